#!/usr/bin/env python3
"""Pin the full-size BASELINE.json configs against the genuine reference (run HERE).

The reference binaries are the ones oracle/build_ref.sh builds from /root/reference
(oracle/_ref/bin/, BEDOPS v2.4.26). Inputs come from the SURVEY.md Appendix D generator
(tools/bedgen.c, through tools/build/libbedgen.so), written contig by contig so no whole
file is ever held in memory. Each config runs ONE reference process on the whole input files
(run (i) of BASELINE.md §3: the reference's own answer, no --chrom splitting involved), file ->
file; the output's rows, bytes and sha256 prefix are recorded, then the inputs are deleted.

    python tools/pin_fullsize.py [config ...]       # default: all
    -> tests/golden/ref_fullsize.json  (merged with what is already there)

Configs (names match bench.py WORKLOADS):
  bedmap          bedmap --count --mean R(50M, seed 7, BED3) M(500M, seed 8, BED5)   configs[2]
  element-of      bedops --element-of 1 A(200M, seed 44) B(200M, seed 45)            configs[3]
  closest         closest-features --closest Q(10M, seed 46) R(1B, seed 47)          configs[4]
  bedmap-decimal  bedmap --count --mean R(5M, seed 7) M(50M, seed 8, decimal scores)
  intersect       bedops --intersect A(100M, seed 42) B(100M, seed 43)               configs[1]
"""
import ctypes
import hashlib
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "bin")
OUT = os.path.join(ROOT, "tests", "golden", "ref_fullsize.json")
WORK = os.environ.get("PIN_WORKDIR", os.path.join(ROOT, "exp", "pin"))

CONFIGS = {
    "intersect": {"tool": "bedops", "args": ["--intersect"], "gen": [(100_000_000, 42, 3), (100_000_000, 43, 3)]},
    "element-of": {"tool": "bedops", "args": ["--element-of", "1"],
                   "gen": [(200_000_000, 44, 3), (200_000_000, 45, 3)]},
    "bedmap": {"tool": "bedmap", "args": ["--count", "--mean"], "gen": [(50_000_000, 7, 3), (500_000_000, 8, 5)]},
    "bedmap-decimal": {"tool": "bedmap", "args": ["--count", "--mean"],
                       "gen": [(5_000_000, 7, 3), (50_000_000, 8, 6)]},
    "closest": {"tool": "closest-features", "args": ["--closest"],
                "gen": [(10_000_000, 46, 3), (1_000_000_000, 47, 3)]},
}


def lib():
    p = os.path.join(ROOT, "tools", "build", "libbedgen.so")
    if not os.path.exists(p):
        subprocess.run(["make", "-s", "tools"], cwd=ROOT, check=True)
    L = ctypes.CDLL(p)
    L.bedgen_buffer_subset.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.bedgen_free.argtypes = [ctypes.c_void_p]
    return L


def write_file(L, path, n, seed, mode):
    """the whole generator file, one contig at a time (identical bytes: jump-ahead streams)"""
    rows = 0
    h = hashlib.sha256()
    with open(path, "wb") as f:
        for c in range(L.bedgen_ncontigs()):
            p, nb, r = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
            if L.bedgen_buffer_subset(n, seed, mode, 0, 1 << c, ctypes.byref(p), ctypes.byref(nb),
                                      ctypes.byref(r)):
                raise RuntimeError("bedgen failed")
            buf = (ctypes.c_char * max(nb.value, 1)).from_address(p.value)
            mv = memoryview(buf)[:nb.value]
            f.write(mv)
            h.update(mv)
            L.bedgen_free(p)
            rows += r.value
    return rows, os.path.getsize(path), h.hexdigest()[:16]


def sha_file(path):
    h, rows = hashlib.sha256(), 0
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 26), b""):
            h.update(chunk)
            rows += chunk.count(b"\n")
    return rows, os.path.getsize(path), h.hexdigest()[:16]


def pin(L, name):
    C = CONFIGS[name]
    d = os.path.join(WORK, name)
    os.makedirs(d, exist_ok=True)
    paths, inputs = [], []
    t0 = time.time()
    for i, (n, seed, mode) in enumerate(C["gen"]):
        p = os.path.join(d, f"in{i}.bed")
        rows, nbytes, sha = write_file(L, p, n, seed, mode)
        paths.append(p)
        inputs.append({"N": n, "seed": seed, "mode": {3: "BED3", 5: "BED5", 6: "BED5-decimal"}[mode],
                       "rows": rows, "bytes": nbytes, "sha16": sha})
    tg = time.time() - t0
    out = os.path.join(d, "out.bed")
    t1 = time.time()
    with open(out, "wb") as fo:
        r = subprocess.run([os.path.join(REF, C["tool"]), *C["args"], *paths], stdout=fo,
                           stderr=subprocess.PIPE)
    tr = time.time() - t1
    if r.returncode:
        raise RuntimeError(f"{name}: reference rc {r.returncode}: {r.stderr[-500:]!r}")
    rows, nbytes, sha = sha_file(out)
    for p in paths + [out]:
        os.unlink(p)
    rec = {"command": f"{C['tool']} {' '.join(C['args'])} <inputs>", "inputs": inputs,
           "output": {"rows": rows, "bytes": nbytes, "sha16": sha},
           "reference": "oracle/_ref/bin (BEDOPS v2.4.26 built by oracle/build_ref.sh), one process, "
                        "whole files, file -> file",
           "reference_seconds": round(tr, 1)}
    print(f"{name}: gen {tg:.0f}s ref {tr:.0f}s -> {rec['output']}", flush=True)
    return name, rec


def main():
    names = sys.argv[1:] or list(CONFIGS)
    L = lib()
    done = json.load(open(OUT)) if os.path.exists(OUT) else {}
    with ThreadPoolExecutor(max_workers=int(os.environ.get("PIN_JOBS", "3"))) as ex:
        for name, rec in ex.map(lambda n: pin(L, n), names):
            done[name] = rec
            with open(OUT, "w") as f:
                json.dump({k: done[k] for k in sorted(done)}, f, indent=1)
                f.write("\n")


if __name__ == "__main__":
    main()
