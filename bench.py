#!/usr/bin/env python3
"""bench.py — headline benchmark of the bedops_amd sweep path on MI355X.

Metric (BASELINE.json): intervals/sec of `bedops --intersect A.bed B.bed`, 100M x 100M
sorted BED3 (SURVEY.md Appendix D generator, seeds 42/43), at 1/2/4/8 GPUs.

One step = one whole pass of the GPU path over the input text already resident in HBM:
load both files (k_scout, k_tokhash, run/dictionary kernels, k_parse_set) -> per-file
components -> intersect (k_mp_partition, k_mp_tile) -> render the sorted BED text back into
HBM (k_fmt_*). With N GPUs (one process per GPU; `--gpus N` starts them itself, or
torch.distributed.run does) the chromosomes are assigned to ranks by
bedops_amd.shard.assign (LPT), every rank runs the step on its chromosomes only and the
ranks exchange their per-chromosome byte counts, which places each rank's text at its
offset of the sorted output (the sharded drop-in then writes it in place, cli_shard.h);
the same steps with the whole text reassembled on rank 0 in strcmp order by
bg_group_gather (bedops_amd/csrc/bg_group.hip: grouped ncclSend/ncclRecv over xGMI) are
timed beside them (`multi_gpu`: placement vs with-gather step time, the gather's cost).
Strong scaling by default: the dataset is the fixed 100M x 100M at every N (`--weak`: N x
100M rows per file). After the timed steps rank 0 hashes the reassembled output against the
reference binary's hash at every N.

Rank 0, N = 1, also times, all file -> file with the inputs
in the page cache and the output written to a file:
  e2e           the drop-in CLI `bedops_amd/bin/bedops --intersect A B > out` (process start,
                HIP init, reads, device work, output write), median of 3, with the
                BEDGPU_STATS phase marks of the median run; `--e2e-devices 0,1,..` also times
                the sharded drop-in (BEDGPU_DEVICES);
  cpu_baseline  the genuine reference (oracle/_ref, built from /root/reference by
                oracle/build_ref.sh): run (ii) one `--chrom` process per chromosome over the
                full files, min(nproc, 25) at a time, outputs concatenated in strcmp order
                (the reference's documented scale-out, bedops.rst:721-726), median of 3; run
                (i) one process on the full inputs; CPU model and core counts;
  gpu_vs_cpu    e2e / run (ii); gpu_vs_cpu_single: e2e / run (i).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "intervals/sec, bedops --intersect 100M×100M BED3 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# reference bedops output for A100M x B100M
REF_INTERSECT = {"rows": 38507974, "bytes": 917848625, "sha16": "2495074965b49d74"}
REF_BEDMAP_R5M = {"rows": 4999998, "bytes": 54515904, "sha16": "899ec7973e166e2d"}
# every workload's full-size output from the genuine reference, one process on the whole
# files (tools/pin_fullsize.py run in the build container -> tests/golden/ref_fullsize.json)
try:
    with open(os.path.join(ROOT, "tests", "golden", "ref_fullsize.json")) as _f:
        REF_PINS = json.load(_f)
    REF_FULL = {k: v["output"] for k, v in REF_PINS.items()}
except OSError:
    REF_PINS, REF_FULL = {}, {}

# bg_prof labels -> kernel names as rocprofv3 reports them (profiles/pmc_traffic.json)
PMC_NAME = {"k_components_count": "k_components<false>", "k_components_write": "k_components<true>",
            "k_parse_set": "k_parse_set_v", "k_parse": "k_parse_rv",
            "k_intersect_count": "k_mp_tile<0, false>", "k_intersect_write": "k_mp_tile<0, true, true>"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- inputs
def bedgen_lib():
    p = os.path.join(ROOT, "tools", "build", "libbedgen.so")
    if not os.path.exists(p):
        subprocess.run(["make", "-s", "tools"], cwd=ROOT, check=True)
    L = ctypes.CDLL(p)
    L.bedgen_buffer_subset.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.bedgen_contig_name.restype = ctypes.c_char_p
    L.bedgen_contig_len.restype = ctypes.c_uint64
    L.bedgen_free.argtypes = [ctypes.c_void_p]
    return L


def contigs(L):
    return [(L.bedgen_contig_name(c).decode(), L.bedgen_contig_len(c)) for c in range(L.bedgen_ncontigs())]


def gen(L, n, seed, mask, mode=3):
    p, nb, rows = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
    rc = L.bedgen_buffer_subset(n, seed, mode, 0, mask, ctypes.byref(p), ctypes.byref(nb),
                                ctypes.byref(rows))
    if rc:
        raise RuntimeError("bedgen failed")
    return p, nb.value, rows.value


def host_bytes(p, nb):
    return memoryview((ctypes.c_char * max(nb, 1)).from_address(p.value))[:nb]


def to_device(torch, p, nb, dev):
    import numpy as np
    host = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(max(nb, 1),))
    t = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    t.copy_(torch.from_numpy(host[:max(nb, 1)]))
    return t


# ----------------------------------------------------------------------------- roofline
def kernel_bytes(name, w):
    """algorithmic HBM bytes per launch of kernel `name` for workload sizes `w`
    (what each kernel must read and write at minimum)."""
    texts, rows, kinds = w["texts"], w["rows"], w["kinds"]
    nf = len(texts)
    col = {0: 16, 1: 28, 2: 24, 3: 0, 4: 36}  # keyed start/end (+ rest span 12 B | score 8 B) per row
    out, obytes, comps = w["out"], w["out_bytes"], w["comps"]
    table = {
        # one launch per input file: text read + columns written (mean over the files)
        "k_parse": sum(t + col[k] * r for t, r, k in zip(texts, rows, kinds)) / nf,
        "k_scout": sum(texts) / nf,
        # BG_BED3_SET: text read + the file's components written (staged once)
        "k_parse_set": (sum(t for t, k in zip(texts, kinds) if k == 3) + 16 * comps)
        / max(1, sum(1 for k in kinds if k == 3)),
        "k_tile_max": 8 * sum(rows) / nf,
        "k_components_count": 16 * sum(rows) / nf,
        "k_components_write": (16 * sum(rows) + 16 * comps) / nf,
        # one launch per step: both component lists read (+ pieces written)
        "k_intersect_count": 16 * comps,
        "k_intersect_write": 16 * comps + 16 * out,
        "k_fmt_count": 16 * out,
        "k_fmt_write": 16 * out + obytes,
        # bedmap: ref keys, map keys + score read; count + sum written
        "k_map_ops": 28 * rows[0] + 24 * rows[-1],
        # closest: every ref row and every candidate read once; left/right written
        "k_closest_chunks": 32 * rows[0] + 16 * rows[-1],
        # element-of: ref keys read + one flag per row; union prefix searched (cached)
        "k_element_flags": 17 * rows[0],
    }
    return table.get(name)


# ----------------------------------------------------------------------------- workloads
# BASELINE.json configs on the GPU path. "intersect" (configs[1]) is the headline metric
# and the default; the others are measured with --workload for DESIGN.md.
# gen: (seed, 3 = BED3 | 5 = BED5 | 6 = BED5 decimal scores) per input; rows: per input.
WORKLOADS = {
    "intersect": {"gen": [(42, 3), (43, 3)], "rows": [100_000_000, 100_000_000],
                  "kinds": [3, 3], "oracle": "bedops_oracle", "args": ["-i"], "cli": "bedops",
                  "ref": REF_INTERSECT,
                  "desc": "bedops --intersect A.bed B.bed: BED3 text in HBM -> parse -> merge -> "
                          "intersect -> BED text in HBM"},
    "element-of": {"gen": [(44, 3), (45, 3)], "rows": [200_000_000, 200_000_000],
                   "kinds": [1, 3], "oracle": "bedops_oracle", "args": ["-e", "1"], "cli": "bedops",
                   "ref": REF_FULL.get("element-of"),
                   "desc": "bedops --element-of 1 A.bed B.bed (configs[3] shape, 200M x 200M)"},
    "bedmap": {"gen": [(7, 3), (8, 5)], "rows": [50_000_000, 500_000_000], "kinds": [0, 2],
               "oracle": "bedmap_oracle", "args": ["--count", "--mean"], "cli": "bedmap",
               "ref": REF_FULL.get("bedmap"), "desc": "bedmap --count --mean ref.bed map.bed (configs[2], 50M x 500M "
                                    "BED5 map)"},
    "bedmap-decimal": {"gen": [(7, 3), (8, 6)], "rows": [5_000_000, 50_000_000], "kinds": [0, 4],
                       "oracle": "bedmap_oracle", "args": ["--count", "--mean"], "cli": "bedmap",
                       "ref": REF_FULL.get("bedmap-decimal"),
                       "desc": "bedmap --count --mean ref.bed map.bed, decimal scores (running "
                               "double replayed in the reference's event order; 5M x 50M)"},
    "closest": {"gen": [(46, 3), (47, 3)], "rows": [10_000_000, 1_000_000_000], "kinds": [1, 1],
                "oracle": "closest_oracle", "args": ["--closest"], "cli": "closest-features",
                "ref": REF_FULL.get("closest"), "desc": "closest-features --closest query.bed ref.bed (configs[4], "
                                     "10M x 1B)"},
}


def run_op(eng, name, s):
    if name == "intersect":
        return eng.op("-i", s, [0, 1])
    if name == "element-of":
        return eng.op("-e", s, [0, 1], "1")
    if name.startswith("bedmap"):
        return eng.map_op(s, ["count", "mean"], 0, 1)
    return eng.closest_op(s, 0, 1, shortest=True)


# ----------------------------------------------------------------------------- process launch
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N rank processes of this script (before any GPU
    call in this process) and exit with the first failing child's status."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        rc = rc or c
    sys.exit(rc)


# ----------------------------------------------------------------------------- baselines
def write_inputs(L, W, td):
    """the full inputs as files (page cache) for the CLI and the CPU fan-out"""
    paths, rows = [], 0
    for i, (seed, mode) in enumerate(W["gen"]):
        p, nb, r = gen(L, W["rows"][i], seed, ~0 & ((1 << 64) - 1), mode)
        path = os.path.join(td, f"in{i}.bed")
        with open(path, "wb") as f:
            f.write(host_bytes(p, nb))
        L.bedgen_free(p)
        paths.append(path)
        rows += r
    return paths, rows


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def _sha16_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 26), b""):
            h.update(chunk)
    return h.hexdigest()[:16]


def _phases(stderr):
    """BEDGPU_STATS=1 marks (bedops_amd/cli/cli_common.h cli_mark, bg_stats): host phase
    deltas and per-stage times, in ms"""
    host, stage = {}, {}
    for ln in stderr.splitlines():
        f = ln.split()
        if len(f) >= 5 and f[0] == "bedgpu" and f[1] == "host" and f[-1].startswith("(+"):
            host[f[2]] = round(float(f[-1][2:-1]), 3)
        elif len(f) >= 5 and f[0] == "bedgpu" and f[1] == "stage":
            stage[f[2]] = round(stage.get(f[2], 0.0) + float(f[3]), 3)
    return {"host_ms": host, "stage_ms": stage}


def _run_pipe(argv, env, cap=None):
    """one CLI run with stdout to a pipe drained by this process; (seconds, sha16, bytes, rc,
    stderr). The clock stops when the process has exited and the pipe is drained; the consumer
    only collects the bytes (a hash while reading would make it the slowest stage, ~1.5 GB/s):
    the output is hashed after the clock stops. cap (the output size of the file run): the
    consumer reads into one buffer allocated and touched before the clock starts, as a C
    reader (`cat`, `gzip`) reads into its own reused buffer — a new 1 MiB bytes object per
    read() made the consumer, not the pipe, the slow end (~4.6 GB/s)."""
    import threading
    buf = bytearray(cap + (1 << 22)) if cap else None
    mv = memoryview(buf) if buf is not None else None
    chunks = []
    off = 0
    t0 = time.perf_counter()
    p = subprocess.Popen(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, bufsize=0)
    err = []
    th = threading.Thread(target=lambda: err.append(p.stderr.read()))
    th.start()
    fd = p.stdout.fileno()
    while True:
        if mv is not None and off + (1 << 22) <= len(buf):
            k = os.readv(fd, [mv[off:off + (1 << 22)]])
            if k == 0:
                break
            off += k
            continue
        b = os.read(fd, 1 << 22)
        if not b:
            break
        chunks.append(b)
    rc = p.wait()
    th.join()
    dt = time.perf_counter() - t0
    h = hashlib.sha256()
    if mv is not None:
        h.update(mv[:off])
    n = off
    for b in chunks:
        h.update(b)
        n += len(b)
    return dt, h.hexdigest()[:16], n, rc, b"".join(err)


def e2e_cli(W, paths, rows, td, runs=3, devices=None, spacing=0.5, sink="file", extra_env=None, pipe_cap=None):
    """the drop-in CLI, file -> file: `bedops_amd/bin/<tool> <args> <files> > out`, input files
    in the page cache, process start + HIP init + reads + device work + output write all
    inside the wall clock. Median of `runs`, with the BEDGPU_STATS phase
    marks of the median run. devices: BEDGPU_DEVICES for the sharded drop-in (None: 1 GPU).
    spacing: seconds between runs (0: back to back, as a shell script of consecutive
    commands runs them); sink "pipe": stdout to a pipe this process drains (`| consumer`);
    extra_env: e.g. BEDGPU_DETACH=0 (the process lifetime includes the GPU teardown)."""
    exe = os.path.join(ROOT, "bedops_amd", "bin", W["cli"])
    out = os.path.join(td, "cli_out.bed")
    args = W["args"] if W["cli"] != "closest-features" else ["--closest"]
    env = {k: v for k, v in os.environ.items() if k != "BEDGPU_DEVICES"}
    env["BEDGPU_STATS"] = "1"
    env.update(extra_env or {})
    if devices:
        env["BEDGPU_DEVICES"] = devices
    times, logs, sha, nbytes = [], [], None, None
    for i in range(runs):
        # by default runs start 0.5 s apart: the drop-in returns once its output is written
        # and its GPU worker tears down detached (bedops_amd/cli/cli_common.h cli_detach,
        # 60-100 ms in the kernel driver); a run started inside that window pays for it in HIP
        # init (measured separately with spacing=0)
        if i and spacing:
            time.sleep(spacing)
        if sink == "pipe":
            dt, sha, nbytes, rc, err = _run_pipe([exe, *args, *paths], env, pipe_cap)
        else:
            with open(out, "wb") as fo:
                t0 = time.perf_counter()
                r = subprocess.run([exe, *args, *paths], stdout=fo, stderr=subprocess.PIPE, env=env)
                dt = time.perf_counter() - t0
            rc, err = r.returncode, r.stderr
        if rc != 0:
            raise RuntimeError(f"CLI failed: {err.decode(errors='replace')[-2000:]}")
        times.append(dt)
        logs.append(err.decode(errors="replace"))
        log(f"e2e run {i} ({sink}, spacing {spacing}, {extra_env or ''}): {dt:.3f} s")
    med = _median(times)
    if sink != "pipe":
        sha, nbytes = _sha16_file(out), os.path.getsize(out)
        os.unlink(out)
    envs = " ".join(f"{k}={v}" for k, v in (extra_env or {}).items())
    rec = {"value": rows / med, "unit": "intervals/s", "median_s": round(med, 4),
           "runs_s": [round(t, 4) for t in times], "spacing_s": spacing, "sink": sink,
           "command": f"{'BEDGPU_DEVICES=' + devices + ' ' if devices else ''}{envs + ' ' if envs else ''}"
                      f"bedops_amd/bin/{W['cli']} {' '.join(args)} <files> "
                      f"{'| reader' if sink == 'pipe' else '> out'}",
           "output_sha16": sha, "output_bytes": nbytes,
           "consumer": (("readv into one preallocated buffer" if pipe_cap else "os.read 4 MiB chunks")
                        if sink == "pipe" else None),
           "phases": _phases(logs[times.index(med)]),
           # the staging ring's own report of the median run (copy issue / drain times, and
           # how long its threads waited on DMA vs copied on the CPU)
           "ring": [ln.strip() for ln in logs[times.index(med)].splitlines()
                    if ln.startswith("bedgpu ring")][:40]}
    return rec


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


def _ref_exe(W):
    """the genuine reference binary built by oracle/build_ref.sh (None: not built)"""
    exe = os.path.join(ROOT, "oracle", "_ref", "bin", {"bedops": "bedops", "bedmap": "bedmap",
                                                        "closest-features": "closest-features"}[W["cli"]])
    return exe if os.access(exe, os.X_OK) else None


def cpu_single(W, paths, rows, td, runs):
    """BASELINE.md run (i): one reference process on the full inputs, file -> file"""
    exe = _ref_exe(W)
    kind = "reference"
    if exe is None:
        exe, kind = os.path.join(ROOT, "oracle", "build", W["oracle"]), "port"
    out = os.path.join(td, "cpu1_out.bed")
    times = []
    for i in range(runs):
        with open(out, "wb") as fo:
            t0 = time.perf_counter()
            subprocess.run([exe, *W["args"], *paths], stdout=fo, check=True)
            times.append(time.perf_counter() - t0)
        log(f"cpu run (i) {i}: {times[-1]:.2f} s")
    sha = _sha16_file(out)
    os.unlink(out)
    med = _median(times)
    return {"value": rows / med, "unit": "intervals/s", "cores": 1, "kind": kind,
            "median_s": round(med, 3), "runs_s": [round(t, 2) for t in times],
            "output_sha16": sha,
            "sample": f"full inputs ({rows} rows), one process: "
                      f"{os.path.relpath(exe, ROOT)} {' '.join(W['args'])} <files> > out, "
                      f"median of {runs}"}


def cpu_single_pinned(workload, rows):
    """run (i) from the pin file: the genuine reference, one process on the same full inputs
    (same generator, seeds and sizes), timed by tools/pin_fullsize.py in the BUILD container
    (not on the GPU box: a 3-8 minute single-process run does not fit a box call)"""
    pin = REF_PINS.get(workload)
    if not pin or not pin.get("reference_seconds"):
        return None
    sec = float(pin["reference_seconds"])
    return {"value": rows / sec, "unit": "intervals/s", "cores": 1, "kind": "reference",
            "median_s": sec, "runs_s": [sec], "output_sha16": pin["output"]["sha16"],
            "measured_in": "build container (tests/golden/ref_fullsize.json), not the GPU box",
            "sample": f"full inputs ({rows} rows), one process: {pin.get('reference', '')}: "
                      f"{pin.get('command', '')}"}


def cpu_fanout_ref(L, W, paths, rows, td, workers, runs):
    """BASELINE.md run (ii), the reference's documented scale-out (bedops.rst:721-726): one
    `--chrom <c>` process per chromosome over the FULL input files (the reference's own
    --chrom seek), `workers` at a time (xargs -P), outputs concatenated in strcmp order,
    file -> file, median of `runs`"""
    exe = _ref_exe(W)
    names = sorted((nm for nm, _ in contigs(L)), key=lambda n: n.encode())
    lens = dict(contigs(L))
    order = sorted(names, key=lambda n: -lens[n])  # longest first, as a scheduler would
    times, sha = [], None
    for i in range(runs):
        outs = {n: os.path.join(td, f"fan_{n}.bed") for n in names}
        t0 = time.perf_counter()
        running, pending = [], list(order)
        while pending or running:
            while pending and len(running) < workers:
                n = pending.pop(0)
                fo = open(outs[n], "wb")
                running.append((subprocess.Popen([exe, "--chrom", n, *W["args"], *paths], stdout=fo), fo))
            p, fo = running.pop(0)
            if p.wait() != 0:
                raise RuntimeError("reference failed in the CPU fan-out")
            fo.close()
        final = os.path.join(td, "fan_out.bed")
        with open(final, "wb") as fo:
            for n in names:
                with open(outs[n], "rb") as fi:
                    while True:
                        b = fi.read(1 << 26)
                        if not b:
                            break
                        fo.write(b)
        times.append(time.perf_counter() - t0)
        log(f"cpu run (ii) {i}: {times[-1]:.2f} s")
        sha = _sha16_file(final)
        for n in names:
            os.unlink(outs[n])
        os.unlink(final)
    med = _median(times)
    return {"value": rows / med, "unit": "intervals/s", "cores": workers, "kind": "reference",
            "median_s": round(med, 3), "runs_s": [round(t, 2) for t in times], "output_sha16": sha,
            "sample": f"full inputs ({rows} rows): {os.path.relpath(exe, ROOT)} --chrom <c> "
                      f"{' '.join(W['args'])} <files>, one process per chromosome ({len(names)}), "
                      f"{workers} at a time, outputs concatenated in strcmp order, file->file, "
                      f"median of {runs}"}


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="intersect")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: N x the workload's rows per file (default: strong)")
    ap.add_argument("--scale", type=float, default=1.0,
                    help="rows per input = scale x the workload's size (tests/smoke)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="processes of the CPU fan-out, run (ii) (default: min(nproc, 25))")
    ap.add_argument("--cpu-single-runs", type=int, default=1,
                    help="runs of the one-process reference, run (i) (median; ~60 s each); 0: take "
                         "run (i) from tests/golden/ref_fullsize.json (timed in the build container)")
    ap.add_argument("--cpu-fanout-runs", type=int, default=3)
    ap.add_argument("--e2e-runs", type=int, default=3)
    ap.add_argument("--e2e-devices", default=None,
                    help="also time the drop-in CLI sharded over BEDGPU_DEVICES (e.g. 0,1)")
    ap.add_argument("--load-only", action="store_true",
                    help="time the loader stage alone (text in HBM -> keyed columns)")
    ap.add_argument("--profile-all", action="store_true",
                    help="time every kernel during the timed steps (default: only the dominant one)")
    ap.add_argument("--share-device", action="store_true",
                    help="(rehearsal of N > 1 on a one-GPU box) every rank on cuda:0, no RCCL "
                         "between ranks: the placement steps only, no gather, no parity hash")
    args = ap.parse_args()
    W = WORKLOADS[args.workload]

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        spawn_ranks(args.gpus)  # does not return
    world = int(env_world or "1")
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
            f"{world}-GPU run as {args.gpus} GPUs")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_device else int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    from bedops_amd.engine import Group, group_uid
    from bedops_amd.shard import assign, member_spans, strcmp_order

    dist = None
    if world > 1:
        import torch.distributed as dist
        # host-side coordination only (uid, barriers, the max over ranks); the data path's
        # exchange is RCCL inside libbedgpu (bg_group_gather)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        uidl = [group_uid() if rank == 0 else None]
        dist.broadcast_object_list(uidl, src=0)
        uid = uidl[0]
    else:
        uid = bytes(128)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    grp = Group(device=local, uid=bytes(128), nranks=1, rank=0) if args.share_device else \
        Group(device=local, uid=uid, nranks=world, rank=rank)
    eng = grp.engines[0]

    L = bedgen_lib()
    cs = contigs(L)
    owner, _ = assign({nm: ln for nm, ln in cs}, world)  # rows per contig ∝ its length
    gnames = strcmp_order([nm for nm, _ in cs])
    mask = sum(1 << c for c, (nm, _) in enumerate(cs) if owner[nm] == rank)
    per_file = [int(r * args.scale) * (world if args.weak else 1) for r in W["rows"]]
    t0 = time.perf_counter()
    bufs, texts, rows = [], [], []
    for (seed, mode), n in zip(W["gen"], per_file):
        p, nb, r = gen(L, n, seed, mask, mode)
        bufs.append(to_device(torch, p, nb, dev))
        L.bedgen_free(p)
        texts.append(nb)
        rows.append(r)
    log(f"[rank {rank}] {args.workload}: generated {rows} rows / {texts} bytes in "
        f"{time.perf_counter() - t0:.1f}s")
    torch.cuda.synchronize(dev)

    state = {}
    inputs = [((t.data_ptr(), nb), k) for t, nb, k in zip(bufs, texts, W["kinds"])]

    def step(gather=False):
        """one pass of the hot path. N > 1: each rank loads, operates and formats its
        chromosomes (the text stays in its HBM, as at N = 1) and the ranks exchange their
        per-chromosome byte counts, which places every rank's spans in the sorted output (what
        the sharded drop-in writes in place with per-device pwrite, cli_shard.h); gather=True
        also reassembles the whole text on rank 0 over RCCL (bg_group_gather)"""
        s = eng.load(inputs)
        if args.load_only:
            state["out_rows"] = state["out_bytes"] = 0
            s.free()
            return
        r = run_op(eng, args.workload, s)
        nbytes = r.format()
        state["out_rows"] = r.rows()
        state["out_bytes"] = nbytes
        if world > 1:
            names = s.chroms()
            offs, lens = member_spans(names, r.chrom_spans(len(names)), gnames)
            if gather or "keep" in state:  # the path's one data exchange: text -> rank 0 (RCCL)
                dptr, _ = r.device_text()
                out, n = grp.gather(len(gnames), [(dptr, offs, lens)])
                if rank == 0:
                    if "keep" in state:
                        state["text"] = read_device(out, n)
                        del state["keep"]
                    eng.device_free(out)
            else:  # placement: every chromosome's byte count from every rank (host, gloo)
                cnt = torch.tensor(lens, dtype=torch.int64)
                allc = [torch.empty_like(cnt) for _ in range(world)]
                dist.all_gather(allc, cnt)
                tot = torch.stack(allc).sum(0)
                before = torch.cumsum(tot, 0) - tot  # output offset of each chromosome
                state["place"] = int(before[[i for i, ln in enumerate(lens) if ln][0]]) if any(lens) else 0
        elif "keep" in state:
            state["text"] = r.text()
            del state["keep"]
        r.free()
        s.free()

    def read_device(dptr, n):
        with tempfile.TemporaryFile() as fo:
            eng.write_device(dptr, n, fo.fileno())
            fo.seek(0)
            return fo.read()

    def barrier():
        eng.sync()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()

    # warmup; every warmup step profiles every kernel: the last (warm) one names the
    # dominant kernel (the first carries code-object loading and first-touch costs — with
    # --warmup 1 it named k_fmt_write, whose first launch faults its output pages in — so at
    # least two untimed steps run)
    eng.prof_enable("*")
    for w in range(max(args.warmup, 2)):
        step()
        last = eng.prof_read()
        eng.prof_enable("*")  # (clears the statistics)
        if w == 0:
            first = last
    eng.prof_enable("")
    dominant = max(last.items(), key=lambda kv: kv[1][1])[0]
    comps = 0
    if args.workload == "intersect":  # component counts size the merge/intersect kernels
        s = eng.load(inputs)
        for f in (0, 1):
            m = eng.op("-m", s, [f])
            comps += m.rows()
            m.free()
        s.free()
    eng.prof_enable("*" if args.profile_all else dominant)
    barrier()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    torch.cuda.synchronize(dev)
    t_end = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t_end - t_start
    total_rows = sum(rows)
    if dist:
        et = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(et, op=dist.ReduceOp.MAX)
        elapsed = float(et.item())
        rt = torch.tensor([sum(rows)], dtype=torch.int64)
        dist.all_reduce(rt)
        total_rows = int(rt.item())
    prof = eng.prof_read()
    # N > 1: the same steps with the whole text reassembled on rank 0 (the RCCL gather the
    # drop-in's pipe output needs), timed the same way, reported beside the placement steps
    multi = None
    if dist and not args.load_only and not args.share_device:
        barrier()
        g0 = time.perf_counter()
        for _ in range(args.steps):
            step(gather=True)
        eng.sync()
        torch.cuda.synchronize(dev)
        g1 = time.perf_counter()
        dist.barrier()
        gt = torch.tensor([g1 - g0], dtype=torch.float64)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        gms = float(gt.item()) / args.steps * 1e3
        ob = torch.tensor([state["out_bytes"]], dtype=torch.int64)
        dist.all_reduce(ob)
        multi = {"step_ms_placement": round(elapsed / args.steps * 1e3, 3),
                 "step_ms_with_gather": round(gms, 3),
                 "gather_ms": round(gms - elapsed / args.steps * 1e3, 3),
                 "output_bytes": int(ob.item()),
                 "value_with_gather": round(total_rows / (gms / 1e3), 1),
                 "rank_rows": rows, "note": "max over ranks; value = placement steps (text left "
                 "in each rank's HBM at its output offset), value_with_gather = every step also "
                 "gathers the text to rank 0 over RCCL"}

    # parity after timing: the reassembled output against the reference hash, at every N
    verify = None
    if not args.no_verify and not args.load_only and args.scale == 1.0 and not args.weak and not args.share_device:
        if rank == 0:
            state["keep"] = True
        step()
        if rank == 0:
            txt = state.pop("text")
            verify = {"rows": txt.count(b"\n"), "bytes": len(txt),
                      "sha16": hashlib.sha256(txt).hexdigest()[:16]}
            if W["ref"]:
                verify["matches_reference"] = all(verify[k] == W["ref"][k] for k in W["ref"])
            del txt
    if dist:
        dist.barrier()

    if rank != 0:
        grp.close()
        # (rank 0 times the sharded drop-in once every rank has released its group)
        dist.barrier()
        dist.destroy_process_group()
        return

    # roofline of the dominant kernel, from its launches inside the timed region
    sizes = {"texts": texts, "rows": rows, "kinds": W["kinds"], "out": state["out_rows"],
             "out_bytes": state["out_bytes"], "comps": comps}
    roof = None
    per_launch = kernel_bytes(dominant, sizes)
    if per_launch is not None and dominant in prof:
        calls, ms = prof[dominant]  # launches inside the timed region only
        avg_s = ms / 1e3 / max(calls, 1)
        gbs = per_launch / avg_s / 1e9
        traffic = None
        # per-launch HBM bytes of the same workload's kernels from the committed PMC passes
        # (tools/gpu_profile_r02.sh -> profiles/pmc_traffic_<workload>.json)
        pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.workload}.json")
        if not os.path.exists(pmc) and args.workload == "intersect":
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc) and world == 1 and args.scale == 1.0:
            try:
                tbl = json.load(open(pmc))
                key = PMC_NAME.get(dominant, dominant)
                ent = tbl.get(key)
                if ent:
                    traffic = ent.get("bytes")
                else:  # template instances (e.g. one k_parse_rv per file kind): launch-weighted mean
                    vs = [v for k, v in tbl.items() if k.startswith(key + "<") and v.get("launches")]
                    if vs:
                        traffic = int(sum(v["bytes"] * v["launches"] for v in vs) / sum(v["launches"] for v in vs))
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dominant,
                "avg_ms": round(avg_s * 1e3, 4), "launches": calls,
                "bytes_per_launch": int(per_launch), "rank": 0}

    e2e = cpu = e2e_sh = None
    if world > 1:
        # N GPUs: the shipped drop-in itself over the same N devices (BEDGPU_DEVICES=0..N-1,
        # one process driving them, chromosome shards, per-device output writes), file ->
        # file, a fresh child process started after every rank has released its group
        grp.close()
        grp = None
        dist.barrier()
        if not args.no_e2e and args.scale == 1.0 and not args.load_only and not args.weak \
                and not args.share_device:
            with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as td:
                paths, nrows = write_inputs(L, W, td)
                e2e_sh = e2e_cli(W, paths, nrows, td, runs=args.e2e_runs,
                                 devices=",".join(str(d) for d in range(world)))
                if W["ref"]:
                    e2e_sh["matches_reference"] = e2e_sh["output_sha16"] == W["ref"]["sha16"]
                for p in paths:
                    os.unlink(p)
    if world == 1 and args.scale == 1.0 and not args.load_only and (
            not args.no_e2e or not args.no_cpu_baseline):
        with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR")) as td:
            paths, nrows = write_inputs(L, W, td)
            if not args.no_e2e:
                e2e = e2e_cli(W, paths, nrows, td, runs=args.e2e_runs)
                # the same command back to back (no spacing: the previous run's detached GPU
                # teardown overlaps the next run's HIP init), with the GPU teardown inside the
                # process lifetime (BEDGPU_DETACH=0), and with stdout to a pipe
                variants = {"back_to_back": {"spacing": 0},
                            "no_detach": {"extra_env": {"BEDGPU_DETACH": "0"}},
                            "pipe": {"sink": "pipe", "pipe_cap": e2e["output_bytes"]}}
                for name, kw in variants.items():
                    v = e2e_cli(W, paths, nrows, td, runs=args.e2e_runs, **kw)
                    e2e[name] = {k: v[k] for k in ("median_s", "runs_s", "command", "output_sha16", "consumer")}
                    e2e[name]["value"] = round(v["value"], 1)
                if W["ref"]:
                    e2e["matches_reference"] = all(x == W["ref"]["sha16"] for x in
                                                   [e2e["output_sha16"]] + [e2e[n]["output_sha16"] for n in variants])
                if args.e2e_devices:
                    e2e_sh = e2e_cli(W, paths, nrows, td, runs=args.e2e_runs, devices=args.e2e_devices)
                    if W["ref"]:
                        e2e_sh["matches_reference"] = e2e_sh["output_sha16"] == W["ref"]["sha16"]
            if not args.no_cpu_baseline:
                info = cpu_info()
                workers = args.cpu_workers or max(1, min(info["affinity_cpus"], 25))
                # cores the fan-out can actually use: its processes, bounded by the CPUs visible
                # and by the cgroup quota
                eff = min(workers, info["affinity_cpus"],
                          int(info["cgroup_cpu_quota"]) if info["cgroup_cpu_quota"] else workers)
                fan = cpu_fanout_ref(L, W, paths, nrows, td, workers, args.cpu_fanout_runs) \
                    if _ref_exe(W) else None
                single = cpu_single(W, paths, nrows, td, args.cpu_single_runs) if args.cpu_single_runs > 0 \
                    else cpu_single_pinned(args.workload, nrows)
                # (a run (i) taken from the pin file was timed in the build container, not on
                # this host: it is reported under cpu_baseline.single only, never as `value`)
                top = fan or (single if single and "measured_in" not in single else None)
                cpu = {"value": top["value"], "unit": "intervals/s",
                       "cores": eff if fan else top["cores"], "processes": top["cores"],
                       "kind": top["kind"], "sample": top["sample"], **info,
                       "single": single, "fanout": fan} if top else None
            for p in paths:
                os.unlink(p)

    ms_per_step = elapsed / args.steps * 1e3
    value = total_rows * args.steps / elapsed
    line = {
        "metric": METRIC if args.workload == "intersect" else
        f"intervals/sec, {W['desc'].split(' (')[0]}",
        "value": round(value, 1), "unit": "intervals/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (SURVEY.md App. D generator, seeds "
                f"{'/'.join(str(g[0]) for g in W['gen'])}; BED text resident in HBM)",
        "config": {"workload": W["desc"] + (" (loader only)" if args.load_only else ""),
                   "rows_per_input": [r * (world if args.weak else 1) for r in
                                      [int(x * args.scale) for x in W["rows"]]],
                   "parallelism": "single GPU" if world == 1 else
                   f"{world} GPUs (one process each), chromosome shards (LPT); each step places "
                   "every rank's spans in the output by a byte-count exchange, the text stays in "
                   "its rank's HBM (the RCCL gather to rank 0 is timed beside it: multi_gpu)",
                   "output_rows": state["out_rows"] if world == 1 else None},
        "roofline": roof, "cpu_baseline": cpu,
        "e2e_intervals_per_s": round(e2e["value"], 1) if e2e else None,
        "e2e": e2e,
        "e2e_sharded": e2e_sh,
        "e2e_sharded_intervals_per_s": round(e2e_sh["value"], 1) if e2e_sh else None,
        "gpu_vs_cpu": round(e2e["value"] / cpu["value"], 2) if (cpu and e2e) else None,
        "gpu_vs_cpu_single": round(e2e["value"] / cpu["single"]["value"], 2)
        if (cpu and e2e and cpu.get("single") and "measured_in" not in cpu["single"]) else None,
        "gpu_vs_cpu_back_to_back": round(e2e["back_to_back"]["value"] / cpu["value"], 2)
        if (cpu and e2e and "back_to_back" in e2e) else None,
        "gpu_vs_cpu_scope": ("file->file CLI (median of runs 0.5 s apart, the front process's "
                             "lifetime) vs the reference file->file: gpu_vs_cpu against run (ii) "
                             "(--chrom fan-out), gpu_vs_cpu_single against run (i) (one process), "
                             "gpu_vs_cpu_back_to_back: runs back to back against run (ii); "
                             "e2e.no_detach includes the GPU teardown, e2e.pipe writes to a pipe")
        if (cpu and e2e) else None,
        "parity": verify,
        "multi_gpu": multi,
        "kernels_first_step_ms": {k: round(v[1], 4) for k, v in
                                  sorted(first.items(), key=lambda kv: -kv[1][1])},
        "kernels_warm_step_ms": {k: round(v[1], 4) for k, v in
                                 sorted(last.items(), key=lambda kv: -kv[1][1])},
    }
    if args.profile_all:  # HIP-event time per timed step of every kernel
        line["kernels_ms_per_step"] = {k: round(v[1] / args.steps, 4) for k, v in
                                       sorted(prof.items(), key=lambda kv: -kv[1][1])}
    print(json.dumps(line), flush=True)
    if grp:
        grp.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
