#!/usr/bin/env python3
"""bench.py — headline benchmark of the bedops_amd sweep path on MI355X.

Metric (BASELINE.json): intervals/sec of `bedops --intersect A.bed B.bed`, 100M x 100M
sorted BED3 (SURVEY.md Appendix D generator, seeds 42/43).

One step = one whole pass of the GPU path over the input text already resident in HBM:
load both files (k_scout, k_tokhash, run/dictionary kernels, k_parse) -> per-file merge
(k_tile_max, k_components_*) -> intersect (k_mp_partition, k_intersect_*) -> render the
sorted BED text back into HBM (k_fmt_*). With N GPUs (one process per GPU,
torch.distributed over RCCL) the dataset is N x 100M rows per file (weak scaling),
chromosomes go to ranks by bedops_amd.shard.assign (LPT), every rank runs the step on its
shard and bedops_amd.shard.gather_text sends the per-chromosome texts to rank 0 over xGMI,
where they land in strcmp chromosome order — the one exchange the path has.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import ctypes
import hashlib
import json
import os
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


# bg_prof labels -> kernel names as rocprofv3 reports them (profiles/pmc_traffic.json)
PMC_NAME = {"k_components_count": "k_components<false>", "k_components_write": "k_components<true>",
            "k_intersect_count": "k_mp_tile<0, false>", "k_intersect_write": "k_mp_tile<0, true>"}


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


def contig_shards(L, world):
    """contig index -> rank: bedops_amd.shard.assign (LPT) on contig length, which is
    proportional to the generator's rows per contig"""
    from bedops_amd.shard import assign
    n = L.bedgen_ncontigs()
    owner, load = assign({L.bedgen_contig_name(c).decode(): L.bedgen_contig_len(c)
                          for c in range(n)}, world)
    return {c: owner[L.bedgen_contig_name(c).decode()] for c in range(n)}, load


def gen(L, n, seed, mask, mode=3):
    p, nb, rows = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
    rc = L.bedgen_buffer_subset(n, seed, mode, 0, mask, ctypes.byref(p), ctypes.byref(nb),
                                ctypes.byref(rows))
    if rc:
        raise RuntimeError("bedgen failed")
    return p, nb.value, rows.value


def to_device(torch, L, p, nb, dev):
    import numpy as np
    host = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(max(nb, 1),))
    t = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    t.copy_(torch.from_numpy(host[:max(nb, 1)]))
    return t


# ----------------------------------------------------------------------------- roofline
def kernel_bytes(name, w):
    """algorithmic HBM bytes per launch of kernel `name` for workload sizes `w`
    (what each kernel must read and write at minimum)."""
    tb, rows, comps, out, obytes = w["text"], w["rows"], w["comps"], w["out"], w["out_bytes"]
    table = {
        # per file (2 launches per step): text read + keyed start/end written
        "k_parse": (tb + 16 * rows) / 2,
        "k_scout": tb / 2,
        "k_tile_max": 8 * rows / 2,
        "k_components_count": 16 * rows / 2,
        "k_components_write": (16 * rows + 16 * comps) / 2,
        # one launch per step: both component lists read (+ pieces written)
        "k_intersect_count": 16 * comps,
        "k_intersect_write": 16 * comps + 16 * out,
        "k_fmt_count": 16 * out,
        "k_fmt_write": 16 * out + obytes,
    }
    return table.get(name)


# ----------------------------------------------------------------------------- cpu baseline
def cpu_baseline(A_bytes, B_bytes, max_rows=35_000_000):
    """Time the CPU oracle (plain-C restatement of the reference sweep; the reference
    itself is not buildable in this image) on a bounded sample: the leading
    whole chromosomes of A and B (same generator, same order) up to ~max_rows rows."""
    exe = os.path.join(ROOT, "oracle", "build", "bedops_oracle")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "oracle"], cwd=ROOT, check=True)
    cut_names = [b"chr12", b"chr11", b"chr10"]
    best = None
    for nm in cut_names:  # largest prefix of whole contigs under max_rows rows
        ia, ib = A_bytes.find(b"\n" + nm + b"\t"), B_bytes.find(b"\n" + nm + b"\t")
        if ia < 0 or ib < 0:
            continue
        ra, rb = A_bytes.count(b"\n", 0, ia + 1), B_bytes.count(b"\n", 0, ib + 1)
        if ra + rb <= max_rows * 2:
            best = (ia + 1, ib + 1, ra, rb, nm)
            break
    if best is None:
        return None
    ia, ib, ra, rb, nm = best
    with tempfile.TemporaryDirectory() as td:
        pa, pb = os.path.join(td, "a.bed"), os.path.join(td, "b.bed")
        with open(pa, "wb") as f:
            f.write(A_bytes[:ia])
        with open(pb, "wb") as f:
            f.write(B_bytes[:ib])
        with open(os.path.join(td, "out.bed"), "wb") as fo:
            t0 = time.perf_counter()
            subprocess.run([exe, "-i", pa, pb], stdout=fo, check=True)
            dt = time.perf_counter() - t0
    return {"value": (ra + rb) / dt, "unit": "intervals/s", "cores": 1, "kind": "port",
            "sample": f"bedops_oracle -i on the contigs before {nm.decode()} of A100M/B100M "
                      f"({ra}+{rb} rows, file->file, {dt:.2f} s, 1 thread)"}


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=100_000_000, help="rows per file per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--load-only", action="store_true",
                    help="time the loader stage alone (text in HBM -> keyed columns)")
    ap.add_argument("--profile-all", action="store_true",
                    help="time every kernel during the timed steps (default: only the dominant one)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    from bedops_amd import BED3, Engine

    L = bedgen_lib()
    owner, _ = contig_shards(L, world)
    mask = sum(1 << c for c, r in owner.items() if r == rank)
    N = args.rows * world
    t0 = time.perf_counter()
    pa, na, ra = gen(L, N, 42, mask)
    pb, nb, rb = gen(L, N, 43, mask)
    log(f"[rank {rank}] generated A {ra} rows/{na} B, B {rb} rows/{nb} B in {time.perf_counter()-t0:.1f}s")
    ta = to_device(torch, L, pa, na, dev)
    tb_ = to_device(torch, L, pb, nb, dev)
    A_bytes = B_bytes = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        A_bytes = bytes((ctypes.c_char * na).from_address(pa.value))
        B_bytes = bytes((ctypes.c_char * nb).from_address(pb.value))
    L.bedgen_free(pa)
    L.bedgen_free(pb)
    torch.cuda.synchronize(dev)

    eng = Engine(local)
    ncontigs = L.bedgen_ncontigs()
    state = {}

    def step():
        s = eng.load([((ta.data_ptr(), na), BED3), ((tb_.data_ptr(), nb), BED3)])
        if args.load_only:
            state["out_rows"] = state["out_bytes"] = 0
            s.free()
            return
        r = eng.op("-i", s, [0, 1])
        nbytes = r.format()
        state["out_rows"] = r.rows()
        state["out_bytes"] = nbytes
        if world > 1:
            gather_to_rank0(r, s, nbytes)
        if "keep" in state:
            state["text"] = r.text()
            del state["keep"]
        r.free()
        s.free()

    contig_names = [L.bedgen_contig_name(c).decode() for c in range(ncontigs)]
    chrom_owner = {contig_names[c]: owner[c] for c in range(ncontigs)}

    def gather_to_rank0(r, s, nbytes):
        # the path's one exchange: per-chromosome text -> rank 0 over RCCL, in strcmp order
        from bedops_amd.shard import gather_text
        names = s.chroms()
        sp = r.chrom_spans(len(names))
        spans = {nm: (sp[g], sp[g + 1]) for g, nm in enumerate(names) if sp[g + 1] > sp[g]}
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        r.copy_to_device(buf.data_ptr(), max(nbytes, 1))
        out = gather_text(dist, buf, spans, contig_names, chrom_owner, rank, world)
        if rank == 0:
            state["gathered"] = int(out.numel())

    # warmup; the first warmup step profiles every kernel to find the dominant one
    eng.prof_enable("*")
    for w in range(max(args.warmup, 1)):
        step()
        if w == 0:
            first = eng.prof_read()
            eng.prof_enable("")
    dominant = max(first.items(), key=lambda kv: kv[1][1])[0]
    # component counts of A and B (sizes the merge/intersect kernels' algorithmic bytes)
    s = eng.load([((ta.data_ptr(), na), BED3), ((tb_.data_ptr(), nb), BED3)])
    comps = 0
    for f in (0, 1):
        m = eng.op("-m", s, [f])
        comps += m.rows()
        m.free()
    s.free()
    eng.prof_enable("*" if args.profile_all else dominant)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    eng.sync()
    torch.cuda.synchronize(dev)
    t_end = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t_end - t_start
    if dist:
        et = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(et, op=dist.ReduceOp.MAX)
        elapsed = float(et.item())
        rows_all = torch.tensor([ra + rb], dtype=torch.int64, device=dev)
        dist.all_reduce(rows_all)
        total_rows = int(rows_all.item())
    else:
        total_rows = ra + rb
    prof = eng.prof_read()

    if rank != 0:
        eng.close()
        dist.destroy_process_group()
        return

    # roofline of the dominant kernel, from its launches inside the timed region
    sizes = {"text": na + nb, "rows": ra + rb, "out": state["out_rows"],
             "out_bytes": state["out_bytes"], "comps": comps}
    roof = None
    pick = dominant
    per_launch = kernel_bytes(pick, sizes)
    if per_launch is not None and pick in prof:
        calls, ms = prof[pick]  # launches inside the timed region only
        avg_s = ms / 1e3 / max(calls, 1)
        gbs = per_launch / avg_s / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get(PMC_NAME.get(pick, pick), {}).get("bytes")
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": pick,
                "avg_ms": round(avg_s * 1e3, 4), "launches": calls,
                "bytes_per_launch": int(per_launch)}

    verify = None
    if world == 1 and not args.no_verify and args.rows == 100_000_000:
        state["keep"] = True
        step()
        txt = state.pop("text")
        verify = {"rows": txt.count(b"\n"), "bytes": len(txt),
                  "sha16": hashlib.sha256(txt).hexdigest()[:16]}
        verify["matches_reference"] = (verify == {**REF_INTERSECT} or
                                       (verify["rows"] == REF_INTERSECT["rows"] and
                                        verify["bytes"] == REF_INTERSECT["bytes"] and
                                        verify["sha16"] == REF_INTERSECT["sha16"]))
        del txt

    cpu = None
    if world == 1 and not args.no_cpu_baseline and A_bytes is not None:
        cpu = cpu_baseline(A_bytes, B_bytes)

    ms_per_step = elapsed / args.steps * 1e3
    value = total_rows * args.steps / elapsed
    line = {
        "metric": METRIC, "value": round(value, 1), "unit": "intervals/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (SURVEY.md App. D generator, seeds 42/43; BED text resident in HBM)",
        "config": {"workload": "bedops --intersect A.bed B.bed: BED3 text in HBM -> parse -> "
                               "merge -> intersect -> BED text in HBM",
                   "rows_per_file": args.rows * world, "rows_per_gpu_per_file": args.rows,
                   "parallelism": "single GPU" if world == 1 else
                   f"{world} GPUs, chromosome shards (LPT) + RCCL gather to rank 0",
                   "output_rows": state["out_rows"] if world == 1 else None},
        "roofline": roof, "cpu_baseline": cpu,
        "gpu_vs_cpu": round(value / cpu["value"], 1) if cpu else None,
        "parity": verify,
        "kernels_first_step_ms": {k: round(v[1], 4) for k, v in
                                  sorted(first.items(), key=lambda kv: -kv[1][1])},
    }
    print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
