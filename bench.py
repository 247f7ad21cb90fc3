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
    texts, rows, kinds = w["texts"], w["rows"], w["kinds"]
    nf = len(texts)
    col = {0: 16, 1: 28, 2: 24, 3: 0}  # keyed start/end (+ rest span 12 B | score 8 B) per row
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


# ----------------------------------------------------------------------------- cpu baseline
def cpu_baseline(L, W, target_s=15.0):
    """Time the CPU oracle (plain-C restatement of the reference; the reference itself is
    not buildable in this image) on a bounded sample of the same workload:
    the leading whole contigs (strcmp order) of every input, about `target_s` seconds of
    single-thread work at the oracle's expected rate."""
    exe = os.path.join(ROOT, "oracle", "build", W["oracle"])
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "oracle"], cwd=ROOT, check=True)
    n = L.bedgen_ncontigs()
    lens = [L.bedgen_contig_len(c) for c in range(n)]
    total = float(sum(lens))
    budget = W["cpu_rate"] * target_s
    rows_all = sum(W["rows"])
    mask, used = 0, 0.0
    for c in range(n):  # contigs in strcmp order
        share = rows_all * lens[c] / total
        if mask and used + share > budget:
            break
        mask |= 1 << c
        used += share
    last = L.bedgen_contig_name(max(c for c in range(n) if (mask >> c) & 1)).decode()
    with tempfile.TemporaryDirectory() as td:
        paths, nrows = [], 0
        for i, (seed, mode) in enumerate(W["gen"]):
            p, nb, r = gen(L, W["rows"][i], seed, mask, mode)
            path = os.path.join(td, f"in{i}.bed")
            with open(path, "wb") as f:
                f.write(memoryview((ctypes.c_char * nb).from_address(p.value)))
            L.bedgen_free(p)
            paths.append(path)
            nrows += r
        with open(os.path.join(td, "out.bed"), "wb") as fo:
            t0 = time.perf_counter()
            subprocess.run([exe, *W["cpu_args"], *paths], stdout=fo, check=True)
            dt = time.perf_counter() - t0
    return {"value": nrows / dt, "unit": "intervals/s", "cores": 1, "kind": "port",
            "sample": f"{W['oracle']} {' '.join(W['cpu_args'])} on contigs chr1..{last} (strcmp "
                      f"order) of the same inputs: {nrows} rows, file->file, {dt:.2f} s, 1 thread"}


# ----------------------------------------------------------------------------- workloads
# BASELINE.json configs on the GPU path. "intersect" (configs[1]) is the headline metric
# and the default; the others are measured with --workload for DESIGN.md.
# gen: (seed, 3 = BED3 | 5 = BED5) per input; rows: per input at N = 1.
WORKLOADS = {
    "intersect": {"gen": [(42, 3), (43, 3)], "rows": [100_000_000, 100_000_000],
                  "kinds": [3, 3], "oracle": "bedops_oracle", "cpu_args": ["-i"],
                  "cpu_rate": 8.5e6, "ref": REF_INTERSECT,
                  "desc": "bedops --intersect A.bed B.bed: BED3 text in HBM -> parse -> merge -> "
                          "intersect -> BED text in HBM"},
    "element-of": {"gen": [(44, 3), (45, 3)], "rows": [200_000_000, 200_000_000],
                   "kinds": [1, 3], "oracle": "bedops_oracle", "cpu_args": ["-e", "1"],
                   "cpu_rate": 3e6, "ref": None,
                   "desc": "bedops --element-of 1 A.bed B.bed (configs[3] shape, 200M x 200M)"},
    "bedmap": {"gen": [(7, 3), (8, 5)], "rows": [50_000_000, 500_000_000], "kinds": [0, 2],
               "oracle": "bedmap_oracle", "cpu_args": ["--count", "--mean"], "cpu_rate": 2e6,
               "ref": None, "desc": "bedmap --count --mean ref.bed map.bed (configs[2], 50M x 500M "
                                    "BED5 map)"},
    "closest": {"gen": [(46, 3), (47, 3)], "rows": [10_000_000, 1_000_000_000], "kinds": [1, 1],
                "oracle": "closest_oracle", "cpu_args": ["--closest"], "cpu_rate": 4e6,
                "ref": None, "desc": "closest-features --closest query.bed ref.bed (configs[4], "
                                     "10M x 1B)"},
}


def run_op(eng, name, s):
    if name == "intersect":
        return eng.op("-i", s, [0, 1])
    if name == "element-of":
        return eng.op("-e", s, [0, 1], "1")
    if name == "bedmap":
        return eng.map_op(s, ["count", "mean"], 0, 1)
    return eng.closest_op(s, 0, 1, shortest=True)


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="intersect")
    ap.add_argument("--scale", type=float, default=1.0,
                    help="rows per input per GPU = scale x the workload's size (tests/smoke)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--load-only", action="store_true",
                    help="time the loader stage alone (text in HBM -> keyed columns)")
    ap.add_argument("--profile-all", action="store_true",
                    help="time every kernel during the timed steps (default: only the dominant one)")
    args = ap.parse_args()
    W = WORKLOADS[args.workload]

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # a first collective over every rank initialises the RCCL communicator, so the
        # later batched point-to-point transfers may involve only a subset of the ranks
        dist.barrier(device_ids=[local])
    dev = torch.device("cuda", local)

    from bedops_amd import Engine

    L = bedgen_lib()
    owner, _ = contig_shards(L, world)
    mask = sum(1 << c for c, r in owner.items() if r == rank)
    per_gpu = [int(r * args.scale) for r in W["rows"]]
    t0 = time.perf_counter()
    bufs, texts, rows = [], [], []
    for (seed, mode), n in zip(W["gen"], per_gpu):
        p, nb, r = gen(L, n * world, seed, mask, mode)
        bufs.append(to_device(torch, L, p, nb, dev))
        L.bedgen_free(p)
        texts.append(nb)
        rows.append(r)
    log(f"[rank {rank}] {args.workload}: generated {rows} rows / {texts} bytes in "
        f"{time.perf_counter() - t0:.1f}s")
    torch.cuda.synchronize(dev)

    eng = Engine(local)
    ncontigs = L.bedgen_ncontigs()
    state = {}
    inputs = [((t.data_ptr(), nb), k) for t, nb, k in zip(bufs, texts, W["kinds"])]

    def step():
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
            gather_to_rank0(r, s, nbytes)
        if "keep" in state:
            state["text"] = r.text()
            del state["keep"]
        r.free()
        s.free()

    contig_names = [L.bedgen_contig_name(c).decode() for c in range(ncontigs)]
    chrom_owner = {contig_names[c]: owner[c] for c in range(ncontigs)}

    size_pg = dist.new_group(backend="gloo") if world > 1 else None

    def gather_to_rank0(r, s, nbytes):
        # the path's one exchange: per-chromosome text -> rank 0 over RCCL, in strcmp order.
        # Pipelined: this batch's transfers are posted and run on RCCL's stream while the
        # next batch is computed; the previous batch's are waited for here.
        from bedops_amd.shard import gather_text_async
        names = s.chroms()
        sp = r.chrom_spans(len(names))
        spans = {nm: (sp[g], sp[g + 1]) for g, nm in enumerate(names) if sp[g + 1] > sp[g]}
        buf = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        r.copy_to_device(buf.data_ptr(), max(nbytes, 1))
        pend = gather_text_async(dist, buf, spans, contig_names, chrom_owner, rank, world, size_pg)
        drain()
        state["pending"] = pend

    def drain():
        p = state.pop("pending", None)
        if p is not None:
            out = p.wait()
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
    comps = 0
    if args.workload == "intersect":  # component counts size the merge/intersect kernels
        s = eng.load(inputs)
        for f in (0, 1):
            m = eng.op("-m", s, [f])
            comps += m.rows()
            m.free()
        s.free()
    eng.prof_enable("*" if args.profile_all else dominant)
    drain()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()  # the last batch's transfers are inside the timed region
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
        rows_all = torch.tensor([sum(rows)], dtype=torch.int64, device=dev)
        dist.all_reduce(rows_all)
        total_rows = int(rows_all.item())
    else:
        total_rows = sum(rows)
    prof = eng.prof_read()

    if rank != 0:
        eng.close()
        dist.destroy_process_group()
        return

    # roofline of the dominant kernel, from its launches inside the timed region
    sizes = {"texts": texts, "rows": rows, "kinds": W["kinds"], "out": state["out_rows"],
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
        if os.path.exists(pmc) and args.workload == "intersect":
            try:
                traffic = json.load(open(pmc)).get(PMC_NAME.get(pick, pick), {}).get("bytes")
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": pick,
                "avg_ms": round(avg_s * 1e3, 4), "launches": calls,
                "bytes_per_launch": int(per_launch)}

    verify = None
    if world == 1 and not args.no_verify and not args.load_only and args.scale == 1.0:
        state["keep"] = True
        step()
        txt = state.pop("text")
        verify = {"rows": txt.count(b"\n"), "bytes": len(txt),
                  "sha16": hashlib.sha256(txt).hexdigest()[:16]}
        if W["ref"]:
            verify["matches_reference"] = all(verify[k] == W["ref"][k] for k in W["ref"])
        del txt

    cpu = None
    if world == 1 and not args.no_cpu_baseline and rank == 0:
        cpu = cpu_baseline(L, W)

    ms_per_step = elapsed / args.steps * 1e3
    value = total_rows * args.steps / elapsed
    line = {
        "metric": METRIC if args.workload == "intersect" else
        f"intervals/sec, {W['desc'].split(' (')[0]}",
        "value": round(value, 1), "unit": "intervals/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (SURVEY.md App. D generator, seeds "
                f"{'/'.join(str(g[0]) for g in W['gen'])}; BED text resident in HBM)",
        "config": {"workload": W["desc"] + (" (loader only)" if args.load_only else ""),
                   "rows_per_input": [r * world for r in per_gpu],
                   "rows_per_gpu_per_input": per_gpu,
                   "parallelism": "single GPU" if world == 1 else
                   f"{world} GPUs, chromosome shards (LPT) + RCCL gather to rank 0",
                   "output_rows": state["out_rows"] if world == 1 else None},
        "roofline": roof, "cpu_baseline": cpu,
        "gpu_vs_cpu": round(value / cpu["value"], 1) if cpu else None,
        "parity": verify,
        "kernels_first_step_ms": {k: round(v[1], 4) for k, v in
                                  sorted(first.items(), key=lambda kv: -kv[1][1])},
    }
    if args.profile_all:  # HIP-event time per timed step of every kernel
        line["kernels_ms_per_step"] = {k: round(v[1] / args.steps, 4) for k, v in
                                       sorted(prof.items(), key=lambda kv: -kv[1][1])}
    print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
