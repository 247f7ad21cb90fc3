"""Per-chromosome sharding plan + rank-0 reassembly model, world size 2 and 3 on CPU with gloo.

Each rank reads the inputs, builds the plan (bedops_amd.shard.assign), runs the oracle on its
own chromosomes only, and describes its output over the global chromosome list with
shard.member_spans — the bookkeeping bg_group_gather does in C (bedops_amd/csrc/
bg_group.hip). The plans are exchanged and must be identical on every rank; rank 0
reassembles with shard.reassemble and must equal the single-run output: the reference's
documented per-chromosome scale-out property. The same path on the GPU
(C sharding in the front-ends, the engine's Group.gather) is tests/test_gpu_shard.py.
"""
import os
import random
import socket
import subprocess
import tempfile

import pytest

import randbed

CHROMS = ["chr1", "chr10", "chr11", "chr2", "chr20", "chr3", "chrM", "chrX", "chrY"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _names_of(text):
    out = []
    for ln in text.splitlines():
        c = ln.split(b"\t", 1)[0].decode()
        if not out or out[-1] != c:
            out.append(c)
    return out


def _offsets(text, names):
    """bg_result_chrom_spans of a formatted text: first byte of each chromosome + total"""
    offs, pos, seen = [], 0, {}
    for ln in text.splitlines(keepends=True):
        c = ln.split(b"\t", 1)[0].decode()
        if c not in seen:
            seen[c] = pos
        pos += len(ln)
    for c in names:
        offs.append(seen.get(c, pos))
    return offs + [pos]


def _worker(rank, world, port, files, mode, exe, outdir):
    import torch.distributed as dist
    from bedops_amd.shard import assign, member_spans, reassemble, strcmp_order

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        texts = [open(f, "rb").read() for f in files]
        weights = {}
        for t in texts:  # bytes per chromosome over all inputs (the C front-ends' weight)
            for line in t.splitlines(keepends=True):
                c = line.split(b"\t", 1)[0].decode()
                weights[c] = weights.get(c, 0) + len(line)
        owner, _ = assign(weights, world)
        plans = [None] * world
        dist.all_gather_object(plans, sorted(owner.items()))
        assert all(p == plans[0] for p in plans), "ranks disagree on the shard plan"
        mine = []
        for i, t in enumerate(texts):  # this rank's chromosomes only (no input exchange)
            keep = b"".join(ln for ln in t.splitlines(keepends=True)
                            if owner[ln.split(b"\t", 1)[0].decode()] == rank)
            p = os.path.join(outdir, f"in{rank}_{i}.bed")
            open(p, "wb").write(keep)
            mine.append(p)
        out = subprocess.run([exe, *mode, *mine], capture_output=True, check=True).stdout
        global_names = strcmp_order(weights)
        local = _names_of(out)
        offs, lens = member_spans(local, _offsets(out, local), global_names)
        pieces = [None] * world
        dist.all_gather_object(pieces, (out, offs, lens))
        if rank == 0:
            got = reassemble(pieces, global_names, owner)
            open(os.path.join(outdir, "gathered.bed"), "wb").write(got)
    finally:
        dist.destroy_process_group()


def _run(world, mode, nfiles, seed, oracle_bin):
    import torch.multiprocessing as mp

    rng = random.Random(seed)
    with tempfile.TemporaryDirectory() as td:
        files = []
        for f in range(nfiles):
            rows = randbed.rows(rng, rng.choice([50, 400, 1500]), chroms=CHROMS, span=3000,
                                maxlen=rng.choice([20, 150]))
            p = os.path.join(td, f"f{f}.bed")
            randbed.write(p, randbed.text(rows, rest="cols" if f == 0 else None, rng=rng))
            files.append(p)
        exe = oracle_bin["bedops"]
        want = subprocess.run([exe, *mode, *files], capture_output=True, check=True).stdout
        mp.start_processes(_worker, args=(world, _free_port(), files, mode, exe, td), nprocs=world,
                           join=True, start_method="spawn")
        got = open(os.path.join(td, "gathered.bed"), "rb").read()
    return want, got


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", [["-i"], ["-m"], ["-d"], ["-e", "1"], ["-n", "50%"]])
def test_sharded_reassembly_equals_single_run(oracle_bin, world, mode):
    want, got = _run(world, mode, 2 if mode != ["-m"] else 3, hash((world, tuple(mode))) & 0xffff,
                     oracle_bin)
    assert got == want


def test_assign_is_lpt_and_deterministic():
    from bedops_amd.shard import assign
    w = {"chr1": 249, "chr2": 242, "chr3": 198, "chrX": 156, "chrM": 1, "chr21": 46}
    owner, load = assign(w, 3)
    assert owner == assign(dict(reversed(list(w.items()))), 3)[0]
    assert sorted(load) == sorted([249 + 46, 242 + 1, 198 + 156]) or max(load) <= 249 + 156
    assert set(owner.values()) == {0, 1, 2}


def test_member_spans_rejects_unsorted_global_list():
    from bedops_amd.shard import member_spans
    with pytest.raises(ValueError):
        member_spans(["chr1"], [0, 5], ["chr2", "chr1"])
