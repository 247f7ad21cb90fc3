"""Per-chromosome sharding + rank-0 reassembly (bedops_amd/shard.py), world size 2 and 3 on
CPU with gloo. Each rank computes its chromosomes' output with the oracle (the GPU engine
is exercised by bench.py on the box; the shard logic is the same code), the texts are
gathered with bedops_amd.shard.gather_text, and rank 0's bytes must equal the single-run
output — the reference's documented per-chromosome scale-out property
(SURVEY.md §8(e))."""
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


def _worker(rank, world, port, files, mode, exe, outdir, pipelined=False):
    import torch
    import torch.distributed as dist
    from bedops_amd.shard import assign, gather_text, gather_text_async, spans_from_text

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        weights = {c: 0 for c in CHROMS}
        texts = [open(f, "rb").read() for f in files]
        for t in texts:
            for line in t.splitlines():
                weights[line.split(b"\t", 1)[0].decode()] += 1
        owner, _ = assign(weights, world)
        mine = []
        for i, t in enumerate(texts):  # this rank's chromosomes only
            keep = b"".join(ln + b"\n" for ln in t.splitlines()
                            if owner[ln.split(b"\t", 1)[0].decode()] == rank)
            p = os.path.join(outdir, f"in{rank}_{i}.bed")
            open(p, "wb").write(keep)
            mine.append(p)
        out = subprocess.run([exe, *mode, *mine], capture_output=True, check=True).stdout
        spans = spans_from_text(out)
        buf = torch.frombuffer(bytearray(out), dtype=torch.uint8) if out else \
            torch.empty(0, dtype=torch.uint8)
        if pipelined:  # two batches in flight before either is waited for (bench.py's loop)
            sg = dist.new_group(backend="gloo")
            p1 = gather_text_async(dist, buf, spans, CHROMS, owner, rank, world, sg)
            p2 = gather_text_async(dist, buf.clone(), spans, CHROMS, owner, rank, world, sg)
            got, got2 = p1.wait(), p2.wait()
            if rank == 0:
                assert bytes(got.numpy()) == bytes(got2.numpy())
        else:
            got = gather_text(dist, buf, spans, CHROMS, owner, rank, world)
        if rank == 0:
            open(os.path.join(outdir, "gathered.bed"), "wb").write(bytes(got.numpy()))
    finally:
        dist.destroy_process_group()


def _run(world, files, mode, exe, outdir, pipelined=False):
    import torch.multiprocessing as mp
    mp.start_processes(_worker, args=(world, _free_port(), files, mode, exe, outdir, pipelined),
                       nprocs=world, start_method="spawn", join=True)
    return open(os.path.join(outdir, "gathered.bed"), "rb").read()


def test_assign_is_lpt_and_deterministic():
    from bedops_amd.shard import assign
    w = {"chr1": 249, "chr2": 242, "chr3": 198, "chrX": 156, "chrM": 0, "chr10": 134}
    owner, load = assign(w, 2)
    assert sorted(owner) == sorted(w)
    assert sum(load) == sum(w.values())
    assert max(load) - min(load) <= max(w.values())
    assert assign(w, 2) == (owner, load)
    assert set(assign(w, 1)[0].values()) == {0}
    assert set(assign(w, 8)[0].values()) <= set(range(8))


def test_spans_from_text():
    from bedops_amd.shard import spans_from_text
    t = b"chr1\t1\t2\nchr1\t3\t4\nchr10\t1\t2\nchrX\t5\t6\n"
    assert spans_from_text(t) == {"chr1": (0, 18), "chr10": (18, 28), "chrX": (28, 37)}
    assert spans_from_text(b"") == {}


@pytest.mark.parametrize("world,mode,pipelined", [(2, ["-i"], False), (2, ["-m"], False),
                                                  (3, ["-d"], False), (2, ["-e", "1"], False),
                                                  (3, ["-n", "50%"], False), (2, ["-i"], True),
                                                  (3, ["-m"], True)])
def test_sharded_equals_single_run(oracle_bin, world, mode, pipelined):
    rng = random.Random(1000 + world)
    with tempfile.TemporaryDirectory() as td:
        files = []
        for i in range(2):
            chroms = CHROMS if i == 0 else CHROMS[:-2]  # chrX/chrY only in file 0
            p = os.path.join(td, f"f{i}.bed")
            randbed.write(p, randbed.text(randbed.rows(rng, 3000, chroms=chroms, span=20000)))
            files.append(p)
        exe = oracle_bin["bedops"]
        want = subprocess.run([exe, *mode, *files], capture_output=True, check=True).stdout
        got = _run(world, files, mode, exe, td, pipelined)
        assert got == want
