"""Multi-GPU path on one GPU: chromosome shards run as separate group members on cuda:0.

The C front-ends under BEDGPU_DEVICES=0,0[,0] split every input by chromosome (bisection),
run each shard on its own member (host thread, context, stream) and reassemble the texts
with bg_group_gather (bedops_amd/cli/cli_shard.h, bedops_amd/csrc/bg_group.hip); with a
device listed twice the members get no RCCL communicator and the transfers are device
copies — the plan, the spans and the reassembly are the code the RCCL path runs. The output
must be byte-identical to the one-device run and to the oracle. The engine-level test drives
engine.Group.gather the way bench.py does under torch.distributed.run.
"""
import os
import random
import subprocess
import sys
import tempfile
import zlib

import pytest

import randbed

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHROMS = ["chr1", "chr10", "chr11", "chr2", "chr20", "chr3", "chrM", "chrX", "chrY"]
MODES = [["-m"], ["-i"], ["-d"], ["-e", "1"], ["-n", "30%"], ["-c"], ["-c", "-L"], ["-w", "7"],
         ["-s"], ["-p"], ["-u"]]


def _cli(exe, args, env_devices):
    env = dict(os.environ)
    env.pop("BEDGPU_DEVICES", None)
    if env_devices:
        env["BEDGPU_DEVICES"] = env_devices
    return subprocess.run([exe, *args], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env,
                          timeout=120)


@pytest.mark.parametrize("mode", MODES)
def test_cli_sharded_equals_single_device(gpu_bin, oracle_bin, mode):
    rng = random.Random(zlib.crc32(repr(mode).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(4):
            files = []
            for f in range(3 if mode[0] in ("-m", "-i", "-u") else 2):
                rows = randbed.rows(rng, rng.choice([1, 40, 600, 3000]),
                                    chroms=rng.sample(CHROMS, rng.choice([1, 4, 9])),
                                    span=rng.choice([500, 5000]), maxlen=rng.choice([10, 120]),
                                    zero_frac=0.05 if mode[0] in ("-i", "-d", "-e", "-n") else 0.0)
                p = os.path.join(td, f"f{trial}_{f}.bed")
                randbed.write(p, randbed.text(rows, rest="cols" if f == 0 else None, rng=rng))
                files.append(p)
            one = _cli(gpu_bin["bedops"], mode + files, None)
            assert one.returncode == 0, one.stderr
            want = subprocess.run([oracle_bin["bedops"], *mode, *files], stdout=subprocess.PIPE,
                                  check=True).stdout
            assert one.stdout == want
            for devs in ("0,0", "0,0,0"):
                got = _cli(gpu_bin["bedops"], mode + files, devs)
                assert got.returncode == 0, got.stderr
                assert got.stdout == want, (mode, trial, devs)


def test_cli_sharded_errors_match_single_device(gpu_bin, tmp_path):
    """an error inside a shard falls back to the one-device run: same message, same line"""
    a = tmp_path / "a.bed"
    b = tmp_path / "b.bed"
    a.write_text("chr1\t1\t5\nchr2\t3\t9\nchr2\t4\tx\nchr3\t1\t2\n")
    b.write_text("chr1\t2\t8\nchr3\t0\t9\n")
    one = _cli(gpu_bin["bedops"], ["-i", str(a), str(b)], None)
    two = _cli(gpu_bin["bedops"], ["-i", str(a), str(b)], "0,0")
    assert one.returncode != 0
    assert (two.returncode, two.stderr, two.stdout) == (one.returncode, one.stderr, one.stdout)


def test_cli_sharded_stdin_and_missing_devices_fall_back(gpu_bin, oracle_bin, tmp_path):
    """BEDGPU_DEVICES naming more GPUs than exist (the group cannot open), or a stdin input
    (not a mappable file), take the one-device path with the same output; stdin is not
    consumed by the declined shard attempt"""
    import torch
    rng = random.Random(9)
    a = randbed.write(str(tmp_path / "a.bed"), randbed.text(randbed.rows(rng, 4000, chroms=CHROMS)))
    b = randbed.write(str(tmp_path / "b.bed"), randbed.text(randbed.rows(rng, 3000, chroms=CHROMS)))
    want = subprocess.run([oracle_bin["bedops"], "-i", a, b], stdout=subprocess.PIPE, check=True).stdout
    n = torch.cuda.device_count()
    got = _cli(gpu_bin["bedops"], ["-i", a, b], ",".join(str(d) for d in range(n + 1)))
    assert got.returncode == 0 and got.stdout == want, got.stderr
    env = dict(os.environ, BEDGPU_DEVICES="0,0")
    with open(a, "rb") as fi:
        got = subprocess.run([gpu_bin["bedops"], "-i", "-", b], stdin=fi, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, env=env, timeout=120)
    assert got.returncode == 0 and got.stdout == want, got.stderr
    wantm = subprocess.run([oracle_bin["bedmap"], "--count", a, b], stdout=subprocess.PIPE, check=True).stdout
    with open(a, "rb") as fi:
        got = subprocess.run([gpu_bin["bedmap"], "--count", "-", b], stdin=fi, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, env=env, timeout=120)
    assert got.returncode == 0 and got.stdout == wantm, got.stderr


# bench.py's workloads (WORKLOADS / run_op): input kinds and the step's operation
BENCH_STEPS = {
    "intersect": ([3, 3], lambda eng, s: eng.op("-i", s, [0, 1])),
    "element-of": ([1, 3], lambda eng, s: eng.op("-e", s, [0, 1], "1")),
    "bedmap": ([0, 2], lambda eng, s: eng.map_op(s, ["count", "mean"], 0, 1)),
    "closest": ([1, 1], lambda eng, s: eng.closest_op(s, 0, 1, shortest=True)),
}


def _bench_texts(rng, workload):
    a = randbed.rows(rng, 3000, chroms=CHROMS, span=20000, maxlen=90)
    b = randbed.rows(rng, 6000 if workload != "closest" else 12000, chroms=CHROMS, span=20000, maxlen=90)
    if workload == "bedmap":  # BED5 map rows, integer scores (configs[2])
        mt = "".join(f"{c}\t{st}\t{e}\tid{i}\t{rng.randint(0, 999)}\n" for i, (c, st, e) in enumerate(b))
        return [randbed.text(a).encode(), mt.encode()]
    return [randbed.text(a).encode(), randbed.text(b).encode()]


def _step_text(eng, workload, texts):
    kinds, op = BENCH_STEPS[workload]
    s = eng.load([(t, k) for t, k in zip(texts, kinds)])
    r = op(eng, s)
    r.format()
    return s, r


@pytest.mark.parametrize("workload", sorted(BENCH_STEPS))
def test_engine_group_gather_equals_single_run(workload):
    """bench.py's multi-rank step on one GPU, for every workload it times: each member loads
    only its chromosomes (LPT owner), runs the workload's operation, formats in HBM;
    Group.gather reassembles on member 0 (member_spans in strcmp order) — byte-identical to the
    one-engine run of the same step (which the reference-fixture and full-size tests pin)"""
    from bedops_amd import Engine
    from bedops_amd.engine import Group
    from bedops_amd.shard import assign, member_spans, strcmp_order

    rng = random.Random(zlib.crc32(workload.encode()))
    texts = _bench_texts(rng, workload)
    e1 = Engine(0)
    try:
        s1, r1 = _step_text(e1, workload, texts)
        want = r1.text()
        r1.free()
        s1.free()
    finally:
        e1.close()
    weights = {}
    for t in texts:
        for ln in t.splitlines(keepends=True):
            c = ln.split(b"\t", 1)[0].decode()
            weights[c] = weights.get(c, 0) + len(ln)
    gnames = strcmp_order(weights)
    for world in (2, 3):
        owner, _ = assign(weights, world)
        g = Group(devices=[0] * world)
        try:
            parts, keep = [], []
            for m, eng in enumerate(g.engines):
                shard = [b"".join(ln for ln in t.splitlines(keepends=True)
                                  if owner[ln.split(b"\t", 1)[0].decode()] == m) for t in texts]
                s, r = _step_text(eng, workload, shard)
                dptr, _ = r.device_text()
                names = s.chroms()
                offs, lens = member_spans(names, r.chrom_spans(len(names)), gnames)
                parts.append((dptr, offs, lens))
                keep.append((s, r))
            out, n = g.gather(len(gnames), parts)
            with tempfile.TemporaryFile() as fo:  # member 0 streams its buffer to a file
                g.engines[0].write_device(out, n, fo.fileno())
                fo.seek(0)
                got = fo.read()
            g.engines[0].device_free(out)
            for s, r in keep:
                r.free()
                s.free()
        finally:
            g.close()
        assert got == want, (workload, world)


def test_engine_group_intersect_matches_oracle(oracle_bin):
    """the gathered intersect (bench.py's headline step) against the oracle itself"""
    from bedops_amd.engine import Group
    from bedops_amd.shard import assign, member_spans, strcmp_order

    rng = random.Random(5)
    texts = [randbed.text(randbed.rows(rng, 4000, chroms=CHROMS, span=20000, maxlen=90)).encode()
             for _ in range(2)]
    weights = {}
    for t in texts:
        for ln in t.splitlines(keepends=True):
            c = ln.split(b"\t", 1)[0].decode()
            weights[c] = weights.get(c, 0) + len(ln)
    gnames = strcmp_order(weights)
    owner, _ = assign(weights, 3)
    g = Group(devices=[0] * 3)
    try:
        parts, keep = [], []
        for m, eng in enumerate(g.engines):
            shard = [b"".join(ln for ln in t.splitlines(keepends=True)
                              if owner[ln.split(b"\t", 1)[0].decode()] == m) for t in texts]
            s, r = _step_text(eng, "intersect", shard)
            dptr, _ = r.device_text()
            names = s.chroms()
            offs, lens = member_spans(names, r.chrom_spans(len(names)), gnames)
            parts.append((dptr, offs, lens))
            keep.append((s, r))
        out, n = g.gather(len(gnames), parts)
        with tempfile.TemporaryFile() as fo:
            g.engines[0].write_device(out, n, fo.fileno())
            fo.seek(0)
            got = fo.read()
        g.engines[0].device_free(out)
        for s, r in keep:
            r.free()
            s.free()
    finally:
        g.close()
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for i, t in enumerate(texts):
            p = os.path.join(td, f"{i}.bed")
            open(p, "wb").write(t)
            paths.append(p)
        want = subprocess.run([oracle_bin["bedops"], "-i", *paths], stdout=subprocess.PIPE, check=True).stdout
    assert got == want


MAP_CASES = [
    ["--count", "--mean", "--sum", "--max"],
    ["--echo", "--echo-map-id", "--bases", "--median"],
    ["--bp-ovr", "5", "--echo-map-score", "--indicator"],
    ["--fraction-both", "0.3", "--stdev", "--echo-map-range"],
    ["--range", "20", "--kth", "0.25", "--tmean", "0.1", "0.2"],
    ["--skip-unmapped", "--min-element", "--max-element"],
    ["--exact", "--count", "--echo-map"],
]


@pytest.mark.parametrize("case", MAP_CASES, ids=lambda c: "_".join(x.strip("-") for x in c))
@pytest.mark.parametrize("decimal", [False, True], ids=["int", "decimal"])
def test_bedmap_sharded_equals_single_device(gpu_bin, oracle_bin, case, decimal):
    """bedmap windows never cross chromosomes; decimal running sums span the whole file
    (the reference's double accumulators), so such a request falls back to one device"""
    rng = random.Random(zlib.crc32(repr((case, decimal)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(3):
            ref = randbed.rows(rng, rng.choice([1, 300, 2000]),
                               chroms=rng.sample(CHROMS, rng.choice([1, 4, 9])), span=4000,
                               maxlen=rng.choice([10, 120]))
            mp = randbed.rows(rng, rng.choice([1, 500, 3000]),
                              chroms=rng.sample(CHROMS, rng.choice([1, 4, 9])), span=4000,
                              maxlen=rng.choice([10, 120]))
            pr = randbed.write(os.path.join(td, f"r{trial}.bed"),
                               randbed.text(ref, rest="cols", rng=rng))
            mtext = randbed.text(mp, rest="bed5", rng=rng)
            if decimal:
                mtext = "".join(ln.rsplit("\t", 1)[0] + f"\t{rng.randint(-999, 999) / 8}\n"
                                for ln in mtext.splitlines())
            pm = randbed.write(os.path.join(td, f"m{trial}.bed"), mtext)
            for files in ([pr, pm], [pm]):   # two files, and single-file mode
                want = subprocess.run([oracle_bin["bedmap"], *case, *files],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE)
                for devs in (None, "0,0", "0,0,0"):
                    got = _cli(gpu_bin["bedmap"], case + files, devs)
                    assert (got.returncode == 0) == (want.returncode == 0), (got.stderr, devs)
                    assert got.stdout == want.stdout, (case, trial, files, devs)


CLOSEST_CASES = [[], ["--closest"], ["--dist"], ["--closest", "--dist", "--no-overlaps"],
                 ["--no-ref", "--dist"], ["--delim", "|", "--closest", "--no-overlaps"]]


@pytest.mark.parametrize("case", CLOSEST_CASES, ids=lambda c: "_".join(x.strip("-|") for x in c) or "plain")
def test_closest_sharded_equals_single_device(gpu_bin, oracle_bin, case):
    """findDistances drops earlier-chromosome candidates and stops at a later chromosome,
    so each chromosome's lines depend on that chromosome alone"""
    rng = random.Random(zlib.crc32(repr(case).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(4):
            files = []
            for f in range(2):
                rows = randbed.rows(rng, rng.choice([1, 200, 2500]),
                                    chroms=rng.sample(CHROMS, rng.choice([1, 4, 9])),
                                    span=rng.choice([3000, 30000]), maxlen=rng.choice([10, 120]),
                                    zero_frac=0.03)
                p = os.path.join(td, f"c{trial}_{f}.bed")
                randbed.write(p, randbed.text(rows, rest="cols" if f == 0 else "bed5", rng=rng))
                files.append(p)
            want = subprocess.run([oracle_bin["closest"], *case, *files], stdout=subprocess.PIPE,
                                  check=True).stdout
            for devs in (None, "0,0", "0,0,0"):
                got = _cli(gpu_bin["closest"], case + files, devs)
                assert got.returncode == 0, got.stderr
                assert got.stdout == want, (case, trial, devs)


_RCCL_SELF_CHILD = r"""
import os, random, sys, tempfile
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import randbed
from bedops_amd.engine import BED3_SET, Group
from bedops_amd.shard import member_spans, strcmp_order
chroms = sys.argv[3].split(",")
rng = random.Random(9)
texts = [randbed.text(randbed.rows(rng, 5000, chroms=chroms, span=30000, maxlen=90)).encode() for _ in range(2)]
gnames = strcmp_order({ln.split(b"\t", 1)[0].decode(): 1 for t in texts for ln in t.splitlines()})
single = sys.argv[2] == "1"
g = Group(devices=[0]) if single else Group(device=0, uid=bytes(128), nranks=1, rank=0)
try:
    eng = g.engines[0]
    s = eng.load([(x, BED3_SET) for x in texts])
    r = eng.op("-i", s, [0, 1])
    r.format()
    dptr, _ = r.device_text()
    names = s.chroms()
    offs, lens = member_spans(names, r.chrom_spans(len(names)), gnames)
    out, n = g.gather(len(gnames), [(dptr, offs, lens)])
    eng.write_device(out, n, 1)
    eng.device_free(out)
    r.free()
    s.free()
finally:
    g.close()
with open(sys.argv[4], "wb") as f:
    for t in texts:
        f.write(t + b"\0")
"""


def test_group_gather_through_rccl_self_communicator(oracle_bin, tmp_path):
    """BEDGPU_RCCL_SELF=1: a one-member group gets a one-rank RCCL communicator and sends its
    own chromosome runs to itself (ncclAllReduce of the sizes, grouped ncclSend/ncclRecv), so
    bg_group_gather's communicator branch runs on this one-GPU box; the reassembled text must
    equal a single run. Each case runs in a child process that loads only the library (as the
    C front-ends do): a process that has also loaded torch's own HIP runtime gives RCCL a
    second one"""
    env = dict(os.environ, BEDGPU_RCCL_SELF="1")
    env.pop("NCCL_DEBUG", None)  # (RCCL prints its log on stdout, where the text goes)
    for single in ("1", "0"):
        inputs = tmp_path / f"inputs{single}.bin"
        r = subprocess.run([sys.executable, "-c", _RCCL_SELF_CHILD, ROOT, single, ",".join(CHROMS), str(inputs)],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=240)
        assert r.returncode == 0, (single, r.stderr.decode(errors="replace")[-3000:])
        got = r.stdout
        texts = inputs.read_bytes().split(b"\0")[:2]
        paths = []
        for i, t in enumerate(texts):
            p = tmp_path / f"in{single}_{i}.bed"
            p.write_bytes(t)
            paths.append(str(p))
        want = subprocess.run([oracle_bin["bedops"], "-i", *paths], stdout=subprocess.PIPE, check=True).stdout
        assert got == want, single


def test_sharded_cli_writes_each_device_part_at_its_offset(gpu_bin, oracle_bin, tmp_path):
    """stdout a regular file: every shard writes its chromosomes' spans straight to their
    offsets (bg_pwrite_device), no gather; a pipe keeps the gather. Both equal the oracle,
    also after bytes already in the file (the output starts at the file position)"""
    rng = random.Random(13)
    a = str(tmp_path / "a.bed")
    b = str(tmp_path / "b.bed")
    open(a, "w").write(randbed.text(randbed.rows(rng, 20000, chroms=CHROMS, span=200000, maxlen=90)))
    open(b, "w").write(randbed.text(randbed.rows(rng, 20000, chroms=CHROMS, span=200000, maxlen=90)))
    want = subprocess.run([oracle_bin["bedops"], "-i", a, b], stdout=subprocess.PIPE, check=True).stdout
    env = dict(os.environ, BEDGPU_DEVICES="0,0,0", BEDGPU_STATS="1")
    out = str(tmp_path / "out.bed")
    with open(out, "wb") as fo:
        fo.write(b"head\n")
        fo.flush()
        r = subprocess.run([gpu_bin["bedops"], "-i", a, b], stdout=fo, stderr=subprocess.PIPE, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    assert open(out, "rb").read() == b"head\n" + want
    assert b"shards" in r.stderr  # the sharded path ran (cli_mark)
    r = subprocess.run([gpu_bin["bedops"], "-i", a, b], stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env,
                       timeout=120)
    assert r.returncode == 0 and r.stdout == want, r.stderr


def test_bench_multi_rank_placement_step_on_one_gpu():
    """bench.py --gpus 2 (two rank processes, gloo coordination) with both ranks on cuda:0:
    the N > 1 placement step (per-chromosome byte counts exchanged, text left in each rank's
    HBM) runs and reports one line for 2 GPUs; the RCCL gather needs distinct devices"""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--scale", "0.002", "--steps", "2", "--warmup", "1", "--no-e2e",
                        "--no-cpu-baseline"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert "byte-count exchange" in line["config"]["parallelism"]
