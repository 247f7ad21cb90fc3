"""The product's host heap replay (bedops_amd/csrc/bg_heap_replay.h, run by bg_heap_addr before
bedmap orders equal rows by address) against the oracle's model (oracle/bedmap_oracle.c +
oracle/heapsim.h, itself pinned to the reference's output by tests/test_ref_fixtures.py): the
simulated address of every map row must agree, on every bedmap fixture's inputs and options
and on random inputs with duplicate rows and remainders in the row objects' chunk sizes.
CPU only: tools/build/heap_replay_check runs the same replay code on the host."""
import os
import random
import subprocess
import tempfile

import pytest

import randbed
import ref_fixtures as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = os.path.join(ROOT, "tools", "build", "heap_replay_check")


@pytest.fixture(scope="module")
def check_bin():
    subprocess.run(["make", "-s", "tools/build/heap_replay_check"], cwd=ROOT, check=True)
    return CHECK


def _addrs(argv):
    r = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)
    assert r.returncode == 0, (argv, r.stderr[:300])
    return r.stdout


def _same(check_bin, oracle_bin, args, paths):
    """None: the oracle stopped early (an element operation on an empty window)"""
    with tempfile.NamedTemporaryFile() as f:
        r = subprocess.run([oracle_bin["bedmap"], "--dump-addr", f.name] + args + paths, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL, timeout=120)
        if r.returncode != 0:
            return None
        want = open(f.name, "rb").read()
    got = _addrs([check_bin] + args + paths)
    return got == want


@pytest.mark.parametrize("suite", ["bedmap", "decimal", "faster"])
def test_replay_matches_oracle_on_fixture_inputs(check_bin, oracle_bin, suite):
    fx = R.load(suite)
    bad, n = [], 0
    with tempfile.TemporaryDirectory() as td:
        for k, c in enumerate(fx["cases"]):
            if c["tool"] != "bedmap" or c["rc"] != 0 or c.get("stdin") is not None:
                continue
            if any(a in c["args"] for a in ("--ec", "--header", "--chrom")):
                continue
            paths = []
            for i in c["files"]:
                p = os.path.join(td, f"g{c['group']}_{i}.bed")
                if not os.path.exists(p):
                    with open(p, "w") as f:
                        f.write(fx["groups"][c["group"]][i])
                paths.append(p)
            n += 1
            if _same(check_bin, oracle_bin, c["args"], paths) is False:
                bad.append((k, c["args"]))
    assert n > 20
    assert not bad, bad[:5]


OPS = ["--echo-map", "--echo-map-size", "--echo-overlap-size", "--echo-map-range", "--bases", "--bases-uniq",
       "--bases-uniq-f", "--count", "--echo", "--echo-map-id", "--echo-map-score", "--min-element", "--wmean"]
CRITS = [[], ["--range", "30"], ["--fraction-map", "0.5"], ["--fraction-ref", "0.3"], ["--bp-ovr", "5"],
         ["--exact"], ["--fraction-either", "0.4"], ["--fraction-both", "0.2"]]


def _rest(rng, i):
    k = rng.choice([0, 3, 20, 30, 36, 45, 52])
    return "" if k == 0 else "\t" + ("x" * k)[:max(0, k - len(str(i)))] + str(i)


@pytest.mark.parametrize("seed", range(6))
def test_replay_matches_oracle_on_random_duplicates(check_bin, oracle_bin, seed):
    """duplicate rows (equal coordinates, equal or different remainders), remainders whose
    strings fall in the row objects' chunk sizes, all three map row types, both sweeps"""
    rng = random.Random(7000 + seed)
    ref = randbed.rows(rng, rng.choice([60, 200]), span=3000, maxlen=rng.choice([30, 120]))
    mp = randbed.rows(rng, rng.choice([200, 500]), span=3000, maxlen=rng.choice([20, 80]))
    mp = sorted(mp + ref[::2] + ref[::3] + mp[::4], key=lambda r: (r[0].encode(), r[1], r[2]))
    bad = []
    with tempfile.TemporaryDirectory() as td:
        rp, mpth = os.path.join(td, "r.bed"), os.path.join(td, "m.bed")
        with open(rp, "w") as f:
            f.write("".join(f"{c}\t{s}\t{e}{_rest(rng, i)}\n" for i, (c, s, e) in enumerate(ref)))
        with open(mpth, "w") as f:
            f.write("".join(f"{c}\t{s}\t{e}\tid{i % 7}\t{rng.randint(0, 9)}{_rest(rng, i)}\n"
                            for i, (c, s, e) in enumerate(mp)))
        for _ in range(16):
            crit = rng.choice(CRITS)
            if rng.random() < 0.3 and crit[:1] in ([], ["--range"], ["--bp-ovr"], ["--exact"], ["--fraction-both"]):
                crit = ["--faster"] + crit
            ops = rng.sample(OPS, rng.choice([1, 2, 3]))
            files = rng.choice([[rp, mpth], [mpth]])
            if _same(check_bin, oracle_bin, crit + ops, files) is False:
                bad.append(crit + ops + [len(files)])
    assert not bad, bad[:5]
