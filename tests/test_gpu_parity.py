"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's own known-answer tests. Bit-exact byte comparison everywhere."""
import hashlib
import os
import random
import subprocess
import tempfile
import zlib

import pytest

import randbed
import testplan_runner

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from bedops_amd import Engine
    e = Engine(0)
    yield e
    e.close()


def run_oracle(binary, args, texts, tmpdir):
    paths = []
    for i, t in enumerate(texts):
        p = os.path.join(tmpdir, f"in{i}.bed")
        with open(p, "wb") as f:
            f.write(t if isinstance(t, bytes) else t.encode())
        paths.append(p)
    r = subprocess.run([binary] + args + paths, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       check=True)
    return r.stdout


# ---------------------------------------------------------------------------------
# reference KATs (applications/bed/bedops/test/TestPlan.xml) through the C front-end
# ---------------------------------------------------------------------------------
def test_testplan_kats_gpu_cli(gpu_bin, tmp_path):
    """all 63 KATs: every operation, --range, --chrom, -L, chop sub-options"""
    res = testplan_runner.run_testplan([gpu_bin["bedops"]], str(tmp_path))
    bad = [r for r in res if not r[2]]
    assert len(res) == 63
    assert not bad, bad


# ---------------------------------------------------------------------------------
# randomized differential tests against the oracle
# ---------------------------------------------------------------------------------
CASES = [("-m", 1), ("-m", 2), ("-m", 3), ("-i", 2), ("-i", 3), ("-d", 2), ("-d", 3),
         ("-e", 2), ("-n", 2), ("-e", 3)]
SPECS = {"-e": [None, "1", "3", "50%", "100%", "0%"], "-n": [None, "1", "25%"]}


@pytest.mark.parametrize("zero_frac", [0.0, 0.06])
@pytest.mark.parametrize("mode,nfiles", CASES)
def test_random_bedops_vs_oracle(eng, oracle_bin, mode, nfiles, zero_frac):
    rng = random.Random(zlib.crc32(repr((mode, nfiles, zero_frac)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(12):
            n = rng.choice([0, 1, 2, 5, 30, 200, 1500])
            texts = []
            for f in range(nfiles):
                rs = randbed.rows(rng, n if f == 0 else rng.choice([0, 3, 40, 300, 1200]),
                                  span=rng.choice([50, 400, 3000]), maxlen=rng.choice([5, 40, 150]),
                                  zero_frac=zero_frac)
                rest = "cols" if (f == 0 and mode in ("-e", "-n")) else None
                texts.append(randbed.text(rs, rest=rest, rng=rng).encode())
            for spec in SPECS.get(mode, [None]):
                args = [mode] + ([spec] if spec else [])
                want = run_oracle(oracle_bin["bedops"], args, texts, td)
                got = eng.bedops(mode, texts, spec=spec)
                assert got == want, (mode, spec, trial, n)


@pytest.mark.parametrize("nfiles", [2, 3, 4])
def test_intersect_zero_length_rows_vs_oracle(eng, oracle_bin, nfiles):
    """nextIntersectLine prints some isolated zero-length pieces ("chr t t") depending on
    its stream state (Bedops.cpp:1105-1181): the GPU replays those calls (k_zi_replay)"""
    rng = random.Random(1000 + nfiles)
    nzero = 0
    with tempfile.TemporaryDirectory() as td:
        for trial in range(40):
            texts = []
            for f in range(nfiles):
                rs = randbed.rows(rng, rng.choice([0, 1, 5, 40, 300, 3000]),
                                  span=rng.choice([40, 300, 5000]), maxlen=rng.choice([3, 12, 60]),
                                  zero_frac=rng.choice([0.05, 0.3, 0.7]))
                texts.append(randbed.text(rs).encode())
            want = run_oracle(oracle_bin["bedops"], ["-i"], texts, td)
            nzero += sum(1 for ln in want.splitlines() if ln.split(b"\t")[1] == ln.split(b"\t")[2])
            assert eng.bedops("-i", texts) == want, trial
    assert nzero > 0  # the trials did exercise the zero-length prints


def test_element_of_wide_rows_slice(eng, oracle_bin):
    """reference rows spanning more components than a workgroup stages in LDS"""
    rng = random.Random(21)
    ref = sorted([("chr1", 0, 90000), ("chr1", 5, 60000), ("chr1", 100, 101)] +
                 randbed.rows(rng, 600, chroms=["chr1"], span=100000, maxlen=50),
                 key=lambda r: (r[1], r[2]))
    other = randbed.rows(rng, 6000, chroms=["chr1"], span=100000, maxlen=8)
    rt = randbed.text(ref, rest="cols", rng=rng).encode()
    ot = randbed.text(other).encode()
    with tempfile.TemporaryDirectory() as td:
        for spec in ("1", "30%", "100%"):
            want = run_oracle(oracle_bin["bedops"], ["-e", spec], [rt, ot], td)
            assert eng.bedops("-e", [rt, ot], spec=spec) == want, spec


def _fields(t):
    for ln in t.decode().splitlines():
        f = ln.split()
        if len(f) >= 3:
            yield f[0], int(f[1]), int(f[2])


@pytest.mark.parametrize("ovr,prec,skip", [(1, 6, False), (5, 6, False), (1, 3, True), (2, 0, False)])
def test_random_bedmap_vs_oracle(eng, oracle_bin, ovr, prec, skip):
    rng = random.Random(ovr * 100 + prec)
    with tempfile.TemporaryDirectory() as td:
        for trial in range(10):
            ref = randbed.rows(rng, rng.choice([0, 1, 20, 400, 2000]), span=rng.choice([300, 3000]),
                               maxlen=rng.choice([10, 80, 300]))
            mp = randbed.rows(rng, rng.choice([0, 1, 50, 800, 4000]), span=rng.choice([300, 3000]),
                              maxlen=rng.choice([10, 80, 300]))
            rt = randbed.text(ref).encode()
            mt = randbed.text(mp, rest="bed5", rng=rng).encode()
            for ops in (["count"], ["mean"], ["count", "mean"], ["mean", "count"]):
                args = [f"--{o}" for o in ops] + ["--bp-ovr", str(ovr), "--prec", str(prec)]
                if skip:
                    args.append("--skip-unmapped")
                want = run_oracle(oracle_bin["bedmap"], args, [rt, mt], td)
                got = eng.bedmap(ops, rt, mt, overlap_bp=ovr, precision=prec, skip_unmapped=skip)
                assert got == want, (ops, trial)


# every bedmap operation on the GPU path under every overlap criterion;
# oracle = restatement of the sweep + fixWindow + visitors (oracle/bedmap_oracle.c)
MAP_OPSETS = [["count", "sum", "min", "max", "indicator"],
              ["bases", "bases-uniq", "bases-uniq-f", "mean"],
              ["echo", "echo-ref-size", "echo-ref-name", "count"],
              ["echo-map", "echo-map-id", "echo-map-size"],
              ["echo-map", "mean", "echo-map-score"],
              ["echo-overlap-size", "echo-map-range", "count"],
              ["median", "variance", "stdev", "cv", ("kth", 0.3), ("kth", 0.05)],
              ["echo-ref-row-id", "echo-map-id-uniq", "echo-ref-row-id", "count"],
              ["mad", ("mad", 1.4826), "median"]]
MAP_CRITS = [("bp-ovr", 1), ("bp-ovr", 7), ("range", 1), ("range", 25), ("fraction-ref", "0.5"),
             ("fraction-map", "0.25"), ("fraction-map", "1"), ("fraction-either", "0.7"),
             ("fraction-both", "0.3"), ("exact", None)]


@pytest.mark.parametrize("crit,val", MAP_CRITS)
def test_random_bedmap_ops_criteria_vs_oracle(eng, oracle_bin, crit, val):
    rng = random.Random(zlib.crc32(repr((crit, val)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(6):
            ref = randbed.rows(rng, rng.choice([0, 1, 30, 500, 2000]), span=rng.choice([300, 3000]),
                               maxlen=rng.choice([10, 80, 300]))
            mp = randbed.rows(rng, rng.choice([0, 1, 50, 800, 3000]), span=rng.choice([300, 3000]),
                              maxlen=rng.choice([10, 80, 300]))
            if trial % 2:  # exact matches, duplicates and nesting
                mp = sorted(mp + ref[::2] + ref[::3], key=lambda r: (r[0].encode(), r[1], r[2]))
            rt = randbed.text(ref, rest="cols", rng=rng).encode()
            mt = "".join(f"{c}\t{s}\t{e}\tid{i % 37}\t{rng.randint(0, 999)}" + ("\tx\t+" if i % 3 == 0 else "")
                         + "\n" for i, (c, s, e) in enumerate(mp)).encode()
            copt = [f"--{crit}"] + ([str(val)] if val is not None else [])
            kw = {"criterion": crit, "value": val}
            if crit == "bp-ovr":
                kw = {"overlap_bp": val}
            for ops in MAP_OPSETS:
                heavy = any(o in ("median", "mad") or isinstance(o, tuple) for o in ops)
                if heavy and len(mp) > 1500:  # O(window^2) selection per row: keep the windows modest
                    continue
                args = [a for o in ops for a in ([f"--{o[0]}", str(o[1])] if isinstance(o, tuple)
                                                 else [f"--{o}"])] + copt
                want = run_oracle(oracle_bin["bedmap"], args, [rt, mt], td)
                got = eng.bedmap(ops, rt, mt, **kw)
                assert got == want, (crit, val, ops, trial)


# bedmap --faster (Bedmap.cpp:287-290, 728-745): the sweep runs with the criterion and the
# visitors see its own calls; the GPU replays it as two one-integer chains (bg_faster.hip).
# Shapes: rows without nesting (what --faster is for), nested rows, duplicates, zero-length
# rows, a chromosome-long reference row (forces the chains' fix-up and serial passes).
FASTER_CRITS = [("bp-ovr", 1), ("bp-ovr", 7), ("range", 25), ("fraction-both", "0.3"), ("exact", None)]


def _flat_rows(rng, n, span, maxlen):
    out, s_, e_ = [], 0, 0
    for _ in range(n):
        s_ += rng.randint(0, max(1, 2 * span // max(n, 1)))
        e_ = max(e_ + rng.randint(0, 3), s_ + rng.randint(1, maxlen))
        out.append(("chr1", s_, e_))
    return out


@pytest.mark.parametrize("crit,val", FASTER_CRITS)
def test_bedmap_faster_vs_oracle(eng, oracle_bin, crit, val):
    rng = random.Random(zlib.crc32(repr(("faster", crit, val)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(10):
            shape = trial % 5
            if shape == 0:
                ref, mp = _flat_rows(rng, 3000, 200000, 90), _flat_rows(rng, 9000, 200000, 40)
            else:
                ref = randbed.rows(rng, rng.choice([1, 40, 600, 3000]), span=rng.choice([300, 5000]),
                                   maxlen=rng.choice([10, 80, 300]), zero_frac=0.1 if shape == 3 else 0.0)
                mp = randbed.rows(rng, rng.choice([1, 60, 900, 4000]), span=rng.choice([300, 5000]),
                                  maxlen=rng.choice([10, 80, 300]), zero_frac=0.1 if shape == 3 else 0.0)
                if shape == 2:
                    mp = sorted(mp + ref[::2] + ref[::3], key=lambda r: (r[0].encode(), r[1], r[2]))
                if shape == 4:  # a chromosome-long row ahead of everything
                    ref = sorted(ref + [("chr1", 0, 6000)], key=lambda r: (r[0].encode(), r[1], r[2]))
            rt = randbed.text(ref, rest="cols", rng=rng).encode()
            mt = "".join(f"{c}\t{s}\t{e}\tid{i % 37}\t{rng.randint(0, 999)}" + ("\tx\t+" if i % 3 == 0 else "")
                         + "\n" for i, (c, s, e) in enumerate(mp)).encode()
            copt = [f"--{crit}"] + ([str(val)] if val is not None else [])
            kw = {"overlap_bp": val} if crit == "bp-ovr" else {"criterion": crit, "value": val}
            for ops in (["count", "sum", "min", "max", "indicator"], ["bases", "bases-uniq", "mean"],
                        ["echo-map-id", "echo-map-score", "echo-overlap-size"], ["median", "stdev"],
                        ["min-element", "count"]):
                if ops[0] == "median" and len(mp) > 1500:
                    continue
                # an element operation stops the reference at the first unmapped row: with
                # --skip-unmapped every window it prints is non-empty
                skip = ops[0] == "min-element"
                args = ["--faster"] + (["--skip-unmapped"] if skip else []) + [f"--{o}" for o in ops] + copt
                want = run_oracle(oracle_bin["bedmap"], args, [rt, mt], td)
                got = eng.bedmap(ops, rt, mt, faster=True, skip_unmapped=skip, **kw)
                assert got == want, (crit, val, ops, trial)
                want = run_oracle(oracle_bin["bedmap"], args, [mt], td)  # one file
                got = eng.bedmap(ops, mt, None, faster=True, skip_unmapped=skip, **kw)
                assert got == want, ("single", crit, val, ops, trial)


@pytest.mark.parametrize("crit,val", MAP_CRITS)
def test_bedmap_zero_length_rows_vs_oracle(eng, oracle_bin, crit, val):
    """zero-length reference/map rows change the reference's sweep window (deleted, popped and
    hiding rows; WindowSweepImpl.cpp:195-237): k_mz_* reproduce it, byte-equal to the oracle"""
    rng = random.Random(zlib.crc32(repr(("zero", crit, val)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(8):
            zr, zm = rng.choice([(0.0, 0.2), (0.2, 0.0), (0.1, 0.1), (0.4, 0.3)])
            ref = randbed.rows(rng, rng.choice([1, 30, 400, 2000]), span=rng.choice([300, 3000]),
                               maxlen=rng.choice([10, 80]), zero_frac=zr)
            mp = randbed.rows(rng, rng.choice([1, 50, 800, 3000]), span=rng.choice([300, 3000]),
                              maxlen=rng.choice([10, 80, 300]), zero_frac=zm)
            rt = randbed.text(ref, rest="cols", rng=rng).encode()
            mt = "".join(f"{c}\t{s}\t{e}\tid{i % 37}\t{rng.randint(0, 999)}\n"
                         for i, (c, s, e) in enumerate(mp)).encode()
            copt = [f"--{crit}"] + ([str(val)] if val is not None else [])
            kw = {"overlap_bp": val} if crit == "bp-ovr" else {"criterion": crit, "value": val}
            for ops in (["count", "sum", "min", "max", "indicator"], ["bases", "bases-uniq", "mean"],
                        ["echo-map", "echo-map-id", "echo-overlap-size"], ["median", "stdev"],
                        ["echo-ref-row-id", "echo-map-id-uniq", "count"]):
                if ops[0] == "median" and len(mp) > 1500:
                    continue
                want = run_oracle(oracle_bin["bedmap"], [f"--{o}" for o in ops] + copt, [rt, mt], td)
                assert eng.bedmap(ops, rt, mt, **kw) == want, (crit, val, ops, trial)


@pytest.mark.parametrize("prec", [0, 3, 6, 12])
def test_bedmap_sci(eng, oracle_bin, prec):
    """--sci: every score-precision value as exact "%.{p}e" (glibc's rounding)"""
    rng = random.Random(prec + 40)
    ref = randbed.rows(rng, 300, span=3000, maxlen=80)
    mp = randbed.rows(rng, 1200, span=3000, maxlen=80)
    rt = randbed.text(ref).encode()
    ints = "".join(f"{c}\t{s}\t{e}\tid{i}\t{rng.choice([0, 1, 7, 999, 123456, -42])}\n"
                   for i, (c, s, e) in enumerate(mp)).encode()
    decs = "".join(f"{c}\t{s}\t{e}\tid{i}\t{rng.choice(['0.5', '-2.25', '0.001', '3.14159', '0.0001', '95'])}\n"
                   for i, (c, s, e) in enumerate(mp)).encode()
    with tempfile.TemporaryDirectory() as td:
        for mt, ops in ((ints, ["mean", "sum", "variance", "stdev", "cv", "bases-uniq-f", "min"]),
                        (decs, ["min", "max", "median", "echo-map-score", "mad"])):
            want = run_oracle(oracle_bin["bedmap"], [f"--{o}" for o in ops] + ["--sci", "--prec", str(prec)],
                              [rt, mt], td)
            assert eng.bedmap(ops, rt, mt, precision=prec, sci=True) == want, ops


def test_bedmap_dense_map_slice(eng, oracle_bin):
    """a workgroup whose candidate slice exceeds the LDS stage (searches in HBM instead)"""
    rng = random.Random(11)
    ref = randbed.rows(rng, 300, chroms=["chr1"], span=2000, maxlen=60)
    mp = randbed.rows(rng, 9000, chroms=["chr1"], span=2000, maxlen=60)
    rt = randbed.text(ref).encode()
    mt = randbed.text(mp, rest="bed5", rng=rng).encode()
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["bedmap"], ["--count", "--mean", "--bases-uniq"], [rt, mt], td)
        assert eng.bedmap(["count", "mean", "bases-uniq"], rt, mt) == want


def test_bedmap_min_max_decimal_scores(eng, oracle_bin):
    """min/max/order statistics take any score (no arithmetic)"""
    rng = random.Random(77)
    ref = randbed.rows(rng, 400, span=2000, maxlen=80)
    mp = randbed.rows(rng, 1500, span=2000, maxlen=80)
    rt = randbed.text(ref).encode()
    mt = "".join(f"{c}\t{s}\t{e}\tid{i}\t{rng.choice(['-', ''])}{rng.randint(0, 9999) / 100}\n"
                 for i, (c, s, e) in enumerate(mp)).encode()
    with tempfile.TemporaryDirectory() as td:
        for prec in (0, 2, 6):
            want = run_oracle(oracle_bin["bedmap"], ["--min", "--max", "--count", "--median", "--kth",
                                                     "0.7", "--mad", "--prec", str(prec)], [rt, mt], td)
            assert eng.bedmap(["min", "max", "count", "median", ("kth", 0.7), "mad"], rt, mt,
                              precision=prec) == want


def _decimal_map(rng, rows):
    out = []
    for i, (c, s, e) in enumerate(rows):
        kind = rng.random()
        if kind < 0.05:
            sc = f"{rng.choice(['', '-'])}{rng.randint(1, 9)}e{rng.randint(8, 16)}"  # mixed magnitudes
        elif kind < 0.5:
            sc = f"{rng.choice(['', '-'])}{rng.randint(0, 99999) / 1000}"
        else:
            sc = f"{rng.randint(0, 10 ** 6) / 10 ** rng.randint(1, 6)}"
        out.append(f"{c}\t{s}\t{e}\tid{rng.randint(0, 5)}\t{sc}" + ("\tx" if i % 4 == 0 else "") + "\n")
    return "".join(out).encode()


@pytest.mark.parametrize("crit,val", [("bp-ovr", 1), ("bp-ovr", 9), ("range", 15), ("fraction-map", "0.5"),
                                      ("fraction-either", "0.3"), ("exact", None)])
def test_bedmap_decimal_running_sums_vs_oracle(eng, oracle_bin, crit, val):
    """decimal scores: the reference's one running double per visitor, replayed in its event
    order (sweep pops in file order, then fixWindow deletes and adds in
    CoordRestAddressCompare order) by k_mev / k_mev_chain; byte-equal to the oracle"""
    rng = random.Random(zlib.crc32(repr(("dec", crit, val)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(6):
            ref = randbed.rows(rng, rng.choice([1, 40, 600, 2500]), span=rng.choice([300, 3000]),
                               maxlen=rng.choice([10, 80]))
            mp = randbed.rows(rng, rng.choice([1, 60, 900, 4000]), span=rng.choice([300, 3000]),
                              maxlen=rng.choice([10, 80, 300]))
            if trial % 2:  # equal coordinates with different ids and scores
                mp = sorted(mp + mp[::3] + mp[::5], key=lambda r: (r[0].encode(), r[1], r[2]))
            rt = randbed.text(ref).encode()
            mt = _decimal_map(rng, mp)
            copt = [f"--{crit}"] + ([str(val)] if val is not None else [])
            kw = {"overlap_bp": val} if crit == "bp-ovr" else {"criterion": crit, "value": val}
            for ops, prec in ((["count", "mean", "sum"], 6), (["variance", "stdev", "cv", "mean"], 9),
                              (["sum"], 0), (["mean", "min"], 17)):
                args = [f"--{o}" for o in ops] + copt + ["--prec", str(prec)]
                want = run_oracle(oracle_bin["bedmap"], args, [rt, mt], td)
                assert eng.bedmap(ops, rt, mt, precision=prec, **kw) == want, (crit, ops, trial)


def test_bedmap_decimal_score_spellings_vs_oracle(eng, oracle_bin):
    """the row parser's decimal fast path (parse_score_fast_ws: `<int>.<frac>` as one
    correctly rounded division) and every spelling it hands to the byte path: trailing zeros,
    integers written with a fraction, leading zeros, long fractions, 17-19 significant
    digits (above 2^53: decimal_exact's 128-bit rounding), signs, exponents, a lone dot side;
    byte-equal to the oracle for sums, means and extremes"""
    spell = ["0.000", "12.000", "1.50", "007.25", "5.", ".5", "3.14159265358979", "0.1", "0.2",
             "0.3", "99.999", "123456789012.5", "1234567.123456789012", "12345678901.12345678",
             "-1.5", "+2.25", "1e3", "2.5e-2", "10.0001", "4503599627370497.5", "0.000001",
             "1.0000000000001", "42", "000", "7.7", "100000.00001", "0.30000000000000004",
             "1.2345678901234567e-05", "9007199254740993", "123456789012345678e-5",
             "6.0221408570000001e+23", "2.2250738585072014e-10"]
    rng = random.Random(4242)
    ref = randbed.rows(rng, 500, chroms=["chr1", "chr2"], span=4000, maxlen=80)
    mp = randbed.rows(rng, 3000, chroms=["chr1", "chr2"], span=4000, maxlen=80)
    rt = randbed.text(ref).encode()
    mt = "".join(f"{c}\t{s}\t{e}\tid{i}\t{spell[i % len(spell)] if i % 3 else rng.choice(spell)}\n"
                 for i, (c, s, e) in enumerate(mp)).encode()
    with tempfile.TemporaryDirectory() as td:
        for ops, prec in ((["count", "sum", "mean"], 6), (["min", "max", "sum"], 17), (["variance", "mean"], 9)):
            want = run_oracle(oracle_bin["bedmap"], [f"--{o}" for o in ops] + ["--prec", str(prec)], [rt, mt], td)
            assert eng.bedmap(ops, rt, mt, precision=prec) == want, ops


def test_bedmap_decimal_drift_fixture(eng):
    """tests/golden/bedmap_drift.json: running-double drift (2|0.350001 where the exact mean
    is 0.35) and CoordRestAddressCompare order of equal rows"""
    import json
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bedmap_drift.json")))
    for c in cases:
        ops = [a[2:] for a in c["args"] if a.startswith("--") and a != "--prec"]
        prec = int(c["args"][c["args"].index("--prec") + 1]) if "--prec" in c["args"] else 6
        got = eng.bedmap(ops, c["ref"].encode(), c["map"].encode(), precision=prec)
        assert got == c["expect"].encode(), c["name"]


def test_bedmap_cli_overlap_options(gpu_bin, oracle_bin, tmp_path):
    rng = random.Random(5)
    ref = randbed.rows(rng, 300, span=3000, maxlen=100)
    mp = randbed.rows(rng, 900, span=3000, maxlen=100)
    r = randbed.write(str(tmp_path / "r.bed"), randbed.text(ref, rest="cols", rng=rng))
    m = randbed.write(str(tmp_path / "m.bed"), randbed.text(mp, rest="bed5", rng=rng))
    for args in (["--fraction-either", "0.4", "--echo", "--bases-uniq", "--max"],
                 ["--multidelim", "::", "--echo-map-id", "--echo-map", "--prec", "2", "--echo-map-score"],
                 ["--range", "10", "--delim", ";", "--indicator", "--sum"],
                 ["--range", "0", "--count"], ["--exact", "--skip-unmapped", "--echo-ref-name", "--count"],
                 ["--skip-unmapped", "--echo-ref-row-id", "--echo-map-id-uniq"]):
        want = subprocess.run([oracle_bin["bedmap"]] + args + [r, m], stdout=subprocess.PIPE,
                              check=True).stdout
        got = subprocess.run([gpu_bin["bedmap"]] + args + [r, m], stdout=subprocess.PIPE,
                             check=True).stdout
        assert got == want, args
    bad = subprocess.run([gpu_bin["bedmap"], "--bp-ovr", "3", "--exact", "--count", r, m],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    assert bad.returncode != 0 and b"More than one overlap specification used." in bad.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["file_wb", "file_rw_offset", "append", "pipe", "stream_env", "stdin"])
def test_cli_io_paths(gpu_bin, oracle_bin, tmp_path, how):
    """inputs mapped and DMA'd from the page cache (or read from stdin), output by parallel
    pwrite(2) into a regular file (write-only and read-write descriptors, at an unaligned
    offset), or streamed through write(2) (pipes, appends, BEDGPU_WRITE_PAR=0): every path
    gives the oracle's bytes, around whatever the file held before"""
    rng = random.Random(hash(how) & 0xffff)
    a = randbed.rows(rng, 120000, span=40_000_000, maxlen=500)
    b = randbed.rows(rng, 90000, span=40_000_000, maxlen=500)
    pa = randbed.write(str(tmp_path / "a.bed"), randbed.text(a))
    pb = randbed.write(str(tmp_path / "b.bed"), randbed.text(b))
    env = dict(os.environ)
    env.pop("BEDGPU_DEVICES", None)
    if how == "stream_env":
        env["BEDGPU_WRITE_PAR"] = "0"
    out = tmp_path / "out.bed"
    for mode in (["--intersect"], ["--everything"], ["--element-of", "1"]):
        want = subprocess.run([oracle_bin["bedops"]] + mode + [pa, pb], stdout=subprocess.PIPE,
                              check=True).stdout
        files = [pa, pb]
        stdin = None
        if how == "stdin":
            files = ["-", pb]
            stdin = open(pa, "rb")
        if how == "pipe":
            got = subprocess.run([gpu_bin["bedops"]] + mode + files, stdout=subprocess.PIPE, check=True,
                                 env=env).stdout
            assert got == want, (mode, how)
            continue
        prefix = b""
        if how == "file_wb" or how == "stream_env" or how == "stdin":
            fo = open(out, "wb")
        elif how == "file_rw_offset":
            fo = open(out, "w+b")
            prefix = b"#" * 12345  # not page aligned
            fo.write(prefix)
            fo.flush()
        else:  # append: O_APPEND
            prefix = b"previous line\n"
            out.write_bytes(prefix)
            fo = open(out, "ab")
        with fo:
            subprocess.run([gpu_bin["bedops"]] + mode + files, stdout=fo, check=True, env=env, stdin=stdin)
        if stdin:
            stdin.close()
        assert out.read_bytes() == prefix + want, (mode, how)


# ---------------------------------------------------------------------------------
# I/O edge cases (Appendix B of SURVEY.md)
# ---------------------------------------------------------------------------------
EDGE = [
    b"",                                                  # empty file
    b"chr1\t5\t10\n",                                     # single row
    b"chr1\t5\t10\nchr1\t20\t30",                         # unterminated last line: dropped
    b"chr1 5 10\nchr1  7   12\n",                         # spaces as separators
    b"chr1\t5\t10\r\nchr1\t11\t12\r\n",                   # CRLF
    b"chr1\t005\t010\tx\ty\n",                            # leading zeros, extra columns
    b"chr1\t5\t5\nchr1\t5\t10\n",                         # zero-length then real row
    b"chr1\t10\t20\nchr1\t20\t30\n",                      # touching rows
    b"  chr1\t1\t2\n",                                    # leading whitespace
    b"chrVeryLongName_" + b"x" * 100 + b"\t1\t9\n",       # long chrom name
]


@pytest.mark.parametrize("k", range(len(EDGE)))
@pytest.mark.parametrize("mode", ["-m", "-i", "-e", "-d"])
def test_io_edge_cases(eng, oracle_bin, k, mode):
    a = EDGE[k]
    b = b"chr1\t4\t8\nchr1\t9\t25\nchr2\t0\t5\n"
    texts = [a] if mode == "-m" else [a, b]
    spec = "1" if mode == "-e" else None
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["bedops"], [mode] + ([spec] if spec else []), texts, td)
    assert eng.bedops(mode, texts, spec=spec) == want


def test_unsorted_input_is_an_error(eng):
    from bedops_amd import BedgpuError
    for bad in (b"chr1\t50\t60\nchr1\t5\t10\n", b"chr2\t1\t2\nchr1\t1\t2\n",
                b"chr1\t1\t2\nchr2\t1\t2\nchr1\t3\t4\n", b"chr1\t50\t60\nchr1\t5\t10\nchr1\t70\t80\n",
                b"".join(b"chr1\t%d\t%d\n" % (i, i + 5) for i in range(300)).replace(b"\t200\t205", b"\t20\t205")):
        with pytest.raises(BedgpuError) as ei:
            eng.bedops("-m", [bad])
        assert ei.value.code == -3


def test_malformed_line_is_an_error(eng):
    from bedops_amd import BedgpuError
    for bad in (b"chr1\t5\n", b"chr1\tx\t10\n", b"chr1\t5\t2\n"):
        with pytest.raises(BedgpuError):
            eng.bedops("-m", [bad])


BLANKS = [b"chr1\t1\t2\n\nchr1\t3\t4\n", b"\nchr1\t1\t2\n", b"chr1\t1\t2\nchr1\t3\t4\n\n\n",
          b" \n\t\n\r\nchr1\t1\t2\n \nchr2\t3\t4\n", b"\n", b"\n\n \n", b"chr1\t1\t2\n\nchr1\t3\t4",
          b"chr1\t1\t2\n  chr1\t3\t9\n\t\n"]


@pytest.mark.parametrize("mode", ["-m", "-i", "-d", "-u", "-e", "-n", "-c", "-s", "-p"])
def test_blank_lines_are_skipped_like_fscanf(eng, oracle_bin, mode):
    """whitespace-only lines without --ec: the reference's fscanf (Bed.hpp:244-255) skips them
    (its --ec rejects them: "Empty line found."); the loader strips them and reloads
    (k_blank_*), in short files and in files of many 4 KiB tiles"""
    rng = random.Random(zlib.crc32(repr(("blank", mode)).encode()))
    big = randbed.text(randbed.rows(rng, 3000)).encode()
    lines = big.splitlines(keepends=True)
    for k in range(0, len(lines), 37):
        lines[k] = rng.choice([b"\n", b" \n", b"\t\t\n", b"\r\n"]) * rng.randint(1, 3) + lines[k]
    big_blank = b"".join(lines) + b"\n \n"
    b = b"chr1\t0\t3\nchr1\t3\t40\nchr2\t0\t5\n"
    cases = [[t] if mode in ("-m", "-c") else [t, b] for t in BLANKS]
    cases += [[big_blank] if mode in ("-m", "-c") else [big_blank, big]]
    spec = "1" if mode in ("-e", "-n") else None
    with tempfile.TemporaryDirectory() as td:
        for texts in cases:
            want = run_oracle(oracle_bin["bedops"], [mode] + ([spec] if spec else []), texts, td)
            assert eng.bedops(mode, texts, spec=spec) == want, (mode, texts[0][:60])


def test_chrom_restriction(eng, oracle_bin):
    rng = random.Random(7)
    a = randbed.text(randbed.rows(rng, 500)).encode()
    b = randbed.text(randbed.rows(rng, 500)).encode()
    with tempfile.TemporaryDirectory() as td:
        for ch in ("chr10", "chrX", "chrNone"):
            want = run_oracle(oracle_bin["bedops"], ["--chrom", ch, "-i"], [a, b], td)
            assert eng.bedops("-i", [a, b], chrom=ch) == want


# ---------------------------------------------------------------------------------
# full-size pinned hashes (produced by the reference binaries)
# ---------------------------------------------------------------------------------
def _gen(bedgen, n, seed, *flags):
    return subprocess.run([bedgen, str(n), str(seed), *flags], stdout=subprocess.PIPE,
                          check=True).stdout


def _h(b):
    return hashlib.sha256(b).hexdigest()[:16]


def test_merge_m1M_reference_hash(eng, bedgen):
    m = _gen(bedgen, 1000000, 1, "--chr1")
    out = eng.bedops("-m", [m])
    assert out.count(b"\n") == 847748 and len(out) == 20437351
    assert _h(out) == "5356e0cdf191310c"


@pytest.mark.slow
def test_bedmap_R5M_M50M_reference_hash(eng, bedgen):
    r = _gen(bedgen, 5000000, 7)
    m = _gen(bedgen, 50000000, 8, "--bed5")
    out = eng.bedmap(["count", "mean"], r, m)
    assert out.count(b"\n") == 4999998 and len(out) == 54515904
    assert _h(out) == "899ec7973e166e2d"


@pytest.mark.slow
def test_intersect_and_element_of_100M_reference_hash(eng, bedgen):
    a = _gen(bedgen, 100000000, 42)
    b = _gen(bedgen, 100000000, 43)
    out = eng.bedops("-i", [a, b])
    assert out.count(b"\n") == 38507974 and len(out) == 917848625
    assert _h(out) == "2495074965b49d74"
    del out
    out = eng.bedops("-e", [a, b], spec="1")
    assert out.count(b"\n") == 90223158 and len(out) == 2150489515
    assert _h(out) == "98a8a1c8a72bf6f5"


# ---------------------------------------------------------------------------------
# closest-features: the GPU replay of the reference's reader cache vs the oracle
# ---------------------------------------------------------------------------------
CLOSEST_OPTS = [[], ["--closest"], ["--dist"], ["--closest", "--dist"], ["--no-overlaps"],
                ["--no-overlaps", "--closest", "--dist"], ["--no-ref"], ["--delim", "\t"]]


def _closest_kwargs(args):
    kw = {"shortest": "--closest" in args, "dist": "--dist" in args,
          "no_ref": "--no-ref" in args, "no_overlaps": "--no-overlaps" in args}
    if "--delim" in args:
        kw["delim"] = args[args.index("--delim") + 1]
    return kw


def test_closest_hand_cases_gpu(eng):
    from test_oracle import CLOSEST_C, CLOSEST_KATS, CLOSEST_Q
    for args, want in CLOSEST_KATS:
        got = eng.closest(CLOSEST_Q.encode(), CLOSEST_C.encode(), **_closest_kwargs(args))
        assert got.decode() == want, args


@pytest.mark.parametrize("shape", ["sparse", "dense", "nested", "zero"])
@pytest.mark.parametrize("args", CLOSEST_OPTS, ids=lambda a: "_".join(a) or "default")
def test_random_closest_vs_oracle(eng, oracle_bin, shape, args):
    rng = random.Random(zlib.crc32(repr((shape, args)).encode()))
    nq, nc, span, ml, zf = {"sparse": (3000, 400, 200000, 100, 0.0),
                            "dense": (2000, 20000, 50000, 60, 0.0),
                            "nested": (3000, 3000, 100000, 3000, 0.0),
                            "zero": (2500, 2500, 10000, 80, 0.1)}[shape]
    q = randbed.text(randbed.rows(rng, nq, span=span, maxlen=ml, zero_frac=zf), rest="cols", rng=rng)
    c = randbed.text(randbed.rows(rng, nc, span=span, maxlen=ml, zero_frac=zf), rest="cols", rng=rng)
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["closest"], args, [q, c], td)
    got = eng.closest(q.encode(), c.encode(), **_closest_kwargs(args))
    assert got == want


def test_closest_edge_inputs(eng, oracle_bin):
    cases = [("", "chr1\t1\t2\n"), ("chr1\t1\t2\n", ""), ("", ""),
             ("chr1\t5\t5\nchr1\t5\t9\n", "chr1\t5\t5\nchr1\t9\t9\n"),
             ("chrA\t10\t20\nchrB\t10\t20\n", "chrB\t1\t2\nchrC\t3\t4\n")]
    for q, c in cases:
        for args in (["--closest", "--dist"], []):
            with tempfile.TemporaryDirectory() as td:
                want = run_oracle(oracle_bin["closest"], args, [q, c], td)
            assert eng.closest(q.encode(), c.encode(), **_closest_kwargs(args)) == want, (q, c, args)


def test_closest_cli_and_chrom(gpu_bin, oracle_bin, tmp_path):
    rng = random.Random(7)
    q = randbed.text(randbed.rows(rng, 5000, span=30000), rest="cols", rng=rng)
    c = randbed.text(randbed.rows(rng, 8000, span=30000), rest="cols", rng=rng)
    pq, pc = tmp_path / "q.bed", tmp_path / "c.bed"
    pq.write_text(q)
    pc.write_text(c)
    for args in (["--closest", "--dist"], ["--chrom", "chr10"], ["--no-overlaps", "--chrom", "chrX"]):
        want = subprocess.run([oracle_bin["closest"], *args, str(pq), str(pc)],
                              stdout=subprocess.PIPE, check=True).stdout
        got = subprocess.run([gpu_bin["closest"], *args, str(pq), str(pc)],
                             stdout=subprocess.PIPE, check=True).stdout
        assert got == want, args


@pytest.mark.slow
def test_closest_large_vs_oracle(eng, oracle_bin, bedgen, tmp_path):
    q = subprocess.run([bedgen, "1000000", "46"], stdout=subprocess.PIPE, check=True).stdout
    c = subprocess.run([bedgen, "20000000", "47"], stdout=subprocess.PIPE, check=True).stdout
    (tmp_path / "q.bed").write_bytes(q)
    (tmp_path / "c.bed").write_bytes(c)
    want = subprocess.run([oracle_bin["closest"], "--closest", str(tmp_path / "q.bed"),
                           str(tmp_path / "c.bed")], stdout=subprocess.PIPE, check=True).stdout
    assert eng.closest(q, c, shortest=True) == want


@pytest.mark.parametrize("crit,val", [("bp-ovr", 1), ("range", 500), ("fraction-ref", "0.2"), ("exact", None)])
def test_bedmap_long_rows_by_class_vs_oracle(eng, oracle_bin, crit, val):
    """map rows longer than 4 KiB are searched per length class (bg_map_cands): every
    operation, in the same visiting order as one window, byte-equal to the oracle"""
    rng = random.Random(zlib.crc32(repr(("long", crit, val)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(4):
            ref = randbed.rows(rng, rng.choice([50, 800]), chroms=["chr1", "chr2"], span=400000, maxlen=2000)
            mp = randbed.rows(rng, rng.choice([200, 3000]), chroms=["chr1", "chr2"], span=400000, maxlen=300)
            for _ in range(rng.choice([1, 5, 40])):  # long rows of many length classes
                c = rng.choice(["chr1", "chr2"])
                s = rng.randrange(0, 300000)
                mp.append((c, s, s + rng.choice([5000, 9000, 20000, 70000, 300000])))
            mp.sort(key=lambda r: (r[0].encode(), r[1], r[2]))
            rt = randbed.text(ref, rest="cols", rng=rng).encode()
            mt = "".join(f"{c}\t{s}\t{e}\tid{i % 17}\t{rng.randint(0, 999)}\n"
                         for i, (c, s, e) in enumerate(mp)).encode()
            copt = [f"--{crit}"] + ([str(val)] if val is not None else [])
            kw = {"overlap_bp": val} if crit == "bp-ovr" else {"criterion": crit, "value": val}
            for ops in (["count", "sum", "min", "max", "mean"], ["bases", "bases-uniq", "bases-uniq-f"],
                        ["echo-map", "echo-map-id", "echo-overlap-size", "echo-map-range"],
                        ["median", ("kth", 0.4), "echo-map-id-uniq"]):
                args = [a for o in ops for a in ([f"--{o[0]}", str(o[1])] if isinstance(o, tuple)
                                                 else [f"--{o}"])] + copt
                want = run_oracle(oracle_bin["bedmap"], args, [rt, mt], td)
                assert eng.bedmap(ops, rt, mt, **kw) == want, (crit, ops, trial)


def test_bedmap_chromosome_length_row_stays_fast(eng, oracle_bin, bedgen):
    """one chromosome-length map row in a 1M x 10M map: same answer as the oracle, and the
    GPU time within 3x of the same input without that row (its own length class; one window
    spanning the chromosome is ~1000x, the margin absorbs a shared box's noise)"""
    import time
    from bedops_amd.engine import BED3, BED5
    ref = subprocess.run([bedgen, "1000000", "7"], stdout=subprocess.PIPE, check=True).stdout
    mp = subprocess.run([bedgen, "10000000", "8", "--bed5"], stdout=subprocess.PIPE, check=True).stdout
    mp_long = b"chr1\t0\t248956422\tidLong\t7\n" + mp  # chr1's rows come first

    def timed(m):
        best = None
        for _ in range(3):
            s = eng.load([(ref, BED3), (m, BED5)])
            eng.sync()
            t0 = time.perf_counter()
            r = eng.map_op(s, ["count", "mean"], 0, 1)
            r.format()
            eng.sync()
            dt = time.perf_counter() - t0
            txt = r.text()
            r.free()
            s.free()
            best = dt if best is None else min(best, dt)
        return best, txt

    t_plain, _ = timed(mp)
    t_long, got = timed(mp_long)
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["bedmap"], ["--count", "--mean"], [ref, mp_long], td)
    assert got == want
    assert t_long < 3 * t_plain + 0.02, (t_long, t_plain)


def test_coordinates_up_to_the_key_limit_vs_oracle(gpu_bin, oracle_bin, tmp_path):
    """coordinates in [10^12, 2^40): 13-digit numbers (above the reference's
    MAX_COORD_VALUE, which only --ec enforces, BEDOPS.Constants.hpp:36) through every
    formatter (set modes, row modes, bedmap columns, closest-features), byte-equal to the
    oracle"""
    rng = random.Random(1340)
    top = (1 << 40) - 1
    for trial in range(3):
        files = []
        for f in range(2):
            rows = []
            for _ in range(rng.choice([20, 200])):
                s = rng.randrange(top - 10 ** 12 - 5000, top - 200)
                rows.append(("chr1", s, s + rng.randint(0, 150)))
            rows += [("chr2", 999_999_999_990 + k, 1_000_000_000_010 + k) for k in range(rng.randint(1, 4))]
            rows.sort(key=lambda r: (r[0].encode(), r[1], r[2]))
            p = tmp_path / f"in{trial}_{f}.bed"
            p.write_text("".join(f"{c}\t{s}\t{e}\tid{i}\t{i % 7}\n" for i, (c, s, e) in enumerate(rows)))
            files.append(str(p))
        for tool, args, nfiles in [("bedops", ["--merge"], 2), ("bedops", ["--intersect"], 2),
                                   ("bedops", ["--element-of", "1"], 2), ("bedops", ["--complement"], 2),
                                   ("bedops", ["--everything"], 2), ("bedmap", ["--echo", "--count", "--mean", "--echo-map"], 2),
                                   ("bedmap", ["--echo-map-range", "--echo-ref-name", "--bases"], 2),
                                   ("closest", ["--closest", "--dist"], 2)]:
            want = subprocess.run([oracle_bin[tool]] + args + files[:nfiles], stdout=subprocess.PIPE,
                                  check=True).stdout
            got = subprocess.run([gpu_bin[tool]] + args + files[:nfiles], stdout=subprocess.PIPE,
                                 check=True).stdout
            assert got == want, (trial, tool, args)
