"""CPU-only checks that pin the oracle (test infrastructure) before it is trusted:
the reference's own KATs and the reference-produced output hashes of SURVEY.md
Appendix D, plus the synthetic generator's input hashes."""
import hashlib
import os
import subprocess

import pytest

import testplan_runner


def _h(b):
    return hashlib.sha256(b).hexdigest()[:16]


def test_testplan_kats_oracle(oracle_bin, tmp_path):
    """All 63 KATs: the hot-path modes and complement/chop/symmdiff/partition/everything
    with --range, --chrom and -L."""
    res = testplan_runner.run_testplan([oracle_bin["bedops"]], str(tmp_path))
    assert len(res) == 63
    bad = [r for r in res if not r[2]]
    assert not bad, bad


def test_testplan_fixture_complete():
    tests = testplan_runner.load_tests()
    assert len(tests) == 63
    modes = [testplan_runner.test_mode(t) for t in tests]
    assert modes.count("m") == 10 and modes.count("i") == 4 and modes.count("d") == 7


def test_generator_matches_survey_hashes(bedgen):
    m = subprocess.run([bedgen, "1000000", "1", "--chr1"], stdout=subprocess.PIPE, check=True).stdout
    assert m.count(b"\n") == 1000000 and len(m) == 24107523 and _h(m) == "be10f5128ea87dfd"
    r = subprocess.run([bedgen, "5000000", "7"], stdout=subprocess.PIPE, check=True).stdout
    assert r.count(b"\n") == 4999998 and len(r) == 119178183 and _h(r) == "8504e875c83bc0b6"


def test_oracle_merge_m1M_reference_hash(oracle_bin, bedgen, tmp_path):
    p = tmp_path / "m1M.bed"
    p.write_bytes(subprocess.run([bedgen, "1000000", "1", "--chr1"], stdout=subprocess.PIPE,
                                 check=True).stdout)
    out = subprocess.run([oracle_bin["bedops"], "-m", str(p)], stdout=subprocess.PIPE,
                         check=True).stdout
    assert out.count(b"\n") == 847748 and len(out) == 20437351
    assert _h(out) == "5356e0cdf191310c"


def test_oracle_bedmap_small_known_answer(oracle_bin, tmp_path):
    # hand-checked: map rows overlapping [10,20) by >= 1 bp are [5,12) s=4 and [19,30) s=9
    ref = tmp_path / "r.bed"
    mp = tmp_path / "m.bed"
    ref.write_text("chr1\t10\t20\nchr1\t40\t50\n")
    mp.write_text("chr1\t5\t12\ta\t4\nchr1\t19\t30\tb\t9\nchr1\t20\t40\tc\t1\n")
    out = subprocess.run([oracle_bin["bedmap"], "--count", "--mean", str(ref), str(mp)],
                         stdout=subprocess.PIPE, check=True).stdout
    assert out == b"2|6.500000\n0|NAN\n"


# hand-worked closest-features cases (ClosestFeature.cpp:260-413, Printers.hpp:46-205):
# q1 [100,200): b [60,90) is the left (distance -(100-90+1) = -11); c [150,160) lies inside
# q1 and starts after its centroid 149.5 (proportion 0 < 0.5, no overlapping left yet), so
# it is the right; --closest prints the overlapping right. q2 [500,510): d [300,400) left
# (-101), e [505,600) hangs over the right edge. q3: no candidate on chr2 -> NA.
CLOSEST_Q = "chr1\t100\t200\tq1\nchr1\t500\t510\tq2\nchr2\t10\t20\tq3\n"
CLOSEST_C = ("chr1\t10\t50\ta\nchr1\t60\t90\tb\nchr1\t150\t160\tc\nchr1\t300\t400\td\n"
             "chr1\t505\t600\te\nchr3\t1\t2\tf\n")
CLOSEST_KATS = [
    ([], "chr1\t100\t200\tq1|chr1\t60\t90\tb|chr1\t150\t160\tc\n"
         "chr1\t500\t510\tq2|chr1\t300\t400\td|chr1\t505\t600\te\n"
         "chr2\t10\t20\tq3|NA|NA\n"),
    (["--closest"], "chr1\t100\t200\tq1|chr1\t150\t160\tc\n"
                    "chr1\t500\t510\tq2|chr1\t505\t600\te\nchr2\t10\t20\tq3|NA\n"),
    (["--dist"], "chr1\t100\t200\tq1|chr1\t60\t90\tb|-11|chr1\t150\t160\tc|0\n"
                 "chr1\t500\t510\tq2|chr1\t300\t400\td|-101|chr1\t505\t600\te|0\n"
                 "chr2\t10\t20\tq3|NA|NA|NA|NA\n"),
    (["--closest", "--dist"], "chr1\t100\t200\tq1|chr1\t150\t160\tc|0\n"
                              "chr1\t500\t510\tq2|chr1\t505\t600\te|0\nchr2\t10\t20\tq3|NA|NA\n"),
    (["--no-overlaps"], "chr1\t100\t200\tq1|chr1\t60\t90\tb|chr1\t300\t400\td\n"
                        "chr1\t500\t510\tq2|chr1\t300\t400\td|NA\nchr2\t10\t20\tq3|NA|NA\n"),
    (["--no-ref", "--closest", "--delim", ";"], "chr1\t150\t160\tc\nchr1\t505\t600\te\nNA\n"),
]


def test_oracle_closest_hand_cases(oracle_bin, tmp_path):
    q, c = tmp_path / "q.bed", tmp_path / "c.bed"
    q.write_text(CLOSEST_Q)
    c.write_text(CLOSEST_C)
    for args, want in CLOSEST_KATS:
        out = subprocess.run([oracle_bin["closest"], *args, str(q), str(c)],
                             stdout=subprocess.PIPE, check=True).stdout.decode()
        assert out == want, args


def test_closest_cache_free_model_is_not_the_reference(oracle_bin, tmp_path):
    """Documents why the GPU replays the reference's cache: a candidate that overlapped an
    earlier row and ends after a later-found left row is dropped by the reference
    (ClosestFeature.cpp:300-304), so a cache-free nearest-left search would differ."""
    import model_closest
    q, c = tmp_path / "q.bed", tmp_path / "c.bed"
    # row 1 [150,170): c0 [79,156) overlaps it; c1 [122,148) is a new best left and
    # empties the kept list, dropping c0. Row 2 [178,202): the true nearest left is c0
    # (ends 156) but the reference reports c1.
    q.write_text("chr1\t150\t170\tr1\nchr1\t178\t202\tr2\n")
    c.write_text("chr1\t79\t156\tc0\nchr1\t122\t148\tc1\n")
    out = subprocess.run([oracle_bin["closest"], "--no-overlaps", str(q), str(c)],
                         stdout=subprocess.PIPE, check=True).stdout.decode().splitlines()
    assert out[1] == "chr1\t178\t202\tr2|chr1\t122\t148\tc1|NA"
    left, _ = model_closest.pick([(79, 156), (122, 148)], (178, 202), allow_overlaps=False)
    assert left == 0  # cache-free answer: c0


# hand-worked bedmap answers for every operation and criterion on the oracle (computed by
# hand from the reference's definitions: BedDistances.hpp, OvrAggregate/OvrUnique visitors)
BEDMAP_HAND_REF = "chr1\t10\t100\ta\tx\nchr1\t50\t60\tb\nchr2\t5\t10\tc\n"
BEDMAP_HAND_MAP = ("chr1\t0\t20\tm1\t5\nchr1\t15\t55\tm2\t-3\nchr1\t58\t70\tm3\t7.5\n"
                   "chr1\t90\t200\tm4\t2\nchr2\t7\t9\tm5\t1\n")
BEDMAP_HAND = [
    (["--count", "--sum", "--min", "--max", "--indicator"],
     "4|11.500000|-3.000000|7.500000|1\n2|4.500000|-3.000000|7.500000|1\n1|1.000000|1.000000|1.000000|1\n"),
    (["--bases", "--bases-uniq", "--bases-uniq-f", "--echo"],
     "72|67|0.744444|chr1\t10\t100\ta\tx\n7|7|0.700000|chr1\t50\t60\tb\n2|2|0.400000|chr2\t5\t10\tc\n"),
    (["--range", "30", "--count", "--echo-ref-name", "--echo-ref-size"],
     "4|chr1:10-100|90\n2|chr1:50-60|10\n1|chr2:5-10|5\n"),
    (["--fraction-map", "0.5", "--count", "--bases"], "3|62\n0|0\n1|2\n"),
    (["--fraction-ref", "0.2", "--count"], "1\n2\n1\n"),
    (["--fraction-both", "0.3", "--count"], "1\n0\n1\n"),
    (["--exact", "--count"], "0\n0\n0\n"),
]


@pytest.mark.parametrize("k", range(len(BEDMAP_HAND)))
def test_bedmap_oracle_hand_cases(oracle_bin, tmp_path, k):
    args, want = BEDMAP_HAND[k]
    r = tmp_path / "r.bed"
    m = tmp_path / "m.bed"
    r.write_text(BEDMAP_HAND_REF)
    m.write_text(BEDMAP_HAND_MAP)
    out = subprocess.run([oracle_bin["bedmap"]] + args + [str(r), str(m)], stdout=subprocess.PIPE,
                         check=True).stdout.decode()
    assert out == want


def test_oracle_bedmap_drift_fixture(oracle_bin, tmp_path):
    """the committed running-double fixture (tests/golden/make_bedmap_drift_fixture.py)"""
    import json
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bedmap_drift.json")))
    assert any(c["expect"].endswith("2|0.350001\n") for c in cases)
    for c in cases:
        pr, pm = tmp_path / "r.bed", tmp_path / "m.bed"
        pr.write_text(c["ref"])
        pm.write_text(c["map"])
        got = subprocess.run([oracle_bin["bedmap"], *c["args"], str(pr), str(pm)],
                             stdout=subprocess.PIPE, check=True).stdout.decode()
        assert got == c["expect"], c["name"]


def test_sortbed_oracle_matches_python_model(oracle_bin, tmp_path):
    """oracle/sortbed_oracle.c against a few-line Python statement of sort-bed's order
    (strcmp chromosome, start, end, rest; no rest first) and printBed's format"""
    import random
    rng = random.Random(4)
    for trial in range(30):
        rows, text = [], []
        for _ in range(rng.choice([0, 3, 200])):
            c = rng.choice(["chr1", "chr10", "chr2", "chrX", "1", "2"])
            s = rng.randrange(1000)
            e = s + rng.randint(1, 30)
            rest = rng.choice([None, "a", "b\t1", "a b", "id3"])
            sep = rng.choice(["\t", " "])
            text.append(f"{c}{sep}{s}{sep}{e}" + ("" if rest is None else f"{sep}{rest}"))
            rows.append((c.encode(), s, e, rest))
        p = tmp_path / f"s{trial}.bed"
        p.write_text("".join(ln + "\n" for ln in text))
        rows.sort(key=lambda r: (r[0], r[1], r[2], (0, "") if r[3] is None else (1, r[3].encode())))
        want = "".join(f"{c.decode()}\t{s}\t{e}" + ("" if r is None else f"\t{r}") + "\n"
                       for c, s, e, r in rows)
        got = subprocess.run([oracle_bin["sortbed"], str(p)], stdout=subprocess.PIPE,
                             check=True).stdout.decode()
        assert got == want, trial


# hand-worked answers for the visitors restated last (ExtremeVisitor with
# ScoreThenGenomicCompare*, TrimmedMeanVisitor, WeightedAverageVisitor, sweep overload 1)
VIS_REF = "chr1\t10\t50\nchr1\t100\t120\nchr1\t300\t400\n"
VIS_MAP = ("chr1\t5\t20\ta\t3\nchr1\t15\t30\tb\t7\nchr1\t15\t30\tc\t7\n"
           "chr1\t40\t60\td\t1.5\nchr1\t105\t110\te\t2\n")


def test_bedmap_oracle_new_visitors_by_hand(oracle_bin, tmp_path):
    r, m = tmp_path / "r.bed", tmp_path / "m.bed"
    r.write_text(VIS_REF)
    m.write_text(VIS_MAP)
    run = lambda *a: subprocess.run([oracle_bin["bedmap"], *a], capture_output=True)
    o = run("--echo", "--max-element", "--min-element", "--tmean", "0.1", "0.1", "--wmean",
            "--max-element-rand", "--skip-unmapped", str(r), str(m))
    # row 1: b and c tie on (7, chr1 15 30): the set keeps b, added first (its full_rest
    # "b" < "c"); -rand: the last of the equal scores here; trimmed mean of 4 with nothing
    # trimmed = 18.5/4; weights .25/.375/.375/.25 of scores 3/7/7/1.5 -> 6.375/1.25
    assert o.stdout.decode() == (
        "chr1\t10\t50|chr1\t15\t30\tb\t7.000000|chr1\t40\t60\td\t1.500000|4.625000|5.100000|chr1\t15\t30\tc\t7.000000\n"
        "chr1\t100\t120|chr1\t105\t110\te\t2.000000|chr1\t105\t110\te\t2.000000|2.000000|2.000000|chr1\t105\t110\te\t2.000000\n")
    # an unmapped row: PrintAllScorePrecision throws on NaN after what precedes it
    o = run("--echo", "--min-element", str(r), str(m))
    assert o.returncode != 0
    assert o.stdout.decode().endswith("chr1\t300\t400|")
    assert o.stderr.decode() == ("May use bedmap --help for more help.\n\n"
                                 "Error: Unable to process a 'NAN' with PrintAllScorePrecision.\n")
    # single-file mode: rows re-printed as B5Rest ("%lf" score); --tmean 0.2 0.3 of {3,7,7}
    # trims one row at the bottom: (3 + 7 - 3) / 1
    o = run("--echo", "--count", "--tmean", "0.2", "0.3", str(m))
    assert o.stdout.decode().splitlines()[0] == "chr1\t5\t20\ta\t3.000000|3|7.000000"
