"""CPU-only checks that pin the oracle (test infrastructure) before it is trusted:
the reference's own KATs and the reference-produced output hashes of SURVEY.md
Appendix D, plus the synthetic generator's input hashes."""
import hashlib
import subprocess

import testplan_runner


def _h(b):
    return hashlib.sha256(b).hexdigest()[:16]


def test_testplan_kats_oracle(oracle_bin, tmp_path):
    res = testplan_runner.run_testplan([oracle_bin["bedops"]], str(tmp_path),
                                       modes={"m", "i", "d", "e", "n"})
    assert len(res) == 28
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
