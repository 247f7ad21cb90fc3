"""Pin the oracle against the genuine reference (CPU only).

tests/golden/ref_*.json.gz hold the output of BEDOPS v2.4.26 itself (built from /root/reference
by oracle/build_ref.sh, run by tests/golden/make_ref_fixtures.py): closest-features under all
option sets, every bedmap operation under every overlap criterion, decimal-score running
doubles, sort-bed ordering and --ec messages. Each oracle restatement must reproduce them
byte for byte, so the GPU tests that compare against the oracle inherit the pin.
"""
import os

import pytest

import ref_fixtures as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Known residual divergence of the oracle's heap-address model (oracle/heapsim.h): the
# reference orders equal-coordinate map rows by heap address; the model replays glibc's
# tcache/fast-bin reuse but not malloc_consolidate, which this case's 150-row window
# triggers when the heap grows. (suite, case index)
KNOWN = {("bedmap", 160)}


def _bin(oracle_bin, tool):
    return oracle_bin[{"bedops": "bedops", "bedmap": "bedmap", "closest": "closest",
                       "sortbed": "sortbed"}[tool]]


@pytest.mark.parametrize("suite", ["closest", "bedmap", "decimal", "sortbed", "faster", "f2", "r6"])
def test_oracle_reproduces_reference(oracle_bin, suite):
    fx = R.load(suite)
    bad = []
    for k, c in enumerate(fx["cases"]):
        if (suite, k) in KNOWN:
            continue
        # argument errors and --ec checks are the drop-in CLI's (tests/test_gpu_ref_fixtures.py);
        # the oracle restates the sweeps
        if c["rc"] != 0 or "--ec" in c["args"] or "--header" in c["args"]:
            continue
        d = R.compare(_bin(oracle_bin, c["tool"]), fx, c, check_stderr=False)
        if d:
            bad.append((k, c["args"], d[:200]))
    assert not bad, bad[:5]
    assert len(fx["cases"]) > 5


def test_known_divergences_still_diverge(oracle_bin):
    """if a KNOWN case starts matching, the list is stale"""
    for suite, k in KNOWN:
        fx = R.load(suite)
        c = fx["cases"][k]
        assert R.compare(_bin(oracle_bin, c["tool"]), fx, c, check_stderr=False) is not None


def test_ec_oracle_messages_match_reference(oracle_bin):
    """oracle/ec_oracle.c's first-error text equals the reference's --ec message (bedops
    --ec --merge over a malformed first file and a clean second one)"""
    import subprocess
    import tempfile
    fx = R.load("ec")
    ec = os.path.join(ROOT, "oracle", "build", "ec_oracle")
    n = 0
    for c in fx["cases"]:
        if c["tool"] != "bedops" or c["args"] != ["--ec", "--merge"]:
            continue
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "in0.bed")
            with open(p, "w") as f:
                f.write(fx["groups"][c["group"]][0])
            r = subprocess.run([ec, "3", "0", p], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        got = (r.stdout + r.stderr).decode().replace(p, "@0")
        if c["rc"] == 0:
            assert r.returncode == 0 and got == "", (c, got)
        else:
            want = c["stderr"].split("Error: ", 1)[1]
            assert r.returncode == 1 and got.strip() == want.strip(), (want, got)
        n += 1
    assert n == len(fx["groups"])


def test_fixture_suites_cover_the_surfaces():
    """every bedmap operation name the reference parser accepts (minus the *-rand ones, which
    the reference randomises) appears in the fixtures, under every criterion"""
    fx = R.load("bedmap")
    ops = {a for c in fx["cases"] for a in c["args"] if a.startswith("--")}
    for o in ["--count", "--mean", "--sum", "--min", "--max", "--indicator", "--bases", "--bases-uniq",
              "--bases-uniq-f", "--echo", "--echo-ref-size", "--echo-ref-name", "--echo-map",
              "--echo-map-id", "--echo-map-id-uniq", "--echo-map-score", "--echo-map-size",
              "--echo-overlap-size", "--echo-map-range", "--median", "--kth", "--mad", "--variance",
              "--stdev", "--cv", "--sci", "--min-element", "--max-element", "--tmean", "--wmean",
              "--echo-ref-row-id", "--skip-unmapped", "--delim", "--prec"]:
        assert o in ops, o
    for crit in ["--bp-ovr", "--range", "--fraction-ref", "--fraction-map", "--fraction-either",
                 "--fraction-both", "--exact"]:
        assert crit in ops, crit
    opts = {tuple(c["args"]) for c in R.load("closest")["cases"]}
    assert len(opts) >= 9
