"""--ec through the drop-in CLIs on the GPU (bg_check): every error class of
tests/test_check.py gives the oracle's message (oracle/ec_oracle.c) with the reference's
error framing and exit status; clean files give the same output as without --ec."""
import os
import subprocess

import pytest

import test_check

pytestmark = pytest.mark.gpu


def _oracle(path, nf, rest):
    return test_check.oracle_text(path, nf, rest)


@pytest.mark.parametrize("mode,nf,rest", [("-m", 3, 0), ("-e", 3, 1)])
def test_bedops_ec_messages(gpu_bin, oracle_bin, tmp_path, mode, nf, rest):
    ok = str(tmp_path / "ok.bed")
    with open(ok, "wb") as f:
        f.write(b"chr1\t1\t3\nchr1\t4\t8\n")
    for i, data in enumerate(test_check.CASES):
        p = str(tmp_path / f"c{i}.bed")
        with open(p, "wb") as f:
            f.write(data)
        want = _oracle(p, nf, rest)
        args = [gpu_bin["bedops"], "--ec", mode, p, ok]
        r = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
        if want:
            assert r.returncode != 0, data
            assert r.stderr == b"May use bedops --help for more help.\n\nError: " + want + b"\n", data
        else:
            assert r.returncode == 0, (data, r.stderr)
            plain = subprocess.run([gpu_bin["bedops"], "--header", mode, p, ok], stdout=subprocess.PIPE)
            assert r.stdout == plain.stdout, data


def test_bedmap_ec_map_fields(gpu_bin, tmp_path):
    ref = str(tmp_path / "r.bed")
    with open(ref, "wb") as f:
        f.write(b"chr1\t1\t30\n")
    for i, data in enumerate(test_check.CASES5):
        p = str(tmp_path / f"m{i}.bed")
        with open(p, "wb") as f:
            f.write(data)
        want = _oracle(p, 5, 1)
        r = subprocess.run([gpu_bin["bedmap"], "--ec", "--mean", ref, p], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE)
        if want:
            assert r.stderr == b"May use bedmap --help for more help.\n\nError: " + want + b"\n", data
        else:
            assert r.returncode == 0, (data, r.stderr)


def test_ec_large_clean_file(gpu_bin, bedgen, tmp_path):
    """a clean 2M-row file passes --ec and gives the plain output"""
    p = str(tmp_path / "a.bed")
    with open(p, "wb") as f:
        subprocess.run([bedgen, "2000000", "11"], stdout=f, check=True)
    r = subprocess.run([gpu_bin["bedops"], "--ec", "-m", p], stdout=subprocess.PIPE, check=True)
    plain = subprocess.run([gpu_bin["bedops"], "-m", p], stdout=subprocess.PIPE, check=True)
    assert r.stdout == plain.stdout


def test_engine_check_matches_oracle(eng_check, tmp_path):
    for i, data in enumerate(test_check.CASES):
        p = str(tmp_path / f"e{i}.bed")
        with open(p, "wb") as f:
            f.write(data)
        got = eng_check.check(data, 3, True, name=p)
        assert (got or b"") == _oracle(p, 3, 1), data


@pytest.fixture(scope="module")
def eng_check():
    from bedops_amd import Engine
    e = Engine(0)
    yield e
    e.close()
