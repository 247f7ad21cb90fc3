"""GPU parity for the remaining bedops operations: --complement [-L],
--chop [bp] [--stagger nt] [-x], --symmdiff, --partition, --everything and --range
padding, through the C ABI, byte-compared with the oracle's restatement of the
reference control flow (oracle/bedops_oracle.c, pinned by all 63 TestPlan KATs)."""
import os
import random
import subprocess
import tempfile
import zlib

import pytest

import randbed

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
            f.write(t)
        paths.append(p)
    return subprocess.run([binary] + args + paths, stdout=subprocess.PIPE, check=True,
                          timeout=120).stdout


RESTS = ["", "\ta", "\tb", "\tab", "\ta\tz", "\tB", "\t+"]


def rest_text(rng, rows):
    """rows with a small vocabulary of remainders, so equal (start, end) rows of
    different files tie and are ordered by strcmp of the remainder"""
    return "".join(f"{c}\t{s}\t{e}{rng.choice(RESTS)}\n" for c, s, e in rows).encode()


def gen(rng, nfiles, zero_frac, rest=False, near_zero=False):
    texts = []
    for _ in range(nfiles):
        n = rng.choice([0, 1, 3, 20, 150, 900])
        span = rng.choice([30, 60]) if near_zero else rng.choice([40, 300, 3000])
        rs = randbed.rows(rng, n, span=span, maxlen=rng.choice([4, 30, 120]), zero_frac=zero_frac)
        if rest:
            texts.append(rest_text(rng, rs))
        else:
            texts.append(randbed.text(rs).encode())
    return texts


def has_zero(texts):
    for t in texts:
        for ln in t.decode().splitlines():
            f = ln.split()
            if int(f[1]) == int(f[2]):
                return True
    return False


MODES = [
    ("-c", [], 1, {}), ("-c", [], 3, {}), ("-c", ["-L"], 2, {"full_left": True}),
    ("-w", [], 1, {}), ("-w", ["5"], 2, {"chop": (5, 0, False)}),
    ("-w", ["7", "--stagger", "3"], 2, {"chop": (7, 3, False)}),
    ("-w", ["4", "-x"], 1, {"chop": (4, 0, True)}),
    ("-w", ["10", "--stagger", "4", "-x"], 3, {"chop": (10, 4, True)}),
    ("-w", ["3", "--stagger", "9"], 2, {"chop": (3, 9, False)}),
    ("-s", [], 2, {}), ("-s", [], 3, {}), ("-s", [], 4, {}),
    ("-p", [], 1, {}), ("-p", [], 2, {}), ("-p", [], 4, {}),
    ("-u", [], 1, {}), ("-u", [], 2, {}), ("-u", [], 4, {}),
]


@pytest.mark.parametrize("zero_frac", [0.0, 0.08])
@pytest.mark.parametrize("mode,extra,nfiles,kw", MODES,
                         ids=lambda v: "_".join(v) if isinstance(v, list) else str(v))
def test_random_modes_vs_oracle(eng, oracle_bin, mode, extra, nfiles, kw, zero_frac):
    rng = random.Random(zlib.crc32(repr((mode, extra, nfiles, zero_frac)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(10):
            texts = gen(rng, nfiles, zero_frac, rest=(mode == "-u"))
            # (--symmdiff over zero-length rows: the stream replay, k_sd_replay)
            want = run_oracle(oracle_bin["bedops"], [mode] + extra, texts, td)
            got = eng.bedops(mode, texts, **kw)
            assert got == want, (mode, extra, trial)


PADS = [(-5, 5), (-100, 100), (5, -8), (-5, -8), (-3, -1), (10, 0), (0, 7), (-20, 0), (3, 3),
        (0, -2), (-1, 40)]


@pytest.mark.parametrize("pad", PADS, ids=lambda p: f"{p[0]}:{p[1]}")
@pytest.mark.parametrize("mode,nfiles", [("-m", 2), ("-u", 2), ("-e", 2), ("-p", 2), ("-c", 1),
                                         ("-w", 1), ("-d", 2), ("-u", 1)])
def test_range_padding_vs_oracle(eng, oracle_bin, mode, nfiles, pad):
    """rows start near base 0 on several chromosomes, so clamping, the re-sort of clamped
    rows, vaporised rows and the first-chromosome-only getFirst of negative pads all occur"""
    from bedops_amd import BedgpuError
    rng = random.Random(zlib.crc32(repr((mode, nfiles, pad)).encode()))
    with tempfile.TemporaryDirectory() as td:
        for trial in range(8):
            texts = gen(rng, nfiles, 0.05, rest=(mode in ("-u", "-e")), near_zero=True)
            # A uint64 wrap of an end inside the reference's getFirst (BedPadReader.hpp:212)
            # yields ends near 2^64 (the reference then prints them, or loops for ~2^64 steps
            # in --chop): such inputs are refused on the GPU path (past the 2^40 key range). The oracle's
            # --everything prints each padded input to detect them.
            huge = False
            for i in range(nfiles):
                if mode == "-e" and i == 0:
                    continue
                out = run_oracle(oracle_bin["bedops"], ["--range", f"{pad[0]}:{pad[1]}", "-u"],
                                 [texts[i]], td)
                huge |= any(int(x) >= 2 ** 40 - 1 for ln in out.decode().splitlines()
                            for x in ln.split("\t")[1:3])
            if huge:
                with pytest.raises(BedgpuError) as ei:
                    eng.bedops(mode, texts, pad=pad)
                assert ei.value.code == -8
                continue
            want = run_oracle(oracle_bin["bedops"], ["--range", f"{pad[0]}:{pad[1]}", mode], texts,
                              td)
            got = eng.bedops(mode, texts, pad=pad)
            assert got == want, (mode, pad, trial)


def test_range_symmetric_shorthand_cli(gpu_bin, oracle_bin, tmp_path):
    rng = random.Random(7)
    a = tmp_path / "a.bed"
    a.write_bytes(rest_text(rng, randbed.rows(rng, 300, span=200, maxlen=30)))
    for args in (["--range", "10", "-u"], ["--range", "-3", "-m"], ["--range", "4:-2", "-c", "-L"]):
        want = subprocess.run([oracle_bin["bedops"]] + args + [str(a)], stdout=subprocess.PIPE,
                              check=True).stdout
        got = subprocess.run([gpu_bin["bedops"]] + args + [str(a)], stdout=subprocess.PIPE,
                             check=True).stdout
        assert got == want, args


@pytest.mark.parametrize("mode,nfiles", [("-p", 3), ("-s", 3), ("-u", 3), ("-c", 2),
                                         ("-w", 2)])
def test_modes_large_vs_oracle(eng, oracle_bin, mode, nfiles):
    """a few hundred thousand rows: many radix-sort tiles, long merge-path passes"""
    rng = random.Random(99)
    texts = []
    for f in range(nfiles):
        rs = randbed.rows(rng, 120000, chroms=randbed.CHROMS + ["chr5", "chrY"], span=400000,
                          maxlen=300)
        texts.append(rest_text(rng, rs) if mode == "-u" else randbed.text(rs).encode())
    extra = ["25", "--stagger", "10"] if mode == "-w" else []
    kw = {"chop": (25, 10, False)} if mode == "-w" else {}
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["bedops"], [mode] + extra, texts, td)
    assert eng.bedops(mode, texts, **kw) == want


@pytest.mark.parametrize("nfiles", [2, 3, 5])
def test_symmdiff_zero_length_replay_vs_oracle(eng, oracle_bin, nfiles):
    """--symmdiff over zero-length rows: the per-segment stream replay (k_sd_replay) against the
    oracle's nextSymmetricDiffLine (Bedops.cpp:1343-1467), dense zero-length, nested and
    duplicated rows near base 0"""
    rng = random.Random(zlib.crc32(repr(("sd-zero", nfiles)).encode()))
    seen = 0
    with tempfile.TemporaryDirectory() as td:
        for trial in range(25):
            texts = gen(rng, nfiles, rng.choice([0.1, 0.3, 0.6]), near_zero=rng.random() < 0.5)
            seen += has_zero(texts)
            want = run_oracle(oracle_bin["bedops"], ["-s"], texts, td)
            assert eng.bedops("-s", texts) == want, (nfiles, trial)
    assert seen >= 10
