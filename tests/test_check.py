"""--ec validation: the GPU grammar (bedops_amd/csrc/bg_check.h, compiled
here with g++) and the library's message wording against the oracle's restatement of
Bed::bed_check_iterator (oracle/ec_oracle.c) on every error class; the GPU run of the same
cases goes through the CLIs (tests/test_gpu_check.py)."""
import ctypes
import os
import random
import subprocess

import pytest

from conftest import ROOT

# one or more lines per error class of BedCheckIterator.hpp:326-624 (3-field BED unless noted)
CASES = [
    b"chr1\t5\t10\n\nchr1\t6\t7\n", b"chr1 \t5\t10\n", b"\tchr1\t5\t10\n", b"chr1\n",
    b"c" * 130 + b"\t1\t2\n", b"chr1\t\t5\n", b"chr1\t-5\t10\n", b"chr1\t5 \t10\n",
    b"chr1\t5x\t10\n", b"chr1\t+5\t10\n", b"chr1\t5\n", b"chr1\t1234567890123\t2\n",
    b"chr1\t5\t\t\n", b"chr1\t5\t-10\n", b"chr1\t5\t10 x\n", b"chr1\t5\t1y0\n",
    b"chr1\t5\t10\r\n", b"chr1\t5\t1234567890123\n", b"chr1\t5\t10\nchr1\t4\t10\n",
    b"chr2\t5\t10\nchr1\t4\t10\n", b"chr1\t5\t10\nchr1\t5\t9\n", b"chr1\t5\t5\n",
    b"chr1\t7\t5\n", b"track name=x\nbrowser position\n#c\n@h\nchr1\t5\t10\n",
    b"chr1\t5\t10\ntrack x\n", b"chr1\t5\t10\n#late\n", b"chr1\t5\t10", b"chr1\t5\t",
    b"TRACK\nchr1\t1\t2\nchr1\t1\t2\n", b"chr1\t5\t10\tb\nchr1\t5\t10\ta\n",
    b"chr1\t5\t10\t0b\nchr1\t5\t010\ta\n", b"chr10\t1\t2\nchr1\t3\t4\n", b"",
]
CASES5 = [  # map files under score operations: 5 fields
    b"chr1\t5\t10\tid\t1\n", b"chr1\t5\t10\n", b"chr1\t5\t10\tid\n", b"chr1\t5\t10\t\t3\n",
    b"chr1\t5\t10\ti d\t3\n", b"chr1\t5\t10\tid\t\n", b"chr1\t5\t10\tid\t1.2.3\n",
    b"chr1\t5\t10\tid\t1e5.0\n", b"chr1\t5\t10\tid\t1e5e3\n", b"chr1\t5\t10\tid\t1 2\n",
    b"chr1\t5\t10\tid\t1-2\n", b"chr1\t5\t10\tid\t1e+-2\n", b"chr1\t5\t10\tid\t1e2-\n",
    b"chr1\t5\t10\tid\t-15\trest\n", b"chr1\t5\t10\tid\t3x\n", b"chr1\t5\t10\tid\t1e5-\n",
]


@pytest.fixture(scope="module")
def check_bin(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("ck") / "ck")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe,
                    os.path.join(ROOT, "tests", "cpu", "check_main.cpp")], check=True)
    return exe


@pytest.fixture(scope="module")
def lib():
    subprocess.run(["make", "-s", "-j8", "lib", "oracle"], cwd=ROOT, check=True,
                   stdout=subprocess.DEVNULL)
    L = ctypes.CDLL(os.path.join(ROOT, "bedops_amd", "lib", "libbedgpu.so"))
    L.bg_check_message.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64]
    return L


def gpu_grammar_text(check_bin, lib, path, data, nf, rest):
    r = subprocess.run([check_bin, str(nf), str(rest), path], stdout=subprocess.PIPE)
    if r.returncode == 0:
        return b""
    row, code, off, ln = map(int, r.stdout.split())
    buf = ctypes.create_string_buffer(4096)
    assert lib.bg_check_message(data[off:off + ln], ln, code, nf, rest, buf, 4096) == 0
    return f"in {path}\n".encode() + buf.value + f"\nSee row: {row}".encode()


def oracle_text(path, nf, rest):
    r = subprocess.run([os.path.join(ROOT, "oracle", "build", "ec_oracle"), str(nf), str(rest), path],
                       stdout=subprocess.PIPE)
    return r.stdout


@pytest.mark.parametrize("nf,rest,cases", [(3, 0, CASES), (3, 1, CASES), (5, 1, CASES5 + CASES)])
def test_check_grammar_matches_oracle(check_bin, lib, tmp_path, nf, rest, cases):
    for i, data in enumerate(cases):
        p = str(tmp_path / f"c{i}.bed")
        with open(p, "wb") as f:
            f.write(data)
        assert gpu_grammar_text(check_bin, lib, p, data, nf, rest) == oracle_text(p, nf, rest), data


def test_check_random_mutations(check_bin, lib, tmp_path):
    rng = random.Random(9)
    alphabet = b"\t \n0123456789-+.eExchr#@\r"
    for trial in range(400):
        rows = sorted((rng.choice(["chr1", "chr2", "chr10"]), s, s + rng.randint(1, 30))
                      for s in rng.sample(range(1000), 12))
        data = bytearray("".join(f"{c}\t{s}\t{e}\tid{k}\t{k}\n" for k, (c, s, e) in enumerate(rows)).encode())
        for _ in range(rng.randint(0, 3)):
            data[rng.randrange(len(data))] = rng.choice(alphabet)
        data = bytes(data)
        p = str(tmp_path / "m.bed")
        with open(p, "wb") as f:
            f.write(data)
        for nf, rest in ((3, 0), (3, 1), (5, 1)):
            assert gpu_grammar_text(check_bin, lib, p, data, nf, rest) == oracle_text(p, nf, rest), (trial, data)
