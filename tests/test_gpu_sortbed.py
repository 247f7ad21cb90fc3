"""sort-bed on the GPU (bedops_amd/csrc/bg_sortbed.hip, bedops_amd/bin/sort-bed) against the
oracle restatement of applications/bed/sort-bed/src (oracle/sortbed_oracle.c): unsorted
multi-file inputs with tab/space separators, remainders, duplicates, headers and blank
lines are sorted byte-identically; every line error gives the reference's message and exit
status. The reference ships no sort-bed output fixtures (its test only checks the exit code,
applications/bed/sort-bed/test/sort-chr-test.bash), so parity is against the oracle."""
import os
import random
import subprocess

import pytest

pytestmark = pytest.mark.gpu

NAMES = ["chr1", "chr10", "chr2", "chrX", "chrY", "chr1_random", "scaffold_7", "chrM", "1", "10", "2"]


def _rand_file(rng, n):
    lines = []
    if rng.random() < 0.3:
        lines.append(rng.choice(["track name=x", "browser position chr1", "# comment", "@hdr"]))
    for _ in range(n):
        c = rng.choice(NAMES)
        s = rng.randrange(0, 5000)
        e = s + rng.randint(1, 60)
        sep = [rng.choice(["\t", " "]) for _ in range(3)]
        st = str(s) if rng.random() < 0.9 else "0" * rng.randint(1, 3) + str(s)
        ln = f"{c}{sep[0]}{st}{sep[1]}{e}"
        r = rng.random()
        if r < 0.3:
            ln += f"{sep[2]}id{rng.randint(0, 9)}"
        elif r < 0.5:
            ln += f"{sep[2]}{rng.choice(['x', 'y', 'id1'])}\t{rng.randint(0, 99)}\t+"
        elif r < 0.55:
            ln += sep[2] + "  "
        lines.append(ln)
        if rng.random() < 0.02:
            lines.append("")
    if lines and rng.random() < 0.5:
        lines = lines * rng.randint(1, 2)  # duplicate rows
        lines = [ln for ln in lines if not (ln.startswith(("track", "browser", "#", "@")))]
    rng.shuffle(lines)
    return "\n".join(lines) + ("\n" if rng.random() < 0.9 or not lines else "\t" if lines else "")


def _run(exe, files):
    return subprocess.run([exe, *files], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=120)


def test_sortbed_random_vs_oracle(gpu_bin, oracle_bin, tmp_path):
    rng = random.Random(11)
    for trial in range(40):
        files = []
        for f in range(rng.choice([1, 1, 2, 3])):
            p = tmp_path / f"t{trial}_{f}.bed"
            p.write_text(_rand_file(rng, rng.choice([0, 1, 5, 100, 3000])))
            files.append(str(p))
        want = _run(oracle_bin["sortbed"], files)
        got = _run(gpu_bin["sortbed"], files)
        assert (got.returncode, got.stdout, got.stderr) == (want.returncode, want.stdout, want.stderr), trial


BAD = ["chr1\t5\t3\n", " chr1\t1\t2\n", "chr1\n", "chr1\t5\n", "chr1\t1234567890123\t1234567890124\n",
       "chr1\t\t5\n", "chr1\t5x\t9\n", "chr1\t5\t9", "chr1\t5\t99999999999999\n", "chr1\t5\t\t9\n",
       "chr1\t5\t9z\n", "chr1\t5\t5\n", "c" * 130 + "\t1\t2\n", "chr1\t1\t2\t" + "i" * 17000 + "\n",
       "chr1\t1\t2\r\n"]


@pytest.mark.parametrize("k", range(len(BAD)))
def test_sortbed_errors_vs_oracle(gpu_bin, oracle_bin, tmp_path, k):
    p = tmp_path / "bad.bed"
    p.write_text("chr1\t1\t2\n#late comment is data\n" if k == 99 else "chr2\t1\t2\n\n" + BAD[k] + "chr3\t4\t5\n")
    want = _run(oracle_bin["sortbed"], [str(p)])
    got = _run(gpu_bin["sortbed"], [str(p)])
    assert want.returncode != 0
    assert (got.returncode, got.stdout, got.stderr) == (want.returncode, want.stdout, want.stderr)


def test_sortbed_large_vs_oracle(gpu_bin, oracle_bin, bedgen, tmp_path):
    """1M rows of two generated files, shuffled line order"""
    rng = random.Random(3)
    files = []
    for seed in (42, 43):
        txt = subprocess.run([bedgen, "500000", str(seed), "--bed5"], stdout=subprocess.PIPE,
                             check=True).stdout.splitlines(keepends=True)
        rng.shuffle(txt)
        p = tmp_path / f"g{seed}.bed"
        p.write_bytes(b"".join(txt))
        files.append(str(p))
    want = _run(oracle_bin["sortbed"], files)
    got = _run(gpu_bin["sortbed"], files)
    assert want.returncode == 0
    assert got.returncode == 0 and got.stdout == want.stdout


def test_sortbed_long_tie_runs_vs_oracle(gpu_bin, oracle_bin, tmp_path):
    """1e5 rows at one coordinate with random rests (amplicon / duplicate-heavy data), rests
    that share long prefixes (several 8-byte refinement rounds) and rows without a rest:
    ordered like the oracle, in seconds (the tie order is radix refinement, not per-run
    insertion)"""
    import time
    rng = random.Random(123)
    lines = [f"chr2\t700\t900\tread{rng.randint(0, 10 ** 9)}\t{rng.randint(0, 60)}" for _ in range(100000)]
    lines += [f"chr2\t700\t900\tshared_prefix_0123456789_{rng.randint(0, 999):03d}" for _ in range(3000)]
    lines += ["chr2\t700\t900"] * 50 + [f"chr1\t5\t9\tx{k % 7}" for k in range(20000)]
    rng.shuffle(lines)
    p = tmp_path / "ties.bed"
    p.write_text("\n".join(lines) + "\n")
    want = subprocess.run([oracle_bin["sortbed"], str(p)], stdout=subprocess.PIPE, check=True).stdout
    t0 = time.time()
    got = subprocess.run([gpu_bin["sortbed"], str(p)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         timeout=120)
    dt = time.time() - t0
    assert got.returncode == 0, got.stderr
    assert got.stdout == want
    assert dt < 30, dt
