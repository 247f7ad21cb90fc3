"""The row loader (k_parse_rv: two waves per 8 KiB tile, one per 4 KiB sub-tile) on the texts
that stress its structure: lines crossing the sub-tile and tile edges, lines longer than a
sub-tile (a wave with no line of its own), several chromosome runs in one sub-tile, chromosome
names of 9-16 and of more than 16 bytes sharing their first 16, numbers past 9 digits, odd
spacing, and BED5 scores of every spelling. Outputs (which print the rows' coordinates, rest
columns and scores back) are compared byte for byte with the oracle; sort errors at the
sub-tile edges must name the same data line the reference's order implies."""
import os
import random
import subprocess
import tempfile
import zlib

import pytest

pytestmark = pytest.mark.gpu

SHORT = ["chr1", "chr2", "chrX"]
MID = ["chrUn_KI27", "chrUn_KI270302", "chrUn_KI270303v1"]          # 9..16 bytes
LONG = ["chrUn_KI270302v1_randomA", "chrUn_KI270302v1_randomB",   # > 16, same first 16
        "chrUn_KI270302v1_random_long_name_x"]


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
    r = subprocess.run([binary] + args + paths, stdout=subprocess.PIPE, stderr=subprocess.PIPE, check=True)
    return r.stdout


SCORES = ["17", "0", "42.5", "-3", "+2.25", "1e3", "0.000", "12.000", "3.14159265358979", "007.25",
          "123456789012345678901234", "9007199254740993", "2.5e-2", ".5", "5."]


def hard_rows(rng, n, chroms, big_coords=False, long_rest=0.0, bed5=False, runs=30):
    """sorted rows: chromosomes in runs of random length, coordinates past 9 digits when
    big_coords, some rest columns longer than a 4 KiB sub-tile, random spacing"""
    chroms = sorted(set(chroms), key=lambda c: c.encode())
    per = [0] * len(chroms)
    for _ in range(n):
        per[min(int(rng.expovariate(1.0 / max(1, len(chroms) / 3))), len(chroms) - 1)] += 1
    out = []
    for c, m in zip(chroms, per):
        s = rng.randrange(10 ** 10) if big_coords and rng.random() < 0.5 else rng.randrange(1000)
        run = []
        for _ in range(m):
            s += rng.choice([0, 0, 1, 3, 40, 700])
            run.append((c, s, s + rng.choice([0, 1, 5, 60, 2000])))
        out += sorted(run, key=lambda r: (r[1], r[2]))
    lines = []
    for i, (c, s, e) in enumerate(out):
        sep = rng.choice(["\t"] * 8 + [" ", "  ", "\t \t"])
        lead = " " if rng.random() < 0.01 else ""
        line = f"{lead}{c}{sep}{s}{sep}{e}"
        if bed5:
            line += f"\tid{i % 97}\t{rng.choice(SCORES) if rng.random() < 0.3 else rng.randint(0, 999)}"
            if rng.random() < 0.1:
                line += "\tx" * rng.randint(1, 4)
        elif rng.random() < 0.5:
            line += f"\tid{i}\t{rng.randint(0, 999)}\t+"
        if rng.random() < long_rest:
            line += "\t" + "y" * rng.choice([300, 4200, 9000])
        lines.append(line + "\n")
    return "".join(lines).encode()


SHAPES = {  # name: (rows, chromosomes, big coordinates, share of long rest columns)
    "short_names": (6000, SHORT, False, 0.0),
    "mid_names": (6000, MID, False, 0.0),
    "long_names": (4000, LONG + SHORT, False, 0.0),
    "many_runs": (6000, [f"chr{k}" for k in range(60)], False, 0.0),
    "big_coords": (5000, SHORT + MID, True, 0.0),
    "long_lines": (2500, SHORT, False, 0.03),
}


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_row_columns_through_bedmap_vs_oracle(eng, oracle_bin, shape):
    """ref rows with rest (--echo), map rows BED5 with rest (--echo-map): every column the
    loader writes is printed back"""
    n, chroms, big, lr = SHAPES[shape]
    rng = random.Random(zlib.crc32(shape.encode()))
    ref = hard_rows(rng, n // 3, chroms, big, lr)
    mp = hard_rows(rng, n, chroms, big, lr, bed5=True)
    with tempfile.TemporaryDirectory() as td:
        for ops in (["echo", "count", "sum", "min", "max"], ["echo-map", "echo-map-score", "mean"]):
            want = run_oracle(oracle_bin["bedmap"], [f"--{o}" for o in ops], [ref, mp], td)
            assert eng.bedmap(ops, ref, mp) == want, (shape, ops)


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_row_columns_through_closest_and_element_of_vs_oracle(eng, oracle_bin, shape):
    n, chroms, big, lr = SHAPES[shape]
    rng = random.Random(zlib.crc32(("ce", shape).__repr__().encode()))
    a = hard_rows(rng, n, chroms, big, lr)
    b = hard_rows(rng, n // 2, chroms, big, lr)
    with tempfile.TemporaryDirectory() as td:
        want = run_oracle(oracle_bin["closest"], ["--closest", "--dist"], [a, b], td)
        assert eng.closest(a, b, shortest=True, dist=True) == want, shape
        want = run_oracle(oracle_bin["bedops"], ["-e", "1"], [a, b], td)
        assert eng.bedops("-e", [a, b], spec="1") == want, shape


def _plain(n, c="chr1"):
    return [f"{c}\t{100 + 7 * i}\t{130 + 7 * i}\n".encode() for i in range(n)]


@pytest.mark.parametrize("edge", [4096, 8192, 12288])
def test_unsorted_rows_at_subtile_edges_name_the_line(eng, edge):
    """two adjacent rows swapped around a sub-tile / tile edge: the error names the second
    row of the pair (wave 1's first line against wave 0's last, k_check_bounds across tiles)"""
    from bedops_amd import BedgpuError
    lines = _plain(1500)
    offs, o = [], 0
    for ln in lines:
        offs.append(o)
        o += len(ln)
    near = [k for k in range(len(lines) - 1) if abs(offs[k + 1] - edge) <= 40]
    assert near
    good = b"".join(_plain(50))
    for k in near:
        bad = lines[:k] + [lines[k + 1], lines[k]] + lines[k + 2:]
        with pytest.raises(BedgpuError) as ei:
            eng.bedmap(["count"], b"".join(bad), good)
        assert ei.value.code == -3
        assert f"data line {k + 2}:" in str(ei.value), (k, str(ei.value))


def test_long_names_sharing_16_bytes_out_of_order_are_an_error(eng):
    """one row of B inside a long run of A (names equal in their first 16 bytes and length),
    away from the tile edges the run records look at: the lean path must not take it for A"""
    from bedops_amd import BedgpuError
    a, b = LONG[0], LONG[1]
    rows = [f"{a}\t{i}\t{i + 5}\n" for i in range(1500)]
    rows[100] = f"{b}\t{100}\t{105}\n"
    with pytest.raises(BedgpuError) as ei:
        eng.bedmap(["count"], "".join(rows).encode(), b"chr1\t1\t2\n")
    assert ei.value.code == -3


def test_short_lines_redo_with_the_wide_parser(eng, oracle_bin):
    """sub-tiles of more than 512 lines (lines under 8 bytes): the load is redone with k_parse"""
    rows = "".join(f"c\t{i}\t{i + 1}\n" for i in range(3000)).encode()  # 8-9 byte lines
    tiny = "".join(f"c\t{i % 10}\t{i % 10 + 1}\n" for i in range(3000))
    tiny = "".join(sorted(tiny.splitlines(keepends=True), key=lambda s: (int(s.split()[1]), int(s.split()[2])))).encode()
    with tempfile.TemporaryDirectory() as td:
        for ref in (rows, tiny):
            want = run_oracle(oracle_bin["bedmap"], ["--echo", "--count"], [ref, rows], td)
            assert eng.bedmap(["echo", "count"], ref, rows) == want
