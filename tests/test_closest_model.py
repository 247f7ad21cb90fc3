"""The one-candidate-at-a-time form of closest-features' scan (cl_run in
bedops_amd/csrc/bg_closest.hip, modelled in tests/model_closest_seq.py) against the
control-flow oracle (oracle/closest_oracle.c) through its printed output, on random nested
inputs; and the kernel's integer centroid test against the reference's double form."""
import random
import subprocess

import model_closest_seq as M


def rand_rows(rng, n, chroms, span, maxlen, nested=0.0):
    rows = []
    for _ in range(n):
        ch = rng.randrange(chroms)
        s = rng.randrange(span)
        ln = rng.randint(1, maxlen) if rng.random() > nested else rng.randint(maxlen, 6 * maxlen)
        rows.append((ch, s, s + ln))
    rows.sort()
    return rows


CASES = [  # (seed, query rows, candidate rows, chroms, span, maxlen, nested)
    (1, 60, 300, 1, 2000, 40, 0.0),
    (2, 80, 400, 2, 3000, 80, 0.1),
    (3, 50, 600, 1, 1500, 30, 0.3),
    (4, 120, 200, 3, 5000, 200, 0.2),
    (5, 40, 900, 1, 2500, 15, 0.05),
]


def _bed(rows, tag):
    return "".join(f"chr{c + 1}\t{s}\t{e}\t{tag}{i}\n" for i, (c, s, e) in enumerate(rows))


def test_sequential_form_matches_oracle(oracle_bin, tmp_path):
    for seed, nq, nc, chroms, span, maxlen, nested in CASES[:3]:
        rng = random.Random(100 + seed)
        Q = rand_rows(rng, nq, chroms, span, maxlen, nested)
        C = rand_rows(rng, nc, chroms, span, maxlen, nested)
        q, c = tmp_path / "q.bed", tmp_path / "c.bed"
        q.write_text(_bed(Q, "q"))
        c.write_text(_bed(C, "c"))
        for overlaps in (True, False):
            args = [] if overlaps else ["--no-overlaps"]
            out = subprocess.run([oracle_bin["closest"], "--no-ref", *args, str(q), str(c)],
                                 stdout=subprocess.PIPE, check=True).stdout.decode().splitlines()
            res, _ = M.run_seq(Q, C, overlaps)
            want = []
            for left, right in res:
                parts = [_bed([C[x]], "c").replace("c0", f"c{x}").rstrip("\n") if x >= 0 else "NA"
                         for x in (left, right)]
                want.append("|".join(parts))
            assert out == want, (seed, overlaps)


def _half_double(bs, be, cs, ce):
    cen = (be - 1.0 + bs) / 2.0  # ClosestFeature.cpp:227-239 in doubles
    prop = 0.0 if cen < cs else (cen + 1 - cs) / float(ce - cs)
    return prop < 0.5


def _half_int(bs, be, cs, ce):  # bg_closest.hip: cl_run
    return 2 * cs > bs + be - 1 or bs + be + 1 - 2 * cs < ce - cs


def test_integer_centroid_test_equals_double():
    """the kernels' integer form of the centroid proportion test equals the reference's
    double computation: random rows, rows at the proportion's boundary (N = L - 1, L, L + 1),
    and coordinates near 2^40 (the key space's limit)"""
    rng = random.Random(11)
    cases = []
    for _ in range(200000):
        top = rng.choice([100, 10**4, 10**9, 1 << 40])
        bs = rng.randrange(top)
        be = bs + rng.randint(1, min(top, 10**6))
        cs = rng.randint(bs, be)  # an "inside" candidate starts inside the ref row
        ce = cs + rng.randint(1, min(top, 10**6))
        cases.append((bs, be, cs, ce))
    for _ in range(50000):  # at the boundary: N = bs + be + 1 - 2cs vs L = ce - cs
        bs = rng.randrange(1 << 40)
        be = bs + rng.randint(1, 10**6)
        cs = rng.randint(bs, be)
        n = bs + be + 1 - 2 * cs
        for L in (n - 1, n, n + 1):
            if L >= 1:
                cases.append((bs, be, cs, cs + L))
    for bs, be, cs, ce in cases:
        assert _half_int(bs, be, cs, ce) == _half_double(bs, be, cs, ce), (bs, be, cs, ce)
