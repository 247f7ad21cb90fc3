"""The wave form of closest-features' scan (k_closest_wave, bedops_amd/csrc/bg_closest.hip)
against the one-candidate-at-a-time form (cl_run): same left/right and the same reader cache
after every ref row, on random nested inputs, windows of 64 and of a few candidates (so every
piece of carried state crosses window edges); and the sequential form against the
control-flow oracle (oracle/closest_oracle.c) through its printed output."""
import random
import subprocess

import model_closest_wave as M


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


def test_wave_form_equals_sequential_form():
    for seed, nq, nc, chroms, span, maxlen, nested in CASES:
        rng = random.Random(seed)
        Q = rand_rows(rng, nq, chroms, span, maxlen, nested)
        C = rand_rows(rng, nc, chroms, span, maxlen, nested)
        for overlaps in (True, False):
            want = M.run_seq(Q, C, overlaps)
            for W in (64, 5, 3, 1):
                got = M.run_wave(Q, C, overlaps, W)
                assert got[0] == want[0], (seed, overlaps, W)
                assert got[1] == want[1], (seed, overlaps, W)


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
