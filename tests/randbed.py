"""Seeded random sorted-BED generators for differential tests (oracle vs GPU).

Shapes exercise what the reference's sweep is sensitive to: several chromosomes in
strcmp order (chr1 < chr10 < chr2 < chrX), duplicates, nesting, touching rows,
zero-length rows, extra columns, and empty files.
"""
import random

CHROMS = ["chr1", "chr10", "chr2", "chrX"]


def rows(rng, n, chroms=CHROMS, span=2000, maxlen=120, zero_frac=0.0):
    out = []
    for _ in range(n):
        c = rng.choice(chroms)
        s = rng.randrange(span)
        if zero_frac and rng.random() < zero_frac:
            ln = 0
        else:
            ln = rng.randint(1, maxlen) if rng.random() < 0.9 else rng.randint(1, 6 * maxlen)
        out.append((c, s, s + ln))
    out.sort(key=lambda r: (r[0].encode(), r[1], r[2]))
    return out


def text(rs, rest=None, rng=None):
    lines = []
    for i, (c, s, e) in enumerate(rs):
        tail = ""
        if rest == "cols":
            tail = f"\tid{i}\t{rng.randint(0, 999) if rng else i % 1000}\t+"
        elif rest == "bed5":
            tail = f"\tid{i}\t{rng.randint(0, 999) if rng else i % 1000}"
        lines.append(f"{c}\t{s}\t{e}{tail}\n")
    return "".join(lines)


def write(path, content):
    with open(path, "w") as f:
        f.write(content)
    return path
