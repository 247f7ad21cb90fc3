"""Cache-free model of closest-features' left/right choice (the form the GPU kernel
computes), checked against the control-flow oracle (oracle/closest_oracle.c) by
tests/test_oracle.py on random inputs.

For a query row b, scan the candidates of b's chromosome in sorted order, apply the
per-element rules of findDistances (ClosestFeature.cpp:300-397) as if every earlier
candidate were still visible, and stop at the first candidate strictly to the right.
"""
INF = float("inf")


def dist(c, b):
    """getDistance(c, b) for rows on the same chromosome (ClosestFeature.cpp:244-255)"""
    if c[1] <= b[0]:
        return -(b[0] - c[1] + 1)
    if b[1] <= c[0]:
        return c[0] - b[1] + 1
    return 0


def pick(cands, b, allow_overlaps=True):
    """cands: [(start, end)] sorted; b: (start, end). returns (left, right) indices or None"""
    left = right = None
    ld, rd = -INF, INF
    cen = (b[1] - 1.0 + b[0]) / 2.0
    for i, c in enumerate(cands):
        d = dist(c, b)
        if d < 0:
            if d >= ld:
                ld, left = d, i
        elif d > 0:
            if d < rd:
                rd, right = d, i
            break
        elif allow_overlaps:
            if c[0] <= b[0]:
                left, ld = i, 0
            elif b[1] <= c[1]:
                right, rd = i, 0
            else:
                ln = c[1] - c[0]
                prop = 0.0 if cen < c[0] else ((cen + 1 - c[0]) / ln if ln else INF)
                if ld == 0:
                    if prop < 0.5:
                        right, rd = i, 0
                elif prop >= 0.5:
                    left, ld = i, 0
                else:
                    right, rd = i, 0
    return left, right
