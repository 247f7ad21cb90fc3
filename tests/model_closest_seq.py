"""A model of closest-features' scan with the reader cache, as the GPU kernel evaluates it
(bedops_amd/csrc/bg_closest.hip): `run_seq` takes one candidate at a time through the branch
chain, as `cl_run` (k_closest_chunks, a thread per chunk of ref rows) evaluates
ClosestFeature.cpp:284-401. tests/test_closest_model.py checks it against the control-flow
oracle (oracle/closest_oracle.c) through its outputs. (Round 5's wave-per-chunk form, every
piece of carried state a prefix function of a 64-candidate window, was exact but slower on
the GPU, 20.5-23.1 vs 18 ms, and was removed in round 6.)

Rows are (chrom, start, end) with integer chrom ids; distances follow getDistance
(ClosestFeature.cpp:244-255): -inf / +inf for an earlier / later chromosome.
"""
MINUS = float("-inf")
PLUS = float("inf")


def dist(c, b):
    if c[0] != b[0]:
        return MINUS if c[0] < b[0] else PLUS
    if c[2] <= b[1]:
        return -((b[1] - c[2]) + 1)
    if b[2] <= c[1]:
        return (c[1] - b[2]) + 1
    return 0


def _half(c, b):
    cen = ((b[2]) - 1.0 + b[1]) / 2.0
    cst = float(c[1])
    prop = 0.0 if cen < cst else (cen + 1 - cst) / float(c[2] - c[1])
    return prop < 0.5


def run_seq(Q, C, overlaps=True):
    """cl_run over every ref row: returns [(left, right)] and the cache after each row"""
    stack, fp, out, caches = [], 0, [], []
    for b in Q:
        ld, rdist, left, right, lce, lc = MINUS, PLUS, -1, -1, 0, False
        kept = []

        def step(ci):
            nonlocal ld, rdist, left, right, lce, lc, kept
            c = C[ci]
            d = dist(c, b)
            if d == MINUS:
                return False
            hasL, hasR = left >= 0, right >= 0
            plus = d == PLUS
            neg = d < 0
            pos = d > 0 and not plus
            newleft = neg and d >= ld
            dropL = neg and not newleft
            firstR = pos and d < rdist
            farR = pos and not firstR
            ovl = d == 0 and overlaps
            noov = d == 0 and not overlaps
            hangL = ovl and c[1] <= b[1]
            hangR = ovl and not hangL and b[2] <= c[2]
            inside = ovl and not hangL and not hangR
            half = _half(c, b) if inside else False
            in_a = inside and ld == 0 and half
            in_b = inside and ld == 0 and not half
            in_c = inside and ld != 0 and not half
            in_d = inside and ld != 0 and half
            reset = newleft or in_c
            keepL = hasL and not lc and (plus or firstR or farR or hangR or in_d or noov or dropL or in_a
                                         or in_b or (hangL and not (lce <= c[2])))
            keepR = hasR and (plus or farR or hangR or in_a or in_d)
            keepC = plus or firstR or farR or in_b or noov
            if reset:
                kept = []
            if keepL:
                kept.append(left)
            if keepR:
                kept.append(right)
            if keepC:
                kept.append(ci)
            lc_hasl = plus or firstR or farR or hangR or in_d
            lc_one = dropL or in_a or in_b or (noov and hasL)
            lc_zero = newleft or hangL or in_c
            lc = False if lc_zero else (True if lc_one else (hasL if lc_hasl else lc))
            if newleft or hangL or in_c:
                left, lce = ci, c[2]
            ld = d if newleft else (0 if (hangL or in_c) else ld)
            if firstR or hangR or in_a or in_d:
                right = ci
            rdist = d if firstR else (0 if (hangR or in_a or in_d) else rdist)
            return plus or pos

        brk = False
        while stack and not brk:
            brk = step(stack.pop())
        eof = False
        while not brk:
            if fp >= len(C):
                eof = True
                break
            fp += 1
            brk = step(fp - 1)
        if eof and left >= 0 and not lc:
            kept.append(left)
        if eof and right >= 0:
            kept.append(right)
        stack.extend(reversed(kept))
        out.append((left, right))
        caches.append((fp, tuple(stack)))
    return out, caches
