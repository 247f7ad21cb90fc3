"""Two models of closest-features' scan with the reader cache, for the GPU's two kernels
(bedops_amd/csrc/bg_closest.hip):

- `run_seq`: one candidate at a time through the branch chain, as `cl_run` (the
  thread-per-chunk kernel) evaluates ClosestFeature.cpp:284-401;
- `run_wave`: the candidates of a ref row taken W at a time (W = 64 on the GPU), every piece
  of carried state computed as a prefix function of the window, as `cw_window`/`cw_run`
  (k_closest_wave) do.

tests/test_closest_wave_model.py checks that the two agree (left, right and the cache after
every row) on random nested inputs, and `run_seq` against the control-flow oracle
(oracle/closest_oracle.c) through its outputs.

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


def _window(C, b, cands, S, overlaps):
    """one window of candidate indices through the chain in prefix form (cw_window).
    S: dict of the carried state; returns (consumed, brk)"""
    n = len(cands)
    rows = [C[ci] for ci in cands]
    d = [dist(c, b) for c in rows]
    live = [x != MINUS for x in d]
    plus = [live[i] and d[i] == PLUS for i in range(n)]
    pos = [live[i] and d[i] > 0 and not plus[i] for i in range(n)]
    B = next((i for i in range(n) if plus[i] or pos[i]), n)
    act = [live[i] and i <= B for i in range(n)]
    plus = [plus[i] and act[i] for i in range(n)]  # (the rows after the break are not read)
    pos = [pos[i] and act[i] for i in range(n)]
    neg = [act[i] and d[i] < 0 for i in range(n)]
    ovl = [act[i] and d[i] == 0 and overlaps for i in range(n)]
    noov = [act[i] and d[i] == 0 and not overlaps for i in range(n)]
    hangL = [ovl[i] and rows[i][1] <= b[1] for i in range(n)]
    hangR = [ovl[i] and not hangL[i] and b[2] <= rows[i][2] for i in range(n)]
    inside = [ovl[i] and not hangL[i] and not hangR[i] for i in range(n)]
    half = [inside[i] and _half(rows[i], b) for i in range(n)]
    zs = [i for i in range(n) if hangL[i] or (inside[i] and not half[i])]
    ld0z = S["ld"] == 0
    Z = -1 if ld0z else (zs[0] if zs else n)
    ldz = [ld0z or i > Z for i in range(n)]
    in_c = [inside[i] and not half[i] and not ldz[i] for i in range(n)]
    in_b = [inside[i] and not half[i] and ldz[i] for i in range(n)]
    in_a = [inside[i] and half[i] and ldz[i] for i in range(n)]
    in_d = [inside[i] and half[i] and not ldz[i] for i in range(n)]
    pm, run = [], S["ld"]
    for i in range(n):  # exclusive prefix max of the negative distances, from the incoming ld
        pm.append(run)
        if neg[i]:
            run = max(run, d[i])
    newleft = [neg[i] and not ldz[i] and d[i] >= pm[i] for i in range(n)]
    dropL = [neg[i] and not newleft[i] for i in range(n)]
    rz = [any(hangR[j] or in_a[j] or in_d[j] for j in range(i)) for i in range(n)]
    firstR = [pos[i] and d[i] < (0 if rz[i] else S["rdist"]) for i in range(n)]
    farR = [pos[i] and not firstR[i] for i in range(n)]

    def last_before(flags, i):
        for j in range(i - 1, -1, -1):
            if flags[j]:
                return j
        return -1

    setleft = [newleft[i] or hangL[i] or in_c[i] for i in range(n)]
    lft = [cands[j] if j >= 0 else S["left"] for j in (last_before(setleft, i) for i in range(n))]
    lce = [rows[j][2] if j >= 0 else S["lce"] for j in (last_before(setleft, i) for i in range(n))]
    hasL = [x >= 0 for x in lft]
    lc_zero = [newleft[i] or hangL[i] or in_c[i] for i in range(n)]
    lc_one = [dropL[i] or in_a[i] or in_b[i] or (noov[i] and hasL[i]) for i in range(n)]
    lc_hasl = [plus[i] or firstR[i] or farR[i] or hangR[i] or in_d[i] for i in range(n)]
    lc_ev = [act[i] and (lc_zero[i] or lc_one[i] or lc_hasl[i]) for i in range(n)]
    lc_after = [False if lc_zero[i] else (True if lc_one[i] else hasL[i]) for i in range(n)]
    lci = [lc_after[j] if j >= 0 else S["lc"] for j in (last_before(lc_ev, i) for i in range(n))]
    setright = [firstR[i] or hangR[i] or in_a[i] or in_d[i] for i in range(n)]
    rgt = [cands[j] if j >= 0 else S["right"] for j in (last_before(setright, i) for i in range(n))]
    hasR = [x >= 0 for x in rgt]
    keepL = [act[i] and hasL[i] and not lci[i] and (plus[i] or firstR[i] or farR[i] or hangR[i] or in_d[i]
                                                    or noov[i] or dropL[i] or in_a[i] or in_b[i] or
                                                    (hangL[i] and not (lce[i] <= rows[i][2])))
             for i in range(n)]
    keepR = [act[i] and hasR[i] and (plus[i] or farR[i] or hangR[i] or in_a[i] or in_d[i]) for i in range(n)]
    keepC = [plus[i] or firstR[i] or farR[i] or in_b[i] or noov[i] for i in range(n)]
    resets = [i for i in range(n) if newleft[i] or in_c[i]]
    R = resets[-1] if resets else -1
    if R >= 0:
        S["kept"] = []
    for i in range(max(R, 0), n):
        if keepL[i]:
            S["kept"].append(lft[i])
        if keepR[i]:
            S["kept"].append(rgt[i])
        if keepC[i]:
            S["kept"].append(cands[i])
    # the state after the window
    if ld0z or zs:
        S["ld"] = 0
    else:
        S["ld"] = max([S["ld"]] + [d[i] for i in range(n) if neg[i]])
    L = last_before(setleft, n)
    if L >= 0:
        S["left"], S["lce"] = cands[L], rows[L][2]
    j = last_before(lc_ev, n)
    if j >= 0:
        S["lc"] = lc_after[j]
    j = last_before(setright, n)
    if j >= 0:
        S["right"] = cands[j]
    if B < n and firstR[B]:
        S["rdist"] = d[B]
    elif any(hangR[i] or in_a[i] or in_d[i] for i in range(n)):
        S["rdist"] = 0
    brk = B < n
    return (B + 1 if brk else n), brk


def run_wave(Q, C, overlaps=True, W=64):
    stack, fp, out, caches = [], 0, [], []
    for b in Q:
        S = {"ld": MINUS, "rdist": PLUS, "left": -1, "right": -1, "lce": 0, "lc": False, "kept": []}
        brk = eof = False
        while not brk:  # a window: the cache from the top, then file rows in the lanes left
            ns = min(W, len(stack))
            nf = min(W - ns, len(C) - fp)
            if ns + nf == 0:
                eof = True
                break
            cands = [stack[len(stack) - 1 - i] for i in range(ns)] + list(range(fp, fp + nf))
            used, brk = _window(C, b, cands, S, overlaps)
            if used <= ns:
                del stack[len(stack) - used:]
            else:
                del stack[len(stack) - ns:]
                fp += used - ns
        if eof and S["left"] >= 0 and not S["lc"]:
            S["kept"].append(S["left"])
        if eof and S["right"] >= 0:
            S["kept"].append(S["right"])
        stack.extend(reversed(S["kept"]))
        out.append((S["left"], S["right"]))
        caches.append((fp, tuple(stack)))
    return out, caches
