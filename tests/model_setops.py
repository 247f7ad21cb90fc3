"""Pure-Python model of the GPU formulation (bedops_amd/csrc/bg_setops.hip).

Not the oracle: this restates what the kernels compute (running-max components,
per-element merge-path pieces, gap enumeration for difference, prefix-sum
element-of) so the formulation itself can be checked against the oracle on the CPU,
without a GPU. Keys are (chrom_rank << 40) | coordinate, as in HBM.
"""
SHIFT = 40


def keyed(rows, names):
    rank = {n: i for i, n in enumerate(sorted(set(names), key=lambda s: s.encode()))}
    return [((rank[c] << SHIFT) | s, (rank[c] << SHIFT) | e) for c, s, e in rows], rank


def components(iv):
    out = []
    run = None
    for s, e in iv:
        if run is None or s > run:
            out.append([s, e])
        else:
            out[-1][1] = max(out[-1][1], e)
        run = e if run is None else max(run, e)
    return [tuple(x) for x in out]


def merged(x, y, x_first):
    """merge by start; ties: X first if x_first else Y first"""
    i = j = 0
    out = []
    while i < len(x) or j < len(y):
        if i < len(x) and (j >= len(y) or (x[i][0] <= y[j][0] if x_first else x[i][0] < y[j][0])):
            out.append(("x", i)); i += 1
        else:
            out.append(("y", j)); j += 1
    return out


def intersect2(x, y):
    out = []
    lastx = lasty = None
    for w, k in merged(x, y, x_first=False):
        s, e = (x if w == "x" else y)[k]
        partner = lasty if w == "x" else lastx
        if w == "x":
            lastx = e
        else:
            lasty = e
        if partner is not None and min(e, partner) > s:
            out.append((s, min(e, partner)))
    return out


def difference2(r, o):
    out = []
    i = j = 0
    while i < len(r) or j < len(o):
        if i < len(r) and (j >= len(o) or r[i][0] < o[j][1]):
            a, b = r[i]
            if j >= len(o) or o[j][0] >= b:
                out.append((a, b))
            elif o[j][0] > a:
                out.append((a, o[j][0]))
            i += 1
        else:
            if i > 0:
                oe, rb = o[j][1], r[i - 1][1]
                if rb > oe:
                    out.append((oe, min(rb, o[j + 1][0]) if j + 1 < len(o) else rb))
            j += 1
    return out


def union_components(files):
    acc = components(files[0])
    for f in files[1:]:
        z = sorted(acc + components(f), key=lambda t: t[0])
        acc = components(z)
    return acc


def element_of(ref, comps, thres, use_pct, invert):
    import bisect
    starts = [c[0] for c in comps]
    ends = [c[1] for c in comps]
    P = [0]
    for s, e in comps:
        P.append(P[-1] + (e - s))
    keep = []
    for idx, (s, e) in enumerate(ref):
        lo = bisect.bisect_right(ends, s)
        if lo >= len(comps):
            k = invert
        else:
            hi = bisect.bisect_left(starts, e)
            ov = 0
            if lo < hi:
                ov = P[hi] - P[lo] - max(0, s - starts[lo]) - max(0, ends[hi - 1] - e)
            rng = float(e - s)
            if use_pct:
                is_el = (float(ov) / rng >= thres) if rng != 0 else False
            else:
                is_el = float(ov) >= thres
            k = (not is_el) if invert else is_el
        if k:
            keep.append(idx)
    return keep


def intersect_zero_len(files):
    """--intersect including nextIntersectLine's zero-length prints (Bedops.cpp:1105-1181),
    as k_zi_mark / k_zi_replay / k_zi_place compute it: the non-empty output is the set
    intersection; zero-length prints come from replaying the calls that follow the
    canonical state after O[m-1] (every head = first piece ending after O[m-1].s, the
    marker file's = first piece ending after O[m-1].e) until O[m] is printed again."""
    import bisect
    P = [components(f) for f in files]
    normal = P[0]
    for f in P[1:]:
        normal = intersect2(normal, f)
    nf = len(P)
    ends = [[p[1] for p in Pi] for Pi in P]

    def call(h):
        if any(h[j] >= len(P[j]) for j in range(nf)):
            return None
        mj = 0
        for j in range(1, nf):
            if P[j][h[j]][0] > P[mj][h[mj]][0]:
                mj = j
        cur = P[mj][h[mj]]
        i, marker, min_e = 0, -1, None
        while i < nf:
            h[i] = max(h[i], bisect.bisect_right(ends[i], cur[0]))
            if h[i] >= len(P[i]):
                return None
            p = P[i][h[i]]
            if p[0] >= cur[1]:
                cur, i, marker, min_e = p, 0, -1, None
                continue
            cur = (max(cur[0], p[0]), min(cur[1], p[1]))
            if min_e is None or p[1] < min_e:
                min_e, marker = p[1], i
            i += 1
        h[marker] += 1
        return cur

    zs = sorted({p[0] for Pi in P for p in Pi if p[0] == p[1]})
    starts = [o[0] for o in normal]
    extra = {}
    for m in sorted({bisect.bisect_left(starts, t) for t in zs}):
        if m == 0:
            h = [0] * nf
        else:
            s, e = normal[m - 1]
            h = [bisect.bisect_right(ends[j], s) for j in range(nf)]
            q = next(j for j in range(nf) if h[j] < len(P[j]) and P[j][h[j]][1] == e)
            h[q] += 1
        em = []
        while True:
            c = call(h)
            if c is None:
                break
            if c[0] == c[1]:
                em.append(c)
                continue
            assert m < len(normal) and c == normal[m]
            break
        extra[m] = em
    out = []
    for m in range(len(normal) + 1):
        out += extra.get(m, [])
        if m < len(normal):
            out.append(normal[m])
    return out


def bedmap_zero_len_window(ref, mp):
    """Sweep-window membership of each map row with zero-length rows present, as
    k_mz_walk / k_mz_member compute it (bg_map.hip): map row j is a window member of
    reference rows [zin[j], zout[j]). ref, mp: keyed (start, end), start-sorted."""
    import bisect
    nr, nm = len(ref), len(mp)
    ms_ = [m[0] for m in mp]
    zmap = [j for j, m in enumerate(mp) if m[0] == m[1]]

    def next_zero(x):
        k = bisect.bisect_left(zmap, x)
        return zmap[k] if k < len(zmap) else nm
    P, p = [], 0
    for s, e in ref:
        c = bisect.bisect_right(ms_, s)
        a = bisect.bisect_left(ms_, e) if e > s else c
        p = min(max(p, a), next_zero(max(p, c)))
        P.append(p)
    zref = [i for i, r in enumerate(ref) if r[0] == r[1]]
    zt = [ref[i][0] for i in zref]
    zin, zout = [], []
    for j, (ms, me) in enumerate(mp):
        i = bisect.bisect_right(P, j)
        added = i < nr and min(ref[i][1], me) > max(ref[i][0], ms)
        zin.append(i if added else None)
        k = max(bisect.bisect_right(zref, i), bisect.bisect_right(zt, ms))
        zout.append(zref[k] if k < len(zref) else nr)
    return zin, zout
