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
