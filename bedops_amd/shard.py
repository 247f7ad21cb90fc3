"""Per-chromosome sharding across GPUs and the reassembly of sorted output on rank 0.

Every operation on this path is chromosome-local: all comparisons start with the chromosome
(`interfaces/general-headers/algorithm/bed/BedCompare.hpp:42-43`,
`BedDistances.hpp:99-100`), so per-chromosome outputs concatenated in strcmp order are the
whole output (the reference's own documented scale-out, `docs/.../bedops.rst:721-726`).

One process per GPU. `assign()` gives each chromosome to one rank (longest processing time
on a weight such as its row count); each rank runs the engine on its chromosomes only (no
input exchange); `gather_text()` is the one exchange of the path: rank 0 receives every
rank's formatted bytes, chromosome by chromosome, straight into its place in the final
strcmp-ordered buffer (sizes via all_gather, then point-to-point send/recv: RCCL over xGMI
with the "nccl" backend, gloo on CPU for the tests).
"""


def assign(weights, world):
    """chrom -> rank. weights: {chrom: weight}. Heaviest first onto the least-loaded rank
    (ties: lowest rank; equal weights: strcmp order of the name), deterministic on every
    rank. Returns (owner, load)."""
    load = [0] * world
    owner = {}
    for name in sorted(weights, key=lambda c: (-weights[c], _key(c))):
        r = min(range(world), key=lambda k: (load[k], k))
        owner[name] = r
        load[r] += weights[name]
    return owner, load


def _key(name):
    return name.encode() if isinstance(name, str) else bytes(name)


def strcmp_order(names):
    return sorted(names, key=_key)


def gather_text(dist, text, spans, names, owner, rank, world):
    """Reassemble sorted output on rank 0.

    text:   this rank's formatted bytes (uint8 torch tensor, on the collective's device).
    spans:  {chrom: (begin, end)} byte range of each of this rank's chromosomes in `text`
            (chromosomes absent from the output may be omitted).
    names:  every chromosome of the job (any order); owner: chrom -> rank.
    Returns the whole output (uint8 tensor) on rank 0, None elsewhere.
    """
    import torch

    dev = text.device
    order = strcmp_order(names)
    idx = {c: i for i, c in enumerate(order)}
    # byte length of every chromosome's output, known to all ranks
    mine = torch.zeros(len(order), dtype=torch.int64)
    for c, (a, b) in spans.items():
        if owner[c] != rank:
            raise ValueError(f"rank {rank} has output for {c!r}, owned by rank {owner[c]}")
        mine[idx[c]] = b - a
    mine = mine.to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    lens = [0] * len(order)
    for i, c in enumerate(order):
        lens[i] = int(parts[owner[c]][i].item())

    if rank != 0:
        ops = []
        for c in order:  # sends in strcmp order; rank 0 posts its receives in the same order
            if owner[c] == rank and lens[idx[c]] > 0:
                a, b = spans[c]
                ops.append(dist.P2POp(dist.isend, text[a:b], 0))
        _run(dist, ops)
        return None

    total = sum(lens)
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    ops = []
    pos = 0
    for i, c in enumerate(order):
        n = lens[i]
        if n > 0:
            if owner[c] == 0:
                a, b = spans[c]
                out[pos:pos + n].copy_(text[a:b])
            else:
                ops.append(dist.P2POp(dist.irecv, out[pos:pos + n], owner[c]))
        pos += n
    _run(dist, ops)
    return out[:total]


def _run(dist, ops):
    # one grouped launch of all point-to-point transfers (ncclGroupStart/End under RCCL)
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()


def spans_from_text(data):
    """{chrom: (begin, end)} of a sorted BED text (bytes), by scanning line starts; used
    where no device-side chromosome spans exist (tests)."""
    spans = {}
    pos = 0
    n = len(data)
    cur, beg = None, 0
    while pos < n:
        nl = data.find(b"\n", pos)
        nl = n if nl < 0 else nl
        line = data[pos:nl]
        t = line.split(None, 1)[0].decode() if line.strip() else None
        if t != cur:
            if cur is not None:
                spans[cur] = (beg, pos)
            cur, beg = t, pos
        pos = nl + 1
    if cur is not None:
        spans[cur] = (beg, min(pos, n))
    return spans
