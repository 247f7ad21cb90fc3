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
with the "nccl" backend, gloo on CPU for the tests). gather_text_async posts the transfers
and returns, so a pipeline can compute the next batch while this one moves.
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


class PendingGather:
    """Transfers of one reassembly in flight; wait() returns the output on rank 0."""

    def __init__(self, works, out, keep):
        self.works, self.out, self._keep = works, out, keep

    def wait(self):
        for w in self.works:
            w.wait()
        self.works, self._keep = [], None
        return self.out


def gather_text_async(dist, text, spans, names, owner, rank, world, size_group=None):
    """Post the reassembly of sorted output on rank 0 and return without waiting.

    text:   this rank's formatted bytes (uint8 torch tensor, on the collective's device).
    spans:  {chrom: (begin, end)} byte range of each of this rank's chromosomes in `text`
            (chromosomes absent from the output may be omitted).
    names:  every chromosome of the job (any order); owner: chrom -> rank.
    size_group: optional process group (e.g. gloo, CPU tensors) for the per-chromosome
            byte counts, so that exchanging them never queues behind earlier transfers.
    The bytes land chromosome by chromosome straight into their place in rank 0's output.
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
    if size_group is None:
        mine = mine.to(dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=size_group)
    parts = [p.cpu() for p in parts]
    lens = [int(parts[owner[c]][i]) for i, c in enumerate(order)]

    if rank != 0:
        ops = []
        for c in order:  # sends in strcmp order; rank 0 posts its receives in the same order
            if owner[c] == rank and lens[idx[c]] > 0:
                a, b = spans[c]
                ops.append(dist.P2POp(dist.isend, text[a:b], 0))
        return PendingGather(_post(dist, ops), None, text)

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
    return PendingGather(_post(dist, ops), out[:total], text)


def gather_text(dist, text, spans, names, owner, rank, world, size_group=None):
    """Reassemble sorted output on rank 0 (blocking form of gather_text_async).
    Returns the whole output (uint8 tensor) on rank 0, None elsewhere."""
    return gather_text_async(dist, text, spans, names, owner, rank, world, size_group).wait()


def _post(dist, ops):
    # one grouped launch of all point-to-point transfers (ncclGroupStart/End under RCCL)
    return dist.batch_isend_irecv(ops) if ops else []


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
