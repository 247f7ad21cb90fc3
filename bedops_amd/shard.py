"""Per-chromosome sharding across GPUs (the host-side plan; the reassembly is in C).

Every operation on this path is chromosome-local: all comparisons start with the chromosome
(`interfaces/general-headers/algorithm/bed/BedCompare.hpp:42-43`,
`BedDistances.hpp:99-100`), so per-chromosome outputs concatenated in strcmp order are the
whole output (the reference's own documented scale-out, `docs/.../bedops.rst:721-726`).

One process per GPU (bench.py under torch.distributed.run) or one process driving every GPU
(the C front-ends under BEDGPU_DEVICES, bedops_amd/cli/cli_shard.h — the same plan in C).
`assign()` gives each chromosome to one member (longest processing time on its weight);
each member runs the engine on its chromosomes only (no input exchange); `member_spans()`
describes a member's formatted output over the GLOBAL chromosome list, and
`engine.Group.gather()` (bg_group_gather, bedops_amd/csrc/bg_group.hip) is the one exchange
of the path: grouped RCCL send/recv of every chromosome's bytes into its place on rank 0.

Modes that are not chromosome-local — `--range` padding with its file-wide break rows
(bg_set_pad), `--chrom` (one chromosome) — are never sharded.
"""


def assign(weights, world):
    """chrom -> member. weights: {chrom: weight}. Heaviest first onto the least-loaded
    member (ties: lowest member; equal weights: strcmp order of the name), deterministic on
    every rank. Returns (owner, load)."""
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


def member_spans(local_names, local_offsets, global_names):
    """A member's output over the global chromosome list.

    local_names: the member's chromosome dictionary (its bg_set, strcmp order);
    local_offsets: bg_result_chrom_spans of its formatted result (len(local_names) + 1).
    Returns (offsets, lengths) indexed like `global_names` (strcmp order): zero length for
    chromosomes the member has no output for."""
    gidx = {c: i for i, c in enumerate(global_names)}
    if list(global_names) != strcmp_order(global_names):
        raise ValueError("global chromosome list must be in strcmp order")
    offs = [0] * len(global_names)
    lens = [0] * len(global_names)
    for q, c in enumerate(local_names):
        if c not in gidx:
            raise ValueError(f"chromosome {c!r} is not in the global list")
        offs[gidx[c]] = local_offsets[q]
        lens[gidx[c]] = local_offsets[q + 1] - local_offsets[q]
    return offs, lens


def reassemble(pieces, global_names, owner):
    """Reference model of bg_group_gather for tests: pieces[m] = (bytes, offsets, lengths)
    of member m; returns rank 0's output (every chromosome's bytes in global order)."""
    out = []
    for g, c in enumerate(global_names):
        m = owner.get(c)
        if m is None:
            continue
        text, offs, lens = pieces[m]
        out.append(text[offs[g]:offs[g] + lens[g]])
    return b"".join(out)
