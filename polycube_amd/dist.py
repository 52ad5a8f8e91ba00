"""Packet-index sharding for one-process-per-GPU runs.

Tables are replicated on every GPU; frames are split into contiguous index
ranges; the only exchange is the per-rule/default counter all-gather (RCCL in
libpcn_ipt.so: pcn_ipt_sync_counters).  These helpers hold the host-side half
so the CPU multi-process tests (gloo) exercise the same partitioning."""


def shard_range(n, world, rank):
    """[lo, hi) of frame indices owned by `rank` (contiguous, sizes differ by <= 1)."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def counter_block(pkts, bytes_, def_pkts, def_bytes):
    """Flatten one rank's counters in the device layout [dp, db, p0, b0, p1, b1, ...]."""
    out = [def_pkts, def_bytes]
    for p, b in zip(pkts, bytes_):
        out += [p, b]
    return out


def sum_blocks(blocks):
    """Element-wise sum of gathered counter blocks (what sum_ranks_kernel computes)."""
    return [sum(col) for col in zip(*blocks)]
