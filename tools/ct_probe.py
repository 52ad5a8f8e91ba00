"""Stateful conntrack batches for profiling (GPU box only).

  python tools/ct_probe.py [--log2n 24] [--flows 65536] [--steps 3]
  rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... --kernel-trace -- python3 tools/ct_probe.py

Builds the bench's stateful leg (config-3 rules, synth.flow_traffic frames)
and prints the wall time per batch and the per-kernel split from HIP events
around the whole classify call.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polycube_amd import Iptables, synth  # noqa: E402


def group_sort(f, n):
    """The frames of each 64-frame group stably ordered by the key bucket of
    their 5-tuple (conntrack.hip key_hash % (2^25 - 1) of the ordered key; ICMP
    taken with zero ports, errors by their own header: an approximation, which
    is all a layout experiment needs)."""
    import numpy as np
    fr = f.reshape(n, 64)
    u32 = lambda o: fr[:, o:o + 4].copy().view("<u4").ravel().astype(np.uint64)
    u16 = lambda o: fr[:, o:o + 2].copy().view("<u2").ravel().astype(np.uint64)
    proto = fr[:, 23].astype(np.uint64)
    a, b = u32(26), u32(30)
    pa, pb = u16(34), u16(36)
    icmp = proto == 1
    pa = np.where(icmp, 0, pa).astype(np.uint64)
    pb = np.where(icmp, 0, pb).astype(np.uint64)
    src, dst = np.minimum(a, b), np.maximum(a, b)
    sp, dp = np.minimum(pa, pb), np.maximum(pa, pb)
    with np.errstate(over="ignore"):
        h = ((src << np.uint64(32)) | dst) * np.uint64(0x9E3779B97F4A7C15)
        h ^= ((proto << np.uint64(32)) | (sp << np.uint64(16)) | dp) * np.uint64(0xC2B2AE3D27D4EB4F)
        h ^= h >> np.uint64(29)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(32)
    key = (h % np.uint64((1 << 25) - 1)).reshape(n // 64, 64)
    order = np.argsort(key, axis=1, kind="stable") + (np.arange(n // 64) * 64)[:, None]
    return np.ascontiguousarray(fr[order.ravel()]).ravel()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=24)
    ap.add_argument("--flows", type=int, default=1 << 16)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--p-icmp", type=float, default=0.1)
    ap.add_argument("--p-err", type=float, default=0.02)
    ap.add_argument("--p-noise", type=float, default=0.05)
    ap.add_argument("--cap-log2", type=int, default=20, help="connection table slots (pcn_ipt_ct_enable)")
    ap.add_argument("--group-sort", action="store_true",
                    help="experiment: order the frames of every 64-frame group by (approximately) their "
                         "key bucket, to see what records grouped by key inside a group would save the walk")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rs = synth.config_rules(3)
    ipt = Iptables(device=0, jit=1)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in rs.rules():
        fw.append(**r)
    fw.default = "DROP"
    fw.apply_rules()
    n = 1 << a.log2n
    f, _ = synth.flow_traffic(n, a.flows, 0xC7, stride=64, rs=rs, p_icmp=a.p_icmp, p_err=a.p_err,
                              p_noise=a.p_noise)
    if a.group_sort:
        f = group_sort(f, n)
    frames = torch.from_numpy(f).to(dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    ipt.ct_enable(a.cap_log2)
    ipt.ct_set_time(1_700_000_000 * 10**9)
    ipt.classify(frames, n=n, verdicts=v)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ipt.classify(frames, n=n, verdicts=v)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"{ms:.3f} ms per batch of 2^{a.log2n}, {a.flows} flows: {n / ms / 1e3:.1f} Mpkt/s, "
          f"{len(ipt.ct_dump())} live entries", flush=True)
    ipt.close()


if __name__ == "__main__":
    main()
