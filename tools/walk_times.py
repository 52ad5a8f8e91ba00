"""Where a long-run walk wave spends its time (GPU box, measurement build only).

  make -C polycube_amd ct_variant NAME=dbgt DEFS=-DPCN_CT_DBG_T=1
  PCN_IPT_LIBRARY=polycube_amd/ab/libpcn_ipt_ct_dbgt.so python tools/walk_times.py

Runs one stateful batch of the bench traffic (as tools/ct_probe.py) and reads
the walk's per-block clocks (100 MHz): block entry, run start (after the plan,
head and key loads), end of the first chunk (prologue + first rounds), end.
Prints percentiles of each phase for the class-0 waves (one per long run) and
how many of them were in flight over the kernel's life.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polycube_amd import Iptables, synth  # noqa: E402
from polycube_amd import ffi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=24)
    ap.add_argument("--flows", type=int, default=1 << 16)
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
    f, _ = synth.flow_traffic(n, a.flows, 0xC7, stride=64, rs=rs)
    frames = torch.from_numpy(f).to(dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    ipt.ct_enable(20)
    ipt.ct_set_time(1_700_000_000 * 10**9)
    lib = ffi.lib()
    for _ in range(3):
        lib.pcn_ipt_dbg_walk_clear()
        ipt.classify(frames, n=n, verdicts=v)
        torch.cuda.synchronize()
    words = 4 << 17
    buf = (C.c_ulonglong * words)()
    assert lib.pcn_ipt_dbg_walk_times(buf, C.c_size_t(words)) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    entry = t[:, 0]
    ran = t[:, 1] != 0
    e0 = entry[entry != 0].min()
    tt = t[ran]
    recs = tt[:, 3] >> 48
    end = tt[:, 3] & ((1 << 48) - 1)
    ph = {"queue (entry - kernel start)": tt[:, 0] - e0, "head (run start - entry)": tt[:, 1] - tt[:, 0],
          "first chunk (first - run start)": tt[:, 2] - tt[:, 1], "rest (end - first)": end - tt[:, 2],
          "wave life (end - entry)": end - tt[:, 0]}
    print(f"class-0 waves {ran.sum()}, records {recs.sum()} (mean {recs.mean():.0f}), kernel span "
          f"{(max(end.max(), 0) - e0) / 100:.1f} us (first entry to last class-0 end)")
    for k, x in ph.items():
        q = np.percentile(x / 100.0, [10, 50, 90, 99])
        print(f"  {k:34s} us p10 {q[0]:8.1f} p50 {q[1]:8.1f} p90 {q[2]:8.1f} p99 {q[3]:8.1f} mean {x.mean() / 100:8.1f}")
    life = end - tt[:, 0]
    top = np.argsort(life)[::-1][:24]
    print("  longest class-0 waves (vb, records, entry us, life us, first chunk us):")
    vbs = np.nonzero(ran)[0]
    for j in top:
        print(f"    vb {vbs[j]:6d} recs {recs[j]:6d} entry {(tt[j, 0] - e0) / 100:7.1f} life {life[j] / 100:7.1f} "
              f"first {(tt[j, 2] - tt[j, 1]) / 100:7.1f}")
    grid = np.linspace(0, (end.max() - e0), 11)
    inflight = [int(((tt[:, 0] - e0 <= g) & (end - e0 > g)).sum()) for g in grid]
    print("  class-0 waves in flight at 0..100 % of the span:", inflight)
    ipt.close()


if __name__ == "__main__":
    main()
