"""Time pcn_ipt_flow_split stages on the headline batch (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from polycube_amd import Iptables, synth

n = 1 << 24
dev = torch.device("cuda", 0)
f, _ = synth.flow_traffic(n, 1 << 16, 0xC7, stride=64, rs=synth.config_rules(3))
frames = torch.from_numpy(f).to(dev)
ipt = Iptables(device=0)
for _ in range(3):
    ipt.flow_split(frames, 8, 0, n=n, stride=64)
t0 = time.perf_counter()
for _ in range(20):
    idx, *_ = ipt.flow_split(frames, 8, 0, n=n, stride=64)
print(f"split {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms, owned {idx.numel()}", flush=True)
ipt.close()
