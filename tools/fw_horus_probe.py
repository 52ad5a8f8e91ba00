"""Time pcn-firewall classify calls with Horus on, variant by variant (GPU box only).

  python tools/fw_horus_probe.py            # prints one line per variant
  rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run -- python3 tools/fw_horus_probe.py

Variants: the config-3 rules (rule 0 keys Horus on its source port: stale
ports needed), the same rules behind a source-/32 rule 0 (no port field), with
conntrack OFF and MANUAL (stateless labels), Horus off for reference.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from polycube_amd import Firewall, synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    import bench
    rs = synth.config_rules(3)
    rules = rs.rules()
    n = 1 << 24
    frames = torch.from_numpy(bench.gen_frames(n, rs, 0x5EED1000)).to(dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    lead = {"src": "203.0.113.9", "action": "DROP"}
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for name, rl, horus, ct in (("ports_key ct_off", rules, True, "OFF"),
                                ("ports_key manual", rules, True, "ON"),
                                ("src_key ct_off", [lead] + rules, True, "OFF"),
                                ("src_key manual", [lead] + rules, True, "ON"),
                                ("horus_off ct_off", rules, False, "OFF")):
        if only and name.replace(" ", "_") != only:
            continue
        f = Firewall(device=0, jit=1)
        f.horus = horus
        f.conntrack = ct
        if ct == "ON":
            f.accept_established = "OFF"
        f.interactive = False
        ing = f.chain("INGRESS")
        for r in rl:
            ing.append(**dict(r, action=r.get("action", "DROP")))
        ing.default = "DROP"
        ing.apply_rules()
        s = torch.cuda.current_stream(dev)
        for _ in range(5):
            f.classify(frames, n=n, verdicts=v, rule_ids=False)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(s)
        for _ in range(20):
            f.classify(frames, n=n, verdicts=v, rule_ids=False)
        b.record(s)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        acc = int(v.sum().item())
        print(f"{name:18s} {ms:.4f} ms/call  accepted {acc}  horus {f.horus_info('INGRESS')}  "
              f"jit {f.jit_info()}", flush=True)
        f.close()
        del t0


if __name__ == "__main__":
    main()
