"""Per-workgroup timeline of one classify launch (measurement tool, GPU box).

  PCN_IPT_DEBUG_CLOCKS=1 python tools/wg_clocks.py --cfg 2 --log2n 20

Runs the config's chain program over its frames with settled clocks, then reads
the per-workgroup s_memrealtime stamps the kernel recorded for its last launch
(pcn_ipt_debug_clocks: start, after the prologue, after the last frame, after the
counter flush; 100 MHz) and prints the launch's anatomy in microseconds: how far
apart the workgroups started (ramp) and finished (drain), and the median
prologue / frame loop / flush of a workgroup."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--log2n", type=int, default=20)
    ap.add_argument("--launches", type=int, default=5, help="timelines to report (one per launch)")
    a = ap.parse_args()
    if os.environ.get("PCN_IPT_DEBUG_CLOCKS") != "1":
        sys.exit("set PCN_IPT_DEBUG_CLOCKS=1")
    import torch
    from polycube_amd import Iptables, ffi, synth
    rs = synth.config_rules(a.cfg)
    ipt = Iptables(device=0, jit=1, max_rules=16384)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in rs.rules():
        fw.append(**r)
    fw.default = "DROP"
    fw.apply_rules()
    n = 1 << a.log2n
    kw = {}
    if a.cfg == 5:   # IMIX offsets / lens (as tools/ablate.py), TC hook with CFG5_HOOK=tc
        buf, off, ln = synth.imix_frames(rs, n, synth.CONFIG_SEEDS[5])
        frames = torch.from_numpy(buf).cuda()
        kw = dict(offsets=torch.from_numpy(off.view(np.int32)).cuda(), lens=torch.from_numpy(ln.view(np.int16)).cuda(),
                  hook=1 if os.environ.get("CFG5_HOOK") == "tc" else 0)
    else:
        cols = synth.make_headers(rs, n, synth.CONFIG_SEEDS[a.cfg], protos=(17,) if a.cfg in (1, 2) else (6, 17))
        frames = torch.from_numpy(synth.build_frames(*cols).reshape(-1)).cuda()
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _ in range(16):
            ipt.classify(frames, n=n, verdicts=v, rule_ids=False, **kw)
        torch.cuda.synchronize()
    for k in range(a.launches):
        ipt.classify(frames, n=n, verdicts=v, rule_ids=False, **kw)
        grid = ffi.lib().pcn_ipt_debug_clocks(ipt._h, None, 0)
        buf = (C.c_uint64 * (4 * grid))()
        assert ffi.lib().pcn_ipt_debug_clocks(ipt._h, buf, 4 * grid) == grid
        c = np.frombuffer(buf, np.uint64).reshape(grid, 4).astype(np.int64)
        us = (c - c[:, 0].min()) / 100.0            # 100 MHz ticks -> us from the first start
        out = {"cfg": a.cfg, "log2n": a.log2n, "workgroups": grid,
               "span_us": round(float(us[:, 3].max()), 2),
               "start_spread_us": round(float(us[:, 0].max()), 2),
               "end_spread_us": round(float(us[:, 3].max() - us[:, 3].min()), 2),
               "prologue_us_median": round(float(np.median(us[:, 1] - us[:, 0])), 2),
               "frames_us_median": round(float(np.median(us[:, 2] - us[:, 1])), 2),
               "frames_us_min_max": [round(float((us[:, 2] - us[:, 1]).min()), 2),
                                     round(float((us[:, 2] - us[:, 1]).max()), 2)],
               "flush_us_median": round(float(np.median(us[:, 3] - us[:, 2])), 2),
               "program": fw.program_info()["deal_window"]}
        # workgroups are dispatched round-robin over the 8 XCDs: per XCD (b % 8)
        # the median frame-loop time and end time
        xcd = np.arange(grid) % 8
        loop = us[:, 2] - us[:, 1]
        out["xcd_frames_us_median"] = [round(float(np.median(loop[xcd == x])), 2) for x in range(8)]
        out["xcd_end_us_median"] = [round(float(np.median(us[xcd == x, 3])), 2) for x in range(8)]
        print(json.dumps(out), flush=True)
    ipt.close()


if __name__ == "__main__":
    main()
