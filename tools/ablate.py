"""Kernel-time ablation of the classify datapath (measurement tool, GPU box).

Runs config 3 (1k rules, 2^24 64-byte frames) through the product library and
through the PCN_ABLATE builds (polycube_amd/build/libpcn_ipt_ablate{1..4}.so:
1 parse only, 2 + field lookups, 3 + summary AND, 4 full minus counters), for
traffic that is all-default (hit 0), the bench mix (hit 0.5) and all-hit (1).
Each variant runs in its own process (one library per process)."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, hit, log2n, iters, cfg, jit):
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    from polycube_amd import ffi
    if lib:
        ffi.LIB_PATH = lib
    from polycube_amd import Iptables, synth
    rs = synth.config_rules(cfg)
    big = dict(max_rules=16384, max_counted_rules=10000, max_action_rules=10000) if cfg == 5 else {}
    ipt = Iptables(device=0, jit=jit, **big)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in rs.rules():
        fw.append(**r)
    fw.default = "DROP"
    fw.apply_rules()
    n = 1 << log2n
    kw = {}
    if cfg == 5:      # IMIX offsets/lens, TC hook when CFG5_HOOK=tc, 64-byte aligned when CFG5_ALIGN=64
        buf, off, ln = synth.imix_frames(rs, n, synth.CONFIG_SEEDS[5], align=int(os.environ.get("CFG5_ALIGN", "1")))
        frames = torch.from_numpy(buf).cuda()
        kw = dict(offsets=torch.from_numpy(off.view(np.int32)).cuda(), lens=torch.from_numpy(ln.view(np.int16)).cuda(),
                  hook=1 if os.environ.get("CFG5_HOOK") == "tc" else 0)
    else:
        cols = synth.make_headers(rs, n, synth.CONFIG_SEEDS[3], hit_frac=hit,
                                  protos=(6, 17) if cfg == 3 else (17,))
        frames = torch.from_numpy(synth.build_frames(*cols).reshape(-1)).cuda()
        stride = int(os.environ.get("FRAME_STRIDE", "64"))   # the frame-size sweep (bench.py frame_sizes)
        if stride != 64:
            frames = synth.spread_frames(frames, n, stride)
            kw = dict(stride=stride, fixed_len=stride)
    v = torch.empty(n, dtype=torch.uint8, device="cuda")
    # clock settle (as bench.py): untimed launches for SETTLE seconds (default 0.5)
    import time
    t0 = time.perf_counter()
    while True:
        for _ in range(16):
            ipt.classify(frames, n=n, verdicts=v, rule_ids=False, **kw)
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= float(os.environ.get("SETTLE", "0.5")):
            break
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record()
        ipt.classify(frames, n=n, verdicts=v, rule_ids=False, **kw)
        b.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
    info = fw.info()
    print(json.dumps({"lib": os.path.basename(lib or "product"), "jit": ipt.jit_info()["launches_jit"] > 0,
                      "cfg": cfg, "log2n": log2n, "image_bytes": info["table_bytes"], "slots_info": info,
                      "defs": os.environ.get("PCN_IPT_JIT_DEFS", ""), "stride": kw.get("stride", 64),
                      "knobs": {k[14:]: v for k, v in os.environ.items() if k.startswith("PCN_IPT_DEBUG_")},
                      "hit": hit, "ms": ms,
                      "gpkt_s": n / ms / 1e6, "frac": 64 * n / (ms * 1e-3) / 8e12}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--lib", default="")
    ap.add_argument("--hit", type=float, default=0.5)
    ap.add_argument("--log2n", type=int, default=24)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--jit", type=int, default=-1)
    ap.add_argument("--variants", default="jit,product,1,2,3,4")
    ap.add_argument("--hits", default="0,0.5,1")
    a = ap.parse_args()
    if a.child:
        child(a.lib, a.hit, a.log2n, a.iters, a.cfg, a.jit)
        return
    for var in a.variants.split(","):
        jit = -1
        env = dict(os.environ)
        if "@" in var:   # ...@KEY=V;KEY2=V2: PCN_IPT_DEBUG_KEY=V environment knobs
            var, knobs = var.split("@", 1)
            for kv in knobs.split(";"):
                k, v = kv.split("=", 1)
                env["PCN_IPT_DEBUG_" + k] = v
        if var == "jit":     # the product library's chain program
            lib, jit = "", 1
        elif var.startswith("jit:"):  # jit:-DX=1+-DY=0: chain program built with extra defines
            lib, jit = "", 1
            env["PCN_IPT_JIT_DEFS"] = var[4:].replace("+", " ")
        elif var.startswith("jit"):   # jitN: chain program built with -DPCN_ABLATE=N
            lib, jit = "", 1
            env["PCN_IPT_JIT_DEFS"] = f"-DPCN_ABLATE={var[3:]}"
        elif var == "product":
            lib = ""
        elif var.startswith("lib:"):   # lib:NAME: polycube_amd/build/ab/libpcn_ipt_NAME.so, chain programs on
            lib, jit = os.path.join(ROOT, "polycube_amd", "build", "ab", f"libpcn_ipt_{var[4:]}.so"), 1
        elif var.startswith("exp_"):   # another build of the product library (A/B), chain programs on
            lib, jit = os.path.join(ROOT, "polycube_amd", "build", f"libpcn_ipt_{var.split(':')[0]}.so"), 1
        else:
            lib = os.path.join(ROOT, "polycube_amd", "build", f"libpcn_ipt_ablate{var}.so")
        for hit in a.hits.split(","):
            r = subprocess.run([sys.executable, __file__, "--child", "--lib", lib, "--hit", hit, "--log2n",
                                str(a.log2n), "--iters", str(a.iters), "--cfg", str(a.cfg), "--jit", str(jit)],
                               capture_output=True, text=True, timeout=300, env=env)
            out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print(out[-1] if out else f"{var} hit={hit} FAILED rc={r.returncode}: {r.stderr[-400:]}", flush=True)


if __name__ == "__main__":
    main()
