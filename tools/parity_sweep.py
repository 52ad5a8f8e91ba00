"""Randomised GPU-vs-oracle parity sweep (measurement/evidence tool, GPU box).

Each trial draws a service (pcn-iptables, or pcn-firewall in one of its three
conntrack modes), quirky rule sets for every chain, defaults, localip, a frame
stride, edge-case frames, a direction, an attach point, optional per-frame
labels and in_port, and whether chain programs run; it then compares verdicts,
rule ids and every counter of the product library against the CPU oracle
(tests/ helpers).  Runs trials until --seconds elapse and prints one JSON line
per trial plus a summary; exits non-zero on the first mismatch.

  python tools/parity_sweep.py --seconds 150 > gpurun_out/parity_sweep.log
"""
import argparse
import errno
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


BIG = False   # --big: chains of 4100-8000 rules (2+ summary blocks: the two-item deal,
              # global counter atomics past the LDS bins)


def trial(seed, torch, dev):
    from oracle.ffi import Oracle
    from polycube_amd import Firewall, Iptables, IptablesError, synth
    from rulegen import PORTS, quirky_rules
    rng = np.random.default_rng(seed)
    fw_mode = int(rng.integers(-1, 3))           # -1: pcn-iptables, else firewall conntrack mode
    jit = int(rng.choice([1, 1, -1]))
    o = Oracle()
    if fw_mode < 0:
        ipt = Iptables(device=0, jit=jit)
        chains = (0, 1, 2)
        localip = [synth.ip_nbo(int(x)) for x in rng.integers(0, 2**32, size=int(rng.integers(0, 6)))]
        localip += [synth.ip_nbo((10 << 24) | (k << 16) | k) for k in range(int(rng.integers(0, 4)))]
        for name, idx in PORTS.items():
            o.add_port(name, idx)
            ipt.add_port(name, idx)
        o.set_localip(localip)
        ipt.set_localip(localip)
    else:
        ipt = Firewall(device=0, jit=jit)
        o.set_service(1, fw_mode)
        if fw_mode == 0:
            ipt.conntrack = "OFF"
        elif fw_mode == 1:
            ipt.accept_established = "OFF"
        chains = (1, 2)
    ipt.interactive = False
    nrules = {}
    for c in chains:
        count = int(rng.integers(4100, 8000)) if BIG else int(rng.integers(0, 260))
        rules = quirky_rules(count, seed * 7 + c, ct=fw_mode != 0, ifaces=fw_mode < 0)
        if fw_mode >= 0:
            for r in rules:
                r.setdefault("action", "DROP")
        if rng.random() < 0.15 and not BIG:
            rules = []
        d = "DROP" if rng.random() < 0.5 else "ACCEPT"
        ch = ipt.chain(c)
        try:
            o.set_chain(c, rules, d)
        except ValueError as e:
            # the oracle refuses a chain the reference's maps cannot hold (an
            # LPM trie past its 1,024 entries, Iptables_IpLookup_dp.c:54-55):
            # the product must refuse it too, for the same reason and at the
            # verb that pushes the maps (non-interactive: apply_rules; the
            # reference's RawTable::set throws "Table set error: No space left
            # on device", libs/polycube/src/table.cpp:61-66)
            refused, why = False, ""
            for r in rules:
                ch.append(**r)             # staged: no map push, must not fail
            ch.default = d
            try:
                ch.apply_rules()
            except IptablesError as pe:
                why = str(pe)
                refused = pe.code == -errno.ENOSPC and "LPM trie full" in why
            ipt.close()
            return {"seed": seed, "service": "iptables" if fw_mode < 0 else f"firewall/ct{fw_mode}",
                    "rules": len(rules), "oracle_refused": str(e), "product_refused": refused,
                    "product_error": why, "mismatches": 0 if refused else 1, "counters_equal": refused}
        if fw_mode < 0:
            o.apply_accept_established(c)
        for r in rules:
            ch.append(**r)
        ch.default = d
        ch.apply_rules()
        nrules[c] = len(rules)
    # (68, 100, 1500: strides the fixed-stride path takes with dword-aligned loads)
    stride = int(rng.choice([64, 96, 128, 68, 100, 1500]))
    n = int(rng.integers(1, 1 << 15))
    frames, lens = synth.fuzz_frames(n, seed, synth.make_rules(64, seed, protos=(6, 17, 1)), stride=stride)
    frames = frames.reshape(-1)
    fixed = rng.random() < 0.4                    # fixed-length frames: the fixed-stride fast path
    hook = int(rng.random() < 0.25) if not fixed else 0
    direction = int(rng.integers(0, 2))
    ct = rng.integers(0, 5, size=n).astype(np.uint8) if rng.random() < 0.4 else None
    in_port = rng.choice(np.array([0, 1, 2, 3, 0xFFFF], np.uint16), size=n) if rng.random() < 0.5 else None
    kw = dict(stride=stride, direction=direction, hook=hook)
    if fixed:
        kw["fixed_len"] = stride
    v_o, r_o = o.classify(frames, n=n, lens=None if fixed else lens, in_port=in_port, ct_status=ct,
                          nthreads=min(16, os.cpu_count() or 1), **kw)

    def t(a, dt=None):
        return None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(dt) if dt else a).to(dev)
    v_g, r_g = ipt.classify(t(frames), n=n, lens=None if fixed else t(lens, np.int16), in_port=t(in_port, np.int16),
                            ct_status=t(ct), **kw)
    torch.cuda.synchronize()
    v_g, r_g = v_g.cpu().numpy(), r_g.cpu().numpy()
    bad = int(np.count_nonzero((v_o != v_g) | (r_o != r_g)))
    ctr_ok = True
    for c in chains:
        a = o.read_counters(c, 8000)
        b = ipt.chain(c).read_counters(8000)
        ctr_ok &= tuple(a) == tuple(b)
    info = ipt.jit_info()
    ipt.close()
    return {"seed": seed, "service": "iptables" if fw_mode < 0 else f"firewall/ct{fw_mode}", "jit": jit,
            "chain_program": info["launches_jit"] > 0, "rules": nrules, "n": n, "stride": stride, "fixed": fixed,
            "hook": hook, "direction": direction, "labels": ct is not None, "in_port": in_port is not None,
            "mismatches": bad, "counters_equal": bool(ctr_ok)}


def stateful_trial(seed, torch, dev):
    """The connection table on both sides: random service, chain with or
    without conntrack rules, interleaved flows in 2-4 batches of random
    direction; verdicts, rule ids, counters and the whole session table."""
    from oracle.ffi import Oracle
    from polycube_amd import Firewall, Iptables, synth
    rng = np.random.default_rng(seed)
    fw_mode = int(rng.choice([-1, 1, 2]))
    now = 1_700_000_000_000_000_000 + int(rng.integers(0, 10**9))
    rs = synth.config_rules(2, seed=seed)
    base = [dict(r, action=r.get("action", "DROP")) for r in rs.rules()][: int(rng.integers(1, 128))]
    ct_rules = [{"conntrack": "ESTABLISHED", "action": "ACCEPT"}, {"conntrack": "NEW", "action": "ACCEPT"},
                {"conntrack": "INVALID", "action": "DROP"}]
    rules = (ct_rules[int(rng.integers(0, 2)):] if rng.random() < 0.6 else []) + base
    o = Oracle()
    ipt = Iptables(device=0, jit=1) if fw_mode < 0 else Firewall(device=0, jit=1)
    chain = 1
    if fw_mode >= 0:
        o.set_service(1, fw_mode)
        if fw_mode == 1:
            ipt.accept_established = "OFF"
    ipt.interactive = False
    d = "DROP" if rng.random() < 0.5 else "ACCEPT"
    o.set_chain(chain, rules, d)
    if fw_mode < 0:
        o.apply_accept_established(chain)
    ch = ipt.chain(chain)
    for r in rules:
        ch.append(**r)
    ch.default = d
    ch.apply_rules()
    o.ct_enable()
    o.ct_set_time(now)
    ipt.ct_enable(16)
    ipt.ct_set_time(now)
    n = int(rng.integers(1000, 20000))
    # half the trials: 64-byte frames of one length, so a batch whose chain has no
    # conntrack rules (one label) and no Horus program takes the fused stage A
    # (the classify pass builds the walk records; the stale ports completed after it)
    short = rng.random() < 0.5
    stride = 64 if short else 128
    f, lens = synth.flow_traffic(n, int(rng.integers(10, 2000)), seed, stride=stride, rs=rs,
                                 lens_mode="fixed" if short else "mixed", p_noise=0.1, p_err=0.05,
                                 p_icmp=float(rng.choice([0.1, 0.5])) if short else 0.1)
    cuts = sorted(set([0, n] + [int(x) for x in rng.integers(1, n, size=int(rng.integers(1, 4)))]))
    bad = 0
    for lo, hi in zip(cuts, cuts[1:]):
        direction = int(rng.integers(0, 2))
        fr = np.ascontiguousarray(f[lo * stride:hi * stride])
        ln = None if short else lens[lo:hi]
        v_o, r_o = o.classify(fr, n=hi - lo, lens=ln, stride=stride, fixed_len=stride, direction=direction)
        v_g, r_g = ipt.classify(torch.from_numpy(fr).to(dev), n=hi - lo,
                                lens=None if short else torch.from_numpy(ln.view(np.int16)).to(dev), stride=stride,
                                fixed_len=stride, direction=direction)
        torch.cuda.synchronize()
        bad += int(np.count_nonzero((v_o != v_g.cpu().numpy()) | (r_o != r_g.cpu().numpy())))
    a, b = o.ct_dump(), ipt.ct_dump()
    tables = len(a) == len(b) and all(np.array_equal(a[k], b[k]) for k in a.dtype.names)
    ctr_ok = tuple(o.read_counters(chain, len(rules) + 1)) == tuple(ch.read_counters(len(rules) + 1))
    fused = int(ipt.ct_info().get("fused_batches", 0))
    ipt.close()
    return {"seed": seed, "stateful": True, "service": "iptables" if fw_mode < 0 else f"firewall/ct{fw_mode}",
            "rules": len(rules), "n": n, "batches": len(cuts) - 1, "stride": stride, "fused_batches": fused,
            "live_entries": int(len(a)), "mismatches": bad, "counters_equal": bool(ctr_ok and tables),
            "tables_equal": bool(tables)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--seed0", type=int, default=1000)
    ap.add_argument("--stateful", action="store_true", help="connection-table trials")
    ap.add_argument("--lib", default="", help="another build of the product library (A/B)")
    ap.add_argument("--trials", type=int, default=0, help="stop after this many trials (0: --seconds)")
    ap.add_argument("--big", action="store_true", help="chains of 4100-8000 rules (2+ summary blocks)")
    a = ap.parse_args()
    global BIG
    BIG = a.big
    import torch
    if a.lib:
        from polycube_amd import ffi
        ffi.LIB_PATH = a.lib
    dev = torch.device("cuda", 0)
    t0 = time.time()
    k = 0
    ok = 0
    while time.time() - t0 < a.seconds and (not a.trials or k < a.trials):
        r = (stateful_trial if a.stateful else trial)(a.seed0 + k, torch, dev)
        print(json.dumps(r), flush=True)
        k += 1
        if r["mismatches"] or not r["counters_equal"]:
            print(json.dumps({"summary": "MISMATCH", "trials": k}), flush=True)
            sys.exit(1)
        ok += 1
    print(json.dumps({"summary": "all equal", "trials": k, "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
