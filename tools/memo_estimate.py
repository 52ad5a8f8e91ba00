"""Offline estimate (CPU, measurement only): would a per-workgroup LDS memo of class tuple -> best
entry shorten the candidate stage?  Classes from the exported config-3 image (tests/image_model.py)
for one workgroup's 2^16 packets of the bench traffic; prints hit rates, waves whose deal pass a
memo would skip, and deal passes with / without it.  Run: python tools/memo_estimate.py"""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
from image_model import ImageModel, MISS
from polycube_amd import Iptables, synth
rs = synth.config_rules(3)
ipt = Iptables(device=-1); ipt.interactive = False
ch = ipt.chain("FORWARD")
for r in rs.rules(): ch.append(**r)
ch.default = "DROP"; ch.apply_rules()
m = ImageModel(ch)
L, p = m.lay, m.present
print("nslots", L["nslots"], "nrw", m.nrw, "nsw", m.nsw)
n = 1 << 16
for hit in (0.5, 1.0):
    cols = synth.make_headers(rs, n, 1234, hit_frac=hit)
    src, dst, proto, sport, dport, flags = cols
    def be16(x): return ((x & 0xff) << 8) | (x >> 8)
    tuples = []
    order = []
    itemsof = {}
    cand = 0
    for i in range(n):
        pr = int(proto[i]); fl = int(flags[i]) if pr == 6 else 0
        ns = L["nslots"]; cls = [m.all] * ns; mi = 0
        if p & 8: mi += m.u8(L["proto_idx"] + pr) * L["stride_proto"]
        if p & 128: mi += (m.u16(L["flags_idx"] + 2 * fl) if pr == 6 else L["flags_skip"]) * L["stride_flags"]
        for j, (bit, key, name) in enumerate(((16, int(sport[i]), "sport"), (32, int(dport[i]), "dport"), (64, 1, "iface"))):
            if not p & bit: continue
            x = m.key_class(j, be16(key) if j < 2 else key)
            if j < 2 and pr not in (6, 17): x = L[f"skip{j}"]
            if L[f"slot{j}"] == 0: mi += x * L[f"stride_{name}"]
            else: cls[L[f"slot{j}"]] = x
        cls[0] = m.u16(L["meta"] + 2 * mi)
        if p & 2: cls[1] = m.ip_class(0, int(src[i]))
        if p & 4: cls[2] = m.ip_class(1, int(dst[i]))
        if MISS in cls: continue
        items = 0
        for k in range(m.nsw):
            live = m.nrw - 64 * k
            mk = (1 << 64) - 1 if live >= 64 else (1 << live) - 1
            for c in cls: mk &= m.u64(L["sf"] + 8 * (c * m.nsw + k))
            items += bin(mk).count("1")
        if not items:
            continue
        itemsof[tuple(cls)] = items
        cand += 1
        tuples.append(tuple(cls)); order.append((i, tuple(cls)))
    for M in (256, 1024, 4096):
        memo = {}
        hits = 0
        for t in tuples:
            h = hash(t) % M
            if memo.get(h) == t: hits += 1
            else: memo[h] = t
        memo = {}; waves = {}
        for i, t in order:
            h = hash(t) % M
            w = i // 64
            waves.setdefault(w, [0, 0, 0, 0])
            waves[w][0] += 1
            waves[w][2] += itemsof[t]
            if memo.get(h) == t: waves[w][1] += 1
            else: memo[h] = t; waves[w][3] += itemsof[t]
        skipped = sum(1 for w in waves.values() if w[0] == w[1])
        p0 = sum(-(-w[2] // 64) for w in waves.values()); p1 = sum(-(-w[3] // 64) for w in waves.values())
        print(f"hit_frac {hit}: {cand}/{n} packets with candidates, {len(set(tuples))} distinct tuples, memo {M}: "
              f"hit rate {hits/max(1,len(tuples)):.3f}; waves with candidates {len(waves)}/{n//64}, deal pass skipped in {skipped}; deal passes {p0} -> {p1}")

