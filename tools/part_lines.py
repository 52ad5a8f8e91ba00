"""Distinct 128-byte lines a wave's candidate stage reads from the dense PART
table, row-major (cell = class * nrw + word, as built) against word-major
(word * classes + class), on config 5's rule set and bench-style traffic.
Analysis tool (CPU, no GPU): the ImageModel walk of tests/image_model.py over
the exported image, counting the PART cells of the slots that can be partial
at each candidate word (the kernel's per-word slot mask, `wfields`)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from image_model import ImageModel, MISS
    from polycube_amd import Iptables, synth
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 14
    rs = synth.config_rules(5)
    ipt = Iptables(device=-1, max_rules=16384)   # host-only context: the image is built on the CPU
    ipt.interactive = False
    ch = ipt.chain("FORWARD")
    for r in rs.rules():
        ch.append(**r)
    ch.default = "DROP"
    ch.apply_rules()
    m = ImageModel(ch)
    L = m.lay
    assert L["part_dense"], "config 5's PART is dense"
    nrw = m.nrw
    part_bytes = (L["pool"] - L["part"]) if L["pool"] > L["part"] else None
    cell_b = 4 if L["part_wide"] else 2
    src, dst, proto, sport, dport, flags = synth.make_headers(rs, n, synth.CONFIG_SEEDS[5], protos=(6, 17))
    cells = []      # per packet: list of (class, word) read from PART
    maxc = 0
    for i in range(n):
        p = int(proto[i])
        fl = int(flags[i]) if p == 6 else 0
        ns = L["nslots"]
        # the model's class computation (run() up to the summary words)
        cls = [m.all] * ns
        mi = 0
        pr = m.present
        if pr & 1:
            mi += m.u8(L["ct_idx"]) * L["stride_ct"]
        if pr & 8:
            mi += m.u8(L["proto_idx"] + p) * L["stride_proto"]
        if pr & 128:
            mi += (m.u16(L["flags_idx"] + 2 * fl) if p == 6 else L["flags_skip"]) * L["stride_flags"]
        l4 = p in (6, 17)
        for j, (bit, key, name) in enumerate(((16, int(sport[i]), "sport"), (32, int(dport[i]), "dport"), (64, 1, "iface"))):
            if not pr & bit:
                continue
            x = m.key_class(j, key)
            if j < 2 and not l4:
                x = L[f"skip{j}"]
            if L[f"slot{j}"] == 0:
                mi += x * L[f"stride_{name}"]
            else:
                cls[L[f"slot{j}"]] = x
        cls[0] = m.u16(L["meta"] + 2 * mi)
        if pr & 2:
            cls[1] = m.ip_class(0, int(src[i]))
        if pr & 4:
            cls[2] = m.ip_class(1, int(dst[i]))
        out = []
        if MISS not in cls:
            maxc = max(maxc, max(cls))
            for k in range(m.nsw):
                live = nrw - 64 * k
                mm = (1 << 64) - 1 if live >= 64 else (1 << live) - 1
                for c in cls:
                    mm &= m.u64(L["sf"] + 8 * (c * m.nsw + k))
                while mm:
                    b = (mm & -mm).bit_length() - 1
                    mm &= mm - 1
                    w = 64 * k + b
                    wf = m.u8(L["wfields"] + w) if L["wfields"] else 0xFF
                    for f, c in enumerate(cls):
                        if (wf >> f) & 1:
                            out.append((c, w))
        cells.append(out)
    ncls = maxc + 1
    rows, words, cands = [], [], []
    for w0 in range(0, n, 64):
        cs = [x for pk in cells[w0:w0 + 64] for x in pk]
        if not cs:
            continue
        rows.append(len({(L["part"] + cell_b * (c * nrw + w)) // 128 for c, w in cs}))
        words.append(len({(L["part"] + cell_b * (w * ncls + c)) // 128 for c, w in cs}))
        cands.append(len(cs))
    print(f"config 5, {n} packets, nrw {nrw}, classes {ncls}, cell {cell_b} B")
    print(f"PART cells read per wave (partial slots): {np.mean(cands):.1f}")
    print(f"distinct 128-B lines per wave: row-major {np.mean(rows):.1f}, word-major {np.mean(words):.1f}")


if __name__ == "__main__":
    main()
