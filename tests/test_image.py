"""The chain image the GPU kernel walks (intervals, hashes, summaries, partial
words, permutation) answers exactly like the oracle — checked on the CPU by
walking the exported bytes with tests/image_model.py (no GPU needed)."""
import numpy as np
import pytest

from oracle.ffi import Oracle
from polycube_amd import FORWARD, Iptables
from polycube_amd import synth
from image_model import ImageModel, model_classify
from rulegen import PORTS, quirky_rules


def build(rules, default="DROP"):
    o = Oracle()
    ipt = Iptables(device=-1)
    for name, idx in PORTS.items():
        o.add_port(name, idx)
        ipt.add_port(name, idx)
    o.set_chain(FORWARD, rules, default)
    ipt.interactive = False
    ch = ipt.chain(FORWARD)
    for r in rules:
        ch.append(**r)
    ch.apply_rules()
    return o, ipt, ch


def check(rules, frames, n):
    o, ipt, ch = build(rules)
    model = ImageModel(ch)
    _, rid = o.classify(frames, n=n, stride=64)
    got = model_classify(model, frames, n)
    bad = np.nonzero(got != rid)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[0]}: model {got[bad[0]]} oracle {rid[bad[0]]}"
    return ch


@pytest.mark.parametrize("cfg,n", [(1, 1500), (2, 1500), (3, 1500)])
def test_image_configs(cfg, n):
    rs = synth.config_rules(cfg)
    frames = synth.config_frames(cfg, n, rs)
    check(rs.rules(), frames, n)


@pytest.mark.parametrize("seed", range(4))
def test_image_random_rulesets(seed):
    rs = synth.make_rules(150 + 200 * seed, seed + 100)
    cols = synth.make_headers(rs, 1000, seed + 7, hit_frac=0.7)
    frames = synth.build_frames(*cols, frame_len=64)
    check(rs.rules(), frames, 1000)


@pytest.mark.parametrize("seed", range(3))
def test_image_quirky_rules(seed):
    # quirky rules (negations, masks with host bits, ports 0, same-prefix
    # overwrite) under well-formed TCP/UDP probes that hit them
    rules = [r for r in quirky_rules(60 + 40 * seed, seed) if "in_iface" not in r and "out_iface" not in r]
    rng = np.random.default_rng(seed)
    n = 800
    src = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    for i, r in enumerate(rules[: n // 2]):
        if "src" in r:
            src[2 * i] = synth_host(r["src"])
        if "dst" in r:
            dst[2 * i] = synth_host(r["dst"])
    proto = rng.choice([6, 17], n).astype(np.int32)
    sport = rng.choice([0, 53, 80, 443, 8080, 1234], n).astype(np.int32)
    dport = rng.choice([0, 53, 80, 443, 8080, 1234], n).astype(np.int32)
    flags = rng.choice([0x02, 0x12, 0x10, 0x01, 0x04, 0x3F], n).astype(np.int32)
    frames = synth.build_frames(src, dst, proto, sport, dport, flags, frame_len=64)
    check(rules, frames, n)


def synth_host(s):
    a, b, c, d = (int(x) & 0xFF for x in s.split("/")[0].split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


def test_ip_buckets_agree_with_a_full_interval_search():
    rs = synth.config_rules(3)
    _, _, ch = build(rs.rules())
    m = ImageModel(ch)
    bkt, bnd_off, cls_off = m.lay["ip_bkt1"], m.lay["ip_bnd1"], m.lay["ip_cls1"]
    ent = np.frombuffer(m.img, np.uint32, 1 << (32 - m.lay["ip_shift1"]), bkt)
    cnt = ent >> 16
    nb = int(((ent & 0xFFFF) + cnt).max())
    bnd = np.frombuffer(m.img, np.uint32, nb, bnd_off)
    assert (np.diff(bnd.astype(np.int64)) > 0).all()
    if m.lay["ip_win1"]:
        assert cnt.max() == m.lay["ip_win1"] <= 4 and m.lay["ip_steps1"] == 0
    else:
        assert cnt.max() < (1 << m.lay["ip_steps1"]) and m.lay["ip_steps1"] <= 3
    rng = np.random.default_rng(5)
    probes = np.concatenate([rng.integers(0, 1 << 32, 3000, dtype=np.uint64),
                             bnd.astype(np.uint64), bnd.astype(np.uint64) - 1]).astype(np.uint32)
    for h in probes:
        want = m.u16(cls_off + 2 * int(np.searchsorted(bnd, h, side="right")))
        assert m.ip_class(1, int(h)) == want


def test_port_hash_two_probe_guarantee():
    rs = synth.make_rules(3000, 9, port_pool=900, p_sport=0.5)
    _, _, ch = build(rs.rules())
    m = ImageModel(ch)
    for i in (0, 1):
        mask = m.lay[f"mask{i}"]
        tab = np.frombuffer(m.img, np.uint32, mask + 2, m.lay[f"hash{i}"])
        assert tab[mask + 1] == tab[0]
        assert (tab[: mask + 1] != 0xFFFFFFFF).sum() > 300
        shift = 32 - mask.bit_length()
        for slot, e in enumerate(tab[: mask + 1]):
            if e == 0xFFFFFFFF:
                continue
            home = ((int(e >> 16) * 0x9E3779B1) & 0xFFFFFFFF) >> shift
            assert slot in (home, (home + 1) & mask)


@pytest.mark.parametrize("n_rules,n_ports,seed,many_flags,merged", [(60, 6, 1, False, 1), (400, 40, 2, True, 0),
                                                                     (400, 300, 3, True, 0)])
def test_image_meta_slot_with_ifaces_flags_conntrack(n_rules, n_ports, seed, many_flags, merged):
    """proto x tcpflags x conntrack (x sport, dport, iface while the table is
    small; own slots otherwise) in the META slot: model == oracle."""
    import random
    rnd = random.Random(seed)
    ports = {f"p{k}": k + 1 for k in range(n_ports)}
    rules = []
    flags = ["SYN", "ACK", "FIN", "RST", "PSH", "URG", "ECE", "CWR"]
    for r in quirky_rules(n_rules, seed, ifaces=False, p_field=0.5 if many_flags else 0.3):
        if rnd.random() < 0.5:
            r["in_iface"] = rnd.choice(list(ports))
        if not many_flags:
            r.pop("tcpflags", None)
        elif rnd.random() < 0.4:
            r["tcpflags"] = " ".join(("!" if rnd.random() < 0.3 else "") + f
                                     for f in rnd.sample(flags, rnd.randint(1, 4)))
        rules.append(r)
    o = Oracle()
    ipt = Iptables(device=-1)
    for name, idx in ports.items():
        o.add_port(name, idx)
        ipt.add_port(name, idx)
    o.set_chain(FORWARD, rules, "DROP")
    ipt.interactive = False
    ch = ipt.chain(FORWARD)
    for r in rules:
        ch.append(**r)
    ch.apply_rules()
    m = ImageModel(ch)
    if merged:
        assert m.lay["slot2"] == 0 and m.lay["stride_iface"] > 0
    else:
        assert m.lay["nslots"] > 3
    rng = np.random.default_rng(seed)
    n = 1200
    src = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    for i, r in enumerate(rules[: n // 2]):
        if "src" in r:
            src[2 * i] = synth_host(r["src"])
        if "dst" in r:
            dst[2 * i] = synth_host(r["dst"])
    proto = rng.choice([6, 17, 1, 47], n).astype(np.int32)
    sport = rng.choice([0, 22, 53, 80, 443, 8080, 65535], n).astype(np.int32)
    dport = rng.choice([0, 22, 53, 80, 443, 8080, 65535], n).astype(np.int32)
    fl = rng.integers(0, 256, n).astype(np.int32)
    frames = synth.build_frames(src, dst, proto, sport, dport, fl, frame_len=96, icmp_type=np.full(n, 8))
    in_port = rng.integers(0, n_ports + 3, n).astype(np.uint16)
    ct = rng.integers(0, 4, n).astype(np.uint8)
    _, rid = o.classify(frames.reshape(-1), n=n, stride=96, fixed_len=96, in_port=in_port, ct_status=ct)
    f = frames.reshape(n, 96)
    for i in range(n):
        if rid[i] == -2:          # decided before the chain (ICMP length checks etc.)
            continue
        row = f[i]
        got = m.run(int.from_bytes(bytes(row[26:30]), "big"), int.from_bytes(bytes(row[30:34]), "big"),
                    int(row[23]), int.from_bytes(bytes(row[34:36]), "big"),
                    int.from_bytes(bytes(row[36:38]), "big"), int(row[47]) if row[23] == 6 else 0,
                    int(in_port[i]), int(ct[i]))[0]
        assert got == rid[i], f"packet {i}: model {got} oracle {rid[i]}"


def test_image_dense_part_config5():
    """10k rules: the image exceeds LDS, so PART is stored dense (a POOL index
    per class and word); the walk through it answers like the oracle."""
    rs = synth.config_rules(5)
    rules = rs.rules()
    o = Oracle(10000, 10000)
    o.set_chain(FORWARD, rules, "DROP")
    ipt = Iptables(device=-1, max_rules=16384, max_counted_rules=10000)
    ipt.interactive = False
    ch = ipt.chain(FORWARD)
    for r in rules:
        ch.append(**r)
    ch.default = "DROP"
    ch.apply_rules()
    model = ImageModel(ch)
    assert model.lay["part_dense"] == 1 and model.lay["pbase"] == model.lay["part"]
    cols = synth.make_headers(rs, 600, 0x5EED, hit_frac=0.8)
    frames = synth.build_frames(*cols, frame_len=64)
    _, rid = o.classify(frames, n=600, stride=64)
    got = model_classify(model, frames, 600)
    assert np.array_equal(got, rid)
    assert (rid >= 0).sum() > 300
