"""Horus on the GPU against the CPU oracle (`pytest -m gpu`).

Bit-exact on verdicts, rule ids (a Horus hit reports PCN_IPT_RID_HORUS0 -
rule id), the chains' counters and the Horus counters, with the Parser's
stale ports carried from packet to packet and batch to batch, through the
generic kernel and the chain programs, stateless and with the connection
table.  The semantics restated are listed in tests/test_oracle_horus.py."""
import numpy as np
import pytest

from helpers import ip_host, ip_nbo, probe_frames
from oracle.ffi import Oracle
from test_gpu_conntrack import NOW, assert_tables
from test_gpu_parity import JIT, assert_counters, assert_same

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
RID_HORUS0 = -4096
HOST = "10.10.0.10"


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def setup(input_rules, forward=(), output=(), defaults=None, jit=0, ct=False):
    """Oracle and GPU cube with horus on; INPUT is updated last, so its update builds the table."""
    from polycube_amd import Iptables
    d = {0: "ACCEPT", 1: "DROP", 2: "ACCEPT"}
    d.update(defaults or {})
    o = Oracle()
    ipt = Iptables(device=0, jit=jit)
    o.set_localip([ip_nbo(HOST)])
    ipt.set_localip([ip_nbo(HOST)])
    o.set_horus(True)
    ipt.horus = "ON"
    ipt.interactive = False
    for c, rules in ((1, forward), (2, output), (0, input_rules)):
        o.set_chain(c, list(rules), d[c])
        ch = ipt.chain(c)
        for r in rules:
            ch.append(**r)
        ch.default = d[c]
        ch.apply_rules()
    assert o.horus_info() == ipt.horus_info()
    if ct:
        o.ct_enable()
        o.ct_set_time(NOW)
        ipt.ct_enable(14)
        ipt.ct_set_time(NOW)
    return o, ipt


PROTO = {"TCP": 6, "UDP": 17, "ICMP": 1, "GRE": 47}


def rule_packets(rng, r):
    """Packets whose packed Horus key is rule r's: source port 0x<s>?? when the
    rule has sport s (< 256), and [.., d >> 8] [d & 0xff, ..] around the
    source/destination port boundary for dport d.  A rule for a protocol
    without ports gets a UDP packet first that leaves the ports behind (Q4)."""
    b34 = r["sport"] & 0xff if "sport" in r else int(rng.integers(0, 256))
    b35 = r["dport"] >> 8 if "dport" in r else int(rng.integers(0, 256))
    b36 = r["dport"] & 0xff if "dport" in r else int(rng.integers(0, 256))
    sport, dport = (b34 << 8) | b35, (b36 << 8) | int(rng.integers(0, 256))
    proto = PROTO[r["l4proto"]] if "l4proto" in r else int(rng.choice([6, 17]))
    base = {"dir": "ingress", "port": 1, "src": r.get("src", "8.8.4.4").split("/")[0],
            "dst": r.get("dst", HOST).split("/")[0], "proto": proto,
            "sport": sport, "dport": dport, "flags": 0x10, "icmp_type": 8,
            "len": {6: 74, 17: 64, 1: 98, 47: 64}[proto]}
    if proto in (6, 17):
        return [base]
    lead = dict(base, proto=17, src="8.8.4.4", len=64)
    return [lead, base]


def traffic(rng, n, addrs, ports, rules=()):
    """Packets from/to the rules' addresses (or random ones), TCP/UDP/ICMP/GRE,
    to the host or forwarded, ports drawn so the packed-key byte quirk
    (source port 0x??pp, destination port 0xqq??) sometimes matches; a share
    built to hit a rule's key exactly (rule_packets)."""
    pk = []
    while len(pk) < n:
        if rules and rng.random() < 0.25:
            pk.extend(rule_packets(rng, rules[int(rng.integers(0, len(rules)))]))
            continue
        proto = int(rng.choice([6, 17, 17, 1, 47]))
        src = addrs[rng.integers(0, len(addrs))] if rng.random() < 0.7 else \
            ".".join(str(int(x)) for x in rng.integers(1, 255, 4))
        dst = HOST if rng.random() < 0.5 else addrs[rng.integers(0, len(addrs))]
        if rng.random() < 0.6 and ports:
            a, b = ports[rng.integers(0, len(ports))]       # key bytes wanted at wire 35/36 (or 34)
            sport = (int(rng.integers(0, 256)) << 8) | a if rng.random() < 0.5 else (a << 8) | int(rng.integers(0, 256))
            dport = (b << 8) | int(rng.integers(0, 256))
        else:
            sport, dport = int(rng.integers(0, 65536)), int(rng.integers(0, 65536))
        length = {6: 74, 17: 64, 1: 98, 47: 64}[proto]
        if proto == 1 and rng.random() < 0.2:
            length = int(rng.choice([40, 66, 70]))
        pk.append({"dir": "ingress", "port": 1, "src": src, "dst": dst, "proto": proto, "sport": sport,
                   "dport": dport, "flags": int(rng.choice([0x02, 0x10, 0x12, 0x11])),
                   "icmp_type": int(rng.choice([0, 3, 8, 11])), "len": length})
    return pk


def run(o, ipt, dev, packets, direction=0):
    f, lens, ports, _ = probe_frames(packets)
    n = len(packets)
    v_o, r_o = o.classify(f, n=n, lens=lens, stride=128, in_port=ports, direction=direction)
    v_g, r_g = ipt.classify(torch.from_numpy(f).to(dev), n=n, lens=torch.from_numpy(lens.view(np.int16)).to(dev),
                            stride=128, fixed_len=128, in_port=torch.from_numpy(ports.view(np.int16)).to(dev),
                            direction=direction)
    torch.cuda.synchronize()
    return v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy()


def assert_horus_counters(o, ipt, n=64):
    assert o.read_horus_counters(n) == ipt.read_horus_counters(n)


ADDRS = ["1.1.1.1", "2.2.2.2", "3.3.3.3", "4.4.4.4", "5.5.5.5", HOST]


def rule_sets():
    a = ADDRS
    return {
        "src": [{"src": a[0], "action": "DROP"}, {"src": a[1], "action": "ACCEPT"}, {"src": a[2], "action": "DROP"},
                {"src": a[1], "action": "DROP"}, {"src": "7.0.0.0/8", "action": "DROP"},
                {"src": a[3], "l4proto": "UDP", "action": "ACCEPT"}],
        "proto_ports": [{"l4proto": "TCP", "dport": 0x5000 | 0x21, "action": "DROP"},
                        {"l4proto": "UDP", "dport": 0x3100 | 0x07, "action": "ACCEPT"},
                        {"l4proto": "ICMP", "dport": 0x1100 | 0x09, "action": "DROP"},
                        {"l4proto": "GRE", "dport": 0x2200 | 0x41, "action": "ACCEPT"},
                        {"src": a[4], "action": "DROP"}],
        "five": [{"src": a[k], "dst": HOST, "l4proto": p, "sport": s, "dport": d, "action": act}
                 for k, (p, s, d, act) in enumerate([("TCP", 0x33, 0x4455, "DROP"), ("UDP", 0x12, 0x7001, "ACCEPT"),
                                                     ("TCP", 0x90, 0x0a0b, "ACCEPT"), ("ICMP", 0x05, 0x6060, "DROP")])]
                + [{"dst": HOST, "action": "DROP"}],
    }


def key_ports(rules):
    """(wire byte 34 or 35, wire byte 36) pairs that make packets match the rules' packed port keys."""
    out = []
    for r in rules:
        if "dport" in r:
            out.append((r["dport"] >> 8, r["dport"] & 0xff))
        if "sport" in r and r["sport"] < 256:
            out.append((r["sport"], r.get("dport", 0) >> 8))
    return out


@JIT
@pytest.mark.parametrize("kind", ["src", "proto_ports", "five"])
def test_horus_parity_across_batches(dev, jit, kind):
    rules = rule_sets()[kind]
    rng = np.random.default_rng(len(kind))
    o, ipt = setup(rules, output=[{"dst": ADDRS[0], "action": "DROP"}], jit=jit)
    info = ipt.horus_info()
    assert info["runtime"] == 1 and info["entries"] >= 3
    ports = key_ports(rules)
    hits = 0
    for k in range(4):
        pk = traffic(rng, 3000 + 777 * k, ADDRS, ports, rules)
        v_o, r_o, v_g, r_g = run(o, ipt, dev, pk)
        assert_same(v_o, r_o, v_g, r_g)
        hits += int((r_o <= RID_HORUS0).sum())
        # egress batches move the shared struct's ports too
        pk = traffic(rng, 500, ADDRS, ports)
        for p in pk:
            p["dir"], p["src"] = "egress", HOST
        v_o, r_o, v_g, r_g = run(o, ipt, dev, pk, direction=1)
        assert_same(v_o, r_o, v_g, r_g)
    assert hits > 500
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_horus_counters(o, ipt)


def test_horus_with_connection_table(dev):
    """Stateful: Horus hits bypass the ChainSelector; an ACCEPT hit is
    labelled and updates the table like PASS_LABELING, a DROP hit does
    neither; verdicts, rule ids, counters, Horus counters and the table."""
    rules = rule_sets()["five"][:4] + [{"conntrack": "ESTABLISHED", "action": "ACCEPT"}]
    rules = [dict(r, dport=r["dport"], sport=r["sport"]) for r in rules[:4]] + rules[4:]
    rng = np.random.default_rng(5)
    o, ipt = setup(rules, jit=1, ct=True)
    ports = key_ports(rules)
    for k in range(3):
        pk = traffic(rng, 2500, ADDRS, ports, rules[:4])
        v_o, r_o, v_g, r_g = run(o, ipt, dev, pk)
        assert_same(v_o, r_o, v_g, r_g)
        assert (r_o <= RID_HORUS0).sum() > 200
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_horus_counters(o, ipt)


def test_chain_stats_take_the_horus_counters(dev):
    """pcn_ipt_chain_stats folds Horus's counters of rule id k into rule k of
    the chain read (ChainStats.cpp:106-121), and flushes them."""
    rules = [{"src": ADDRS[0], "action": "DROP"}, {"src": ADDRS[1], "action": "ACCEPT"}]
    o, ipt = setup(rules)
    pk = [{"dir": "ingress", "port": 1, "src": ADDRS[k % 3], "dst": HOST, "proto": 17, "sport": 1, "dport": 2,
           "flags": 0, "len": 64 + k % 3} for k in range(30)]
    v_o, r_o, v_g, r_g = run(o, ipt, dev, pk)
    assert_same(v_o, r_o, v_g, r_g)
    hp, hb = ipt.read_horus_counters(2)
    assert hp == [10, 10]
    st = ipt.chain("INPUT").stats()
    assert [x[1] for x in st[:2]] == [10, 10] and [x[2] for x in st[:2]] == hb
    assert ipt.read_horus_counters(2)[0] == [0, 0]


def test_turning_horus_off_takes_effect_at_the_next_update(dev):
    rules = [{"src": ADDRS[1], "action": "ACCEPT"}]
    o, ipt = setup(rules)
    fwd = [{"dir": "ingress", "port": 1, "src": ADDRS[1], "dst": "9.9.9.9", "proto": 17, "sport": 1, "dport": 2,
            "flags": 0, "len": 64}]
    assert run(o, ipt, dev, fwd)[2][0] == 1              # Horus ACCEPT beats FORWARD's default DROP
    ipt.horus = "OFF"
    o.set_horus(False)
    assert run(o, ipt, dev, fwd)[2][0] == 1              # still in place
    ipt.chain("INPUT").apply_rules()
    o.set_chain(0, rules, "ACCEPT")
    v_o, r_o, v_g, r_g = run(o, ipt, dev, fwd)
    assert_same(v_o, r_o, v_g, r_g)
    assert v_g[0] == 0 and ipt.horus_info()["runtime"] == 0


# ---- pcn-firewall: one program per chain, natural port key, conntrack compiled in ----
FW_IN, FW_EG = 1, 2


def fw_rule_packets(rng, r, direction):
    """Packets whose key is rule r's (pcn-firewall: the ports as on the wire).
    A rule for a protocol without ports gets a UDP packet first that leaves
    its ports behind (Q4)."""
    proto = PROTO[r["l4proto"]] if "l4proto" in r else int(rng.choice([6, 17]))
    sport = r.get("sport", int(rng.integers(0, 65536)))
    dport = r.get("dport", int(rng.integers(0, 65536)))
    src = r.get("src", ADDRS[int(rng.integers(0, 5))]).split("/")[0]
    dst = r.get("dst", HOST).split("/")[0]
    base = {"dir": direction, "port": 1, "src": src, "dst": dst, "proto": proto, "sport": sport, "dport": dport,
            "flags": int(rng.choice([0x02, 0x10, 0x12])), "icmp_type": 8,
            "len": {6: 74, 17: 64, 1: 98, 47: 64}[proto]}
    if proto in (6, 17):
        return [base]
    return [dict(base, proto=17, src="8.8.4.4", len=64), base]


def fw_traffic(rng, n, rules, direction):
    ports = [r[k] for r in rules for k in ("sport", "dport") if k in r] or [80]
    pk = []
    while len(pk) < n:
        if rules and rng.random() < 0.3:
            pk.extend(fw_rule_packets(rng, rules[int(rng.integers(0, len(rules)))], direction))
            continue
        proto = int(rng.choice([6, 17, 17, 1, 47]))
        a = ADDRS[rng.integers(0, len(ADDRS))] if rng.random() < 0.7 else \
            ".".join(str(int(x)) for x in rng.integers(1, 255, 4))
        b = HOST if rng.random() < 0.6 else ADDRS[rng.integers(0, len(ADDRS))]
        src, dst = (a, b) if direction == "ingress" else (b, a)
        pick = lambda: int(rng.choice(ports)) if rng.random() < 0.4 else int(rng.integers(0, 65536))  # noqa: E731
        length = {6: 74, 17: 64, 1: 98, 47: 64}[proto]
        if proto == 1 and rng.random() < 0.2:
            length = int(rng.choice([40, 66, 70]))
        pk.append({"dir": direction, "port": 1, "src": src, "dst": dst, "proto": proto, "sport": pick(),
                   "dport": pick(), "flags": int(rng.choice([0x02, 0x10, 0x12, 0x11])),
                   "icmp_type": int(rng.choice([0, 3, 8, 11])), "len": length})
    return pk


FW_EGRESS_RULES = [{"dst": ADDRS[0], "l4proto": "UDP", "action": "ACCEPT"},
                   {"dst": ADDRS[1], "l4proto": "UDP", "action": "DROP"},
                   {"dst": ADDRS[2], "l4proto": "TCP", "action": "ACCEPT"},
                   {"dst": ADDRS[3], "l4proto": "ICMP", "action": "DROP"}]


def fw_setup(ingress, egress, jit, stateful, defaults=("DROP", "ACCEPT")):
    from polycube_amd import Firewall
    o = Oracle()
    o.set_service(1, 2)
    f = Firewall(device=0, jit=jit)
    if stateful:
        o.ct_enable()
        o.ct_set_time(NOW)
        f.ct_enable(14)
        f.ct_set_time(NOW)
    for c, name, rules, d in ((FW_IN, "INGRESS", ingress, defaults[0]), (FW_EG, "EGRESS", egress, defaults[1])):
        ch = f.chain(name)
        ch.default = d
        for r in rules:
            ch.append(**r)
        o.set_chain(c, list(rules), d)
        assert o.horus_info(c) == f.horus_info(name)
    return o, f


def fw_mode(o, f, mode):
    """0 DISABLED / 1 MANUAL / 2 AUTOMATIC on both (Firewall.cpp:112-191)."""
    if mode == 0:
        f.conntrack = "OFF"
    else:
        f.conntrack = "ON"
        f.accept_established = "ON" if mode == 2 else "OFF"
    o.set_service(1, mode)
    assert f.conntrack_mode == mode


def fw_compare(o, f, dev, pk, direction):
    v_o, r_o, v_g, r_g = run(o, f, dev, pk, direction=direction)
    assert_same(v_o, r_o, v_g, r_g)
    return int((r_o <= RID_HORUS0).sum())


@JIT
@pytest.mark.parametrize("stateful", [False, True], ids=["stateless", "table"])
@pytest.mark.parametrize("kind", ["src", "proto_ports", "five"])
def test_firewall_horus_parity_across_modes(dev, jit, kind, stateful):
    """Both chains' programs, every conntrack mode switch the REST API allows
    and a rebuild while conntrack is off (ACCEPT hits then final, misses
    dropped while it stays off): verdicts, rule ids, the chains' and the Horus
    counters, and the session table."""
    ingress = rule_sets()[kind]
    rng = np.random.default_rng(7 + len(kind) + 10 * stateful)
    o, f = fw_setup(ingress, FW_EGRESS_RULES, jit, stateful)
    assert f.horus_info("INGRESS")["runtime"] == 1 and f.horus_info("EGRESS")["entries"] == 4
    hits = 0
    for k, mode in enumerate([2, 1, 0, "rebuild", 0, 1, 2]):
        if mode == "rebuild":          # two INGRESS updates while conntrack is off: built without it
            f.chain("INGRESS").append(src="6.6.6.6", action="DROP")
            f.chain("INGRESS").delete(len(ingress))
            o.set_chain(FW_IN, list(ingress), "DROP")
            assert f.horus_info("INGRESS") == o.horus_info(FW_IN) and o.horus_info(FW_IN)["conntrack"] == 0
            continue
        fw_mode(o, f, mode)
        hits += fw_compare(o, f, dev, fw_traffic(rng, 1500 + 300 * k, ingress, "ingress"), 0)
        hits += fw_compare(o, f, dev, fw_traffic(rng, 700, FW_EGRESS_RULES, "egress"), 1)
    assert hits > 800
    assert_counters(o, f, chains=(FW_IN, FW_EG), n=len(ingress) + 1)
    for c, name in ((FW_IN, "INGRESS"), (FW_EG, "EGRESS")):
        assert o.read_horus_counters(64, chain=c) == f.read_horus_counters(64, chain=name)
    if stateful:
        assert_tables(o, f)
    f.close()


def test_firewall_chain_stats_fold_their_own_program(dev):
    """pcn-firewall ChainStats::fetchCounters: each chain takes its own
    program's counters (ChainStats.cpp:127-143); reset_counters flushes them
    (Chain.cpp:139-152); a default change keeps the program (Chain.cpp:60-82)."""
    o, f = fw_setup([{"src": ADDRS[0], "action": "ACCEPT"}], [{"dst": ADDRS[0], "action": "ACCEPT"}], -1, False)
    fw_compare(o, f, dev, [pkt_fw(ADDRS[0], HOST, "ingress")] * 3, 0)
    fw_compare(o, f, dev, [pkt_fw(HOST, ADDRS[0], "egress")] * 2, 1)
    f.chain("INGRESS").default = "ACCEPT"
    assert f.horus_info("INGRESS")["runtime"] == 1
    assert [x[1] for x in f.chain("INGRESS").stats()[:1]] == [3]
    assert [x[1] for x in f.chain("EGRESS").stats()[:1]] == [2]
    fw_compare(o, f, dev, [pkt_fw(HOST, ADDRS[0], "egress")] * 4, 1)
    f.chain("EGRESS").reset_counters()
    assert f.read_horus_counters(1, chain="EGRESS")[0] == [0]
    assert [x[1] for x in f.chain("EGRESS").stats()[:1]] == [0]
    f.close()


def pkt_fw(src, dst, direction, proto=17):
    return {"dir": direction, "port": 1, "src": src, "dst": dst, "proto": proto, "sport": 1, "dport": 2,
            "flags": 0, "len": 64}


def run_fixed(o, ipt, dev, packets, direction=0):
    """Fixed stride and length (the bench's launch shape: the FIXED kernel path)."""
    f, _, ports, _ = probe_frames(packets)
    n = len(packets)
    v_o, r_o = o.classify(f, n=n, stride=128, fixed_len=64, in_port=ports, direction=direction)
    v_g, r_g = ipt.classify(torch.from_numpy(f).to(dev), n=n, stride=128, fixed_len=64,
                            in_port=torch.from_numpy(ports.view(np.int16)).to(dev), direction=direction)
    torch.cuda.synchronize()
    return v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy()


@JIT
@pytest.mark.parametrize("fixed", [False, True], ids=["lens", "fixed"])
@pytest.mark.parametrize("nrules", [2, 1100], ids=["lds_bins", "global_fallback"])
def test_horus_counters_hot_key(dev, jit, nrules, fixed):
    """A hot key (most packets hit one rule id) through both counting paths:
    the workgroup LDS bins, and -- when the chain's rule bins leave no room
    (1100 INPUT rule bins + 1100 Horus ids > 2048) -- one global atomic pair
    per distinct id of a wave.  Counters exact against the oracle."""
    rules = [{"l4proto": "UDP", "dport": 1000 + i, "action": "DROP" if i % 2 else "ACCEPT"} for i in range(nrules)]
    o, ipt = setup(rules, jit=jit)
    assert ipt.horus_info()["entries"] == nrules
    rng = np.random.default_rng(nrules)
    for k in range(3):
        n = 6000
        pick = np.where(rng.random(n) < 0.8, 0, rng.integers(0, nrules, n))
        pk = []
        for j in pick:
            p = rule_packets(rng, rules[int(j)])[0]
            p["dst"] = HOST if rng.random() < 0.5 else "9.9.9.9"
            p["len"] = int(rng.choice([64, 74, 128]))
            pk.append(p)
        v_o, r_o, v_g, r_g = (run_fixed if fixed else run)(o, ipt, dev, pk)
        assert_same(v_o, r_o, v_g, r_g)
        assert (r_o == RID_HORUS0).sum() > 3000
    assert o.read_horus_counters(nrules) == ipt.read_horus_counters(nrules)
    assert_counters(o, ipt, n=nrules + 1)


@JIT
@pytest.mark.parametrize("fixed", [False, True], ids=["lens", "fixed"])
def test_stale_ports_across_long_runs(dev, jit, fixed):
    """The in-kernel stale ports (classify.hip stale_lookback) where a frame's
    last TCP/UDP predecessor is many 64-frame groups back, or in an earlier
    batch: long ICMP runs, an all-ICMP batch, runs ending at group edges."""
    rules = [{"l4proto": "ICMP", "dport": 0x1100 | 0x09, "action": "DROP"},
             {"l4proto": "ICMP", "dport": 0x2200 | 0x41, "action": "ACCEPT"},
             {"l4proto": "UDP", "dport": 0x3100 | 0x07, "action": "DROP"}]
    o, ipt = setup(rules, jit=jit)
    rng = np.random.default_rng(17)
    go = run_fixed if fixed else run

    def icmp():
        return {"dir": "ingress", "port": 1, "src": "8.8.8.8", "dst": HOST, "proto": 1, "sport": 0, "dport": 0,
                "flags": 0, "icmp_type": 8, "len": 98}

    def lead(r):                     # the UDP packet rule_packets puts before an ICMP rule's packet
        return rule_packets(rng, r)[0]

    batches = []
    b = [lead(rules[0])] + [icmp() for _ in range(3000)] + [lead(rules[1])] + [icmp() for _ in range(127)]
    batches.append(b)                                  # a 47-group run, then a run ending on a group edge
    batches.append([icmp() for _ in range(2000)])      # all ICMP: the carry of the previous batch
    mixed = []
    for k in range(60):
        mixed += [lead(rules[k % 2])] + [icmp() for _ in range(int(rng.integers(0, 200)))]
    batches.append(mixed)
    hits = 0
    for pk in batches:
        for p in pk:
            p["len"] = 98 if p["proto"] == 1 else 64
        v_o, r_o, v_g, r_g = go(o, ipt, dev, pk)
        assert_same(v_o, r_o, v_g, r_g)
        hits += int((r_o <= RID_HORUS0).sum())
    assert hits > 4000
    assert o.read_horus_counters(3) == ipt.read_horus_counters(3)


def test_stale_ports_across_a_split_launch(dev):
    """A batch with per-frame lengths longer than one launch holds (the u32
    histogram bound splits it, classify.hip launch_classify): the stale-port
    groups of the second launch look back into the first one's
    (LaunchArgs::gbase).  2^24 + 2^17 frames, an ICMP run across the split,
    bit-exact against the oracle on every frame."""
    from polycube_amd import synth
    rules = [{"l4proto": "ICMP", "dport": 0x1100 | 0x09, "action": "DROP"},
             {"l4proto": "UDP", "dport": 0x3100 | 0x07, "action": "DROP"}]
    o, ipt = setup(rules, jit=1)
    n = (1 << 24) + (1 << 17)
    rng = np.random.default_rng(23)
    proto = np.where(rng.random(n) < 0.2, 1, 17).astype(np.int32)
    split = 65536 * 256                                    # frames per launch at 64 B per frame, 256 CUs
    lo = split - 5000
    proto[lo:split + 3000] = 1                             # one run across the split (any CU count up to 256)
    sport = rng.integers(0, 65536, n).astype(np.int32)
    dport = rng.integers(0, 65536, n).astype(np.int32)
    key = rng.random(n) < 0.3                              # UDP frames carrying the ICMP rule's key bytes
    sport = np.where(key, (sport & 0xff00) | 0x11, sport)
    dport = np.where(key, (0x09 << 8) | (dport & 0xff), dport)
    sport[lo - 1], dport[lo - 1], proto[lo - 1] = 0x0011, 0x0900, 17
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = np.full(n, ip_host(HOST), np.uint32)
    f = synth.build_frames(src, dst, proto, sport, dport, np.zeros(n, np.int32), frame_len=64,
                           icmp_type=np.full(n, 8, np.int32)).reshape(-1)
    lens = np.full(n, 64, np.uint16)
    v_o, r_o = o.classify(f, n=n, lens=lens, stride=64)
    v_g, r_g = ipt.classify(torch.from_numpy(f).to(dev), n=n, lens=torch.from_numpy(lens.view(np.int16)).to(dev),
                            stride=64)
    torch.cuda.synchronize()
    assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
    assert (r_o[lo:split + 3000] == RID_HORUS0).all()
    assert o.read_horus_counters(2) == ipt.read_horus_counters(2)


def test_horus_off_program_in_place_keys_on_table_ports(dev):
    """horus turned OFF, the program still in place (no update since), conntrack
    on: an ICMP packet's Horus key reads the ports the connection table's
    copy of the Parser struct holds (Q4), as in the oracle."""
    rules = rule_sets()["proto_ports"]
    o, ipt = setup(rules, ct=True)
    ipt.horus = "OFF"
    o.set_horus(False)
    assert ipt.horus_info()["runtime"] == 1
    rng = np.random.default_rng(5)
    pk = []
    for _ in range(40):
        pk += rule_packets(rng, rules[2]) + rule_packets(rng, rules[0])    # UDP lead, ICMP; TCP
    v_o, r_o, v_g, r_g = run(o, ipt, dev, pk)
    assert_same(v_o, r_o, v_g, r_g)
    assert (r_o == RID_HORUS0 - 2).sum() > 0               # the ICMP rule hit on the stale ports
    assert_horus_counters(o, ipt)


@pytest.mark.parametrize("fixed", [False, True], ids=["lens", "fixed"])
def test_stale_ports_ragged_batches(dev, fixed):
    """Batch sizes that leave the last workgroup's waves past the batch end
    (1, 63, 100, 193, 1000, 2^16 + 1): those waves publish no stale-port group
    word (the host holds n / 64 + 1 words), and every frame stays bit-exact."""
    rules = rule_sets()["proto_ports"]
    o, ipt = setup(rules)
    rng = np.random.default_rng(9)
    go = run_fixed if fixed else run
    for n in (1, 63, 100, 193, 1000, (1 << 16) + 1):
        pk = traffic(rng, n, ADDRS, key_ports(rules), rules)[:n]
        v_o, r_o, v_g, r_g = go(o, ipt, dev, pk)
        assert_same(v_o, r_o, v_g, r_g)
    assert_horus_counters(o, ipt)


@pytest.mark.parametrize("fixed", [False, True], ids=["lens", "fixed"])
def test_stale_groups_stay_inside_their_words(dev, fixed, monkeypatch):
    """No stale-port group word is written past the n / 64 + 1 words the host
    holds for a batch (pcn_ipt.cpp sizes them, classify.hip publishes them):
    guard words past them keep their pattern (pcn_ipt_debug_stale_canary), for
    n = 100 and 2^20 + 1 on a fresh context, then for smaller batches after the
    large one with every word past each batch guarded.  The large batch tiles
    4096 probe packets."""
    from polycube_amd import ffi
    monkeypatch.setenv("PCN_IPT_DEBUG_STALE_CANARY", "1")
    rules = rule_sets()["proto_ports"]
    rng = np.random.default_rng(17)
    pk = traffic(rng, 4096, ADDRS, key_ports(rules), rules)[:4096]
    f0, lens0, ports0, _ = probe_frames(pk)
    for sizes in ((100,), ((1 << 20) + 1, 100, 193, 64, 1)):
        o, ipt = setup(rules)
        for n in sizes:
            reps = -(-n // 4096)
            f = np.tile(f0.reshape(4096, -1), (reps, 1))[:n].reshape(-1)
            lens = np.tile(lens0, reps)[:n]
            ports = np.tile(ports0, reps)[:n]
            kw = dict(stride=128, fixed_len=64) if fixed else dict(stride=128, fixed_len=128)
            lo = {} if fixed else dict(lens=lens)
            v_o, r_o = o.classify(f, n=n, in_port=ports, **lo, **kw)
            lg = {} if fixed else dict(lens=torch.from_numpy(lens.view(np.int16)).to(dev))
            v_g, r_g = ipt.classify(torch.from_numpy(f).to(dev), n=n,
                                    in_port=torch.from_numpy(ports.view(np.int16)).to(dev), **lg, **kw)
            torch.cuda.synchronize()
            assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
            assert ffi.lib().pcn_ipt_debug_stale_canary(ipt._h) == 0, f"guard word overwritten at n={n}"
        assert_horus_counters(o, ipt)
        ipt.close()
