"""Horus on the CPU oracle (CPU only).

The reference pins Horus with one integration script (local_test_horus1.sh,
replayed from scenarios.json by test_oracle_golden.py); its probes pass with
or without Horus.  The cases here restate what the reference's Horus code
does beyond that script -- parity unpinned except through the restatement,
each case citing the lines it follows:
  * the map: leading INPUT rules with rule 0's set-field pattern, a /32
    address or nothing, stop at a conntrack rule, first rule of a repeated
    key wins (Utils.cpp:537-630);
  * when it runs: horus on, INPUT rules, empty FORWARD; any chain update
    rebuilds or drops it (Chain.cpp:505-592);
  * where it runs: after the Parser, before the ChainSelector, ingress only
    (Iptables_Parser_dp.c:145-147): forwarded traffic meets INPUT rules;
  * the key's ports: read through a packed struct from the naturally aligned
    one the Parser writes (Iptables_Horus_dp.c:23-33 vs Parser_dp.c:27-37),
    and stale for non-TCP/UDP packets (Q4).
"""
import numpy as np
import pytest

from helpers import ip_nbo, probe_frames
from oracle.ffi import Oracle

RID_HORUS0 = -4096
HOST = "10.10.0.10"
A, B, C = "1.1.1.1", "2.2.2.2", "3.3.3.3"


def pkt(src, dst, proto=17, sport=1000, dport=2000, flags=0x10, icmp_type=8, length=None, direction="ingress"):
    return {"dir": direction, "port": 1, "src": src, "dst": dst, "proto": proto, "sport": sport, "dport": dport,
            "flags": flags, "icmp_type": icmp_type,
            "len": length if length is not None else (98 if proto == 1 else 74 if proto == 6 else 64)}


def run(o, packets, direction=0):
    f, lens, ports, _ = probe_frames(packets)
    return o.classify(f, n=len(packets), lens=lens, stride=128, in_port=ports, direction=direction)


def cube(input_rules, forward=(), defaults=None, horus=True):
    o = Oracle()
    o.set_localip([ip_nbo(HOST)])
    d = {0: "ACCEPT", 1: "DROP", 2: "ACCEPT"}
    d.update(defaults or {})
    o.set_horus(horus)
    o.set_chain(1, list(forward), d[1])
    o.set_chain(2, [], d[2])
    o.set_chain(0, list(input_rules), d[0])
    return o


def test_forwarded_traffic_meets_input_rules():
    """Horus runs before the ChainSelector (Parser_dp.c:145-147; the
    reference's own TODO at Chain.cpp:494): a forwarded packet from A takes
    INPUT rule 0 (DROP) and one from B INPUT rule 1 (ACCEPT, through
    PASS_LABELING), although FORWARD's default is DROP."""
    rules = [{"src": A, "action": "DROP"}, {"src": B, "action": "ACCEPT"}]
    o = cube(rules)
    assert o.horus_info() == {"enabled": 1, "runtime": 1, "entries": 2, "fields": 1, "conntrack": 0}
    pk = [pkt(A, "9.9.9.9"), pkt(B, "9.9.9.9"), pkt(C, "9.9.9.9"), pkt(B, HOST, length=80)]
    v, r = run(o, pk)
    assert list(v) == [0, 1, 0, 1]
    assert list(r) == [RID_HORUS0, RID_HORUS0 - 1, -1, RID_HORUS0 - 1]
    hp, hb = o.read_horus_counters(2)
    assert hp == [1, 2] and hb == [64, 64 + 80]
    # the chain's own counters saw only the packet Horus missed
    _, _, dp, _ = o.read_counters(1, 2)
    assert dp == 1
    off = cube(rules, horus=False)
    v, r = run(off, pk)
    assert list(v) == [0, 0, 0, 1] and list(r) == [-1, -1, -1, 1]


def test_egress_is_never_filtered_by_horus():
    """The egress Parser's tail call lands on an empty program slot (Horus is
    loaded into the ingress program array only, Chain.cpp:545-552)."""
    o = cube([{"src": HOST, "action": "DROP"}], defaults={2: "ACCEPT"})
    o.set_localip([ip_nbo(HOST)])
    v, r = run(o, [pkt(HOST, A, direction="egress")], direction=1)
    assert list(v) == [1]


@pytest.mark.parametrize("rules,entries,fields", [
    # the pattern of rule 0; the first rule with another pattern ends the map
    ([{"src": A, "action": "DROP"}, {"src": B, "l4proto": "TCP", "action": "ACCEPT"}, {"src": C, "action": "DROP"}],
     1, 1),
    # a conntrack match ends it (fromRuleToHorusKeyValue returns false)
    ([{"src": A, "action": "DROP"}, {"src": B, "conntrack": "NEW", "action": "DROP"}, {"src": C, "action": "DROP"}],
     1, 1),
    # a non-/32 address is not part of the key: rule 0 sets no field, no map
    ([{"src": "10.0.0.0/8", "action": "DROP"}], 0, 0),
    # ... and with a protocol the key is the protocol alone
    ([{"src": "10.0.0.0/8", "l4proto": "TCP", "action": "DROP"},
      {"src": "20.0.0.0/16", "l4proto": "UDP", "action": "ACCEPT"}, {"src": A, "l4proto": "UDP", "action": "DROP"}],
     2, 4),
    # tcpflags and interfaces are not part of the key either
    ([{"dst": HOST, "tcpflags": "SYN", "action": "DROP"}, {"dst": A, "in_iface": "veth1", "action": "DROP"}], 2, 2),
    # a repeated key keeps its first rule (std::map::insert)
    ([{"src": A, "dport": 80, "action": "DROP"}, {"src": A, "dport": 80, "action": "ACCEPT"},
      {"src": B, "dport": 80, "action": "ACCEPT"}], 2, 1 | 16),
])
def test_map_from_leading_rules(rules, entries, fields):
    o = Oracle()
    o.add_port("veth1", 1)
    o.set_horus(True)
    o.set_chain(0, rules, "ACCEPT")
    info = o.horus_info()
    assert (info["entries"], info["fields"], info["runtime"]) == (entries, fields, int(entries > 0))


def test_protocol_only_key_ignores_the_rules_address():
    """Rule 0 = {src 10.0.0.0/8, TCP, DROP}: the key is the protocol, so every
    TCP packet takes rule 0, from any source."""
    o = cube([{"src": "10.0.0.0/8", "l4proto": "TCP", "action": "DROP"}], defaults={0: "ACCEPT", 1: "ACCEPT"})
    v, r = run(o, [pkt("99.0.0.1", HOST, proto=6), pkt("99.0.0.1", HOST, proto=17)])
    assert list(v) == [0, 1] and list(r) == [RID_HORUS0, -1]


def test_when_it_runs():
    o = cube([{"src": A, "action": "DROP"}])
    assert o.horus_info()["runtime"] == 1
    o.set_chain(2, [{"dst": B, "action": "DROP"}], "ACCEPT")      # any other chain update drops it
    assert o.horus_info()["runtime"] == 0
    o.set_chain(0, [{"src": A, "action": "DROP"}], "ACCEPT")      # the next INPUT update builds it again
    assert o.horus_info()["runtime"] == 1
    o.set_chain(1, [{"src": B, "action": "DROP"}], "DROP")        # FORWARD rules: no Horus
    o.set_chain(0, [{"src": A, "action": "DROP"}], "ACCEPT")
    assert o.horus_info()["runtime"] == 0
    o.set_chain(1, [], "DROP")
    o.set_horus(False)                                            # the flag alone changes nothing ...
    assert o.horus_info()["runtime"] == 0
    o.set_horus(True)
    o.set_chain(0, [{"src": A, "action": "DROP"}], "ACCEPT")
    assert o.horus_info()["runtime"] == 1
    o.set_horus(False)
    assert o.horus_info()["runtime"] == 1                         # ... until the next update
    o.set_chain(0, [{"src": A, "action": "DROP"}], "ACCEPT")
    assert o.horus_info()["runtime"] == 0


def test_counters_go_with_the_program():
    o = cube([{"src": A, "action": "DROP"}])
    run(o, [pkt(A, HOST)] * 3)
    assert o.read_horus_counters(1)[0] == [3]
    o.set_chain(0, [{"src": A, "action": "DROP"}, {"src": B, "action": "DROP"}], "ACCEPT")
    assert o.read_horus_counters(2)[0] == [0, 0]


def test_packed_key_port_bytes():
    """Rule {TCP, dport 80}: the map key holds htons(80) = bytes 00 50
    (modules/Horus.cpp:49-51); the datapath key's dstPort is bytes 11-12 of
    the aligned struct = the packet's second source-port byte and first
    destination-port byte.  So the rule matches a packet with source port
    0x??00 and destination port 0x50??, and not a packet to port 80."""
    o = cube([{"l4proto": "TCP", "dport": 80, "action": "DROP"}], defaults={0: "ACCEPT", 1: "ACCEPT"})
    assert o.horus_info()["fields"] == 4 | 16
    pk = [pkt(A, HOST, proto=6, sport=0x0400, dport=0x50AB), pkt(A, HOST, proto=6, sport=0x0401, dport=0x50AB),
          pkt(A, HOST, proto=6, sport=0x0400, dport=80)]
    v, r = run(o, pk)
    # 1: Horus DROP; 2: miss, pipeline: dport 0x50ab != 80 -> default ACCEPT; 3: miss, the pipeline's rule 0 drops
    assert list(r) == [RID_HORUS0, -1, 0] and list(v) == [0, 1, 0]
    # source port: key bytes 9-10 = [padding 00, first source-port byte]
    o = cube([{"l4proto": "UDP", "sport": 5, "action": "DROP"}], defaults={0: "ACCEPT", 1: "ACCEPT"})
    v, r = run(o, [pkt(A, HOST, sport=0x05EE), pkt(A, HOST, sport=5)])
    assert list(r) == [RID_HORUS0, 0]


def test_stale_ports_for_icmp():
    """An ICMP packet's key takes the ports the last TCP/UDP packet left in
    the per-CPU struct (Parser_dp.c:122-143, Q4), across batches too."""
    rules = [{"l4proto": "ICMP", "dport": 80, "action": "DROP"}]
    o = cube(rules, defaults={0: "ACCEPT", 1: "ACCEPT"})
    icmp = pkt(A, HOST, proto=1)
    v, r = run(o, [pkt(B, HOST, proto=17, sport=0x0100, dport=0x5000), icmp,
                   pkt(B, HOST, proto=17, sport=0x0101, dport=0x5000), icmp])
    # the second ICMP packet misses Horus and meets the same rule in the chain,
    # where the port modules are skipped for ICMP (Q3)
    assert list(r) == [-1, RID_HORUS0, -1, 0]
    run(o, [pkt(B, HOST, proto=6, sport=0x0700, dport=0x5001)])
    v, r = run(o, [icmp])
    assert list(r) == [RID_HORUS0]
    # an accepted ICMP hit still meets ConntrackLabel's length checks
    o = cube([{"l4proto": "ICMP", "action": "ACCEPT"}], defaults={0: "DROP", 1: "DROP"})
    v, r = run(o, [pkt(A, HOST, proto=1, icmp_type=3, length=66), pkt(A, HOST, proto=1, icmp_type=3, length=70)])
    assert list(v) == [0, 1] and list(r) == [RID_HORUS0, RID_HORUS0]
    assert o.read_horus_counters(1)[0] == [2]


def test_horus_with_conntrack_accepts_through_pass_labeling():
    """Stateful: a Horus ACCEPT labels and updates the table like a PASS
    (ConntrackLabel_dp.c:581-585 -> ChainForwarder -> ConntrackTableUpdate);
    a Horus DROP does neither."""
    o = cube([{"src": A, "l4proto": "UDP", "action": "ACCEPT"}, {"src": B, "l4proto": "UDP", "action": "DROP"}])
    o.ct_enable()
    o.ct_set_time(1)
    v, r = run(o, [pkt(A, HOST), pkt(B, HOST)])
    assert list(v) == [1, 0] and list(r) == [RID_HORUS0, RID_HORUS0 - 1]
    tab = o.ct_dump()
    assert len(tab) == 1 and tab[0]["l4proto"] == 17


def test_product_control_plane_matches_the_oracle():
    """The library's Horus bookkeeping (pcn_ipt.cpp horus_update, on a
    device-less context: no GPU work) follows the same chain-update sequence
    as the oracle: the same table size, key fields and on/off state after
    every step of random rule edits, flag flips and default changes."""
    from polycube_amd import Iptables
    rng = np.random.default_rng(3)
    o, ipt = Oracle(), Iptables(device=-1)
    rules = {0: [], 1: [], 2: []}
    pool = [{"src": A, "action": "DROP"}, {"src": B, "action": "ACCEPT"}, {"src": C, "dport": 80, "action": "DROP"},
            {"src": "9.0.0.0/8", "action": "DROP"}, {"dst": HOST, "l4proto": "UDP", "action": "ACCEPT"},
            {"conntrack": "NEW", "action": "ACCEPT"}, {"src": A, "action": "ACCEPT"}]
    for step in range(300):
        k = rng.integers(0, 10)
        if k == 0:
            on = bool(rng.random() < 0.7)
            o.set_horus(on)
            ipt.horus = on
            continue
        c = int(rng.choice([0] * 8 + [1, 2]))
        if c == 1 and rules[1]:
            k = 7                                 # FORWARD rules stop Horus: delete them again soon
        if k <= 6 or not rules[c]:
            r = pool[int(rng.integers(0, len(pool)))]
            rules[c].append(r)
            ipt.chain(c).append(**r)
        elif k <= 8:
            i = int(rng.integers(0, len(rules[c])))
            rules[c].pop(i)
            ipt.chain(c).delete(i)
        else:
            d = "DROP" if rng.integers(0, 2) else "ACCEPT"
            if ipt.chain(c).default == (0 if d == "DROP" else 1):
                continue                          # Chain::setDefault to the same action: no update
            ipt.chain(c).default = d
        o.set_chain(c, rules[c], ipt.chain(c).default)
        a, b = o.horus_info(), ipt.horus_info()
        assert a == b, (step, a, b)
        seen_on = locals().get("seen_on", 0) + a["runtime"]
    assert seen_on > 20
    ipt.close()
