"""pcn-firewall's Horus on the CPU oracle (CPU only).

pcn-firewall runs Horus from the start (horus_enabled = true, no knob:
Firewall.h:337).  Two reference scripts pin it: general/test_counters.sh and
test_counters_reload.sh expect EGRESS rule 0 to count the echo replies, which
only the Horus counters can do under the default AUTOMATIC conntrack mode
(tests/golden/make_fw_scenarios.py; replayed by test_oracle_firewall.py).  The
cases here restate the rest of its code -- parity unpinned except through the
restatement, each case citing the lines it follows:
  * one program per chain, rebuilt by that chain's updates (Chain.cpp:173-306),
    not by a default change (Chain.cpp:60-82);
  * the Parser calls it in both directions, before ConntrackLabel
    (Firewall_Parser_dp.c:154-165), so it also runs before the AUTOMATIC
    accept-established short cut;
  * its key holds the ports as stored: packed struct on both sides
    (Firewall_Horus_dp.c:28-57, Firewall_Parser_dp.c:32-43); stale for
    non-TCP/UDP packets (Q4);
  * the conntrack setting is compiled in when the program is built
    (modules/Horus.cpp:135-139); setConntrack(OFF) deletes ConntrackLabel
    (Firewall.cpp:151-174), so Horus's tail calls into it fail: a miss drops,
    and so does an ACCEPT hit of a program built with conntrack on.
"""
import numpy as np
import pytest

from helpers import ct_probe_frames
from oracle.ffi import Oracle

RID_HORUS0 = -4096
INGRESS, EGRESS = 1, 2          # chain slots
HOST, NS1 = "10.0.0.2", "10.0.0.1"
A, B, C = "1.1.1.1", "2.2.2.2", "3.3.3.3"


def pkt(src, dst, proto=17, sport=1000, dport=2000, flags=0x10, icmp_type=8, length=None, direction="ingress"):
    return {"dir": direction, "port": 1, "src": src, "dst": dst, "proto": proto, "sport": sport, "dport": dport,
            "flags": flags, "icmp_type": icmp_type,
            "len": length if length is not None else (98 if proto == 1 else 74 if proto == 6 else 64)}


def run(o, packets, direction=0):
    f, lens, ports = ct_probe_frames(packets)
    return o.classify(f, n=len(packets), lens=lens, stride=128, in_port=ports, direction=direction)


def fw(ingress=(), egress=(), mode=2, ct=False, defaults=("DROP", "DROP")):
    o = Oracle()
    o.set_service(1, mode)
    if ct:
        o.ct_enable()
        o.ct_set_time(1)
    o.set_chain(INGRESS, list(ingress), defaults[0])
    o.set_chain(EGRESS, list(egress), defaults[1])
    return o


def test_on_from_the_start_one_program_per_chain():
    o = fw([{"src": A, "action": "DROP"}, {"src": B, "action": "ACCEPT"}], [{"dst": C, "action": "DROP"}])
    assert o.horus_info(INGRESS) == {"enabled": 1, "runtime": 1, "entries": 2, "fields": 1, "conntrack": 1}
    assert o.horus_info(EGRESS) == {"enabled": 1, "runtime": 1, "entries": 1, "fields": 2, "conntrack": 1}
    v, r = run(o, [pkt(A, HOST), pkt(B, HOST), pkt(C, HOST)])
    # B: PASS_LABELING -> accept; C misses and meets INGRESS's default DROP
    assert list(v) == [0, 1, 0] and list(r) == [RID_HORUS0, RID_HORUS0 - 1, -1]
    v, r = run(o, [pkt(HOST, C, direction="egress"), pkt(HOST, A, direction="egress")], direction=1)
    assert list(v) == [0, 0] and list(r) == [RID_HORUS0, -1]
    assert o.read_horus_counters(2, chain=INGRESS)[0] == [1, 1]
    assert o.read_horus_counters(1, chain=EGRESS)[0] == [1]
    # an update of one chain leaves the other's program alone
    o.set_chain(EGRESS, [], "DROP")
    assert o.horus_info(EGRESS)["runtime"] == 0 and o.horus_info(INGRESS)["runtime"] == 1
    assert o.read_horus_counters(2, chain=INGRESS)[0] == [1, 1]


def test_natural_port_key():
    """Both sides packed: the key's ports are the packet's, and htons(80) of
    the rule (modules/Horus.cpp:43-52) matches a packet to port 80."""
    o = fw([{"l4proto": "TCP", "dport": 80, "action": "DROP"}], defaults=("ACCEPT", "ACCEPT"))
    assert o.horus_info(INGRESS)["fields"] == 4 | 16
    v, r = run(o, [pkt(A, HOST, proto=6, dport=80), pkt(A, HOST, proto=6, sport=0x0400, dport=0x50AB)])
    assert list(r) == [RID_HORUS0, -1] and list(v) == [0, 1]


def test_horus_runs_before_accept_established():
    """AUTOMATIC mode: an ESTABLISHED reply is accepted before the chain
    (Firewall_ConntrackLabel_dp.c:474-478) -- unless Horus, which the Parser
    calls first, drops it."""
    rules = [{"src": A, "l4proto": "UDP", "action": "DROP"}]
    for horus, want in ((True, (0, RID_HORUS0)), (False, (1, -3))):
        o = Oracle()
        o.set_service(1, 2)
        o.set_horus(horus)
        o.ct_enable()
        o.ct_set_time(1)
        o.set_chain(INGRESS, rules, "DROP")
        o.set_chain(EGRESS, [], "ACCEPT")
        run(o, [pkt(HOST, A, sport=2000, dport=1000, direction="egress")], direction=1)   # creates the entry
        v, r = run(o, [pkt(A, HOST)])
        assert (int(v[0]), int(r[0])) == want


def test_conntrack_setting_is_compiled_in():
    rules = [{"src": A, "action": "ACCEPT"}, {"src": B, "action": "DROP"}]
    probe = [pkt(A, HOST), pkt(B, HOST), pkt(C, HOST)]
    # built with conntrack on, then turned off: ACCEPT hits and misses reach a
    # ConntrackLabel program that no longer exists -> RX_DROP
    o = fw(rules, mode=2, defaults=("ACCEPT", "ACCEPT"))
    o.set_service(1, 0)
    v, r = run(o, probe)
    assert list(v) == [0, 0, 0] and list(r) == [RID_HORUS0, RID_HORUS0 - 1, -2]
    # built with conntrack off: an ACCEPT hit is RX_OK, a miss still drops
    o = fw(rules, mode=0, defaults=("ACCEPT", "ACCEPT"))
    assert o.horus_info(INGRESS)["conntrack"] == 0
    v, r = run(o, probe)
    assert list(v) == [1, 0, 0] and list(r) == [RID_HORUS0, RID_HORUS0 - 1, -2]
    # ... and stays RX_OK after conntrack comes back on: no label, no entry
    o.set_service(1, 1)
    o.ct_enable()
    o.ct_set_time(1)
    v, r = run(o, [pkt(A, HOST), pkt(C, HOST)])
    assert list(v) == [1, 1] and list(r) == [RID_HORUS0, -1]
    tab = o.ct_dump()
    assert len(tab) == 1 and int(tab[0]["src_ip"]) != 0        # C's packet (default ACCEPT) made the only entry
    # the next INGRESS update compiles conntrack in
    o.set_chain(INGRESS, rules, "ACCEPT")
    assert o.horus_info(INGRESS)["conntrack"] == 1
    run(o, [pkt(A, HOST)])
    assert len(o.ct_dump()) == 2


def test_default_change_keeps_the_program():
    """Chain::setDefault reloads DefaultAction only (Chain.cpp:60-82)."""
    o = fw([{"src": A, "action": "ACCEPT"}], mode=2, defaults=("ACCEPT", "ACCEPT"))
    run(o, [pkt(A, HOST)] * 2)
    o.set_service(1, 0)
    o.set_default(INGRESS, "DROP")
    assert o.horus_info(INGRESS)["conntrack"] == 1
    assert o.read_horus_counters(1, chain=INGRESS)[0] == [2]
    v, r = run(o, [pkt(A, HOST)])
    assert int(v[0]) == 0 and int(r[0]) == RID_HORUS0
    o.set_chain(INGRESS, [{"src": A, "action": "ACCEPT"}], "DROP")   # a rule update rebuilds it
    assert o.horus_info(INGRESS)["conntrack"] == 0
    assert o.read_horus_counters(1, chain=INGRESS)[0] == [0]


def test_stale_ports_and_length_checks():
    """An ICMP packet's key carries the last TCP/UDP ports (Q4); an accepted
    hit still meets ConntrackLabel's ICMP length checks."""
    o = fw([{"l4proto": "ICMP", "dport": 80, "action": "DROP"}], defaults=("ACCEPT", "ACCEPT"))
    icmp = pkt(A, HOST, proto=1)
    v, r = run(o, [pkt(B, HOST, dport=80), icmp, pkt(B, HOST, dport=81), icmp])
    # the second ICMP packet misses Horus and meets the same rule in the chain (ports skipped, Q3)
    assert list(r) == [-1, RID_HORUS0, -1, 0]
    run(o, [pkt(B, HOST, proto=6, dport=80)])
    assert list(run(o, [icmp])[1]) == [RID_HORUS0]
    o = fw([{"l4proto": "ICMP", "action": "ACCEPT"}])
    v, r = run(o, [pkt(A, HOST, proto=1, icmp_type=3, length=66), pkt(A, HOST, proto=1, icmp_type=3, length=70)])
    assert list(v) == [0, 1] and list(r) == [RID_HORUS0, RID_HORUS0]


def test_pass_labeling_updates_the_table():
    o = fw([{"src": A, "l4proto": "UDP", "action": "ACCEPT"}, {"src": B, "l4proto": "UDP", "action": "DROP"}],
           mode=1, ct=True)
    v, r = run(o, [pkt(A, HOST), pkt(B, HOST)])
    assert list(v) == [1, 0] and list(r) == [RID_HORUS0, RID_HORUS0 - 1]
    tab = o.ct_dump()
    assert len(tab) == 1 and tab[0]["l4proto"] == 17


def test_product_control_plane_matches_the_oracle():
    """The library's per-chain Horus bookkeeping (device-less context) follows
    the oracle through random rule edits, default changes and conntrack
    switches: the same table size, key fields, compiled-in conntrack setting."""
    from polycube_amd import Firewall
    rng = np.random.default_rng(11)
    o, f = Oracle(), Firewall(device=-1)
    o.set_service(1, 2)
    mode = 2
    rules = {INGRESS: [], EGRESS: []}
    names = {INGRESS: "INGRESS", EGRESS: "EGRESS"}
    defaults = {INGRESS: "ACCEPT", EGRESS: "ACCEPT"}
    pool = [{"src": A, "action": "DROP"}, {"src": B, "action": "ACCEPT"}, {"src": C, "dport": 80, "action": "DROP"},
            {"src": "9.0.0.0/8", "action": "DROP"}, {"dst": HOST, "l4proto": "UDP", "action": "ACCEPT"},
            {"src": A, "action": "ACCEPT"}, {"l4proto": "TCP", "tcpflags": "SYN", "action": "DROP"}]
    seen = 0
    for step in range(300):
        k = int(rng.integers(0, 12))
        if k == 0:
            on = bool(rng.random() < 0.5)
            f.conntrack = "ON" if on else "OFF"
            mode = (mode or 1) if on else 0
            o.set_service(1, mode)
            continue
        c = int(rng.choice([INGRESS, EGRESS]))
        ch = f.chain(names[c])
        if k <= 6 or not rules[c]:
            r = pool[int(rng.integers(0, len(pool)))]
            rules[c].append(r)
            ch.append(**r)
        elif k <= 9:
            i = int(rng.integers(0, len(rules[c])))
            rules[c].pop(i)
            ch.delete(i)
        else:
            d = "DROP" if defaults[c] == "ACCEPT" else "ACCEPT"
            defaults[c] = d
            ch.default = d
            o.set_default(c, d)
            continue
        o.set_chain(c, rules[c], defaults[c])
        for cc in (INGRESS, EGRESS):
            a, b = o.horus_info(cc), f.horus_info(names[cc])
            assert a == b, (step, cc, a, b)
            seen += a["runtime"]
    assert seen > 100
    f.close()


def test_iptables_context_names_input_only():
    o = Oracle()
    with pytest.raises(AssertionError):
        o.horus_info(INGRESS)
