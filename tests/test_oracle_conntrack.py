"""Stateful conntrack on the CPU oracle (test infrastructure).

* ct_scenarios.json — the reference's conntrack integration tests
  (local_test_conntrack_{tcp,udp}_*.sh) as packet exchanges with the scripts'
  own pass/fail and session-table (TIME_WAIT) assertions.
* Restated quirks of Iptables_ConntrackLabel_dp.c / Iptables_ConntrackTableUpdate_dp.c
  that no reference test covers (parity unpinned beyond the restatement).
"""
import numpy as np
import pytest

from helpers import CHAINS, OracleCube, ct_probe_frames, ip_nbo, load_ct_scenarios, session_states
from oracle.ffi import CT_STATES, Oracle

CT = load_ct_scenarios()


def cube():
    c = OracleCube(Oracle(), CT["ports"], CT["localip"])
    c.o.ct_enable()
    c.o.ct_set_time(1_700_000_000_000_000_000)
    return c


@pytest.mark.parametrize("sc", CT["scenarios"], ids=[s["name"] for s in CT["scenarios"]])
def test_reference_conntrack_scenarios_on_oracle(sc):
    c = cube()
    for k, st in enumerate(sc["steps"]):
        for op in st["ops"]:
            c.op(op)
        if "probe" in st:
            v = c.ct_probe(st["probe"])
            got = "pass" if all(x == 1 for x in v) else "fail"
            if "drop_at" in st:                  # exchange-tagged: every packet before it passed
                d = st["drop_at"]
                assert v[d] == 0 and all(x == 1 for x in v[:d]), f"{sc['name']} step {k}: {v}"
            elif st["expect"] == "fail":
                assert v[0] == 0, f"{sc['name']} step {k}: {v}"
            assert got == st["expect"], f"{sc['name']} step {k} ({st.get('ref_line')}): {v}"
        if "session" in st:
            states = session_states(c.o.ct_dump(), st["session"]["match"])
            assert st["session"]["state"] in states, states


def run(o, pkts, direction=0):
    f, lens, ports = ct_probe_frames(pkts)
    return o.classify(f, n=len(pkts), lens=lens, stride=128, in_port=ports, direction=direction)


def P(src, dst, proto, sport=0, dport=0, flags=0, seq=0, ack=0, icmp_type=None, length=None, inner=None):
    p = {"dir": "ingress", "port": 1, "src": src, "dst": dst, "proto": proto, "sport": sport, "dport": dport,
         "flags": flags, "seq": seq, "ack": ack,
         "len": length or (74 if proto == 6 else 42 if proto == 17 else 98)}
    if icmp_type is not None:
        p["icmp_type"] = icmp_type
    if inner:
        p["inner"] = inner
    return p


def fresh(rules=(), default="ACCEPT"):
    o = Oracle()
    o.set_chain(CHAINS["FORWARD"], list(rules), default)
    o.apply_accept_established(CHAINS["FORWARD"])
    o.ct_enable()
    o.ct_set_time(1000)
    return o


def test_tcp_close_reaches_time_wait_and_ttls():
    o = fresh()
    A, B = "10.0.1.1", "10.0.2.1"
    X, Y = 100, 5000
    seqs = [P(A, B, 6, 40000, 80, 0x02, X, 0), P(B, A, 6, 80, 40000, 0x12, Y, X + 1),
            P(A, B, 6, 40000, 80, 0x10, X + 1, Y + 1), P(A, B, 6, 40000, 80, 0x11, X + 1, Y + 1),
            P(B, A, 6, 80, 40000, 0x11, Y + 1, X + 2), P(A, B, 6, 40000, 80, 0x10, X + 2, Y + 2)]
    want = ["SYN_SENT", "SYN_RECV", "ESTABLISHED", "FIN_WAIT_1", "LAST_ACK", "TIME_WAIT"]
    ttl = [120e9, 60e9, 432000e9, 120e9, 30e9, 30e9]
    for p, w, t in zip(seqs, want, ttl):
        v, _ = run(o, [p])
        assert v[0] == 1
        (e,) = o.ct_dump()
        assert CT_STATES[e["state"]] == w
        assert int(e["ttl"]) == 1000 + int(t)


def test_seq_plus_be_one_quirk():
    """sequence = seqN + 0x1000000 on the network-order word (ConntrackTableUpdate_dp.c:546):
    an ISN whose low byte is 0xFF makes the SYN-ACK's correct ack INVALID."""
    rules = [{"conntrack": "INVALID", "action": "DROP"}]
    for isn, ok in ((0x100, 1), (0x1FF, 0)):
        o = fresh(rules)
        run(o, [P("10.0.0.1", "10.0.0.2", 6, 1000, 80, 0x02, isn, 0)])
        v, _ = run(o, [P("10.0.0.2", "10.0.0.1", 6, 80, 1000, 0x12, 7, isn + 1)])
        assert v[0] == ok


def test_udp_new_then_established_and_insert_noexist():
    o = fresh([{"conntrack": "NEW", "l4proto": "UDP", "action": "ACCEPT"},
               {"conntrack": "ESTABLISHED", "l4proto": "UDP", "action": "DROP"}], "DROP")
    a = P("10.0.0.1", "10.0.0.2", 17, 1000, 53)
    b = P("10.0.0.2", "10.0.0.1", 17, 53, 1000)
    assert list(run(o, [a, a])[1]) == [0, 0]      # forward again while NEW: still NEW
    v, r = run(o, [b])                             # reverse: ESTABLISHED -> rule 1 drops
    assert (v[0], r[0]) == (0, 1)
    (e,) = o.ct_dump()
    assert CT_STATES[e["state"]] == "NEW"          # dropped packets do not update
    o.set_chain(CHAINS["FORWARD"], [], "ACCEPT")
    run(o, [b])
    (e,) = o.ct_dump()
    assert CT_STATES[e["state"]] == "ESTABLISHED"


def test_icmp_key_takes_stale_ports_from_last_tcp_udp_packet():
    """Q4: the Parser leaves srcPort/dstPort stale for ICMP, so the echo's key
    carries the previous TCP/UDP packet's ports (Iptables_Parser_dp.c:122-143)."""
    o = fresh()
    run(o, [P("9.9.9.9", "8.8.8.8", 17, 1111, 2222), P("10.0.0.1", "10.0.0.2", 1, icmp_type=8)])
    icmp = [e for e in o.ct_dump() if e["l4proto"] == 1]
    assert len(icmp) == 1
    ports = {int(icmp[0]["sport"]), int(icmp[0]["dport"])}
    assert ports == {int.from_bytes((1111).to_bytes(2, "big"), "little"),
                     int.from_bytes((2222).to_bytes(2, "big"), "little")}


def test_echo_reply_established_deletes_entry_and_related_errors():
    o = fresh([{"conntrack": "ESTABLISHED", "action": "ACCEPT"}, {"conntrack": "RELATED", "action": "ACCEPT"}],
              "DROP")
    req = P("10.0.0.1", "10.0.0.2", 1, icmp_type=8)
    rep = P("10.0.0.2", "10.0.0.1", 1, icmp_type=0)
    assert o.accept_established(CHAINS["FORWARD"])
    v, r = run(o, [req])                           # NEW -> default DROP, no entry
    assert v[0] == 0 and len(o.ct_dump()) == 0
    o.set_chain(CHAINS["FORWARD"], [], "ACCEPT")
    run(o, [req])
    assert len(o.ct_dump()) == 1
    o.set_chain(CHAINS["FORWARD"], [{"conntrack": "ESTABLISHED", "action": "ACCEPT"}], "DROP")
    o.apply_accept_established(CHAINS["FORWARD"])
    v, r = run(o, [rep])                           # ports 0/0 -> portRev = ipRev -> reverse -> EST
    assert (v[0], r[0]) == (1, -3)                 # accept-established short cut
    assert o.read_accept_established(CHAINS["FORWARD"]) == (1, 98)
    assert len(o.ct_dump()) == 0                   # echo reply deletes the entry
    # an ICMP error quoting a live UDP flow is RELATED
    o.set_chain(CHAINS["FORWARD"], [{"conntrack": "RELATED", "action": "ACCEPT"}], "ACCEPT")
    run(o, [P("10.0.0.1", "10.0.0.2", 17, 1000, 53)])
    q = {"src": "10.0.0.1", "dst": "10.0.0.2", "proto": 17, "sport": 1000, "dport": 53}
    o.set_chain(CHAINS["FORWARD"], [{"conntrack": "RELATED", "action": "ACCEPT"}], "DROP")
    v, r = run(o, [P("10.0.0.2", "10.0.0.1", 1, icmp_type=3, length=70, inner=q),
                   P("10.0.0.2", "10.0.0.1", 1, icmp_type=3, length=70, inner=dict(q, sport=999)),
                   P("10.0.0.2", "10.0.0.1", 1, icmp_type=3, length=69, inner=q)])
    assert list(v) == [1, 0, 0] and list(r) == [0, -1, -2]


def test_accept_established_disable_falls_through():
    """Iptables::disableAcceptEstablished has no `break` (Iptables.cpp:404-449)."""
    o = Oracle()
    ae = [{"conntrack": "ESTABLISHED", "action": "ACCEPT"}]
    for ch in (2, 1, 0):
        o.set_chain(ch, ae, "ACCEPT")
        o.apply_accept_established(ch)
    assert [o.accept_established(c) for c in range(3)] == [True, True, True]
    o.set_chain(0, [], "ACCEPT")
    o.apply_accept_established(0)
    assert [o.accept_established(c) for c in range(3)] == [False, False, False]
    o.set_chain(1, ae + [{"src": "1.2.3.4", "action": "DROP"}], "ACCEPT")
    o.apply_accept_established(1)
    o.set_chain(1, [{"conntrack": "ESTABLISHED", "action": "ACCEPT", "l4proto": "TCP"}], "ACCEPT")
    o.apply_accept_established(1)                  # not equal: extra field
    assert not o.accept_established(1)


def test_flow_traffic_matches_between_one_and_two_batches():
    """State carries across batches: one batch == the same packets in two."""
    from polycube_amd import synth
    rs = synth.config_rules(2)
    f, lens = synth.flow_traffic(6000, 300, 11, rs=rs, lens_mode="mixed")
    outs = []
    for cut in (6000, 2500):
        o = Oracle()
        o.set_chain(1, rs.rules(), "DROP")
        o.ct_enable()
        o.ct_set_time(77)
        v1, r1 = o.classify(f[:cut * 128], n=cut, stride=128, lens=lens[:cut])
        v2, r2 = o.classify(f[cut * 128:], n=6000 - cut, stride=128, lens=lens[cut:])
        outs.append((np.concatenate([v1, v2]), np.concatenate([r1, r2]), o.ct_dump()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert np.array_equal(outs[0][2], outs[1][2])
    assert ip_nbo("1.2.3.4") != 0


def test_lru_keeps_the_most_recently_touched_entries():
    """Capacity at batch granularity (Iptables_ConntrackLabel_dp.c:112, an
    lru_hash of 65536): after a batch the live entries touched longest ago are
    deleted down to max_entries; a touch is a packet after which its entry is
    live; within a batch nothing is evicted."""
    o = fresh()
    o.ct_set_max_entries(2)
    A, B, C, D = ("10.0.0.%d" % k for k in (1, 2, 3, 4))
    H = "10.9.9.9"

    def udp(src, sport):
        return P(src, H, 17, sport, 53)
    run(o, [udp(A, 1000), udp(B, 1001), udp(C, 1002)])       # three inserts in one batch
    info = o.ct_info()
    assert (info["live"], info["evicted"]) == (2, 1)
    live = {int(e["src_ip"]) for e in o.ct_dump()}
    assert live == {ip_nbo(B), ip_nbo(C)}                     # A: touched first
    run(o, [udp(B, 1001), udp(D, 1003)])                      # B touched again, D inserted
    assert {int(e["src_ip"]) for e in o.ct_dump()} == {ip_nbo(B), ip_nbo(D)}   # C: oldest touch
    # an evicted connection starts over: its next datagram is NEW again
    v, r = run(o, [udp(A, 1000)])
    assert o.ct_info()["evicted"] == 3
    o.ct_set_max_entries(0)                                   # unbounded from the next batch on
    run(o, [udp(C, 1002), udp(A, 1005)])
    assert o.ct_info()["live"] == 4


def test_lru_within_a_batch_nothing_is_evicted():
    """The reply of an evicted-at-batch-end flow in the same batch still finds
    its entry (ESTABLISHED): eviction happens between batches."""
    rules = [{"conntrack": "ESTABLISHED", "action": "ACCEPT"}, {"conntrack": "NEW", "l4proto": "UDP",
                                                                "action": "ACCEPT"}]
    o = fresh(rules, "DROP")
    o.ct_set_max_entries(1)
    H = "10.9.9.9"
    pk = [P("10.0.0.1", H, 17, 1000, 53), P("10.0.0.2", H, 17, 1001, 53), P(H, "10.0.0.1", 17, 53, 1000)]
    v, r = run(o, pk)
    assert list(r) == [1, 1, -3]                              # the reply: ESTABLISHED (accept-established)
    assert o.ct_info()["live"] == 1
    v, r = run(o, [P(H, "10.0.0.2", 17, 53, 1001)])          # 10.0.0.2's entry was evicted
    assert list(r) == [1]                                     # NEW again: rule 1
