"""Transcribe the reference's conntrack integration tests into replayable fixtures.

Source: /root/reference/src/services/pcn-iptables/test/local_test_conntrack_{tcp_1..4,udp_1..2}.sh
(read as text).  Topology (helpers.bash:28-42): ns1 10.0.1.1 behind veth1, ns2
10.0.2.1 behind veth2, the host forwards between them, so the cube's FORWARD
chain sees both directions at ingress.  Each connectivity assertion becomes a
probe: the packets that exchange puts through the cube, in order, and the
script's own expected outcome ("pass" = every packet ACCEPTed, "fail" = the
first packet DROPped, so the exchange never gets further).  The scripts also
read the session table (`polycubectl pcn-iptables session-table show | grep
10.0.1.1`, column 6 = state) after a closed TCP connection and expect
TIME_WAIT (tcp_3.sh:54-60, tcp_4.sh:56-62).  Expected outcomes are the
reference's assertions, not oracle output.

Packets:
  * `netcat -nvz 10.0.2.1 <port>` from ns1 (connect, then close at once):
    SYN, SYN-ACK, ACK, FIN-ACK (client), FIN-ACK (server), ACK, with
    consistent sequence numbers;
  * `nping --udp -c 1 ... <dst>`: one UDP datagram; nothing listens, so the
    answer is an ICMP port-unreachable (type 3) quoting the datagram's IP
    header and 8 bytes (70-byte frame).

Run:  python tests/golden/make_ct_scenarios.py   (writes ct_scenarios.json next to it)
"""
import json
import os

NS1, NS2 = "10.0.1.1", "10.0.2.1"
PORTS = {"veth1": 1, "veth2": 2}
LOCAL = ["10.0.1.254", "10.0.2.254"]


def tcp(src, dst, sport, dport, flags, seq, ack, port):
    return {"dir": "ingress", "port": PORTS[port], "src": src, "dst": dst, "proto": 6, "sport": sport,
            "dport": dport, "flags": flags, "seq": seq, "ack": ack, "len": 74}


def netcat(cport, sport, isn_c=0x1A2B3C00, isn_s=0x5D6E7F00):
    """ns1:cport -> ns2:sport, connect and close (netcat -z)."""
    X, Y = isn_c, isn_s
    c = lambda fl, s, a: tcp(NS1, NS2, cport, sport, fl, s, a, "veth1")   # noqa: E731
    s = lambda fl, sq, a: tcp(NS2, NS1, sport, cport, fl, sq, a, "veth2")  # noqa: E731
    return [c(0x02, X, 0), s(0x12, Y, X + 1), c(0x10, X + 1, Y + 1), c(0x11, X + 1, Y + 1),
            s(0x11, Y + 1, X + 2), c(0x10, X + 2, Y + 2)]


def syn_only(cport, sport, isn_c=0x1A2B3C00):
    return netcat(cport, sport, isn_c)[:1]


def udp(src, dst, sport, dport, port):
    return {"dir": "ingress", "port": PORTS[port], "src": src, "dst": dst, "proto": 17, "sport": sport,
            "dport": dport, "flags": 0, "len": 42}


def port_unreach(frm, port, quoted):
    """ICMP type 3 from `frm` quoting the UDP datagram `quoted`."""
    return {"dir": "ingress", "port": PORTS[port], "src": frm, "dst": quoted["src"], "proto": 1, "sport": 0,
            "dport": 0, "flags": 0, "icmp_type": 3, "len": 70,
            "inner": {"src": quoted["src"], "dst": quoted["dst"], "proto": 17, "sport": quoted["sport"],
                      "dport": quoted["dport"]}}


def nping(src, dst, sport, dport):
    """nping --udp -c 1 from src: the datagram, then the port-unreachable reply."""
    d = udp(src, dst, sport, dport, "veth1" if src == NS1 else "veth2")
    return [d, port_unreach(dst, "veth2" if src == NS1 else "veth1", d)]


def A(**r):
    return ["append", "FORWARD", r]


def I(**r):  # noqa: E743 (pcn-iptables -I FORWARD: insert at 0)
    return ["insert", "FORWARD", 0, r]


def D(**r):
    return ["deletes", "FORWARD", r]


def P(chain, action):
    return ["default", chain, action]


def tagged(*exchanges):
    """Exchange-tagged probe (tests/helpers.py exchange_replay): a dropped
    packet ends its exchange, so what it would have caused is never sent."""
    return [dict(p, ex=k) for k, ex in enumerate(exchanges) for p in ex]


def icmp(src, dst, icmp_type, port):
    return {"dir": "ingress", "port": PORTS[port], "src": src, "dst": dst, "proto": 1, "sport": 0, "dport": 0,
            "flags": 0, "icmp_type": icmp_type, "len": 98}


def ping_ns1(count=2):
    """`ip netns exec ns1 ping 10.0.2.1 -c 2`: each request forwarded from
    veth1, its reply from veth2 (the cube's FORWARD chain sees both at ingress)."""
    return tagged(*[[icmp(NS1, NS2, 8, "veth1"), icmp(NS2, NS1, 0, "veth2")] for _ in range(count)])


def step(ops=(), probe=None, expect=None, line=None, session=None):
    s = {"ops": list(ops)}
    if probe is not None:
        s["probe"], s["expect"] = probe, expect
    if session is not None:
        s["session"] = session
    if line:
        s["ref_line"] = line
    return s


def tcp_rules(first, second):
    """Allow connections started by `second` only (tcp_1.sh:43-49, 55-61)."""
    return [A(src=first, l4proto="TCP", conntrack="ESTABLISHED", action="ACCEPT"),
            A(src=first, l4proto="TCP", conntrack="INVALID", action="DROP"),
            A(src=second, l4proto="TCP", conntrack="NEW", action="ACCEPT"),
            A(src=second, l4proto="TCP", conntrack="ESTABLISHED", action="ACCEPT"),
            A(src=second, l4proto="TCP", conntrack="INVALID", action="DROP")]


def scenarios():
    out = []
    for k in (1, 2, 3, 4):
        t = f"src/services/pcn-iptables/test/local_test_conntrack_tcp_{k}.sh"
        steps = [step([["default", "FORWARD", "DROP"]], syn_only(40000, 9090), "fail", f"{t}:test_tcp_fail 9090"),
                 step(tcp_rules(NS2, NS1), netcat(40001, 9091), "pass", f"{t}:test_tcp 9091")]
        if k in (3, 4):
            steps.append(step(session={"match": NS1, "state": "TIME_WAIT"}, line=f"{t}:timewait"))
        steps.append(step([["flush", "FORWARD"]] + tcp_rules(NS1, NS2), syn_only(40002, 9092), "fail",
                          f"{t}:test_tcp_fail 9092"))
        out.append({"name": f"conntrack_tcp_{k}", "source": t, "steps": steps})
    t = "src/services/pcn-iptables/test/local_test_conntrack_udp_1.sh"
    rules = [A(src=NS1, l4proto="UDP", conntrack="ESTABLISHED", action="ACCEPT"),
             A(src=NS1, l4proto="ICMP", action="ACCEPT"),
             A(src=NS2, l4proto="UDP", conntrack="NEW", action="ACCEPT"),
             A(src=NS2, l4proto="UDP", conntrack="ESTABLISHED", action="ACCEPT"),
             A(src=NS2, l4proto="ICMP", action="ACCEPT")]
    out.append({"name": "conntrack_udp_1", "source": t, "steps": [
        step([["default", "FORWARD", "DROP"]] + rules, nping(NS1, NS2, 50001, 50002)[:1], "fail", f"{t}:(1)"),
        step([], nping(NS2, NS1, 50002, 50001), "pass", f"{t}:(2)"),
        step([], nping(NS1, NS2, 50001, 50002), "pass", f"{t}:(3)"),
        step([], nping(NS1, NS2, 50001, 50002), "pass", f"{t}:(4)"),
    ]})
    t = "src/services/pcn-iptables/test/local_test_conntrack_udp_2.sh"
    out.append({"name": "conntrack_udp_2", "source": t, "steps": [
        step([["default", "FORWARD", "DROP"]] + rules, nping(NS2, NS1, 50000, 50000), "pass", f"{t}:(1)"),
        step([], nping(NS1, NS2, 50000, 50000), "pass", f"{t}:(2)"),
    ]})
    # ---------------- local_test6_iptables.sh: ctstate NEW/ESTABLISHED in FORWARD ----------------
    # test_tcp (:17-22) = netcat -nvz 10.0.2.1 60123 from ns1 (a new client port
    # each time); test_tcp_fail (:24-29) expects it to fail.  drop_at: the
    # packet whose drop ends the exchange (derived from the rules, not asserted
    # by the script, which only sees the connect fail).
    t = "src/services/pcn-iptables/test/local_test6_iptables.sh"
    ns = [P("INPUT", "DROP"), P("OUTPUT", "DROP")]

    def nc(k):
        return tagged(netcat(41000 + k, 60123, isn_c=0x11110000 * (k + 1), isn_s=0x22220000 * (k + 1)))
    steps = [step([], ping_ns1(), "pass", f"{t}:54"),
             step(ns, ping_ns1(), "pass", f"{t}:59"),
             step([], nc(0), "pass", f"{t}:61"),
             step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT"), P("FORWARD", "DROP")], nc(1), "fail", f"{t}:67"),
             step(ns + [A(conntrack="ESTABLISHED", action="ACCEPT")], nc(2), "fail", f"{t}:74"),
             step([I(conntrack="NEW", action="ACCEPT")], nc(3), "pass", f"{t}:78"),
             step([D(conntrack="NEW", action="ACCEPT")], nc(4), "fail", f"{t}:82"),
             step([A(conntrack="NEW", action="ACCEPT")], nc(5), "pass", f"{t}:86"),
             step([D(conntrack="NEW", action="ACCEPT"), D(conntrack="ESTABLISHED", action="ACCEPT")], nc(6), "fail",
                  f"{t}:91"),
             step([A(src=NS1, dst=NS2, action="ACCEPT")], nc(7), "fail", f"{t}:95"),
             step([I(conntrack="ESTABLISHED", action="ACCEPT")], nc(8), "pass", f"{t}:99")]
    for st, at in zip(steps, [None, None, None, 0, 0, None, 0, None, 0, 1, None]):
        if at is not None:
            st["drop_at"] = at
    out.append({"name": "local_test6_iptables", "source": t, "steps": steps})
    # ---------------- local_test7_iptables.sh: the same topology, address rules (table on) ----------------
    t = "src/services/pcn-iptables/test/local_test7_iptables.sh"
    out.append({"name": "local_test7_iptables_ct", "source": t, "steps": [
        step([], ping_ns1(), "pass", f"{t}:57"),
        step(ns, ping_ns1(), "pass", f"{t}:62"),
        dict(step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT"), P("FORWARD", "DROP")], ping_ns1(), "fail",
                  f"{t}:68"), drop_at=0),
        step(ns + [A(src=NS1, action="ACCEPT"), A(src=NS2, action="ACCEPT")], ping_ns1(), "pass", f"{t}:76"),
    ]})
    return out


if __name__ == "__main__":
    doc = {"generator": "tests/golden/make_ct_scenarios.py", "ports": PORTS, "localip": LOCAL,
           "scenarios": scenarios()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ct_scenarios.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(f"wrote {path}: {len(doc['scenarios'])} scenarios")
