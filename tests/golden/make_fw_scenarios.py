"""Transcribe the reference's pcn-firewall integration tests into replayable fixtures.

Source: /root/reference/src/services/pcn-firewall/test/{general,ping,tcp,conntrack}/*.sh
(read as text).  Topology (helpers.bash:13-22): ns1 holds veth1_ = 10.0.0.1,
the host side veth1 = 10.0.0.2, and the firewall is attached to veth1
(`polycubectl attach fw veth1`).  A packet from ns1 reaches the cube on its
INGRESS program, a packet the host sends to ns1 on its EGRESS program.

Every connectivity assertion becomes a *probe*: the packets that traffic puts
through the cube, in order, with the script's expected outcome ("pass" = every
packet accepted, "fail" = at least one dropped).  A probe is replayed in order,
one packet at a time, because most of these scripts run with the firewall's
default connection tracking (AUTOMATIC: conntrack ON, accept-established ON,
Firewall.h:323).  Counter assertions (`stats <id> show pkts|bytes`,
`stats show` for the DEFAULT row) are kept with the step they follow.

Ops:  ["default", CHAIN, ACTION] ["append", CHAIN, rule] ["insert", CHAIN, id|None, rule]
      ["add", CHAIN, id, rule] (rule add <id>: Chain::addRule) ["delete", CHAIN, id]
      ["deletes", CHAIN, rule] ["batch", CHAIN, [op dicts]] ["reset_counters", CHAIN]
      ["conntrack", "ON"|"OFF"] ["accept_established", "ON"|"OFF"]
An op the script runs under `set +e` and that the reference refuses is wrapped
as ["expect_error", op].

Run:  python tests/golden/make_fw_scenarios.py   (writes fw_scenarios.json next to it)
"""
import json
import os

NS1, HOST = "10.0.0.1", "10.0.0.2"
SRC = "src/services/pcn-firewall/test/"
ICMP_ACCEPT_IN = {"src": NS1, "dst": HOST, "l4proto": "ICMP", "action": "ACCEPT"}
ICMP_ACCEPT_OUT = {"src": HOST + "/32", "dst": NS1 + "/32", "l4proto": "ICMP", "action": "ACCEPT"}


def pkt(direction, src, dst, proto, sport=0, dport=0, flags=0, icmp_type=None, length=None, seq=None,
        ack=None):
    p = {"dir": direction, "port": 1, "src": src, "dst": dst, "proto": proto, "sport": sport, "dport": dport,
         "flags": flags}
    if icmp_type is not None:
        p["icmp_type"] = icmp_type
    if seq is not None:
        p["seq"], p["ack"] = seq, ack
    p["len"] = length if length is not None else (98 if proto == 1 else 74)
    return p


def ping_from_ns1(n=2):
    """`ip netns exec ns1 ping 10.0.0.2 -c n`: echo request in, echo reply out (98-byte frames)."""
    out = []
    for _ in range(n):
        out += [pkt("ingress", NS1, HOST, 1, icmp_type=8), pkt("egress", HOST, NS1, 1, icmp_type=0)]
    return out


def ping_from_host(n=2):
    """`ping 10.0.0.1 -c n` on the host: echo request out, echo reply in."""
    out = []
    for _ in range(n):
        out += [pkt("egress", HOST, NS1, 1, icmp_type=8), pkt("ingress", NS1, HOST, 1, icmp_type=0)]
    return out


def netcat_from_ns1(port):
    """`ip netns exec ns1 netcat -nvz 10.0.0.2 <port>`: the handshake (SYN in, SYN-ACK out, ACK in)."""
    return [pkt("ingress", NS1, HOST, 6, 40000, port, 0x02, length=74, seq=1000, ack=0),
            pkt("egress", HOST, NS1, 6, port, 40000, 0x12, length=74, seq=5000, ack=1001),
            pkt("ingress", NS1, HOST, 6, 40000, port, 0x10, length=66, seq=1001, ack=5001)]


def tagged(*exchanges):
    """Exchange-tagged probe (tests/helpers.py exchange_replay): packets go one
    at a time and a dropped packet ends its exchange -- a dropped echo request
    has no reply, a dropped SYN no SYN-ACK -- so connection state only ever
    sees what the real exchange would have put through the cube."""
    return [dict(p, ex=k) for k, ex in enumerate(exchanges) for p in ex]


def pings_from_ns1(n=2):
    return tagged(*[[pkt("ingress", NS1, HOST, 1, icmp_type=8), pkt("egress", HOST, NS1, 1, icmp_type=0)]
                    for _ in range(n)])


def pings_from_host(n=2):
    return tagged(*[[pkt("egress", HOST, NS1, 1, icmp_type=8), pkt("ingress", NS1, HOST, 1, icmp_type=0)]
                    for _ in range(n)])


def nping_udp(src_side, sport=50000, dport=50000):
    """`nping --udp -c 1 -p <dport> -g <sport>` from ns1 ("ns1") or the host:
    the 42-byte datagram; nothing listens, so the peer answers with an ICMP
    port-unreachable (type 3) quoting the datagram's IP header + 8 bytes
    (70-byte frame).  "Rcvd: 1" means that answer came back."""
    if src_side == "ns1":
        d = pkt("ingress", NS1, HOST, 17, sport, dport, length=42)
        e = pkt("egress", HOST, NS1, 1, icmp_type=3, length=70)
    else:
        d = pkt("egress", HOST, NS1, 17, sport, dport, length=42)
        e = pkt("ingress", NS1, HOST, 1, icmp_type=3, length=70)
    e["inner"] = {"src": d["src"], "dst": d["dst"], "proto": 17, "sport": sport, "dport": dport}
    return tagged([d, e])


def netcat_session(client, port, cport=40100, close=True, isn_c=0x3C4D0000, isn_s=0x7A8B0000):
    """`nc -nvz <server> <port>` from `client` ("ns1" or "host"): SYN, SYN-ACK,
    ACK and, with close, the -z close (FIN-ACK, FIN-ACK, ACK), sequence
    numbers consistent; one exchange."""
    out_dir, in_dir = ("ingress", "egress") if client == "ns1" else ("egress", "ingress")
    c_ip, s_ip = (NS1, HOST) if client == "ns1" else (HOST, NS1)
    X, Y = isn_c, isn_s

    def c(fl, sq, ak, ln=74):
        return pkt(out_dir, c_ip, s_ip, 6, cport, port, fl, length=ln, seq=sq, ack=ak)

    def sv(fl, sq, ak, ln=74):
        return pkt(in_dir, s_ip, c_ip, 6, port, cport, fl, length=ln, seq=sq, ack=ak)
    ex = [c(0x02, X, 0), sv(0x12, Y, X + 1), c(0x10, X + 1, Y + 1, 66)]
    if close:
        ex += [c(0x11, X + 1, Y + 1, 66), sv(0x11, Y + 1, X + 2, 66), c(0x10, X + 2, Y + 2, 66)]
    return tagged(ex)


def step(ops, probe=None, expect=None, line=None, counters=None):
    s = {"ops": ops}
    if probe is not None:
        s["probe"], s["expect"] = probe, expect
    if counters is not None:
        s["counters"] = counters
    if line is not None:
        s["ref_line"] = SRC + line
    return s


def ctr(chain, rule, pkts, bytes_, divergence=None):
    c = {"chain": chain, "rule": rule, "pkts": pkts, "bytes": bytes_}
    if divergence:
        c.update(divergence)
    return c


FWSETUP = [["default", "INGRESS", "DROP"], ["default", "EGRESS", "DROP"]]   # fwsetup in every script

# The EGRESS counter assertions of test_counters.sh / test_counters_reload.sh
# expect the echo replies to be counted by EGRESS rule 0.  Through the
# pipeline alone they would not be: with the default AUTOMATIC mode a reply
# whose request created a connection entry is labelled ESTABLISHED and
# accepted before the chain, uncounted (Firewall_ConntrackLabel_dp.c:474-478).
# They are counted because pcn-firewall's Horus is on from the start
# (Firewall.h:337): EGRESS rule 0 {src/32, dst/32, ICMP} is a Horus key, the
# Parser calls Horus before ConntrackLabel (Firewall_Parser_dp.c:154-157), the
# hit bumps Horus's counter of rule 0 (Firewall_Horus_dp.c:143-146), and the
# chain's stats fold it in (ChainStats.cpp:127-143).  The script's numbers are
# the datapath's.


def batch_rules(n_first, first, ins_id, ins, lo2, hi2, second):
    ops = [dict(first(i), operation="append") for i in range(n_first)]
    ops += [dict(r, operation="insert", id=ins_id + k) for k, r in enumerate(ins)]
    ops += [dict(second(i), operation="append") for i in range(lo2, hi2 + 1)]
    return ops


def r_10(i, mask, flags):
    r = {"src": f"10.1.{i % 2}.{i % 255}/{mask}", "dst": f"10.1.{i % 2}.{i % 255}", "l4proto": "TCP",
         "sport": i, "dport": i, "action": "DROP"}
    if flags:
        r["tcpflags"] = flags
    return r


def r_11(i, dst_mask, flags):
    r = {"src": f"11.1.0.{i % 255}", "dst": f"11.1.0.{i % 255}" + (f"/{dst_mask}" if dst_mask else ""),
         "l4proto": "TCP", "sport": i, "dport": i, "action": "DROP"}
    if flags:
        r["tcpflags"] = flags
    return r


def scenarios():
    S = []
    S.append({"name": "general/test_append", "steps": [
        step(FWSETUP + [["append", "INGRESS", ICMP_ACCEPT_IN], ["append", "EGRESS", ICMP_ACCEPT_OUT]],
             ping_from_ns1(), "pass", "general/test_append.sh:34")]})
    drop_in = dict(ICMP_ACCEPT_IN, action="DROP")
    S.append({"name": "general/test_insert", "steps": [
        step(FWSETUP + [["insert", "INGRESS", None, ICMP_ACCEPT_IN], ["insert", "EGRESS", None, ICMP_ACCEPT_OUT]],
             ping_from_ns1(), "pass", "general/test_insert.sh:32"),
        step([["insert", "INGRESS", None, drop_in]], ping_from_ns1(), "fail", "general/test_insert.sh:37"),
        step([["deletes", "INGRESS", drop_in]], ping_from_ns1(), "pass", "general/test_insert.sh:44"),
        step([["insert", "INGRESS", 1, drop_in]], ping_from_ns1(), "pass", "general/test_insert.sh:51"),
        # under `set +e`: id 2 == size is allowed, id 5 > size and id -1 are refused
        step([["insert", "INGRESS", 2, drop_in], ["expect_error", ["insert", "INGRESS", 5, drop_in]],
              ["expect_error", ["insert", "INGRESS", -1, drop_in]]],
             ping_from_ns1(), "pass", "general/test_insert.sh:62")]})
    S.append({"name": "general/test_delete", "steps": [
        step(FWSETUP + [["conntrack", "OFF"], ["append", "INGRESS", ICMP_ACCEPT_IN],
                        ["append", "EGRESS", ICMP_ACCEPT_OUT]], ping_from_ns1(), "pass", "general/test_delete.sh:35"),
        step([["delete", "EGRESS", 0]], ping_from_ns1(), "fail", "general/test_delete.sh:39"),
        step([["append", "EGRESS", ICMP_ACCEPT_OUT]], ping_from_ns1(), "pass", "general/test_delete.sh:46"),
        step([["append", "EGRESS", {"src": "10.0.0.0/24", "dst": NS1 + "/32", "l4proto": "ICMP",
                                    "action": "ACCEPT"}]], ping_from_ns1(), "pass", "general/test_delete.sh:53"),
        step([["delete", "EGRESS", 1]], ping_from_ns1(), "pass", "general/test_delete.sh:61"),
        step([["delete", "EGRESS", 0]], ping_from_ns1(), "fail", "general/test_delete.sh:68"),
        step([["append", "EGRESS", ICMP_ACCEPT_OUT]], ping_from_ns1(), "pass", "general/test_delete.sh:76"),
        step([["append", "EGRESS", {"src": "10.0.0.0/24", "dst": NS1 + "/32", "l4proto": "ICMP",
                                    "action": "ACCEPT"}]], ping_from_ns1(), "pass", "general/test_delete.sh:83"),
        step([["delete", "EGRESS", 0]], ping_from_ns1(), "pass", "general/test_delete.sh:91"),
        step([["delete", "EGRESS", 0]], ping_from_ns1(), "fail", "general/test_delete.sh:98")]})
    S.append({"name": "general/test_replace", "steps": [
        step(FWSETUP + [["conntrack", "OFF"], ["append", "INGRESS", ICMP_ACCEPT_IN],
                        ["append", "EGRESS", ICMP_ACCEPT_OUT]], ping_from_ns1(), "pass", "general/test_replace.sh:34"),
        step([["delete", "EGRESS", 0]], ping_from_ns1(), "fail", "general/test_replace.sh:39"),
        step([["append", "EGRESS", ICMP_ACCEPT_OUT]], ping_from_ns1(), "pass", "general/test_replace.sh:46"),
        step([["add", "EGRESS", 0, dict(ICMP_ACCEPT_OUT, src="20.0.0.2/32")]], ping_from_ns1(), "fail",
             "general/test_replace.sh:53"),
        step([["delete", "EGRESS", 0]], ping_from_ns1(), "fail", "general/test_replace.sh:61"),
        step([["append", "EGRESS", ICMP_ACCEPT_OUT]], ping_from_ns1(), "pass", "general/test_replace.sh:66")]})
    S.append({"name": "general/test_removerule", "steps": [
        step(FWSETUP + [["append", "INGRESS", drop_in], ["append", "INGRESS", ICMP_ACCEPT_IN],
                        ["add", "EGRESS", 0, dict(ICMP_ACCEPT_OUT, action="DROP")],
                        ["add", "EGRESS", 1, ICMP_ACCEPT_OUT], ["delete", "INGRESS", 0], ["delete", "EGRESS", 0]],
             ping_from_ns1(), "pass", "general/test_removerule.sh:38")]})
    S.append({"name": "general/test_ipslpm", "steps": [
        step(FWSETUP + [["append", "INGRESS", {"src": "10.0.0.0/8", "action": "DROP"}],
                        ["append", "EGRESS", {"src": "10.0.0.0/8", "action": "DROP"}],
                        ["append", "INGRESS", {"src": NS1, "action": "ACCEPT"}],
                        ["append", "EGRESS", {"src": NS1, "action": "ACCEPT"}],
                        ["append", "INGRESS", {"src": HOST, "action": "ACCEPT"}],
                        ["append", "EGRESS", {"src": HOST, "action": "ACCEPT"}]],
             ping_from_ns1(), "fail", "general/test_ipslpm.sh:39")]})
    S.append({"name": "general/test_wrong_position", "steps": [
        step(FWSETUP + [["append", "INGRESS", ICMP_ACCEPT_IN]] + [["append", "EGRESS", ICMP_ACCEPT_OUT]] * 4 +
             [["expect_error", ["delete", "EGRESS", i]] for i in (-1, 4, 5, 10)] +
             [["expect_error", ["delete", "INGRESS", i]] for i in (-1, 1, 2, 10)],
             line="general/test_wrong_position.sh:38-61")]})
    S[-1]["steps"][0]["nrules"] = {"INGRESS": 1, "EGRESS": 4}   # "test fw to be still alive"
    S.append({"name": "general/test_counters", "steps": [
        step(FWSETUP + [["add", "INGRESS", 0, ICMP_ACCEPT_IN], ["add", "EGRESS", 0, ICMP_ACCEPT_OUT]],
             ping_from_ns1(), "pass", "general/test_counters.sh:34",
             counters=[ctr("INGRESS", 0, 2, 196), ctr("EGRESS", 0, 2, 196)])]})
    for name in ("general/test_counters_default", "general/test_counters_default_2"):
        S.append({"name": name, "steps": [
            step(FWSETUP, ping_from_ns1(), "fail", name + (".sh:30" if name.endswith("default") else ".sh:29"),
                 counters=[ctr("INGRESS", "DEFAULT", 2, 196)])]})
    S.append({"name": "general/test_counters_flush", "steps": [
        step(FWSETUP + [["add", "INGRESS", 0, ICMP_ACCEPT_IN], ["add", "EGRESS", 0, ICMP_ACCEPT_OUT]],
             ping_from_ns1(), "pass", "general/test_counters_flush.sh:33"),
        step([["reset_counters", "INGRESS"], ["reset_counters", "EGRESS"]], line="general/test_counters_flush.sh:35",
             counters=[ctr("INGRESS", 0, 0, 0), ctr("EGRESS", 0, 0, 0)])]})
    S.append({"name": "general/test_counters_reload", "steps": [
        step(FWSETUP + [["add", "INGRESS", 0, ICMP_ACCEPT_IN], ["add", "EGRESS", 0, ICMP_ACCEPT_OUT]],
             ping_from_ns1(), "pass", "general/test_counters_reload.sh:31"),
        step([["add", "INGRESS", 1, {"dst": HOST, "l4proto": "TCP", "sport": 1000, "action": "ACCEPT"}],
              ["append", "EGRESS", {"src": HOST + "/32", "dst": NS1 + "/32", "l4proto": "UDP", "dport": 1000,
                                    "action": "ACCEPT"}]], line="general/test_counters_reload.sh:37",
             counters=[ctr("INGRESS", 0, 2, 196), ctr("EGRESS", 0, 2, 196)])]})
    # ping/test_ping_1.sh: 63 TCP decoys, the ICMP accept inserted at 63, 65 more decoys (INGRESS);
    # 64 decoys, accept at 64, 65 more (EGRESS); one batch each
    ing = batch_rules(63, lambda i: r_10(i, 31, "SYN"), 63, [ICMP_ACCEPT_IN], 64, 128, lambda i: r_11(i, None, None))
    egr = batch_rules(64, lambda i: r_10(i, 32, "SYN"), 64, [ICMP_ACCEPT_OUT], 65, 129, lambda i: r_11(i, 16, "!ACK"))
    S.append({"name": "ping/test_ping_1", "steps": [
        step(FWSETUP + [["batch", "INGRESS", ing], ["batch", "EGRESS", egr]], ping_from_ns1(), "pass",
             "ping/test_ping_1.sh:81")]})
    ing = batch_rules(126, lambda i: r_10(i, 31, "SYN"), 126, [ICMP_ACCEPT_IN], 127, 250, lambda i: r_11(i, None, None))
    egr = batch_rules(63, lambda i: r_10(i, 32, "!SYN"), 63, [ICMP_ACCEPT_OUT], 64, 129,
                      lambda i: r_11(i, 16, "!ACK"))
    S.append({"name": "ping/test_ping_2", "steps": [
        step(FWSETUP + [["batch", "INGRESS", ing], ["batch", "EGRESS", egr]], ping_from_ns1(), "pass",
             "ping/test_ping_2.sh:77")]})
    tcp_in = [{"src": NS1, "dst": HOST, "l4proto": "TCP", "dport": 60123, "tcpflags": f, "action": "ACCEPT"}
              for f in ("SYN, !ACK, !RST, !FIN", "!SYN, ACK, !RST, !FIN", "!SYN, !RST, FIN")]
    tcp_out = [{"src": HOST, "dst": NS1, "l4proto": "TCP", "sport": 60123, "tcpflags": f, "action": "ACCEPT"}
               for f in ("SYN, ACK, !RST", "ACK, !SYN", "FIN, !SYN")]
    ing = batch_rules(62, lambda i: r_10(i, 31, "SYN"), 62, tcp_in, 65, 128, lambda i: r_11(i, None, None))
    egr = batch_rules(63, lambda i: r_10(i, 32, "!SYN"), 63, tcp_out, 66, 129, lambda i: r_11(i, 16, "!ACK"))
    S.append({"name": "tcp/test_tcp_1", "steps": [
        step(FWSETUP + [["batch", "INGRESS", ing], ["batch", "EGRESS", egr]], netcat_from_ns1(60123), "pass",
             "tcp/test_tcp_1.sh:88")]})
    ct_rules = [["accept_established", "OFF"],
                ["append", "INGRESS", {"conntrack": "NEW", "action": "DROP"}],
                ["append", "INGRESS", {"conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                ["append", "EGRESS", {"conntrack": "NEW", "action": "ACCEPT"}],
                ["append", "EGRESS", {"conntrack": "ESTABLISHED", "action": "ACCEPT"}]]
    S.append({"name": "conntrack/test_icmp_echo", "steps": [
        step(FWSETUP + ct_rules, ping_from_ns1(), "fail", "conntrack/test_icmp_echo.sh:38"),
        step([], ping_from_host(), "pass", "conntrack/test_icmp_echo.sh:45")]})
    S.append({"name": "conntrack/test_disable_enable", "steps": [
        step(FWSETUP + [["conntrack", "OFF"], ["append", "INGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                        ["append", "EGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}]],
             ping_from_host(), "pass", "conntrack/test_disable_enable.sh:32"),
        step([["conntrack", "ON"], ["accept_established", "ON"],
              ["add", "INGRESS", 0, {"l4proto": "ICMP", "conntrack": "NEW", "action": "DROP"}],
              ["add", "EGRESS", 0, {"l4proto": "ICMP", "conntrack": "NEW", "action": "ACCEPT"}]],
             ping_from_ns1(), "fail", "conntrack/test_disable_enable.sh:49"),
        step([], ping_from_host(), "pass", "conntrack/test_disable_enable.sh:56"),
        step([["accept_established", "OFF"],
              ["add", "INGRESS", 0, {"conntrack": "NEW", "action": "DROP"}],
              ["add", "INGRESS", 1, {"conntrack": "ESTABLISHED", "action": "ACCEPT"}],
              ["add", "EGRESS", 0, {"conntrack": "NEW", "action": "ACCEPT"}],
              ["add", "EGRESS", 1, {"conntrack": "ESTABLISHED", "action": "ACCEPT"}]],
             ping_from_ns1(), "fail", "conntrack/test_disable_enable.sh:74"),
        step([], ping_from_host(), "pass", "conntrack/test_disable_enable.sh:81")]})
    # ---- conntrack/: the stateful tests not transcribed before (round 3) ----
    # ICMP errors: the RELATED label (Firewall_ConntrackLabel_dp.c, the
    # pcn-iptables code at Iptables_ConntrackLabel_dp.c:482-531)
    err_rules = [["append", "INGRESS", {"l4proto": "UDP", "action": "ACCEPT"}],
                 ["append", "INGRESS", {"l4proto": "ICMP", "conntrack": "RELATED", "action": "ACCEPT"}],
                 ["append", "INGRESS", {"l4proto": "ICMP", "action": "DROP"}],
                 ["append", "EGRESS", {"l4proto": "UDP", "action": "ACCEPT"}],
                 ["append", "EGRESS", {"l4proto": "ICMP", "conntrack": "RELATED", "action": "ACCEPT"}],
                 ["append", "EGRESS", {"l4proto": "ICMP", "action": "DROP"}]]
    for name in ("conntrack/test_icmp_error", "conntrack/test_icmp_error_2"):
        S.append({"name": name, "steps": [
            step(FWSETUP + err_rules, nping_udp("ns1"), "pass", name + ".sh:37-41"),
            step([], nping_udp("ns1"), "pass", name + ".sh:46-50"),
            step([], pings_from_ns1(), "fail", name + ".sh:54-58"),
            step([], pings_from_host(), "fail", name + ".sh:61-65")]})
    # TCP handshakes started by the host towards ns1 (nc exit status only: no close asserted)
    S.append({"name": "conntrack/test_tcp_handshake_1", "steps": [
        step(FWSETUP + [["append", "INGRESS", {"l4proto": "TCP", "conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                        ["append", "INGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                        ["append", "EGRESS", {"l4proto": "TCP", "conntrack": "NEW", "action": "ACCEPT"}],
                        ["append", "EGRESS", {"l4proto": "TCP", "conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                        ["append", "EGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}]],
             netcat_session("host", 60123, close=False), "pass", "conntrack/test_tcp_handshake_1.sh:39-44")]})
    S.append({"name": "conntrack/test_tcp_handshake_2", "steps": [
        step(FWSETUP + [["accept_established", "ON"],
                        ["append", "INGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                        ["append", "EGRESS", {"l4proto": "TCP", "conntrack": "NEW", "action": "ACCEPT"}],
                        ["append", "EGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}]],
             netcat_session("host", 60123, close=False), "pass", "conntrack/test_tcp_handshake_2.sh:39-44")]})

    # TCP connections with the graceful close the scripts check ((2): the server exited)
    def complete(server_side, est_chain, new_chain, auto):
        ops = FWSETUP + ([["accept_established", "ON"]] if auto else [])
        ops += [["append", est_chain, {"l4proto": "TCP", "conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                ["append", est_chain, {"conntrack": "INVALID", "action": "DROP"}],
                ["append", new_chain, {"l4proto": "TCP", "conntrack": "NEW", "action": "ACCEPT"}],
                ["append", new_chain, {"l4proto": "TCP", "conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                ["append", new_chain, {"conntrack": "INVALID", "action": "DROP"}]]
        return ops
    S.append({"name": "conntrack/test_tcp_complete_2", "steps": [
        step(complete("host", "EGRESS", "INGRESS", False), netcat_session("ns1", 60123), "pass",
             "conntrack/test_tcp_complete_2.sh:42-55")]})
    S.append({"name": "conntrack/test_tcp_complete_3", "steps": [
        step(complete("ns1", "INGRESS", "EGRESS", True), netcat_session("host", 60123), "pass",
             "conntrack/test_tcp_complete_3.sh:44-57")]})
    S.append({"name": "conntrack/test_tcp_complete_4", "steps": [
        step(complete("host", "EGRESS", "INGRESS", True), netcat_session("ns1", 60123), "pass",
             "conntrack/test_tcp_complete_4.sh:44-57")]})
    # UDP: (1) a NEW datagram from ns1 is refused; (2) the host's datagram opens the
    # connection; (3)-(4) ns1's datagrams are then ESTABLISHED
    udp_manual = [["accept_established", "OFF"],
                  ["append", "INGRESS", {"l4proto": "UDP", "conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                  ["append", "INGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                  ["default", "INGRESS", "DROP"],
                  ["append", "EGRESS", {"l4proto": "UDP", "conntrack": "NEW", "action": "ACCEPT"}],
                  ["append", "EGRESS", {"l4proto": "UDP", "conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                  ["append", "EGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                  ["default", "EGRESS", "DROP"]]
    udp_auto = [["accept_established", "ON"],
                ["append", "INGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                ["default", "INGRESS", "DROP"],
                ["append", "EGRESS", {"l4proto": "UDP", "conntrack": "NEW", "action": "ACCEPT"}],
                ["append", "EGRESS", {"l4proto": "ICMP", "action": "ACCEPT"}],
                ["default", "EGRESS", "DROP"]]
    for name, rules, l1 in (("conntrack/test_udp", udp_manual, 39), ("conntrack/test_udp_2", udp_manual, 39),
                            ("conntrack/test_udp_3", udp_auto, 38), ("conntrack/test_udp_4", udp_auto, 37)):
        S.append({"name": name, "steps": [
            step(FWSETUP + rules, nping_udp("ns1"), "fail", f"{name}.sh:{l1}"),
            step([], nping_udp("host"), "pass", f"{name}.sh:{l1 + 8}"),
            step([], nping_udp("ns1"), "pass", f"{name}.sh:{l1 + 15}"),
            step([], nping_udp("ns1"), "pass", f"{name}.sh:{l1 + 25}")]})
    # ICMP echo: the NEW request from ns1 is refused, the host's ping passes
    echo_manual = [["accept_established", "OFF"],
                   ["append", "INGRESS", {"conntrack": "NEW", "action": "DROP"}],
                   ["append", "INGRESS", {"conntrack": "ESTABLISHED", "action": "ACCEPT"}],
                   ["append", "EGRESS", {"conntrack": "NEW", "action": "ACCEPT"}],
                   ["append", "EGRESS", {"conntrack": "ESTABLISHED", "action": "ACCEPT"}]]
    echo_auto = [["accept_established", "ON"],
                 ["append", "INGRESS", {"l4proto": "ICMP", "conntrack": "NEW", "action": "DROP"}],
                 ["append", "EGRESS", {"l4proto": "ICMP", "conntrack": "NEW", "action": "ACCEPT"}]]
    for name, rules, l1 in (("conntrack/test_icmp_echo_2", echo_manual, 37),
                            ("conntrack/test_icmp_echo_3", echo_auto, 35),
                            ("conntrack/test_icmp_echo_4", echo_auto, 36)):
        S.append({"name": name, "steps": [
            step(FWSETUP + rules, pings_from_ns1(), "fail", f"{name}.sh:{l1}"),
            step([], pings_from_host(), "pass", f"{name}.sh:{l1 + 7}")]})
    # ---- ping/ ----
    # test_ping_11.sh sends its second batch (the EGRESS-style rules) to INGRESS too
    # (:56): EGRESS stays empty with default DROP, and the replies pass as
    # ESTABLISHED under the default AUTOMATIC mode
    ing = batch_rules(2, lambda i: r_10(i, 31, "SYN"), 2, [ICMP_ACCEPT_IN], 3, 2, None)
    ing2 = batch_rules(2, lambda i: r_10(i, 32, "!SYN"), 2, [ICMP_ACCEPT_OUT], 3, 2, None)
    S.append({"name": "ping/test_ping_11", "steps": [
        step(FWSETUP + [["batch", "INGRESS", ing], ["batch", "INGRESS", ing2]], pings_from_ns1(), "pass",
             "ping/test_ping_11.sh:59")]})
    S.append({"name": "ping/test_ping_21.1", "steps": [
        step(FWSETUP + [["add", "INGRESS", i, r_10(i, 31, "SYN")] for i in range(2)] +
             [["add", "INGRESS", 2, ICMP_ACCEPT_IN]] +
             [["add", "EGRESS", i, r_10(i, 32, "!SYN")] for i in range(2)] +
             [["add", "EGRESS", 2, ICMP_ACCEPT_OUT]], pings_from_ns1(), "pass", "ping/test_ping_21.1.sh:48")]})
    # test_ping_5.1.sh: 4000 / 4000 rules per chain, an accept-all rule at 3500 / 3501
    ing = [dict(r_10(i, 31, "SYN"), operation="append") for i in range(3500)]
    ing += [{"operation": "append", "action": "ACCEPT"}]
    ing += [dict(r_11(i, None, None), operation="append") for i in range(3501, 4001)]
    egr = [dict(r_10(i, 32, "!SYN"), operation="append") for i in range(3501)]
    egr += [{"operation": "append", "action": "ACCEPT"}]
    egr += [dict(r_11(i, 16, "!ACK"), operation="append") for i in range(3502, 4001)]
    S.append({"name": "ping/test_ping_5.1", "steps": [
        step(FWSETUP + [["accept_established", "OFF"], ["batch", "INGRESS", ing], ["batch", "EGRESS", egr]],
             pings_from_ns1(), "pass", "ping/test_ping_5.1.sh:77"),
        step([], pings_from_host(), "pass", "ping/test_ping_5.1.sh:78")]})
    S.append({"name": "ping/test_ping_7", "steps": [
        step(FWSETUP + [["add", "INGRESS", 0, ICMP_ACCEPT_IN], ["add", "EGRESS", 0, ICMP_ACCEPT_OUT]],
             pings_from_ns1(), "pass", "ping/test_ping_7.sh:36"),
        step([], pings_from_host(), "pass", "ping/test_ping_7.sh:37")]})
    # test_ping_1_xdp.sh runs test_ping_1.sh with an argument test_ping_1.sh never reads:
    # the same rules and probe (replayed at the XDP hook, as every probe here)
    S.append(dict(next(x for x in S if x["name"] == "ping/test_ping_1"), name="ping/test_ping_1_xdp"))
    # ---- tcp/ ----
    tcp_in = [{"src": NS1, "dst": HOST, "l4proto": "TCP", "dport": 60123, "tcpflags": f, "action": "ACCEPT"}
              for f in ("SYN, !ACK, !RST, !FIN", "!SYN, ACK, !RST, !FIN", "!SYN, !RST, FIN")]
    tcp_out = [{"src": HOST, "dst": NS1, "l4proto": "TCP", "sport": 60123, "tcpflags": f, "action": "ACCEPT"}
               for f in ("SYN, ACK, !RST", "ACK, !SYN", "FIN, !SYN")]
    # test_tcp_2.sh: its netcat client runs in the background and is not asserted
    ing = batch_rules(126, lambda i: r_10(i, 31, "SYN"), 126, tcp_in, 129, 512, lambda i: r_11(i, None, None))
    egr = batch_rules(127, lambda i: r_10(i, 32, "!SYN"), 127, tcp_out, 130, 260, lambda i: r_11(i, 16, "!ACK"))
    S.append({"name": "tcp/test_tcp_2", "asserted": False, "steps": [
        step(FWSETUP + [["batch", "INGRESS", ing], ["batch", "EGRESS", egr]], netcat_session("ns1", 60123),
             "pass", "tcp/test_tcp_2.sh:91 (background, unasserted)")]})
    ing = batch_rules(6001, lambda i: r_10(i, 31, "SYN"), 6001, tcp_in, 6004, 6999, lambda i: r_11(i, None, None))
    egr = batch_rules(6997, lambda i: r_10(i, 32, "!SYN"), 127, tcp_out, 1, 0, None)
    S.append({"name": "tcp/test_tcp_4", "steps": [
        step(FWSETUP + [["accept_established", "OFF"], ["batch", "INGRESS", ing], ["batch", "EGRESS", egr]],
             netcat_session("ns1", 60123), "pass", "tcp/test_tcp_4.sh:86")]})
    ing = batch_rules(101, lambda i: r_10(i, 31, "SYN"), 101, [{"action": "ACCEPT"}], 102, 200,
                      lambda i: r_11(i, None, None))
    egr = [dict(r_10(i, 32, "!SYN"), operation="append") for i in range(63)]
    egr += [{"operation": "append", "id": 63, "action": "ACCEPT"}]
    egr += [dict({"src": f"10.1.0.{i % 255}", "dst": f"10.1.0.{i % 255}/16", "l4proto": "TCP", "sport": i,
                  "dport": i, "tcpflags": "!ACK", "action": "DROP"}, operation="append") for i in range(64, 129)]
    S.append({"name": "tcp/test_tcp_5", "steps": [
        step(FWSETUP + [["accept_established", "OFF"], ["batch", "INGRESS", ing], ["batch", "EGRESS", egr]],
             netcat_session("ns1", 60123), "pass", "tcp/test_tcp_5.sh:84")]})
    S.append({"name": "test1", "steps": [
        step(FWSETUP + [["add", "INGRESS", 0, ICMP_ACCEPT_IN], ["add", "EGRESS", 0, ICMP_ACCEPT_OUT]],
             pings_from_ns1(), "pass", "test1.sh:34")]})
    return S


def main():
    out = {"generator": "tests/golden/make_fw_scenarios.py", "ns1": NS1, "host": HOST,
           "scenarios": scenarios()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fw_scenarios.json")
    with open(path, "w") as fh:
        json.dump(out, fh, separators=(",", ":"))        # compact: the rule batches hold ~30 K rules
    print(f"wrote {path}: {len(out['scenarios'])} scenarios")


if __name__ == "__main__":
    main()
