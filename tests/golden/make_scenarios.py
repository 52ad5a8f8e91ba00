"""Transcribe the reference's pcn-iptables integration tests into replayable fixtures.

Source: /root/reference/src/services/pcn-iptables/test/local_test*.sh (read as text).
Each reference script builds namespaces/veths, edits rules with pcn-iptables /
polycubectl, and asserts connectivity: a plain `ping`/`netcat`/`nping` line must
succeed, a `test_fail ...` line must fail (helpers.bash:68-78).  Here every such
assertion becomes a *probe*: the packets that traffic puts through the cube, in
the direction and on the port where the cube sees them, plus the expected
outcome taken from the script ("pass" = every packet ACCEPTed, "fail" = at least
one DROPped).  The expected outcomes are the reference's own assertions, not
oracle output, so replaying them pins the oracle and the GPU datapath.

Topology constants (helpers.bash:28-42): ns1 10.0.1.1 behind host veth1
(10.0.1.254), ns2 10.0.2.1 behind host veth2 (10.0.2.254); the host's default
route leaves through eth0 (10.10.0.10 here); `$ip` = 8.8.8.8.  pcn-iptables
numbers rules from 1 (-D CHAIN 2 deletes id 1); -I without a number inserts at 0.

Run:  python tests/golden/make_scenarios.py   (writes scenarios.json next to it)
"""
import json
import os

HOST = "10.10.0.10"
PORTS = {"veth1": 1, "veth2": 2, "eth0": 3}
LOCAL = [HOST, "10.0.1.254", "10.0.2.254"]
IP = "8.8.8.8"


def pkt(direction, port, src, dst, proto, sport=0, dport=0, flags=0, icmp_type=None, length=None,
        ct=None):
    p = {"dir": direction, "port": PORTS[port], "src": src, "dst": dst, "proto": proto,
         "sport": sport, "dport": dport, "flags": flags}
    if icmp_type is not None:
        p["icmp_type"] = icmp_type
    p["len"] = length if length is not None else (98 if proto == 1 else 64 if proto == 17 else 74)
    if ct is not None:
        p["ct"] = ct
    return p


def ping_host():
    """`ping $ip` from the host: echo request out of eth0 (OUTPUT), reply in (INPUT)."""
    return [pkt("egress", "eth0", HOST, IP, 1, icmp_type=8),
            pkt("ingress", "eth0", IP, HOST, 1, icmp_type=0)]


def ping_fwd():
    """`ip netns exec ns1 ping 10.0.2.1`: forwarded both ways (FORWARD), PASS on egress."""
    return [pkt("ingress", "veth1", "10.0.1.1", "10.0.2.1", 1, icmp_type=8),
            pkt("egress", "veth2", "10.0.1.1", "10.0.2.1", 1, icmp_type=8),
            pkt("ingress", "veth2", "10.0.2.1", "10.0.1.1", 1, icmp_type=0),
            pkt("egress", "veth1", "10.0.2.1", "10.0.1.1", 1, icmp_type=0)]


def ping_fwd_rev():
    """`ip netns exec ns2 ping 10.0.1.1`: the same exchange started from ns2."""
    return [pkt("ingress", "veth2", "10.0.2.1", "10.0.1.1", 1, icmp_type=8),
            pkt("egress", "veth1", "10.0.2.1", "10.0.1.1", 1, icmp_type=8),
            pkt("ingress", "veth1", "10.0.1.1", "10.0.2.1", 1, icmp_type=0),
            pkt("egress", "veth2", "10.0.1.1", "10.0.2.1", 1, icmp_type=0)]


def tcp_fwd(port):
    """`netcat -nvz 10.0.2.1 <port>` from ns1: SYN forward, SYN-ACK back."""
    return [pkt("ingress", "veth1", "10.0.1.1", "10.0.2.1", 6, 40000, port, 0x02),
            pkt("ingress", "veth2", "10.0.2.1", "10.0.1.1", 6, port, 40000, 0x12)]


def nping_udp():
    """`ip netns exec ns2 nping --udp 10.0.1.1`: 5 UDP probes (sport 53, dport 40125), NEW."""
    return [pkt("ingress", "veth2", "10.0.2.1", "10.0.1.1", 17, 53, 40125, ct=0) for _ in range(5)]


def step(ops, probe=None, expect=None, line=None, counters=None):
    s = {"ops": ops}
    if probe is not None:
        s["probe"] = probe
        s["expect"] = expect
    if counters is not None:
        s["counters"] = counters
    if line is not None:
        s["ref_line"] = line
    return s


def A(chain, **r):
    return ["append", chain, r]


def I(chain, idx=0, **r):  # noqa: E743
    return ["insert", chain, idx, r]


def D(chain, **r):
    return ["deletes", chain, r]


def P(chain, action):
    return ["default", chain, action]


def scenarios():
    out = []
    # ---------------- local_test1.sh ----------------
    t = "src/services/pcn-iptables/test/local_test1.sh"
    out.append({"name": "local_test1", "source": t, "steps": [
        step([], ping_host(), "pass", f"{t}:21"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_host(), "pass", f"{t}:26"),
        step([P("INPUT", "DROP")], ping_host(), "fail", f"{t}:30"),
        step([A("INPUT", src=IP, dst="10.0.22.0/24", l4proto="TCP", sport=80, dport=90, tcpflags="SYN",
                action="ACCEPT")], ping_host(), "fail", f"{t}:34"),
        step([A("INPUT", src=IP, dst=IP, l4proto="TCP", sport=80, dport=90, tcpflags="SYN", action="ACCEPT")],
             ping_host(), "fail", f"{t}:38"),
        step([A("INPUT", src=IP, l4proto="ICMP", action="ACCEPT")], ping_host(), "pass", f"{t}:42"),
        step([P("OUTPUT", "DROP")], ping_host(), "fail", f"{t}:48"),
        step([A("OUTPUT", dst=IP, src="10.0.22.0/24", l4proto="TCP", sport=80, dport=90, tcpflags="SYN",
                action="ACCEPT")], ping_host(), "fail", f"{t}:52"),
        step([A("OUTPUT", src=IP, dst=IP, l4proto="TCP", sport=80, dport=90, tcpflags="SYN", action="ACCEPT")],
             ping_host(), "fail", f"{t}:56"),
        step([A("OUTPUT", dst=IP, l4proto="ICMP", action="ACCEPT")], ping_host(), "pass", f"{t}:60"),
    ]})
    # ---------------- local_test3_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test3_iptables.sh"
    out.append({"name": "local_test3_iptables", "source": t, "steps": [
        step([], ping_host(), "pass"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_host(), "pass"),
        step([P("INPUT", "DROP")], ping_host(), "fail"),
        step([A("INPUT", src=IP, action="ACCEPT")], ping_host(), "pass"),
        step([I("INPUT", 0, src=IP, action="DROP")], ping_host(), "fail"),
        step([D("INPUT", src=IP, action="ACCEPT")], ping_host(), "fail"),
        step([D("INPUT", src=IP, action="DROP")], ping_host(), "fail"),
        step([P("INPUT", "ACCEPT")], ping_host(), "pass"),
        step([P("INPUT", "DROP")], ping_host(), "fail"),
        step([["flush", "INPUT"], P("INPUT", "ACCEPT")], ping_host(), "pass"),
        step([P("INPUT", "DROP")], ping_host(), "fail"),
        step([A("INPUT", src=IP, l4proto="TCP", action="DROP")], ping_host(), "fail"),
        step([A("INPUT", src=IP, action="ACCEPT")], ping_host(), "pass"),
        step([A("INPUT", src=IP, l4proto="UDP", action="DROP")], ping_host(), "pass"),
        step([["delete", "INPUT", 1]], ping_host(), "fail"),
        step([P("INPUT", "ACCEPT")]),
    ]})
    # ---------------- local_test8_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test8_iptables.sh"
    out.append({"name": "local_test8_iptables", "source": t, "steps": [
        step([], ping_fwd(), "pass"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP")], ping_fwd(), "pass"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT"), P("FORWARD", "DROP")], ping_fwd(), "fail"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP"), I("FORWARD", 0, src="10.0.0.0/8", action="ACCEPT")],
             ping_fwd(), "pass"),
        step([D("FORWARD", src="10.0.0.0/8", action="ACCEPT")], ping_fwd(), "fail"),
        step([A("FORWARD", src="10.0.0.0/8", action="ACCEPT")], ping_fwd(), "pass"),
        step([D("FORWARD", src="10.0.0.0/8", action="ACCEPT")], ping_fwd(), "fail"),
        step([I("FORWARD", 0, src="10.0.0.0/8", action="ACCEPT")], ping_fwd(), "pass"),
        step([D("FORWARD", src="10.0.0.0/8", action="ACCEPT")], ping_fwd(), "fail"),
    ]})
    # ---------------- local_test9_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test9_iptables.sh"
    out.append({"name": "local_test9_iptables", "source": t, "steps": [
        step([], ping_fwd(), "pass"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP")], ping_fwd(), "pass"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT"), P("FORWARD", "DROP")], ping_fwd(), "fail"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP"), A("FORWARD", src="10.0.1.1", action="ACCEPT"),
              A("FORWARD", src="10.0.2.1", action="ACCEPT")], ping_fwd(), "pass"),
        step([I("FORWARD", 0, src="10.0.0.0/8", action="DROP")], ping_fwd(), "fail"),
        step([D("FORWARD", src="10.0.0.0/8", action="DROP")], ping_fwd(), "pass"),
        step([A("FORWARD", src="10.0.0.0/8", action="DROP")], ping_fwd(), "pass"),
        step([I("FORWARD", 0, src="10.0.1.0/24", action="DROP")], ping_fwd(), "fail"),
        step([I("FORWARD", 0, src="10.0.2.0/24", action="DROP")], ping_fwd(), "fail"),
    ]})
    # ---------------- local_test20_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test20_iptables.sh"
    out.append({"name": "local_test20_iptables", "source": t, "steps": [
        step([], ping_fwd(), "pass"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP"), P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT"),
              P("FORWARD", "DROP"), P("INPUT", "DROP"), P("OUTPUT", "DROP")], tcp_fwd(81), "fail"),
        step([A("FORWARD", src="10.0.1.1", dst="10.0.2.1", l4proto="TCP", dport=80, action="ACCEPT"),
              A("FORWARD", dst="10.0.1.1", src="10.0.2.1", l4proto="TCP", sport=80, action="ACCEPT")],
             tcp_fwd(80), "pass"),
        step([D("FORWARD", src="10.0.1.1", dst="10.0.2.1", l4proto="TCP", dport=80, action="ACCEPT"),
              D("FORWARD", dst="10.0.1.1", src="10.0.2.1", l4proto="TCP", sport=80, action="ACCEPT")],
             tcp_fwd(80), "fail"),
        step([P("FORWARD", "ACCEPT")], tcp_fwd(91), "pass"),
        step([A("FORWARD", src="10.0.1.0/24", dst="10.0.2.1", l4proto="TCP", dport=90, action="DROP")],
             tcp_fwd(90), "fail"),
    ]})
    # ---------------- local_test_interfaces1.sh ----------------
    t = "src/services/pcn-iptables/test/local_test_interfaces1.sh"
    out.append({"name": "local_test_interfaces1", "source": t, "steps": [
        step([], ping_fwd(), "pass"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP")], ping_fwd(), "pass"),
        step([P("FORWARD", "DROP")], ping_fwd(), "fail"),
        step([A("FORWARD", in_iface="veth1", action="ACCEPT")], ping_fwd(), "fail"),
        step([A("FORWARD", in_iface="veth2", action="ACCEPT")], ping_fwd(), "pass"),
        step([D("FORWARD", in_iface="veth1", action="ACCEPT")], ping_fwd(), "fail"),
        step([D("FORWARD", in_iface="veth2", action="ACCEPT")], ping_fwd(), "fail"),
        step([P("FORWARD", "ACCEPT")], ping_fwd(), "pass"),
        step([["flush", "FORWARD"]], ping_fwd(), "pass"),
        step([P("FORWARD", "DROP")], ping_fwd(), "fail"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_host(), "pass"),
        step([A("INPUT", in_iface="eth0", action="DROP")], ping_host(), "fail"),
        step([D("INPUT", in_iface="eth0", action="DROP")], ping_host(), "pass"),
        step([A("OUTPUT", out_iface="eth0", action="DROP")], ping_host(), "fail"),
        step([D("OUTPUT", out_iface="eth0", action="DROP")], ping_host(), "pass"),
    ]})
    # ---------------- local_test30_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test30_iptables.sh"
    big = [A("FORWARD", conntrack="ESTABLISHED", action="ACCEPT"),
           A("FORWARD", conntrack="NEW", src="10.0.2.1", action="ACCEPT")]
    big += [A("FORWARD", conntrack="NEW", src=f"192.168.10.{k}", action="ACCEPT") for k in range(3, 12)]
    big += [A("FORWARD", dst=f"192.168.10.{h}", l4proto="UDP", dport=p, action="ACCEPT")
            for h in range(2, 13) for p in range(8080, 8089)]
    out.append({"name": "local_test30_iptables", "source": t, "ports_note": "nping --udp: sport 53 dport 40125",
                "steps": [
        step([], nping_udp(), "pass"),
        step([A("FORWARD", conntrack="ESTABLISHED", action="ACCEPT"),
              A("FORWARD", conntrack="NEW", src="10.0.2.1", action="ACCEPT")], nping_udp(), "pass",
             counters={"chain": "FORWARD", "rule": 1, "pkts": 5}),
        step([["flush", "FORWARD"], ["interactive", False]] + big + [["apply", "FORWARD"]], nping_udp(), "pass",
             counters={"chain": "FORWARD", "rule": 1, "pkts": 5}),
    ]})
    # ---------------- local_test1_iptables.sh ----------------
    # local_test1.sh through the pcn-iptables CLI; `--tcp-flags SYN SYN` (mask
    # SYN, set SYN) is the tcpflags='SYN' of local_test1.sh:30-34
    t = "src/services/pcn-iptables/test/local_test1_iptables.sh"
    out.append({"name": "local_test1_iptables", "source": t, "steps": [
        step([], ping_host(), "pass", f"{t}:19"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_host(), "pass", f"{t}:24"),
        step([P("INPUT", "DROP")], ping_host(), "fail", f"{t}:29"),
        step([A("INPUT", src=IP, dst="10.0.22.0/24", l4proto="TCP", sport=80, dport=90, tcpflags="SYN",
                action="ACCEPT")], ping_host(), "fail", f"{t}:33"),
        step([A("INPUT", src=IP, dst=IP, l4proto="TCP", sport=80, dport=90, tcpflags="SYN", action="ACCEPT")],
             ping_host(), "fail", f"{t}:37"),
        step([A("INPUT", src=IP, l4proto="ICMP", action="ACCEPT")], ping_host(), "pass", f"{t}:41"),
        step([P("OUTPUT", "DROP")], ping_host(), "fail", f"{t}:46"),
        step([A("OUTPUT", dst=IP, src="10.0.22.0/24", l4proto="TCP", sport=80, dport=90, tcpflags="SYN",
                action="ACCEPT")], ping_host(), "fail", f"{t}:50"),
        step([A("OUTPUT", src=IP, dst=IP, l4proto="TCP", sport=80, dport=90, tcpflags="SYN", action="ACCEPT")],
             ping_host(), "fail", f"{t}:54"),
        step([A("OUTPUT", dst=IP, l4proto="ICMP", action="ACCEPT")], ping_host(), "pass", f"{t}:59"),
    ]})
    # ---------------- local_test2_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test2_iptables.sh"
    out.append({"name": "local_test2_iptables", "source": t, "steps": [
        step([], ping_host(), "pass", f"{t}:18"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_host(), "pass", f"{t}:23"),
        step([P("INPUT", "DROP")], ping_host(), "fail", f"{t}:27"),
        step([A("INPUT", src=IP, action="ACCEPT")], ping_host(), "pass", f"{t}:31"),
        step([I("INPUT", 0, src=IP, action="DROP")], ping_host(), "fail", f"{t}:35"),
        step([D("INPUT", src=IP, action="DROP")], ping_host(), "pass", f"{t}:39"),
    ]})
    # ---------------- local_test4_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test4_iptables.sh"
    out.append({"name": "local_test4_iptables", "source": t, "steps": [
        step([], ping_fwd(), "pass", f"{t}:41"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP")], ping_fwd(), "pass", f"{t}:46"),
        step([P("FORWARD", "DROP")], ping_fwd(), "fail", f"{t}:50"),
    ]})
    # ---------------- local_test5_iptables.sh ----------------
    # bidirectional FORWARD drops with insert/delete; both ping directions asserted
    t = "src/services/pcn-iptables/test/local_test5_iptables.sh"
    both = ping_fwd() + ping_fwd_rev()
    out.append({"name": "local_test5_iptables", "source": t, "steps": [
        step([], ping_fwd(), "pass", f"{t}:41"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP")], ping_fwd(), "pass", f"{t}:46"),
        step([P("FORWARD", "DROP")], ping_fwd(), "fail", f"{t}:50"),
        step([A("FORWARD", dst="10.0.2.1", src="10.0.1.1", action="DROP")], ping_fwd(), "fail", f"{t}:54"),
        step([], ping_fwd_rev(), "fail", f"{t}:55"),
        step([I("FORWARD", 0, src="10.0.2.1", dst="10.0.1.1", action="DROP")], ping_fwd(), "fail", f"{t}:59"),
        step([], ping_fwd_rev(), "fail", f"{t}:60"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_fwd(), "fail", f"{t}:65"),
        step([], ping_fwd_rev(), "fail", f"{t}:66"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP"), I("FORWARD", 0, src="10.0.2.1", action="ACCEPT"),
              I("FORWARD", 0, src="10.0.1.1", action="ACCEPT")], both, "pass", f"{t}:74-75"),
        step([D("FORWARD", src="10.0.2.1", action="ACCEPT"), D("FORWARD", src="10.0.1.1", action="ACCEPT")],
             ping_fwd(), "fail", f"{t}:80"),
        step([], ping_fwd_rev(), "fail", f"{t}:81"),
        step([D("FORWARD", dst="10.0.2.1", src="10.0.1.1", action="DROP"),
              D("FORWARD", src="10.0.2.1", dst="10.0.1.1", action="DROP")], ping_fwd(), "fail", f"{t}:86"),
        step([], ping_fwd_rev(), "fail", f"{t}:87"),
        step([P("FORWARD", "DROP"), A("FORWARD", l4proto="ICMP", action="ACCEPT")], both, "pass", f"{t}:93-94"),
    ]})
    # ---------------- local_test7_iptables.sh ----------------
    t = "src/services/pcn-iptables/test/local_test7_iptables.sh"
    out.append({"name": "local_test7_iptables", "source": t, "steps": [
        step([], ping_fwd(), "pass", f"{t}:57"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP")], ping_fwd(), "pass", f"{t}:62"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT"), P("FORWARD", "DROP")], ping_fwd(), "fail", f"{t}:68"),
        step([P("INPUT", "DROP"), P("OUTPUT", "DROP"), A("FORWARD", src="10.0.1.1", action="ACCEPT"),
              A("FORWARD", src="10.0.2.1", action="ACCEPT")], ping_fwd(), "pass", f"{t}:76"),
    ]})
    # ---------------- local_test_horus1.sh ----------------
    # `polycubectl pcn-iptables set horus=ON|OFF` only sets the flag
    # (Iptables::setHorus); the next INPUT update builds the Horus program.
    t = "src/services/pcn-iptables/test/local_test_horus1.sh"
    out.append({"name": "local_test_horus1", "source": t, "steps": [
        step([], ping_host(), "pass", f"{t}:16"),
        step([P("INPUT", "ACCEPT"), P("OUTPUT", "ACCEPT")], ping_host(), "pass", f"{t}:21"),
        step([P("INPUT", "DROP")], ping_host(), "fail", f"{t}:25"),
        step([P("INPUT", "ACCEPT"), ["horus", "ON"]], ping_host(), "pass", f"{t}:31"),
        step([A("INPUT", src=IP, action="DROP")], ping_host(), "fail", f"{t}:35"),
        step([D("INPUT", src=IP, action="DROP")], ping_host(), "pass", f"{t}:41"),
        step([["horus", "OFF"]], ping_host(), "pass", f"{t}:47"),
        step([A("INPUT", src=IP, action="DROP")], ping_host(), "fail", f"{t}:51"),
        step([D("INPUT", src=IP, action="DROP")], ping_host(), "pass", f"{t}:55"),
    ]})
    return out


if __name__ == "__main__":
    doc = {"generator": "tests/golden/make_scenarios.py", "ports": PORTS, "localip": LOCAL,
           "scenarios": scenarios()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenarios.json")
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(f"wrote {path}: {len(doc['scenarios'])} scenarios")
