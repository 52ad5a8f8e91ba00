"""Pin the oracle's pcn-firewall mode against the reference's own firewall tests (CPU only).

fw_scenarios.json transcribes src/services/pcn-firewall/test/{general,ping,tcp,conntrack}
(make_fw_scenarios.py): every connectivity assertion must come out as the script
expects, replayed packet by packet through the oracle with its connection table.
"""
import pytest

from helpers import OracleFwCube, load_fw_scenarios
from oracle.ffi import Oracle

SCEN = load_fw_scenarios()


def check_counters(cube, st, where):
    for c in st.get("counters", []):
        rules, dflt = cube.chain_stats(c["chain"])
        got = dflt if c["rule"] == "DEFAULT" else rules[c["rule"]]
        want = (c.get("datapath_pkts", c["pkts"]), c.get("datapath_bytes", c["bytes"]))
        assert tuple(got) == want, f"{where}: counters {c}: {got}"


@pytest.mark.parametrize("sc", SCEN["scenarios"], ids=[s["name"] for s in SCEN["scenarios"]])
def test_reference_firewall_scenarios_on_oracle(sc):
    cube = OracleFwCube(Oracle())
    for k, st in enumerate(sc["steps"]):
        where = f"{sc['name']} step {k} ({st.get('ref_line', '')})"
        for op in st["ops"]:
            cube.op(op)
        if "probe" in st:
            verdicts, _ = cube.probe(st["probe"])
            got = "pass" if all(v == 1 for v in verdicts) else "fail"
            assert got == st["expect"], f"{where}: {verdicts}"
        for c, n in st.get("nrules", {}).items():
            assert len(cube.rules[c]) == n, where
        check_counters(cube, st, where)


def test_divergent_counter_assertions_are_the_auto_accepted_replies():
    """The two EGRESS counter assertions the datapath cannot meet (see
    make_fw_scenarios.AUTO_REPLY) are met once accept-established is OFF:
    the replies then run the EGRESS chain (ESTABLISHED is still their label)."""
    sc = next(s for s in SCEN["scenarios"] if s["name"] == "general/test_counters")
    cube = OracleFwCube(Oracle())
    cube.op(["accept_established", "OFF"])
    st = sc["steps"][0]
    for op in st["ops"]:
        cube.op(op)
    verdicts, labels = cube.probe(st["probe"])
    assert verdicts == [1] * 4 and labels == [0, 1, 0, 1]
    for c in st["counters"]:
        rules, _ = cube.chain_stats(c["chain"])
        assert rules[c["rule"]] == (c["pkts"], c["bytes"])


def test_firewall_dispatch_differs_from_iptables_where_the_reference_does():
    """No localip / allow logic; empty chain counts its default; no ICMP
    length checks with conntrack off."""
    from helpers import ct_probe_frames
    o = Oracle()
    o.set_service(1, 0)                          # conntrack DISABLED
    o.set_chain(1, [], "ACCEPT")
    o.set_chain(2, [], "DROP")
    short_icmp = {"dir": "ingress", "port": 1, "src": "1.1.1.1", "dst": "2.2.2.2", "proto": 1, "sport": 0,
                  "dport": 0, "flags": 0, "icmp_type": 3, "len": 40}
    f, lens, ports = ct_probe_frames([short_icmp])
    v, r = o.classify(f, n=1, lens=lens, stride=128, in_port=ports, direction=0)
    assert (v[0], r[0]) == (1, -1)               # classified: empty INGRESS -> default ACCEPT, counted
    _, _, dp, db = o.read_counters(1, 0)
    assert (dp, db) == (1, 40)
    o.set_service(1, 1)                          # conntrack ON: the ICMP length check drops first
    v, r = o.classify(f, n=1, lens=lens, stride=128, in_port=ports, direction=0)
    assert (v[0], r[0]) == (0, -2)
    udp = dict(short_icmp, proto=17, sport=53, dport=53, len=64)
    f, lens, ports = ct_probe_frames([udp])
    v, r = o.classify(f, n=1, lens=lens, stride=128, in_port=ports, direction=1)
    assert (v[0], r[0]) == (0, -1)               # egress always runs EGRESS (pcn-iptables: PASS w/o localip)
    o.set_service(0, 0)
    o.set_chain(2, [], "DROP")
    assert tuple(o.classify(f, n=1, lens=lens, stride=128, in_port=ports, direction=1)[0]) == (1,)
