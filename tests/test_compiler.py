"""The product rule compiler (C++, libpcn_ipt.so) emits exactly the per-field
{key -> bitvector} maps of the reference compiler (Utils.cpp:223-732), as
restated by the oracle — CPU only, control-plane context (device=-1)."""
import pytest

from oracle.ffi import Oracle
from polycube_amd import FORWARD, OUTPUT, Iptables, IptablesError
from polycube_amd import synth
from rulegen import PORTS, quirky_rules

FIELDS = range(8)


def both(rules, chain, default="DROP"):
    o = Oracle()
    ipt = Iptables(device=-1)
    for name, idx in PORTS.items():
        o.add_port(name, idx)
        ipt.add_port(name, idx)
    o.set_chain(chain, rules, default)
    ipt.interactive = False
    ch = ipt.chain(chain)
    for r in rules:
        ch.append(**r)
    ch.apply_rules()
    return o, ch


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("chain", [FORWARD, OUTPUT])
def test_maps_equal_oracle_quirky(seed, chain):
    rules = quirky_rules(20 + 37 * seed, seed)
    o, ch = both(rules, chain)
    for f in FIELDS:
        ok, op, ov, onrw = o.export_map(chain, f)
        pk, pp, pv, pnrw = ch.export_map(f)
        assert onrw == pnrw
        assert pk == ok, f"field {f} keys"
        if f in (1, 2):
            assert pp == op, f"field {f} prefix lengths"
        assert pv == ov, f"field {f} vectors"


@pytest.mark.parametrize("cfg", [1, 2, 3])
def test_maps_equal_oracle_configs(cfg):
    rules = synth.config_rules(cfg).rules()
    o, ch = both(rules, FORWARD)
    for f in FIELDS:
        assert ch.export_map(f)[:3] == o.export_map(FORWARD, f)[:3]


def test_rule_count_beyond_64_uses_multiword_vectors():
    rules = [{"dst": f"192.168.10.{h}", "l4proto": "UDP", "dport": p, "action": "ACCEPT"}
             for h in range(2, 13) for p in range(8080, 8089)]
    o, ch = both(rules, FORWARD)
    keys, _, vecs, nrw = ch.export_map(5)
    assert nrw == 2 and len(rules) == 99
    assert vecs == o.export_map(FORWARD, 5)[2]


def test_invalid_rules_are_rejected_like_the_reference():
    ipt = Iptables(device=-1)
    fw = ipt.chain("FORWARD")
    bad = [dict(src="10.0.0.0/33"), dict(dst="1.2.3"), dict(l4proto="SCTP"),
           dict(tcpflags="SYN !SYN"), dict(in_iface="nope"), dict(action="LOG"), dict(sport=70000),
           dict(conntrack="BOGUS")]
    for b in bad:
        with pytest.raises(IptablesError):
            fw.append(**b)
    assert len(fw) == 0
    # glibc "%hhu" wraps 300 to 44, so the reference accepts this address (utils.cpp:43)
    fw.append(src="300.1.1.1")
    assert fw.export_map(1)[0] == [0x0101012C]
    fw.flush()
    with pytest.raises(IptablesError):
        fw.insert(3, src="1.1.1.1")          # Chain.cpp:238-240 "id not allowed"
    with pytest.raises(IptablesError):
        fw.delete(0)                          # "There is no rule 0"
    fw.append(src="1.1.1.1", action="DROP")
    fw.deletes(src="2.2.2.2", action="DROP")  # no match: silently nothing (Chain.cpp:334-352)
    assert len(fw) == 1
    fw.deletes(src="1.1.1.1")                 # action unset == DROP
    assert len(fw) == 0


def test_insert_delete_keep_reference_ids():
    ipt = Iptables(device=-1)
    fw = ipt.chain("FORWARD")
    fw.append(src="10.0.0.1", action="ACCEPT")
    fw.append(src="10.0.0.2", action="ACCEPT")
    fw.insert(1, src="10.0.0.3", action="DROP")
    keys, plen, vecs, _ = fw.export_map(1)
    # rule ids after insert: 0 -> .1, 1 -> .3, 2 -> .2
    by = {k: v[0] for k, v in zip(keys, vecs)}
    nbo = synth.ip_nbo
    assert by[nbo(0x0A000001)] == 1 << 0 and by[nbo(0x0A000003)] == 1 << 1 and by[nbo(0x0A000002)] == 1 << 2
    fw.delete(0)
    keys, _, vecs, _ = fw.export_map(1)
    by = {k: v[0] for k, v in zip(keys, vecs)}
    assert by == {nbo(0x0A000003): 1, nbo(0x0A000002): 2}


def test_non_interactive_stages_until_apply():
    ipt = Iptables(device=-1)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    fw.append(dport=80)
    assert fw.export_map(5)[0] == []
    fw.apply_rules()
    assert fw.export_map(5)[0] == [80]
