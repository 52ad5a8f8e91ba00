"""Chains the reference's maps cannot hold are refused like the reference refuses
them: an IP field with more than 1,024 distinct prefixes overflows the kernel LPM
trie (Iptables_IpLookup_dp.c:54-55); the map push in Chain::updateChain
(modules/IpLookup.cpp:130-140) then throws "Table set error: No space left on
device" (libs/polycube/src/table.cpp:61-66) at the verb that runs the update:
every append / insert in interactive mode, apply_rules otherwise.  The product
returns -ENOSPC with "LPM trie full" at that verb; the oracle refuses the same
rule set.  Control plane only (no GPU)."""
import errno

import pytest

from oracle.ffi import Oracle
from polycube_amd import Firewall, Iptables, IptablesError

CAP = 1024


def _rules(n, field="src"):
    return [{field: f"10.{k >> 8 & 255}.{k & 255}.1/32", "action": "ACCEPT"} for k in range(n)]


def _refused(exc):
    return exc.value.code == -errno.ENOSPC and "LPM trie full" in str(exc.value)


@pytest.mark.parametrize("field", ["src", "dst"])
def test_interactive_append_past_the_trie_is_refused_at_that_append(field):
    ipt = Iptables(device=-1)
    ch = ipt.chain("FORWARD")
    rules = _rules(CAP + 1, field)
    for r in rules[:CAP]:
        ch.append(**r)
    with pytest.raises(IptablesError) as e:
        ch.append(**rules[CAP])
    assert _refused(e)
    o = Oracle()
    o.set_chain(1, rules[:CAP], "DROP")
    with pytest.raises(ValueError, match="rc=-28"):
        o.set_chain(1, rules, "DROP")
    ipt.close()


def test_non_interactive_chain_is_refused_at_apply_rules():
    ipt = Iptables(device=-1)
    ipt.interactive = False
    ch = ipt.chain("INPUT")
    for r in _rules(CAP + 40):
        ch.append(**r)                      # staged: nothing pushed yet
    with pytest.raises(IptablesError) as e:
        ch.apply_rules()
    assert _refused(e)
    ipt.close()


def test_same_prefix_twice_is_one_trie_entry():
    """(len, prefix) is the trie key: repeats of a prefix take no extra entry."""
    ipt = Iptables(device=-1)
    ipt.interactive = False
    ch = ipt.chain("FORWARD")
    rules = _rules(CAP) + _rules(CAP)[:50]
    for r in rules:
        ch.append(**r)
    ch.apply_rules()
    Oracle().set_chain(1, rules, "DROP")
    ipt.close()


def test_firewall_chain_past_the_trie_is_refused():
    fw = Firewall(device=-1)
    fw.interactive = False
    ch = fw.chain("INGRESS")
    for r in _rules(CAP + 1):
        ch.append(**r)
    with pytest.raises(IptablesError) as e:
        ch.apply_rules()
    assert _refused(e)
    o = Oracle()
    o.set_service(1, 2)
    with pytest.raises(ValueError, match="rc=-28"):
        o.set_chain(1, _rules(CAP + 1), "DROP")
    fw.close()
