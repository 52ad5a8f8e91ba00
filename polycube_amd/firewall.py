"""Python host mirroring the pcn-firewall cube API over the same C ABI.

pcn-firewall (src/services/pcn-firewall) is the transparent-cube sibling of
pcn-iptables: the same field modules, BitScan, ActionLookup and rule compiler,
with two chains selected by the packet's direction.  A context switched to the
firewall service (pcn_ipt_set_service) runs them through the same kernel.

  Firewall                 -> Firewall.cpp:20-82 (INGRESS + EGRESS chains, AUTOMATIC conntrack)
  Firewall.conntrack       -> Firewall.cpp:144-195 (getConntrack / setConntrack)
  Firewall.accept_established -> Firewall.cpp:112-142
  FwChain.append           -> Chain.cpp:89-108 (action required)
  FwChain.insert           -> Chain.cpp:691-758
  FwChain.add / replace    -> Chain.cpp:612-658 (addRule: replace at id, append at id == size)
  FwChain.delete / deletes -> Chain.cpp:660-683, 760-771 (no match is an error)
  FwChain.flush            -> Chain.cpp:685-689 (delRuleList)
  FwChain.batch            -> Chain.cpp:773-819 (INSERT/APPEND/DELETE/UPDATE, one reload)
  FwChain.default          -> Chain.cpp:60-82
  FwChain.stats            -> Chain.cpp:527-569 (DEFAULT row last)
  FwChain.reset_counters   -> Chain.cpp:110-167
Invalid input raises IptablesError, like a handler's {kGenericError, msg}.
"""
import ctypes as C

from . import ffi
from .iptables import ACCEPT, DROP, FORWARD, OUTPUT, Chain, Iptables, IptablesError, _check, make_rule

SERVICE_IPTABLES, SERVICE_FIREWALL = 0, 1
INGRESS_CHAIN, EGRESS_CHAIN = FORWARD, OUTPUT       # PCN_FW_INGRESS / PCN_FW_EGRESS slots
CT_DISABLED, CT_MANUAL, CT_AUTOMATIC = 0, 1, 2       # ConntrackModes (defines.h:56-58)
_FW_CHAINS = {"INGRESS": INGRESS_CHAIN, "EGRESS": EGRESS_CHAIN}


class FwChain(Chain):
    """One pcn-firewall chain (INGRESS or EGRESS)."""

    def add(self, id, **fields):  # noqa: A002 (REST leaf name)
        """`chain <C> rule add <id> ...`: Chain::addRule -- replace the rule at
        id (its counters carry on) or append when id == number of rules."""
        _check(ffi.lib().pcn_fw_chain_update(self._h(), self.id, id, C.byref(make_rule(**fields))))

    replace = add

    def batch(self, ops):
        """Chain::batch: ops are dicts with 'operation' (insert/append/delete/
        update) plus rule fields and 'id'.  Every op runs, the chain is
        compiled once, and failed ops are reported by their 1-based position
        (Chain.cpp:773-819)."""
        ipt = self._ipt
        was = ipt.interactive
        ipt.interactive = False
        failed = []
        try:
            for k, op in enumerate(ops, 1):
                op = dict(op)
                kind = str(op.pop("operation", "")).lower()
                rid = op.pop("id", None)
                try:
                    if kind == "delete":
                        if rid is not None:
                            self.delete(rid)
                        else:
                            self.deletes(**op)
                    elif kind == "insert" and rid is not None:
                        self.insert(rid, **op)
                    elif kind == "append":
                        self.append(**op)
                    elif kind == "update" and rid is not None:
                        self.add(rid, **op)
                    else:
                        failed.append(k)
                except IptablesError:
                    failed.append(k)
        finally:
            ipt.interactive = was
            self.apply_rules()
        if failed:
            raise IptablesError(-22, f"Chain::ChainBatchOutput: you required {len(ops)} operations, but the "
                                     f"following nth{{1-{len(ops)}}} ones in the list failed: "
                                     f"[{', '.join(map(str, failed))}]")


class Firewall(Iptables):
    """One pcn-firewall cube bound to one GPU (device=-1: control plane only).

    classify(direction=INGRESS) runs the INGRESS chain, EGRESS the EGRESS
    chain; the rest of the datapath API (rings, counters, RCCL sync) is the
    pcn-iptables one."""

    def __init__(self, device=0, max_counted_rules=0, max_action_rules=0, max_rules=0, jit=0):
        super().__init__(device, max_counted_rules, max_action_rules, max_rules, jit)
        _check(ffi.lib().pcn_ipt_set_service(self._h, SERVICE_FIREWALL))
        self.chains = {name: FwChain(self, cid) for name, cid in _FW_CHAINS.items()}

    def chain(self, name):
        return self.chains[name.upper()] if isinstance(name, str) else FwChain(self, name)

    _HORUS_CHAIN = INGRESS_CHAIN

    def _horus_chain(self, chain):
        """Horus programs are per chain here (INGRESS / EGRESS; Firewall.h:333-340)."""
        if chain is None:
            return self._HORUS_CHAIN
        return _FW_CHAINS[chain.upper()] if isinstance(chain, str) else int(chain)

    @property
    def conntrack_mode(self):
        return _check(ffi.lib().pcn_fw_get_conntrack_mode(self._h))

    @property
    def conntrack(self):
        return "OFF" if self.conntrack_mode == CT_DISABLED else "ON"

    @conntrack.setter
    def conntrack(self, v):
        on = v if isinstance(v, bool) else str(v).upper() == "ON"
        _check(ffi.lib().pcn_fw_set_conntrack(self._h, int(on)))

    @property
    def accept_established(self):
        return "ON" if self.conntrack_mode == CT_AUTOMATIC else "OFF"

    @accept_established.setter
    def accept_established(self, v):
        on = v if isinstance(v, bool) else str(v).upper() == "ON"
        _check(ffi.lib().pcn_fw_set_accept_established(self._h, int(on)))


__all__ = ["Firewall", "FwChain", "INGRESS_CHAIN", "EGRESS_CHAIN", "CT_DISABLED", "CT_MANUAL",
           "CT_AUTOMATIC", "ACCEPT", "DROP"]
