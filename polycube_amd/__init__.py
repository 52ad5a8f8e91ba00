"""polycube_amd — MI355X-native pcn-iptables (and pcn-firewall) classification datapath.

The product is the C-ABI library ``libpcn_ipt.so`` (HIP kernels for gfx950 +
the C++ control-plane mirror, see include/pcn_ipt.h).  This package is the thin
Python host over that ABI, mirroring the reference's pcn-iptables REST verbs
(Chain append/insert/delete/default/stats, services/pcn-iptables/src/Chain.cpp)
so the parity tests read like the reference's own scenario tests.
"""
from .ffi import lib, LibraryMissing  # noqa: F401
from .iptables import Iptables, Chain, IptablesError, INPUT, FORWARD, OUTPUT  # noqa: F401
from .iptables import INGRESS, EGRESS, DROP, ACCEPT, XDP, TC  # noqa: F401
from .firewall import Firewall, FwChain  # noqa: F401

__all__ = ["lib", "LibraryMissing", "Iptables", "Chain", "IptablesError", "INPUT", "FORWARD",
           "OUTPUT", "INGRESS", "EGRESS", "DROP", "ACCEPT", "XDP", "TC", "Firewall", "FwChain"]
