"""ctypes wrapper of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")


class _Rule(C.Structure):
    _fields_ = [
        ("src", C.c_char_p), ("dst", C.c_char_p), ("l4proto", C.c_char_p),
        ("tcpflags", C.c_char_p), ("in_iface", C.c_char_p), ("out_iface", C.c_char_p),
        ("conntrack", C.c_char_p), ("sport", C.c_int32), ("dport", C.c_int32),
        ("action", C.c_int32),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        h = C.CDLL(LIB_PATH)
        vp, u8p, u16p, u32p, u64p, i32p = (C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint16),
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                           C.POINTER(C.c_int32))
        h.orc_create.restype = vp
        h.orc_create.argtypes = [C.c_uint32, C.c_uint32]
        h.orc_destroy.argtypes = [vp]
        h.orc_add_port.argtypes = [vp, C.c_char_p, C.c_uint16]
        h.orc_set_chain.argtypes = [vp, C.c_int, C.POINTER(_Rule), C.c_uint32, C.c_int]
        h.orc_set_localip.argtypes = [vp, u32p, C.c_uint32]
        h.orc_set_service.argtypes = [vp, C.c_int, C.c_int]
        h.orc_classify.argtypes = [vp, C.c_int, C.c_int, vp, vp, vp, C.c_uint32, C.c_uint32, vp, C.c_uint16,
                                   vp, C.c_uint64, vp, vp, C.c_int]
        h.orc_classify_labels.argtypes = [vp, C.c_int, C.c_int, vp, vp, vp, C.c_uint32, C.c_uint32, vp,
                                          C.c_uint16, vp, C.c_uint64, vp, vp, vp, C.c_int]
        h.orc_read_counters.argtypes = [vp, C.c_int, u64p, u64p, C.c_uint32, u64p, u64p, C.c_int]
        h.orc_export_map.argtypes = [vp, C.c_int, C.c_int, u32p, u8p, u64p, C.c_uint32, C.c_uint32]
        h.orc_chain_nrw.restype = C.c_uint32
        h.orc_chain_nrw.argtypes = [vp, C.c_int]
        h.orc_index64.argtypes = [u16p]
        h.orc_ct_enable.argtypes = [vp, C.c_int]
        h.orc_ct_set_time.argtypes = [vp, C.c_uint64]
        h.orc_ct_dump.argtypes = [vp, vp, C.c_uint32]
        h.orc_ct_set_max_entries.argtypes = [vp, C.c_uint64]
        h.orc_ct_info.argtypes = [vp, u64p]
        h.orc_apply_accept_established.argtypes = [vp, C.c_int]
        h.orc_set_accept_established.argtypes = [vp, C.c_int, C.c_int]
        h.orc_get_accept_established.argtypes = [vp, C.c_int]
        h.orc_read_accept_established.argtypes = [vp, C.c_int, u64p, u64p, C.c_int]
        h.orc_set_horus.argtypes = [vp, C.c_int]
        h.orc_horus_info.argtypes = [vp, C.c_int, u32p]
        h.orc_read_horus_counters.argtypes = [vp, C.c_int, u64p, u64p, C.c_uint32, C.c_int]
        h.orc_set_default.argtypes = [vp, C.c_int, C.c_int]
        _lib = h
    return _lib


# orc_ct_entry / pcn_ipt_ct_entry (same layout)
CT_ENTRY = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
                     ("l4proto", "u1"), ("state", "u1"), ("ip_rev", "u1"), ("port_rev", "u1"),
                     ("sequence", "<u4"), ("ttl", "<u8")], align=True)
CT_STATES = ["NEW", "ESTABLISHED", "RELATED", "INVALID", "SYN_SENT", "SYN_RECV", "FIN_WAIT_1",
             "FIN_WAIT_2", "LAST_ACK", "TIME_WAIT"]


def _enc(v):
    return None if v is None else str(v).encode()


def _rule(d):
    act = d.get("action")
    if isinstance(act, str):
        act = {"DROP": 0, "ACCEPT": 1}[act.upper()]
    g = d.get
    return _Rule(_enc(g("src")), _enc(g("dst")), _enc(g("l4proto")), _enc(g("tcpflags")),
                 _enc(g("in_iface")), _enc(g("out_iface")), _enc(g("conntrack")),
                 -1 if g("sport") is None else int(g("sport")),
                 -1 if g("dport") is None else int(g("dport")), -1 if act is None else int(act))


def _ptr(a):
    return None if a is None else a.ctypes.data


class Oracle:
    """Reference-semantics classifier on the CPU (see pcn_ipt_oracle.c)."""

    def __init__(self, max_counted_rules=0, max_action_rules=0):
        self._h = lib().orc_create(max_counted_rules, max_action_rules)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_destroy(self._h)
            self._h = None

    def add_port(self, name, index):
        assert lib().orc_add_port(self._h, name.encode(), index) == 0

    def set_chain(self, chain, rules, default="ACCEPT"):
        d = {"DROP": 0, "ACCEPT": 1}[default.upper()] if isinstance(default, str) else int(default)
        arr = (_Rule * max(len(rules), 1))(*[_rule(r) for r in rules])
        rc = lib().orc_set_chain(self._h, chain, arr, len(rules), d)
        if rc:
            raise ValueError(f"oracle rejected chain (rc={rc})")

    def set_service(self, service, fw_ct_mode=0):
        """0 = pcn-iptables, 1 = pcn-firewall with conntrack mode 0 DISABLED /
        1 MANUAL / 2 AUTOMATIC (pcn-firewall defines.h:56-58)."""
        assert lib().orc_set_service(self._h, service, fw_ct_mode) == 0

    def set_localip(self, ips):
        a = (C.c_uint32 * max(len(ips), 1))(*ips)
        assert lib().orc_set_localip(self._h, a, len(ips)) == 0

    def classify(self, frames, n=None, offsets=None, lens=None, stride=64, fixed_len=64,
                 in_port=None, const_in_port=1, direction=0, ct_status=None, nthreads=1, hook=0,
                 with_labels=False):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        if n is None:
            n = len(offsets) if offsets is not None else frames.size // stride
        offsets = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint32)
        lens = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
        in_port = None if in_port is None else np.ascontiguousarray(in_port, dtype=np.uint16)
        ct_status = None if ct_status is None else np.ascontiguousarray(ct_status, dtype=np.uint8)
        verdicts = np.zeros(n, dtype=np.uint8)
        rule_ids = np.zeros(n, dtype=np.int32)
        labels = np.zeros(n, dtype=np.uint8) if with_labels else None
        lib().orc_classify_labels(self._h, direction, hook, _ptr(frames), _ptr(offsets), _ptr(lens), stride,
                                  fixed_len, _ptr(in_port), const_in_port, _ptr(ct_status), n,
                                  _ptr(verdicts), _ptr(rule_ids), _ptr(labels), nthreads)
        if with_labels:
            return verdicts, rule_ids, labels
        return verdicts, rule_ids

    def read_counters(self, chain, n, flush=False):
        pk = (C.c_uint64 * max(n, 1))()
        by = (C.c_uint64 * max(n, 1))()
        dp, db = C.c_uint64(), C.c_uint64()
        lib().orc_read_counters(self._h, chain, pk, by, n, C.byref(dp), C.byref(db), int(flush))
        return list(pk[:n]), list(by[:n]), dp.value, db.value

    # ---- stateful conntrack ----
    def ct_enable(self, on=True):
        assert lib().orc_ct_enable(self._h, int(on)) == 0

    def ct_set_time(self, ns):
        assert lib().orc_ct_set_time(self._h, int(ns)) == 0

    def ct_set_max_entries(self, m):
        """Live entries kept after each batch (LRU over the touches; 0: unbounded)."""
        assert lib().orc_ct_set_max_entries(self._h, int(m)) == 0

    def ct_info(self):
        out = (C.c_uint64 * 4)()
        assert lib().orc_ct_info(self._h, out) == 0
        return {"live": out[0], "evicted": out[1], "max_entries": out[2], "seq": out[3]}

    def ct_dump(self, cap=1 << 20):
        out = np.zeros(cap, CT_ENTRY)
        n = lib().orc_ct_dump(self._h, out.ctypes.data, cap)
        assert n >= 0, n
        return out[:n]

    def apply_accept_established(self, chain):
        assert lib().orc_apply_accept_established(self._h, chain) == 0

    def set_accept_established(self, chain, on):
        assert lib().orc_set_accept_established(self._h, chain, int(on)) == 0

    def accept_established(self, chain):
        return bool(lib().orc_get_accept_established(self._h, chain))

    def read_accept_established(self, chain, flush=False):
        pk, by = C.c_uint64(), C.c_uint64()
        lib().orc_read_accept_established(self._h, chain, C.byref(pk), C.byref(by), int(flush))
        return pk.value, by.value

    def set_default(self, chain, default):
        """pcn-firewall Chain::setDefault: the default action alone, no chain update."""
        d = {"DROP": 0, "ACCEPT": 1}[default.upper()] if isinstance(default, str) else int(default)
        assert lib().orc_set_default(self._h, chain, d) == 0

    # ---- Horus (Iptables_Horus_dp.c, Firewall_Horus_dp.c) ----
    def set_horus(self, on):
        assert lib().orc_set_horus(self._h, int(on)) == 0

    def horus_info(self, chain=0):
        """chain: 0 (pcn-iptables INPUT), 1 / 2 (pcn-firewall INGRESS / EGRESS)."""
        out = (C.c_uint32 * 5)()
        assert lib().orc_horus_info(self._h, chain, out) == 0
        return {"enabled": out[0], "runtime": out[1], "entries": out[2], "fields": out[3], "conntrack": out[4]}

    def read_horus_counters(self, n, flush=False, chain=0):
        pk = (C.c_uint64 * max(n, 1))()
        by = (C.c_uint64 * max(n, 1))()
        assert lib().orc_read_horus_counters(self._h, chain, pk, by, n, int(flush)) == 0
        return list(pk[:n]), list(by[:n])

    def export_map(self, chain, field, cap=70000):
        nrw = lib().orc_chain_nrw(self._h, chain)
        keys = (C.c_uint32 * cap)()
        plen = (C.c_uint8 * cap)()
        vecs = (C.c_uint64 * (cap * max(nrw, 1)))()
        n = lib().orc_export_map(self._h, chain, field, keys, plen, vecs, cap, nrw)
        assert n >= 0
        return ([keys[i] for i in range(n)], [plen[i] for i in range(n)],
                [list(vecs[i * nrw:(i + 1) * nrw]) for i in range(n)], nrw)


def index64():
    out = (C.c_uint16 * 64)()
    lib().orc_index64(out)
    return list(out)
