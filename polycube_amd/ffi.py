"""ctypes binding of include/pcn_ipt.h (the product C ABI).

Loading fails loudly: there is no Python or CPU fallback for the datapath.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCN_IPT_LIBRARY: an alternative build of the same library (A/B measurements, tools/)
LIB_PATH = os.environ.get("PCN_IPT_LIBRARY") or os.path.join(_HERE, "libpcn_ipt.so")


class LibraryMissing(RuntimeError):
    pass


class Rule(C.Structure):
    _fields_ = [
        ("src", C.c_char_p), ("dst", C.c_char_p), ("l4proto", C.c_char_p),
        ("tcpflags", C.c_char_p), ("in_iface", C.c_char_p), ("out_iface", C.c_char_p),
        ("conntrack", C.c_char_p), ("sport", C.c_int32), ("dport", C.c_int32),
        ("action", C.c_int32),
    ]


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("max_counted_rules", C.c_uint32),
                ("max_action_rules", C.c_uint32), ("max_rules", C.c_uint32), ("jit", C.c_int)]


class Batch(C.Structure):
    _fields_ = [
        ("frames", C.c_void_p), ("frames_bytes", C.c_uint64), ("offsets", C.c_void_p),
        ("lens", C.c_void_p), ("stride", C.c_uint32), ("fixed_len", C.c_uint32),
        ("in_port", C.c_void_p), ("const_in_port", C.c_uint16), ("direction", C.c_uint16),
        ("hook", C.c_uint16), ("reserved", C.c_uint16),
        ("ct_status", C.c_void_p), ("n", C.c_uint64), ("verdicts", C.c_void_p),
        ("rule_ids", C.c_void_p),
    ]


class FieldMap(C.Structure):
    _fields_ = [("n", C.c_uint32), ("keys", C.POINTER(C.c_uint32)),
                ("plen", C.POINTER(C.c_uint8)), ("vecs", C.POINTER(C.c_uint64))]


class Tables(C.Structure):
    _fields_ = [("nrules", C.c_uint32), ("default_action", C.c_int),
                ("actions", C.POINTER(C.c_uint8)), ("maps", FieldMap * 8)]


class JitInfo(C.Structure):
    _fields_ = [("launches_generic", C.c_uint64), ("launches_jit", C.c_uint64),
                ("programs_ready", C.c_uint32), ("programs_failed", C.c_uint32), ("launches_split", C.c_uint64)]


class RingConfig(C.Structure):
    _fields_ = [("slots", C.c_uint32), ("slot_frames", C.c_uint32), ("slot_bytes", C.c_uint64),
                ("streams", C.c_uint32), ("flags", C.c_uint32), ("pack_threads", C.c_uint32)]


class RingSlot(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("frames", C.POINTER(C.c_uint8)), ("offsets", C.POINTER(C.c_uint32)),
                ("lens", C.POINTER(C.c_uint16)), ("in_port", C.POINTER(C.c_uint16))]


class RingStats(C.Structure):
    _fields_ = [("submits", C.c_uint64), ("frames", C.c_uint64), ("h2d_bytes", C.c_uint64), ("d2h_bytes", C.c_uint64),
                ("zc_bytes", C.c_uint64), ("pack_ns", C.c_uint64), ("submit_ns", C.c_uint64)]


class RingBatch(C.Structure):
    _fields_ = [("n", C.c_uint64), ("frames_bytes", C.c_uint64), ("stride", C.c_uint32), ("fixed_len", C.c_uint32),
                ("use_offsets", C.c_uint8), ("use_lens", C.c_uint8), ("use_in_port", C.c_uint8),
                ("hdr_skip", C.c_uint8), ("const_in_port", C.c_uint16), ("direction", C.c_uint16),
                ("hook", C.c_uint16), ("hdr_bytes", C.c_uint16)]


class ChainInfo(C.Structure):
    _fields_ = [("nrules", C.c_uint32), ("nrw", C.c_uint32), ("nsw", C.c_uint32), ("nvec", C.c_uint32),
                ("ngroups", C.c_uint32), ("present", C.c_uint32), ("table_bytes", C.c_uint32),
                ("part_bytes", C.c_uint64)]


class CtInfo(C.Structure):
    _fields_ = [("enabled", C.c_uint32), ("capacity_log2", C.c_uint32), ("now", C.c_uint64),
                ("inserts_lost", C.c_uint64), ("max_entries", C.c_uint64), ("evicted", C.c_uint64),
                ("fused_batches", C.c_uint64)]


class CommInfo(C.Structure):
    _fields_ = [("nccl_version", C.c_int), ("nranks", C.c_int), ("rank", C.c_int), ("device", C.c_int),
                ("pci_bus_id", C.c_char * 32), ("rccl_path", C.c_char * 256), ("gathers_timed", C.c_uint64),
                ("gather_ms_total", C.c_double), ("gathers_untimed", C.c_uint64)]


class HorusInfo(C.Structure):
    _fields_ = [("enabled", C.c_uint32), ("runtime", C.c_uint32), ("entries", C.c_uint32), ("fields", C.c_uint32),
                ("conntrack", C.c_uint32)]


class ProgramInfo(C.Structure):
    _fields_ = [("ready", C.c_int32), ("vgpr_count", C.c_int32), ("agpr_count", C.c_int32),
                ("sgpr_count", C.c_int32), ("vgpr_spill_count", C.c_int32), ("sgpr_spill_count", C.c_int32),
                ("scratch_bytes", C.c_uint32), ("static_lds_bytes", C.c_uint32), ("dynamic_lds_bytes", C.c_uint32),
                ("code_bytes", C.c_uint32), ("deal_window", C.c_uint32), ("hdr_asm", C.c_uint32)]


# name -> (restype, argtypes); every symbol declared in include/pcn_ipt.h
ABI_VERSION = 10           # PCN_IPT_ABI_VERSION of include/pcn_ipt.h this binding mirrors

SIGNATURES = {
    "pcn_ipt_abi_version": (C.c_int, []),
    "pcn_ipt_last_error": (C.c_char_p, []),
    "pcn_ipt_create": (C.c_int, [C.POINTER(Config), C.POINTER(C.c_void_p)]),
    "pcn_ipt_destroy": (None, [C.c_void_p]),
    "pcn_ipt_add_port": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint16]),
    "pcn_ipt_set_localip": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.c_size_t]),
    "pcn_ipt_chain_append": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Rule)]),
    "pcn_ipt_chain_insert": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(Rule)]),
    "pcn_ipt_chain_delete_id": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32]),
    "pcn_ipt_chain_delete_match": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Rule)]),
    "pcn_ipt_chain_flush": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_chain_set_default": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "pcn_ipt_set_interactive": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_chain_apply_rules": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_chain_nrules": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_load_chain": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Tables)]),
    "pcn_ipt_export_map": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.c_uint32,
                                     C.c_uint32]),
    "pcn_ipt_chain_nrw": (C.c_uint32, [C.c_void_p, C.c_int]),
    "pcn_ipt_chain_get_info": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(ChainInfo)]),
    "pcn_ipt_chain_get_image": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint8), C.c_uint32,
                                          C.POINTER(C.c_uint32), C.c_uint32]),
    "pcn_ipt_classify": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.c_void_p]),
    "pcn_ipt_synchronize": (C.c_int, [C.c_void_p]),
    "pcn_ipt_get_jit_info": (C.c_int, [C.c_void_p, C.POINTER(JitInfo)]),
    "pcn_ipt_debug_stale_canary": (C.c_int, [C.c_void_p]),
    "pcn_ipt_debug_ct_walk_passes": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]),
    "pcn_ipt_chain_program_compile": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_chain_program_compile_for": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Batch)]),
    "pcn_ipt_get_program_info": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(ProgramInfo)]),
    "pcn_ipt_embedded_source": (C.c_char_p, [C.c_int]),
    "pcn_ipt_build_sha256": (C.c_char_p, []),
    "pcn_ipt_release_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pcn_ipt_debug_clocks": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint32]),
    "pcn_ipt_debug_sort_pairs": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]),
    "pcn_ipt_read_counters": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64), C.c_int, C.c_int]),
    "pcn_ipt_chain_stats": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64)]),
    "pcn_ipt_chain_reset_counters": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_ring_create": (C.c_int, [C.c_void_p, C.POINTER(RingConfig), C.POINTER(C.c_void_p)]),
    "pcn_ipt_ring_destroy": (None, [C.c_void_p]),
    "pcn_ipt_ring_acquire": (C.c_int, [C.c_void_p, C.POINTER(RingSlot)]),
    "pcn_ipt_ring_submit": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(RingBatch)]),
    "pcn_ipt_ring_complete": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                        C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.POINTER(C.c_int32))]),
    "pcn_ipt_ring_release": (C.c_int, [C.c_void_p, C.c_uint32]),
    "pcn_ipt_ring_get_stats": (C.c_int, [C.c_void_p, C.POINTER(RingStats), C.c_int]),
    "pcn_ipt_set_horus": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_get_horus_info": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(HorusInfo)]),
    "pcn_ipt_read_horus_counters": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                              C.c_uint32, C.c_int]),
    "pcn_ipt_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "pcn_ipt_comm_init": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
    "pcn_ipt_sync_counters": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pcn_ipt_comm_get_info": (C.c_int, [C.c_void_p, C.POINTER(CommInfo)]),
    "pcn_ipt_counter_block_words": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_snapshot_counters": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "pcn_ipt_sum_counter_blocks": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_uint32, C.c_uint64,
                                             C.c_void_p]),
    "pcn_ipt_flow_owner": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.c_uint32, C.c_void_p, C.c_void_p]),
    "pcn_ipt_flow_split": (C.c_int, [C.c_void_p, C.POINTER(Batch), C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p]),
    "pcn_ipt_ct_enable": (C.c_int, [C.c_void_p, C.c_uint32]),
    "pcn_ipt_ct_disable": (C.c_int, [C.c_void_p]),
    "pcn_ipt_ct_clear": (C.c_int, [C.c_void_p]),
    "pcn_ipt_ct_set_max_entries": (C.c_int, [C.c_void_p, C.c_uint64]),
    "pcn_ipt_ct_set_time": (C.c_int, [C.c_void_p, C.c_uint64]),
    "pcn_ipt_ct_dump": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "pcn_ipt_ct_get_info": (C.c_int, [C.c_void_p, C.POINTER(CtInfo)]),
    "pcn_ipt_set_accept_established": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "pcn_ipt_get_accept_established": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_read_accept_established": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64),
                                                  C.POINTER(C.c_uint64), C.c_int]),
    "pcn_ipt_set_service": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_ipt_get_service": (C.c_int, [C.c_void_p]),
    "pcn_fw_set_conntrack": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_fw_set_accept_established": (C.c_int, [C.c_void_p, C.c_int]),
    "pcn_fw_get_conntrack_mode": (C.c_int, [C.c_void_p]),
    "pcn_fw_chain_update": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(Rule)]),
}

_lib = None


def lib():
    """Load libpcn_ipt.so (built by __graft_entry__.build() / `make -C polycube_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch (if already imported) owns the process's HIP runtime; libpcn_ipt.so
        # binds to the same libamdhip64.so.7 soname, so device pointers are shared.
        h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if h.pcn_ipt_abi_version() != ABI_VERSION:   # a stale build would mis-read the structs
            raise LibraryMissing(f"{LIB_PATH} has ABI {h.pcn_ipt_abi_version()}, this binding expects {ABI_VERSION}: rebuild")
        _lib = h
    return _lib


def last_error():
    msg = lib().pcn_ipt_last_error()
    return msg.decode() if msg else ""
