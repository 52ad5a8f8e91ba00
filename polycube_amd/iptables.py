"""Python host mirroring the pcn-iptables cube API over the C ABI.

Names and error behaviour follow the reference REST surface:
  Iptables            -> services/pcn-iptables/src/Iptables.cpp (cube, ports, localip)
  Chain.append/insert -> Chain.cpp:139-300
  Chain.delete/deletes-> Chain.cpp:302-352, 1039-1064
  Chain.flush         -> Chain.cpp:1066-1073 (delRuleList)
  Chain.default       -> Chain.cpp:79-127 (setDefault)
  Chain.apply_rules   -> Chain.cpp:382-392 (applyRules)
  Chain.stats         -> Chain.cpp:931-976 (getStats/getStatsList, DEFAULT row last)
  Chain.reset_counters-> Chain.cpp:354-380
Invalid input raises IptablesError, like a handler's {kGenericError, msg}.
"""
import ctypes as C

from . import ffi

INPUT, FORWARD, OUTPUT = 0, 1, 2
INGRESS, EGRESS = 0, 1
XDP, TC = 0, 1            # attach point (pcn_ipt_batch.hook)
DROP, ACCEPT = 0, 1
_CHAIN_NAMES = {"INPUT": INPUT, "FORWARD": FORWARD, "OUTPUT": OUTPUT}
_ACTIONS = {"DROP": DROP, "ACCEPT": ACCEPT}


def _ct_entry_dtype():
    import numpy as np
    # pcn_ipt_ct_entry (include/pcn_ipt.h)
    return np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
                     ("l4proto", "u1"), ("state", "u1"), ("ip_rev", "u1"), ("port_rev", "u1"),
                     ("sequence", "<u4"), ("ttl", "<u8")], align=True)


CT_ENTRY = _ct_entry_dtype()
CT_STATES = ["NEW", "ESTABLISHED", "RELATED", "INVALID", "SYN_SENT", "SYN_RECV", "FIN_WAIT_1",
             "FIN_WAIT_2", "LAST_ACK", "TIME_WAIT"]


class IptablesError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (errno {-code})")
        self.code = code


def _check(rc):
    if rc < 0:
        raise IptablesError(rc, ffi.last_error())
    return rc


def _enc(v):
    return None if v is None else str(v).encode()


def comm_info(handle=None):
    """pcn_ipt_comm_get_info as a dict; without a context handle only the RCCL facts."""
    out = ffi.CommInfo()
    _check(ffi.lib().pcn_ipt_comm_get_info(handle, C.byref(out)))
    d = {k: getattr(out, k) for k, _ in ffi.CommInfo._fields_}
    for k in ("pci_bus_id", "rccl_path"):
        d[k] = d[k].decode(errors="replace")
    v = d["nccl_version"]
    d["rccl_version"] = f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v else None
    return d


def embedded_kernel_hash():
    """sha-256 (16 hex digits) of classify.hip + devchain.h + image.cpp as the LOADED
    library carries them (pcn_ipt_embedded_source): what decides the bytes a classify
    launch reads, taken from the build that runs, not from the files on disk."""
    import hashlib
    h = hashlib.sha256()
    for which in (0, 1, 3):
        h.update(ffi.lib().pcn_ipt_embedded_source(which))
    return h.hexdigest()[:16]


def build_sha256():
    """sha-256 of every library source at the loaded library's build time."""
    return ffi.lib().pcn_ipt_build_sha256().decode()


def make_rule(src=None, dst=None, l4proto=None, sport=None, dport=None, tcpflags=None,
              in_iface=None, out_iface=None, conntrack=None, action=None):
    """Build a pcn_ipt_rule from REST-style fields (None = not set)."""
    if isinstance(action, str):
        if action.upper() not in _ACTIONS:
            raise IptablesError(-22, f"Action not supported: {action}")
        action = _ACTIONS[action.upper()]
    r = ffi.Rule(_enc(src), _enc(dst), _enc(l4proto), _enc(tcpflags), _enc(in_iface),
                 _enc(out_iface), _enc(conntrack), -1 if sport is None else int(sport),
                 -1 if dport is None else int(dport), -1 if action is None else int(action))
    return r


class Chain:
    def __init__(self, ipt, cid):
        self._ipt = ipt
        self.id = cid

    def _h(self):
        return self._ipt._h

    def append(self, **fields):
        _check(ffi.lib().pcn_ipt_chain_append(self._h(), self.id, C.byref(make_rule(**fields))))

    def insert(self, id=0, **fields):  # noqa: A002 (REST leaf name)
        _check(ffi.lib().pcn_ipt_chain_insert(self._h(), self.id, id, C.byref(make_rule(**fields))))

    def delete(self, id):  # noqa: A002
        _check(ffi.lib().pcn_ipt_chain_delete_id(self._h(), self.id, id))

    def deletes(self, **fields):
        _check(ffi.lib().pcn_ipt_chain_delete_match(self._h(), self.id, C.byref(make_rule(**fields))))

    def flush(self):
        _check(ffi.lib().pcn_ipt_chain_flush(self._h(), self.id))

    @property
    def default(self):
        return self._ipt._defaults[self.id]

    @default.setter
    def default(self, action):
        a = _ACTIONS[action.upper()] if isinstance(action, str) else int(action)
        _check(ffi.lib().pcn_ipt_chain_set_default(self._h(), self.id, a))
        self._ipt._defaults[self.id] = a

    def apply_rules(self):
        _check(ffi.lib().pcn_ipt_chain_apply_rules(self._h(), self.id))

    def __len__(self):
        return _check(ffi.lib().pcn_ipt_chain_nrules(self._h(), self.id))

    def stats(self):
        """[(id, pkts, bytes), ...] + [("DEFAULT", pkts, bytes)] (getStatsList)."""
        n = len(self)
        pk = (C.c_uint64 * max(n, 1))()
        by = (C.c_uint64 * max(n, 1))()
        dp, db = C.c_uint64(), C.c_uint64()
        _check(ffi.lib().pcn_ipt_chain_stats(self._h(), self.id, pk, by, n, C.byref(dp), C.byref(db)))
        return [(i, pk[i], by[i]) for i in range(n)] + [("DEFAULT", dp.value, db.value)]

    def reset_counters(self):
        _check(ffi.lib().pcn_ipt_chain_reset_counters(self._h(), self.id))

    @property
    def accept_established(self):
        """Accept-established optimization on for this chain (Iptables.h accept_established_enabled_*)."""
        return bool(_check(ffi.lib().pcn_ipt_get_accept_established(self._h(), self.id)))

    @accept_established.setter
    def accept_established(self, on):
        _check(ffi.lib().pcn_ipt_set_accept_established(self._h(), self.id, int(bool(on))))

    def read_accept_established(self, flush=False):
        """(pkts, bytes) of pkts/bytes_acceptestablished_<Chain>."""
        pk, by = C.c_uint64(), C.c_uint64()
        _check(ffi.lib().pcn_ipt_read_accept_established(self._h(), self.id, C.byref(pk), C.byref(by),
                                                          int(flush)))
        return pk.value, by.value

    def read_counters(self, n, flush=False, scope=0):
        """Raw datapath counters: (pkts[n], bytes[n], def_pkts, def_bytes)."""
        pk = (C.c_uint64 * max(n, 1))()
        by = (C.c_uint64 * max(n, 1))()
        dp, db = C.c_uint64(), C.c_uint64()
        _check(ffi.lib().pcn_ipt_read_counters(self._h(), self.id, pk, by, n, C.byref(dp),
                                               C.byref(db), int(flush), int(scope)))
        return list(pk[:n]), list(by[:n]), dp.value, db.value

    def info(self):
        """Shape of the compiled device image (pcn_ipt_chain_get_info)."""
        out = ffi.ChainInfo()
        _check(ffi.lib().pcn_ipt_chain_get_info(self._h(), self.id, C.byref(out)))
        return {k: getattr(out, k) for k, _ in ffi.ChainInfo._fields_}

    def program_info(self):
        """Resources of this chain's chain program (pcn_ipt_get_program_info): VGPRs,
        SGPRs, scratch and LDS bytes, deal window; ready = 1 once compiled."""
        out = ffi.ProgramInfo()
        _check(ffi.lib().pcn_ipt_get_program_info(self._h(), self.id, C.byref(out)))
        return {k: getattr(out, k) for k, _ in ffi.ProgramInfo._fields_}

    def compile_program(self, n=None, offsets=False, lens=False, stride=64, fixed_len=64, in_port=False,
                        ct_status=False, direction=None, hook=XDP):
        """Compile this chain's chain program now: for its usual launch shape
        (pcn_ipt_chain_program_compile), or, given any shape argument, for the launch
        shape of such a batch (pcn_ipt_chain_program_compile_for; IMIX: offsets=lens=True)."""
        if n is None and not (offsets or lens or in_port or ct_status or hook or direction is not None
                              or stride != 64 or fixed_len != 64):
            _check(ffi.lib().pcn_ipt_chain_program_compile(self._h(), self.id))
            return
        fake = 1 << 12      # never read: a plan reads no buffer
        b = ffi.Batch()
        b.n = n or (1 << 20)
        b.offsets = fake if offsets else None
        b.lens = fake if lens else None
        b.stride, b.fixed_len = stride, fixed_len
        b.in_port = fake if in_port else None
        b.ct_status = fake if ct_status else None
        b.const_in_port = 1
        b.direction = (EGRESS if self.id == 2 else INGRESS) if direction is None else direction
        b.hook = hook
        _check(ffi.lib().pcn_ipt_chain_program_compile_for(self._h(), self.id, C.byref(b)))

    def export_map(self, field, cap=70000):
        nrw = ffi.lib().pcn_ipt_chain_nrw(self._h(), self.id)
        keys = (C.c_uint32 * cap)()
        plen = (C.c_uint8 * cap)()
        vecs = (C.c_uint64 * (cap * max(nrw, 1)))()
        n = _check(ffi.lib().pcn_ipt_export_map(self._h(), self.id, field, keys, plen, vecs, cap, nrw))
        return ([keys[i] for i in range(n)], [plen[i] for i in range(n)],
                [list(vecs[i * nrw:(i + 1) * nrw]) for i in range(n)], nrw)


class Iptables:
    """One pcn-iptables cube bound to one GPU (device=-1: control plane only)."""

    def __init__(self, device=0, max_counted_rules=0, max_action_rules=0, max_rules=0, jit=0):
        """jit: 0 chain programs compiled in the background, 1 compiled before the
        first launch of a new shape, -1 generic kernel only (pcn_ipt_config.jit)."""
        cfg = ffi.Config(device, max_counted_rules, max_action_rules, max_rules, jit)
        h = C.c_void_p()
        _check(ffi.lib().pcn_ipt_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.device = device
        self._defaults = [ACCEPT, ACCEPT, ACCEPT]
        self.chains = {name: Chain(self, cid) for name, cid in _CHAIN_NAMES.items()}

    def chain(self, name):
        return self.chains[name.upper()] if isinstance(name, str) else Chain(self, name)

    def close(self):
        if self._h:
            ffi.lib().pcn_ipt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def release_stream(self, stream):
        """pcn_ipt_release_stream: before destroying a stream that carried batches."""
        _check(ffi.lib().pcn_ipt_release_stream(self._h, stream))

    def add_port(self, name, index):
        _check(ffi.lib().pcn_ipt_add_port(self._h, name.encode(), index))

    def set_localip(self, ips_nbo):
        arr = (C.c_uint32 * max(len(ips_nbo), 1))(*ips_nbo)
        _check(ffi.lib().pcn_ipt_set_localip(self._h, arr, len(ips_nbo)))

    @property
    def interactive(self):
        return self._interactive if hasattr(self, "_interactive") else True

    @interactive.setter
    def interactive(self, v):
        _check(ffi.lib().pcn_ipt_set_interactive(self._h, int(bool(v))))
        self._interactive = bool(v)

    def load_chain(self, chain, tables):
        _check(ffi.lib().pcn_ipt_load_chain(self._h, chain, C.byref(tables)))

    # ---- Horus (the `horus` leaf, iptables.yang:112-118) ----
    _HORUS_CHAIN = 0           # the chain whose program horus_info() / read_horus_counters() name by default

    @property
    def horus(self):
        """"ON" / "OFF" (Iptables::getHorus); setting it takes effect at the next chain update."""
        return "ON" if self.horus_info()["enabled"] else "OFF"

    @horus.setter
    def horus(self, v):
        on = v if isinstance(v, bool) else str(v).upper() == "ON"
        _check(ffi.lib().pcn_ipt_set_horus(self._h, int(on)))

    def _horus_chain(self, chain):
        if chain is None:
            return self._HORUS_CHAIN
        return _CHAIN_NAMES[chain.upper()] if isinstance(chain, str) else int(chain)

    def horus_info(self, chain=None):
        """The Horus program of `chain` (pcn-iptables: INPUT)."""
        out = ffi.HorusInfo()
        _check(ffi.lib().pcn_ipt_get_horus_info(self._h, self._horus_chain(chain), C.byref(out)))
        return {k: getattr(out, k) for k, _ in ffi.HorusInfo._fields_}

    def read_horus_counters(self, n, flush=False, chain=None):
        """pkts_horus / bytes_horus of rule ids 0..n-1 (lists)."""
        pk = (C.c_uint64 * max(n, 1))()
        by = (C.c_uint64 * max(n, 1))()
        _check(ffi.lib().pcn_ipt_read_horus_counters(self._h, self._horus_chain(chain), pk, by, n, int(flush)))
        return list(pk[:n]), list(by[:n])

    # ---- datapath (device pointers; torch tensors accepted for convenience) ----
    def classify_ptrs(self, frames, frames_bytes, n, verdicts, rule_ids=None, offsets=None,
                      lens=None, stride=64, fixed_len=64, in_port=None, const_in_port=1,
                      direction=INGRESS, ct_status=None, stream=None, hook=XDP):
        b = ffi.Batch(frames, frames_bytes, offsets, lens, stride, fixed_len, in_port, const_in_port,
                      direction, hook, 0, ct_status, n, verdicts, rule_ids)
        _check(ffi.lib().pcn_ipt_classify(self._h, C.byref(b), stream))

    def classify(self, frames, n=None, verdicts=None, rule_ids=None, offsets=None, lens=None,
                 stride=64, fixed_len=64, in_port=None, const_in_port=1, direction=INGRESS,
                 ct_status=None, stream=None, hook=XDP):
        """Classify device-resident frames (torch uint8 tensor on cuda).  Returns
        (verdicts, rule_ids) tensors; the call is asynchronous on `stream`."""
        import torch
        if n is None:
            n = offsets.numel() if offsets is not None else frames.numel() // stride
        dev = frames.device
        if verdicts is None:
            verdicts = torch.empty(n, dtype=torch.uint8, device=dev)
        if rule_ids is None:
            rule_ids = torch.empty(n, dtype=torch.int32, device=dev)

        def p(t):
            return None if t is None else t.data_ptr()
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        self.classify_ptrs(frames.data_ptr(), frames.numel(), n, verdicts.data_ptr(),
                           p(rule_ids) if rule_ids is not False else None, p(offsets), p(lens),
                           stride, fixed_len, p(in_port), const_in_port, direction, p(ct_status), s, hook)
        return verdicts, rule_ids

    def jit_info(self):
        """Chain-program statistics (pcn_ipt_get_jit_info)."""
        out = ffi.JitInfo()
        _check(ffi.lib().pcn_ipt_get_jit_info(self._h, C.byref(out)))
        return {k: getattr(out, k) for k, _ in ffi.JitInfo._fields_}

    def synchronize(self):
        _check(ffi.lib().pcn_ipt_synchronize(self._h))

    def ring(self, slots=4, slot_frames=1 << 20, slot_bytes=None, streams=0, rule_ids=False, zero_copy=False,
             host_pack=False, pack_threads=0):
        """Host ingest ring (pcn_ipt_ring_*): pinned slots -> HBM -> classify -> verdicts.
        zero_copy: the kernel reads the frames in the pinned slots over PCIe (PCN_IPT_RING_ZERO_COPY);
        host_pack: header-only submits pack the windows on host threads, one contiguous copy
        (PCN_IPT_RING_HOST_PACK)."""
        return IngestRing(self, slots, slot_frames, slot_bytes or 64 * slot_frames, streams, rule_ids, zero_copy,
                          host_pack, pack_threads)

    # ---- stateful connection tracking ----
    def ct_enable(self, capacity_log2=0):
        _check(ffi.lib().pcn_ipt_ct_enable(self._h, capacity_log2))

    def ct_disable(self):
        _check(ffi.lib().pcn_ipt_ct_disable(self._h))

    def ct_clear(self):
        _check(ffi.lib().pcn_ipt_ct_clear(self._h))

    def ct_set_time(self, ns):
        _check(ffi.lib().pcn_ipt_ct_set_time(self._h, int(ns)))

    def ct_set_max_entries(self, m):
        """Live entries kept after each batch (LRU over the touches; 0: unbounded)."""
        _check(ffi.lib().pcn_ipt_ct_set_max_entries(self._h, int(m)))

    def ct_dump(self):
        """Live connections (session table), as a numpy array of CT_ENTRY, sorted by key."""
        import numpy as np
        n = _check(ffi.lib().pcn_ipt_ct_dump(self._h, None, 0))
        out = np.zeros(max(n, 1), CT_ENTRY)
        n = _check(ffi.lib().pcn_ipt_ct_dump(self._h, out.ctypes.data, len(out)))
        return out[:n]

    def ct_info(self):
        out = ffi.CtInfo()
        _check(ffi.lib().pcn_ipt_ct_get_info(self._h, C.byref(out)))
        return {k: getattr(out, k) for k, _ in ffi.CtInfo._fields_}

    # ---- multi-GPU counters over RCCL ----
    @staticmethod
    def comm_unique_id():
        buf = (C.c_uint8 * 128)()
        _check(ffi.lib().pcn_ipt_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, nranks, rank, uid):
        buf = (C.c_uint8 * 128)(*uid)
        _check(ffi.lib().pcn_ipt_comm_init(self._h, nranks, rank, buf))

    def sync_counters(self, stream=None):
        _check(ffi.lib().pcn_ipt_sync_counters(self._h, stream))

    def comm_info(self):
        """RCCL version and library path, device ordinal and PCI bus id, and the all-gather steps'
        summed duration on the communicator stream (pcn_ipt_comm_get_info)."""
        return comm_info(self._h)

    def counter_block_words(self, chain):
        """u64 words of `chain`'s counter block [dp, db, p0, b0, ...] (pcn_ipt_counter_block_words)."""
        return _check(ffi.lib().pcn_ipt_counter_block_words(self._h, self._chain_id(chain)))

    def snapshot_counters(self, chain, block=None, stream=None):
        """This GPU's counter block of `chain` as an int64 tensor on the device (the send half of
        sync_counters; pcn_ipt_snapshot_counters)."""
        import torch
        cid = self._chain_id(chain)
        if block is None:
            block = torch.empty(self.counter_block_words(cid), dtype=torch.int64, device=f"cuda:{self.device}")
        s = stream if stream is not None else torch.cuda.current_stream(block.device).cuda_stream
        _check(ffi.lib().pcn_ipt_snapshot_counters(self._h, cid, block.data_ptr(), s))
        return block

    def sum_counter_blocks(self, chain, blocks, stream=None):
        """Sum gathered blocks (a [nranks, words] int64 device tensor, rank-major) into the
        scope=1 counters of `chain` (the receive half of sync_counters; pcn_ipt_sum_counter_blocks)."""
        import torch
        cid = self._chain_id(chain)
        blocks = blocks.contiguous()
        s = stream if stream is not None else torch.cuda.current_stream(blocks.device).cuda_stream
        _check(ffi.lib().pcn_ipt_sum_counter_blocks(self._h, cid, blocks.data_ptr(), blocks.shape[0],
                                                     blocks.shape[1], s))

    @staticmethod
    def _chain_id(chain):
        return _CHAIN_NAMES[chain.upper()] if isinstance(chain, str) else int(chain)

    # ---- flow-affinity split (stateful conntrack on N GPUs) ----
    @staticmethod
    def _frames_batch(frames, n, offsets, lens, stride, fixed_len, in_port, const_in_port, hook):
        def p(t):
            return None if t is None else t.data_ptr()
        if n is None:
            n = offsets.numel() if offsets is not None else frames.numel() // stride
        return n, ffi.Batch(frames.data_ptr(), frames.numel(), p(offsets), p(lens), stride, fixed_len, p(in_port),
                            const_in_port, INGRESS, hook, 0, None, n, None, None)

    def flow_owner(self, frames, nranks, n=None, offsets=None, lens=None, stride=64, fixed_len=64, hook=XDP,
                   stream=None):
        """Owner rank of every frame (pcn_ipt_flow_owner): a uint8 tensor on the frames' device."""
        import torch
        n, b = self._frames_batch(frames, n, offsets, lens, stride, fixed_len, None, 1, hook)
        owner = torch.empty(n, dtype=torch.uint8, device=frames.device)
        s = stream if stream is not None else torch.cuda.current_stream(frames.device).cuda_stream
        _check(ffi.lib().pcn_ipt_flow_owner(self._h, C.byref(b), nranks, owner.data_ptr(), s))
        return owner

    def flow_split(self, frames, nranks, rank, n=None, offsets=None, lens=None, stride=64, fixed_len=64,
                   in_port=None, const_in_port=1, hook=XDP, stream=None):
        """This rank's frames in batch order (pcn_ipt_flow_split): returns (index, offsets, lens,
        in_port) tensors of the owned count, ready for classify(frames, offsets=, lens=, in_port=)."""
        import torch
        n, b = self._frames_batch(frames, n, offsets, lens, stride, fixed_len, in_port, const_in_port, hook)
        dev = frames.device
        index = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        offs = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        ls = torch.empty(max(n, 1), dtype=torch.int16, device=dev)
        ports = torch.empty(max(n, 1), dtype=torch.int16, device=dev)
        m = C.c_uint64(0)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        _check(ffi.lib().pcn_ipt_flow_split(self._h, C.byref(b), nranks, rank, index.data_ptr(), offs.data_ptr(),
                                            ls.data_ptr(), ports.data_ptr(), C.byref(m), s))
        k = m.value
        return index[:k], offs[:k], ls[:k], ports[:k]


class IngestRing:
    """Pinned host slots feeding the GPU classifier (include/pcn_ipt.h, ring).

    acquire() returns (slot, frames, offsets, lens, in_port) as numpy views of
    the slot's pinned memory; submit(slot, n, ...) copies it in and classifies
    it; complete() returns the oldest slot's (slot, verdicts[, rule_ids]) views,
    valid until release(slot)."""

    def __init__(self, ipt, slots, slot_frames, slot_bytes, streams, rule_ids, zero_copy=False, host_pack=False,
                 pack_threads=0):
        import numpy as np
        self._np = np
        self._ipt = ipt
        self.slot_frames = slot_frames
        self.slot_bytes = slot_bytes
        flags = (1 if rule_ids else 0) | (2 if zero_copy else 0) | (4 if host_pack else 0)
        cfg = ffi.RingConfig(slots, slot_frames, slot_bytes, streams, flags, pack_threads)
        h = C.c_void_p()
        _check(ffi.lib().pcn_ipt_ring_create(ipt._h, C.byref(cfg), C.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            ffi.lib().pcn_ipt_ring_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def acquire(self):
        np = self._np
        s = ffi.RingSlot()
        _check(ffi.lib().pcn_ipt_ring_acquire(self._h, C.byref(s)))
        f = self.slot_frames
        return (s.slot, np.ctypeslib.as_array(s.frames, (self.slot_bytes,)),
                np.ctypeslib.as_array(s.offsets, (f,)), np.ctypeslib.as_array(s.lens, (f,)),
                np.ctypeslib.as_array(s.in_port, (f,)))

    def submit(self, slot, n, *, frames_bytes=0, stride=64, fixed_len=64, offsets=False, lens=False,
               in_port=False, const_in_port=1, direction=INGRESS, hook=XDP, hdr_bytes=0, hdr_skip=0):
        """hdr_bytes: copy only each frame's first hdr_bytes over PCIe (pcn_ipt_ring_batch.hdr_bytes);
        hdr_skip: of those, leave the first hdr_skip (0 or 12: the Ethernet addresses) on the host."""
        b = ffi.RingBatch(n, frames_bytes, stride, fixed_len, int(offsets), int(lens), int(in_port), hdr_skip,
                          const_in_port, direction, hook, hdr_bytes)
        _check(ffi.lib().pcn_ipt_ring_submit(self._h, slot, C.byref(b)))

    def complete(self, wait=True):
        """(slot, verdicts, rule_ids or None), or None when nothing is ready (wait=False)."""
        np = self._np
        slot, n = C.c_uint32(), C.c_uint64()
        v, r = C.POINTER(C.c_uint8)(), C.POINTER(C.c_int32)()
        rc = ffi.lib().pcn_ipt_ring_complete(self._h, int(wait), C.byref(slot), C.byref(n), C.byref(v), C.byref(r))
        if rc == -11 and not wait:     # -EAGAIN
            return None
        _check(rc)
        k = int(n.value)
        verdicts = np.ctypeslib.as_array(v, (k,)) if k else np.zeros(0, np.uint8)
        rids = np.ctypeslib.as_array(r, (k,)) if (k and bool(r)) else None
        return slot.value, verdicts, rids

    def release(self, slot):
        _check(ffi.lib().pcn_ipt_ring_release(self._h, slot))

    def stats(self, reset=False):
        """pcn_ipt_ring_get_stats: what the submits moved over PCIe and what their host side
        (pack, submit) cost since creation or the last reset."""
        st = ffi.RingStats()
        _check(ffi.lib().pcn_ipt_ring_get_stats(self._h, C.byref(st), int(reset)))
        return {k: getattr(st, k) for k, _ in ffi.RingStats._fields_}
