"""Headline benchmark: device-resident pcn-iptables classification on MI355X.

Workload (BASELINE.json configs[2], the metric's config): a 1,000-rule FORWARD
chain (synth.config_rules(3), default DROP) over 2^24 synthetic 64-byte IPv4
frames per GPU, 50/50 TCP/UDP, half built to hit a rule and half uniform random.
One step = one classify pass over the resident batch (verdicts + per-rule and
default counters); with N > 1 GPUs each rank owns its own 2^24-frame shard
(weak scaling) and every step ends with the RCCL all-gather of the per-rule
counters over xGMI (pcn_ipt_sync_counters).  Frames are in HBM before the timed
region starts; the PCIe-inclusive rate is reported separately under "e2e".

Run: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no
WORLD_SIZE in the environment it launches its N ranks itself (torch.distributed.run,
before any GPU call); under an external launcher it is one of the ranks.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkt/s device-resident classify @64B, 1k-rule chain, 1 GPU; %HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_PKT = 64             # algorithmic bytes: the 64-byte frame slot
WORKLOADS = {
    2: "config2: 128-rule FORWARD chain, 64B IPv4/UDP frames resident in HBM",
    3: "config3: 1k-rule FORWARD chain, 64B IPv4 50/50 TCP/UDP frames resident in HBM",
    5: "config5: 10k-rule FORWARD chain, IMIX 64/576/1500B frames (30% 802.1Q, 30% IPv6) resident in HBM",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


DATA = {
    2: "synthetic (seeded synth.config_rules(2) + synth.make_headers, UDP only; no captured traffic)",
    3: "synthetic (seeded synth.config_rules(3) + synth.make_headers, 50/50 TCP/UDP; no captured traffic)",
    5: "synthetic (seeded synth.config_rules(5) + synth.imix_frames; no captured traffic)",
}
# the sources that decide what the classify kernel reads per launch: a PMC
# traffic figure (profiles/pmc_traffic.json) is reported only for the build it
# was measured on
KERNEL_SOURCES = ("polycube_amd/csrc/classify.hip", "polycube_amd/csrc/devchain.h", "polycube_amd/csrc/image.cpp")


def kernel_src_hash():
    """sha-256 (16 hex digits) of classify.hip + devchain.h + image.cpp as the loaded
    libpcn_ipt.so carries them (pcn_ipt_embedded_source): the build that runs, not the
    files on disk (a stale library reports its own hash, see disk_src_hash)."""
    from polycube_amd.iptables import embedded_kernel_hash
    return embedded_kernel_hash()


def disk_src_hash():
    """The same hash over the files on disk (differs from kernel_src_hash when the
    library is stale)."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def rccl_libraries():
    """Every librccl the process has mapped (torch ships its own; libpcn_ipt.so links
    /opt/rocm/lib's): which RCCL serves a call depends on symbol resolution order."""
    seen = []
    try:
        with open("/proc/self/maps") as fh:
            for ln in fh:
                path = ln.split()[-1] if len(ln.split()) >= 6 else ""
                if "librccl" in path and path not in seen:
                    seen.append(path)
    except OSError:
        pass
    return seen


def torch_rccl():
    import torch
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception as e:   # noqa: BLE001 (a report field, never fatal)
        return f"unavailable: {e}"


def traffic_key(cfg, hook):
    return f"config{cfg}" + ("_tc" if hook else "")


def load_traffic(cfg, hook, n, key=None):
    """(HBM bytes per launch, note) from profiles/pmc_traffic.json when it was measured on this
    build's kernel sources and this batch size; (None, why) otherwise.  key: another entry
    than the config's own (the frame-size sweep's config3_stride<S>)."""
    key = key or traffic_key(cfg, hook)
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(tf):
        return None, "no profiles/pmc_traffic.json"
    with open(tf) as fh:
        pm = json.load(fh).get("configs", {}).get(key)
    if not pm:
        return None, f"no PMC entry for {key}"
    if pm.get("src_hash") != kernel_src_hash():
        return None, f"PMC entry measured on kernel sources {pm.get('src_hash')}, this build is {kernel_src_hash()}"
    if pm.get("frames") != n:
        return None, f"PMC entry measured at {pm.get('frames')} frames, this run has {n}"
    return pm["hbm_bytes_per_launch"], (f"rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE on kernel sources {pm['src_hash']} "
                                        f"({pm.get('profile', '')})")


def gen_frames(n, rs, seed, chunk=1 << 22, protos=(6, 17), hit_frac=0.5):
    from polycube_amd import synth
    out = np.empty((n, 64), np.uint8)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        cols = synth.make_headers(rs, m, seed + s // chunk, protos=protos, hit_frac=hit_frac)
        out[s:s + m] = synth.build_frames(*cols, frame_len=64)
    return out.reshape(-1)


def cpu_baseline(rules, frames, n, threads, min_seconds=8.0, offsets=None, lens=None, hook=0, big=None):
    """The oracle (scalar C restatement of the reference eBPF algorithm) on the host cores:
    passes over the same batch until min_seconds have gone by.  Returns (Mpkt/s, frames, seconds)."""
    from oracle.ffi import Oracle
    big = big or {}
    o = Oracle(big.get("max_counted_rules", 0), big.get("max_action_rules", 0))
    o.set_chain(1, rules, "DROP")
    done, t0 = 0, time.perf_counter()
    while True:
        if offsets is None:
            o.classify(frames, n=n, nthreads=threads, hook=hook)
        else:
            o.classify(frames, n=n, offsets=offsets[:n], lens=lens[:n], nthreads=threads, hook=hook)
        done += n
        el = time.perf_counter() - t0
        if el >= min_seconds:
            break
    return done / el / 1e6, done, el


def cgroup_cpus():
    """CPUs the cgroup's CFS quota grants (cgroup v2 cpu.max / v1 cfs_quota_us), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            per = int(fh.read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def host_cores():
    """(threads the baseline runs on, nproc): the CPUs this process may run on --
    its affinity set, capped by the cgroup's CPU quota (a GPU box shows the whole
    machine in nproc but grants a share of it) -- and the machine's count."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = cgroup_cpus()
    return (min(usable, quota) if quota else usable), os.cpu_count() or usable


def cpu_rates(rules, frames, n, label, offsets=None, lens=None, hook=0, big=None, s1=3.0, sall=6.0,
              with_nproc=False):
    """cpu_baseline object: every core this process is granted, and one core, on the same
    batch; with_nproc also times nproc threads (more than the grant: oversubscribed)."""
    cores, nproc = host_cores()
    kw = dict(offsets=offsets, lens=lens, hook=hook, big=big)
    one = min(n, 1 << 20)
    v1, done1, el1 = cpu_baseline(rules, frames, one, 1, min_seconds=s1, **kw)
    vT, doneT, elT = cpu_baseline(rules, frames, n, cores, min_seconds=sall, **kw)
    out = {"value": round(vT, 2), "unit": "Mpkt/s", "cores": cores, "nproc": nproc, "kind": "port",
           "sample": f"{label}: {doneT} frames ({doneT // n} passes over the same {n}-frame batch) in {elT:.1f}s "
                     f"on {cores} threads (the CPUs granted to this process: affinity set capped by the cgroup "
                     f"quota {cgroup_cpus()}; nproc {nproc})",
           "single_core": {"value": round(v1, 2), "cores": 1,
                           "sample": f"{done1} frames (passes over the batch's first {one}) in {el1:.1f}s"}}
    if with_nproc and nproc != cores:
        vN, doneN, elN = cpu_baseline(rules, frames, n, nproc, min_seconds=s1, **kw)
        out["nproc_threads"] = {"value": round(vN, 2), "cores": nproc,
                                "sample": f"{doneN} frames in {elN:.1f}s on {nproc} threads (beyond the grant)"}
    return out


def secondary_cpu_baselines(log):
    """configs 1, 2 and 5: the oracle at one core and all cores, each on its
    own config's rules and frames (config 5: 2^20 of its IMIX frames, XDP hook)."""
    from polycube_amd import synth
    out = {}
    for cfg, n in ((1, 1 << 22), (2, 1 << 20), (5, 1 << 20)):
        t = time.perf_counter()
        rs = synth.config_rules(cfg)
        rules = rs.rules()
        if cfg == 5:
            frames, offs, lens = synth.imix_frames(rs, n, synth.CONFIG_SEEDS[5])
            big = dict(max_counted_rules=10000, max_action_rules=10000)
        else:
            frames, offs, lens, big = synth.config_frames(cfg, n, rs).reshape(-1), None, None, None
        out[f"config{cfg}"] = dict(cpu_rates(rules, frames, n, f"config {cfg}, {len(rules)} rules", offs, lens,
                                             big=big, s1=2.0, sall=3.0), rules=len(rules), frames=n)
        log(f"[bench] cpu baseline config {cfg}: {out[f'config{cfg}']['value']} Mpkt/s "
            f"({time.perf_counter() - t:.1f}s)")
    return out


def parity_sample(o_rules, frames, v_dev, r_dev, offsets=None, lens=None, hook=0, big=None, k=1 << 16):
    from oracle.ffi import Oracle
    big = big or {}
    o = Oracle(big.get("max_counted_rules", 0), big.get("max_action_rules", 0))
    o.set_chain(1, o_rules, "DROP")
    if offsets is None:
        v, r = o.classify(frames[:k * 64], n=k, nthreads=4, hook=hook)
    else:
        v, r = o.classify(frames, n=k, offsets=offsets[:k], lens=lens[:k], nthreads=4, hook=hook)
    return bool(np.array_equal(v, v_dev[:k]) and np.array_equal(r, r_dev[:k]))


def e2e_rate(ipt, frames_host, n, chunk=1 << 21, slots=4, reps=3, stride=64, frame_len=64, hdr_bytes=0,
             zero_copy=False, host_pack=False, pack_threads=0, hdr_skip=0):
    """Host ingest ring (pcn_ipt_ring_*): pinned slots -> hipMemcpyAsync H2D ->
    classify -> D2H verdicts, `slots` slots in flight over as many streams.
    The frames are placed in the pinned slots once, as a NIC's RX DMA would
    write them (not timed); each timed pass submits n frames in chunk-frame
    slots and waits for every verdict to be back in host memory.  hdr_bytes:
    only each frame's first hdr_bytes cross PCIe (a strided hipMemcpy2DAsync, or with
    host_pack the windows packed on pack_threads host threads, then one contiguous copy;
    the pack runs inside each timed submit); hdr_skip 12: the Ethernet addresses stay on
    the host too (hdr_bytes - 12 bytes a frame cross PCIe)."""
    from polycube_amd import IptablesError
    ring = ipt.ring(slots=slots, slot_frames=chunk, slot_bytes=stride * chunk, zero_copy=zero_copy,
                    host_pack=host_pack, pack_threads=pack_threads)
    held = [ring.acquire() for _ in range(slots)]
    m = frames_host.size // stride
    for k, (slot, frames, _, _, _) in enumerate(held):
        lo = (k * chunk) % m
        take = min(chunk, m - lo)
        for r in range(0, chunk, take):
            q = min(take, chunk - r)
            frames[r * stride:(r + q) * stride] = frames_host[lo * stride:(lo + q) * stride]
        ring.release(slot)
    nsub = max(1, n // chunk)
    best, best_st, best_el = 0.0, None, 0.0
    for _ in range(reps):
        submitted = completed = 0
        ring.stats(reset=True)
        t0 = time.perf_counter()
        while completed < nsub:
            while submitted < nsub:
                try:
                    slot = ring.acquire()[0]
                except IptablesError as e:        # -EAGAIN: every slot in flight
                    if e.code != -11:
                        raise
                    break
                ring.submit(slot, chunk, stride=stride, fixed_len=frame_len, hdr_bytes=hdr_bytes, hdr_skip=hdr_skip)
                submitted += 1
            slot = ring.complete(wait=True)[0]
            ring.release(slot)
            completed += 1
        el = time.perf_counter() - t0
        rate = nsub * chunk / el / 1e6
        if rate > best:
            best, best_st, best_el = rate, ring.stats(), el
    ring.close()
    st = best_st
    sub = max(1, st["submits"])
    info = {"mpkt_s": round(best, 2),
            "h2d_gb_s": round(st["h2d_bytes"] / best_el / 1e9, 2),
            "d2h_gb_s": round(st["d2h_bytes"] / best_el / 1e9, 2),
            "submit_ms_per_chunk": round(st["submit_ns"] / sub / 1e6, 4),
            "submit_share_of_wall": round(st["submit_ns"] / 1e9 / best_el, 3)}
    if zero_copy:
        info["pcie_read_gb_s"] = round(st["zc_bytes"] / best_el / 1e9, 2)
    if host_pack:
        info["pack_ms_per_chunk"] = round(st["pack_ns"] / sub / 1e6, 4)
        info["pack_share_of_wall"] = round(st["pack_ns"] / 1e9 / best_el, 3)
    return info


def e2e_legs(ipt, frames_host, n, rs, log):
    """The e2e rate with whole frames and with header-only transfers, for the
    headline's 64-byte frames and for 1500-byte frames (one slot's worth,
    1536-byte stride) of the same traffic."""
    from polycube_amd import synth
    out = {}
    threads = host_cores()[0]
    legs = (("whole_frames", 0, False, False, 0), ("header_only_48", 48, False, False, 0),
            ("zero_copy", 0, True, False, 0), ("header_pack_48", 48, False, True, 0),
            ("header_pack_36", 48, False, True, 12))
    detail = {}
    for name, hb, zc, hp, sk in legs:
        detail[name] = e2e_rate(ipt, frames_host, n, hdr_bytes=hb, zero_copy=zc, host_pack=hp,
                                pack_threads=min(threads, 16), hdr_skip=sk)
        out[name] = detail[name]["mpkt_s"]
        log(f"[bench] e2e 64B {name}: {detail[name]}")
    out["pack_threads"] = min(threads, 16)
    out["legs"] = detail
    out["pcie_h2d_ceiling_gb_s"] = pcie_h2d_ceiling()
    m = 1 << 16
    cols = synth.make_headers(rs, m, synth.CONFIG_SEEDS[3] + 1)
    big = synth.build_frames(*cols, frame_len=1536).reshape(-1)
    out["frames_1500"] = {}
    for name, hb, zc in (("whole_frames", 0, False), ("header_only_64", 64, False), ("zero_copy", 0, True)):
        d = e2e_rate(ipt, big, 1 << 20, chunk=m, stride=1536, frame_len=1500, hdr_bytes=hb, zero_copy=zc)
        out["frames_1500"][name] = d["mpkt_s"]
        out["frames_1500"].setdefault("legs", {})[name] = d
        log(f"[bench] e2e 1500B {name}: {d}")
    out["kept"] = max((k for k, _, _, _, _ in legs), key=lambda k: out[k])
    # what bounds the kept leg: its PCIe bytes against the copy ceiling, its host submit
    # (pack) time against the wall time
    kd = detail[out["kept"]]
    pcie = kd.get("h2d_gb_s", 0) + kd.get("pcie_read_gb_s", 0)
    host = kd.get("pack_share_of_wall", kd.get("submit_share_of_wall", 0))
    out["bound"] = (f"PCIe: {pcie} GB/s in against a {out['pcie_h2d_ceiling_gb_s']} GB/s pinned-copy ceiling"
                    if pcie >= 0.8 * out["pcie_h2d_ceiling_gb_s"] else
                    f"host: the submits' {'pack' if 'pack_share_of_wall' in kd else 'host'} time is "
                    f"{host:.0%} of the wall time" if host >= 0.8 else
                    f"neither saturated: PCIe {pcie} GB/s of {out['pcie_h2d_ceiling_gb_s']}, host {host:.0%}")
    out["value"] = out[out["kept"]]
    out["unit"] = "Mpkt/s"
    out["what"] = ("host ingest ring (pcn_ipt_ring): pinned slots -> H2D -> classify -> D2H verdicts, 4 slots x 2^21 "
                   "64-byte frames in flight over 4 streams; whole frames vs. only each frame's first 48 bytes over "
                   "PCIe (pcn_ipt_ring_batch.hdr_bytes, a strided copy) vs. zero copy (PCN_IPT_RING_ZERO_COPY: the "
                   "classify kernel reads the pinned slots over PCIe) vs. header pack (PCN_IPT_RING_HOST_PACK: each "
                   "submit packs the 48-byte windows into contiguous pinned rows on pack_threads host threads, then "
                   "one contiguous 48-byte-stride copy; the pack is inside the timed loop); header_pack_36: the same "
                   "without the 12 Ethernet-address bytes no stage of the path reads (pcn_ipt_ring_batch.hdr_skip: "
                   "36 bytes a frame cross PCIe); frames_1500: 4 slots x "
                   "2^16 1500-byte frames at a 1536-byte stride, the first three")
    return out


def pcie_h2d_ceiling(mb=256, streams=4, reps=5):
    """Pinned host -> device copy rate (GB/s) with `streams` copies of mb MB in flight:
    the PCIe ceiling the e2e legs are set against (the DMA engines of one GPU)."""
    import torch
    dev = torch.device("cuda", torch.cuda.current_device())
    src = [torch.empty(mb << 20, dtype=torch.uint8).pin_memory() for _ in range(streams)]
    dst = [torch.empty(mb << 20, dtype=torch.uint8, device=dev) for _ in range(streams)]
    ss = [torch.cuda.Stream(dev) for _ in range(streams)]
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s, a, b in zip(ss, src, dst):
            with torch.cuda.stream(s):
                b.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, streams * (mb << 20) / (time.perf_counter() - t0) / 1e9)
    return round(best, 2)


def gather_ceiling(frames, offsets, lens, n, s_ptr, kern_ms):
    """Config 5: the read ceiling of its own access pattern on the same device
    buffers -- per frame the offset, the length and the 52-byte header window,
    one verdict byte out, no classification (tools/gather_ceiling.hip, four
    lanes per frame, 16-byte loads).  None when the probe library is absent."""
    import ctypes
    import torch
    path = os.path.join(ROOT, "tools", "libgather_ceiling.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.gather_ceiling_ms.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)]
    out = torch.empty(n, dtype=torch.uint8, device=frames.device)
    ms = ctypes.c_float(0)
    rc = lib.gather_ceiling_ms(frames.data_ptr(), offsets.data_ptr(), lens.data_ptr(), out.data_ptr(), n, 200, 50,
                               ctypes.c_void_p(s_ptr), ctypes.byref(ms))
    if rc != 0:
        return {"error": rc}
    return {"ms": round(ms.value, 4), "frac_of_ceiling": round(ms.value / kern_ms, 4),
            "what": "tools/gather_ceiling.hip on the same buffers: offset + length + 52-byte header window per "
                    "frame (4 lanes x 16-byte loads), one byte out, no classification"}


def ct_rate(ipt, rs, n, dev, steps=5, warmup=2, flows=1 << 16, seed=0xC7):
    """Stateful conntrack (pcn_ipt_ct_*) on the same chain: n 64-byte frames of
    `flows` interleaved connections (TCP handshakes/closes, UDP, ICMP), the
    table carried across steps.  Returns (Mpkt/s, ms per step, live entries)."""
    import torch

    from polycube_amd import synth
    f, _ = synth.flow_traffic(n, flows, seed, stride=64, rs=rs)
    frames = torch.from_numpy(f).to(dev)
    verdicts = torch.empty(n, dtype=torch.uint8, device=dev)
    ipt.ct_enable(20)
    ipt.ct_set_time(1_700_000_000 * 10**9)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(warmup):
        ipt.classify(frames, n=n, verdicts=verdicts, stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ipt.classify(frames, n=n, verdicts=verdicts, stream=stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    live = len(ipt.ct_dump())
    # flow-affinity split (pcn_ipt_flow_split) of the same batch over 8 tables,
    # and the owned share's stateful classify on a fresh table
    ipt.ct_clear()
    split = ipt.flow_split(frames, 8, 0, n=n, stride=64)
    t0 = time.perf_counter()
    for _ in range(steps):
        split = ipt.flow_split(frames, 8, 0, n=n, stride=64)
    split_ms = (time.perf_counter() - t0) / steps * 1e3
    idx, offs, lens, ports = split
    m = idx.numel()
    ipt.classify(frames, n=m, verdicts=verdicts, offsets=offs, lens=lens, in_port=ports, stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ipt.classify(frames, n=m, verdicts=verdicts, offsets=offs, lens=lens, in_port=ports, stream=stream)
    torch.cuda.synchronize()
    share_ms = (time.perf_counter() - t0) / steps * 1e3
    ipt.ct_disable()
    return n * steps / el / 1e6, el / steps * 1e3, live, {"split_ms": round(split_ms, 3), "share_frames": m,
                                                           "share_ms": round(share_ms, 3)}


def ct_single_flow(ipt, rs, n, dev, steps=3):
    """The stateful leg's worst case for the walk: the whole batch one TCP connection
    (handshake, data, close; no noise, no ICMP), so every segment of its one run is
    walked speculatively and chained by ct_seg_fix.  ms per batch."""
    import torch

    from polycube_amd import synth
    f, _ = synth.flow_traffic(n, 1, 0xC7, stride=64, rs=rs, p_noise=0.0, p_icmp=0.0, p_err=0.0)
    frames = torch.from_numpy(f).to(dev)
    verdicts = torch.empty(n, dtype=torch.uint8, device=dev)
    ipt.ct_enable(20)
    ipt.ct_set_time(1_700_000_000 * 10**9)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ipt.classify(frames, n=n, verdicts=verdicts, stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ipt.classify(frames, n=n, verdicts=verdicts, stream=stream)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    ipt.ct_disable()
    return ms


def fw_rate(rules, frames, n, dev, s_ptr, jit, steps=20, horus=False, settle=0.5):
    """The headline rules in a pcn-firewall INGRESS chain (conntrack OFF), same
    resident frames: time per pcn_ipt_classify call (one HIP event pair around
    `steps` calls, after `settle` seconds of untimed calls) and Mpkt/s.
    horus=False turns pcn-firewall's Horus off (it is on from the start in the
    reference, Firewall.h:337) so the rule pipeline itself is measured."""
    import torch
    from polycube_amd import Firewall
    fw = Firewall(device=dev.index, jit=jit)
    fw.horus = horus
    fw.conntrack = "OFF"
    fw.interactive = False
    ing = fw.chain("INGRESS")
    for r in rules:
        ing.append(**dict(r, action=r.get("action", "DROP")))
    ing.default = "DROP"
    ing.apply_rules()
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    # the chain program was just compiled with the GPU idle: settle the clocks
    # first, as the headline does, then one event pair around the timed calls
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < settle:
        for _ in range(32):
            fw.classify(frames, n=n, verdicts=v, rule_ids=False, stream=s_ptr)
        torch.cuda.synchronize()
    for _ in range(3):
        fw.classify(frames, n=n, verdicts=v, rule_ids=False, stream=s_ptr)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(steps):
        fw.classify(frames, n=n, verdicts=v, rule_ids=False, stream=s_ptr)
    b.record(stream)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / steps
    info = fw.horus_info("INGRESS")
    fw.close()
    return n / (ms * 1e-3) / 1e6, ms, info


def timed_calls(fn, steps, stream, settle=0.3):
    """Kernel ms per call: `settle` seconds of untimed calls, then one HIP event pair on the
    launch stream around `steps` calls (as the headline is timed)."""
    import torch
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < settle:
        for _ in range(16):
            fn()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(steps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def hit_rate_sweep(ipt, chain, rs, n, dev, stream, base_ms, seed, steps=20, hits=(0.0, 1.0)):
    """The headline chain over batches built with other rule-hit shares (synth.make_headers
    hit_frac: that share of the frames is built from a random rule's fields, the rest uniform),
    the same kernel timing as the headline.  Reports kernel ms, Gpkt/s, the roofline fraction
    and the share of frames that matched a rule (from the counters)."""
    import torch
    alt = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    s_ptr = stream.cuda_stream
    out = {"0.5": {"kernel_ms": round(base_ms, 4), "gpkt_s": round(n / base_ms / 1e6, 2),
                   "frac": round(BYTES_PER_PKT * n / (base_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "what": "the headline batch (timed above)"}}
    for h in hits:
        alt.copy_(torch.from_numpy(gen_frames(n, rs, seed, hit_frac=h)))
        ms = timed_calls(lambda: ipt.classify(alt, n=n, verdicts=v, rule_ids=False, stream=s_ptr), steps, stream)
        chain.read_counters(len(rs.rules()), flush=True)
        ipt.classify(alt, n=n, verdicts=v, rule_ids=False, stream=s_ptr)
        torch.cuda.synchronize()
        pk = chain.read_counters(len(rs.rules()), flush=True)[0]   # (the default counters are never flushed)
        out[str(h)] = {"kernel_ms": round(ms, 4), "gpkt_s": round(n / ms / 1e6, 2),
                       "frac": round(BYTES_PER_PKT * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                       "matched_rule_share": round(sum(pk) / n, 4)}
    del alt
    return out


FRAME_SIZES = (64, 128, 256, 576, 1024, 1500)


def frame_size_sweep(ipt, rules, frames, n, dev, stream, log, steps=20, sizes=FRAME_SIZES):
    """north_star's "Mpkt/s on synthetic 64 B-1500 B frames": the headline chain and
    traffic as fixed-size frames of each size (stride = size, packet_len = size;
    synth.spread_frames lays the resident 64-byte frames out on the device, IP / UDP
    lengths rewritten), 2^log2n frames in HBM, timed as the headline (settle, one event
    pair around `steps` launches).  The roofline is the 64-byte header sector per frame
    (the Parser reads bytes 0..47, Iptables_Parser_dp.c:126-143): `frac` = 64 B x n /
    time / peak.  `lines_128b` is the count of 128-byte lines a frame's 48-byte window
    touches (1500 B: 48 of every 128 windows cross into a second line): every L2 fill is a
    128-byte request, so a frame at a stride of 128 B or more moves at least one whole line
    (tools/gather_calib.hip: TCC_EA0_RDREQ = the lines touched), and
    `line_frac` = lines x 128 B x n / time / peak is the roofline of that access pattern;
    `traffic` the PMC HBM bytes per frame where profiles/pmc_traffic.json holds an entry
    for this build.  Each size's first 2^16 frames are checked against
    the oracle (verdicts and rule ids)."""
    import torch

    from polycube_amd import synth
    big = torch.empty(n * max(sizes), dtype=torch.uint8, device=dev)
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    rid = torch.empty(n, dtype=torch.int32, device=dev)
    s_ptr = stream.cuda_stream
    out = {}
    from oracle.ffi import Oracle
    o = Oracle()
    o.set_chain(1, rules, "DROP")
    k = 1 << 16
    for size in sizes:
        buf = synth.spread_frames(frames, n, size, out=big)
        ms = timed_calls(lambda: ipt.classify(buf, n=n, verdicts=v, rule_ids=False, stride=size, fixed_len=size,
                                              stream=s_ptr), steps, stream)
        ipt.classify(buf, n=n, verdicts=v, rule_ids=rid, stride=size, fixed_len=size, stream=s_ptr)
        torch.cuda.synchronize()
        w = min(size, 128)
        host = buf.view(n, size)[:k, :w].cpu().numpy().reshape(-1)
        vo, ro = o.classify(host, n=k, stride=w, fixed_len=size, nthreads=4)
        ok = bool(np.array_equal(vo, v[:k].cpu().numpy()) and np.array_equal(ro, rid[:k].cpu().numpy()))
        offs = np.arange(n, dtype=np.int64) * size
        lines = float(np.mean(1 + ((offs + 47) // 128 - offs // 128)))
        traffic, note = load_traffic(3, 0, n, key=None if size == 64 else f"config3_stride{size}")
        out[str(size)] = {"kernel_ms": round(ms, 4), "mpkt_s": round(n / ms / 1e3, 1),
                          "frac": round(BYTES_PER_PKT * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "line_frac": round(lines * 128 * n / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "frame_gb_s": round(size * n / (ms * 1e-3) / 1e9, 1),
                          "lines_128b_per_frame": round(lines, 4),
                          "line_gb_s": round(lines * 128 * n / (ms * 1e-3) / 1e9, 1),
                          "path": "fixed-stride" if size % 4 == 0 else "generic gather (any byte offset)",
                          "traffic_bytes_per_frame": None if traffic is None else round(traffic / n, 2),
                          "traffic_from": note, "parity_sample_vs_oracle": ok}
        log(f"[bench] frame size {size}: {out[str(size)]}")
    del big
    torch.cuda.empty_cache()
    out["frames"] = n
    out["what"] = frame_size_sweep.__doc__.split("\n", 1)[1].strip()
    return out


def rule_update_latency(dev, log):
    """Rule-update latency, the analogue of the reference's per-update timer
    (Chain::updateChain, Chain.cpp:436,920-928: rule compile, bcc compile + load of the
    chain's eBPF programs, map pushes).  Here, per config (1k and 10k rules):
      apply_ms       pcn_ipt_chain_apply_rules of the whole chain (rule compiler, table image,
                     upload to the inactive slot, flip), non-interactive mode
      compile_ms     pcn_ipt_chain_program_compile: the chain program (hiprtc) for the launch shape
      first_ms       the first classify launch after that (program load) until its verdicts are in
      append_ms      one more rule appended in interactive mode (Chain::append -> updateChain):
                     the whole chain recompiled and uploaded
      append_first_ms  the next launch (jit=0: the generic kernel runs while the new chain
                     program compiles in the background, as pcn_ipt_config.jit = 0 does)
      append_program_ms  until that background compile is ready"""
    import torch
    from polycube_amd import Iptables, synth
    out = {}
    for cfg in (3, 5):
        rs = synth.config_rules(cfg)
        rules = rs.rules()
        big = dict(max_rules=16384, max_counted_rules=10000, max_action_rules=10000) if cfg == 5 else {}
        m = 1 << 16
        kw = {}
        if cfg == 5:
            buf, off, ln = synth.imix_frames(rs, m, synth.CONFIG_SEEDS[5])
            frames = torch.from_numpy(buf).to(dev)
            kw = dict(offsets=torch.from_numpy(off.view(np.int32)).to(dev),
                      lens=torch.from_numpy(ln.view(np.int16)).to(dev))
        else:
            frames = torch.from_numpy(gen_frames(m, rs, synth.CONFIG_SEEDS[3])).to(dev)
        v = torch.empty(m, dtype=torch.uint8, device=dev)
        ipt = Iptables(device=dev.index, jit=1, **big)
        ipt.interactive = False
        ch = ipt.chain("FORWARD")
        for r in rules:
            ch.append(**r)
        ch.default = "DROP"
        torch.cuda.synchronize()
        t = time.perf_counter()
        ch.apply_rules()
        apply_ms = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        ch.compile_program()
        compile_ms = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        ipt.classify(frames, n=m, verdicts=v, rule_ids=False, **kw)
        ipt.synchronize()
        first_ms = (time.perf_counter() - t) * 1e3
        ready0 = ipt.jit_info()["programs_ready"]
        ipt.close()
        # interactive one-rule update on a jit=0 context (background compiles)
        ipt = Iptables(device=dev.index, jit=0, **big)
        ipt.interactive = False
        ch = ipt.chain("FORWARD")
        for r in rules:
            ch.append(**r)
        ch.default = "DROP"
        ch.apply_rules()
        ch.compile_program()
        ipt.classify(frames, n=m, verdicts=v, rule_ids=False, **kw)
        ipt.synchronize()
        ipt.interactive = True
        ready = ipt.jit_info()["programs_ready"]
        t = time.perf_counter()
        ch.append(**dict(rules[len(rules) // 2], action="ACCEPT"))
        append_ms = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        ipt.classify(frames, n=m, verdicts=v, rule_ids=False, **kw)
        ipt.synchronize()
        append_first_ms = (time.perf_counter() - t) * 1e3
        prog_ms = None
        while time.perf_counter() - t < 30:
            if ipt.jit_info()["programs_ready"] > ready:
                prog_ms = (time.perf_counter() - t) * 1e3
                break
            time.sleep(0.005)
        ipt.close()
        out[f"config{cfg}"] = {"rules": len(rules), "apply_ms": round(apply_ms, 2), "compile_ms": round(compile_ms, 1),
                               "first_ms": round(first_ms, 2), "programs_ready": ready0,
                               "append_ms": round(append_ms, 2), "append_first_ms": round(append_first_ms, 2),
                               "append_program_ms": None if prog_ms is None else round(prog_ms, 1)}
        log(f"[bench] rule update config {cfg}: {out[f'config{cfg}']}")
    out["what"] = rule_update_latency.__doc__.split("\n", 1)[1].strip()
    return out


def spawn_ranks(n):
    """Run this script as N ranks (torch.distributed.run, one process per GPU,
    rendezvous on 127.0.0.1); rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n}: launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--log2n", type=int, default=24, help="frames per GPU = 2^log2n")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe end-to-end leg")
    ap.add_argument("--config", type=int, default=3, choices=(2, 3, 5),
                    help="BASELINE.json config: 3 = the headline (default); 2 and 5 are secondary measurements")
    ap.add_argument("--imix-align", type=int, default=1, choices=(1, 64),
                    help="config 5 layout: 1 = frames packed back to back (default), 64 = each at a 64-byte "
                         "boundary, as NIC RX buffers place them")
    ap.add_argument("--hook", default="xdp", choices=("xdp", "tc"),
                    help="attach-point semantics (tc: outer VLAN tags stripped before classification)")
    ap.add_argument("--no-ct", action="store_true", help="skip the stateful-conntrack leg")
    ap.add_argument("--no-fw", action="store_true", help="skip the pcn-firewall leg")
    ap.add_argument("--no-hits", action="store_true", help="skip the hit-rate 0 / 1 sweep (config 3)")
    ap.add_argument("--no-update", action="store_true", help="skip the rule-update latency leg")
    ap.add_argument("--no-sizes", action="store_true", help="skip the 64-1500 B frame-size sweep (config 3)")
    ap.add_argument("--jit", type=int, default=1,
                    help="chain programs: 1 compiled before the first launch (default), 0 background, -1 off")
    ap.add_argument("--settle", type=float, default=1.0,
                    help="seconds of untimed steps before the W warmup steps, so the GPU clocks reach their "
                         "steady state (a datapath runs continuously); 0 disables")
    ap.add_argument("--step-events", action="store_true",
                    help="bracket every timed step with its own HIP event pair (adds the events' cost to the "
                         "timed loop) instead of one pair around the whole timed region")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start N ranks under torch.distributed.run as
        # children, before this process touches the GPU, and exit with their code
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    from polycube_amd import Iptables, synth
    from polycube_amd import dist as pdist
    from polycube_amd.iptables import build_sha256

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "PCN_BENCH_DEVICE" in os.environ:   # test hook: several ranks on one GPU (RCCL refuses that)
        local = int(os.environ["PCN_BENCH_DEVICE"])
    if args.gpus != world:
        log(f"[rank {rank}] --gpus {args.gpus} but WORLD_SIZE={world}: measuring {world} rank(s)")
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    cfg = args.config
    if cfg == 5 and args.log2n == 24:
        args.log2n = 22                      # config 5 is 2^22 IMIX frames
    if cfg == 2 and args.log2n == 24:
        args.log2n = 20                      # BASELINE.json configs[1]: 1M frames
    n = 1 << args.log2n
    hook = 1 if args.hook == "tc" else 0
    rs = synth.config_rules(cfg)
    rules = rs.rules()
    big = dict(max_rules=16384, max_counted_rules=10000, max_action_rules=10000) if cfg == 5 else {}
    ipt = Iptables(device=local, jit=args.jit, **big)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in rules:
        fw.append(**r)
    fw.default = "DROP"
    fw.apply_rules()
    collective = "RCCL all-gather of the per-rule counter blocks (pcn_ipt_sync_counters)"
    use_rccl = world > 1
    if world > 1:
        uid = [Iptables.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        err = ""
        try:
            ipt.comm_init(world, rank, uid[0])
        except Exception as e:           # keep the scaling line, say how it was made
            err = str(e)
        ok = torch.tensor([0 if err else 1])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        use_rccl = bool(ok.item())
        if not use_rccl:
            collective = (f"gloo all-gather of the counter blocks through the host (pcn_ipt_snapshot_counters -> "
                          f"gloo -> pcn_ipt_sum_counter_blocks; RCCL init failed: {err[:160]})")
            log(f"[rank {rank}] {collective}")

    t = time.perf_counter()
    offsets_host = lens_host = None
    if cfg == 5:
        frames_host, offsets_host, lens_host = synth.imix_frames(rs, n, synth.CONFIG_SEEDS[5] + 7919 * rank,
                                                                 align=args.imix_align)
    else:
        frames_host = gen_frames(n, rs, synth.CONFIG_SEEDS[cfg] + 7919 * rank,
                                 protos=(synth.UDP,) if cfg == 2 else (synth.TCP, synth.UDP))
    log(f"[rank {rank}] generated {n} frames in {time.perf_counter() - t:.1f}s")
    frames = torch.from_numpy(frames_host).to(dev)
    offsets = None if offsets_host is None else torch.from_numpy(offsets_host.view(np.int32)).to(dev)
    lens = None if lens_host is None else torch.from_numpy(lens_host.view(np.int16)).to(dev)
    verdicts = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    s_ptr = stream.cuda_stream

    def classify(rid=False):
        ipt.classify(frames, n=n, verdicts=verdicts, rule_ids=rid, offsets=offsets, lens=lens, stream=s_ptr,
                     hook=hook)

    host_ex = [0.0]   # seconds spent in the gloo fallback's host exchange

    def exchange():
        if world == 1:
            return
        if use_rccl:
            ipt.sync_counters(s_ptr)
        else:   # fallback: the same per-step exchange, the blocks moved through the host by gloo
            t = time.perf_counter()
            blk = ipt.snapshot_counters("FORWARD", stream=s_ptr).cpu()
            parts = [torch.empty_like(blk) for _ in range(world)]
            dist.all_gather(parts, blk)
            ipt.sum_counter_blocks("FORWARD", torch.stack(parts).to(dev), stream=s_ptr)
            host_ex[0] += time.perf_counter() - t

    def step():
        classify()
        exchange()

    # clock settle: untimed steps until the GPU has run the workload for `settle` seconds
    # (every rank runs the same number of steps: each step may hold a collective,
    # so the ranks agree after each chunk whether to go on)
    settle_steps, t_settle = 0, time.perf_counter()
    while True:
        go = time.perf_counter() - t_settle < args.settle
        if world > 1:
            flag = torch.tensor([int(go)])
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            go = bool(flag.item())
        if not go:
            break
        for _ in range(64):
            step()
        settle_steps += 64
        torch.cuda.synchronize()
    settle_s = time.perf_counter() - t_settle
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    nev = args.steps if args.step_events else 1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nev)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    cinfo0 = ipt.comm_info() if use_rccl else None    # folds the settle/warmup gathers' times in
    host_ex[0] = 0.0
    t0 = time.perf_counter()
    if args.step_events:
        for k in range(args.steps):
            ev[k][0].record(stream)
            classify()
            ev[k][1].record(stream)
            exchange()
    else:
        # one event pair on the launch stream around the K steps: the average
        # launch duration below includes the launch-to-launch boundaries, so it
        # is an upper bound of the kernel time (a lower bound of `achieved`)
        ev[0][0].record(stream)
        for k in range(args.steps):
            classify()
            exchange()
        ev[0][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = (float(np.mean([a.elapsed_time(b) for a, b in ev])) if args.step_events
               else ev[0][0].elapsed_time(ev[0][1]) / args.steps)
    multi = None
    if world > 1:
        # per rank: device ordinal and PCI bus id (each rank must hold its own GPU unless the
        # one-GPU test hook put them on one), the RCCL that serves the calls, the exchange time
        ci = ipt.comm_info()
        if use_rccl:
            g = ci["gathers_timed"] - cinfo0["gathers_timed"]
            ex_ms = (ci["gather_ms_total"] - cinfo0["gather_ms_total"]) / max(1, g)
        else:
            g, ex_ms = args.steps, host_ex[0] / args.steps * 1e3
        mine = {"rank": rank, "local_rank": local, "device": ci["device"], "pci_bus_id": ci["pci_bus_id"],
                "exchange_ms_per_step": round(ex_ms, 4), "steps_timed": g}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        shared = "PCN_BENCH_DEVICE" in os.environ
        distinct = len({r["pci_bus_id"] for r in ranks}) == world
        if not shared and not distinct:
            raise SystemExit(f"[rank {rank}] ranks share a GPU: {ranks}")
        multi = {"rccl_version": ci["rccl_version"], "rccl_path": ci["rccl_path"], "ranks": ranks,
                 "devices_distinct": distinct,
                 "devices_shared_by_test_hook": shared,
                 "exchange_ms_per_step_max": max(r["exchange_ms_per_step"] for r in ranks),
                 "exchange_what": ("RCCL all-gather + device rank sum on the communicator stream (an event pair per "
                                   "step there; it overlaps the next step's classify)" if use_rccl else
                                   "gloo fallback: host wall time of snapshot + gloo all_gather + device sum per "
                                   "step (on the classify path)")}
    if world > 1:
        tt = torch.tensor([elapsed])
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    sum_ok = None
    if world > 1:
        # the summed (scope 1) view must equal the sum of every rank's own counters
        k = min(len(rules), 8000)
        mine = torch.tensor(pdist.counter_block(*fw.read_counters(k, scope=0)), dtype=torch.int64)
        total = mine.clone()
        dist.all_reduce(total)
        got = torch.tensor(pdist.counter_block(*fw.read_counters(k, scope=1)), dtype=torch.int64)
        ok = torch.tensor([int(torch.equal(got, total))])
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        sum_ok = bool(ok.item())

    value = n * world * args.steps / elapsed / 1e6
    bytes_per_pkt = BYTES_PER_PKT + (6 if cfg == 5 else 0)   # + offset and length per frame (§8d)
    achieved = bytes_per_pkt * n / (kern_ms * 1e-3) / 1e9
    traffic, traffic_note = load_traffic(cfg, hook, n)

    jit_info = ipt.jit_info()
    kernel = (f"pcn_classify_jit (chain program, config-{cfg} layout baked in)"
              if jit_info["launches_jit"] > args.warmup else "classify_kernel (generic)")
    # every rank: one untimed pass with rule ids, its first 2^16 frames checked against the
    # oracle (each rank classifies its own shard), then the verdict of all ranks together
    rid = torch.empty(n, dtype=torch.int32, device=dev)
    fw.read_counters(len(rules), flush=True)
    classify(rid)
    torch.cuda.synchronize()
    ok = parity_sample(rules, frames_host, verdicts[: 1 << 16].cpu().numpy(), rid[: 1 << 16].cpu().numpy(),
                       offsets_host, lens_host, hook, big)
    parity_ranks = [ok]
    if world > 1:
        parity_ranks = [None] * world
        dist.all_gather_object(parity_ranks, bool(ok))
        ok = all(parity_ranks)
    program = fw.program_info()
    if rank == 0:
        line = {
            "metric": METRIC if world == 1 else METRIC.replace("1 GPU", f"{world} GPUs"), "value": round(value, 2), "unit": "Mpkt/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": DATA[cfg],
            "config": {"workload": WORKLOADS[cfg] + (", TC hook" if hook else ""),
                       "rules": len(rules), "frames_per_gpu": n,
                       "frame_bytes": "IMIX 64/576/1500 (7:4:1)" if cfg == 5 else 64,
                       "layout": ("packed back to back" if args.imix_align == 1 else "64-byte aligned")
                       if cfg == 5 else "64-byte stride",
                       "parallelism": (f"dp{world} (packet-index shards, "
                                       + ("RCCL counter all-gather)" if use_rccl else "host gloo counter all-reduce)")
                                       if world > 1 else "dp1 (one packet shard, no exchange)"),
                       "collective": collective if world > 1 else None},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_from": traffic_note, "kernel_src_hash": kernel_src_hash(),
                         "kernel_src_hash_from": "classify.hip + devchain.h + image.cpp text embedded in the loaded "
                                                 "libpcn_ipt.so (pcn_ipt_embedded_source)",
                         "disk_src_hash": disk_src_hash(), "library_build_sha256": build_sha256()[:16],
                         "program": {k: program[k] for k in ("ready", "vgpr_count", "agpr_count", "sgpr_count",
                                                             "vgpr_spill_count", "sgpr_spill_count", "scratch_bytes",
                                                             "static_lds_bytes", "dynamic_lds_bytes", "code_bytes",
                                                             "deal_window", "hdr_asm")},
                         "kernel": kernel, "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_from": ("a HIP event pair around each timed step" if args.step_events else
                                            "one HIP event pair around the K timed steps on the launch stream "
                                            "(includes the launch boundaries)"),
                         "bytes_per_unit": bytes_per_pkt, "units_per_launch": n},
            "parity_sample_vs_oracle": ok,
            "parity_sample_per_rank": parity_ranks,
            "parity_sample_what": ("each rank's first 2^16 frames of its own shard, verdicts and rule ids against the "
                                   "oracle, after the timed loop; the AND over ranks"),
            "counters_summed_over_ranks_ok": sum_ok,
            "settle": {"seconds": round(settle_s, 2), "steps": settle_steps,
                       "what": "untimed steps before the warmup steps, until the GPU clocks reach steady state"},
        }
        from polycube_amd.iptables import comm_info
        ci = comm_info()
        line["rccl"] = {"library_resolved": {"version": ci["rccl_version"], "path": ci["rccl_path"]},
                        "torch": torch_rccl(), "mapped": rccl_libraries(),
                        "what": "library_resolved: the RCCL libpcn_ipt.so's ncclCommInitRank binds to (dladdr) and "
                                "ncclGetVersion reports -- the one that serves pcn_ipt_sync_counters; torch: "
                                "torch.cuda.nccl.version(); mapped: every librccl in the process"}
        if multi:
            line["multi_gpu"] = multi
        if world == 1 and cfg == 3 and not args.no_hits:
            line["hit_rates"] = hit_rate_sweep(ipt, fw, rs, n, dev, stream, kern_ms, synth.CONFIG_SEEDS[3])
        if world == 1 and cfg == 3 and not args.no_sizes:
            line["frame_sizes"] = frame_size_sweep(ipt, rules, frames, n, dev, stream, log)
        if cfg == 5:
            line["roofline"]["gather_ceiling"] = gather_ceiling(frames, offsets, lens, n, s_ptr, kern_ms)
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_rates(rules, frames_host, n, WORKLOADS[cfg], offsets_host, lens_host, hook,
                                             big or None, with_nproc=True)
            if cfg == 3:
                line["cpu_baselines"] = secondary_cpu_baselines(log)
        if world == 1 and not args.no_e2e and cfg != 5:
            line["e2e"] = e2e_legs(ipt, frames_host, n, rs, log)
        if world == 1 and not args.no_fw and cfg == 3:
            rate, ms, _ = fw_rate(rules, frames, n, dev, s_ptr, args.jit)
            hrate, hms, hinfo = fw_rate(rules, frames, n, dev, s_ptr, args.jit, horus=True)
            line["firewall"] = {
                "value": round(rate, 2), "unit": "Mpkt/s", "ms_per_call": round(ms, 4),
                "what": "the same rules and frames through the pcn-firewall personality (pcn_ipt_set_service): "
                        "INGRESS chain, conntrack OFF, Horus off (the rule pipeline)",
                "horus_default": {
                    "value": round(hrate, 2), "ms_per_call": round(hms, 4), "table": hinfo,
                    "what": "as the reference runs it: Horus on (Firewall.h:337). Rule 0 keys the table on its source "
                            "port, so every frame needs the Parser's stale ports (computed in the classify kernel, "
                            "which also leaves the carry for the next batch) and, with conntrack OFF, each Horus "
                            "miss drops (the tail call into the deleted ConntrackLabel)"}}
        if world == 1 and not args.no_ct and cfg == 3:
            rate, ms, live, shard = ct_rate(ipt, rs, n, dev)
            one_ms = ct_single_flow(ipt, rs, n, dev)
            line["stateful_conntrack"] = {
                "single_flow_ms": round(one_ms, 3),
                "single_flow_what": ct_single_flow.__doc__.split("\n", 1)[0] + " " +
                                    ct_single_flow.__doc__.split("\n", 1)[1].strip(),
                "value": round(rate, 2), "unit": "Mpkt/s", "ms_per_step": round(ms, 3),
                "flow_split_8": dict(shard, what="pcn_ipt_flow_split of the whole batch for rank 0 of 8 (split_ms, "
                                                 "incl. its count read-back), then rank 0's owned frames through "
                                                 "its own fresh connection table (share_ms)"),
                "what": f"same chain with the connection table on (pcn_ipt_ct_enable): 2^{args.log2n} 64B frames of "
                        f"2^16 interleaved flows, labels from and updates to the HBM table in batch order "
                        f"({live} live entries after the run)"}
        if world == 1 and cfg == 3 and not args.no_update:
            line["rule_update"] = rule_update_latency(dev, log)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ipt.close()


if __name__ == "__main__":
    main()
