"""GPU parity: the HIP datapath (through the C ABI) against the CPU oracle.

Bit-exact on verdicts, matched rule ids and every counter.  Runs in one process
on one MI355X (`pytest -m gpu`)."""
import ctypes as C
import os

import numpy as np
import pytest

from helpers import GpuCube, ip_nbo, load_scenarios
from oracle.ffi import Oracle
from polycube_amd import ffi, synth
from rulegen import PORTS, quirky_rules

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def make_pair(rules_by_chain, defaults=None, localip=(), ports=PORTS, **cfg):
    from polycube_amd import Iptables
    defaults = defaults or {}
    o = Oracle(cfg.get("max_counted_rules", 0), cfg.get("max_action_rules", 0))
    ipt = Iptables(device=0, **cfg)
    for name, idx in ports.items():
        o.add_port(name, idx)
        ipt.add_port(name, idx)
    o.set_localip(list(localip))
    ipt.set_localip(list(localip))
    ipt.interactive = False
    for chain in (0, 1, 2):
        rules = rules_by_chain.get(chain, [])
        d = defaults.get(chain, "ACCEPT")
        o.set_chain(chain, rules, d)
        o.apply_accept_established(chain)          # Chain::applyRules (Chain.cpp:408)
        ch = ipt.chain(chain)
        for r in rules:
            ch.append(**r)
        ch.default = d
        ch.apply_rules()
    return o, ipt


def run_both(o, ipt, dev, frames, n, *, stride=64, fixed_len=64, offsets=None, lens=None, in_port=None,
             const_in_port=1, direction=0, ct=None, hook=0):
    v_o, r_o = o.classify(frames, n=n, offsets=offsets, lens=lens, stride=stride, fixed_len=fixed_len,
                          in_port=in_port, const_in_port=const_in_port, direction=direction, ct_status=ct,
                          nthreads=NTHREADS, hook=hook)

    def t(a, dt=None):
        if a is None:
            return None
        a = np.ascontiguousarray(a)
        if dt is not None:
            a = a.view(dt)
        return torch.from_numpy(a).to(dev)
    v_g, r_g = ipt.classify(t(frames), n=n, offsets=t(offsets, np.int32), lens=t(lens, np.int16),
                            stride=stride, fixed_len=fixed_len, in_port=t(in_port, np.int16),
                            const_in_port=const_in_port, direction=direction, ct_status=t(ct), hook=hook)
    torch.cuda.synchronize()
    return v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy()


def assert_same(v_o, r_o, v_g, r_g):
    bad = np.nonzero((v_o != v_g) | (r_o != r_g))[0]
    assert bad.size == 0, (f"{bad.size} mismatches, first at {bad[:5]}: oracle {v_o[bad[:5]]}/{r_o[bad[:5]]} "
                           f"gpu {v_g[bad[:5]]}/{r_g[bad[:5]]}")


def assert_counters(o, ipt, chains=(0, 1, 2), n=None):
    for c in chains:
        k = n or 8000
        po, bo, dpo, dbo = o.read_counters(c, k)
        pg, bg, dpg, dbg = ipt.chain(c).read_counters(k)
        assert (dpo, dbo) == (dpg, dbg), f"default counters chain {c}"
        assert po == pg, f"pkts chain {c}"
        assert bo == bg, f"bytes chain {c}"


SCEN = load_scenarios()


JIT = pytest.mark.parametrize("jit", [-1, 1], ids=["generic", "chainprog"])


def assert_jit_used(ipt, jit):
    info = ipt.jit_info()
    if jit == 1:
        assert info["launches_jit"] > 0 and info["programs_failed"] == 0, info
    else:
        assert info["launches_jit"] == 0, info


@JIT
@pytest.mark.parametrize("sc", SCEN["scenarios"], ids=[s["name"] for s in SCEN["scenarios"]])
def test_reference_scenarios_on_gpu(dev, sc, jit):
    from polycube_amd import Iptables
    cube = GpuCube(Iptables(device=0, jit=jit), SCEN["ports"], SCEN["localip"])
    for k, st in enumerate(sc["steps"]):
        for op in st["ops"]:
            cube.op(op)
        if "probe" not in st:
            continue
        verdicts = cube.probe(st["probe"])
        got = "pass" if all(v == 1 for v in verdicts) else "fail"
        assert got == st["expect"], f"{sc['name']} step {k}: {verdicts}"
        if "counters" in st:
            c = st["counters"]
            stats = cube.ipt.chain(c["chain"]).stats()
            assert stats[c["rule"]][1] == c["pkts"]


@JIT
@pytest.mark.parametrize("cfg,n", [(1, 1 << 16), (2, 1 << 20), (3, 1 << 20)])
def test_config_parity(dev, cfg, n, jit):
    rs = synth.config_rules(cfg)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=jit)
    frames = synth.config_frames(cfg, n, rs).reshape(-1)
    assert_same(*run_both(o, ipt, dev, frames, n))
    assert_counters(o, ipt)
    assert_jit_used(ipt, jit)


@JIT
@pytest.mark.parametrize("seed", range(10))
def test_fuzz_parity(dev, seed, jit):
    """Quirky rules in all three chains, short/odd frames, random ports/ct, both directions."""
    rng = np.random.default_rng(seed)
    rules = {c: quirky_rules(int(rng.integers(0, 150)), seed * 10 + c) for c in (0, 1, 2)}
    if seed == 0:
        rules[0], rules[1] = [], []          # _INGRESS_ALLOWLOGIC
    if seed == 1:
        rules[1] = []                        # empty FORWARD, default DROP counters
    defaults = {c: ("DROP" if (seed + c) % 2 else "ACCEPT") for c in (0, 1, 2)}
    if seed == 0:
        defaults[0] = defaults[1] = "ACCEPT"
    localip = [ip_nbo(f"10.0.{k}.{k}") for k in range(0, 40)] + [ip_nbo("8.8.8.8")]
    o, ipt = make_pair(rules, defaults, localip, jit=jit)
    n = 1 << 16
    rs = synth.make_rules(64, seed, protos=(6, 17, 1))
    frames, lens = synth.fuzz_frames(n, seed, rs, stride=96)
    # steer some traffic at local addresses so INPUT/OUTPUT are exercised
    loc = rng.random(n) < 0.3
    pick = np.array([synth.ip_nbo(0)], np.uint32)
    f = frames.copy()
    for col in (26, 30):
        ips = rng.choice(np.array([(10 << 24) | (k << 16) | (0 << 8) | k for k in range(40)], np.uint32), size=n)
        be = np.stack([(ips >> 24) & 255, (ips >> 16) & 255, (ips >> 8) & 255, ips & 255], axis=1).astype(np.uint8)
        f[loc, col:col + 4] = be[loc]
    del pick
    in_port = rng.choice(np.array([0, 1, 2, 3, 7, 0xFFFF], np.uint16), size=n)
    ct = rng.integers(0, 4, size=n).astype(np.uint8) if seed % 2 else None
    for direction in (0, 1):
        res = run_both(o, ipt, dev, f.reshape(-1), n, stride=96, lens=lens, in_port=in_port,
                       direction=direction, ct=ct)
        assert_same(*res)
    assert_counters(o, ipt)


@pytest.mark.parametrize("seed", range(4))
def test_split_launch_edge_frames(dev, seed):
    """Split launches (a gather kernel, then a rule kernel over its 16-byte records:
    offsets / lens batches of a chain whose image exceeds LDS; opt-in, measured slower
    than the fused kernel) on edge-case frames:
    config 5's 10k rules in FORWARD and 3-6k in OUTPUT, INPUT empty (localip steers
    a share of the ingress frames to its default and of the egress frames to
    OUTPUT), short / odd frames, VLAN and IPv6, random in_port and ct_status arrays
    (odd seeds), both directions, the TC hook on seeds 2-3.  Bit-exact against the
    oracle: verdicts, rule ids and every counter."""
    rng = np.random.default_rng(seed)
    rs = synth.config_rules(5)
    rules = rs.rules()
    big = dict(max_rules=16384, max_counted_rules=10000, max_action_rules=10000)
    localip = [ip_nbo(f"10.0.{k}.{k}") for k in range(40)]
    os.environ["PCN_IPT_DEBUG_SPLIT"] = "1"      # read when the context is created (off by default)
    try:
        o, ipt = make_pair({1: rules, 2: rules[: 3000 + 1000 * seed]}, {0: "ACCEPT", 1: "DROP", 2: "ACCEPT"},
                           localip, jit=1, **big)
    finally:
        del os.environ["PCN_IPT_DEBUG_SPLIT"]
    n = 1 << 18
    frames, lens = synth.fuzz_frames(n, 100 + seed, rs, stride=96)
    f = frames.reshape(n, 96).copy()
    ips = rng.choice(np.array([(10 << 24) | (k << 16) | k for k in range(40)], np.uint32), size=n)
    be = np.stack([(ips >> 24) & 255, (ips >> 16) & 255, (ips >> 8) & 255, ips & 255], axis=1).astype(np.uint8)
    for col in (26, 30):                 # local sources (OUTPUT) and destinations (INPUT)
        loc = rng.random(n) < 0.2
        f[loc, col:col + 4] = be[loc]
    offsets = (np.arange(n, dtype=np.uint64) * 96).astype(np.uint32)
    in_port = rng.choice(np.array([0, 1, 2, 3, 7, 0xFFFF], np.uint16), size=n) if seed % 2 else None
    ct = rng.integers(0, 4, size=n).astype(np.uint8) if seed % 2 else None
    hook = 1 if seed >= 2 else 0
    for direction in (0, 1):
        res = run_both(o, ipt, dev, f.reshape(-1), n, stride=96, offsets=offsets, lens=lens, in_port=in_port,
                       direction=direction, ct=ct, hook=hook)
        assert_same(*res)
    assert_counters(o, ipt, n=10000)
    info = ipt.jit_info()
    assert info["launches_split"] >= 1 and info["programs_failed"] == 0, info


@JIT
@pytest.mark.parametrize("hook", [0, 1], ids=["xdp", "tc"])
@pytest.mark.parametrize("align", [1, 64], ids=["packed", "aligned"])
def test_imix_config5_parity(dev, jit, hook, align):
    """10k rules (extended limits), IMIX 64/576/1500 with VLAN/IPv6 mixed in
    (variable offsets), packed back to back or 64-byte aligned.  XDP: tagged
    and IPv6 frames pass unclassified; TC: the outer VLAN tag is stripped first
    and the inner IPv4 is classified."""
    rs = synth.config_rules(5)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, max_rules=16384, max_counted_rules=10000,
                       max_action_rules=10000, jit=jit)
    n = 1 << 17
    buf, offsets, lens = synth.imix_frames(rs, n, 5, align=align)
    v_o, r_o, v_g, r_g = run_both(o, ipt, dev, buf, n, offsets=offsets, lens=lens, hook=hook)
    assert_same(v_o, r_o, v_g, r_g)
    assert_counters(o, ipt, n=10000)
    assert_jit_used(ipt, jit)
    tagged = np.frombuffer(buf, np.uint8)[offsets.astype(np.int64) + 12] == 0x81
    assert (r_o[tagged] >= 0).any() == (hook == 1)      # TC classifies tagged frames, XDP passes them


@pytest.mark.parametrize("seed", range(2))
def test_tc_hook_fuzz_parity(dev, seed):
    """TC hook on fuzzed frames: VLAN tags (0x8100 / 0x88A8, short tagged
    frames), odd offsets and lengths, all three chains."""
    rng = np.random.default_rng(100 + seed)
    rules = {c: quirky_rules(int(rng.integers(20, 150)), 300 + seed * 10 + c) for c in (0, 1, 2)}
    localip = [ip_nbo(f"10.0.{k}.{k}") for k in range(0, 40)]
    o, ipt = make_pair(rules, {0: "DROP", 1: "ACCEPT", 2: "DROP"}, localip, jit=1)
    n = 1 << 15
    frames, lens = synth.fuzz_frames(n, 200 + seed, synth.make_rules(64, seed, protos=(6, 17, 1)), stride=96)
    f = frames.copy().reshape(n, 96)
    tag = rng.random(n) < 0.4
    f[tag, 16:96] = f[tag, 12:92].copy()
    f[tag, 12:14] = np.where(rng.random((int(tag.sum()), 1)) < 0.7, [0x81, 0x00], [0x88, 0xA8])
    f[tag, 14:16] = (0x00, 0x07)
    lens = lens.copy()
    lens[tag] = np.minimum(lens[tag].astype(np.int64) + 4, 96).astype(lens.dtype)
    short = rng.random(n) < 0.02
    lens[short] = rng.integers(12, 20, int(short.sum()))
    for direction in (0, 1):
        assert_same(*run_both(o, ipt, dev, f.reshape(-1), n, stride=96, lens=lens, direction=direction, hook=1))
    assert_counters(o, ipt)


def test_full_size_headline_config3(dev):
    """Config 3 at its bench size (2^24 frames), through the chain program the
    bench runs: bit-exact verdicts, rule ids and counters."""
    rs = synth.config_rules(3)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=1)
    n = 1 << 24
    frames = synth.config_frames(3, n, rs).reshape(-1)
    assert_same(*run_both(o, ipt, dev, frames, n))
    assert_counters(o, ipt)
    assert_jit_used(ipt, 1)


@pytest.mark.parametrize("stride,log2n", [(1500, 24), (1536, 22), (1024, 22), (576, 22), (256, 22), (128, 22),
                                          (1500, 16), (1501, 16)],
                         ids=["1500-full", "1536", "1024", "576", "256", "128", "1500-small", "1501-odd"])
def test_frame_size_sweep_parity(dev, stride, log2n):
    """The north_star frame sizes (bench.py frame_sizes): config 3's rules over
    fixed-size frames of `stride` bytes (packet_len = stride), 1500 B at the full
    2^24 batch (25 GB of frames in HBM).  16-byte multiples run the fixed-stride
    path, 1500 / 1501 the generic gather (a window at any byte offset).  A quarter
    of the batch is edge-case frames (fuzz_frames: odd ethertypes, VLAN / IPv6,
    ICMP types, GRE, odd protocols), the rest the bench's TCP/UDP mix.  The oracle
    reads each frame's first 128 bytes (the parse reads at most 76: an ICMP
    error's quoted header) with packet_len = stride.  Bit-exact verdicts, rule ids
    and counters (bytes = pkts * stride), through the chain program."""
    rs = synth.config_rules(3)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=1)
    n = 1 << log2n
    hdr = synth.config_frames(3, n, rs, seed=stride)
    rng = np.random.default_rng(stride)
    m = n // 4
    fz, _ = synth.fuzz_frames(m, stride, rs, stride=64)
    hdr[rng.choice(n, m, replace=False)] = fz.reshape(m, 64)
    buf = synth.spread_frames(torch.from_numpy(hdr.reshape(-1)).to(dev), n, stride)
    del hdr
    w = min(stride, 128)
    host = buf.view(n, stride)[:, :w].cpu().numpy().reshape(-1)
    for _ in range(2):                 # twice: the counters add up over launches
        v_o, r_o = o.classify(host, n=n, stride=w, fixed_len=stride, nthreads=NTHREADS)
        v_g, r_g = ipt.classify(buf, n=n, stride=stride, fixed_len=stride)
        torch.cuda.synchronize()
        assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
    assert_counters(o, ipt, chains=(1,), n=len(rs.rules()))
    assert_jit_used(ipt, 1)
    del buf
    torch.cuda.empty_cache()


@pytest.mark.parametrize("hook", [0, 1], ids=["xdp", "tc"])
def test_full_size_config5(dev, hook):
    """Config 5 at its bench size (2^22 IMIX frames packed back to back, 10k
    rules, VLAN and IPv6 mixed in), through the chain program the bench runs
    (two-item deal, packed counter copies): bit-exact verdicts, rule ids and
    every counter, at both hooks."""
    rs = synth.config_rules(5)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, max_rules=16384, max_counted_rules=10000,
                       max_action_rules=10000, jit=1)
    n = 1 << 22
    buf, offsets, lens = synth.imix_frames(rs, n, 5, align=1)
    for _ in range(2):                 # twice: the counters add up over launches
        assert_same(*run_both(o, ipt, dev, buf, n, offsets=offsets, lens=lens, hook=hook))
    assert_counters(o, ipt, n=10000)
    assert_jit_used(ipt, 1)


def test_table_level_boundary(dev):
    """pcn_ipt_load_chain with the maps the reference compiler emits (oracle export)."""
    rules = quirky_rules(180, 99)
    o, ipt = make_pair({1: rules}, {1: "DROP"})
    from polycube_amd import Iptables
    ipt2 = Iptables(device=0)
    keep = []
    t = ffi.Tables()
    t.nrules = len(rules)
    t.default_action = 0
    acts = (C.c_uint8 * len(rules))(*[1 if r.get("action") == "ACCEPT" else 0 for r in rules])
    t.actions = acts
    for f in range(8):
        keys, plen, vecs, nrw = o.export_map(1, f)
        if not keys:
            continue
        ka = (C.c_uint32 * len(keys))(*keys)
        pa = (C.c_uint8 * len(keys))(*plen)
        va = (C.c_uint64 * (len(keys) * nrw))(*[w for v in vecs for w in v])
        keep += [ka, pa, va]
        t.maps[f] = ffi.FieldMap(len(keys), ka, pa, va)
    ipt2.load_chain(1, t)
    n = 1 << 16
    frames, lens = synth.fuzz_frames(n, 3, synth.make_rules(32, 3), stride=96)
    in_port = np.random.default_rng(1).choice(np.array([1, 2, 3, 9], np.uint16), size=n)
    v_o, r_o, _, _ = run_both(o, ipt, dev, frames.reshape(-1), n, stride=96, lens=lens, in_port=in_port)
    _, _, v_g, r_g = run_both(o, ipt2, dev, frames.reshape(-1), n, stride=96, lens=lens, in_port=in_port)
    assert_same(v_o, r_o, v_g, r_g)


def test_counters_flush_stats_and_double_buffer(dev):
    rs = synth.config_rules(2)
    rules = rs.rules()
    o, ipt = make_pair({1: rules}, {1: "DROP"})
    ipt.interactive = True
    n = 1 << 18
    frames = synth.config_frames(2, n, rs).reshape(-1)
    tf = torch.from_numpy(frames).to(dev)
    v1, r1 = ipt.classify(tf, n=n)
    torch.cuda.synchronize()
    r1 = r1.cpu().numpy()
    fw = ipt.chain("FORWARD")
    pk, by, dp, db = fw.read_counters(len(rules), flush=True)
    assert sum(pk) == int((r1 >= 0).sum()) and dp == int((r1 == -1).sum())
    assert fw.read_counters(len(rules))[0] == [0] * len(rules)       # read-and-flush
    assert fw.read_counters(1)[2] == dp                                # default counters persist
    ipt.classify(tf, n=n)
    fw.insert(0, src="203.0.113.7", action="DROP")                     # stats shift with the insert
    st = fw.stats()
    want = np.bincount(r1[r1 >= 0], minlength=len(rules))
    assert [s[1] for s in st[1:-1]] == list(want) and st[0][1] == 0
    assert st[-1][0] == "DEFAULT" and st[-1][1] == 2 * dp
    # reload while batches are queued: every batch sees one complete table set
    outs = []
    for k in range(6):
        outs.append(ipt.classify(tf, n=n)[1])
        fw.default = "ACCEPT" if k % 2 else "DROP"
    torch.cuda.synchronize()
    for rr in outs:
        assert int((rr.cpu().numpy() == -2).sum()) == 0


def test_rccl_single_rank_counter_sync(dev):
    from polycube_amd import Iptables
    rs = synth.config_rules(2)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"})
    uid = Iptables.comm_unique_id()
    ipt.comm_init(1, 0, uid)
    n = 1 << 16
    frames = synth.config_frames(2, n, rs).reshape(-1)
    tf = torch.from_numpy(frames).to(dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):          # the all-gather of step k overlaps classify k+1 (comm stream)
        ipt.classify(tf, n=n, stream=s)
        ipt.sync_counters(s)
        o.classify(frames, n=n, nthreads=4)
    torch.cuda.synchronize()
    fw = ipt.chain("FORWARD")
    assert fw.read_counters(128, scope=1) == fw.read_counters(128, scope=0)
    assert fw.read_counters(128, scope=1) == o.read_counters(1, 128)


def test_u32_bins_split_launch_counts_exactly(dev):
    """2^26 jumbo-length frames (lens 65535) all hitting one rule: the per-
    workgroup u32 byte bins would wrap, so the launch is split; every counter
    must still come out exact (n pkts, n * 65535 bytes)."""
    rules = [{"dst": "10.1.0.0/16", "l4proto": "UDP", "dport": 53, "action": "ACCEPT"},
             {"src": "192.0.2.0/24", "action": "DROP"}]
    o, ipt = make_pair({1: rules}, {1: "DROP"})
    one = synth.build_frames(np.array([0xC0000201], np.uint32), np.array([0x0A010203], np.uint32),
                             np.array([17]), np.array([4000]), np.array([53]), np.array([0]),
                             frame_len=64).reshape(-1)
    n = 1 << 26
    frames = torch.from_numpy(one).to(dev)
    offsets = torch.zeros(n, dtype=torch.int32, device=dev)
    lens = torch.full((n,), -1, dtype=torch.int16, device=dev)      # 65535 as u16
    v, r = ipt.classify(frames, n=n, offsets=offsets, lens=lens)
    torch.cuda.synchronize()
    assert int((r == 0).sum()) == n and int((v == 1).sum()) == n
    pk, by, dp, db = ipt.chain("FORWARD").read_counters(2)
    assert pk == [n, 0] and by == [n * 65535, 0] and dp == 0 and db == 0
    del offsets, lens, v, r


def test_packed_counter_copies_fold_across_launches_and_streams(dev, monkeypatch):
    """Each workgroup adds a counter pair as one packed u64 (packets << 38 |
    bytes) into its copy of the chain's block; the host folds the copies into
    the plain block before any field could overflow.  With the test limit of
    2^14 packets per copy a 2^20-frame launch splits in two and every launch
    folds first, after waiting for the other stream's launches (two streams
    alternate).  Every counter must equal the oracle's over all launches."""
    monkeypatch.setenv("PCN_IPT_DEBUG_PACK_MAX_PKTS", str(1 << 14))
    rs = synth.config_rules(3)
    rules = rs.rules()
    o, ipt = make_pair({1: rules}, {1: "DROP"})
    n = 1 << 20
    frames = synth.config_frames(3, n, rs).reshape(-1)
    tf = torch.from_numpy(frames).to(dev)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(6):
        outs.append(ipt.classify(tf, n=n, stream=streams[k % 2].cuda_stream))
        o.classify(frames, n=n, nthreads=NTHREADS)
    torch.cuda.synchronize()
    assert_counters(o, ipt, chains=(1,), n=len(rules))
    # IMIX lengths: the byte field bounds the copies (test limit 2^20 bytes)
    n5 = 1 << 17
    buf, offsets, lens = synth.imix_frames(rs, n5, 7)
    for k in range(4):
        v_o, r_o, v_g, r_g = run_both(o, ipt, dev, buf, n5, offsets=offsets, lens=lens)
        assert_same(v_o, r_o, v_g, r_g)
    assert_counters(o, ipt, chains=(1,), n=len(rules))


def test_adaptive_deal_window_follows_the_traffic(dev):
    """A one-block chain's chain program deals 64 candidates a pass; when the
    previous launch's waves mostly held more (hit rate 1: 64-110 candidate words
    per wave) the 128-candidate program runs instead, and the 64 one again once
    the traffic falls back (hit rate 0.5: never more than 63).  The choice reads
    the kernel's own per-workgroup counts from host-mapped memory; results are
    identical either way."""
    import time
    rs = synth.config_rules(3)
    rules = rs.rules()
    o, ipt = make_pair({1: rules}, {1: "DROP"}, jit=1)
    chain = ipt.chain("FORWARD")
    n = 1 << 20
    frames = {}
    for h in (1.0, 0.5):
        cols = synth.make_headers(rs, n, 33, hit_frac=h)
        frames[h] = synth.build_frames(*cols, frame_len=64).reshape(-1)
    windows = []
    for h in (1.0, 0.5):
        tf = torch.from_numpy(frames[h]).to(dev)
        for k in range(8):
            v_g, r_g = ipt.classify(tf, n=n)
            torch.cuda.synchronize()
            if k in (0, 7):
                v_o, r_o = o.classify(frames[h], n=n, nthreads=NTHREADS)
                assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
            else:
                o.classify(frames[h], n=n, nthreads=NTHREADS)
            if k == 3:
                time.sleep(1.0)       # the 128-candidate program compiles in the background
        windows.append(chain.program_info()["deal_window"])
    assert windows == [128, 64], windows
    assert_counters(o, ipt, chains=(1,), n=len(rules))


def test_stream_of_a_closed_ring_is_never_touched(dev, monkeypatch):
    """A ring whose one stream carried batches, closed (its stream destroyed), then
    batches on the NULL stream and on a new stream: the context must not record an
    event on the dead stream (pcn_ipt_ring_destroy releases it first), and every
    counter still equals the oracle's -- with a fold before every launch (test
    limit), so the folds wait on the streams that remain."""
    monkeypatch.setenv("PCN_IPT_DEBUG_PACK_MAX_PKTS", str(1 << 13))
    rs = synth.config_rules(2)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=1)
    ring = ipt.ring(slots=2, slot_frames=1 << 14, slot_bytes=(1 << 14) * 64, streams=1)
    for k in range(3):
        slot, frames, _, _, _ = ring.acquire()
        f = synth.config_frames(2, 1 << 14, rs, seed=k).reshape(-1)
        frames[:f.size] = f
        ring.submit(slot, 1 << 14)
        o.classify(f, n=1 << 14, nthreads=NTHREADS)
        done, _, _ = ring.complete()
        ring.release(done)
    ring.close()
    n = 1 << 16
    frames = synth.config_frames(2, n, rs, seed=9).reshape(-1)
    tf = torch.from_numpy(frames).to(dev)
    side = torch.cuda.Stream()
    for stream in (None, side.cuda_stream, None):
        v_g, r_g = ipt.classify(tf, n=n, stream=stream)
        v_o, r_o = o.classify(frames, n=n, nthreads=NTHREADS)
        torch.cuda.synchronize()
        assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
    ipt.release_stream(side.cuda_stream)
    assert_counters(o, ipt, chains=(1,), n=len(rs.rules()))


def test_fold_waits_for_a_stream_that_was_alone(dev, monkeypatch):
    """A user stream U, then a two-stream ring (U + A + B known: events recorded),
    the ring closed (A, B released: U alone records nothing), more batches on U,
    then a new stream whose launches fold before every launch (test limit): the fold
    must wait for U's later batches, not for U's event from before the ring closed.
    Counters equal the oracle's."""
    monkeypatch.setenv("PCN_IPT_DEBUG_PACK_MAX_PKTS", str(1 << 13))
    rs = synth.config_rules(2)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=1)
    n = 1 << 16
    user = torch.cuda.Stream()
    batches = [synth.config_frames(2, n, rs, seed=20 + k).reshape(-1) for k in range(3)]
    dbatches = [torch.from_numpy(f).to(dev) for f in batches]
    torch.cuda.synchronize()
    ipt.classify(dbatches[0], n=n, stream=user.cuda_stream, rule_ids=False)
    o.classify(batches[0], n=n, nthreads=NTHREADS)
    ring = ipt.ring(slots=2, slot_frames=1 << 14, slot_bytes=(1 << 14) * 64, streams=2)
    for k in range(4):
        slot, frames, _, _, _ = ring.acquire()
        f = synth.config_frames(2, 1 << 14, rs, seed=40 + k).reshape(-1)
        frames[:f.size] = f
        ring.submit(slot, 1 << 14)
        o.classify(f, n=1 << 14, nthreads=NTHREADS)
        done, _, _ = ring.complete()
        ring.release(done)
    ring.close()
    for k in (1, 2):       # U alone again: several batches queued back to back
        for _ in range(4):
            ipt.classify(dbatches[k], n=n, stream=user.cuda_stream, rule_ids=False)
            o.classify(batches[k], n=n, nthreads=NTHREADS)
    side = torch.cuda.Stream()
    for _ in range(3):
        ipt.classify(dbatches[0], n=n, stream=side.cuda_stream, rule_ids=False)
        o.classify(batches[0], n=n, nthreads=NTHREADS)
    torch.cuda.synchronize()
    ipt.release_stream(side.cuda_stream)
    ipt.release_stream(user.cuda_stream)
    assert_counters(o, ipt, chains=(1,), n=len(rs.rules()))


def test_localip_input_output_from_lds(dev):
    """INPUT/OUTPUT selection by a 200-address localip set staged in LDS."""
    rs = synth.config_rules(2)
    rules = rs.rules()
    rng = np.random.default_rng(11)
    n = 1 << 16
    frames = synth.config_frames(2, n, rs).reshape(n, 64)
    dsts = frames[:, 30:34].copy().view(">u4").reshape(-1)
    local = sorted({int(synth.ip_nbo(int(x))) for x in rng.choice(dsts, 200, replace=False)})
    o, ipt = make_pair({0: rules[:64], 1: rules[64:], 2: rules[::2]}, {0: "DROP", 1: "ACCEPT", 2: "DROP"},
                       localip=local)
    for direction in (0, 1):
        v_o, r_o, v_g, r_g = run_both(o, ipt, dev, frames.reshape(-1), n, direction=direction)
        assert_same(v_o, r_o, v_g, r_g)
    assert_counters(o, ipt)


@pytest.mark.parametrize("zero_copy", [False, True], ids=["copy", "zero_copy"])
def test_ingest_ring_parity(dev, zero_copy):
    """Host ingest ring: frames filled into pinned slots, copied in (or, zero
    copy, read by the kernel in the pinned slots over PCIe), classified and the
    verdicts / rule ids copied back -- fixed-stride slots and IMIX slots
    (offsets, lens, in_port, TC hook) interleaved; equal to the oracle,
    counters included."""
    rs = synth.config_rules(2)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=1)
    ring = ipt.ring(slots=3, slot_frames=1 << 14, slot_bytes=(1 << 14) * 1600, rule_ids=True, zero_copy=zero_copy)
    expect = {}
    for k in range(8):
        slot, frames, offsets, lens, in_port = ring.acquire()
        n = (1 << 14) - 37 * k
        if k % 2 == 0:
            f = synth.config_frames(2, n, rs, seed=k).reshape(-1)
            frames[:f.size] = f
            ring.submit(slot, n)
            expect[slot] = o.classify(f, n=n, nthreads=NTHREADS)
        else:
            buf, off, ln = synth.imix_frames(rs, n, 40 + k)
            frames[:buf.size] = buf
            offsets[:n] = off
            lens[:n] = ln
            ports = np.random.default_rng(k).choice(np.array([0, 1, 2], np.uint16), size=n)
            in_port[:n] = ports
            ring.submit(slot, n, frames_bytes=buf.size, offsets=True, lens=True, in_port=True, hook=1)
            expect[slot] = o.classify(buf, n=n, offsets=off, lens=ln, in_port=ports, hook=1, nthreads=NTHREADS)
        if k >= 2:
            done, v, r = ring.complete()
            v_o, r_o = expect.pop(done)
            assert_same(v_o, r_o, v.copy(), r.copy())
            ring.release(done)
    while expect:
        done, v, r = ring.complete()
        v_o, r_o = expect.pop(done)
        assert_same(v_o, r_o, v.copy(), r.copy())
        ring.release(done)
    ring.close()
    assert_counters(o, ipt)


@pytest.mark.parametrize("skip", [0, 12], ids=["whole_window", "no_mac"])
@pytest.mark.parametrize("pack", [False, True], ids=["strided", "host_pack"])
@pytest.mark.parametrize("hook,hdr", [(0, 48), (1, 64)], ids=["xdp48", "tc64"])
def test_ingest_ring_header_only(dev, hook, hdr, pack, skip):
    """pcn_ipt_ring_batch.hdr_bytes: only each frame's first hdr bytes cross
    PCIe (a strided copy, packed on the device) while the lengths still come
    from fixed_len / lens: equal to the oracle on the whole frames.  64-byte
    frames at a 64-byte stride (the bench's slots, the fixed-stride kernel),
    fuzz frames (every protocol, edge lengths) at a 96-byte stride and up to
    1536-byte frames; too few header bytes and offsets batches are refused.
    hdr_skip 12: the Ethernet addresses stay on the host too (36 / 52 bytes a
    frame cross PCIe; the device rows sit at a 36 / 52-byte stride, each frame
    starting 12 bytes before its row), with the same verdicts."""
    from polycube_amd import IptablesError
    rs = synth.config_rules(3)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=1)
    ring = ipt.ring(slots=2, slot_frames=1 << 13, slot_bytes=(1 << 13) * 1536, rule_ids=True, host_pack=pack,
                    pack_threads=3)
    for k, stride in enumerate((64, 96, 1536, 64)):
        slot, frames, offsets, lens, in_port = ring.acquire()
        n = (1 << 13) - 5 * k
        if stride == 64:
            f = synth.config_frames(3, n, rs, seed=k).reshape(-1)
            ln, kw = None, {}
        else:
            f, ln = synth.fuzz_frames(n, 70 + k, rs, stride=stride)
            f = f.reshape(-1)
            lens[:n] = ln
            kw = dict(lens=True)
        frames[:f.size] = f
        ring.submit(slot, n, stride=stride, fixed_len=stride, hook=hook, hdr_bytes=hdr, hdr_skip=skip, **kw)
        v_o, r_o = o.classify(f, n=n, lens=ln, stride=stride, fixed_len=stride, hook=hook, nthreads=NTHREADS)
        done, v, r = ring.complete()
        assert done == slot
        assert_same(v_o, r_o, v.copy(), r.copy())
        ring.release(done)
    slot = ring.acquire()[0]
    for bad in (dict(hdr_bytes=hdr - 16), dict(hdr_bytes=hdr + 8), dict(hdr_bytes=hdr, offsets=True),
                dict(hdr_skip=12), dict(hdr_bytes=hdr, hdr_skip=4)):
        with pytest.raises(IptablesError) as e:
            ring.submit(slot, 16, stride=128, fixed_len=128, hook=hook, **bad)
        assert e.value.code == -22
    ring.release(slot)
    ring.close()
    assert_counters(o, ipt)


@JIT
def test_ragged_batch_sizes_fixed_stride(dev, jit):
    """Batches that end inside a wave's 64-frame group and inside a workgroup's
    row (the prefetch's clamped tail, lanes past n), from 1 frame up to more
    than one grid stride, on the fixed-stride fast path."""
    rs = synth.config_rules(3)
    o, ipt = make_pair({1: rs.rules()}, {1: "DROP"}, jit=jit)
    frames_all = synth.config_frames(3, 300_017, rs).reshape(-1)
    for n in (1, 2, 63, 64, 65, 777, 1025, 4097, 65_553, 262_147, 300_017):
        frames = frames_all[: n * 64]
        assert_same(*run_both(o, ipt, dev, frames, n))
    assert_counters(o, ipt)
    assert_jit_used(ipt, jit)
