"""GPU parity of stateful conntrack (conntrack.hip) against the CPU oracle.

Bit-exact on verdicts, rule ids, per-rule / default / accept-established
counters and the whole session table (keys, states, sequence numbers, ttl),
with state carried across batches.  One process, one MI355X (`pytest -m gpu`)."""
import ctypes

import numpy as np
import pytest

from helpers import GpuCube, ct_probe_frames, load_ct_scenarios, session_states
from oracle.ffi import Oracle
from polycube_amd import synth
from rulegen import quirky_rules
from test_gpu_parity import JIT, assert_counters, assert_same, make_pair

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
CT = load_ct_scenarios()
NOW = 1_700_000_000_123_456_789


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def t(dev, a, dt=None):
    if a is None:
        return None
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(dt) if dt is not None else a).to(dev)


def ct_pair(rules_by_chain, defaults=None, localip=(), cap_log2=16, **cfg):
    o, ipt = make_pair(rules_by_chain, defaults, localip, **cfg)
    o.ct_enable()
    o.ct_set_time(NOW)
    ipt.ct_enable(cap_log2)
    ipt.ct_set_time(NOW)
    return o, ipt


def run_ct(o, ipt, dev, frames, n, *, stride=128, lens=None, in_port=None, direction=0, hook=0, fixed_len=None):
    fixed_len = fixed_len or stride
    v_o, r_o = o.classify(frames, n=n, lens=lens, stride=stride, fixed_len=fixed_len, in_port=in_port,
                          direction=direction, hook=hook)
    v_g, r_g = ipt.classify(t(dev, frames), n=n, lens=t(dev, lens, np.int16), stride=stride, fixed_len=fixed_len,
                            in_port=t(dev, in_port, np.int16), direction=direction, hook=hook)
    torch.cuda.synchronize()
    return v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy()


def assert_tables(o, ipt):
    a, b = o.ct_dump(), ipt.ct_dump()
    assert len(a) == len(b), (len(a), len(b))
    for f in a.dtype.names:
        bad = np.nonzero(a[f] != b[f])[0]
        assert bad.size == 0, f"session table field {f}: {bad.size} differ, first {a[bad[:3]]} vs {b[bad[:3]]}"


def assert_ae(o, ipt):
    for c in range(3):
        assert o.read_accept_established(c) == ipt.chain(c).read_accept_established(), f"ae counters chain {c}"


@pytest.mark.parametrize("sc", CT["scenarios"], ids=[s["name"] for s in CT["scenarios"]])
def test_reference_conntrack_scenarios_on_gpu(dev, sc):
    from polycube_amd import Iptables
    ipt = Iptables(device=0, jit=1)
    ipt.ct_enable(12)
    ipt.ct_set_time(NOW)
    cube = GpuCube(ipt, CT["ports"], CT["localip"])
    for k, st in enumerate(sc["steps"]):
        for op in st["ops"]:
            cube.op(op)
        if "probe" in st:
            v = cube.ct_probe(st["probe"])
            got = "pass" if all(x == 1 for x in v) else "fail"
            assert got == st["expect"], f"{sc['name']} step {k} ({st.get('ref_line')}): {v}"
            if "drop_at" in st:
                d = st["drop_at"]
                assert v[d] == 0 and all(x == 1 for x in v[:d]), f"{sc['name']} step {k}: {v}"
        if "session" in st:
            assert st["session"]["state"] in session_states(ipt.ct_dump(), st["session"]["match"])


CT_RULES = [{"conntrack": "ESTABLISHED", "action": "ACCEPT"},
            {"conntrack": "INVALID", "action": "DROP"},
            {"conntrack": "RELATED", "l4proto": "ICMP", "action": "ACCEPT"},
            {"conntrack": "NEW", "l4proto": "TCP", "tcpflags": "SYN !ACK", "action": "ACCEPT"}]


@JIT
@pytest.mark.parametrize("mode", ["plain", "ct_rules", "accept_established"])
def test_flow_traffic_parity_across_batches(dev, jit, mode):
    rs = synth.config_rules(2)
    rules = rs.rules()
    if mode == "ct_rules":
        rules = CT_RULES[1:] + rules
    elif mode == "accept_established":
        rules = CT_RULES + rules
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, jit=jit)
    assert ipt.chain(1).accept_established == (mode == "accept_established")
    f, lens = synth.flow_traffic(30000, 1500, 5, rs=rs, lens_mode="mixed")
    for lo, hi in ((0, 7000), (7000, 7001), (7001, 30000)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, f[lo * 128:hi * 128], hi - lo, lens=lens[lo:hi])
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)
    assert ipt.ct_info()["inserts_lost"] == 0


@pytest.mark.parametrize("offset", [0, 1])
def test_counters_of_a_10k_rule_chain_with_rule_ids_at_any_alignment(dev, offset):
    """ct_count over the final rule ids: rule ids above the 1024 LDS bins (global
    counters), ragged batch ends (the 16-byte loads' tail), and a caller's rule-id
    buffer 4 bytes off 16-byte alignment (the 4-byte-load kernel)."""
    rs = synth.config_rules(5)
    rules = rs.rules()
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, jit=1, max_rules=16384, max_counted_rules=10000,
                     max_action_rules=10000)
    f, lens = synth.flow_traffic(30000, 2000, 11, rs=rs, lens_mode="mixed")
    for lo, hi in ((0, 9001), (9001, 9003), (9003, 30000)):
        n = hi - lo
        buf = torch.empty(n + 4, dtype=torch.int32, device=dev)
        rid = buf[offset:offset + n]
        assert (rid.data_ptr() % 16 != 0) == (offset != 0)
        v_o, r_o = o.classify(f[lo * 128:hi * 128], n=n, lens=lens[lo:hi], stride=128, fixed_len=128)
        v_g, r_g = ipt.classify(t(dev, f[lo * 128:hi * 128]), n=n, lens=t(dev, lens[lo:hi], np.int16), stride=128,
                                fixed_len=128, rule_ids=rid)
        torch.cuda.synchronize()
        assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
    assert (r_o >= 1024).any()
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)


@pytest.mark.parametrize("mode", ["plain", "ct_rules"])
def test_fixed_stride_64_with_lengths(dev, mode):
    """ct_prep's coalesced path (frames at a 64-byte stride, windows and walk records
    transposed through LDS) with per-frame lengths, ragged batches whose last group falls
    back to per-lane windows, and, with conntrack rules, four stage-A outcomes per record."""
    rs = synth.config_rules(2)
    rules = rs.rules()
    if mode == "ct_rules":
        rules = CT_RULES[1:] + rules
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, jit=1)
    n = 20000
    f, lens = synth.flow_traffic(n, 800, 9, stride=64, rs=rs, lens_mode="mixed", p_noise=0.1)
    lens = np.minimum(lens, 64).astype(np.uint16)
    for lo, hi in ((0, 6001), (6001, 6064), (6064, n)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, f[lo * 64:hi * 64], hi - lo, stride=64, lens=lens[lo:hi])
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)


@pytest.mark.parametrize("seed", [1, 2])
def test_fuzz_quirky_rules_both_directions_and_hooks(dev, seed):
    """Quirky rules with conntrack fields in all chains, localip, INPUT/FORWARD/OUTPUT,
    XDP and TC hooks, short frames, ICMP errors quoting live flows."""
    rng = np.random.default_rng(seed)
    rules = {c: quirky_rules(40, seed * 10 + c) for c in range(3)}
    rules[1] = CT_RULES + rules[1]
    localip = [synth.ip_nbo(int(x)) for x in rng.integers(0, 2**32, size=8)]
    o, ipt = ct_pair(rules, {0: "DROP", 1: "DROP", 2: "ACCEPT"}, localip=localip, jit=1)
    f, lens = synth.flow_traffic(12000, 700, seed, stride=128, lens_mode="mixed", p_noise=0.2, p_err=0.05)
    nb = f.reshape(12000, 128)
    # some packets towards / from the host (INPUT / OUTPUT)
    sel = rng.random(12000) < 0.2
    nb[sel, 30:34] = np.frombuffer(np.array(localip[:1], np.uint32).tobytes(), np.uint8)
    ports = rng.integers(0, 4, size=12000).astype(np.uint16)
    for k, (lo, hi) in enumerate(((0, 4000), (4000, 8000), (8000, 12000))):
        for direction in (0, 1):
            hook = k % 2
            v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo, lens=lens[lo:hi],
                                        in_port=ports[lo:hi], direction=direction, hook=hook)
            assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    for c in range(3):
        assert_counters(o, ipt, chains=(c,), n=len(rules[c]) + 1)
    assert_ae(o, ipt)


def test_long_echo_replies_read_the_quoted_flow(dev):
    """Echo replies >= 70 B whose own entry is not reversed take ICMP_MISS and
    look up the quoted header's key (ConntrackLabel_dp.c:450-531).  Quoting
    flows with packets in the same batch, most of them go to ct_tail (the
    walk stops at the first, one wave takes the rest in order)."""
    rng = np.random.default_rng(9)
    o, ipt = ct_pair({1: [{"conntrack": "RELATED", "action": "ACCEPT"},
                          {"conntrack": "INVALID", "action": "DROP"}]}, {1: "ACCEPT"})
    n = 4000
    f, lens = synth.flow_traffic(n, 100, 3, stride=128, p_icmp=0.4, p_err=0.1)
    nb = f.reshape(n, 128)
    icmp = nb[:, 23] == 1
    # make echo replies quote random live flows and be long
    rep = icmp & (rng.random(n) < 0.5)
    nb[rep, 34] = 0
    src = nb[:, 26:30].copy()
    dst = nb[:, 30:34].copy()
    q = rng.integers(0, n, size=n)
    nb[rep, 42] = 0x45
    nb[rep, 51] = nb[q[rep], 23]
    nb[rep, 54:58] = src[q[rep]]
    nb[rep, 58:62] = dst[q[rep]]
    nb[rep, 62:66] = nb[q[rep], 34:38]
    lens = np.where(rep, rng.choice(np.array([70, 98, 128]), size=n), 128).astype(np.uint16)
    for lo, hi in ((0, 1500), (1500, 4000)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo, lens=lens[lo:hi])
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=3)


def test_stateless_accept_established_with_given_labels(dev):
    """Labels supplied per packet (conntrack off): rule 0 {ESTABLISHED, ACCEPT}
    hits move to the accept-established path (rule id -3, its counters)."""
    rs = synth.config_rules(2)
    rules = CT_RULES + rs.rules()
    o, ipt = make_pair({1: rules}, {1: "DROP"})
    n = 20000
    frames = synth.config_frames(2, n, rs).reshape(-1)
    ct = np.random.default_rng(4).integers(0, 4, size=n).astype(np.uint8)
    v_o, r_o = o.classify(frames, n=n, ct_status=ct)
    v_g, r_g = ipt.classify(t(dev, frames), n=n, ct_status=t(dev, ct))
    torch.cuda.synchronize()
    assert_same(v_o, r_o, v_g.cpu().numpy(), r_g.cpu().numpy())
    assert (r_o == -3).sum() > 1000
    assert_counters(o, ipt, n=len(rules))
    assert_ae(o, ipt)
    # ChainStats: rule 0 = its counters + the accept-established ones (ChainStats.cpp:64-103)
    st = ipt.chain(1).stats()
    assert st[0][1] == int((r_o == -3).sum())


@pytest.mark.parametrize("setup", ["forward", "local_in_out", "allow_logic", "empty_input_drop"])
def test_stage_a_builds_the_walk_records(dev, setup):
    """Batches of 64-byte frames with one label: the classify pass (stage A) builds
    the walk records, key buckets and {len, cinfo} words itself (devchain.h
    ct_walk_rec) and advances the stale-port carry, so ct_prep never runs and the
    frames are read once.  ICMP-heavy traffic (each echo keys on the stale ports of
    the last TCP/UDP frame before it, Q4, across 64-frame groups and batches), odd
    batch sizes, noise, both directions, and chain selections: FORWARD only; local
    addresses (INPUT / OUTPUT); allow logic (all PASS_LABELING); an empty INPUT
    chain with DROP (DROP_NO_LABELING).  Bit-exact against the oracle: verdicts,
    rule ids, counters and the whole table, and every batch took the fused path."""
    from test_gpu_parity import ip_nbo
    rs = synth.config_rules(3)
    rules = rs.rules()
    localip, chains, defaults = (), {1: rules}, {1: "DROP"}
    if setup == "local_in_out":
        localip = [ip_nbo(f"10.0.{k}.{k}") for k in range(40)]
        chains = {0: rules[:300], 1: rules[300:], 2: rules[::3]}
        defaults = {0: "ACCEPT", 1: "DROP", 2: "DROP"}
    elif setup == "allow_logic":
        chains, defaults = {2: rules[:100]}, {0: "ACCEPT", 1: "ACCEPT", 2: "ACCEPT"}
    elif setup == "empty_input_drop":
        localip = [ip_nbo(f"10.0.{k}.{k}") for k in range(40)]
        chains, defaults = {1: rules}, {0: "DROP", 1: "ACCEPT"}
    o, ipt = ct_pair(chains, defaults, localip, cap_log2=18, jit=1)
    rng = np.random.default_rng(7)
    n = 1 << 18
    f, _ = synth.flow_traffic(n, 3000, 11, stride=64, rs=rs, p_icmp=0.3, p_noise=0.1, p_err=0.05)
    fr = f.reshape(n, 64)
    if localip:
        ips = rng.choice(np.array([(10 << 24) | (k << 16) | k for k in range(40)], np.uint32), size=n)
        be = np.stack([(ips >> 24) & 255, (ips >> 16) & 255, (ips >> 8) & 255, ips & 255], axis=1).astype(np.uint8)
        for col in (26, 30):
            loc = rng.random(n) < 0.15
            fr[loc, col:col + 4] = be[loc]
    cuts = [0, 1, 64, 129, 1000, 1 << 16, (1 << 16) + 7, n]
    nb = 0
    for direction in (0, 1):
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, fr[lo:hi].reshape(-1), hi - lo, stride=64, direction=direction)
            assert_same(v_o, r_o, v_g, r_g)
            nb += 1
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)
    assert ipt.ct_info()["fused_batches"] == nb, ipt.ct_info()


def test_stage_a_records_from_the_generic_kernel(dev):
    """The fused stage A through the generic classify kernel (no chain program: jit
    -1), which carries the same record building and stale-port publication: ICMP-heavy
    64-byte frames over ragged batches, bit-exact against the oracle, tables included."""
    rs = synth.config_rules(3)
    rules = rs.rules()
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, cap_log2=18, jit=-1)
    n = 1 << 16
    f, _ = synth.flow_traffic(n, 1500, 31, stride=64, rs=rs, p_icmp=0.4, p_noise=0.1, p_err=0.05)
    fr = f.reshape(n, 64)
    cuts = [0, 63, 64, 4100, 30001, n]
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, fr[lo:hi].reshape(-1), hi - lo, stride=64)
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert ipt.ct_info()["fused_batches"] == len(cuts) - 1, ipt.ct_info()
    assert ipt.jit_info()["launches_jit"] == 0, ipt.jit_info()


def test_stage_a_stale_ports_across_icmp_only_stretches(dev):
    """The fused stage A's stale ports (Q4) where whole runs of 64-frame groups hold
    no TCP/UDP frame: every ICMP frame there keys on the ports of the last TCP/UDP
    frame before the stretch, in this batch or (a batch that starts with the stretch,
    and an all-ICMP batch) in an earlier one -- what conntrack.hip ct_stale_agg /
    ct_stale_fix resolve after the launch, across its 4096-group runs.  Bit-exact
    against the oracle, tables and counters included, every batch on the fused path."""
    rs = synth.config_rules(3)
    rules = rs.rules()
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, cap_log2=18, jit=1)
    mixed, _ = synth.flow_traffic(1 << 18, 2000, 21, stride=64, rs=rs, p_icmp=0.3, p_noise=0.05, p_err=0.05)
    icmp, _ = synth.flow_traffic(1 << 19, 3000, 22, stride=64, rs=rs, p_icmp=1.0, p_noise=0.0, p_err=0.0)
    mixed, icmp = mixed.reshape(-1, 64), icmp.reshape(-1, 64)
    assert set(np.unique(icmp[:, 23])) == {1}, "the stretch is all ICMP"
    batches = [
        np.concatenate([mixed[:5000], icmp[:300000], mixed[5000:5100]]),   # > 4096 ICMP-only groups mid-batch
        icmp[300000:400001],                                              # a batch of ICMP only: the carry
        np.concatenate([icmp[400001:400100], mixed[5100:90000]]),          # starts with the stretch
        mixed[90000:90037],
    ]
    nb = 0
    for fr in batches:
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, np.ascontiguousarray(fr).reshape(-1), len(fr), stride=64)
        assert_same(v_o, r_o, v_g, r_g)
        nb += 1
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert ipt.ct_info()["fused_batches"] == nb, ipt.ct_info()


def test_headline_size_flows_parity(dev):
    """2^22 packets of 2^16 interleaved flows, 64-byte frames, config-3 rules."""
    rs = synth.config_rules(3)
    o, ipt = ct_pair({1: rs.rules()}, {1: "DROP"}, cap_log2=18, jit=1)
    n = 1 << 22
    f, _ = synth.flow_traffic(n, 1 << 16, 21, stride=64, rs=rs)
    v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, f, n, stride=64)
    assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=1001)


@pytest.mark.parametrize("p_icmp", [0.0, 0.1])
def test_long_runs_walk_a_wave_each(dev, p_icmp):
    """Keys with more than PCN_CT_LONG_RUN (128) packets in one batch get a whole wave
    (conntrack.hip walk_long: records staged in LDS 64 at a time, eligible
    segments labelled in parallel); interleaved with many short flows, TCP
    noise (INVALID paths, FIN/RST) and, with ICMP, echo replies that split the
    batch into segments.  Bit-exact vs the oracle across batches."""
    rs = synth.config_rules(2)
    rules = CT_RULES + rs.rules()
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, jit=1)
    rng = np.random.default_rng(31)
    n_long, n_short = 48000, 16000
    fl, _ = synth.flow_traffic(n_long, 12, 31, stride=64, rs=rs, p_icmp=p_icmp, p_noise=0.03, p_err=0.0)
    fs, _ = synth.flow_traffic(n_short, 2000, 32, stride=64, rs=rs, p_icmp=p_icmp, p_noise=0.05)
    n = n_long + n_short
    slot = np.zeros(n, bool)
    slot[rng.choice(n, size=n_short, replace=False)] = True
    nb = np.empty((n, 64), np.uint8)
    nb[~slot] = fl.reshape(n_long, 64)
    nb[slot] = fs.reshape(n_short, 64)
    # the long flows give runs far past the threshold inside one batch
    ip = nb[:30000, 26:34].view(">u4")
    pt = nb[:30000, 34:38].view(">u2")
    key = np.stack([ip.min(1), ip.max(1), pt.min(1), pt.max(1), nb[:30000, 23]], 1).astype(np.int64)
    _, cnt = np.unique(key, axis=0, return_counts=True)
    assert (cnt >= 1000).sum() >= 5, np.sort(cnt)[-12:]
    for lo, hi in ((0, 30000), (30000, 30001), (30001, n)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo, stride=64)
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)


def test_long_runs_resume_across_echo_reply_segments(dev):
    """Long echo replies (>= 70 B) quoting flows of the same batch: the walk
    stops every run at the first of them, and ct_tail resumes the long runs
    (walk_long) and the short ones from their cursors between them, bit-exact
    vs the oracle."""
    rng = np.random.default_rng(41)
    o, ipt = ct_pair({1: [{"conntrack": "RELATED", "action": "ACCEPT"},
                          {"conntrack": "INVALID", "action": "DROP"}] + synth.config_rules(2).rules()},
                     {1: "ACCEPT"}, jit=1)
    n = 40000
    f, _ = synth.flow_traffic(n, 10, 41, stride=128, p_icmp=0.2, p_err=0.02, p_noise=0.03)
    nb = f.reshape(n, 128)
    icmp = nb[:, 23] == 1
    rep = icmp & (rng.random(n) < 0.02)               # ~80 long echo replies: ~80 segments
    nb[rep, 34] = 0
    q = rng.integers(0, n, size=n)
    nb[rep, 42] = 0x45
    nb[rep, 51] = nb[q[rep], 23]
    nb[rep, 54:58] = nb[q[rep], 26:30]
    nb[rep, 58:62] = nb[q[rep], 30:34]
    nb[rep, 62:66] = nb[q[rep], 34:38]
    lens = np.where(rep, 98, 128).astype(np.uint16)
    for lo, hi in ((0, 25000), (25000, n)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo, lens=lens[lo:hi])
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(synth.config_rules(2).rules()) + 3)


def test_errors_quoting_the_all_zero_key_among_inserts(dev):
    """ICMP errors quoting proto 0 between 0.0.0.0 and itself, ports 0: the one
    key a stale (zero) read of a slot claimed in the same launch could match,
    so conntrack.hip's table_slot re-reads it after an acquire.  Interleaved
    with a fresh table's worth of inserts, it stays a miss (INVALID) as in the
    oracle."""
    o, ipt = ct_pair({1: [{"conntrack": "RELATED", "action": "ACCEPT"},
                          {"conntrack": "INVALID", "action": "DROP"}]}, {1: "ACCEPT"}, cap_log2=12)
    rng = np.random.default_rng(17)
    n = 24000
    f, _ = synth.flow_traffic(n, 3000, 17, stride=128, p_icmp=0.0, p_err=0.0)
    nb = f.reshape(n, 128)
    err = rng.random(n) < 0.1
    nb[err, 23] = 1
    nb[err, 34] = 3                                   # destination unreachable
    zero = np.zeros(n, np.int64)
    synth.set_icmp_inner(nb, err, zero, zero, zero, zero, zero)
    for lo, hi in ((0, 12000), (12000, n)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo)
        assert_same(v_o, r_o, v_g, r_g)
        assert (r_o[err[lo:hi]] == 1).all()          # INVALID -> DROP rule
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=3)


def test_full_table_inserts_and_misses_stay_bounded(dev):
    """A full table: every further insert and miss stops after 512 probes
    (conntrack.hip kMaxProbe) instead of scanning the whole table, and the
    live entries stay findable."""
    import time
    o, ipt = ct_pair({1: []}, {1: "ACCEPT"}, cap_log2=14)
    n = 40000
    f, _ = synth.flow_traffic(n, n, 23, stride=64, p_icmp=0.0, p_noise=0.0, p_err=0.0)   # one packet per flow
    ipt.classify(t(dev, f), n=n, stride=64, fixed_len=64)
    torch.cuda.synchronize()
    assert ipt.ct_info()["inserts_lost"] > 0
    live = len(ipt.ct_dump())
    assert 0 < live <= 1 << 14
    g, _ = synth.flow_traffic(n, n, 24, stride=64, p_icmp=0.0, p_noise=0.0, p_err=0.0)
    t0 = time.perf_counter()
    ipt.classify(t(dev, g), n=n, stride=64, fixed_len=64)
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 10.0
    assert len(ipt.ct_dump()) >= live


def test_full_table_drops_inserts_without_faulting(dev):
    o, ipt = ct_pair({1: []}, {1: "ACCEPT"}, cap_log2=10)
    f, _ = synth.flow_traffic(20000, 5000, 8, stride=64, p_icmp=0.0, p_noise=0.0)
    ipt.classify(t(dev, f), n=20000, stride=64, fixed_len=64)
    torch.cuda.synchronize()
    info = ipt.ct_info()
    assert info["inserts_lost"] > 0
    assert 1000 < len(ipt.ct_dump()) <= 1024


def test_ring_over_many_streams_keeps_batch_order(dev):
    """A stateful context fed by the ingest ring, one stream per slot: the
    batches share the connection table and the conntrack scratch, so each
    one's stage A waits for the previous batch's last conntrack kernel.  Four
    slots are submitted back to back with no wait between them; verdicts,
    rule ids, counters and the session table equal one sequential oracle."""
    rs = synth.config_rules(2)
    rules = CT_RULES + rs.rules()
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, jit=1)
    n_all, nb = 32000, 4
    f, lens = synth.flow_traffic(n_all, 900, 17, rs=rs, lens_mode="mixed")
    per = n_all // nb
    ring = ipt.ring(slots=nb, slot_frames=per, slot_bytes=per * 128, streams=nb, rule_ids=True)
    expect = {}
    for k in range(nb):
        slot, frames, _, lns, _ = ring.acquire()
        lo, hi = k * per, (k + 1) * per
        frames[:per * 128] = f[lo * 128:hi * 128]
        lns[:per] = lens[lo:hi]
        ring.submit(slot, per, stride=128, fixed_len=128, lens=True)
        expect[slot] = o.classify(f[lo * 128:hi * 128], n=per, lens=lens[lo:hi], stride=128, fixed_len=128)
    while expect:
        done, v, r = ring.complete()
        v_o, r_o = expect.pop(done)
        assert_same(v_o, r_o, v.copy(), r.copy())
        ring.release(done)
    ring.close()
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)


def test_ping_replies_of_98_bytes_walk_in_their_runs(dev):
    """Ordinary pings: 98-byte echo replies (>= 70 B, so ICMP_MISS may read
    their payload as a quoted header) whose payload quotes nothing of the
    batch -- walked inside their own key's run with a direct read of the
    quoted key (ct_hard_split), no tail.  A few replies quote live flows of the
    batch (the tail).  Verdicts, rule ids, counters and the table vs the oracle."""
    rng = np.random.default_rng(77)
    rules = [{"conntrack": "RELATED", "action": "ACCEPT"}, {"conntrack": "INVALID", "action": "DROP"},
             {"l4proto": "ICMP", "conntrack": "NEW", "action": "ACCEPT"}] + synth.config_rules(2).rules()
    o, ipt = ct_pair({1: rules}, {1: "ACCEPT"}, cap_log2=18, jit=1)
    n = 1 << 18
    f, _ = synth.flow_traffic(n, 4000, 77, stride=128, p_icmp=0.5, p_err=0.01, p_noise=0.02)
    nb = f.reshape(n, 128)
    icmp = nb[:, 23] == 1
    reply = icmp & (nb[:, 34] == 0)
    lens = np.where(icmp, 98, 128).astype(np.uint16)
    nb[reply, 42:98] = rng.integers(0, 256, size=(int(reply.sum()), 56), dtype=np.uint8)   # ping payload
    quote = reply & (rng.random(n) < 0.001)                 # a few quote a flow of the batch
    q = rng.integers(0, n, size=n)
    nb[quote, 42] = 0x45
    nb[quote, 51] = nb[q[quote], 23]
    nb[quote, 54:62] = nb[q[quote], 26:34]
    nb[quote, 62:66] = nb[q[quote], 34:38]
    assert reply.sum() > 20000
    for lo, hi in ((0, n // 2), (n // 2, n)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo, lens=lens[lo:hi])
        assert_same(v_o, r_o, v_g, r_g)
    assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)


def test_stateful_classify_is_stream_asynchronous(dev):
    """pcn_ipt_classify with the connection table on queues the whole pipeline
    (plan and walk sized on the device, no read-back): right after the call on
    a 2^24-frame batch the stream still has work, and the call returns in a
    fraction of the batch's time."""
    import time
    rs = synth.config_rules(3)
    from polycube_amd import Iptables
    ipt = Iptables(device=0, jit=1)
    ipt.interactive = False
    ch = ipt.chain("FORWARD")
    for r in rs.rules():
        ch.append(**r)
    ch.default = "DROP"
    ch.apply_rules()
    ipt.ct_enable(20)
    ipt.ct_set_time(NOW)
    base, _ = synth.flow_traffic(1 << 20, 1 << 14, 5, stride=64, rs=rs)
    frames = torch.from_numpy(base).to(dev).repeat(16)
    n = 1 << 24
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        ipt.classify(frames, n=n, verdicts=v, stream=s.cuda_stream)     # warm: scratch allocations
        s.synchronize()
        t0 = time.perf_counter()
        ipt.classify(frames, n=n, verdicts=v, stream=s.cuda_stream)
        t_call = time.perf_counter() - t0
        busy = not s.query()
        s.synchronize()
        t_all = time.perf_counter() - t0
    assert busy, "the stream was idle right after the call: the call waited for the batch"
    assert t_call < 0.5 * t_all, (t_call, t_all)
    ipt.close()


@pytest.mark.parametrize("max_entries", [700, 2000])
def test_lru_capacity_evicts_like_the_oracle(dev, max_entries):
    """More live connections than max_entries: after every batch both drop the
    least recently touched entries down to max_entries (conntrack.hip ct_ev_*:
    a radix select over the touch stamps).  Verdicts, rule ids, counters, the
    whole table and the eviction count equal the oracle's, batch after batch,
    with ICMP errors (touching the quoted key), long runs and echo replies."""
    rules = CT_RULES + synth.config_rules(2).rules()
    o, ipt = ct_pair({1: rules}, {1: "DROP"}, cap_log2=15, jit=1)
    o.ct_set_max_entries(max_entries)
    ipt.ct_set_max_entries(max_entries)
    f, lens = synth.flow_traffic(60000, 9000, 13, stride=128, lens_mode="mixed", p_err=0.05, p_icmp=0.2)
    nb = f.reshape(60000, 128)
    for lo, hi in ((0, 15000), (15000, 15001), (15001, 40000), (40000, 60000)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb[lo:hi].reshape(-1), hi - lo, lens=lens[lo:hi])
        assert_same(v_o, r_o, v_g, r_g)
        assert_tables(o, ipt)
        assert len(ipt.ct_dump()) <= max_entries
    assert ipt.ct_info()["evicted"] == o.ct_info()["evicted"]
    assert o.ct_info()["evicted"] > 0
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)


def test_lru_crosses_the_reference_capacity(dev):
    """The default max_entries is the reference's 65536 (lru_hash,
    Iptables_ConntrackLabel_dp.c:112): 2^17 UDP connections over three
    batches leave exactly 65536 live entries, the most recently touched ones."""
    rs = synth.config_rules(2)
    o, ipt = ct_pair({1: rs.rules()}, {1: "ACCEPT"}, cap_log2=19)
    assert ipt.ct_info()["max_entries"] == o.ct_info()["max_entries"] == 65536
    n = 3 * (1 << 17)
    rng = np.random.default_rng(3)
    src = rng.integers(0, 2**32, size=1 << 17, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(1024, 65535, size=1 << 17)
    pick = np.concatenate([np.arange(1 << 17), rng.integers(0, 1 << 17, size=n - (1 << 17))])
    f = synth.build_frames(src[pick], np.full(n, 0x0A000001, np.uint32), np.full(n, 17), sp[pick],
                           np.full(n, 53), np.zeros(n, np.int32), frame_len=64).reshape(-1)
    for lo, hi in ((0, 1 << 17), (1 << 17, 2 << 17), (2 << 17, n)):
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, f[lo * 64:hi * 64], hi - lo, stride=64)
        assert_same(v_o, r_o, v_g, r_g)
        assert_tables(o, ipt)
    assert len(ipt.ct_dump()) == 65536
    assert ipt.ct_info()["evicted"] == o.ct_info()["evicted"]


def _elephants(rng, flows, phase, per, *, close_at=None, reopen_at=None):
    """`per` packets of each long flow (proto, src, dst, sport, dport, X, Y) in
    arrival order, randomly interleaved: phase "open" starts TCP with its
    handshake, "data" continues it; a flow in `close_at` (flow -> fraction)
    sends FIN-ACK, FIN-ACK, ACK there and data after it, one in `reopen_at`
    a new SYN.  UDP flows alternate directions."""
    cols = {k: [] for k in ("t", "src", "dst", "proto", "sport", "dport", "flags", "seq", "ack")}
    for f, (proto, a, b, pa, pb, X, Y) in enumerate(flows):
        t = np.sort(rng.random(per))
        rev = (np.arange(per) % 2).astype(bool)
        flags = np.where(rng.random(per) < 0.3, 0x18, 0x10)
        seq = np.where(rev, Y + 1, X + 1)
        ack = np.where(rev, X + 1, Y + 1)
        if proto == synth.TCP and phase == "open":
            rev[:3] = (False, True, False)
            flags[:3] = (0x02, 0x12, 0x10)
            seq[:3] = (X, Y, X + 1)
            ack[:3] = (0, X + 1, Y + 1)
        if proto == synth.TCP and close_at and f in close_at:
            c = int(per * close_at[f])
            rev[c:c + 3] = (False, True, False)
            flags[c:c + 3] = (0x11, 0x11, 0x10)
            seq[c:c + 3] = (X + 1, Y + 1, X + 2)
            ack[c:c + 3] = (Y + 1, X + 2, Y + 2)
        if proto == synth.TCP and reopen_at and f in reopen_at:
            c = int(per * reopen_at[f])
            rev[c], flags[c], seq[c], ack[c] = False, 0x02, X + 7, 0
        cols["t"].append(t)
        cols["src"].append(np.where(rev, b, a))
        cols["dst"].append(np.where(rev, a, b))
        cols["sport"].append(np.where(rev, pb, pa))
        cols["dport"].append(np.where(rev, pa, pb))
        cols["proto"].append(np.full(per, proto))
        cols["flags"].append(np.where(proto == synth.TCP, flags, 0))
        cols["seq"].append(seq & 0xFFFFFFFF)
        cols["ack"].append(ack & 0xFFFFFFFF)
    c = {k: np.concatenate(v) for k, v in cols.items()}
    o = np.argsort(c["t"], kind="stable")
    c = {k: v[o] for k, v in c.items()}
    f = synth.build_frames(c["src"].astype(np.uint32), c["dst"].astype(np.uint32), c["proto"].astype(np.int32),
                           c["sport"], c["dport"], c["flags"].astype(np.int32), frame_len=128)
    synth.set_tcp_seq(f, c["proto"] == synth.TCP, c["seq"].astype(np.uint64), c["ack"].astype(np.uint64))
    return f


def test_long_runs_in_speculative_segments(dev):
    """Runs of thousands of packets cut every PCN_CT_SEG (512) sorted positions:
    the head wave walks to the first cut, every later segment is walked at once
    from the key's entry as the batch found it, and ct_seg_fix chains them,
    re-walking those whose guess did not hold.  Batch 1 opens the flows (no
    guess holds), batch 2 continues them under a new clock (every guess holds,
    the ttl set anew), batch 3 closes some mid-run (FIN) and reopens one (SYN),
    batch 4 adds ICMP errors quoting them and long echo replies quoting them
    (the walk stops at the first; ct_tail resumes).  Interleaved with short
    flows.  Bit-exact vs the oracle: verdicts, rule ids, counters, the table."""
    rng = np.random.default_rng(57)
    rules = CT_RULES + synth.config_rules(2).rules()
    o, ipt = ct_pair({1: rules}, {1: "ACCEPT"}, cap_log2=16, jit=1)
    ips = rng.integers(1, 2**32, size=(9, 2), dtype=np.uint64)
    flows = [(synth.TCP if k < 6 else synth.UDP, int(ips[k, 0]), int(ips[k, 1]), 1000 + k, 80 + k,
              int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))) for k in range(9)]
    short, _ = synth.flow_traffic(8000 * 4, 2000, 58, stride=128, p_icmp=0.1, p_err=0.02)
    short = short.reshape(-1, 128)
    phases = [("open", {}, {}), ("data", {}, {}), ("data", {0: 0.4, 2: 0.05, 4: 0.93}, {2: 0.7}), ("data", {}, {})]
    for k, (phase, close, reopen) in enumerate(phases):
        ipt.ct_set_time(NOW + k * 10**9)
        o.ct_set_time(NOW + k * 10**9)
        el = _elephants(rng, flows, phase, 3000, close_at=close, reopen_at=reopen)
        n = len(el) + 8000
        nb = np.empty((n, 128), np.uint8)
        slot = np.zeros(n, bool)
        slot[rng.choice(n, size=8000, replace=False)] = True
        nb[~slot] = el
        nb[slot] = short[k * 8000:(k + 1) * 8000]
        lens = np.full(n, 128, np.uint16)
        if k == 3:
            # ICMP errors quoting the long flows (their runs), and long echo
            # replies quoting them (their quoted bucket is in the batch: ct_tail)
            m = rng.choice(n, size=300, replace=False)
            err, rep = m[:250], m[250:]
            q = rng.integers(0, 9, size=300)
            qa = np.array([flows[j][1] for j in q], np.uint64)
            qb = np.array([flows[j][2] for j in q], np.uint64)
            mask = np.zeros(n, bool)
            mask[m] = True
            nb[m, 23] = 1
            nb[err, 34] = 3
            nb[rep, 34] = 0
            nb[m, 35] = 0
            isrc = np.zeros(n, np.uint64)
            idst = np.zeros(n, np.uint64)
            ipr = np.zeros(n, np.int64)
            isp = np.zeros(n, np.int64)
            idp = np.zeros(n, np.int64)
            isrc[m], idst[m] = qa, qb
            ipr[m] = [flows[j][0] for j in q]
            isp[m] = [flows[j][3] for j in q]
            idp[m] = [flows[j][4] for j in q]
            synth.set_icmp_inner(nb, mask, isrc, idst, ipr, isp, idp)
            lens[rep] = 98
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, nb.reshape(-1), n, lens=lens)
        assert_same(v_o, r_o, v_g, r_g)
        assert_tables(o, ipt)
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)


def _key_bucket(a, b, pa, pb, proto, kbits):
    """conntrack.hip key_hash % (2^kbits - 1) of a connection's ordered key
    (ConntrackLabel_dp.c:200-228: lower IP first, lower port first, each compared
    as the little-endian load of its network-order bytes), numpy u64."""
    a = a.astype(np.uint32).byteswap().astype(np.uint64)
    b = b.astype(np.uint32).byteswap().astype(np.uint64)
    pa = pa.astype(np.uint16).byteswap().astype(np.uint64)
    pb = pb.astype(np.uint16).byteswap().astype(np.uint64)
    src, dst = np.minimum(a, b), np.maximum(a, b)
    sp, dp = np.minimum(pa, pb), np.maximum(pa, pb)
    with np.errstate(over="ignore"):
        h = ((src << np.uint64(32)) | dst) * np.uint64(0x9E3779B97F4A7C15)
        h ^= ((np.uint64(proto) << np.uint64(32)) | (sp << np.uint64(16)) | dp) * np.uint64(0xC2B2AE3D27D4EB4F)
        h ^= h >> np.uint64(29)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(32)
    return h % np.uint64((1 << kbits) - 1)


def test_long_runs_of_colliding_connections(dev):
    """One key bucket holding several long connections (hash collisions): the
    head wave walks them one pass per connection (conntrack.hip PassKeys), and
    past kPassKeys (4) takes the rest as one sequence.  Buckets of 6, 3 and 2
    colliding TCP/UDP flows of 80 packets each, over three batches that open
    them, continue them and close some mid-run.  Bit-exact vs the oracle:
    verdicts, rule ids, counters, the table (and its LRU stamps' order).
    The batch (880 records) is shorter than a speculative segment cut needs
    (kSeg = 512 records on both sides), so every bucket is walked by its head
    wave in passes; the walk's pass counters say that both the per-connection
    passes and the rest-as-one-sequence walk ran."""
    rng = np.random.default_rng(61)
    rules = CT_RULES + synth.config_rules(2).rules()
    o, ipt = ct_pair({1: rules}, {1: "ACCEPT"}, cap_log2=16, jit=1)
    from polycube_amd import ffi
    per, groups = 80, (6, 3, 2)
    stats = (ctypes.c_uint64 * 2)()
    assert ffi.lib().pcn_ipt_debug_ct_walk_passes(ipt._h, stats, 1) == 0   # reset
    n = per * sum(groups)
    kbits = 8                      # conntrack.hip ct_run: 2^kbits >= n
    while (1 << kbits) < n:
        kbits += 1
    flows = []
    for g, size in enumerate(groups):
        proto = synth.TCP if g != 1 else synth.UDP
        m = 1 << 18
        a = rng.integers(1, 2**32, size=m, dtype=np.uint64)
        b = rng.integers(1, 2**32, size=m, dtype=np.uint64)
        pa = rng.integers(1024, 65535, size=m)
        pb = rng.integers(1, 1024, size=m)
        bk = _key_bucket(a, b, pa, pb, proto, kbits)
        target = np.bincount(bk.astype(np.int64)).argmax()
        pick = np.nonzero(bk == target)[0][:size]
        assert len(pick) == size
        for j in pick:
            flows.append((proto, int(a[j]), int(b[j]), int(pa[j]), int(pb[j]),
                          int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32))))
    phases = [("open", {}), ("data", {}), ("data", {0: 0.3, 4: 0.6, 9: 0.5})]
    for k, (phase, close) in enumerate(phases):
        ipt.ct_set_time(NOW + k * 10**9)
        o.ct_set_time(NOW + k * 10**9)
        f = _elephants(rng, flows, phase, per, close_at=close)
        v_o, r_o, v_g, r_g = run_ct(o, ipt, dev, f.reshape(-1), n)
        assert_same(v_o, r_o, v_g, r_g)
        assert_tables(o, ipt)
        assert ffi.lib().pcn_ipt_debug_ct_walk_passes(ipt._h, stats, 1) == 0
        # buckets of 6 / 3 / 2 connections: passes for their 2nd-4th / 2nd-3rd / 2nd, and the
        # 6-bucket's 5th and 6th as one sequence
        assert stats[0] >= 3 + 2 + 1 and stats[1] >= 1, (k, list(stats))
    assert_counters(o, ipt, n=len(rules) + 1)
    assert_ae(o, ipt)
