"""pcn-firewall on the GPU: the same kernel behind the firewall personality, checked
against the oracle's firewall mode (verdicts, rule ids, per-rule and default
counters) and against the reference's own firewall tests (fw_scenarios.json)."""
import os

import numpy as np
import pytest

from helpers import GpuFwCube, OracleFwCube, load_fw_scenarios
from oracle.ffi import Oracle
from polycube_amd import synth
from rulegen import quirky_rules

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
NTHREADS = min(16, os.cpu_count() or 1)
JIT = pytest.mark.parametrize("jit", [-1, 1], ids=["generic", "chainprog"])
SCEN = load_fw_scenarios()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@JIT
@pytest.mark.parametrize("sc", SCEN["scenarios"], ids=[s["name"] for s in SCEN["scenarios"]])
def test_reference_firewall_scenarios_on_gpu(dev, sc, jit):
    """Replay every script: the GPU takes each packet's label from the oracle's
    connection table (batch.ct_status) and must give the oracle's verdicts, the
    script's outcome and the same counters."""
    from polycube_amd import Firewall
    ocube = OracleFwCube(Oracle())
    gcube = GpuFwCube(Firewall(device=0, jit=jit))
    for k, st in enumerate(sc["steps"]):
        where = f"{sc['name']} step {k} ({st.get('ref_line', '')})"
        for op in st["ops"]:
            ocube.op(op)
            gcube.op(op)
        assert gcube.fw.conntrack_mode == ocube.mode, where
        if "probe" in st:
            v_o, labels = ocube.probe(st["probe"])
            v_g, _ = gcube.probe(st["probe"], labels)
            assert v_g == v_o, f"{where}: oracle {v_o} gpu {v_g}"
            got = "pass" if all(v == 1 for v in v_g) else "fail"
            assert got == st["expect"], where
        for c, n in st.get("nrules", {}).items():
            assert len(gcube.fw.chain(c)) == n, where
        for c in ("INGRESS", "EGRESS"):
            assert gcube.chain_stats(c) == ocube.chain_stats(c), f"{where}: {c} stats"


def make_fw_pair(rules_by_chain, defaults, mode, jit):
    from polycube_amd import Firewall
    o = Oracle()
    o.set_service(1, mode)
    fw = Firewall(device=0, jit=jit)
    if mode == 0:
        fw.conntrack = "OFF"
    elif mode == 1:
        fw.accept_established = "OFF"
    fw.interactive = False
    for name, slot in (("INGRESS", 1), ("EGRESS", 2)):
        rules = rules_by_chain.get(name, [])
        o.set_chain(slot, rules, defaults[name])
        ch = fw.chain(name)
        for r in rules:
            ch.append(**r)
        ch.default = defaults[name]
        ch.apply_rules()
    return o, fw


@JIT
@pytest.mark.parametrize("mode", [0, 1, 2], ids=["ct_off", "manual", "automatic"])
@pytest.mark.parametrize("seed", range(3))
def test_firewall_fuzz_parity(dev, seed, mode, jit):
    """Quirky rules (no interface fields; conntrack matches only with conntrack
    on), edge-case frames, both directions, labels supplied or not."""
    rng = np.random.default_rng(100 + seed)
    rules = {}
    for k, name in enumerate(("INGRESS", "EGRESS")):
        rs = quirky_rules(int(rng.integers(0, 200)), 1000 + seed * 10 + k, ifaces=False, ct=mode != 0)
        for r in rs:
            r.setdefault("action", "DROP")
        rules[name] = rs
    if seed == 1:
        rules["EGRESS"] = []                  # empty chain: DefaultAction + its counters
    defaults = {"INGRESS": "DROP" if seed % 2 else "ACCEPT", "EGRESS": "ACCEPT" if seed % 2 else "DROP"}
    o, fw = make_fw_pair(rules, defaults, mode, jit)
    n = 1 << 15
    frames, lens = synth.fuzz_frames(n, 200 + seed, synth.make_rules(64, seed, protos=(6, 17, 1)), stride=96)
    for direction in (0, 1):
        for ct in (None, rng.integers(0, 5, size=n).astype(np.uint8)):
            v_o, r_o = o.classify(frames.reshape(-1), n=n, lens=lens, stride=96, direction=direction,
                                  ct_status=ct, nthreads=NTHREADS)
            v_g, r_g = fw.classify(torch.from_numpy(frames.reshape(-1)).to(dev), n=n,
                                   lens=torch.from_numpy(lens.view(np.int16)).to(dev), stride=96,
                                   direction=direction,
                                   ct_status=None if ct is None else torch.from_numpy(ct).to(dev))
            torch.cuda.synchronize()
            v_g, r_g = v_g.cpu().numpy(), r_g.cpu().numpy()
            bad = np.nonzero((v_o != v_g) | (r_o != r_g))[0]
            assert bad.size == 0, (f"dir {direction} ct {ct is not None}: {bad.size} mismatches at {bad[:5]}: "
                                   f"oracle {v_o[bad[:5]]}/{r_o[bad[:5]]} gpu {v_g[bad[:5]]}/{r_g[bad[:5]]}")
            if mode == 2 and ct is not None:
                assert np.any(r_g == -3)       # AUTOMATIC accepted some ESTABLISHED packets
    for name, slot in (("INGRESS", 1), ("EGRESS", 2)):
        po, bo, dpo, dbo = o.read_counters(slot, 8000)
        pg, bg, dpg, dbg = fw.chain(name).read_counters(8000)
        assert (dpo, dbo) == (dpg, dbg) and po == pg and bo == bg, name


def test_firewall_headline_shape_fixed_stride(dev):
    """The headline workload (config 3 rules, 64-byte frames, fixed stride, chain
    program) through the firewall INGRESS chain equals the oracle."""
    rs = synth.config_rules(3)
    rules = [dict(r, action=r.get("action", "DROP")) for r in rs.rules()]
    o, fw = make_fw_pair({"INGRESS": rules}, {"INGRESS": "DROP", "EGRESS": "ACCEPT"}, 0, 1)
    n = 1 << 20
    frames = synth.config_frames(3, n, rs).reshape(-1)
    v_o, r_o = o.classify(frames, n=n, stride=64, fixed_len=64, nthreads=NTHREADS)
    v_g, r_g = fw.classify(torch.from_numpy(frames).to(dev), n=n)
    torch.cuda.synchronize()
    assert np.array_equal(v_o, v_g.cpu().numpy()) and np.array_equal(r_o, r_g.cpu().numpy())
    assert fw.jit_info()["launches_jit"] > 0
    po, bo, dpo, dbo = o.read_counters(1, 1000)
    pg, bg, dpg, dbg = fw.chain("INGRESS").read_counters(1000)
    assert (po, bo, dpo, dbo) == (pg, bg, dpg, dbg)


# ---- stateful: the connection table on the GPU (conntrack.hip) ----
NOW = 1_700_000_000_123_456_789


def assert_tables(o, fw):
    a, b = o.ct_dump(), fw.ct_dump()
    assert len(a) == len(b), (len(a), len(b))
    for f in a.dtype.names:
        bad = np.nonzero(a[f] != b[f])[0]
        assert bad.size == 0, f"session table field {f}: {bad.size} differ"


@pytest.mark.parametrize("sc", SCEN["scenarios"], ids=[s["name"] for s in SCEN["scenarios"]])
def test_reference_firewall_scenarios_stateful_gpu(dev, sc):
    """The scripts again, now labelled from the GPU's own connection table
    (pcn_ipt_ct_enable): verdicts, outcomes, counters and the session table
    equal the oracle's."""
    from polycube_amd import Firewall
    ocube = OracleFwCube(Oracle())
    fw = Firewall(device=0, jit=1)
    fw.ct_enable(16)
    ocube.o.ct_set_time(NOW)
    fw.ct_set_time(NOW)
    gcube = GpuFwCube(fw)
    for k, st in enumerate(sc["steps"]):
        where = f"{sc['name']} step {k} ({st.get('ref_line', '')})"
        for op in st["ops"]:
            ocube.op(op)
            gcube.op(op)
        if "probe" in st:
            v_o, _ = ocube.probe(st["probe"])
            v_g, _ = gcube.probe(st["probe"], None)
            assert v_g == v_o, f"{where}: oracle {v_o} gpu {v_g}"
            got = "pass" if all(v == 1 for v in v_g) else "fail"
            assert got == st["expect"], where
        for c in ("INGRESS", "EGRESS"):
            assert gcube.chain_stats(c) == ocube.chain_stats(c), f"{where}: {c} stats"
        assert_tables(ocube.o, fw)


CT_RULES = [{"conntrack": "ESTABLISHED", "action": "ACCEPT"}, {"conntrack": "NEW", "l4proto": "TCP", "action": "ACCEPT"},
            {"conntrack": "INVALID", "action": "DROP"}]


@pytest.mark.parametrize("mode", [1, 2], ids=["manual", "automatic"])
def test_firewall_stateful_flow_parity(dev, mode):
    """Interleaved flows (handshakes, replies, ICMP errors quoting live flows,
    noise) through INGRESS and EGRESS in several batches; conntrack rules in
    INGRESS; the table carried across batches and directions."""
    rs = synth.config_rules(2)
    base = [dict(r, action=r.get("action", "DROP")) for r in rs.rules()]
    o, fw = make_fw_pair({"INGRESS": CT_RULES + base, "EGRESS": base[:40]},
                         {"INGRESS": "DROP", "EGRESS": "ACCEPT"}, mode, 1)
    o.ct_enable()
    o.ct_set_time(NOW)
    fw.ct_enable(16)
    fw.ct_set_time(NOW)
    n = 24000
    f, lens = synth.flow_traffic(n, 900, 11 + mode, rs=rs, lens_mode="mixed", p_noise=0.1, p_err=0.05)
    nb = f.reshape(n, 128)
    for k, (lo, hi) in enumerate(((0, 6000), (6000, 6001), (6001, 15000), (15000, 24000))):
        direction = k % 2
        fr = np.ascontiguousarray(nb[lo:hi]).reshape(-1)
        v_o, r_o = o.classify(fr, n=hi - lo, lens=lens[lo:hi], stride=128, fixed_len=128, direction=direction)
        v_g, r_g = fw.classify(torch.from_numpy(fr).to(dev), n=hi - lo,
                               lens=torch.from_numpy(lens[lo:hi].view(np.int16)).to(dev), stride=128,
                               fixed_len=128, direction=direction)
        torch.cuda.synchronize()
        v_g, r_g = v_g.cpu().numpy(), r_g.cpu().numpy()
        bad = np.nonzero((v_o != v_g) | (r_o != r_g))[0]
        assert bad.size == 0, f"batch {k}: {bad.size} mismatches at {bad[:5]}"
        if mode == 2 and k > 0:
            assert np.any(r_g == -3)
    assert_tables(o, fw)
    for name, slot, nr in (("INGRESS", 1, len(base) + 3), ("EGRESS", 2, 40)):
        po, bo, dpo, dbo = o.read_counters(slot, nr)
        pg, bg, dpg, dbg = fw.chain(name).read_counters(nr)
        assert (po, bo, dpo, dbo) == (pg, bg, dpg, dbg), name
    assert fw.ct_info()["inserts_lost"] == 0
