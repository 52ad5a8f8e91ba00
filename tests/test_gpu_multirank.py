"""The N-rank counter exchange on one GPU.

pcn_ipt_sync_counters = snapshot (pcn_ipt_snapshot_counters) -> RCCL
all-gather -> device rank sum (pcn_ipt_sum_counter_blocks).  RCCL refuses two
ranks on one GPU, so on a one-GPU box the all-gather is what these tests leave
out: they feed the rank sum N = 2, 4, 8 blocks laid out as ncclAllGather lays
them out, and run N shard contexts on the one GPU whose blocks, summed, must
equal one unsharded oracle pass.  The reference's only reduction is the control
plane's sum over per-CPU counters (modules/ActionLookup.cpp:78-96)."""
import numpy as np
import pytest

from oracle.ffi import Oracle
from polycube_amd import dist as pdist
from polycube_amd import synth

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _cube(rules, default="DROP"):
    from polycube_amd import Iptables
    ipt = Iptables(device=0)
    ipt.interactive = False
    ch = ipt.chain("FORWARD")
    for r in rules:
        ch.append(**r)
    ch.default = default
    ch.apply_rules()
    return ipt


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_rank_sum_of_gathered_blocks(dev, nranks):
    rs = synth.config_rules(2)
    ipt = _cube(rs.rules())
    w = ipt.counter_block_words("FORWARD")
    assert w == 2 + 2 * 128
    rng = np.random.default_rng(nranks)
    blocks = rng.integers(0, 1 << 40, size=(nranks, w), dtype=np.int64)
    ipt.sum_counter_blocks("FORWARD", torch.from_numpy(blocks).to(dev))
    torch.cuda.synchronize()
    got = pdist.counter_block(*ipt.chain("FORWARD").read_counters(128, scope=1))
    assert got == pdist.sum_blocks(blocks.tolist())
    # the local (scope 0) counters are untouched by the sum
    assert ipt.chain("FORWARD").read_counters(128, scope=0) == ([0] * 128, [0] * 128, 0, 0)
    ipt.close()


def test_rank_sum_refuses_a_wrong_block_size(dev):
    from polycube_amd import IptablesError
    ipt = _cube(synth.config_rules(2).rules())
    w = ipt.counter_block_words("FORWARD")
    with pytest.raises(IptablesError) as e:
        ipt.sum_counter_blocks("FORWARD", torch.zeros((2, w + 2), dtype=torch.int64, device=dev))
    assert e.value.code == -22
    ipt.close()


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_shard_contexts_summed_equal_one_pass(dev, nranks):
    """Each shard [lo, hi) of the batch through its own context (a rank), the
    snapshots stacked rank-major and summed: verdicts, rule ids and every
    counter equal a single oracle pass over the whole batch."""
    rs = synth.config_rules(3)
    rules = rs.rules()
    n = (1 << 18) + 5          # ragged shards
    frames = np.ascontiguousarray(synth.config_frames(3, n, rs).reshape(-1))
    tf = torch.from_numpy(frames).to(dev)
    ranks = [_cube(rules) for _ in range(nranks)]
    v = torch.empty(n, dtype=torch.uint8, device=dev)
    r = torch.empty(n, dtype=torch.int32, device=dev)
    snaps = []
    for k, ipt in enumerate(ranks):
        lo, hi = pdist.shard_range(n, nranks, k)
        ipt.classify(tf[lo * 64:hi * 64], n=hi - lo, verdicts=v[lo:hi], rule_ids=r[lo:hi])
        snaps.append(ipt.snapshot_counters("FORWARD"))
    ranks[0].sum_counter_blocks("FORWARD", torch.stack(snaps))
    torch.cuda.synchronize()
    o = Oracle()
    o.set_chain(1, rules, "DROP")
    vo, ro = o.classify(frames, n=n, nthreads=8)
    assert np.array_equal(v.cpu().numpy(), vo)
    assert np.array_equal(r.cpu().numpy(), ro)
    want = o.read_counters(1, len(rules))
    assert ranks[0].chain("FORWARD").read_counters(len(rules), scope=1) == want
    # and the blocks themselves are each rank's own counters
    per = [pdist.counter_block(*ipt.chain("FORWARD").read_counters(len(rules))) for ipt in ranks]
    assert [s.cpu().tolist() for s in snaps] == per
    assert pdist.sum_blocks(per) == pdist.counter_block(*want)
    for ipt in ranks:
        ipt.close()
