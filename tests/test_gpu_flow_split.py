"""Stateful conntrack sharded over N tables by flow affinity (pcn_ipt_flow_split).

The reference runs its datapath per CPU behind the NIC's RSS queue choice: the
connection table is shared, the Parser's `packet` struct is per CPU
(Iptables_Parser_dp.c:45).  Here each rank owns a connection table and the
split sends every connection's packets to one rank in batch order, so:
  - with TCP/UDP traffic the merged results equal ONE sequential oracle over
    the whole batch (verdicts, rule ids, summed counters, the union of the
    session tables);
  - with ICMP in the mix, whose keys carry the stale ports of the previous
    TCP/UDP packet on the same CPU (quirk Q4), each rank equals an oracle run
    on that rank's packets, which is the reference's per-CPU semantics.
Several contexts on one MI355X stand in for the ranks (`pytest -m gpu`)."""
import numpy as np
import pytest

from polycube_amd import synth
from test_gpu_conntrack import CT_RULES, NOW, assert_same, ct_pair, t
from test_gpu_parity import make_pair

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _fmix32(h):
    h = h.astype(np.uint64)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


def host_owner(frames, n, stride, lens, nranks, hook=0):
    """Restatement of the owner rule in include/pcn_ipt.h.  At the TC hook an
    outer 802.1Q / 802.1ad tag is stripped first (conntrack.hip flow_owner_of,
    the parse() untag): the fields move 4 bytes on and the length drops by 4."""
    f = frames.reshape(n, stride)
    L = lens.astype(np.int64) if lens is not None else np.full(n, stride, np.int64)
    et0 = (f[:, 12].astype(np.int64) << 8) | f[:, 13]
    tag = (hook == 1) & (L >= 14) & ((et0 == 0x8100) | (et0 == 0x88A8))
    short_tag = tag & (L < 18)
    shifted = np.concatenate([f[:, 4:], np.zeros((n, 4), np.uint8)], axis=1)
    f = np.where(tag[:, None], shifted, f)
    L = np.where(tag, L - 4, L)
    le32 = lambda o: f[:, o:o + 4].copy().view("<u4")[:, 0].astype(np.uint64)   # noqa: E731
    et = (f[:, 12].astype(np.int64) << 8) | f[:, 13]
    proto, icmp = f[:, 23], f[:, 34]
    ok = (L >= 34) & (et == 0x0800) & ~short_tag
    ok &= ~((proto == 6) & (L < 54)) & ~((proto == 17) & (L < 42))
    err = (proto == 1) & (L >= 70) & (icmp != 0) & (icmp != 8) & ~((icmp >= 13) & (icmp <= 18))
    a = np.where(err, le32(54), le32(26))
    c = np.where(err, le32(58), le32(30))
    lo, hi = np.minimum(a, c), np.maximum(a, c)
    h = _fmix32(_fmix32(lo ^ np.uint64(0x9E3779B9)) ^ hi)
    return np.where(ok, (h * np.uint64(nranks)) >> np.uint64(32), 0).astype(np.uint8)


def vlan_tag(frames, n, stride, lens, frac, seed):
    """Put an outer 802.1Q or 802.1ad tag on a `frac` share of the frames (as
    synth.imix_frames does): bytes 12.. move 4 on, the length grows by 4 (at
    most the stride).  A flow's packets are tagged independently, so one
    connection arrives both tagged and untagged."""
    rng = np.random.default_rng(seed)
    f = frames.reshape(n, stride).copy()
    sel = rng.random(n) < frac
    f[sel, 16:] = f[sel, 12:stride - 4]
    qinq = rng.random(int(sel.sum())) < 0.5
    f[sel, 12] = np.where(qinq, 0x88, 0x81)
    f[sel, 13] = np.where(qinq, 0xA8, 0x00)
    f[sel, 14:16] = (0x00, 0x07)
    lens = lens.copy()
    lens[sel] = np.minimum(lens[sel].astype(np.int64) + 4, stride).astype(lens.dtype)
    return f.reshape(-1), lens


@pytest.mark.parametrize("hook", [0, 1], ids=["xdp", "tc"])
def test_owner_matches_host_restatement(dev, hook):
    _, ipt = make_pair({1: []})
    n = 20000
    f, lens = synth.flow_traffic(n, 900, 11, stride=128, lens_mode="mixed", p_noise=0.2, p_err=0.1)
    f, lens = vlan_tag(f, n, 128, lens, 0.3, 5)
    for nranks in (1, 2, 3, 8):
        got = ipt.flow_owner(t(dev, f), nranks, n=n, lens=t(dev, lens, np.int16), stride=128,
                             hook=hook).cpu().numpy()
        want = host_owner(f, n, 128, lens, nranks, hook)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (nranks, bad[:5], got[bad[:5]], want[bad[:5]])
        if nranks > 1:
            assert np.bincount(got, minlength=nranks).min() > 0


@pytest.mark.parametrize("hook", [0, 1], ids=["xdp", "tc"])
def test_split_partitions_the_batch_in_order(dev, hook):
    _, ipt = make_pair({1: []})
    n = 30001
    f, lens = synth.flow_traffic(n, 2000, 4, stride=128, lens_mode="mixed", p_noise=0.2)
    ports = np.random.default_rng(1).integers(0, 4, n).astype(np.uint16)
    fd, ld, pd = t(dev, f), t(dev, lens, np.int16), t(dev, ports, np.int16)
    owner = ipt.flow_owner(fd, 3, n=n, lens=ld, stride=128, hook=hook).cpu().numpy()
    seen = []
    for r in range(3):
        idx, offs, ls, ps = (x.cpu().numpy() for x in ipt.flow_split(fd, 3, r, n=n, lens=ld, stride=128,
                                                                      in_port=pd, hook=hook))
        idx = idx.view(np.uint32)
        assert np.array_equal(idx, np.nonzero(owner == r)[0])
        assert np.array_equal(offs.view(np.uint32), idx * 128)
        assert np.array_equal(ls.view(np.uint16), lens[idx])
        assert np.array_equal(ps.view(np.uint16), ports[idx])
        seen.append(idx)
    assert np.array_equal(np.sort(np.concatenate(seen)), np.arange(n))
    # an offsets batch splits the same way (offsets carried over)
    offsets = np.arange(n, dtype=np.uint32) * 128
    idx, offs, _, _ = ipt.flow_split(fd, 3, 1, offsets=t(dev, offsets, np.int32), lens=ld, hook=hook)
    assert np.array_equal(offs.cpu().numpy().view(np.uint32), offsets[idx.cpu().numpy()])
    idx0, _, _, _ = ipt.flow_split(fd, 3, 0, n=0, stride=128)
    assert idx0.numel() == 0


def test_bad_ranks_are_refused(dev):
    """flow_args / pcn_ipt_flow_split: nranks must be 1..255 and rank < nranks
    (-EINVAL before any launch), on a context that has a device."""
    import ctypes as C
    from polycube_amd import ffi
    _, ipt = make_pair({1: []})
    f = torch.zeros(64 * 4, dtype=torch.uint8, device=dev)
    out = torch.zeros(16, dtype=torch.int32, device=dev)
    b = ffi.Batch(f.data_ptr(), f.numel(), None, None, 64, 64, None, 1, 0, 0, 0, None, 4, None, None)
    m = C.c_uint64(7)
    lib = ffi.lib()
    p = out.data_ptr()
    for nranks, rank in ((0, 0), (256, 0), (3, 3), (2, 5)):
        assert lib.pcn_ipt_flow_split(ipt._h, C.byref(b), nranks, rank, p, p, p, None, C.byref(m), None) == -22, \
            (nranks, rank)
    for nranks in (0, 256):
        assert lib.pcn_ipt_flow_owner(ipt._h, C.byref(b), nranks, p, None) == -22, nranks
    assert lib.pcn_ipt_flow_split(ipt._h, C.byref(b), 2, 1, p, p, p, None, None, None) == -22   # n_out required
    torch.cuda.synchronize()
    assert int(out.abs().sum()) == 0      # nothing was written


def _key_sorted(tab):
    return np.sort(tab, order=[x for x in ("src_ip", "dst_ip", "sport", "dport", "l4proto") if x in tab.dtype.names])


def _sharded(rules, nranks, f, lens, n, stride, dev, batches, oracle_per_rank, hook=0):
    o, _ = ct_pair({1: rules}, {1: "DROP"}, jit=1)
    cubes = [ct_pair({1: rules}, {1: "DROP"}, jit=1) for _ in range(nranks)]
    v_all = np.zeros(n, np.uint8)
    r_all = np.zeros(n, np.int32)
    v_o = np.zeros(n, np.uint8)
    r_o = np.zeros(n, np.int32)
    for lo, hi in batches:
        fb, lb = f[lo * stride:hi * stride], lens[lo:hi]
        fd, ld = t(dev, fb), t(dev, lb, np.int16)
        if not oracle_per_rank:
            v, r = o.classify(fb, n=hi - lo, lens=lb, stride=stride, fixed_len=stride, hook=hook)
            v_o[lo:hi], r_o[lo:hi] = v, r
        for rank, (orc, ipt) in enumerate(cubes):
            idx, offs, ls, ps = ipt.flow_split(fd, nranks, rank, n=hi - lo, lens=ld, stride=stride, hook=hook)
            if idx.numel() == 0:
                continue
            v, r = ipt.classify(fd, n=idx.numel(), offsets=offs, lens=ls, in_port=ps, hook=hook)
            torch.cuda.synchronize()
            gi = idx.cpu().numpy().view(np.uint32) + lo
            v_all[gi], r_all[gi] = v.cpu().numpy(), r.cpu().numpy()
            if oracle_per_rank:
                ov, orr = orc.classify(fb, offsets=offs.cpu().numpy().view(np.uint32),
                                       lens=ls.cpu().numpy().view(np.uint16), in_port=ps.cpu().numpy().view(np.uint16),
                                       hook=hook)
                v_o[gi], r_o[gi] = ov, orr
    return o, cubes, v_o, r_o, v_all, r_all


@pytest.mark.parametrize("nranks,hook", [(2, 0), (3, 0), (2, 1), (3, 1)],
                         ids=["2-xdp", "3-xdp", "2-tc-vlan", "3-tc-vlan"])
def test_sharded_tcp_udp_equals_one_sequential_table(dev, nranks, hook):
    """At the TC hook a third of the frames carry an outer VLAN tag, so one
    connection's packets arrive tagged and untagged and must meet one owner."""
    rs = synth.config_rules(2)
    rules = CT_RULES + rs.rules()
    n = 24000
    f, lens = synth.flow_traffic(n, 1500, 7, rs=rs, lens_mode="mixed", p_icmp=0.0, p_err=0.0)
    if hook == 1:
        f, lens = vlan_tag(f, n, 128, lens, 0.33, 3)
    o, cubes, v_o, r_o, v_g, r_g = _sharded(rules, nranks, f, lens, n, 128, dev,
                                            ((0, 9000), (9000, 9001), (9001, n)), False, hook)
    assert_same(v_o, r_o, v_g, r_g)
    # the union of the per-rank session tables is the single table
    union = _key_sorted(np.concatenate([ipt.ct_dump() for _, ipt in cubes]))
    want = _key_sorted(o.ct_dump())
    assert len(union) == len(want)
    for fld in want.dtype.names:
        assert np.array_equal(union[fld], want[fld]), fld
    # per-rule, default and accept-established counters sum to the single datapath's
    k = len(rules) + 1
    po, bo, dpo, dbo = o.read_counters(1, k)
    parts = [ipt.chain(1).read_counters(k) for _, ipt in cubes]
    assert np.array_equal(np.sum([np.asarray(p[0], np.uint64) for p in parts], 0), np.asarray(po, np.uint64))
    assert np.array_equal(np.sum([np.asarray(p[1], np.uint64) for p in parts], 0), np.asarray(bo, np.uint64))
    assert (sum(p[2] for p in parts), sum(p[3] for p in parts)) == (dpo, dbo)
    ae = [ipt.chain(1).read_accept_established() for _, ipt in cubes]
    assert tuple(map(sum, zip(*ae))) == tuple(o.read_accept_established(1))


def test_sharded_with_icmp_equals_per_rank_oracles(dev):
    rs = synth.config_rules(2)
    rules = CT_RULES + rs.rules()
    n = 16000
    f, lens = synth.flow_traffic(n, 800, 9, rs=rs, lens_mode="mixed", p_icmp=0.3, p_err=0.1, p_noise=0.1)
    _, cubes, v_o, r_o, v_g, r_g = _sharded(rules, 2, f, lens, n, 128, dev, ((0, 5000), (5000, n)), True)
    assert_same(v_o, r_o, v_g, r_g)
    for orc, ipt in cubes:
        a, b = _key_sorted(orc.ct_dump()), _key_sorted(ipt.ct_dump())
        assert len(a) == len(b)
        for fld in a.dtype.names:
            assert np.array_equal(a[fld], b[fld]), fld
