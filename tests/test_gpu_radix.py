"""The stateful pipeline's hand-written sort (polycube_amd/csrc/radix.hip) on its
own: keys sorted stably with their batch indices, against numpy's stable
argsort, across sub-tile and super-tile boundaries (8192 keys a sub-tile, one
super-tile per CU), 1-4 digit passes and batches where one "hot" bucket
(packets that need no table) dominates.  The
conntrack tests exercise it inside the pipeline, batch after batch."""
import ctypes as C

import numpy as np
import pytest

from polycube_amd import ffi

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ipt():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from polycube_amd import Iptables
    x = Iptables(device=0)
    yield x
    x.close()


def _sort(ipt, keys, kbits):
    dev = torch.device("cuda", 0)
    k = torch.from_numpy(keys.view(np.int32)).to(dev)
    ko = torch.empty_like(k)
    io = torch.empty_like(k)
    rc = ffi.lib().pcn_ipt_debug_sort_pairs(ipt._h, C.c_void_p(k.data_ptr()), len(keys), kbits,
                                           C.c_void_p(ko.data_ptr()), C.c_void_p(io.data_ptr()))
    assert rc == 0, ffi.last_error()
    assert torch.equal(k, torch.from_numpy(keys.view(np.int32)).to(dev))     # input left as it was
    return ko.cpu().numpy().view(np.uint32), io.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,kbits,hot", [
    (1, 8, 0.0), (5, 9, 0.0), (8191, 13, 0.3), (8192, 18, 0.0), (8193, 18, 0.5), (100_003, 25, 0.6),
    ((1 << 20) + 7, 25, 0.4), (300_000, 27, 0.0), (70_000, 32, 0.1), (1 << 22, 25, 0.9)])
def test_radix_sort_is_a_stable_sort(ipt, n, kbits, hot):
    rng = np.random.default_rng(n ^ kbits)
    top = (1 << kbits) - 1
    keys = rng.integers(0, top + 1, size=n, dtype=np.uint64).astype(np.uint32)
    keys[rng.random(n) < hot] = top                   # the sentinel bucket
    if n > 1000:
        keys[: n // 50] = keys[n // 50]               # a long run of one key
    ko, io = _sort(ipt, keys, kbits)
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(io, order.astype(np.uint32))
    assert np.array_equal(ko, keys[order])


def test_radix_sort_refuses_bad_arguments(ipt):
    from polycube_amd import IptablesError  # noqa: F401
    k = np.zeros(4, np.uint32)
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(k.view(np.int32)).to(dev)
    rc = ffi.lib().pcn_ipt_debug_sort_pairs(ipt._h, C.c_void_p(t.data_ptr()), 4, 0, C.c_void_p(t.data_ptr()),
                                           C.c_void_p(t.data_ptr()))
    assert rc == -22
