"""World-size-2 gloo run of the multi-GPU partitioning on CPU.

Each rank classifies its contiguous shard (the oracle stands in for its GPU:
there is none here), lays its counters out as the library's block
(pcn_ipt_counter_block_words), the ranks all-gather the blocks (the RCCL
all-gather of pcn_ipt_sync_counters, here over gloo) and sum them.  The same
exchange through the library on a GPU: tests/test_gpu_multirank.py.  The result must equal a
single unsharded pass: verdicts are a pure function of each packet (no conntrack
state), so sharding by index changes nothing."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from polycube_amd import dist as pdist
from polycube_amd import synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.ffi import Oracle
    rs = synth.config_rules(2)
    rules = rs.rules()
    frames = synth.config_frames(2, n, rs)
    lo, hi = pdist.shard_range(n, world, rank)
    o = Oracle()
    o.set_chain(1, rules, "DROP")
    v, r = o.classify(frames[lo:hi].reshape(-1), n=hi - lo)
    blk = torch.tensor(pdist.counter_block(*o.read_counters(1, len(rules))), dtype=torch.int64)
    # the block has the library's layout and size (what pcn_ipt_snapshot_counters sends)
    from polycube_amd import Iptables
    ipt = Iptables(device=-1)
    ipt.interactive = False
    ch = ipt.chain("FORWARD")
    for r in rules:
        ch.append(**r)
    ch.apply_rules()
    assert blk.numel() == ipt.counter_block_words("FORWARD")
    ipt.close()
    gathered = [torch.zeros_like(blk) for _ in range(world)]
    dist.all_gather(gathered, blk)
    vs = [torch.zeros(pdist.shard_range(n, world, k)[1] - pdist.shard_range(n, world, k)[0],
                      dtype=torch.uint8) for k in range(world)]
    dist.all_gather(vs, torch.from_numpy(v)) if all(x.numel() == vs[0].numel() for x in vs) else None
    if rank == 0:
        total = pdist.sum_blocks([g.tolist() for g in gathered])
        q.put((total, torch.cat(vs).numpy().tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_counters_equal_single_pass():
    n, world = 1 << 15, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    total, vbytes = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.ffi import Oracle
    rs = synth.config_rules(2)
    rules = rs.rules()
    o = Oracle()
    o.set_chain(1, rules, "DROP")
    v, _ = o.classify(synth.config_frames(2, n, rs).reshape(-1), n=n)
    assert total == pdist.counter_block(*o.read_counters(1, len(rules)))
    assert np.frombuffer(vbytes, np.uint8).tolist() == v.tolist()


def test_shard_range_partitions():
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            spans = [pdist.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
