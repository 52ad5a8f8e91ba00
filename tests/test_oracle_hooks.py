"""XDP vs TC attach-point semantics of the oracle (CPU only).

XDP sees the wire frame: an 802.1Q / 802.1ad-tagged frame is not IPv4 and is
passed unclassified (Iptables_Parser_dp.c:102-106).  At the TC hook the kernel
has already stripped the outer tag (skb_vlan_untag, Linux net/core/dev.c; not
in /root/reference, so this half is "parity unpinned": restated kernel
behaviour), so the inner IPv4 packet is classified and packet_len = skb->len
excludes the tag (cube_tc.cpp:374-432)."""
import numpy as np

from oracle.ffi import Oracle
from polycube_amd import synth

RULES = [{"dst": "10.1.0.0/16", "l4proto": "UDP", "dport": 53, "action": "ACCEPT"}]


def frame(dst, tags=(), length=64):
    f = synth.build_frames(np.array([0xC0000201], np.uint32), np.array([dst], np.uint32), np.array([17]),
                           np.array([4000]), np.array([53]), np.array([0]), frame_len=length).reshape(-1)
    for tpid in reversed(tags):
        f = np.concatenate([f[:12], np.array([tpid >> 8, tpid & 0xFF, 0x00, 0x05], np.uint8), f[12:]])[:length]
    return np.ascontiguousarray(f)


def run(f, hook, length=None):
    o = Oracle()
    o.set_chain(1, RULES, "DROP")
    n = 1
    L = np.array([length or len(f)], np.uint16)
    v, r = o.classify(f, n=n, offsets=np.zeros(1, np.uint32), lens=L, hook=hook)
    pk, by, dp, db = o.read_counters(1, 1)
    return int(v[0]), int(r[0]), pk[0], by[0], dp, db


def test_untagged_frames_are_the_same_at_both_hooks():
    f = frame(0x0A010203)
    assert run(f, 0) == run(f, 1) == (1, 0, 1, 64, 0, 0)


def test_tagged_frame_passes_at_xdp_and_is_classified_at_tc():
    for tpid in (0x8100, 0x88A8):
        f = frame(0x0A010203, tags=(tpid,), length=68)
        assert run(f, 0) == (1, -2, 0, 0, 0, 0)             # not IPv4 on the wire: RX_OK, no counters
        assert run(f, 1) == (1, 0, 1, 64, 0, 0)             # inner IPv4 hits rule 0; skb->len = 64


def test_tagged_miss_takes_the_default_at_tc():
    f = frame(0xC0000299, tags=(0x8100,), length=68)
    assert run(f, 0)[:2] == (1, -2)
    assert run(f, 1) == (0, -1, 0, 0, 1, 64)                # DROP default, default counters


def test_short_tagged_frame_is_dropped_by_the_untag_at_tc():
    f = frame(0x0A010203, tags=(0x8100,), length=68)
    assert run(f, 1, length=17)[:2] == (0, -2)
    assert run(f, 0, length=17)[:2] == (1, -2)


def test_only_the_outer_tag_is_stripped():
    f = frame(0x0A010203, tags=(0x88A8, 0x8100), length=72)
    assert run(f, 1)[:2] == (1, -2)                          # inner ethertype 0x8100: not IPv4
