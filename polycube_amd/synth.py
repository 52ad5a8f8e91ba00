"""Seeded synthetic rule chains and packet streams for the BASELINE.json configs.

Rule sets are lists of REST-style dicts (the body of
POST /polycube/v1/iptables/<cube>/chain/<CHAIN>/append/, iptables.yang:221-230).
Packets are L2 frames laid out exactly as the reference Parser reads them
(Iptables_Parser_dp.c:94-153): Ethernet 14 B + IPv4 20 B (IHL 5) + TCP 20 B /
UDP 8 B, zero payload.  Everything is vectorised numpy so 2^24 frames build in
seconds; no network data is used (there is none on the box).
"""
import numpy as np

TCP, UDP, ICMP, GRE = 6, 17, 1, 47
_PROTO_NAME = {TCP: "TCP", UDP: "UDP", ICMP: "ICMP", GRE: "GRE"}
_FLAG_BITS = ["FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR"]

CONFIG_SEEDS = {1: 0x5EED0016, 2: 0x5EED0128, 3: 0x5EED1000, 5: 0x5EED10000}


def ip_str(host_order):
    h = int(host_order)
    return f"{(h >> 24) & 255}.{(h >> 16) & 255}.{(h >> 8) & 255}.{h & 255}"


def ip_nbo(host_order):
    """NBO bytes read as a little-endian u32 (how the reference stores IPs)."""
    h = int(host_order)
    return int.from_bytes(h.to_bytes(4, "big"), "little")


class RuleSet:
    """Column form of a generated chain (for packet synthesis) + REST dicts."""

    def __init__(self, n):
        self.n = n
        self.src = np.zeros(n, np.uint32)
        self.src_len = np.full(n, -1, np.int32)
        self.dst = np.zeros(n, np.uint32)
        self.dst_len = np.full(n, -1, np.int32)
        self.proto = np.zeros(n, np.int32)      # 0 = unset
        self.sport = np.full(n, -1, np.int32)
        self.dport = np.full(n, -1, np.int32)
        self.fset = np.zeros(n, np.int32)       # tcpflags set mask (-1 unset)
        self.fnot = np.zeros(n, np.int32)
        self.has_flags = np.zeros(n, bool)
        self.action = np.zeros(n, np.int32)

    def rules(self):
        out = []
        for i in range(self.n):
            r = {"action": "ACCEPT" if self.action[i] else "DROP"}
            if self.src_len[i] >= 0:
                r["src"] = f"{ip_str(self.src[i])}/{self.src_len[i]}"
            if self.dst_len[i] >= 0:
                r["dst"] = f"{ip_str(self.dst[i])}/{self.dst_len[i]}"
            if self.proto[i]:
                r["l4proto"] = _PROTO_NAME[int(self.proto[i])]
            if self.sport[i] >= 0:
                r["sport"] = int(self.sport[i])
            if self.dport[i] >= 0:
                r["dport"] = int(self.dport[i])
            if self.has_flags[i]:
                toks = [_FLAG_BITS[b] for b in range(8) if self.fset[i] >> b & 1]
                toks += ["!" + _FLAG_BITS[b] for b in range(8) if self.fnot[i] >> b & 1]
                r["tcpflags"] = " ".join(toks)
            out.append(r)
        return out


def _prefix_pool(rng, count, lens, aligned=True):
    lens = rng.choice(lens, size=count)
    base = rng.integers(0, 2**32, size=count, dtype=np.uint64).astype(np.uint32)
    if aligned:
        sh = (32 - np.clip(lens, 1, 32)).astype(np.uint64)
        mask = np.where(lens == 0, np.uint64(0), (np.uint64(0xFFFFFFFF) << sh) & np.uint64(0xFFFFFFFF))
        base = (base.astype(np.uint64) & mask).astype(np.uint32)
    return base, lens.astype(np.int32)


def make_rules(n, seed, *, p_src=0.5, p_dst=0.7, protos=(TCP, UDP), p_proto=0.8, p_dport=0.6,
               p_sport=0.1, p_flags=0.1, prefix_lens=(8, 16, 16, 24, 24, 24, 32, 32), aligned=True,
               pool_size=None, port_pool=64, min_prefix=16):
    """The SURVEY.md §8d rule mix: prefixes /8 /16 /24 /32 (octet aligned),
    proto in {TCP, UDP, unset}, dport from a 64-value pool or unset, sport
    mostly unset, a few tcpflags rules, action 50/50.  Distinct prefixes per
    field stay <= 1023 (the 1024-entry LPM trie)."""
    rng = np.random.default_rng(seed)
    rs = RuleSet(n)
    pool_size = pool_size or min(1000, max(8, n // 2))
    sp, sl = _prefix_pool(rng, pool_size, prefix_lens, aligned)
    dp, dl = _prefix_pool(rng, pool_size, prefix_lens, aligned)
    ports = rng.integers(1, 65536, size=port_pool)
    pick = rng.integers(0, pool_size, size=n)
    use = rng.random(n) < p_src
    rs.src = np.where(use, sp[pick], 0).astype(np.uint32)
    rs.src_len = np.where(use, sl[pick], -1).astype(np.int32)
    pick = rng.integers(0, pool_size, size=n)
    use = rng.random(n) < p_dst
    rs.dst = np.where(use, dp[pick], 0).astype(np.uint32)
    rs.dst_len = np.where(use, dl[pick], -1).astype(np.int32)
    # every rule pins at least one address prefix of /16 or longer, so uniform
    # random traffic mostly falls through to the default action
    none = (rs.src_len < 0) & (rs.dst_len < 0)
    rs.dst = np.where(none, dp[pick], rs.dst).astype(np.uint32)
    rs.dst_len = np.where(none, dl[pick], rs.dst_len).astype(np.int32)
    if min_prefix:
        for a, ln in ((rs.src, rs.src_len), (rs.dst, rs.dst_len)):
            short = (ln >= 0) & (ln < min_prefix)
            other = rs.dst_len if ln is rs.src_len else rs.src_len
            grow = short & ((other < 0) | (other < min_prefix))
            ln[grow] = min_prefix
    use = rng.random(n) < p_proto
    rs.proto = np.where(use, rng.choice(np.array(protos), size=n), 0).astype(np.int32)
    l4 = (rs.proto == TCP) | (rs.proto == UDP) | (rs.proto == 0)
    rs.dport = np.where(l4 & (rng.random(n) < p_dport), rng.choice(ports, size=n), -1).astype(np.int32)
    rs.sport = np.where(l4 & (rng.random(n) < p_sport), rng.choice(ports, size=n), -1).astype(np.int32)
    rs.has_flags = (rs.proto == TCP) & (rng.random(n) < p_flags)
    fl_choices = np.array([[0x02, 0x10], [0x10, 0x00], [0x02, 0x00], [0x01, 0x00], [0x04, 0x00], [0x12, 0x00]])
    fc = fl_choices[rng.integers(0, len(fl_choices), size=n)]
    rs.fset = np.where(rs.has_flags, fc[:, 0], 0).astype(np.int32)
    rs.fnot = np.where(rs.has_flags, fc[:, 1], 0).astype(np.int32)
    rs.action = rng.integers(0, 2, size=n).astype(np.int32)
    return rs


def config_rules(cfg, seed=None):
    seed = CONFIG_SEEDS.get(cfg, 0) if seed is None else seed
    if cfg == 1:
        return make_rules(16, seed, protos=(UDP,), pool_size=16)
    if cfg == 2:
        return make_rules(128, seed, protos=(UDP,))
    if cfg == 3:
        return make_rules(1000, seed)
    if cfg == 5:
        return make_rules(10000, seed, pool_size=480)
    raise ValueError(cfg)


def _be16(col):
    return np.stack([(col >> 8) & 255, col & 255], axis=1).astype(np.uint8)


def _be32(col):
    col = col.astype(np.uint64)
    return np.stack([(col >> 24) & 255, (col >> 16) & 255, (col >> 8) & 255, col & 255],
                    axis=1).astype(np.uint8)


def build_frames(src, dst, proto, sport, dport, flags, frame_len=64, ethertype=0x0800, out=None,
                 icmp_type=None):
    """Write n frames of `frame_len` bytes (stride frame_len) into a new/out array."""
    n = len(src)
    f = np.zeros((n, frame_len), np.uint8) if out is None else out
    f[:, 0:6] = (0x02, 0x00, 0x00, 0x00, 0x00, 0x02)
    f[:, 6:12] = (0x02, 0x00, 0x00, 0x00, 0x00, 0x01)
    f[:, 12:14] = _be16(np.full(n, ethertype, np.int64) if np.isscalar(ethertype) else ethertype)
    f[:, 14] = 0x45
    f[:, 16:18] = _be16(np.full(n, frame_len - 14, np.int64))
    f[:, 20] = 0x40
    f[:, 22] = 64
    f[:, 23] = proto
    f[:, 26:30] = _be32(src)
    f[:, 30:34] = _be32(dst)
    f[:, 34:36] = _be16(sport)
    f[:, 36:38] = _be16(dport)
    tcp = proto == TCP
    f[tcp, 46] = 0x50
    f[:, 47] = np.where(tcp, flags, f[:, 47])
    udp = proto == UDP
    f[udp, 38:40] = _be16(np.full(int(udp.sum()), frame_len - 34, np.int64))
    if icmp_type is not None:
        ic = proto == ICMP
        f[ic, 34] = icmp_type[ic]
        f[ic, 35] = 0
    return f


def make_headers(rs, n, seed, *, hit_frac=0.5, protos=(TCP, UDP)):
    """Header columns: `hit_frac` built from a random rule's fields, the rest uniform."""
    rng = np.random.default_rng(seed ^ 0xA5A5)
    nh = int(n * hit_frac)
    src = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    proto = rng.choice(np.array(protos), size=n).astype(np.int32)
    sport = rng.integers(1024, 65536, size=n).astype(np.int32)
    dport = rng.integers(1, 65536, size=n).astype(np.int32)
    flags = rng.integers(0, 256, size=n).astype(np.int32)
    if nh and rs is not None and rs.n:
        r = rng.integers(0, rs.n, size=nh)

        def fill(col, val, ln):
            ln = ln[r]
            m = ln >= 0
            sh = (32 - np.clip(ln, 1, 32)).astype(np.uint64)
            mask = np.where(ln <= 0, np.uint64(0), (np.uint64(0xFFFFFFFF) << sh) & np.uint64(0xFFFFFFFF))
            cur = col[:nh].astype(np.uint64)
            v = (val[r].astype(np.uint64) & mask) | (cur & ~mask & np.uint64(0xFFFFFFFF))
            col[:nh] = np.where(m, v, cur).astype(np.uint32)
        fill(src, rs.src, rs.src_len)
        fill(dst, rs.dst, rs.dst_len)
        rp = rs.proto[r]
        proto[:nh] = np.where(rp > 0, rp, proto[:nh])
        sport[:nh] = np.where(rs.sport[r] >= 0, rs.sport[r], sport[:nh])
        dport[:nh] = np.where(rs.dport[r] >= 0, rs.dport[r], dport[:nh])
        fl = flags[:nh]
        fl = np.where(rs.has_flags[r], (fl | rs.fset[r]) & ~rs.fnot[r] & 0xFF, fl)
        flags[:nh] = fl
        perm = rng.permutation(n)
        src, dst, proto, sport, dport, flags = (a[perm] for a in (src, dst, proto, sport, dport, flags))
    return src, dst, proto, sport, dport, flags


def config_frames(cfg, n, rs=None, seed=None):
    """Fixed 64-byte frames for configs 1-3 (UDP for 1/2, 50/50 TCP/UDP for 3)."""
    seed = CONFIG_SEEDS.get(cfg, 0) if seed is None else seed
    protos = (UDP,) if cfg in (1, 2) else (TCP, UDP)
    cols = make_headers(rs, n, seed, protos=protos)
    return build_frames(*cols, frame_len=64)


def spread_frames(frames64, n, stride, out=None, fix_lengths=True):
    """Fixed-size frames of `stride` bytes (>= 64) on the device from n 64-byte
    frames (a uint8 torch tensor of n*64 bytes, on the device): each frame's first
    64 bytes copied to i*stride, the rest zero (payload).  fix_lengths rewrites the
    IPv4 total length (and, for UDP, the UDP length) of untagged IPv4 frames for
    a frame of `stride` bytes.  `out` (>= n*stride bytes) is reused when given.
    The frame-size sweep's layout (bench.py frame_sizes, tests): the classify
    kernel reads only a frame's first 48-52 bytes (Iptables_Parser_dp.c:126-143),
    so a larger frame changes the access pattern, not what is read."""
    import torch
    if stride < 64:
        raise ValueError("stride must be >= 64")
    buf = (torch.empty(n * stride, dtype=torch.uint8, device=frames64.device) if out is None
           else out[: n * stride])
    v = buf.view(n, stride)
    if stride > 64:
        v[:, 64:].zero_()
    src = frames64[: n * 64].view(n, 64)
    v[:, :64] = src
    if fix_lengths:
        ipv4 = (src[:, 12] == 8) & (src[:, 13] == 0)
        tot, ul = stride - 14, stride - 34

        def put16(col, val, mask):
            v[:, col] = torch.where(mask, torch.full_like(src[:, col], (val >> 8) & 255), src[:, col])
            v[:, col + 1] = torch.where(mask, torch.full_like(src[:, col], val & 255), src[:, col + 1])
        put16(16, tot, ipv4)
        put16(38, ul, ipv4 & (src[:, 23] == UDP))
    return buf


def imix_frames(rs, n, seed, *, vlan_frac=0.3, ipv6_frac=0.3, align=1):
    """Config 5: IMIX 7:4:1 of 64/576/1500-byte frames packed back to back, with
    802.1Q-tagged and IPv6 frames mixed in.  align=64 starts every frame at a
    64-byte boundary instead (how NIC RX buffers place them); the frames and
    their lengths are the same.  Returns (buffer, offsets, lens)."""
    rng = np.random.default_rng(seed ^ 0x1111)
    sizes = rng.choice(np.array([64, 576, 1500]), p=[7 / 12, 4 / 12, 1 / 12], size=n).astype(np.int64)
    slots = (sizes + align - 1) // align * align
    offsets = np.zeros(n, np.int64)
    offsets[1:] = np.cumsum(slots)[:-1]
    total = int(slots.sum())
    buf = np.zeros(total + 64, np.uint8)
    cols = make_headers(rs, n, seed)
    hdr = build_frames(*cols, frame_len=64)
    kind = rng.random(n)
    vlan = kind < vlan_frac
    ipv6 = (kind >= vlan_frac) & (kind < vlan_frac + ipv6_frac)
    hdr[vlan, 16:64] = hdr[vlan, 12:60]           # insert a 4-byte 802.1Q tag
    hdr[vlan, 12:14] = (0x81, 0x00)
    hdr[vlan, 14:16] = (0x00, 0x05)
    hdr[ipv6, 12:14] = (0x86, 0xDD)
    hdr[ipv6, 14] = 0x60
    idx = offsets[:, None] + np.arange(64)[None, :]
    buf[idx] = hdr
    if total > 2**32 - 1:
        raise ValueError("IMIX buffer exceeds 32-bit offsets")
    return buf, offsets.astype(np.uint32), sizes.astype(np.uint16)


def fuzz_frames(n, seed, rs=None, stride=96):
    """Edge-case frames: every length 0..stride, random/odd ethertypes, ICMP types,
    GRE, short TCP/UDP/ICMP headers; in_port and lens returned alongside."""
    rng = np.random.default_rng(seed)
    src, dst, proto, sport, dport, flags = make_headers(rs, n, seed, protos=(TCP, UDP, ICMP, GRE, 0, 99))
    icmp_type = rng.choice(np.array([0, 3, 5, 8, 11, 13, 14, 15, 16, 17, 18, 30]), size=n)
    et = rng.choice(np.array([0x0800, 0x0800, 0x0800, 0x0800, 0x86DD, 0x8100, 0x0806, 0x0008]), size=n)
    f = build_frames(src, dst, proto, sport, dport, flags, frame_len=stride, ethertype=et,
                     icmp_type=icmp_type)
    lens = rng.integers(0, stride + 1, size=n)
    common = rng.random(n) < 0.5
    lens = np.where(common, rng.choice(np.array([13, 14, 33, 34, 41, 42, 53, 54, 61, 62, 69, 70, 64, 96]), size=n),
                    lens).astype(np.uint16)
    return f, lens


# ---------------------------------------------------------------------------
# Stateful traffic (conntrack): flows with handshakes, replies and ICMP errors
# ---------------------------------------------------------------------------

def set_tcp_seq(frames, mask, seq, ack):
    """TCP sequence/ack numbers (host order in, network order in the frame)."""
    f = frames.reshape(len(mask), -1)
    f[mask, 38:42] = _be32(np.asarray(seq, np.uint64)[mask])
    f[mask, 42:46] = _be32(np.asarray(ack, np.uint64)[mask])


def set_icmp_inner(frames, mask, isrc, idst, iproto, isport, idport):
    """The offending IP header + 8 payload bytes an ICMP error carries at byte 42
    (what ConntrackLabel_dp.c:491-529 reads)."""
    f = frames.reshape(len(mask), -1)
    m = np.asarray(mask)
    f[m, 42] = 0x45
    f[m, 50] = 64
    f[m, 51] = np.asarray(iproto)[m]
    f[m, 54:58] = _be32(np.asarray(isrc, np.uint64)[m])
    f[m, 58:62] = _be32(np.asarray(idst, np.uint64)[m])
    f[m, 62:64] = _be16(np.asarray(isport, np.int64)[m])
    f[m, 64:66] = _be16(np.asarray(idport, np.int64)[m])


def flow_traffic(n, nflows, seed, *, stride=128, rs=None, hit_frac=0.5, p_noise=0.05, p_icmp=0.1,
                 p_err=0.02, lens_mode="fixed"):
    """n frames from `nflows` interleaved connections, in packet-arrival order.

    TCP flows run SYN, SYN-ACK, ACK, data, FIN-ACK, FIN-ACK, ACK with consistent
    sequence numbers; UDP flows alternate directions; ICMP flows are echo
    request/reply pairs.  A `p_noise` fraction of packets get random flags or a
    swapped direction (INVALID paths), and `p_err` are ICMP errors quoting
    another flow's header (RELATED lookups).  A `hit_frac` share of the flows
    take their endpoints from a rule of `rs` so the chain's rules are exercised.
    Returns (frames [n*stride], lens u16 or None)."""
    rng = np.random.default_rng(seed)
    nflows = max(1, min(nflows, n))
    src, dst, proto, sport, dport, _ = make_headers(rs, nflows, seed, hit_frac=hit_frac)
    kind = rng.random(nflows)
    proto = np.where(kind < p_icmp, ICMP, proto).astype(np.int32)
    # packets per flow: a multinomial split of n
    per = rng.multinomial(n, np.full(nflows, 1.0 / nflows))
    fid = np.repeat(np.arange(nflows), per)
    pos = np.arange(n) - np.repeat(np.cumsum(per) - per, per)      # index inside the flow
    last = np.repeat(per, per) - 1
    # arrival order: each flow starts at a random time and spreads its packets out
    t0 = rng.random(nflows)[fid]
    span = (rng.random(nflows) * 0.5 + 0.05)[fid]
    t = t0 + span * (pos + rng.random(n) * 0.5) / np.maximum(last + 1, 1)
    order = np.argsort(t, kind="stable")
    fid, pos, last = fid[order], pos[order], last[order]
    p = proto[fid]
    # direction: TCP script, UDP/ICMP alternate
    tcp_dir = np.select([pos == 0, pos == 1, pos == 2, pos == last - 1], [0, 1, 0, 1], pos % 2)
    tcp_dir = np.where((pos == last) & (last >= 5), 0, tcp_dir)
    rev = np.where(p == TCP, tcp_dir, pos % 2).astype(bool)
    swap = rng.random(n) < p_noise
    rev ^= swap
    a_ip, b_ip = src[fid], dst[fid]
    a_pt, b_pt = sport[fid], dport[fid]
    s_ip = np.where(rev, b_ip, a_ip).astype(np.uint32)
    d_ip = np.where(rev, a_ip, b_ip).astype(np.uint32)
    s_pt = np.where(rev, b_pt, a_pt)
    d_pt = np.where(rev, a_pt, b_pt)
    # TCP flags and sequence numbers (client X, server Y)
    X = rng.integers(0, 2**32, size=nflows, dtype=np.uint64)[fid]
    Y = rng.integers(0, 2**32, size=nflows, dtype=np.uint64)[fid]
    M = np.uint64(0xFFFFFFFF)
    fin_c = (pos == last - 2) & (last >= 5)
    fin_s = (pos == last - 1) & (last >= 5)
    ack_l = (pos == last) & (last >= 5)
    flags = np.select([pos == 0, pos == 1, fin_c | fin_s], [0x02, 0x12, 0x11], 0x10)
    flags = np.where((~(pos <= 2)) & (~fin_c) & (~fin_s) & (~ack_l) & (rng.random(n) < 0.3), 0x18, flags)
    seq = np.select([pos == 0, pos == 1, fin_s, ack_l], [X, Y, (Y + 1) & M, (X + 2) & M],
                    np.where(rev, (Y + 1) & M, (X + 1) & M))
    ack = np.select([pos == 0, pos == 1, fin_s, ack_l], [np.zeros_like(X), (X + 1) & M, (X + 2) & M, (Y + 2) & M],
                    np.where(rev, (X + 1) & M, (Y + 1) & M))
    noisy = rng.random(n) < p_noise
    flags = np.where(noisy, rng.integers(0, 256, size=n), flags).astype(np.int32)
    # ICMP: echo request / reply; some packets become errors quoting another flow
    itype = np.where(rev, 0, 8)
    err = rng.random(n) < p_err
    p = np.where(err, ICMP, p).astype(np.int32)
    itype = np.where(err, rng.choice(np.array([3, 11, 5, 13]), size=n), itype)
    f = build_frames(s_ip, d_ip, p, s_pt, d_pt, flags, frame_len=stride, icmp_type=itype)
    tcp = p == TCP
    set_tcp_seq(f, tcp, seq, ack)
    if stride >= 66:
        q = rng.integers(0, nflows, size=n)      # the quoted flow (its forward direction)
        qrev = rng.random(n) < 0.5
        set_icmp_inner(f, err, np.where(qrev, dst[q], src[q]), np.where(qrev, src[q], dst[q]), proto[q],
                       np.where(qrev, dport[q], sport[q]), np.where(qrev, sport[q], dport[q]))
    lens = None
    if lens_mode == "mixed":
        lens = np.where(rng.random(n) < 0.2, rng.choice(np.array([41, 42, 54, 61, 62, 69, 70, 98]), size=n),
                        stride).astype(np.uint16)
    return f.reshape(-1), lens
