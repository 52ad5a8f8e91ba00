"""Scalar CPU model of the kernel's chain stage over an exported table image.

TEST INFRASTRUCTURE ONLY: it reads the bytes libpcn_ipt.so builds for the GPU
(pcn_ipt_chain_get_image) and walks them exactly as classify.hip's run_chain
does, so the image builder can be checked against the oracle without a GPU.
It is never part of the product path."""
import ctypes as C
import struct

import numpy as np

from polycube_amd import ffi

LAYOUT = ["bytes", "ip_bkt0", "ip_bkt1", "ip_shift0", "ip_shift1", "ip_steps0", "ip_steps1", "ip_win0", "ip_win1", "ip_bnd0", "ip_bnd1", "ip_cls0", "ip_cls1",
          "hash0", "hash1", "hash2", "mask0", "mask1", "mask2", "wild0", "wild1", "wild2", "skip0", "skip1",
          "slot0", "slot1", "slot2", "nslots", "proto_idx", "flags_idx", "ct_idx", "flags_skip", "meta",
          "stride_proto", "stride_flags", "stride_ct", "stride_sport", "stride_dport", "stride_iface",
          "sf", "pbase", "part", "part_wide", "part_direct", "part_dense", "pool", "zero", "perm", "wfields"]
MISS = 0xFFFF
EMPTY = 0xFFFFFFFF


class ImageModel:
    def __init__(self, chain):
        lib = ffi.lib()
        n = lib.pcn_ipt_chain_get_image(chain._h(), chain.id, None, 0, None, 0)
        buf = (C.c_uint8 * max(n, 1))()
        desc = (C.c_uint32 * 64)()
        assert lib.pcn_ipt_chain_get_image(chain._h(), chain.id, buf, n, desc, 64) == n
        self.img = bytes(buf)[:n]
        d = list(desc)
        self.lay = dict(zip(LAYOUT, d[:len(LAYOUT)]))
        self.nrw, self.nsw, self.present, self.all = d[len(LAYOUT):len(LAYOUT) + 4]

    def u16(self, off):
        return struct.unpack_from("<H", self.img, off)[0]

    def u32(self, off):
        return struct.unpack_from("<I", self.img, off)[0]

    def u64(self, off):
        return struct.unpack_from("<Q", self.img, off)[0]

    def ip_class(self, side, h):
        L = self.lay
        e = self.u32(L[f"ip_bkt{side}"] + 4 * (h >> L[f"ip_shift{side}"]))
        win = L[f"ip_win{side}"]
        if win:
            first = e & 0xFFFF
            n = sum(self.u32(L[f"ip_bnd{side}"] + 4 * (first + k)) <= h for k in range(win))
            return self.u16(L[f"ip_cls{side}"] + 2 * (first + min(n, e >> 16)))
        lo = e & 0xFFFF
        end = lo + (e >> 16)
        for k in reversed(range(L[f"ip_steps{side}"])):
            probe = lo + (1 << k)
            if probe <= end and self.u32(L[f"ip_bnd{side}"] + 4 * (probe - 1)) <= h:
                lo = probe
        return self.u16(L[f"ip_cls{side}"] + 2 * lo)

    def key_class(self, i, key):
        L = self.lay
        mask = L[f"mask{i}"]
        shift = 32 - mask.bit_length()
        h = ((key * 0x9E3779B1) & 0xFFFFFFFF) >> shift
        for e in (self.u32(L[f"hash{i}"] + 4 * h), self.u32(L[f"hash{i}"] + 4 * h + 4)):
            if e != EMPTY and e >> 16 == key:
                return e & 0xFFFF
        return L[f"wild{i}"]

    def u8(self, off):
        return self.img[off]

    def run(self, saddr_h, daddr_h, proto, sport, dport, flags, port=1, ct=0):
        """-> (rule id or -1 for default, action bit or None).  Slots as in
        classify.hip chain_classes: meta, src, dst, then own-slot key fields."""
        L, p = self.lay, self.present
        ns = L["nslots"]
        cls = [self.all] * ns
        mi = 0
        if p & 1:
            mi += self.u8(L["ct_idx"] + ct) * L["stride_ct"]
        if p & 8:
            mi += self.u8(L["proto_idx"] + proto) * L["stride_proto"]
        if p & 128:
            mi += (self.u16(L["flags_idx"] + 2 * flags) if proto == 6 else L["flags_skip"]) * L["stride_flags"]
        l4 = proto in (6, 17)
        for i, (bit, key, name) in enumerate(((16, sport, "sport"), (32, dport, "dport"), (64, port, "iface"))):
            if not p & bit:
                continue
            x = self.key_class(i, key)
            if i < 2 and not l4:
                x = L[f"skip{i}"]
            if L[f"slot{i}"] == 0:
                mi += x * L[f"stride_{name}"]
            else:
                cls[L[f"slot{i}"]] = x
        cls[0] = self.u16(L["meta"] + 2 * mi)
        if p & 2:
            cls[1] = self.ip_class(0, saddr_h)
        if p & 4:
            cls[2] = self.ip_class(1, daddr_h)
        if MISS in cls:
            return -1, None
        best = None
        for k in range(self.nsw):
            live = self.nrw - 64 * k
            m = (1 << 64) - 1 if live >= 64 else (1 << live) - 1
            recs = [c * self.nsw + k for c in cls]
            for r in recs:
                m &= self.u64(L["sf"] + 8 * r)
            while m:
                bit = (m & -m).bit_length() - 1
                m &= m - 1
                acc = (1 << 64) - 1
                if L["part_dense"]:                               # POOL index per (class, word)
                    for c in cls:
                        cell = c * self.nrw + 64 * k + bit
                        q = self.u32(L["part"] + 4 * cell) if L["part_wide"] else self.u16(L["part"] + 2 * cell)
                        acc &= self.u64(L["pool"] + 8 * q)
                    recs = []
                for r in recs:
                    part = self.u64(L["pbase"] + 16 * r)        # PM: partial words
                    if not part >> bit & 1:
                        continue                                  # FULL at this word
                    rank = bin(part & ((1 << bit) - 1)).count("1")
                    j = self.u32(L["pbase"] + 16 * r + 8) + rank
                    if L["part_direct"]:
                        acc &= self.u64(L["part"] + 8 * j)
                        continue
                    q = self.u32(L["part"] + 4 * j) if L["part_wide"] else self.u16(L["part"] + 2 * j)
                    acc &= self.u64(L["pool"] + 8 * q)
                if acc:
                    low = (acc & -acc).bit_length() - 1
                    e = self.u16(L["perm"] + 2 * ((64 * k + bit) * 63 + low))
                    best = e if best is None else min(best, e)
        if best is None:
            return -1, None
        return best >> 1, best & 1


def model_classify(model, frames, n, stride=64):
    """Rule ids for well-formed IPv4 TCP/UDP frames (fields at fixed offsets)."""
    f = np.asarray(frames, np.uint8).reshape(n, stride)
    out = np.empty(n, np.int32)
    for i in range(n):
        row = f[i]
        s = int.from_bytes(bytes(row[26:30]), "big")
        d = int.from_bytes(bytes(row[30:34]), "big")
        proto = int(row[23])
        sp = int.from_bytes(bytes(row[34:36]), "big")
        dp = int.from_bytes(bytes(row[36:38]), "big")
        fl = int(row[47]) if proto == 6 else 0
        ct = (0 if (fl & 2 and (fl | 2) == 2) else 3) if proto == 6 else 0
        out[i] = model.run(s, d, proto, sp, dp, fl, 1, ct)[0]
    return out
