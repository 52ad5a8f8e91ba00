// devchain.h — device-side layout of one compiled chain ("chain image") and the
// classify launch arguments.  Shared by the host image builder and the HIP kernel.
//
// The reference keeps one BPF map per field module (LPM trie / hash / array of
// 1,048-byte bitvectors, Iptables_*Lookup_dp.c) and walks them with ~12 tail
// calls per packet.  Here a chain is one contiguous HBM blob:
//   * IP fields: DIR-16-8-8 tables (u32 entries) giving the kernel-LPM answer
//     for any /32 key (longest prefix, same-prefix last-writer-wins);
//   * port / interface fields: direct 65,536-entry u16 class tables with the
//     wildcard fallback (key 0 / 0xffff) already folded in;
//   * proto / tcp-flags / conntrack: 256/256/4-entry u16 class tables;
//   * a deduplicated bitvector pool [nvec][nrw] (63 rule bits per word) plus a
//     per-vector summary [nvec][nsw] (bit w set iff word w != 0).
// A class id of PCN_CLS_MISS means "lookup miss with no wildcard" => default.
#pragma once
#include <cstdint>

#define PCN_CLS_MISS 0xFFFFu
#define PCN_IP_PTR 0x80000000u
#define PCN_MAX_LOCALIP 256

namespace pcn {

struct DevChain {
  const uint32_t *ip_l1[2];      // [0]=src [1]=dst: 65536 entries, index = host-order ip >> 16
  const uint32_t *ip_blk[2];     // 256-entry blocks for /17../32
  const uint16_t *key_cls[3];    // [0]=sport [1]=dport [2]=iface, 65536 entries each
  const uint16_t *proto_cls;     // 256
  const uint16_t *flags_cls;     // 256
  const uint16_t *ct_cls;        // 4
  const uint64_t *pool;          // [nvec][nrw]
  const uint64_t *summ;          // [nvec][nsw]
  const uint8_t *actions;        // [nrules] 0 DROP / 1 ACCEPT
  unsigned long long *ctr;       // [2 + 2*ncounted]: def_pkts, def_bytes, pkts0, bytes0, ...
  uint32_t nrules, nrw, nsw, present;
  uint32_t ncounted, max_action;
  int32_t default_action;
  int32_t lds_base;              // first LDS bin of this chain's rules; -1 => global atomics
};

struct LaunchArgs {
  DevChain ch[3];
  const uint8_t *frames;
  uint64_t frames_bytes;
  const uint32_t *offsets;
  const uint16_t *lens;
  const uint16_t *in_port;
  const uint8_t *ct_status;
  uint8_t *verdicts;
  int32_t *rule_ids;
  const uint32_t *localip;       // sorted NBO u32
  uint64_t n;
  uint32_t stride, fixed_len;
  uint32_t nlocal;
  uint32_t nbins;                // LDS bins (3 default bins + rule bins)
  uint16_t const_in_port;
  uint16_t direction;
  uint32_t allow_logic;          // _INGRESS_ALLOWLOGIC (modules/ChainSelector.cpp:190-202)
};

}  // namespace pcn
