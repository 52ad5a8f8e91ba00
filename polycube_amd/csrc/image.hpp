// image.hpp — lowers compiled chain tables (ruleset.hpp) into the HBM chain
// image consumed by the classify kernel (devchain.h).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "ruleset.hpp"

namespace pcn {

constexpr size_t kNoSection = ~size_t(0);

struct HostImage {
  std::vector<uint8_t> blob;     // all sections, 256-byte aligned
  size_t off_ip_l1[2] = {kNoSection, kNoSection};
  size_t off_ip_blk[2] = {kNoSection, kNoSection};
  size_t off_key[3] = {kNoSection, kNoSection, kNoSection};
  size_t off_proto = kNoSection, off_flags = kNoSection, off_ct = kNoSection;
  size_t off_pool = kNoSection, off_summ = kNoSection, off_actions = kNoSection;
  uint32_t nrules = 0, nrw = 0, nsw = 0, present = 0, nvec = 0;
  int default_action = 1;
};

// Throws std::runtime_error (e.g. ENOSPC-style: > 1024 LPM entries per field,
// the kernel trie capacity of Iptables_IpLookup_dp.c:54-55; or > 65534 vectors).
HostImage build_image(const ChainTables &t);

// Kernel-LPM view of an IP map (what the BPF trie holds after updateMap):
// (prefix len, host-order masked prefix) -> vector index into t.maps[f].vecs.
struct LpmEntry { uint8_t len; uint32_t prefix; uint32_t vec; };
std::vector<LpmEntry> lpm_entries(const FieldMap &m);

}  // namespace pcn
