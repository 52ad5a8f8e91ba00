// image.hpp — lowers compiled chain tables (ruleset.hpp) into the chain image
// consumed by the classify kernel (devchain.h).
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "devchain.h"
#include "ruleset.hpp"

namespace pcn {

struct HostImage {
  std::vector<uint8_t> tables;   // table image (TableLayout offsets)
  TableLayout lay{};
  uint32_t nrules = 0, nrw = 0, nsw = 0, present = 0, nvec = 0, ngroups = 0, all_cls = 0;
  uint32_t part_words = 0;       // partial (neither zero nor full) vector words
  uint32_t pool_words = 0;       // distinct partial words stored
  uint64_t part_bytes = 0;       // PART indices + POOL bytes
  uint32_t meta_entries = 0;     // proto x flags x conntrack (x iface) table size
  int default_action = 1;
};

// A table the reference's BPF map could not hold: its map push fails with
// ENOSPC ("Table set error: No space left on device", libs/polycube/src/
// table.cpp:61-66) at the verb that runs Chain::updateChain.  The C ABI
// returns -ENOSPC for it.
struct TableFull : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Throws TableFull (> 1024 LPM entries per field — the kernel trie capacity of
// Iptables_IpLookup_dp.c:54-55) or std::runtime_error (> 65534 distinct vectors).
HostImage build_image(const ChainTables &t);

// Kernel-LPM view of an IP map (what the BPF trie holds after updateMap):
// one entry per (len, masked prefix), the last pushed value winning.
struct LpmEntry { uint8_t len; uint32_t prefix; uint32_t vec; };
std::vector<LpmEntry> lpm_entries(const FieldMap &m);

// The LPM function as disjoint intervals: class[j] holds on [bnd[j-1], bnd[j])
// (bnd[-1] = 0, bnd[m] = 2^32); class = index into m.vecs or -1 (miss).
struct Intervals { std::vector<uint32_t> bnd; std::vector<int32_t> cls; };
Intervals lpm_intervals(const FieldMap &m);

}  // namespace pcn
