// ruleset.hpp — host rule model and LBVS rule compiler for the pcn-iptables
// classification path (product code; no dependency on oracle/).
//
// Rule model:    ChainRule (services/pcn-iptables/src/ChainRule.cpp:29-83, ChainRule.h:127-154)
// Compiler:      Chain::*FromRulesToMap (Utils.cpp:223-732) as driven by
//                Chain::updateChain (Chain.cpp:600-874)
// Output:        per-field {key -> rule bitvector} maps, 63 rule bits per u64
//                word (defines.h:165-168), exactly what updateChain pushes with
//                RawTable::set, plus the action table.
#pragma once
#include <cstdint>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "pcn_ipt.h"

namespace pcn {

constexpr uint32_t kBitsPerWord = 63;                       // defines.h:168
inline uint32_t words_for_rules(uint32_t n) { return (n + kBitsPerWord - 1) / kBitsPerWord; }

struct IpPrefix {                                           // defines.h:84-114 IpAddr
  uint32_t ip = 0;       // network byte order bytes read as a little-endian u32
  uint8_t len = 32;
  bool operator<(const IpPrefix &o) const { return ip != o.ip ? ip < o.ip : len < o.len; }
  bool operator==(const IpPrefix &o) const { return ip == o.ip && len == o.len; }
  static IpPrefix parse(const std::string &s);              // throws std::runtime_error
};

// Ports known to the cube: name -> polycube port index (Iptables::interfaceNameToIndex).
class PortTable {
 public:
  void add(const std::string &name, uint16_t index) { idx_[name] = index; }
  std::optional<uint16_t> find(const std::string &name) const {
    auto it = idx_.find(name);
    if (it == idx_.end()) return std::nullopt;
    return it->second;
  }
 private:
  std::map<std::string, uint16_t> idx_;
};

struct TcpFlagsMask { uint8_t set = 0, not_set = 0; };

struct Rule {
  std::optional<IpPrefix> src, dst;
  std::optional<uint8_t> l4proto;
  std::optional<uint16_t> sport, dport;
  std::optional<TcpFlagsMask> tcpflags;
  std::optional<std::string> in_iface, out_iface;
  std::optional<uint8_t> conntrack;                         // 0 NEW .. 3 INVALID
  uint8_t action = PCN_IPT_DROP;

  // ChainRule::update semantics (throws std::runtime_error on invalid input).
  static Rule from_c(const pcn_ipt_rule &r, const PortTable &ports);
  // ChainRule::equal (used by Chain::deletes)
  bool operator==(const Rule &o) const;
};

uint8_t protocol_from_string(const std::string &p);        // Utils.cpp:45-57
TcpFlagsMask flags_from_string(const std::string &flags);  // Utils.cpp:73-140

using BitVec = std::vector<uint64_t>;

struct FieldMap {
  std::vector<uint32_t> keys;
  std::vector<uint8_t> plen;   // IP fields only
  std::vector<BitVec> vecs;
  bool present() const { return !keys.empty(); }
};

struct ChainTables {
  uint32_t nrules = 0;
  uint32_t nrw = 0;            // NR_ELEMENTS = ceil(nrules / 63)
  int default_action = PCN_IPT_ACCEPT;
  std::vector<uint8_t> actions;
  FieldMap maps[PCN_IPT_NFIELDS];
};

// Chain::updateChain's compile step for one chain.
ChainTables compile_chain(const std::vector<Rule> &rules, int chain, int default_action,
                          const PortTable &ports);

}  // namespace pcn
