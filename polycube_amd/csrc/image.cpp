// image.cpp — chain tables -> HBM chain image (see devchain.h for the layout).
#include "image.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>

#include "devchain.h"

namespace pcn {
namespace {

constexpr size_t kAlign = 256;
constexpr uint32_t kTrieCapacity = 1024;   // Iptables_IpLookup_dp.c:54-55

// Vector dedup across all fields of a chain: identical bitvectors share one
// pool slot (and one summary).
class VecPool {
 public:
  explicit VecPool(uint32_t nrw) : nrw_(nrw) {}
  uint16_t intern(const BitVec &v) {
    BitVec key(v.begin(), v.begin() + nrw_);
    auto it = ids_.find(key);
    if (it != ids_.end()) return it->second;
    if (vecs_.size() >= PCN_CLS_MISS) throw std::runtime_error("too many distinct rule bitvectors");
    uint16_t id = static_cast<uint16_t>(vecs_.size());
    ids_.emplace(key, id);
    vecs_.push_back(std::move(key));
    return id;
  }
  const std::vector<BitVec> &vecs() const { return vecs_; }
 private:
  uint32_t nrw_;
  std::map<BitVec, uint16_t> ids_;
  std::vector<BitVec> vecs_;
};

struct Blob {
  std::vector<uint8_t> bytes;
  template <typename T>
  size_t add(const std::vector<T> &v) {
    size_t off = (bytes.size() + kAlign - 1) / kAlign * kAlign;
    bytes.resize(off + v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(bytes.data() + off, v.data(), v.size() * sizeof(T));
    return off;
  }
};

inline uint32_t host_order(uint32_t nbo) { return __builtin_bswap32(nbo); }
inline uint32_t prefix_mask(uint8_t len) { return len == 0 ? 0u : ~uint32_t(0) << (32 - len); }

// DIR-16-8-8 expansion.  Prefixes are painted shortest first, so a longer
// prefix always overwrites the shorter ones it nests in (= longest match).
struct DirTable {
  std::vector<uint32_t> l1 = std::vector<uint32_t>(65536, PCN_CLS_MISS);
  std::vector<uint32_t> blk;

  uint32_t push_block(uint32_t fill) {
    uint32_t id = static_cast<uint32_t>(blk.size() / 256);
    blk.insert(blk.end(), 256, fill);
    return id;
  }
  // Turn a leaf slot into a pointer to a fresh block filled with the leaf;
  // returns the block id.  (Slots are addressed by index: push_block may
  // reallocate `blk`.)
  uint32_t descend_l1(uint32_t s) {
    if (!(l1[s] & PCN_IP_PTR)) l1[s] = PCN_IP_PTR | push_block(l1[s]);
    return l1[s] & ~PCN_IP_PTR;
  }
  uint32_t descend_blk(size_t at) {
    if (!(blk[at] & PCN_IP_PTR)) {
      uint32_t id = push_block(blk[at]);
      blk[at] = PCN_IP_PTR | id;
    }
    return blk[at] & ~PCN_IP_PTR;
  }
  void paint(uint32_t prefix, uint8_t len, uint32_t cls) {
    if (len <= 16) {
      uint32_t first = prefix >> 16, count = 1u << (16 - len);
      for (uint32_t s = first; s < first + count; ++s) l1[s] = cls;
      return;
    }
    uint32_t b2 = descend_l1(prefix >> 16);
    uint32_t mid = (prefix >> 8) & 0xff;
    if (len <= 24) {
      uint32_t count = 1u << (24 - len);
      for (uint32_t j = mid; j < mid + count; ++j) blk[b2 * 256 + j] = cls;
      return;
    }
    uint32_t b3 = descend_blk(size_t(b2) * 256 + mid);
    uint32_t lo = prefix & 0xff, count = 1u << (32 - len);
    for (uint32_t k = lo; k < lo + count; ++k) blk[b3 * 256 + k] = cls;
  }
};

}  // namespace

std::vector<LpmEntry> lpm_entries(const FieldMap &m) {
  // updateMap pushes the std::map in (ip, netmask) order; the trie keeps one
  // node per (len, first len bits) and a later set replaces the value.
  std::map<std::pair<uint8_t, uint32_t>, uint32_t> trie;
  for (size_t k = 0; k < m.keys.size(); ++k) {
    uint8_t len = m.plen[k];
    trie[{len, host_order(m.keys[k]) & prefix_mask(len)}] = static_cast<uint32_t>(k);
  }
  if (trie.size() > kTrieCapacity)
    throw std::runtime_error("LPM trie full: " + std::to_string(trie.size()) + " prefixes > 1024");
  std::vector<LpmEntry> out;
  for (auto &[key, vec] : trie) out.push_back({key.first, key.second, vec});
  return out;   // sorted by (len, prefix): shortest first
}

HostImage build_image(const ChainTables &t) {
  HostImage img;
  img.nrules = t.nrules;
  img.nrw = t.nrw;
  img.nsw = (t.nrw + 63) / 64;
  img.default_action = t.default_action;
  Blob blob;
  VecPool pool(t.nrw);
  if (t.nrules > 0) {
    for (int f = 0; f < PCN_IPT_NFIELDS; ++f)
      if (t.maps[f].present()) img.present |= 1u << f;

    for (int side = 0; side < 2; ++side) {
      const FieldMap &m = t.maps[side == 0 ? PCN_IPT_F_IPSRC : PCN_IPT_F_IPDST];
      if (!m.present()) continue;
      DirTable dir;
      for (const LpmEntry &e : lpm_entries(m)) dir.paint(e.prefix, e.len, pool.intern(m.vecs[e.vec]));
      img.off_ip_l1[side] = blob.add(dir.l1);
      if (dir.blk.empty()) dir.blk.assign(256, PCN_CLS_MISS);
      img.off_ip_blk[side] = blob.add(dir.blk);
    }
    // ports (L4PortLookup.cpp:44-56 wildcard key 0) and interfaces
    // (InterfaceLookup.cpp:44-56 wildcard key 0xffff): the miss fallback is folded in.
    const int key_fields[3] = {PCN_IPT_F_SPORT, PCN_IPT_F_DPORT, PCN_IPT_F_IFACE};
    const uint32_t wild[3] = {0, 0, 0xffff};
    for (int i = 0; i < 3; ++i) {
      const FieldMap &m = t.maps[key_fields[i]];
      if (!m.present()) continue;
      std::vector<uint16_t> tab(65536, PCN_CLS_MISS);
      for (size_t k = 0; k < m.keys.size(); ++k)
        if (m.keys[k] == wild[i]) std::fill(tab.begin(), tab.end(), pool.intern(m.vecs[k]));
      for (size_t k = 0; k < m.keys.size(); ++k) tab[m.keys[k] & 0xffff] = pool.intern(m.vecs[k]);
      img.off_key[i] = blob.add(tab);
    }
    // L4ProtocolLookup_dp.c:95-103: a miss retries with key 0 (the wildcard).
    if (t.maps[PCN_IPT_F_L4PROTO].present()) {
      const FieldMap &m = t.maps[PCN_IPT_F_L4PROTO];
      std::vector<uint16_t> tab(256, PCN_CLS_MISS);
      for (size_t k = 0; k < m.keys.size(); ++k)
        if (m.keys[k] == 0) std::fill(tab.begin(), tab.end(), pool.intern(m.vecs[k]));
      for (size_t k = 0; k < m.keys.size(); ++k) tab[m.keys[k] & 0xff] = pool.intern(m.vecs[k]);
      img.off_proto = blob.add(tab);
    }
    if (t.maps[PCN_IPT_F_TCPFLAGS].present()) {
      const FieldMap &m = t.maps[PCN_IPT_F_TCPFLAGS];
      std::vector<uint16_t> tab(256, PCN_CLS_MISS);
      for (size_t k = 0; k < m.keys.size(); ++k) tab[m.keys[k] & 0xff] = pool.intern(m.vecs[k]);
      img.off_flags = blob.add(tab);
    }
    if (t.maps[PCN_IPT_F_CONNTRACK].present()) {
      const FieldMap &m = t.maps[PCN_IPT_F_CONNTRACK];
      std::vector<uint16_t> tab(4, PCN_CLS_MISS);
      for (size_t k = 0; k < m.keys.size() && k < 4; ++k) tab[m.keys[k] & 3] = pool.intern(m.vecs[k]);
      img.off_ct = blob.add(tab);
    }
    const auto &vecs = pool.vecs();
    img.nvec = static_cast<uint32_t>(vecs.size());
    std::vector<uint64_t> flat, summ;
    flat.reserve(size_t(img.nvec) * t.nrw);
    summ.assign(size_t(img.nvec) * img.nsw, 0);
    for (uint32_t v = 0; v < img.nvec; ++v) {
      for (uint32_t w = 0; w < t.nrw; ++w) {
        flat.push_back(vecs[v][w]);
        if (vecs[v][w]) summ[size_t(v) * img.nsw + w / 64] |= uint64_t(1) << (w % 64);
      }
    }
    if (flat.empty()) flat.push_back(0);
    if (summ.empty()) summ.push_back(0);
    img.off_pool = blob.add(flat);
    img.off_summ = blob.add(summ);
  }
  std::vector<uint8_t> actions(t.actions);
  if (actions.empty()) actions.push_back(0);
  img.off_actions = blob.add(actions);
  img.blob = std::move(blob.bytes);
  return img;
}

}  // namespace pcn
