// image.cpp — chain tables -> chain image (see devchain.h for the layout).
#include "image.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <set>
#include <stdexcept>
#include <string>

namespace pcn {
namespace {

constexpr size_t kAlign = 16;
constexpr uint32_t kTrieCapacity = 1024;   // Iptables_IpLookup_dp.c:54-55
constexpr size_t kGroupAlignMin = 8;       // densest packing: smaller type groups share words
constexpr uint32_t kHashMul = 0x9E3779B1u;
constexpr size_t kMetaMaxEntries = 8192;   // key fields join the meta slot while its table stays this small
constexpr size_t kMetaMaxClasses = 1024;   // ... and holds at most this many distinct vectors
constexpr size_t kDirectMaxBytes = 96 * 1024;
// Dense PART: when the image with records and indexed PART exceeds the LDS of
// a CU (it is then read from L2 in part anyway), up to 4 MiB of L2 (one XCD's)
constexpr size_t kDenseMinBytes = 160 * 1024;
constexpr size_t kDenseMaxBytes = 4 * 1024 * 1024;
constexpr uint32_t kIpWindowMax = 4;           // IP buckets read whole up to this many boundaries

// Measurement knob (tools/ablate.py experiments): PCN_IPT_DEBUG_COMPACT=1
// builds the smallest image (indexed partial words, searched IP buckets of at
// most 2^10) to try two workgroups per CU.
bool compact_images() {
  static const bool v = std::getenv("PCN_IPT_DEBUG_COMPACT") != nullptr;
  return v;
}
// ... PCN_IPT_DEBUG_IPSEARCH=1: searched IP buckets only; PCN_IPT_DEBUG_JOIN=m:
// join exactly the key fields in mask m (1 sport, 2 dport, 4 iface) to META.
bool ip_search_only() {
  static const bool v = std::getenv("PCN_IPT_DEBUG_IPSEARCH") != nullptr;
  return v;
}
// PCN_IPT_DEBUG_IP_BITS=b: IP bucket tables of at most 2^b entries (A/B).
uint32_t ip_bits_max() {
  static const uint32_t v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_IP_BITS");
    const long b = e ? std::strtol(e, nullptr, 10) : 0;
    return b >= 4 && b <= PCN_IP_BUCKET_BITS_MAX ? static_cast<uint32_t>(b) : uint32_t(PCN_IP_BUCKET_BITS_MAX);
  }();
  return v;
}
// PCN_IPT_DEBUG_CLUSTER=0: pack a type group's rules into words in rule-id
// order (A/B of the value clustering in make_permutation)
bool cluster_rules() {
  static const bool v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_CLUSTER");
    return !(e && *e == '0');
  }();
  return v;
}
int forced_join() {
  static const int v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_JOIN");
    return e ? std::atoi(e) : -1;
  }();
  return v;
}   // images up to this size store partial words directly

inline uint32_t host_order(uint32_t nbo) { return __builtin_bswap32(nbo); }
inline uint32_t prefix_mask(uint8_t len) { return len == 0 ? 0u : ~uint32_t(0) << (32 - len); }
inline bool test_bit(const BitVec &v, uint32_t id) { return (v[id / kBitsPerWord] >> (id % kBitsPerWord)) & 1; }

struct Blob {
  std::vector<uint8_t> bytes;
  template <typename T>
  uint32_t add(const std::vector<T> &v) {
    size_t off = (bytes.size() + kAlign - 1) / kAlign * kAlign;
    bytes.resize(off + std::max<size_t>(v.size() * sizeof(T), kAlign));
    if (!v.empty()) std::memcpy(bytes.data() + off, v.data(), v.size() * sizeof(T));
    return static_cast<uint32_t>(off);
  }
};

// Rule -> bit position permutation.  Rules are ordered by the set of fields
// they constrain (their "type"), larger type groups start on a fresh 63-bit
// word, and each word lists its rules in ascending id.
struct Permutation {
  uint32_t nrw = 0;
  std::vector<uint32_t> pos;        // rule id -> bit position
  std::vector<uint16_t> perm;       // bit position -> id << 1 | action (PCN pad: 0xFFFF)
  std::vector<uint64_t> valid;      // per word: bits holding a rule
  uint32_t ngroups = 0;
};

Permutation make_permutation(const ChainTables &t, const std::vector<std::vector<const BitVec *>> &field_vecs) {
  const uint32_t n = t.nrules;
  std::vector<uint32_t> type(n, 0);
  for (int f = 0; f < PCN_IPT_NFIELDS; ++f) {
    const auto &vs = field_vecs[f];
    if (vs.empty()) continue;
    BitVec all(t.nrw, ~uint64_t(0));
    for (const BitVec *v : vs)
      for (uint32_t w = 0; w < t.nrw; ++w) all[w] &= (*v)[w];
    for (uint32_t r = 0; r < n; ++r)
      if (!test_bit(all, r)) type[r] |= 1u << f;   // r is not a wildcard in field f
  }
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  // Inside a type group the rules that share a word are free to choose (a
  // word keeps its bits in ascending rule id, and the packet's rule is the
  // minimum over its matching words): rules with equal field values are put
  // next to each other, so a word's rules agree on their values and a field's
  // summary bits are set for few words of a class -- fewer candidate words
  // whose fields each match some rule of the word but no rule all of them.
  // A rule's value in field f is the first map entry whose vector holds it
  // (its own key; for IP fields its own prefix, the shortest entry holding it).
  std::vector<std::vector<uint32_t>> first(PCN_IPT_NFIELDS);
  const int cluster_order[] = {PCN_IPT_F_DPORT, PCN_IPT_F_IPDST, PCN_IPT_F_IPSRC, PCN_IPT_F_L4PROTO,
                               PCN_IPT_F_SPORT, PCN_IPT_F_TCPFLAGS, PCN_IPT_F_IFACE, PCN_IPT_F_CONNTRACK};
  if (cluster_rules()) {
    for (int f : cluster_order) {
      const auto &vs = field_vecs[f];
      if (vs.empty()) continue;
      first[f].assign(n, ~0u);
      for (size_t e = 0; e < vs.size(); ++e)
        for (uint32_t w = 0; w < t.nrw && w < vs[e]->size(); ++w) {
          uint64_t bits = (*vs[e])[w];
          while (bits) {
            const uint32_t r = w * kBitsPerWord + static_cast<uint32_t>(__builtin_ctzll(bits));
            bits &= bits - 1;
            if (r < n && first[f][r] == ~0u) first[f][r] = static_cast<uint32_t>(e);
          }
        }
    }
  }
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    if (type[a] != type[b]) return type[a] < type[b];
    for (int f : cluster_order) {
      if (first[f].empty()) continue;
      if (first[f][a] != first[f][b]) return first[f][a] < first[f][b];
    }
    return false;
  });
  std::map<uint32_t, size_t> group_size;
  for (uint32_t r = 0; r < n; ++r) group_size[type[r]]++;
  // Pack type groups into words.  A word mixing types can pass every field's
  // summary with no rule matching (rule A wild in src, rule B wild in dst...),
  // so each group gets words of its own unless that costs an extra 64-word
  // summary block; then groups smaller than `min_own` share words.
  auto pack = [&](size_t min_own) {
    std::vector<std::vector<uint32_t>> ws;
    uint32_t cur_type = ~0u;
    for (uint32_t r : order) {
      bool fresh = ws.empty() || ws.back().size() == kBitsPerWord;
      if (type[r] != cur_type) {
        cur_type = type[r];
        if (group_size[cur_type] >= min_own) fresh = true;
      }
      if (fresh) ws.emplace_back();
      ws.back().push_back(r);
    }
    return ws;
  };
  std::vector<std::vector<uint32_t>> words = pack(kGroupAlignMin);
  const size_t blocks = (words.size() + 63) / 64;
  for (size_t min_own : {size_t(1), size_t(2), size_t(4)}) {
    auto ws = pack(min_own);
    if ((ws.size() + 63) / 64 <= blocks) { words = std::move(ws); break; }
  }
  for (auto &w : words) std::sort(w.begin(), w.end());
  Permutation p;
  p.ngroups = static_cast<uint32_t>(group_size.size());
  p.nrw = static_cast<uint32_t>(words.size());
  p.pos.assign(n, 0);
  p.perm.assign(size_t(p.nrw) * kBitsPerWord, 0xFFFF);
  p.valid.assign(p.nrw, 0);
  for (uint32_t w = 0; w < p.nrw; ++w) {
    for (uint32_t j = 0; j < words[w].size(); ++j) {
      uint32_t r = words[w][j];
      uint32_t bit = w * kBitsPerWord + j;
      p.pos[r] = bit;
      p.perm[bit] = static_cast<uint16_t>((r << 1) | (t.actions[r] ? 1u : 0u));
      p.valid[w] |= uint64_t(1) << j;
    }
  }
  return p;
}

class VecPool {
 public:
  VecPool(const Permutation &p, uint32_t n) : p_(p), n_(n) {}
  uint16_t intern(const BitVec &orig) {
    BitVec v(p_.nrw, 0);
    for (uint32_t w = 0; w * kBitsPerWord < n_ && w < orig.size(); ++w) {
      uint64_t bits = orig[w];
      while (bits) {
        uint32_t r = w * kBitsPerWord + static_cast<uint32_t>(__builtin_ctzll(bits));
        bits &= bits - 1;
        if (r < n_) { uint32_t q = p_.pos[r]; v[q / kBitsPerWord] |= uint64_t(1) << (q % kBitsPerWord); }
      }
    }
    auto it = ids_.find(v);
    if (it != ids_.end()) return it->second;
    if (vecs_.size() >= PCN_CLS_MISS) throw std::runtime_error("too many distinct rule bitvectors");
    uint16_t id = static_cast<uint16_t>(vecs_.size());
    ids_.emplace(v, id);
    vecs_.push_back(std::move(v));
    return id;
  }
  const std::vector<BitVec> &vecs() const { return vecs_; }
 private:
  const Permutation &p_;
  uint32_t n_;
  std::map<BitVec, uint16_t> ids_;
  std::vector<BitVec> vecs_;
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
    throw TableFull("LPM trie full: " + std::to_string(trie.size()) +
                    " prefixes > 1024 (Table set error: No space left on device)");
  std::vector<LpmEntry> out;
  for (auto &[key, vec] : trie) out.push_back({key.first, key.second, vec});
  return out;   // sorted by (len, prefix): shortest first
}

Intervals lpm_intervals(const FieldMap &m) {
  std::vector<LpmEntry> es = lpm_entries(m);
  std::vector<uint64_t> pts{0};
  for (const LpmEntry &e : es) {
    uint64_t lo = e.prefix, hi = uint64_t(e.prefix) + (uint64_t(1) << (32 - e.len));
    pts.push_back(lo);
    if (hi <= 0xFFFFFFFFull) pts.push_back(hi);
  }
  std::sort(pts.begin(), pts.end());
  pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
  Intervals iv;
  for (uint64_t s : pts) {
    // longest prefix covering s (entries are sorted by length: keep the last hit)
    int32_t cls = -1;
    for (const LpmEntry &e : es)
      if ((uint32_t(s) & prefix_mask(e.len)) == e.prefix) cls = static_cast<int32_t>(e.vec);
    if (!iv.cls.empty() && iv.cls.back() == cls) continue;
    if (s != 0) iv.bnd.push_back(static_cast<uint32_t>(s));
    iv.cls.push_back(cls);
  }
  return iv;
}

namespace {

// One image; key field i joins the meta slot when bit i of `join` is set and
// the meta table stays within kMetaMaxEntries entries / kMetaMaxClasses
// distinct vectors.
HostImage build_image_with(const ChainTables &t, uint32_t join) {
  HostImage img;
  img.nrules = t.nrules;
  img.default_action = t.default_action;
  Blob blob;
  TableLayout &lay = img.lay;
  std::memset(&lay, 0, sizeof lay);
  for (int i = 0; i < 3; ++i) lay.hash_wild[i] = PCN_CLS_MISS;

  if (t.nrules == 0) {
    img.nrw = img.nsw = 0;
    blob.add(std::vector<uint32_t>(4, 0));
    lay.bytes = static_cast<uint32_t>(blob.bytes.size());
    img.tables = std::move(blob.bytes);
    return img;
  }
  for (int f = 0; f < PCN_IPT_NFIELDS; ++f)
    if (t.maps[f].present()) img.present |= 1u << f;

  // the classes each slot can hold (wfields below): 0 meta, 1/2 IP, 3.. own-slot key fields
  std::vector<std::set<uint32_t>> slot_cls(6);
  // vectors visible to the datapath, per field (IP: after the trie collapse)
  std::vector<LpmEntry> lpm[2];
  std::vector<std::vector<const BitVec *>> field_vecs(PCN_IPT_NFIELDS);
  for (int f = 0; f < PCN_IPT_NFIELDS; ++f) {
    const FieldMap &m = t.maps[f];
    if (!m.present()) continue;
    if (f == PCN_IPT_F_IPSRC || f == PCN_IPT_F_IPDST) {
      auto &es = lpm[f - PCN_IPT_F_IPSRC];
      es = lpm_entries(m);
      for (const LpmEntry &e : es) field_vecs[f].push_back(&m.vecs[e.vec]);
    } else {
      for (const BitVec &v : m.vecs) field_vecs[f].push_back(&v);
    }
  }
  Permutation perm = make_permutation(t, field_vecs);
  img.nrw = perm.nrw;
  img.nsw = (perm.nrw + 63) / 64;
  img.ngroups = perm.ngroups;
  VecPool pool(perm, t.nrules);

  // IP fields: interval tables
  for (int side = 0; side < 2; ++side) {
    const FieldMap &m = t.maps[PCN_IPT_F_IPSRC + side];
    if (!m.present()) continue;
    Intervals iv = lpm_intervals(m);
    std::vector<uint16_t> cls;
    for (int32_t c : iv.cls) cls.push_back(c < 0 ? PCN_CLS_MISS : pool.intern(m.vecs[c]));
    slot_cls[1 + side].insert(cls.begin(), cls.end());
    // Bucket entry (count << 16) | first: the boundaries inside the bucket
    // are bnd[first, first + count).  The kernel runs a branchless upper-bound
    // search of ip_steps[side] steps (a wave-uniform trip count), so the bucket
    // count is the smallest 2^4..2^12 keeping every bucket at <= 3 boundaries
    // (2 steps), else <= 7 (3 steps), else 2^12.
    if (iv.bnd.size() > 0x7FFF) throw std::runtime_error("too many LPM intervals");
    auto first_of = [&](uint32_t bits) {
      const uint32_t nb = 1u << bits;
      std::vector<uint32_t> first(nb + 1);
      for (uint32_t b = 0; b <= nb; ++b) {
        uint64_t start = uint64_t(b) << (32 - bits);
        first[b] = static_cast<uint32_t>(std::lower_bound(iv.bnd.begin(), iv.bnd.end(), start) - iv.bnd.begin());
      }
      return first;
    };
    auto max_count = [](const std::vector<uint32_t> &first) {
      uint32_t mc = 0;
      for (size_t b = 0; b + 1 < first.size(); ++b) mc = std::max(mc, first[b + 1] - first[b]);
      return mc;
    };
    // Window mode first: when some 2^4..2^12 buckets keep every bucket at <=
    // kIpWindowMax boundaries, the kernel reads them all at once and counts
    // (one dependent read instead of a search).  A prefix's two boundaries
    // usually share a bucket, so this is the common case.
    uint32_t bits = 0, win = 0;
    const uint32_t max_bits = compact_images() ? 10 : ip_bits_max();
    for (uint32_t b = 4; b <= max_bits && !bits && !compact_images() && !ip_search_only(); ++b)
      if (max_count(first_of(b)) <= kIpWindowMax) bits = b;
    if (bits) {
      win = std::max(1u, max_count(first_of(bits)));
    } else {
      for (uint32_t limit : {3u, 7u}) {
        for (uint32_t b = 4; b <= max_bits && !bits; ++b)
          if (max_count(first_of(b)) <= limit) bits = b;
        if (bits) break;
      }
    }
    if (!bits) bits = max_bits;
    const std::vector<uint32_t> first = first_of(bits);
    uint32_t steps = 0;
    while ((1u << steps) - 1 < max_count(first)) ++steps;
    if (win) {   // padding: window reads past the last boundary see values no address exceeds
      steps = 0;
      iv.bnd.insert(iv.bnd.end(), win, 0xFFFFFFFFu);
    }
    const uint32_t nb = 1u << bits;
    std::vector<uint32_t> bkt(nb);
    for (uint32_t b = 0; b < nb; ++b) bkt[b] = ((first[b + 1] - first[b]) << 16) | first[b];
    lay.ip_shift[side] = 32 - bits;
    lay.ip_steps[side] = steps;
    lay.ip_win[side] = win;
    lay.ip_bkt[side] = blob.add(bkt);
    lay.ip_bnd[side] = blob.add(iv.bnd);
    lay.ip_cls[side] = blob.add(cls);
  }
  // the all-ones vector: fields a packet skips (or the chain lacks)
  BitVec ones(t.nrw, 0);
  for (uint32_t r = 0; r < t.nrules; ++r) ones[r / kBitsPerWord] |= uint64_t(1) << (r % kBitsPerWord);
  img.all_cls = pool.intern(ones);

  // ---- the meta slot ----
  // proto, tcpflags and conntrack always, and each of sport / dport / iface
  // while the table stays small: every such field maps its packet value to an
  // index into its list of distinct vectors (nullptr = no entry: the packet
  // takes the default action), and the meta table holds the class of their
  // AND.  Fewer slots mean fewer summary and partial-word reads per packet,
  // and the summary of an AND is tighter than the AND of summaries.  A key
  // field that does not join keeps a slot of its own and its hash holds
  // classes.
  struct Small {
    std::vector<const BitVec *> vecs;
    uint32_t index(const BitVec *v) {
      for (size_t k = 0; k < vecs.size(); ++k)
        if (vecs[k] == v || (v && vecs[k] && *vecs[k] == *v)) return static_cast<uint32_t>(k);
      vecs.push_back(v);
      return static_cast<uint32_t>(vecs.size() - 1);
    }
  };
  Small P, F, Cn;
  std::vector<uint8_t> pidx(256, 0), cidx(4, 0);
  std::vector<uint16_t> fidx(256, 0);   // up to 256 distinct flag vectors + the skip entry
  // L4ProtocolLookup_dp.c:95-103: a miss retries with key 0 (the wildcard).
  if (t.maps[PCN_IPT_F_L4PROTO].present()) {
    const FieldMap &m = t.maps[PCN_IPT_F_L4PROTO];
    std::vector<const BitVec *> by(256, nullptr);
    for (size_t k = 0; k < m.keys.size(); ++k)
      if (m.keys[k] == 0) std::fill(by.begin(), by.end(), &m.vecs[k]);
    for (size_t k = 0; k < m.keys.size(); ++k) by[m.keys[k] & 0xff] = &m.vecs[k];
    for (int v = 0; v < 256; ++v) pidx[v] = static_cast<uint8_t>(P.index(by[v]));
  } else {
    P.index(&ones);
  }
  // TcpFlagsLookup_dp.c:93-97: skipped (all rules pass) unless the packet is TCP
  if (t.maps[PCN_IPT_F_TCPFLAGS].present()) {
    const FieldMap &m = t.maps[PCN_IPT_F_TCPFLAGS];
    std::vector<const BitVec *> by(256, nullptr);
    for (size_t k = 0; k < m.keys.size(); ++k) by[m.keys[k] & 0xff] = &m.vecs[k];
    for (int v = 0; v < 256; ++v) fidx[v] = static_cast<uint16_t>(F.index(by[v]));
  }
  lay.flags_skip = F.index(&ones);
  if (t.maps[PCN_IPT_F_CONNTRACK].present()) {
    const FieldMap &m = t.maps[PCN_IPT_F_CONNTRACK];
    std::vector<const BitVec *> by(4, nullptr);
    for (size_t k = 0; k < m.keys.size(); ++k)
      if (m.keys[k] < 4) by[m.keys[k]] = &m.vecs[k];
    for (int v = 0; v < 4; ++v) cidx[v] = static_cast<uint8_t>(Cn.index(by[v]));
  } else {
    Cn.index(&ones);
  }
  if (P.vecs.size() > 256 || Cn.vecs.size() > 256) throw std::runtime_error("meta index overflow");

  // sport / dport / iface: hash of explicit keys; the wildcard key (0 / 0 /
  // 0xffff) becomes the miss value (L4PortLookup.cpp:44-56,
  // InterfaceLookup.cpp:44-56); ports are skipped for non-TCP/UDP packets
  // (L4PortLookup_dp.c:99-103).
  const int key_fields[3] = {PCN_IPT_F_SPORT, PCN_IPT_F_DPORT, PCN_IPT_F_IFACE};
  const uint32_t wild[3] = {0, 0, 0xffff};
  Small K[3];
  const BitVec *miss_vec[3] = {nullptr, nullptr, nullptr};
  bool key_present[3] = {false, false, false};
  for (int i = 0; i < 3; ++i) {
    const FieldMap &m = t.maps[key_fields[i]];
    if (!m.present()) continue;
    key_present[i] = true;
    for (size_t k = 0; k < m.keys.size(); ++k) {
      if (m.keys[k] == wild[i]) miss_vec[i] = &m.vecs[k];
      else K[i].index(&m.vecs[k]);
    }
    K[i].index(miss_vec[i]);
    if (i < 2) K[i].index(&ones);
  }
  bool merged[3] = {false, false, false};
  auto meta_dims = [&](const bool mg[3]) {
    std::vector<const std::vector<const BitVec *> *> dims{&P.vecs, &F.vecs, &Cn.vecs};
    for (int i = 0; i < 3; ++i)
      if (mg[i]) dims.push_back(&K[i].vecs);
    return dims;
  };
  auto for_each_entry = [&](const std::vector<const std::vector<const BitVec *> *> &dims, auto &&fn) {
    std::vector<size_t> at(dims.size(), 0);
    BitVec v(t.nrw);
    for (;;) {
      bool miss = false;
      for (size_t d = 0; d < dims.size(); ++d) miss |= (*dims[d])[at[d]] == nullptr;
      if (miss) {
        fn(nullptr);
      } else {
        for (uint32_t w = 0; w < t.nrw; ++w) {
          uint64_t x = ~uint64_t(0);
          for (size_t d = 0; d < dims.size(); ++d) x &= (*(*dims[d])[at[d]])[w];
          v[w] = x;
        }
        fn(&v);
      }
      size_t d = dims.size();
      while (d-- > 0) {            // row-major: the last dimension varies fastest
        if (++at[d] < dims[d]->size()) break;
        at[d] = 0;
      }
      if (d == size_t(-1)) break;
    }
  };
  for (int i = 0; i < 3; ++i) {
    if (!key_present[i] || !((join >> i) & 1)) continue;
    bool mg[3] = {merged[0], merged[1], merged[2]};
    mg[i] = true;
    const auto dims = meta_dims(mg);
    size_t entries = 1;
    for (auto *d : dims) entries *= d->size();
    if (entries > kMetaMaxEntries) continue;
    std::set<BitVec> distinct;
    for_each_entry(dims, [&](const BitVec *v) { if (v) distinct.insert(*v); });
    if (distinct.size() <= kMetaMaxClasses) merged[i] = true;
  }
  // slots: 0 meta, 1 src, 2 dst, then key fields that keep their own slot
  lay.nslots = 3;
  for (int i = 0; i < 3; ++i) lay.key_slot[i] = (key_present[i] && !merged[i]) ? lay.nslots++ : 0;
  for (int i = 0; i < 3; ++i) {
    const FieldMap &m = t.maps[key_fields[i]];
    if (!key_present[i]) continue;
    auto value = [&](const BitVec *v) -> uint32_t {
      if (merged[i]) return K[i].index(v);
      return v ? pool.intern(*v) : PCN_CLS_MISS;
    };
    lay.hash_wild[i] = value(miss_vec[i]);
    if (!merged[i]) slot_cls[lay.key_slot[i]].insert(lay.hash_wild[i]);
    if (i < 2) lay.key_skip[i] = merged[i] ? K[i].index(&ones) : img.all_cls;
    size_t nk = 0;
    for (size_t k = 0; k < m.keys.size(); ++k)
      if (m.keys[k] != wild[i]) ++nk;
    // load <= 1/4 and every key within two probes of its home slot (the
    // kernel reads slots h and h+1 and never loops); slot `size` mirrors slot 0
    std::vector<uint32_t> tab;
    for (uint32_t size = 16;; size <<= 1) {
      if (size < 4 * nk) continue;
      const uint32_t shift = static_cast<uint32_t>(__builtin_clz(size - 1));
      tab.assign(size + 1, PCN_HASH_EMPTY);
      bool ok = true;
      for (size_t k = 0; k < m.keys.size() && ok; ++k) {
        if (m.keys[k] == wild[i]) continue;
        uint32_t key = m.keys[k] & 0xffff;
        uint32_t h = (key * kHashMul) >> shift;
        if (tab[h] != PCN_HASH_EMPTY) h = (h + 1) & (size - 1);
        if (tab[h] != PCN_HASH_EMPTY) { ok = false; break; }
        tab[h] = (key << 16) | value(&m.vecs[k]);
        if (!merged[i]) slot_cls[lay.key_slot[i]].insert(tab[h] & 0xffff);
      }
      if (!ok) continue;
      tab[size] = tab[0];
      lay.hash_mask[i] = size - 1;
      break;
    }
    lay.hash[i] = blob.add(tab);
  }
  // meta index = sum of field index x stride (row-major over the joined fields)
  {
    const auto dims = meta_dims(merged);
    const int field_of_dim[6] = {0, 1, 2, 3, 4, 5};   // proto, flags, ct, then joined sport/dport/iface
    std::vector<int> fields{0, 1, 2};
    for (int i = 0; i < 3; ++i)
      if (merged[i]) fields.push_back(3 + i);
    (void)field_of_dim;
    uint32_t stride = 1;
    for (size_t d = dims.size(); d-- > 0;) {
      lay.meta_stride[fields[d]] = stride;
      stride *= static_cast<uint32_t>(dims[d]->size());
    }
    std::vector<uint16_t> meta;
    meta.reserve(stride);
    for_each_entry(dims, [&](const BitVec *v) { meta.push_back(v ? pool.intern(*v) : PCN_CLS_MISS); });
    slot_cls[0].insert(meta.begin(), meta.end());
    lay.proto_idx = blob.add(pidx);
    lay.flags_idx = blob.add(fidx);
    lay.ct_idx = blob.add(cidx);
    lay.meta = blob.add(meta);
    img.meta_entries = static_cast<uint32_t>(meta.size());
  }
  // Per class and 64-word block: SUMM (bit w: word w != 0), read by every
  // packet's summary AND, and the candidate record {PM, PBASE}: PM (bit w:
  // word w is partial -- neither zero nor every rule of its word) and the
  // start of the class's partial words in PART, stored in word order (rank =
  // popcount of PM below w).  At a candidate word every field's SUMM bit is
  // set, so PM alone tells partial from FULL there, and one 16-byte read
  // serves a field of the candidate stage.
  const auto &vecs = pool.vecs();
  img.nvec = static_cast<uint32_t>(vecs.size());
  const size_t nrec = size_t(img.nvec) * img.nsw;
  std::vector<uint64_t> summ(nrec, 0), words{~uint64_t(0)};
  std::vector<uint32_t> cand(4 * nrec, 0), part;                 // {PM lo, PM hi, PBASE, 0} per record
  std::vector<uint32_t> dense(size_t(img.nvec) * img.nrw, 0);     // POOL index per (class, word)
  std::map<uint64_t, uint32_t> word_id{{~uint64_t(0), 0}};
  for (uint32_t v = 0; v < img.nvec; ++v) {
    for (uint32_t w = 0; w < img.nrw; ++w) {
      const size_t rec = size_t(v) * img.nsw + w / 64;
      if (w % 64 == 0) cand[4 * rec + 2] = static_cast<uint32_t>(part.size());
      const uint64_t x = vecs[v][w];
      if (x) summ[rec] |= uint64_t(1) << (w % 64);
      if (x && x != perm.valid[w]) {
        cand[4 * rec + (w % 64) / 32] |= uint32_t(1) << (w % 32);
        auto it = word_id.emplace(x, static_cast<uint32_t>(words.size())).first;
        if (it->second == words.size()) words.push_back(x);
        part.push_back(it->second);
        dense[size_t(v) * img.nrw + w] = it->second;
      }
    }
  }
  img.part_words = static_cast<uint32_t>(part.size());
  lay.sf = blob.add(summ);
  // Partial words stored directly (one dependent LDS read less per field in
  // the candidate stage) while the whole image stays within kDirectMaxBytes.
  const size_t direct_bytes = blob.bytes.size() + cand.size() * 4 + part.size() * 8 + perm.perm.size() * 2 +
                              5 * kAlign;
  lay.part_direct = direct_bytes <= kDirectMaxBytes && !compact_images();
  lay.part_wide = !lay.part_direct && words.size() > 0xFFFF;
  if (lay.part_direct) {
    lay.pbase = blob.add(cand);
    std::vector<uint64_t> direct(part.size());
    for (size_t k = 0; k < part.size(); ++k) direct[k] = words[part[k]];
    lay.part = blob.add(direct);
    words.resize(1);   // POOL[0] = all-ones: what a FULL field reads
    lay.pool = blob.add(words);
    lay.zero = blob.add(std::vector<uint32_t>(4, 0));
    lay.perm = blob.add(perm.perm);
  } else {
    // An image this size may not fit LDS whole: POOL, the zero cell and PERM
    // go before the candidate tables, so the staged prefix [0, pbase) holds
    // every table but those.  When the image with {PM, PBASE} records and
    // indexed PART would exceed LDS anyway, PART is stored dense instead (a
    // POOL index per class and word, larger but L2-resident), so a candidate
    // field costs one L2 read rather than a record read and an index read.
    const size_t iw = lay.part_wide ? 4 : 2;
    const size_t indexed_bytes = blob.bytes.size() + words.size() * 8 + perm.perm.size() * 2 + cand.size() * 4 +
                                 part.size() * iw + 5 * kAlign;
    lay.part_dense = indexed_bytes > kDenseMinBytes && dense.size() * iw <= kDenseMaxBytes && !compact_images();
    if (lay.part_dense) {
      // Per word, the slots whose classes can be partial there (a word's rules
      // constrain ~3 of config 5's 5 slots): a candidate field outside them is
      // FULL whatever the class, and its PART cell is not read from L2.
      std::vector<uint8_t> wf(img.nrw, 0);
      for (uint32_t f = 0; f < lay.nslots; ++f)
        for (uint32_t c : slot_cls[f]) {
          if (c >= img.nvec) continue;   // PCN_CLS_MISS: no entry, the packet takes the default
          for (uint32_t w = 0; w < img.nrw; ++w)
            if (dense[size_t(c) * img.nrw + w]) wf[w] |= uint8_t(1u << f);
        }
      lay.wfields = blob.add(wf);
    }
    lay.pool = blob.add(words);
    lay.zero = blob.add(std::vector<uint32_t>(4, 0));
    lay.perm = blob.add(perm.perm);
    if (lay.part_dense) {
      if (lay.part_wide) lay.part = blob.add(dense);
      else lay.part = blob.add(std::vector<uint16_t>(dense.begin(), dense.end()));
      lay.pbase = lay.part;
    } else {
      lay.pbase = blob.add(cand);
      if (lay.part_wide) lay.part = blob.add(part);
      else lay.part = blob.add(std::vector<uint16_t>(part.begin(), part.end()));
    }
  }
  img.pool_words = static_cast<uint32_t>(words.size());
  img.part_bytes = (lay.part_dense ? dense.size() : part.size()) * (lay.part_direct ? 8 : lay.part_wide ? 4 : 2) +
                   words.size() * 8;
  lay.bytes = static_cast<uint32_t>((blob.bytes.size() + kAlign - 1) / kAlign * kAlign);
  blob.bytes.resize(lay.bytes);
  img.tables = std::move(blob.bytes);
  return img;
}

}  // namespace

// Joining key fields to the meta slot saves a slot (fewer summary and
// partial-word reads per packet) but can grow the image; join greedily, one
// field at a time, while the image keeps its partial words direct (i.e.
// stays within kDirectMaxBytes, comfortably inside LDS).
HostImage build_image(const ChainTables &t) {
  if (forced_join() >= 0) return build_image_with(t, static_cast<uint32_t>(forced_join()));
  HostImage best = build_image_with(t, 0);
  if (t.nrules == 0 || !best.lay.part_direct) return best;
  uint32_t join = 0;
  for (;;) {
    HostImage pick;
    uint32_t pick_join = 0;
    bool found = false;
    for (uint32_t i = 0; i < 3; ++i) {
      if ((join >> i) & 1) continue;
      const uint32_t j = join | (1u << i);
      HostImage trial = build_image_with(t, j);
      if (trial.lay.nslots >= best.lay.nslots || !trial.lay.part_direct) continue;
      if (!found || trial.lay.bytes < pick.lay.bytes) {
        pick = std::move(trial);
        pick_join = j;
        found = true;
      }
    }
    if (!found) return best;
    best = std::move(pick);
    join = pick_join;
  }
}

}  // namespace pcn
