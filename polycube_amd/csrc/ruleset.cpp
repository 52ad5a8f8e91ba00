// ruleset.cpp — rule parsing and the LBVS bitvector compiler (see ruleset.hpp).
#include "ruleset.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace pcn {
namespace {

// libs/polycube/src/utils.cpp:38-50 ip_string_to_nbo_uint (+ get_ip_from_string :233-239):
// the address part is scanned with "%hhu.%hhu.%hhu.%hhu%n" and must be consumed whole.
uint32_t ip_string_to_nbo(const std::string &s) {
  std::string addr = s.substr(0, s.find('/'));
  unsigned char a[4];
  int last = -1;
  int rc = std::sscanf(addr.c_str(), "%hhu.%hhu.%hhu.%hhu%n", a + 0, a + 1, a + 2, a + 3, &last);
  if (rc != 4 || static_cast<int>(addr.size()) != last)
    throw std::runtime_error("Not an ipv4 address " + s);
  return uint32_t(a[3]) << 24 | uint32_t(a[2]) << 16 | uint32_t(a[1]) << 8 | uint32_t(a[0]);
}

inline void set_rule_bit(BitVec &v, uint32_t id) {        // SET_BIT(bv[id/63], id%63)
  v[id / kBitsPerWord] |= uint64_t(1) << (id % kBitsPerWord);
}

// Utils.cpp:294-318: the containment test masks the NBO-as-integer address with
// the LOW `len` bits (quirk Q6 in SURVEY.md §8a) — reproduced on purpose.
inline bool ip_rule_covers(const IpPrefix &key, const IpPrefix &rule) {
  uint32_t mask = rule.len == 32 ? 0xffffffffu : ((uint32_t(1) << rule.len) - 1);
  return (key.ip & mask) == (rule.ip & mask) && rule.len <= key.len;
}

// Utils.cpp:223-375 ipFromRulesToMap
FieldMap compile_ip(const std::vector<Rule> &rules, bool src, uint32_t nrw) {
  std::map<IpPrefix, BitVec> ips;
  bool any_dont_care = false;
  for (const Rule &r : rules) {
    const auto &f = src ? r.src : r.dst;
    if (f) ips.emplace(*f, BitVec(nrw, 0)); else any_dont_care = true;
  }
  if (!ips.empty() && any_dont_care) ips.emplace(IpPrefix{0, 0}, BitVec(nrw, 0));
  for (auto &[key, vec] : ips) {
    for (uint32_t id = 0; id < rules.size(); ++id) {
      const auto &f = src ? rules[id].src : rules[id].dst;
      if (ip_rule_covers(key, f ? *f : IpPrefix{0, 0})) set_rule_bit(vec, id);
    }
  }
  FieldMap m;
  for (auto &[key, vec] : ips) {
    m.keys.push_back(key.ip);
    m.plen.push_back(key.len);
    m.vecs.push_back(std::move(vec));
  }
  return m;
}

// Utils.cpp:381-526: a keyed exact-match map; rules without the field are
// "don't care" and are set in every entry, under an extra wildcard key.
template <typename KeyOf>
FieldMap compile_keyed(const std::vector<Rule> &rules, uint32_t nrw, uint32_t wildcard_key,
                       KeyOf key_of) {
  std::map<uint32_t, BitVec> m;
  std::vector<uint32_t> dont_care;
  for (uint32_t id = 0; id < rules.size(); ++id) {
    std::optional<uint32_t> k = key_of(rules[id]);
    if (!k) { dont_care.push_back(id); continue; }
    auto it = m.try_emplace(*k, BitVec(nrw, 0)).first;
    set_rule_bit(it->second, id);
  }
  if (!m.empty() && !dont_care.empty()) {
    m.try_emplace(wildcard_key, BitVec(nrw, 0));
    for (uint32_t id : dont_care)
      for (auto &kv : m) set_rule_bit(kv.second, id);
  }
  FieldMap out;
  for (auto &[k, v] : m) { out.keys.push_back(k); out.vecs.push_back(std::move(v)); }
  return out;
}

// Utils.cpp:680-732 flagsFromRulesToMap: a full 256-entry array.
FieldMap compile_flags(const std::vector<Rule> &rules, uint32_t nrw) {
  FieldMap out;
  bool any = std::any_of(rules.begin(), rules.end(), [](const Rule &r) { return bool(r.tcpflags); });
  if (!any) return out;
  out.vecs.assign(256, BitVec(nrw, 0));
  for (uint32_t j = 0; j < 256; ++j) out.keys.push_back(j);
  for (uint32_t id = 0; id < rules.size(); ++id) {
    const Rule &r = rules[id];
    if (!r.tcpflags) {
      for (auto &v : out.vecs) set_rule_bit(v, id);
      continue;
    }
    uint8_t need = r.tcpflags->set ? r.tcpflags->set : 0xff;   // :714-717 (quirk Q10)
    uint8_t forbid = r.tcpflags->not_set;
    for (uint32_t c = 0; c < 256; ++c)
      if ((c & need) == need && (c & forbid) == 0) set_rule_bit(out.vecs[c], id);
  }
  return out;
}

// Utils.cpp:642-678 conntrackFromRulesToMap: 4 states, wildcard rules in all.
FieldMap compile_conntrack(const std::vector<Rule> &rules, uint32_t nrw) {
  FieldMap out;
  bool any = std::any_of(rules.begin(), rules.end(), [](const Rule &r) { return bool(r.conntrack); });
  if (!any) return out;
  for (uint32_t s = 0; s < 4; ++s) {
    BitVec v(nrw, 0);
    for (uint32_t id = 0; id < rules.size(); ++id)
      if (!rules[id].conntrack || *rules[id].conntrack == s) set_rule_bit(v, id);
    out.keys.push_back(s);
    out.vecs.push_back(std::move(v));
  }
  return out;
}

}  // namespace

IpPrefix IpPrefix::parse(const std::string &s) {
  IpPrefix p;
  size_t slash = s.find('/');
  uint8_t len = 32;
  if (slash != std::string::npos) {
    const char *b = s.c_str() + slash + 1;
    char *end = nullptr;
    long v = std::strtol(b, &end, 10);                         // std::stol
    if (end == b) throw std::runtime_error("invalid netmask in " + s);
    len = static_cast<uint8_t>(v);                             // stored into a uint8_t
  }
  if (len > 32) throw std::runtime_error("Netmask can't be bigger than 32");
  p.ip = ip_string_to_nbo(s);
  p.len = len;
  return p;
}

uint8_t protocol_from_string(const std::string &p) {
  if (p == "TCP" || p == "tcp") return 6;
  if (p == "UDP" || p == "udp") return 17;
  if (p == "ICMP" || p == "icmp") return 1;
  if (p == "GRE" || p == "gre") return 47;
  throw std::runtime_error("Protocol not supported.");
}

TcpFlagsMask flags_from_string(const std::string &flags) {
  static const char *kNames[8] = {"FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR"};
  std::string s = flags;
  TcpFlagsMask m;
  for (int bit = 0; bit < 8; ++bit) {           // negated flags are consumed first
    std::string neg = std::string("!") + kNames[bit];
    size_t at = s.find(neg);
    if (at != std::string::npos) { s.erase(at, neg.size()); m.not_set |= uint8_t(1u << bit); }
  }
  for (int bit = 0; bit < 8; ++bit)
    if (s.find(kNames[bit]) != std::string::npos) m.set |= uint8_t(1u << bit);
  if (m.set & m.not_set) throw std::runtime_error("A flag can't be both set and not set!");
  return m;
}

Rule Rule::from_c(const pcn_ipt_rule &c, const PortTable &ports) {
  Rule r;
  if (c.conntrack) {
    std::string s = c.conntrack;
    if (s == "NEW") r.conntrack = 0;
    else if (s == "ESTABLISHED") r.conntrack = 1;
    else if (s == "RELATED") r.conntrack = 2;
    else if (s == "INVALID") r.conntrack = 3;
    else throw std::runtime_error("invalid conntrack status " + s);
  }
  if (c.src) r.src = IpPrefix::parse(c.src);
  if (c.dst) r.dst = IpPrefix::parse(c.dst);
  if (c.sport >= 0) {
    if (c.sport > 65535) throw std::runtime_error("sport out of range");
    r.sport = static_cast<uint16_t>(c.sport);
  }
  if (c.dport >= 0) {
    if (c.dport > 65535) throw std::runtime_error("dport out of range");
    r.dport = static_cast<uint16_t>(c.dport);
  }
  if (c.tcpflags) r.tcpflags = flags_from_string(c.tcpflags);
  if (c.l4proto) r.l4proto = protocol_from_string(c.l4proto);
  if (c.in_iface) {
    if (!ports.find(c.in_iface)) throw std::runtime_error(std::string("no port ") + c.in_iface);
    r.in_iface = c.in_iface;
  }
  if (c.out_iface) {
    if (!ports.find(c.out_iface)) throw std::runtime_error(std::string("no port ") + c.out_iface);
    r.out_iface = c.out_iface;
  }
  if (c.action < 0) r.action = PCN_IPT_DROP;
  else if (c.action == PCN_IPT_DROP || c.action == PCN_IPT_ACCEPT) r.action = uint8_t(c.action);
  else throw std::runtime_error("Action not supported.");   // Utils.cpp:200-207
  return r;
}

bool Rule::operator==(const Rule &o) const {
  auto flags_eq = [](const std::optional<TcpFlagsMask> &a, const std::optional<TcpFlagsMask> &b) {
    if (bool(a) != bool(b)) return false;
    return !a || (a->set == b->set && a->not_set == b->not_set);
  };
  return src == o.src && dst == o.dst && sport == o.sport && dport == o.dport &&
         l4proto == o.l4proto && flags_eq(tcpflags, o.tcpflags) && in_iface == o.in_iface &&
         out_iface == o.out_iface && conntrack == o.conntrack && action == o.action;
}

ChainTables compile_chain(const std::vector<Rule> &rules, int chain, int default_action,
                          const PortTable &ports) {
  ChainTables t;
  t.nrules = static_cast<uint32_t>(rules.size());
  t.nrw = words_for_rules(t.nrules);
  t.default_action = default_action;
  t.actions.reserve(rules.size());
  for (const Rule &r : rules) t.actions.push_back(r.action);
  if (t.nrules == 0) return t;
  const uint32_t nrw = t.nrw;
  t.maps[PCN_IPT_F_CONNTRACK] = compile_conntrack(rules, nrw);
  t.maps[PCN_IPT_F_IPSRC] = compile_ip(rules, true, nrw);
  t.maps[PCN_IPT_F_IPDST] = compile_ip(rules, false, nrw);
  t.maps[PCN_IPT_F_L4PROTO] = compile_keyed(rules, nrw, 0, [](const Rule &r) {
    return r.l4proto ? std::optional<uint32_t>(*r.l4proto) : std::nullopt;
  });
  t.maps[PCN_IPT_F_SPORT] = compile_keyed(rules, nrw, 0, [](const Rule &r) {
    return r.sport ? std::optional<uint32_t>(*r.sport) : std::nullopt;
  });
  t.maps[PCN_IPT_F_DPORT] = compile_keyed(rules, nrw, 0, [](const Rule &r) {
    return r.dport ? std::optional<uint32_t>(*r.dport) : std::nullopt;
  });
  // Utils.cpp:483-501: INPUT/FORWARD match in-iface, OUTPUT matches out-iface;
  // a name that no longer resolves is treated as don't-care (the catch block).
  const bool out = chain == PCN_IPT_OUTPUT;
  t.maps[PCN_IPT_F_IFACE] = compile_keyed(rules, nrw, 0xffff, [&](const Rule &r) {
    const auto &name = out ? r.out_iface : r.in_iface;
    if (!name) return std::optional<uint32_t>();
    auto idx = ports.find(*name);
    return idx ? std::optional<uint32_t>(*idx) : std::nullopt;
  });
  t.maps[PCN_IPT_F_TCPFLAGS] = compile_flags(rules, nrw);
  return t;
}

}  // namespace pcn
