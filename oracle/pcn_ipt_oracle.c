/*
 * pcn_ipt_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker, CPU baseline).
 *
 * A deliberately literal, scalar C restatement of the reference pcn-iptables
 * datapath and rule compiler.  Every function cites the reference file:line it
 * follows (paths relative to src/services/pcn-iptables/src/ unless noted).
 * It is never linked into the product library.
 *
 * Semantics restated:
 *   rule parsing      ChainRule.cpp:29-83, defines.h:84-114 (IpAddr),
 *                     libs/polycube/src/utils.cpp:38-50,233-239, Utils.cpp:19-200
 *   rule compiler     Utils.cpp:223-732 (*FromRulesToMap), Chain.cpp:431-929
 *   datapath          datapaths/Iptables_{Parser,ChainSelector,ConntrackLabel,
 *                     IpLookup,L4ProtocolLookup,L4PortLookup,InterfaceLookup,
 *                     TcpFlagsLookup,ConntrackMatch,BitScan,ActionLookup}_dp.c
 *   kernel LPM trie   longest prefix wins, MSB-first over the key bytes, an
 *                     insert with an equal (prefixlen, prefix) replaces the value;
 *                     1024-entry capacity (Iptables_IpLookup_dp.c:54-55).
 *                     Linux kernel/bpf/lpm_trie.c is not in /root/reference;
 *                     this is its published behaviour.
 * The module order chosen by Chain.cpp:624-849 does not change verdicts or
 * counters (every module ANDs into one vector; any miss/zero exits to the
 * default action once), so modules run in the fixed defines.h order here.
 */
#define _GNU_SOURCE
#include "pcn_ipt_oracle.h"

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NCHAINS 3
#define REF_MAX_RULES 8192 /* Iptables.h:173 */
#define NRULES_TO_NELEMS(x) ((x) / 63 + ((x) % 63 != 0 ? 1 : 0)) /* defines.h:168 */
#define TRIE_MAX 1024     /* Iptables_IpLookup_dp.c:54-55 */

enum { F_CT = 0, F_IPSRC, F_IPDST, F_PROTO, F_SPORT, F_DPORT, F_IFACE, F_FLAGS, NFIELDS };
enum { RX_OK = 0, RX_DROP = 2 };
enum { CT_NEW = 0, CT_ESTABLISHED = 1, CT_RELATED = 2, CT_INVALID = 3 };

typedef struct { uint32_t ip; uint8_t netmask; } ipaddr_t; /* defines.h:84-114 */

typedef struct {
  int src_set, dst_set, proto_set, sport_set, dport_set, flags_set_, in_set, out_set, ct_set;
  ipaddr_t src, dst;
  int proto;
  uint16_t sport, dport;
  uint8_t fset, fnot;
  char in_iface[64], out_iface[64];
  int ct;
  int action;
} prule_t;

typedef struct tnode {
  struct tnode *ch[2];
  int has;
  int vec; /* index into chain pool */
} tnode_t;

typedef struct {      /* one compiled map, as pushed by updateMap */
  int n;
  uint32_t *key;      /* map key in push order */
  uint8_t *plen;
  int *vec;           /* pool index */
} omap_t;

typedef struct {
  int nrules, default_action, nrw, vlen;
  prule_t *rules;
  uint64_t *pool; int npool, cappool;
  int present[NFIELDS];
  omap_t maps[NFIELDS];
  /* datapath views */
  tnode_t *trie[2]; int trie_nodes[2];
  int proto_tab[256];
  int sport_tab[65536], dport_tab[65536], iface_tab[65536];
  int sport_wild, dport_wild, iface_wild; /* pool idx or -1 */
  int flags_tab[256];
  int ct_tab[4];
  uint8_t *actions; /* per rule */
  /* counters (ActionLookup_dp.c:55-56, Parser_dp.c:47-58) */
  uint64_t *pkts, *bytes;
  uint64_t def_pkts, def_bytes;
} ochain_t;

typedef struct { char name[64]; uint16_t index; } port_t;

/* One Horus entry: the set fields of the key as the datapath's packed
 * horusKey holds them (sk/dk: the port's two network-order bytes read as a
 * little-endian u16, i.e. the htons() of modules/Horus.cpp:44-51), the
 * HorusValue {action, ruleID} (defines.h:161-164). */
#define HZ_MAX 2048                              /* HorusConst::MAX_RULE_SIZE_FOR_HORUS, defines.h:127 */
typedef struct { uint32_t src, dst; uint8_t proto; uint16_t sk, dk; uint8_t action; uint32_t rule; } hzent_t;
/* One Horus program: pcn-iptables has one (ingress, from INPUT); pcn-firewall
 * one per chain (INGRESS / EGRESS, Firewall.h:333-340). */
typedef struct {
  int runtime;                               /* horus_runtime_enabled_ */
  int ct;                                    /* pcn-firewall: _CONNTRACK_ENABLED when it was built */
  uint32_t fields; int n;
  hzent_t ent[HZ_MAX];
  uint64_t pkts[HZ_MAX], bytes[HZ_MAX];      /* pkts_horus / bytes_horus (Horus_dp.c:77-78) */
} hzprog_t;

struct orc_ctx {
  int service;                           /* ORC_SVC_IPTABLES / ORC_SVC_FIREWALL */
  int fw_ct_mode;                        /* pcn-firewall conntrackMode (defines.h:56-58) */
  ochain_t ch[NCHAINS];
  port_t ports[1024]; int nports;
  uint32_t localip[256]; int nlocal;
  uint32_t max_counted, max_action;
  uint16_t index64[64];
  pthread_mutex_t mu;
  /* stateful conntrack (see "conntrack" below) */
  struct ctstate *ct;
  int ae[NCHAINS];                       /* accept_established_enabled_<chain>_ (Iptables.h) */
  uint64_t ae_pkts[NCHAINS], ae_bytes[NCHAINS]; /* pkts_/bytes_acceptestablished_<Chain> */
  /* Horus (Iptables.h:183-188; pcn-firewall Firewall.h:333-340) */
  int hz_enabled;
  hzprog_t hz[2];                            /* [0] iptables INPUT / firewall INGRESS, [1] firewall EGRESS */
  /* the shared per-CPU `packet` struct's ports while conntrack is off (the
   * Horus key reads them for packets the Parser wrote no ports for, Q4) */
  uint16_t hz_stale[2];
};

/* ---------------- rule parsing ---------------- */

/* libs/polycube/src/utils.cpp:38-50 (+ get_ip_from_string :233-239) */
static int ip_string_to_nbo_uint(const char *s, uint32_t *out) {
  char buf[128];
  const char *slash = strchr(s, '/');
  size_t len = slash ? (size_t)(slash - s) : strlen(s);
  if (len >= sizeof buf) return -EINVAL;
  memcpy(buf, s, len); buf[len] = 0;
  unsigned char a[4]; int last = -1;
  int rc = sscanf(buf, "%hhu.%hhu.%hhu.%hhu%n", a + 0, a + 1, a + 2, a + 3, &last);
  if (rc != 4 || (int)len != last) return -EINVAL;
  *out = (uint32_t)a[3] << 24 | (uint32_t)a[2] << 16 | (uint32_t)a[1] << 8 | (uint32_t)a[0];
  return 0;
}

/* defines.h:91-109 IpAddr::fromString (netmask via std::stol into a uint8_t) */
static int ipaddr_from_string(const char *s, ipaddr_t *o) {
  const char *slash = strchr(s, '/');
  uint8_t nm = 32;
  if (slash) {
    char *end; errno = 0;
    long v = strtol(slash + 1, &end, 10);
    if (end == slash + 1 || errno) return -EINVAL; /* std::stol throws */
    nm = (uint8_t)v;
  }
  if (nm > 32) return -EINVAL;
  uint32_t ip;
  if (ip_string_to_nbo_uint(s, &ip)) return -EINVAL;
  o->ip = ip; o->netmask = nm;
  return 0;
}

static int strieq2(const char *a, const char *up, const char *lo) {
  return strcmp(a, up) == 0 || strcmp(a, lo) == 0;
}

/* Utils.cpp:45-57 ChainRule::protocolFromStringToInt */
static int proto_from_string(const char *p, int *out) {
  if (strieq2(p, "TCP", "tcp")) { *out = 6; return 0; }
  if (strieq2(p, "UDP", "udp")) { *out = 17; return 0; }
  if (strieq2(p, "ICMP", "icmp")) { *out = 1; return 0; }
  if (strieq2(p, "GRE", "gre")) { *out = 47; return 0; }
  return -EINVAL;
}

/* erase the first occurrence of pat from s (std::string::erase(find(pat), len)) */
static int erase_first(char *s, const char *pat) {
  char *p = strstr(s, pat);
  if (!p) return 0;
  size_t l = strlen(pat);
  memmove(p, p + l, strlen(p + l) + 1);
  return 1;
}

/* Utils.cpp:73-140 ChainRule::flagsFromStringToMasks */
static int flags_from_string(const char *flags, uint8_t *set, uint8_t *notset) {
  static const char *names[8] = {"FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR"};
  char buf[256];
  if (strlen(flags) >= sizeof buf) return -EINVAL;
  strcpy(buf, flags);
  uint8_t ns = 0, s = 0;
  for (int i = 0; i < 8; i++) {
    char neg[8]; snprintf(neg, sizeof neg, "!%s", names[i]);
    if (erase_first(buf, neg)) ns |= (uint8_t)(1u << i);
  }
  for (int i = 0; i < 8; i++)
    if (strstr(buf, names[i])) s |= (uint8_t)(1u << i);
  if (s & ns) return -EINVAL;
  *set = s; *notset = ns;
  return 0;
}

static int ct_from_string(const char *s, int *o) {
  if (!strcmp(s, "NEW")) *o = CT_NEW;
  else if (!strcmp(s, "ESTABLISHED")) *o = CT_ESTABLISHED;
  else if (!strcmp(s, "RELATED")) *o = CT_RELATED;
  else if (!strcmp(s, "INVALID")) *o = CT_INVALID;
  else return -EINVAL;
  return 0;
}

static int port_index(orc_ctx *c, const char *name, uint16_t *idx) {
  for (int i = 0; i < c->nports; i++)
    if (!strcmp(c->ports[i].name, name)) { *idx = c->ports[i].index; return 0; }
  return -ENOENT; /* Iptables.cpp:480-484 get_port throws */
}

/* ChainRule.cpp:29-83 ChainRule::update */
static int parse_rule(orc_ctx *c, const orc_rule *r, prule_t *p) {
  memset(p, 0, sizeof *p);
  if (r->conntrack) { if (ct_from_string(r->conntrack, &p->ct)) return -EINVAL; p->ct_set = 1; }
  if (r->src) { if (ipaddr_from_string(r->src, &p->src)) return -EINVAL; p->src_set = 1; }
  if (r->dst) { if (ipaddr_from_string(r->dst, &p->dst)) return -EINVAL; p->dst_set = 1; }
  if (r->sport >= 0) { if (r->sport > 65535) return -EINVAL; p->sport = (uint16_t)r->sport; p->sport_set = 1; }
  if (r->dport >= 0) { if (r->dport > 65535) return -EINVAL; p->dport = (uint16_t)r->dport; p->dport_set = 1; }
  if (r->tcpflags) { if (flags_from_string(r->tcpflags, &p->fset, &p->fnot)) return -EINVAL; p->flags_set_ = 1; }
  if (r->l4proto) { if (proto_from_string(r->l4proto, &p->proto)) return -EINVAL; p->proto_set = 1; }
  uint16_t dummy;
  if (r->in_iface) {
    if (strlen(r->in_iface) >= 64 || port_index(c, r->in_iface, &dummy)) return -EINVAL;
    strcpy(p->in_iface, r->in_iface); p->in_set = 1;
  }
  if (r->out_iface) {
    if (strlen(r->out_iface) >= 64 || port_index(c, r->out_iface, &dummy)) return -EINVAL;
    strcpy(p->out_iface, r->out_iface); p->out_set = 1;
  }
  if (r->action < 0) p->action = 0;            /* ChainRule.cpp:76-82: unset => DROP */
  else if (r->action <= 1) p->action = r->action;
  else return -EINVAL;                         /* Utils.cpp:200-207 (LOG throws) */
  return 0;
}

/* ---------------- compiler ---------------- */

static int pool_new(ochain_t *ch) {
  if (ch->npool == ch->cappool) {
    int nc = ch->cappool ? ch->cappool * 2 : 64;
    uint64_t *np = realloc(ch->pool, (size_t)nc * ch->vlen * 8);
    if (!np) return -1;
    ch->pool = np; ch->cappool = nc;
  }
  memset(ch->pool + (size_t)ch->npool * ch->vlen, 0, (size_t)ch->vlen * 8);
  return ch->npool++;
}
static inline uint64_t *VEC(ochain_t *ch, int i) { return ch->pool + (size_t)i * ch->vlen; }
/* defines.h:165 SET_BIT on bitVector[id/63], bit id%63 (Utils.cpp:316) */
static inline void setbit(uint64_t *v, uint32_t id) { v[id / 63] |= (uint64_t)1 << (id % 63); }

static void omap_push(omap_t *m, uint32_t key, uint8_t plen, int vec) {
  m->key = realloc(m->key, (size_t)(m->n + 1) * 4);
  m->plen = realloc(m->plen, (size_t)(m->n + 1));
  m->vec = realloc(m->vec, (size_t)(m->n + 1) * sizeof(int));
  m->key[m->n] = key; m->plen[m->n] = plen; m->vec[m->n] = vec; m->n++;
}

static int cmp_ipaddr(const void *a, const void *b) { /* defines.h:110-113 operator< */
  const ipaddr_t *x = a, *y = b;
  if (x->ip != y->ip) return x->ip < y->ip ? -1 : 1;
  return (int)x->netmask - (int)y->netmask;
}
static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return x < y ? -1 : x > y;
}

/* Utils.cpp:294-318 containment test (with its NBO-as-integer mask quirk) */
static int ip_contains(ipaddr_t addr, ipaddr_t rule) {
  uint32_t mask = rule.netmask == 32 ? 0xffffffffu : (((uint32_t)1 << rule.netmask) - 1);
  return ((addr.ip & mask) == (rule.ip & mask)) && (rule.netmask <= addr.netmask);
}

/* Utils.cpp:223-375 Chain::ipFromRulesToMap */
static void compile_ip(ochain_t *ch, int field) {
  int is_src = field == F_IPSRC;
  ipaddr_t *keys = malloc(sizeof(ipaddr_t) * (ch->nrules + 1));
  int nk = 0, ndc = 0;
  for (int i = 0; i < ch->nrules; i++) {
    prule_t *r = &ch->rules[i];
    int set = is_src ? r->src_set : r->dst_set;
    if (!set) { ndc++; continue; }
    keys[nk++] = is_src ? r->src : r->dst;
  }
  qsort(keys, nk, sizeof(ipaddr_t), cmp_ipaddr);
  int nu = 0;
  for (int i = 0; i < nk; i++)
    if (nu == 0 || cmp_ipaddr(&keys[nu - 1], &keys[i]) != 0) keys[nu++] = keys[i];
  if (nu != 0 && ndc != 0) { /* :326-374 wildcard 0.0.0.0/0 (insert keeps an existing key) */
    ipaddr_t w = {0, 0};
    int found = 0;
    for (int i = 0; i < nu; i++) if (keys[i].ip == 0 && keys[i].netmask == 0) found = 1;
    if (!found) {
      keys[nu++] = w;
      qsort(keys, nu, sizeof(ipaddr_t), cmp_ipaddr);
    }
  }
  omap_t *m = &ch->maps[field];
  for (int k = 0; k < nu; k++) {
    int v = pool_new(ch);
    for (int i = 0; i < ch->nrules; i++) {
      prule_t *r = &ch->rules[i];
      int set = is_src ? r->src_set : r->dst_set;
      ipaddr_t rip = set ? (is_src ? r->src : r->dst) : (ipaddr_t){0, 0};
      if (ip_contains(keys[k], rip)) setbit(VEC(ch, v), (uint32_t)i);
    }
    omap_push(m, keys[k].ip, keys[k].netmask, v);
  }
  ch->present[field] = nu > 0;
  free(keys);
}

static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

/* kernel LPM trie insert, modules/IpLookup.cpp:122-140 updateMap order */
static int trie_insert(ochain_t *ch, int t, uint32_t ip_nbo, uint8_t plen, int vec) {
  if (!ch->trie[t]) ch->trie[t] = calloc(1, sizeof(tnode_t));
  tnode_t *n = ch->trie[t];
  uint32_t h = bswap32(ip_nbo);
  for (int b = 0; b < plen; b++) {
    int bit = (h >> (31 - b)) & 1;
    if (!n->ch[bit]) n->ch[bit] = calloc(1, sizeof(tnode_t));
    n = n->ch[bit];
  }
  if (!n->has) {
    if (ch->trie_nodes[t] >= TRIE_MAX) return -ENOSPC;
    ch->trie_nodes[t]++;
  }
  n->has = 1; n->vec = vec;
  return 0;
}
static int trie_lookup(const tnode_t *n, uint32_t ip_nbo) {
  uint32_t h = bswap32(ip_nbo);
  int best = -1;
  for (int b = 0; n; b++) {
    if (n->has) best = n->vec;
    if (b == 32) break;
    n = n->ch[(h >> (31 - b)) & 1];
  }
  return best;
}
static void trie_free(tnode_t *n) {
  if (!n) return;
  trie_free(n->ch[0]); trie_free(n->ch[1]); free(n);
}

typedef int (*getkey_fn)(orc_ctx *, const prule_t *, int chain, uint32_t *key);
static int gk_proto(orc_ctx *c, const prule_t *r, int chain, uint32_t *k) {
  (void)c; (void)chain; if (!r->proto_set) return 0; *k = (uint32_t)r->proto; return 1;
}
static int gk_sport(orc_ctx *c, const prule_t *r, int chain, uint32_t *k) {
  (void)c; (void)chain; if (!r->sport_set) return 0; *k = r->sport; return 1;
}
static int gk_dport(orc_ctx *c, const prule_t *r, int chain, uint32_t *k) {
  (void)c; (void)chain; if (!r->dport_set) return 0; *k = r->dport; return 1;
}
/* Utils.cpp:483-501: IN_TYPE for INPUT/FORWARD, OUT_TYPE for OUTPUT (Chain.cpp:611) */
static int gk_iface(orc_ctx *c, const prule_t *r, int chain, uint32_t *k) {
  const char *nm = chain == ORC_OUTPUT ? (r->out_set ? r->out_iface : NULL)
                                        : (r->in_set ? r->in_iface : NULL);
  uint16_t idx;
  if (!nm || port_index(c, nm, &idx)) return 0;
  *k = idx; return 1;
}

/* Utils.cpp:381-429 / 431-474 / 476-526: keyed bitvector maps with a wildcard key */
static void compile_keyed(orc_ctx *c, ochain_t *ch, int chain, int field, getkey_fn gk,
                          uint32_t wildkey) {
  uint32_t *keys = malloc(sizeof(uint32_t) * (ch->nrules + 1));
  int nk = 0, ndc = 0;
  for (int i = 0; i < ch->nrules; i++) {
    uint32_t k;
    if (gk(c, &ch->rules[i], chain, &k)) keys[nk++] = k; else ndc++;
  }
  qsort(keys, nk, 4, cmp_u32);
  int nu = 0;
  for (int i = 0; i < nk; i++) if (nu == 0 || keys[nu - 1] != keys[i]) keys[nu++] = keys[i];
  if (nu != 0 && ndc != 0) {
    int found = 0;
    for (int i = 0; i < nu; i++) if (keys[i] == wildkey) found = 1;
    if (!found) { keys[nu++] = wildkey; qsort(keys, nu, 4, cmp_u32); }
  }
  omap_t *m = &ch->maps[field];
  for (int k = 0; k < nu; k++) omap_push(m, keys[k], 0, pool_new(ch));
  for (int i = 0; i < ch->nrules; i++) {
    uint32_t kk;
    if (gk(c, &ch->rules[i], chain, &kk)) {
      for (int k = 0; k < nu; k++) if (keys[k] == kk) setbit(VEC(ch, m->vec[k]), (uint32_t)i);
    } else if (nu != 0) { /* don't-care rules are in all entries */
      for (int k = 0; k < nu; k++) setbit(VEC(ch, m->vec[k]), (uint32_t)i);
    }
  }
  ch->present[field] = nu > 0;
  free(keys);
}

/* Utils.cpp:680-732 Chain::flagsFromRulesToMap */
static void compile_flags(ochain_t *ch) {
  int any = 0;
  for (int i = 0; i < ch->nrules; i++) if (ch->rules[i].flags_set_) any = 1;
  if (!any) return;
  omap_t *m = &ch->maps[F_FLAGS];
  for (int j = 0; j < 256; j++) omap_push(m, (uint32_t)j, 0, pool_new(ch));
  for (int i = 0; i < ch->nrules; i++) {
    prule_t *r = &ch->rules[i];
    if (!r->flags_set_) {
      for (int j = 0; j < 256; j++) setbit(VEC(ch, m->vec[j]), (uint32_t)i);
      continue;
    }
    uint8_t fs = r->fset, fn = r->fnot;
    if (fs == 0) fs = 255; /* :714-717 */
    for (int j = 0; j < 256; j++) {
      uint8_t cand = (uint8_t)j; /* possible_flags_combinations_[j] == j */
      if ((cand & fs) == fs && (cand & fn) == 0) setbit(VEC(ch, m->vec[cand]), (uint32_t)i);
    }
  }
  ch->present[F_FLAGS] = 1;
}

/* Utils.cpp:642-678 Chain::conntrackFromRulesToMap */
static void compile_ct(ochain_t *ch) {
  int any = 0;
  for (int i = 0; i < ch->nrules; i++) if (ch->rules[i].ct_set) any = 1;
  if (!any) return;
  omap_t *m = &ch->maps[F_CT];
  for (int s = 0; s < 4; s++) {
    int v = pool_new(ch);
    for (int i = 0; i < ch->nrules; i++) {
      prule_t *r = &ch->rules[i];
      if (!r->ct_set || r->ct == s) setbit(VEC(ch, v), (uint32_t)i);
    }
    omap_push(m, (uint32_t)s, 0, v);
  }
  ch->present[F_CT] = 1;
}

static void chain_free(ochain_t *ch) {
  free(ch->rules); free(ch->pool); free(ch->actions); free(ch->pkts); free(ch->bytes);
  for (int f = 0; f < NFIELDS; f++) {
    free(ch->maps[f].key); free(ch->maps[f].plen); free(ch->maps[f].vec);
  }
  trie_free(ch->trie[0]); trie_free(ch->trie[1]);
  memset(ch, 0, sizeof *ch);
}

/* Chain::updateChain, Chain.cpp:600-874 */
static int compile_chain(orc_ctx *c, int chain) {
  ochain_t *ch = &c->ch[chain];
  int n = ch->nrules;
  ch->nrw = NRULES_TO_NELEMS(n);
  int mr = NRULES_TO_NELEMS(REF_MAX_RULES);
  ch->vlen = ch->nrw > mr ? ch->nrw : mr;
  compile_ct(ch);
  compile_ip(ch, F_IPSRC);
  compile_ip(ch, F_IPDST);
  compile_keyed(c, ch, chain, F_PROTO, gk_proto, 0);
  compile_keyed(c, ch, chain, F_SPORT, gk_sport, 0);
  compile_keyed(c, ch, chain, F_DPORT, gk_dport, 0);
  compile_keyed(c, ch, chain, F_IFACE, gk_iface, 0xffff);
  compile_flags(ch);
  /* datapath views */
  for (int t = 0; t < 2; t++) {
    omap_t *m = &ch->maps[t == 0 ? F_IPSRC : F_IPDST];
    for (int k = 0; k < m->n; k++) {
      int rc = trie_insert(ch, t, m->key[k], m->plen[k], m->vec[k]);
      if (rc) return rc;
    }
  }
  for (int i = 0; i < 256; i++) ch->proto_tab[i] = -1;
  for (int k = 0; k < ch->maps[F_PROTO].n; k++)
    ch->proto_tab[ch->maps[F_PROTO].key[k] & 0xff] = ch->maps[F_PROTO].vec[k];
  int *tabs[3] = {ch->sport_tab, ch->dport_tab, ch->iface_tab};
  int *wild[3] = {&ch->sport_wild, &ch->dport_wild, &ch->iface_wild};
  int fl[3] = {F_SPORT, F_DPORT, F_IFACE};
  uint32_t wk[3] = {0, 0, 0xffff};
  for (int t = 0; t < 3; t++) {
    for (int i = 0; i < 65536; i++) tabs[t][i] = -1;
    *wild[t] = -1;
    omap_t *m = &ch->maps[fl[t]];
    for (int k = 0; k < m->n; k++) {
      tabs[t][m->key[k]] = m->vec[k];
      if (m->key[k] == wk[t]) *wild[t] = m->vec[k]; /* L4PortLookup.cpp:44-56, InterfaceLookup.cpp:44-56 */
    }
  }
  for (int i = 0; i < 256; i++) ch->flags_tab[i] = -1;
  for (int k = 0; k < ch->maps[F_FLAGS].n; k++) ch->flags_tab[k] = ch->maps[F_FLAGS].vec[k];
  for (int i = 0; i < 4; i++) ch->ct_tab[i] = -1;
  for (int k = 0; k < ch->maps[F_CT].n; k++) ch->ct_tab[k] = ch->maps[F_CT].vec[k];
  ch->actions = calloc((size_t)n + 1, 1);
  for (int i = 0; i < n; i++) ch->actions[i] = (uint8_t)ch->rules[i].action;
  return 0;
}

/* ---------------- public control API ---------------- */

static void build_index64(uint16_t t[64]) {
  /* BitScan_dp.c:97: idx = ((b ^ (b-1)) * 0x03f79d71b4cb0a89) >> 58; index64[idx] = ctz(b) */
  for (int p = 0; p < 64; p++) {
    uint64_t b = (uint64_t)1 << p;
    int idx = (int)(((b ^ (b - 1)) * 0x03f79d71b4cb0a89ull) >> 58);
    t[idx] = (uint16_t)p;
  }
}

orc_ctx *orc_create(uint32_t max_counted, uint32_t max_action) {
  orc_ctx *c = calloc(1, sizeof *c);
  if (!c) return NULL;
  c->max_counted = max_counted ? max_counted : 8000;  /* ActionLookup_dp.c:55-56 */
  c->max_action = max_action ? max_action : 10000;    /* ActionLookup_dp.c:36 */
  build_index64(c->index64);
  pthread_mutex_init(&c->mu, NULL);
  for (int i = 0; i < NCHAINS; i++) {
    c->ch[i].default_action = 1; /* Iptables.cpp:33-38: chains start ACCEPT */
    c->ch[i].pkts = calloc(c->max_counted, 8);
    c->ch[i].bytes = calloc(c->max_counted, 8);
  }
  return c;
}

static void ct_free(struct ctstate *t);
void orc_destroy(orc_ctx *c) {
  if (!c) return;
  ct_free(c->ct);
  for (int i = 0; i < NCHAINS; i++) chain_free(&c->ch[i]);
  free(c);
}

int orc_add_port(orc_ctx *c, const char *name, uint16_t index) {
  if (c->nports >= 1024 || strlen(name) >= 64) return -ENOSPC;
  strcpy(c->ports[c->nports].name, name);
  c->ports[c->nports].index = index;
  c->nports++;
  return 0;
}

static void horus_update(orc_ctx *c, int chain);
int orc_set_chain(orc_ctx *c, int chain, const orc_rule *rules, uint32_t n, int def) {
  if (chain < 0 || chain >= NCHAINS || (def != 0 && def != 1)) return -EINVAL;
  prule_t *pr = calloc((size_t)n + 1, sizeof(prule_t));
  for (uint32_t i = 0; i < n; i++)
    if (parse_rule(c, &rules[i], &pr[i])) { free(pr); return -EINVAL; }
  ochain_t *ch = &c->ch[chain];
  uint64_t *pk = ch->pkts, *by = ch->bytes;
  /* the default counters live outside the reloaded rule modules
   * (pkts_/bytes_default_<CHAIN> are shared tables, Iptables_Parser_dp.c:47-58;
   * pcn-firewall's DefaultAction is not part of the chain, Firewall.cpp:60-70):
   * they survive Chain::updateChain.  The per-rule ActionLookup counters do not. */
  const uint64_t dp = ch->def_pkts, db = ch->def_bytes;
  ch->pkts = ch->bytes = NULL;
  chain_free(ch);
  ch->pkts = pk; ch->bytes = by;
  ch->def_pkts = dp; ch->def_bytes = db;
  memset(pk, 0, c->max_counted * 8); memset(by, 0, c->max_counted * 8);
  ch->rules = pr; ch->nrules = (int)n; ch->default_action = def;
  int rc = compile_chain(c, chain);
  horus_update(c, chain);
  return rc;
}

/* ---------------- Horus ---------------- */

static inline uint16_t bswap16(uint16_t x) { return (uint16_t)(x >> 8 | x << 8); }

/* Chain::fromRuleToHorusKeyValue + horusFromRulesToMap (pcn-iptables
 * Utils.cpp:537-630; pcn-firewall Utils.cpp:483-577, the same rule): the
 * leading rules whose key sets the same fields as rule 0 (a /32 address,
 * protocol, ports; anything else the rule matches on is not part of the key),
 * up to the first rule with a conntrack match; std::map::insert keeps the
 * first rule of a repeated key. */
static void horus_build(const ochain_t *in, hzprog_t *h) {
  uint32_t set_fields = 0;
  hzent_t key;
  memset(&key, 0, sizeof key);        /* one HorusRule reused for every rule (Utils.cpp:604) */
  h->n = 0;
  for (int i = 0; i < in->nrules && i < HZ_MAX; i++) {
    const prule_t *r = &in->rules[i];
    if (r->ct_set) break;             /* fromRuleToHorusKeyValue returns false: stop */
    uint32_t f = 0;
    if (r->src_set && r->src.netmask == 32) { f |= ORC_HZ_SRCIP; key.src = r->src.ip; }
    if (r->dst_set && r->dst.netmask == 32) { f |= ORC_HZ_DSTIP; key.dst = r->dst.ip; }
    if (r->proto_set) { f |= ORC_HZ_L4PROTO; key.proto = (uint8_t)r->proto; }
    if (r->sport_set) { f |= ORC_HZ_SRCPORT; key.sk = bswap16(r->sport); }
    if (r->dport_set) { f |= ORC_HZ_DSTPORT; key.dk = bswap16(r->dport); }
    key.action = r->action == 0 ? 0 : 1;
    key.rule = (uint32_t)i;           /* rule->getId(): dense ids (Q12) */
    if (i == 0) {
      if (!f) break;
      set_fields = f;
    }
    if (f != set_fields) break;
    int dup = 0;
    for (int k = 0; k < h->n && !dup; k++) {
      const hzent_t *e = &h->ent[k];
      dup = e->src == key.src && e->dst == key.dst && e->proto == key.proto && e->sk == key.sk && e->dk == key.dk;
    }
    if (!dup) h->ent[h->n++] = key;
  }
  h->fields = set_fields;
}

/* The Horus program a chain's updates rebuild: pcn-iptables INPUT -> [0];
 * pcn-firewall INGRESS (FORWARD slot) -> [0], EGRESS (OUTPUT slot) -> [1]. */
static int horus_slot(const orc_ctx *c, int chain) {
  if (c->service == ORC_SVC_FIREWALL) return chain == ORC_FORWARD ? 0 : chain == ORC_OUTPUT ? 1 : -1;
  return chain == ORC_INPUT ? 0 : -1;
}

/* The Horus program a batch's Parser calls: pcn-iptables ingress only (the
 * egress Parser's tail call lands on an empty program slot); pcn-firewall the
 * direction's own. */
static hzprog_t *horus_of_batch(orc_ctx *c, int dir) {
  hzprog_t *h = c->service == ORC_SVC_FIREWALL ? &c->hz[dir == ORC_INGRESS ? 0 : 1]
                                               : dir == ORC_INGRESS ? &c->hz[0] : NULL;
  return h && h->runtime ? h : NULL;
}

static void horus_reset(hzprog_t *h) {
  h->runtime = 0;                     /* the old program goes, and its counters with it */
  h->n = 0;
  h->fields = 0;
  memset(h->pkts, 0, sizeof h->pkts);
  memset(h->bytes, 0, sizeof h->bytes);
}

/* Chain::updateChain's Horus part, run for every chain update.
 * pcn-iptables (Chain.cpp:505-592): any update drops the program; an INPUT
 * update with horus on, >= 1 INPUT rule (MIN_RULE_SIZE_FOR_HORUS) and an empty
 * FORWARD rule list builds a new one.
 * pcn-firewall (Chain.cpp:232-306): an update of INGRESS / EGRESS rebuilds that
 * chain's own program when horus is on (always: Firewall.h:337) and the chain
 * has >= 1 rule, and the program keeps the conntrack setting it was compiled
 * with (modules/Horus.cpp:135-139; setConntrack does not reload it,
 * Firewall.cpp:151-191). */
static void horus_update(orc_ctx *c, int chain) {
  if (c->service == ORC_SVC_FIREWALL) {
    const int k = horus_slot(c, chain);
    if (k < 0) return;
    hzprog_t *h = &c->hz[k];
    horus_reset(h);
    if (!c->hz_enabled || c->ch[chain].nrules < 1) return;
    horus_build(&c->ch[chain], h);
    h->ct = c->fw_ct_mode != FW_CT_DISABLED;
    if (h->n >= 1) h->runtime = 1;
    return;
  }
  hzprog_t *h = &c->hz[0];
  horus_reset(h);
  if (chain != ORC_INPUT || !c->hz_enabled) return;
  if (c->ch[ORC_INPUT].nrules < 1 || c->ch[ORC_FORWARD].nrules != 0) return;
  horus_build(&c->ch[ORC_INPUT], h);
  if (h->n >= 1) h->runtime = 1;
}

int orc_set_horus(orc_ctx *c, int on) {
  c->hz_enabled = on != 0;
  return 0;
}

int orc_horus_info(orc_ctx *c, int chain, uint32_t out[5]) {
  const int k = horus_slot(c, chain);
  if (k < 0) return -EINVAL;
  const hzprog_t *h = &c->hz[k];
  out[0] = (uint32_t)c->hz_enabled; out[1] = (uint32_t)h->runtime;
  out[2] = (uint32_t)h->n; out[3] = h->fields; out[4] = (uint32_t)(h->runtime && h->ct);
  return 0;
}

int orc_read_horus_counters(orc_ctx *c, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n, int flush) {
  const int k = horus_slot(c, chain);
  if (k < 0) return -EINVAL;
  hzprog_t *h = &c->hz[k];
  for (uint32_t i = 0; i < n; i++) {
    const int ok = i < HZ_MAX;
    if (pkts) pkts[i] = ok ? h->pkts[i] : 0;
    if (bytes) bytes[i] = ok ? h->bytes[i] : 0;
    if (ok && flush) { h->pkts[i] = 0; h->bytes[i] = 0; }   /* Horus::flushCounters */
  }
  return 0;
}

/* The Horus key of the per-CPU packet struct; rs/rd are the Parser's
 * srcPort/dstPort as stored (wire bytes 34-35, 36-37).
 * pcn-iptables (Iptables_Horus_dp.c:112-133): the Parser writes the naturally
 * aligned struct (srcPort at bytes 10-11, dstPort at 12-13, byte 9 padding
 * that nothing writes), and Horus reads it through a packed declaration
 * (srcPort at 9-10, dstPort at 11-12).
 * pcn-firewall (Firewall_Horus_dp.c:112-133): both sides declare the struct
 * packed (Firewall_Parser_dp.c:32-43), so the key holds the ports as stored. */
static const hzent_t *horus_lookup(const orc_ctx *c, const hzprog_t *h, uint32_t saddr, uint32_t daddr,
                                   uint8_t proto, uint16_t rs, uint16_t rd) {
  const uint32_t F = h->fields;
  uint16_t sk = rs, dk = rd;
  if (c->service != ORC_SVC_FIREWALL) {
    sk = (uint16_t)((rs & 0xff) << 8);                /* bytes 9-10: [0, wire34] */
    dk = (uint16_t)((rs >> 8) | ((rd & 0xff) << 8));  /* bytes 11-12: [wire35, wire36] */
  }
  for (int k = 0; k < h->n; k++) {
    const hzent_t *e = &h->ent[k];
    if ((F & ORC_HZ_SRCIP) && e->src != saddr) continue;
    if ((F & ORC_HZ_DSTIP) && e->dst != daddr) continue;
    if ((F & ORC_HZ_L4PROTO) && e->proto != proto) continue;
    if ((F & ORC_HZ_SRCPORT) && e->sk != sk) continue;
    if ((F & ORC_HZ_DSTPORT) && e->dk != dk) continue;
    return e;
  }
  return NULL;
}

/* pcn-firewall Chain::setDefault (Chain.cpp:60-82): only the DefaultAction
 * program is reloaded -- no Chain::updateChain, so the rule modules, their
 * counters and the Horus program stay as they are. */
int orc_set_default(orc_ctx *c, int chain, int def) {
  if (chain < 0 || chain >= NCHAINS || (def != 0 && def != 1)) return -EINVAL;
  c->ch[chain].default_action = def;
  return 0;
}

int orc_set_service(orc_ctx *c, int service, int fw_ct_mode) {
  if (service != ORC_SVC_IPTABLES && service != ORC_SVC_FIREWALL) return -EINVAL;
  if (fw_ct_mode < FW_CT_DISABLED || fw_ct_mode > FW_CT_AUTOMATIC) return -EINVAL;
  /* pcn-firewall's horus_enabled is true from the start and has no knob
   * (Firewall.h:337); pcn-iptables' leaf is OFF by default (Iptables.h:185) */
  if (service != c->service) c->hz_enabled = service == ORC_SVC_FIREWALL;
  c->service = service;
  c->fw_ct_mode = fw_ct_mode;
  return 0;
}

int orc_set_localip(orc_ctx *c, const uint32_t *ips, uint32_t n) {
  if (n > 256) return -ENOSPC; /* ChainSelector_dp.c:54 hash(256) */
  memcpy(c->localip, ips, n * 4); c->nlocal = (int)n;
  return 0;
}

uint32_t orc_chain_nrw(orc_ctx *c, int chain) { return (uint32_t)c->ch[chain].nrw; }

void orc_index64(uint16_t out[64]) { build_index64(out); }

int orc_export_map(orc_ctx *c, int chain, int field, uint32_t *keys, uint8_t *plen,
                   uint64_t *vecs, uint32_t cap, uint32_t nrw) {
  if (chain < 0 || chain >= NCHAINS || field < 0 || field >= NFIELDS) return -EINVAL;
  ochain_t *ch = &c->ch[chain];
  omap_t *m = &ch->maps[field];
  if ((uint32_t)m->n > cap) return -ENOSPC;
  for (int k = 0; k < m->n; k++) {
    keys[k] = m->key[k]; plen[k] = m->plen[k];
    for (uint32_t w = 0; w < nrw; w++)
      vecs[(size_t)k * nrw + w] = (int)w < ch->vlen ? VEC(ch, m->vec[k])[w] : 0;
  }
  return m->n;
}

int orc_read_counters(orc_ctx *c, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n,
                      uint64_t *dp, uint64_t *db, int flush) {
  if (chain < 0 || chain >= NCHAINS) return -EINVAL;
  ochain_t *ch = &c->ch[chain];
  for (uint32_t i = 0; i < n; i++) {
    int ok = i < c->max_counted;
    if (pkts) pkts[i] = ok ? ch->pkts[i] : 0;
    if (bytes) bytes[i] = ok ? ch->bytes[i] : 0;
    if (ok && flush) { ch->pkts[i] = 0; ch->bytes[i] = 0; } /* ActionLookup.cpp:124-151 */
  }
  if (dp) *dp = ch->def_pkts;
  if (db) *db = ch->def_bytes;
  return 0;
}

/* ---------------- datapath ---------------- */

typedef struct {        /* per-CPU counters (percpu arrays) */
  uint64_t *pkts[NCHAINS], *bytes[NCHAINS];
  uint64_t dpk[NCHAINS], dby[NCHAINS];
  uint64_t ae_pkts[NCHAINS], ae_bytes[NCHAINS];   /* pkts_/bytes_acceptestablished_<Chain> */
  uint64_t *hz_pkts, *hz_bytes;                   /* pkts_horus / bytes_horus */
} pcpu_t;

static inline uint16_t be16(const uint8_t *p) { return (uint16_t)(p[0] << 8 | p[1]); }
static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

static int localip_has(const orc_ctx *c, uint32_t ip) {
  for (int i = 0; i < c->nlocal; i++) if (c->localip[i] == ip) return 1;
  return 0;
}

/* ConntrackLabel_dp.c:190-531 with an empty `connections` table (stateless). */
static int ct_label_empty(int proto, uint8_t flags, int icmp_type) {
  if (proto == 6) /* TCP_MISS :372-383 */
    return ((flags & 0x02) && (flags | 0x02) == 0x02) ? CT_NEW : CT_INVALID;
  if (proto == 17) return CT_NEW;            /* UDP_MISS :428-432 */
  if (proto == 1) return icmp_type == 8 ? CT_NEW : CT_INVALID;
  return CT_INVALID;                         /* :562-566 */
}

/* ---------------- conntrack (stateful mode) ----------------
 * The `connections` table (Iptables_ConntrackLabel_dp.c:111-113: BPF lru_hash
 * of 65536 `ct_k` -> `ct_v`), ConntrackLabel (:190-531) and
 * ConntrackTableUpdate (Iptables_ConntrackTableUpdate_dp.c:141-655), run for
 * one packet at a time in batch order, as one CPU would run them.
 *  - Entries never expire: the datapath writes `ttl` but nothing compares it
 *    (the control plane only lists it, Iptables.cpp:527-566).  `now` is the
 *    `timestamp` percpu value the control plane refreshes every second
 *    (modules/ConntrackTableUpdate.cpp:108-137); tests set it explicitly.
 *  - Capacity (the lru_hash's 65536 entries, :112): restated at batch
 *    granularity.  A packet touches its table key (its own, or for an ICMP
 *    error the quoted one) when the entry is live after the packet; the touch
 *    stamp is (batch sequence << 32 | index in the batch).  After a batch, if
 *    more than max_entries are live, the live entries with the oldest stamps
 *    are deleted down to max_entries (exact LRU over the touches; within a
 *    batch nothing is evicted, so a connection the kernel would evict mid-batch
 *    stays visible to the batch's later packets).  The kernel's own LRU is
 *    approximate (per-CPU free lists, reference bits), so no order is more
 *    faithful than this one; the GPU applies the same rule (conntrack.hip).
 *  - `packet` is one per-CPU struct shared by ingress and egress
 *    (Iptables_Parser_dp.c:44-56): the Parser writes srcPort/dstPort only for
 *    TCP/UDP (:122-143), so an ICMP packet's conntrack key carries the ports
 *    of the last TCP/UDP packet parsed before it (quirk Q4). */
enum { ST_NEW = 0, ST_ESTABLISHED, ST_RELATED, ST_INVALID, ST_SYN_SENT, ST_SYN_RECV,
       ST_FIN_WAIT_1, ST_FIN_WAIT_2, ST_LAST_ACK, ST_TIME_WAIT };
#define TCPHDR_FIN 0x01
#define TCPHDR_SYN 0x02
#define TCPHDR_RST 0x04
#define TCPHDR_ACK 0x10
#define HEX_BE_ONE 0x1000000u
/* ConntrackTableUpdate_dp.c:38-48 (ns) */
#define UDP_ESTABLISHED_TIMEOUT 180000000000ull
#define UDP_NEW_TIMEOUT 30000000000ull
#define ICMP_TIMEOUT 30000000000ull
#define TCP_ESTABLISHED 432000000000000ull
#define TCP_SYN_SENT 120000000000ull
#define TCP_SYN_RECV 60000000000ull
#define TCP_LAST_ACK 30000000000ull
#define TCP_FIN_WAIT 120000000000ull

typedef struct { uint32_t src, dst; uint8_t proto; uint16_t sport, dport; } ctk_t;  /* struct ct_k */
typedef struct { uint64_t ttl; uint8_t state, ipRev, portRev; uint32_t seq; } ctv_t; /* struct ct_v */
typedef struct { ctk_t k; ctv_t v; int used; uint64_t touch; } cte_t;    /* used: 0 empty, 1 live, 2 deleted */

struct ctstate {
  cte_t *tab; size_t cap, live, used;
  uint64_t now;
  uint64_t bseq, max_entries, evicted;  /* LRU at batch granularity (see above) */
  ctk_t tkey; int has_tkey;             /* the current packet's table key */
  /* the shared per-CPU `packet` struct: fields the Parser leaves stale */
  uint16_t sport, dport; uint32_t seq, ack; uint8_t flags;
};

static void ct_free(struct ctstate *t) {
  if (!t) return;
  free(t->tab); free(t);
}

static uint64_t ctk_hash(const ctk_t *k) {
  uint64_t h = ((uint64_t)k->src << 32 | k->dst) * 0x9E3779B97F4A7C15ull;
  h ^= ((uint64_t)k->proto << 32 | (uint64_t)k->sport << 16 | k->dport) * 0xC2B2AE3D27D4EB4Full;
  return h ^ (h >> 29);
}
static int ctk_eq(const ctk_t *a, const ctk_t *b) {
  return a->src == b->src && a->dst == b->dst && a->proto == b->proto && a->sport == b->sport &&
         a->dport == b->dport;
}
static cte_t *ct_find(struct ctstate *t, const ctk_t *k) {     /* connections.lookup */
  if (!t->cap) return NULL;
  for (size_t i = ctk_hash(k) & (t->cap - 1), s = 0; s < t->cap; s++, i = (i + 1) & (t->cap - 1)) {
    cte_t *e = &t->tab[i];
    if (e->used == 0) return NULL;
    if (e->used == 1 && ctk_eq(&e->k, k)) return e;
  }
  return NULL;
}
static void ct_grow(struct ctstate *t) {
  size_t oc = t->cap;
  cte_t *old = t->tab;
  t->cap = oc ? oc * 2 : 1024;
  t->tab = calloc(t->cap, sizeof(cte_t));
  t->used = t->live = 0;
  for (size_t i = 0; i < oc; i++) {
    if (old[i].used != 1) continue;
    size_t j = ctk_hash(&old[i].k) & (t->cap - 1);
    while (t->tab[j].used) j = (j + 1) & (t->cap - 1);
    t->tab[j] = old[i];
    t->used++; t->live++;
  }
  free(old);
}
/* connections.update (BPF_ANY) / .insert (BPF_NOEXIST: an existing key is left as is) */
static void ct_put(struct ctstate *t, const ctk_t *k, const ctv_t *v, int noexist) {
  cte_t *e = ct_find(t, k);
  if (e) { if (!noexist) e->v = *v; return; }
  if ((t->used + 1) * 2 > t->cap) ct_grow(t);
  size_t i = ctk_hash(k) & (t->cap - 1);
  while (t->tab[i].used == 1) i = (i + 1) & (t->cap - 1);
  if (t->tab[i].used == 0) t->used++;
  t->tab[i].k = *k; t->tab[i].v = *v; t->tab[i].used = 1;
  t->live++;
}
static void ct_delete(struct ctstate *t, const ctk_t *k) {        /* connections.delete */
  cte_t *e = ct_find(t, k);
  if (e) { e->used = 2; t->live--; }
}

typedef struct {          /* struct packetHeaders as the conntrack modules read it */
  uint32_t src, dst; uint8_t proto; uint16_t sport, dport; uint8_t flags; uint32_t seq, ack;
} ctpkt_t;

/* ConntrackLabel_dp.c:200-228 and ConntrackTableUpdate_dp.c:166-194: the key
 * orders IPs and ports as little-endian loads of their network-order bytes. */
static ctk_t ct_key(const ctpkt_t *p, uint8_t *ipRev, uint8_t *portRev) {
  ctk_t k;
  if (p->src <= p->dst) { k.src = p->src; k.dst = p->dst; *ipRev = 0; }
  else { k.src = p->dst; k.dst = p->src; *ipRev = 1; }
  k.proto = p->proto;
  if (p->sport < p->dport) { k.sport = p->sport; k.dport = p->dport; *portRev = 0; }
  else if (p->sport > p->dport) { k.sport = p->dport; k.dport = p->sport; *portRev = 1; }
  else { k.sport = p->sport; k.dport = p->dport; *portRev = *ipRev; }
  return k;
}
static inline int syn_only(uint8_t f) { return (f & TCPHDR_SYN) && (f | TCPHDR_SYN) == TCPHDR_SYN; }
static inline int ack_only(uint8_t f) { return (f & TCPHDR_ACK) && (f | TCPHDR_ACK) == TCPHDR_ACK; }
static inline int synack_only(uint8_t f) {
  return (f & TCPHDR_ACK) && (f & TCPHDR_SYN) && (f | (TCPHDR_SYN | TCPHDR_ACK)) == (TCPHDR_SYN | TCPHDR_ACK);
}
static inline uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

/* The key a labelled packet is tracked under for the LRU touch: its own, or
 * an ICMP error's quoted header's; none for packets that never reach the table
 * (short ICMP dropped, timestamp/info types, other protocols). */
static void ct_note_key(struct ctstate *t, const ctpkt_t *p, const uint8_t *f, uint32_t L) {
  uint8_t a, b;
  t->has_tkey = 0;
  if (p->proto == 6 || p->proto == 17) {
    t->tkey = ct_key(p, &a, &b);
    t->has_tkey = 1;
  } else if (p->proto == 1 && L >= 42) {
    const uint8_t type = f[34];
    if (type == 8 || type == 0) {
      t->tkey = ct_key(p, &a, &b);
      t->has_tkey = 1;
    } else if (!(type >= 13 && type <= 18) && L >= 70) {
      uint32_t is = ld32(f + 54), id = ld32(f + 58);
      uint16_t x = ld16(f + 62), y = ld16(f + 64);
      t->tkey = (ctk_t){is <= id ? is : id, is <= id ? id : is, f[51], x <= y ? x : y, x <= y ? y : x};
      t->has_tkey = 1;
    }
  }
}

/* After a batch: delete the least recently touched live entries down to
 * max_entries (0: unbounded); then the next batch's sequence number. */
static int cmp_touch(const void *a, const void *b) {
  const uint64_t x = (*(cte_t *const *)a)->touch, y = (*(cte_t *const *)b)->touch;
  return x < y ? -1 : x > y;
}
static void ct_end_batch(struct ctstate *t) {
  if (t->max_entries && t->live > t->max_entries) {
    cte_t **ls = malloc(t->live * sizeof *ls);
    size_t m = 0;
    for (size_t i = 0; i < t->cap; i++)
      if (t->tab[i].used == 1) ls[m++] = &t->tab[i];
    qsort(ls, m, sizeof *ls, cmp_touch);
    const size_t k = m - t->max_entries;
    for (size_t i = 0; i < k; i++) ls[i]->used = 2;
    t->live -= k;
    t->evicted += k;
    free(ls);
  }
  t->bseq++;
}

/* ConntrackLabel_dp.c:190-531: the packet's connStatus, or -1 for RX_DROP
 * (the ICMP length checks, :441-443, :486-505). */
static int ct_label(struct ctstate *t, const ctpkt_t *p, const uint8_t *f, uint32_t L) {
  uint8_t ipRev, portRev;
  ctk_t key = ct_key(p, &ipRev, &portRev);
  cte_t *e;
  if (p->proto == 6) {
    e = ct_find(t, &key);
    if (e && e->v.ipRev == ipRev && e->v.portRev == portRev) {            /* TCP_FORWARD :245 */
      if (p->flags & TCPHDR_RST) return ST_ESTABLISHED;
      uint8_t s = e->v.state;
      if (s == ST_SYN_SENT) return syn_only(p->flags) ? ST_NEW : ST_INVALID;
      if (s == ST_SYN_RECV) return ack_only(p->flags) && p->ack == e->v.seq ? ST_ESTABLISHED : ST_INVALID;
      if (s == ST_ESTABLISHED || s == ST_FIN_WAIT_1 || s == ST_FIN_WAIT_2 || s == ST_LAST_ACK)
        return ST_ESTABLISHED;
      if (s == ST_TIME_WAIT && syn_only(p->flags)) return ST_NEW;
      return ST_INVALID;
    }
    if (e && e->v.ipRev != ipRev && e->v.portRev != portRev) {            /* TCP_REVERSE :310 */
      if (p->flags & TCPHDR_RST) return ST_ESTABLISHED;
      uint8_t s = e->v.state;
      if (s == ST_SYN_SENT || s == ST_SYN_RECV)
        return synack_only(p->flags) && p->ack == e->v.seq ? ST_ESTABLISHED : ST_INVALID;
      if (s == ST_ESTABLISHED || s == ST_FIN_WAIT_1 || s == ST_FIN_WAIT_2 || s == ST_LAST_ACK)
        return ST_ESTABLISHED;
      if (s == ST_TIME_WAIT && syn_only(p->flags)) return ST_NEW;
      return ST_INVALID;
    }
    return syn_only(p->flags) ? ST_NEW : ST_INVALID;                      /* TCP_MISS :372-383 */
  }
  if (p->proto == 17) {
    e = ct_find(t, &key);
    if (e && e->v.ipRev == ipRev && e->v.portRev == portRev)              /* UDP_FORWARD */
      return e->v.state == ST_NEW ? ST_NEW : ST_ESTABLISHED;
    if (e && e->v.ipRev != ipRev && e->v.portRev != portRev) return ST_ESTABLISHED; /* UDP_REVERSE */
    return ST_NEW;                                                       /* UDP_MISS */
  }
  if (p->proto == 1) {
    if (L < 42) return -1;
    uint8_t type = f[34];
    if (type == 8) return ST_NEW;
    if (type == 0) {
      e = ct_find(t, &key);
      if (!e) return ST_INVALID;
      if (e->v.ipRev != ipRev && e->v.portRev != portRev) return ST_ESTABLISHED;
      /* else ICMP_MISS (:468) */
    }
    if (type >= 13 && type <= 18) return ST_INVALID;
    if (L < 62) return -1;
    /* the encapsulated IP header and 8 bytes of its payload (:491-529) */
    uint32_t is = ld32(f + 54), id = ld32(f + 58);
    ctk_t ik;
    if (is <= id) { ik.src = is; ik.dst = id; } else { ik.src = id; ik.dst = is; }
    ik.proto = f[51];
    if (L < 70) return -1;
    uint16_t a = ld16(f + 62), b = ld16(f + 64);
    if (a <= b) { ik.sport = a; ik.dport = b; } else { ik.sport = b; ik.dport = a; }
    return ct_find(t, &ik) ? ST_RELATED : ST_INVALID;
  }
  return ST_INVALID;                                                     /* :562-566 */
}

/* ConntrackTableUpdate_dp.c:141-655, run for every accepted labelled packet. */
static void ct_update(struct ctstate *t, const ctpkt_t *p, const uint8_t *f, int label) {
  if (label == ST_INVALID) return;
  uint8_t ipRev, portRev;
  ctk_t key = ct_key(p, &ipRev, &portRev);
  const uint64_t now = t->now;
  ctv_t nv = {0, 0, 0, 0, 0};
  if (p->proto == 6) {
    if (p->flags & TCPHDR_RST) return;
    cte_t *e = ct_find(t, &key);
    int dir = !e ? 0 : (e->v.ipRev == ipRev && e->v.portRev == portRev) ? 1
                     : (e->v.ipRev != ipRev && e->v.portRev != portRev) ? 2 : 0;
    if (dir) {
      ctv_t *v = &e->v;
      if (v->state == ST_SYN_SENT) {
        if (dir == 1) { if (syn_only(p->flags)) v->ttl = now + TCP_SYN_SENT; return; }
        if (synack_only(p->flags) && p->ack == v->seq) {
          v->state = ST_SYN_RECV; v->ttl = now + TCP_SYN_RECV; v->seq = p->seq + HEX_BE_ONE;
        }
        return;
      }
      if (v->state == ST_SYN_RECV) {
        if (dir == 1) {
          if (ack_only(p->flags) && p->ack == v->seq) { v->state = ST_ESTABLISHED; v->ttl = now + TCP_ESTABLISHED; }
        } else if (synack_only(p->flags) && p->ack == v->seq) {
          v->ttl = now + TCP_SYN_RECV;
        }
        return;
      }
      if (v->state == ST_ESTABLISHED) {
        if (p->flags & TCPHDR_FIN) { v->state = ST_FIN_WAIT_1; v->ttl = now + TCP_FIN_WAIT; v->seq = p->ack; }
        else v->ttl = now + TCP_ESTABLISHED;
        return;
      }
      if (v->state == ST_FIN_WAIT_1) {
        if ((p->flags & TCPHDR_ACK) && p->seq == v->seq) { v->state = ST_FIN_WAIT_2; v->ttl = now + TCP_FIN_WAIT; }
        else return;
        /* no goto: falls into the FIN_WAIT_2 test (:259-281) */
      }
      if (v->state == ST_FIN_WAIT_2) {
        if (p->flags & TCPHDR_FIN) { v->state = ST_LAST_ACK; v->ttl = now + TCP_LAST_ACK; v->seq = p->ack; }
        else v->ttl = now + TCP_FIN_WAIT;
        return;
      }
      if (v->state == ST_LAST_ACK) {
        if ((p->flags & TCPHDR_ACK) && p->seq == v->seq) v->state = ST_TIME_WAIT;
        v->ttl = now + TCP_LAST_ACK;
        return;
      }
      if (v->state == ST_TIME_WAIT) {
        if (label != ST_NEW) return;
        /* goto TCP_MISS */
      } else {
        return;
      }
    }
    if (syn_only(p->flags)) {                                            /* TCP_MISS :540-555 */
      nv.state = ST_SYN_SENT; nv.ttl = now + TCP_SYN_SENT; nv.seq = p->seq + HEX_BE_ONE;
      nv.ipRev = ipRev; nv.portRev = portRev;
      ct_put(t, &key, &nv, 0);
    }
    return;
  }
  if (p->proto == 17) {
    cte_t *e = ct_find(t, &key);
    if (e && e->v.ipRev == ipRev && e->v.portRev == portRev) {
      e->v.ttl = now + (e->v.state == ST_NEW ? UDP_NEW_TIMEOUT : UDP_ESTABLISHED_TIMEOUT);
      return;
    }
    if (e && e->v.ipRev != ipRev && e->v.portRev != portRev) {
      if (e->v.state == ST_NEW) { e->v.ttl = now + UDP_NEW_TIMEOUT; e->v.state = ST_ESTABLISHED; }
      else e->v.ttl = now + UDP_ESTABLISHED_TIMEOUT;
      return;
    }
    nv.ttl = now + UDP_NEW_TIMEOUT; nv.state = ST_NEW; nv.ipRev = ipRev; nv.portRev = portRev;
    ct_put(t, &key, &nv, 1);                                             /* UDP_MISS insert */
    return;
  }
  if (p->proto == 1) {
    uint8_t type = f[34];
    if (type == 8) {
      nv.ttl = now + ICMP_TIMEOUT; nv.state = ST_NEW; nv.ipRev = ipRev; nv.portRev = portRev;
      ct_put(t, &key, &nv, 1);
    } else if (type == 0) {
      ct_delete(t, &key);
    }
  }
}

/* ChainRule::acceptEstablishedOptimizationFound (ChainRule.cpp:218-238): rule 0
 * is exactly {conntrack ESTABLISHED, action ACCEPT}. */
static int ae_found(const ochain_t *ch) {
  if (ch->nrules == 0) return 0;
  const prule_t *r = &ch->rules[0];
  return r->ct_set && r->ct == CT_ESTABLISHED && r->action == 1 && !r->src_set && !r->dst_set &&
         !r->proto_set && !r->sport_set && !r->dport_set && !r->flags_set_ && !r->in_set && !r->out_set;
}

/* default action tail: Program.cpp:88-111 (+ default counters from each module) */
static inline int default_verdict(const ochain_t *ch, pcpu_t *pc, int chain, uint32_t L,
                                  int32_t *rid) {
  pc->dpk[chain] += 1; pc->dby[chain] += L;
  *rid = -1;
  return ch->default_action == 0 ? RX_DROP : RX_OK;
}

/* st != NULL: stateful conntrack (labels from and updates to st, one packet
 * at a time); else labels come from ct_in or an empty table. */
static int classify_one(const orc_ctx *c, int dir, int hook, const uint8_t *f, uint32_t L, uint16_t port,
                        int ct_in, pcpu_t *pc, int32_t *rid, struct ctstate *st, int *label, uint16_t *hzp,
                        const hzprog_t *hz) {
  *rid = -2;
  *label = 255;
  /* TC hook: the receive path strips the outer 802.1Q / 802.1ad tag before
   * the program runs (skb_vlan_untag; a frame too short to hold the tag is
   * dropped there), and packet_len = skb->len no longer counts it. */
  uint8_t untagged[128];
  if (hook == ORC_HOOK_TC && L >= 14 && (be16(f + 12) == 0x8100 || be16(f + 12) == 0x88A8)) {
    if (L < 18) return RX_DROP;
    uint32_t keep = L - 4 < sizeof untagged ? L - 4 : (uint32_t)sizeof untagged;
    memcpy(untagged, f, 12);
    memcpy(untagged + 12, f + 16, keep - 12);
    f = untagged;
    L -= 4;
  }
  /* Parser_dp.c:94-153 */
  if (L < 14) return RX_DROP;
  if (be16(f + 12) != 0x0800) return RX_OK;
  if (L < 34) return RX_DROP;
  uint32_t saddr = ld32(f + 26), daddr = ld32(f + 30);
  int proto = f[23];
  uint16_t sport = 0, dport = 0;
  uint8_t flags = 0;
  if (proto == 6) {
    if (L < 54) return RX_DROP;
    memcpy(&sport, f + 34, 2); memcpy(&dport, f + 36, 2);
    flags = f[47];
    if (st) { st->sport = sport; st->dport = dport; st->seq = ld32(f + 38); st->ack = ld32(f + 42); st->flags = flags; }
  } else if (proto == 17) {
    if (L < 42) return RX_DROP;
    memcpy(&sport, f + 34, 2); memcpy(&dport, f + 36, 2);
    if (st) { st->sport = sport; st->dport = dport; }
  }
  if (!st && hzp && (proto == 6 || proto == 17)) { hzp[0] = sport; hzp[1] = dport; }
  ctpkt_t cp;
  if (st) cp = (ctpkt_t){saddr, daddr, (uint8_t)proto, st->sport, st->dport, st->flags, st->seq, st->ack};
  /* Horus (pcn-iptables Parser_dp.c:145-147 -> Horus_dp.c:97-167, ingress
   * only: the egress Parser's tail call lands on an empty program slot;
   * pcn-firewall Firewall_Parser_dp.c:154-157 -> Firewall_Horus_dp.c:97-175,
   * each direction its own).  hz: the batch's program in place, or NULL. */
  int pass_labeling = 0, chain = -1, ct;
  const int fwsvc = c->service == ORC_SVC_FIREWALL;
  if (hz) {
    uint16_t rs = sport, rd = dport;                       /* written by this packet */
    if (proto != 6 && proto != 17) {                       /* stale (Q4) */
      rs = st ? st->sport : hzp ? hzp[0] : 0;
      rd = st ? st->dport : hzp ? hzp[1] : 0;
    }
    const hzent_t *e = horus_lookup(c, hz, saddr, daddr, (uint8_t)proto, rs, rd);
    if (e) {
      pc->hz_pkts[e->rule] += 1; pc->hz_bytes[e->rule] += L;
      *rid = ORC_RID_HORUS0 - (int32_t)e->rule;
      if (e->action == 0) return RX_DROP;
      pass_labeling = 1;                                   /* PASS_LABELING -> ConntrackLabel */
      if (!fwsvc) goto labeling;
      /* pcn-firewall, compiled with conntrack off: RX_OK (Firewall_Horus_dp.c:162-164);
       * with it on, PASS_LABELING tail-calls ConntrackLabel (:157-161), which
       * setConntrack(OFF) has deleted since (Firewall.cpp:163-171): the tail
       * call fails and the program returns RX_DROP */
      if (!hz->ct) return RX_OK;
      if (c->fw_ct_mode == FW_CT_DISABLED) return RX_DROP;
    } else if (fwsvc && c->fw_ct_mode == FW_CT_DISABLED) {
      /* a miss always tail-calls ConntrackLabel (Firewall_Horus_dp.c:170-174):
       * with conntrack off that program does not exist, so RX_DROP */
      return RX_DROP;
    }
  }
  /* ports as the NBO u16 the eBPF hash keys hold; the maps store ntohs(port) */
  sport = (uint16_t)(sport >> 8 | sport << 8);
  dport = (uint16_t)(dport >> 8 | dport << 8);

  if (c->service == ORC_SVC_FIREWALL) {
    /* pcn-firewall: Firewall_Parser_dp.c:94-165 -> [ConntrackLabel, when the
     * conntrack mode is not DISABLED (modules/Parser.cpp:41-45)] ->
     * ChainForwarder (Firewall_ChainForwarder_dp.c:20-42).  The chain is the
     * program's direction: INGRESS or EGRESS, kept in the FORWARD / OUTPUT
     * slots.  No localip, no allow logic. */
    chain = dir == ORC_INGRESS ? ORC_FORWARD : ORC_OUTPUT;
    if (c->fw_ct_mode == FW_CT_DISABLED) st = NULL;   /* ConntrackTableUpdate: "conntrack disabled - pass" */
    ct = ct_in >= 0 ? ct_in : CT_NEW; /* DISABLED: connStatus is never written (per-CPU zero) */
    if (c->fw_ct_mode != FW_CT_DISABLED) {
      if (st) {
        ct_note_key(st, &cp, f, L);
        ct = ct_label(st, &cp, f, L);                  /* Firewall_ConntrackLabel_dp.c:116-460 */
        if (ct < 0) return RX_DROP;
      } else {
        int icmp_type = -1;                            /* the same ICMP length checks */
        if (proto == 1) {
          if (L < 42) return RX_DROP;
          icmp_type = f[34];
          if (icmp_type != 8 && icmp_type != 0 && !(icmp_type >= 13 && icmp_type <= 18) && L < 70) return RX_DROP;
        }
        ct = ct_in >= 0 ? ct_in : ct_label_empty(proto, flags, icmp_type);
      }
      *label = ct;
      /* PASS_LABELING (a Horus ACCEPT) -> ConntrackTableUpdate -> RX_OK in
       * both modes (Firewall_ConntrackLabel_dp.c:463-489) */
      if (pass_labeling) {
        if (st) ct_update(st, &cp, f, ct);
        return RX_OK;
      }
      /* _CONNTRACK_MODE == 2 (AUTOMATIC): ESTABLISHED -> ConntrackTableUpdate
       * -> RX_OK, before any chain and without counters
       * (Firewall_ConntrackLabel_dp.c:474-478) */
      if (c->fw_ct_mode == FW_CT_AUTOMATIC && ct == CT_ESTABLISHED) {
        *rid = -3;
        if (st) ct_update(st, &cp, f, ct);
        return RX_OK;
      }
    }
    *label = ct;
    if (c->ch[chain].nrules == 0) {
      /* _NR_ELEMENTS_<CHAIN> == 0: DefaultAction (Firewall_DefaultAction_dp.c:37-43) */
      int v = default_verdict(&c->ch[chain], pc, chain, L, rid);
      if (st && v == RX_OK) ct_update(st, &cp, f, ct);
      return v;
    }
    goto rules;
  }
  /* ChainSelector_dp.c:131-298 */
  if (dir == ORC_INGRESS) {
    const ochain_t *in = &c->ch[ORC_INPUT], *fw = &c->ch[ORC_FORWARD];
    if (in->default_action == 1 && fw->default_action == 1 && in->nrules == 0 &&
        fw->nrules == 0) { /* _INGRESS_ALLOWLOGIC, modules/ChainSelector.cpp:190-202 */
      chain = -1; pass_labeling = 1;
    } else {
      chain = localip_has(c, daddr) ? ORC_INPUT : ORC_FORWARD;
    }
  } else {
    if (!localip_has(c, saddr)) return RX_OK; /* PASS */
    chain = ORC_OUTPUT;
  }
  if (chain >= 0 && c->ch[chain].nrules == 0) {
    pc->dpk[chain] += 1; pc->dby[chain] += L;
    *rid = -1;
    if (c->ch[chain].default_action == 0) return RX_DROP; /* DROP_NO_LABELING */
    pass_labeling = 1;
  }
labeling:
  if (st) {
    ct_note_key(st, &cp, f, L);
    ct = ct_label(st, &cp, f, L);                    /* ConntrackLabel_dp.c:190-531 */
    if (ct < 0) return RX_DROP;
    *label = ct;
    /* PASS_LABELING → ChainForwarder → ConntrackTableUpdate → RX_OK */
    if (pass_labeling) { ct_update(st, &cp, f, ct); return RX_OK; }
    /* _CONNTRACK_MODE_<CHAIN> == ON: accept established (ConntrackLabel_dp.c:580-616) */
    if (c->ae[chain] && ct == ST_ESTABLISHED) {
      pc->ae_pkts[chain] += 1; pc->ae_bytes[chain] += L;
      *rid = -3;
      ct_update(st, &cp, f, ct);
      return RX_OK;
    }
  } else {
    /* ConntrackLabel_dp.c:436-531: ICMP length checks (stateless: empty table) */
    int icmp_type = -1;
    if (proto == 1) {
      if (L < 42) return RX_DROP;
      icmp_type = f[34];
      if (icmp_type != 8 && icmp_type != 0 && !(icmp_type >= 13 && icmp_type <= 18)) {
        if (L < 62) return RX_DROP;
        if (L < 70) return RX_DROP;
      }
    }
    ct = ct_in >= 0 ? ct_in : ct_label_empty(proto, flags, icmp_type);
    *label = ct;
    if (pass_labeling) return RX_OK; /* ChainForwarder → ConntrackTableUpdate → RX_OK */
    if (c->ae[chain] && ct == CT_ESTABLISHED) {
      pc->ae_pkts[chain] += 1; pc->ae_bytes[chain] += L;
      *rid = -3;
      return RX_OK;
    }
  }

rules:;
  const ochain_t *ch = &c->ch[chain];
  int nrw = ch->nrw;
  uint64_t v[1024];
  uint64_t *vv = nrw <= 1024 ? v : malloc((size_t)nrw * 8);
  for (int i = 0; i < nrw; i++) vv[i] = 0x7FFFFFFFFFFFFFFFull; /* ChainSelector_dp.c:205-218 */
  int verdict = -1;
  for (int fld = 0; fld < NFIELDS && verdict < 0; fld++) {
    if (!ch->present[fld]) continue;
    int e = -1;
    switch (fld) {
    case F_CT: /* ConntrackMatch_dp.c:90-153 */
      if (ct < 0 || ct > 3) { verdict = RX_DROP; *rid = -2; continue; }
      e = ch->ct_tab[ct]; break;
    case F_IPSRC: e = trie_lookup(ch->trie[0], saddr); break; /* IpLookup_dp.c:98-104 */
    case F_IPDST: e = trie_lookup(ch->trie[1], daddr); break;
    case F_PROTO: /* L4ProtocolLookup_dp.c:95-103 */
      e = ch->proto_tab[proto];
      if (e < 0) e = ch->proto_tab[0];
      break;
    case F_SPORT: case F_DPORT: /* L4PortLookup_dp.c:99-135 */
      if (proto != 6 && proto != 17) continue;
      e = fld == F_SPORT ? ch->sport_tab[sport] : ch->dport_tab[dport];
      if (e < 0) e = fld == F_SPORT ? ch->sport_wild : ch->dport_wild;
      break;
    case F_IFACE: /* InterfaceLookup_dp.c:103-135 */
      e = ch->iface_tab[port];
      if (e < 0) e = ch->iface_wild;
      break;
    case F_FLAGS: /* TcpFlagsLookup_dp.c:93-110 */
      if (proto != 6) continue;
      e = ch->flags_tab[flags];
      break;
    }
    if (e < 0) { verdict = default_verdict(ch, pc, chain, L, rid); break; }
    const uint64_t *ev = ch->pool + (size_t)e * ch->vlen;
    int allzero = 1;
    for (int i = 0; i < nrw; i++) { vv[i] &= ev[i]; if (vv[i]) allzero = 0; }
    if (allzero) verdict = default_verdict(ch, pc, chain, L, rid);
  }
  if (verdict < 0) {
    /* BitScan_dp.c:88-110 */
    int rule = -1;
    for (int i = 0; i < nrw; i++) {
      uint64_t b = vv[i];
      if (b) {
        int idx = (int)(((b ^ (b - 1)) * 0x03f79d71b4cb0a89ull) >> 58);
        rule = c->index64[idx] + i * 63;
        break;
      }
    }
    if (rule < 0) {
      verdict = default_verdict(ch, pc, chain, L, rid);
    } else if ((uint32_t)rule >= c->max_action) { /* ActionLookup_dp.c:90-94 lookup miss */
      verdict = RX_DROP; *rid = -2;
    } else {
      /* ActionLookup_dp.c:96-111 */
      if ((uint32_t)rule < c->max_counted) { pc->pkts[chain][rule] += 1; pc->bytes[chain][rule] += L; }
      *rid = rule;
      verdict = ch->actions[rule] == 0 ? RX_DROP : RX_OK;
    }
  }
  if (vv != v) free(vv);
  /* ActionLookup / default ACCEPT → ConntrackTableUpdate (ActionLookup_dp.c:100-104, Program.cpp:88-111) */
  if (st && verdict == RX_OK) ct_update(st, &cp, f, ct);
  return verdict;
}

typedef struct {
  const orc_ctx *c; int dir; int hook; const uint8_t *frames; const uint32_t *offsets; const uint16_t *lens;
  uint32_t stride, fixed_len; const uint16_t *in_port; uint16_t const_port; const uint8_t *ct;
  uint64_t lo, hi; uint8_t *verdicts; int32_t *rule_ids; pcpu_t pc; struct ctstate *st; uint8_t *labels;
  uint16_t *hzp;   /* stale ports for Horus keys while conntrack is off (NULL: not tracked) */
  const hzprog_t *hz;   /* the batch's Horus program, or NULL */
} job_t;

static void *run_job(void *arg) {
  job_t *j = arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint8_t *f = j->frames + (j->offsets ? j->offsets[i] : i * (uint64_t)j->stride);
    uint32_t L = j->lens ? j->lens[i] : j->fixed_len;
    uint16_t port = j->in_port ? j->in_port[i] : j->const_port;
    int ct = j->ct ? j->ct[i] : -1;
    int32_t rid;
    int lab;
    if (j->st) j->st->has_tkey = 0;
    int v = classify_one(j->c, j->dir, j->hook, f, L, port, ct, &j->pc, &rid, j->st, &lab, j->hzp, j->hz);
    if (j->st && j->st->has_tkey) {         /* the LRU touch: the entry is live after this packet */
      cte_t *e = ct_find(j->st, &j->st->tkey);
      if (e) e->touch = j->st->bseq << 32 | i;
    }
    if (j->labels) j->labels[i] = (uint8_t)lab;
    j->verdicts[i] = v == RX_DROP ? 0 : 1;
    if (j->rule_ids) j->rule_ids[i] = rid;
  }
  return NULL;
}

int orc_classify(orc_ctx *c, int dir, int hook, const uint8_t *frames, const uint32_t *offsets,
                 const uint16_t *lens, uint32_t stride, uint32_t fixed_len,
                 const uint16_t *in_port, uint16_t const_port, const uint8_t *ct_status,
                 uint64_t n, uint8_t *verdicts, int32_t *rule_ids, int nthreads) {
  return orc_classify_labels(c, dir, hook, frames, offsets, lens, stride, fixed_len, in_port, const_port,
                             ct_status, n, verdicts, rule_ids, NULL, nthreads);
}

int orc_classify_labels(orc_ctx *c, int dir, int hook, const uint8_t *frames, const uint32_t *offsets,
                        const uint16_t *lens, uint32_t stride, uint32_t fixed_len,
                        const uint16_t *in_port, uint16_t const_port, const uint8_t *ct_status,
                        uint64_t n, uint8_t *verdicts, int32_t *rule_ids, uint8_t *labels, int nthreads) {
  if (c->ct && ct_status) return -EINVAL;   /* labels come from the table */
  if (c->ct) nthreads = 1;                   /* one packet at a time, in batch order */
  /* with horus on, the Parser's stale ports (read by Horus keys) are tracked
   * from packet to packet: one packet at a time too.  They are tracked only
   * while horus is on (or conntrack, which keeps its own): the GPU does the same. */
  uint16_t *hzp = c->hz_enabled && !c->ct ? c->hz_stale : NULL;
  if (hzp) nthreads = 1;
  hzprog_t *hz = horus_of_batch(c, dir);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  job_t *jobs = calloc((size_t)nthreads, sizeof(job_t));
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job_t *j = &jobs[t];
    *j = (job_t){c, dir, hook, frames, offsets, lens, stride, fixed_len, in_port, const_port, ct_status,
                 n * t / nthreads, n * (t + 1) / nthreads, verdicts, rule_ids,
                 {{0}, {0}, {0}, {0}, {0}, {0}, NULL, NULL}, c->ct, labels, hzp, hz};
    for (int k = 0; k < NCHAINS; k++) {
      j->pc.pkts[k] = calloc(c->max_counted, 8);
      j->pc.bytes[k] = calloc(c->max_counted, 8);
    }
    j->pc.hz_pkts = calloc(HZ_MAX, 8);
    j->pc.hz_bytes = calloc(HZ_MAX, 8);
  }
  for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, run_job, &jobs[t]);
  run_job(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  /* control plane sums per-CPU counters (ActionLookup.cpp:78-96) */
  for (int t = 0; t < nthreads; t++) {
    for (int k = 0; k < NCHAINS; k++) {
      for (uint32_t r = 0; r < c->max_counted; r++) {
        c->ch[k].pkts[r] += jobs[t].pc.pkts[k][r];
        c->ch[k].bytes[r] += jobs[t].pc.bytes[k][r];
      }
      c->ch[k].def_pkts += jobs[t].pc.dpk[k];
      c->ch[k].def_bytes += jobs[t].pc.dby[k];
      c->ae_pkts[k] += jobs[t].pc.ae_pkts[k];
      c->ae_bytes[k] += jobs[t].pc.ae_bytes[k];
      free(jobs[t].pc.pkts[k]); free(jobs[t].pc.bytes[k]);
    }
    for (int r = 0; hz && r < HZ_MAX; r++) {
      hz->pkts[r] += jobs[t].pc.hz_pkts[r];
      hz->bytes[r] += jobs[t].pc.hz_bytes[r];
    }
    free(jobs[t].pc.hz_pkts); free(jobs[t].pc.hz_bytes);
  }
  free(jobs); free(th);
  /* a batch that ran the table (pcn-firewall DISABLED does not) */
  if (c->ct && n && !(c->service == ORC_SVC_FIREWALL && c->fw_ct_mode == FW_CT_DISABLED)) ct_end_batch(c->ct);
  return 0;
}

/* ---------------- conntrack control ---------------- */

int orc_ct_enable(orc_ctx *c, int on) {
  if (on && !c->ct) {
    c->ct = calloc(1, sizeof(struct ctstate));
    if (!c->ct) return -ENOMEM;
    c->ct->bseq = 1;
    c->ct->max_entries = 65536;               /* connections: lru_hash of 65536 (ConntrackLabel_dp.c:112) */
  } else if (!on && c->ct) {
    ct_free(c->ct);
    c->ct = NULL;
  }
  return 0;
}

int orc_ct_set_time(orc_ctx *c, uint64_t ns) {
  if (!c->ct) return -EINVAL;
  c->ct->now = ns;
  return 0;
}

int orc_ct_set_max_entries(orc_ctx *c, uint64_t max) {
  if (!c->ct) return -EINVAL;
  c->ct->max_entries = max;
  return 0;
}

int orc_ct_info(orc_ctx *c, uint64_t out[4]) {
  if (!c->ct) return -EINVAL;
  out[0] = c->ct->live; out[1] = c->ct->evicted; out[2] = c->ct->max_entries; out[3] = c->ct->bseq;
  return 0;
}

static int cmp_entry(const void *a, const void *b) {
  const orc_ct_entry *x = a, *y = b;
  if (x->src_ip != y->src_ip) return x->src_ip < y->src_ip ? -1 : 1;
  if (x->dst_ip != y->dst_ip) return x->dst_ip < y->dst_ip ? -1 : 1;
  if (x->l4proto != y->l4proto) return x->l4proto < y->l4proto ? -1 : 1;
  if (x->sport != y->sport) return x->sport < y->sport ? -1 : 1;
  if (x->dport != y->dport) return x->dport < y->dport ? -1 : 1;
  return 0;
}

/* The live `connections` entries (Iptables::getSessionTableList reads them,
 * Iptables.cpp:527-566), as stored (key order fields), sorted by key. */
int orc_ct_dump(orc_ctx *c, orc_ct_entry *out, uint32_t cap) {
  if (!c->ct) return -EINVAL;
  struct ctstate *t = c->ct;
  if (t->live > cap) return -ENOSPC;
  uint32_t n = 0;
  for (size_t i = 0; i < t->cap; i++) {
    const cte_t *e = &t->tab[i];
    if (e->used != 1) continue;
    out[n++] = (orc_ct_entry){e->k.src, e->k.dst, e->k.sport, e->k.dport, e->k.proto, e->v.state,
                              e->v.ipRev, e->v.portRev, e->v.seq, e->v.ttl};
  }
  qsort(out, n, sizeof *out, cmp_entry);
  return (int)n;
}

/* ChainRule::applyAcceptEstablishedOptimization (ChainRule.cpp:211-216) →
 * Iptables::enable/disableAcceptEstablished (Iptables.cpp:351-449).  The
 * disable switch has no `break`: disabling INPUT also disables FORWARD and
 * OUTPUT, disabling FORWARD also disables OUTPUT. */
int orc_apply_accept_established(orc_ctx *c, int chain) {
  if (chain < 0 || chain >= NCHAINS) return -EINVAL;
  if (ae_found(&c->ch[chain])) {
    c->ae[chain] = 1;
  } else {
    for (int k = chain; k < NCHAINS; k++) c->ae[k] = 0;
  }
  return 0;
}

int orc_set_accept_established(orc_ctx *c, int chain, int on) {
  if (chain < 0 || chain >= NCHAINS) return -EINVAL;
  c->ae[chain] = on != 0;
  return 0;
}

int orc_get_accept_established(orc_ctx *c, int chain) {
  if (chain < 0 || chain >= NCHAINS) return -EINVAL;
  return c->ae[chain];
}

/* pkts_/bytes_acceptestablished_<Chain> (ConntrackLabel.cpp:38-112): read, and
 * flush when asked (ChainStats::fetchCounters for id 0, ChainStats.cpp:64-103). */
int orc_read_accept_established(orc_ctx *c, int chain, uint64_t *pkts, uint64_t *bytes, int flush) {
  if (chain < 0 || chain >= NCHAINS) return -EINVAL;
  if (pkts) *pkts = c->ae_pkts[chain];
  if (bytes) *bytes = c->ae_bytes[chain];
  if (flush) c->ae_pkts[chain] = c->ae_bytes[chain] = 0;
  return 0;
}
