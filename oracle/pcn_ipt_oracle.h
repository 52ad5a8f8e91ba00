/*
 * pcn_ipt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference pcn-iptables classification path, used as
 * the parity checker for the MI355X datapath.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library.  The product library
 * (polycube_amd/libpcn_ipt.so) never links or calls it.
 *
 * Parity status: pinned by the reference's own integration-test scenarios
 * (src/services/pcn-iptables/test/local_test*.sh, transcribed into
 * tests/golden/scenarios.json) and by the reference BitScan index64 known-answer
 * table (modules/BitScan.cpp:32-49 → tests/golden/index64.json).  The reference
 * eBPF itself is unbuildable here (no BPF backend in llc, no bcc); see DESIGN.md.
 */
#ifndef PCN_IPT_ORACLE_H
#define PCN_IPT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Rule as received by the REST surface (ChainRuleJsonObject, iptables.yang:221-230).
 * NULL string / negative integer = field not set. */
typedef struct {
  const char *src;       /* "a.b.c.d" or "a.b.c.d/n" */
  const char *dst;
  const char *l4proto;   /* "TCP"/"UDP"/"ICMP"/"GRE" (either case) */
  const char *tcpflags;  /* e.g. "SYN !ACK" */
  const char *in_iface;  /* port name */
  const char *out_iface;
  const char *conntrack; /* "NEW"/"ESTABLISHED"/"RELATED"/"INVALID" */
  int32_t sport;         /* -1 unset, else 0..65535 */
  int32_t dport;
  int32_t action;        /* -1 unset (=> DROP), 0 DROP, 1 ACCEPT */
} orc_rule;

typedef struct orc_ctx orc_ctx;

enum { ORC_INPUT = 0, ORC_FORWARD = 1, ORC_OUTPUT = 2 };
enum { ORC_INGRESS = 0, ORC_EGRESS = 1 };
/* Attach point: XDP (frames as on the wire: an 802.1Q/802.1ad frame is not
 * IPv4, Iptables_Parser_dp.c:102-106) or TC (the kernel receive path has
 * removed the outer VLAN tag before the TC hook: skb_vlan_untag, Linux
 * net/core/dev.c, outside /root/reference; md->packet_len = skb->len,
 * polycubed/src/cube_tc.cpp:374-432). */
enum { ORC_HOOK_XDP = 0, ORC_HOOK_TC = 1 };

orc_ctx *orc_create(uint32_t max_counted_rules, uint32_t max_action_rules);
void orc_destroy(orc_ctx *c);
int orc_add_port(orc_ctx *c, const char *name, uint16_t index);
/* Replace a chain's rule list and default action and run the rule compiler
 * (Chain::updateChain).  Returns 0 or a negative errno. */
int orc_set_chain(orc_ctx *c, int chain, const orc_rule *rules, uint32_t n,
                  int default_action);
/* Service personality.  ORC_SVC_FIREWALL restates pcn-firewall
 * (src/services/pcn-firewall/src/datapaths/Firewall_*_dp.c): the same field
 * modules, BitScan and ActionLookup, but the chain is the program's direction
 * (INGRESS chain in the ORC_FORWARD slot, EGRESS in ORC_OUTPUT), there is no
 * localip / allow logic, and the ConntrackLabel stage (ICMP length checks,
 * labels) runs only when fw_ct_mode != FW_CT_DISABLED; FW_CT_AUTOMATIC
 * accepts ESTABLISHED packets before the chain, uncounted (rule id -3). */
enum { ORC_SVC_IPTABLES = 0, ORC_SVC_FIREWALL = 1 };
enum { FW_CT_DISABLED = 0, FW_CT_MANUAL = 1, FW_CT_AUTOMATIC = 2 };   /* defines.h:56-58 */
int orc_set_service(orc_ctx *c, int service, int fw_ct_mode);
int orc_set_localip(orc_ctx *c, const uint32_t *ips_nbo, uint32_t n);
/* Classify a batch (host pointers).  offsets==NULL => packet i at i*stride;
 * lens==NULL => every packet fixed_len bytes; in_port==NULL => const_port;
 * ct_status==NULL => connection status from an empty conntrack table. */
int orc_classify(orc_ctx *c, int direction, int hook, const uint8_t *frames,
                 const uint32_t *offsets, const uint16_t *lens, uint32_t stride,
                 uint32_t fixed_len, const uint16_t *in_port,
                 uint16_t const_port, const uint8_t *ct_status, uint64_t n,
                 uint8_t *verdicts, int32_t *rule_ids, int nthreads);
/* Horus.  pcn-iptables: the `horus` leaf (iptables.yang:112-118, OFF by
 * default, Iptables.h:185); orc_set_horus only sets the flag
 * (Iptables::setHorus, Iptables.cpp:400-406); like Chain::updateChain
 * (Chain.cpp:505-592) every orc_set_chain drops the Horus program and its
 * counters, and an INPUT update with horus on, INPUT rules and an empty
 * FORWARD chain builds a new one from the leading INPUT rules that set the
 * same fields (Utils.cpp:537-630).  pcn-firewall: on from the start with no
 * knob (Firewall.h:337; orc_set_horus still turns it off, for tests), one
 * program per chain, rebuilt by that chain's orc_set_chain (Chain.cpp:232-306)
 * and keeping the conntrack setting it was built with.  A hit reports rule id
 * ORC_RID_HORUS0 - <rule id> and counts into the program's counters
 * (Iptables_Horus_dp.c:80-90, 136-161; Firewall_Horus_dp.c:85-95, 137-167).
 * `chain` names the program: ORC_INPUT for pcn-iptables, ORC_FORWARD
 * (INGRESS) / ORC_OUTPUT (EGRESS) for pcn-firewall. */
#define ORC_RID_HORUS0 (-4096)
enum { ORC_HZ_SRCIP = 1, ORC_HZ_DSTIP = 2, ORC_HZ_L4PROTO = 4, ORC_HZ_SRCPORT = 8, ORC_HZ_DSTPORT = 16 };
int orc_set_horus(orc_ctx *c, int on);
/* out[0] enabled, out[1] runtime enabled, out[2] entries, out[3] set fields
 * (ORC_HZ_*), out[4] pcn-firewall: built with conntrack on */
int orc_horus_info(orc_ctx *c, int chain, uint32_t out[5]);
int orc_read_horus_counters(orc_ctx *c, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n, int flush);
/* pcn-firewall Chain::setDefault: the default action alone (no chain update) */
int orc_set_default(orc_ctx *c, int chain, int default_action);

/* orc_classify that also reports each packet's connection label (0..3, the
 * connStatus the field modules see), or 255 when the packet was decided
 * before labelling (parser, PASS, ICMP length checks). */
int orc_classify_labels(orc_ctx *c, int direction, int hook, const uint8_t *frames,
                        const uint32_t *offsets, const uint16_t *lens, uint32_t stride,
                        uint32_t fixed_len, const uint16_t *in_port, uint16_t const_port,
                        const uint8_t *ct_status, uint64_t n, uint8_t *verdicts,
                        int32_t *rule_ids, uint8_t *labels, int nthreads);
/* Per-rule counters (read-and-flush when flush != 0) and default counters. */
int orc_read_counters(orc_ctx *c, int chain, uint64_t *pkts, uint64_t *bytes,
                      uint32_t n, uint64_t *def_pkts, uint64_t *def_bytes,
                      int flush);
/* Export the compiled per-field map of a chain, in the order the reference
 * pushes it (std::map order / array index).  field: 0 conntrack, 1 ipsrc,
 * 2 ipdst, 3 l4proto, 4 sport, 5 dport, 6 iface, 7 tcpflags.  keys get the map
 * key (IP: NBO u32 as stored by the reference), plen the prefix length (IP only),
 * vecs nrw words per entry.  Returns the number of entries, 0 if the module is
 * absent, negative on error. */
int orc_export_map(orc_ctx *c, int chain, int field, uint32_t *keys,
                   uint8_t *plen, uint64_t *vecs, uint32_t cap, uint32_t nrw);
uint32_t orc_chain_nrw(orc_ctx *c, int chain);
/* ---- stateful conntrack (ConntrackLabel / ConntrackTableUpdate) ----
 * on: packets are labelled from, and accepted packets update, a connection
 * table, one packet at a time in batch order (orc_classify ignores nthreads;
 * ct_status must be NULL).  off: stateless labels (ct_status or empty table). */
typedef struct {
  uint32_t src_ip, dst_ip;   /* ct_k: ordered, network-order u32 as stored */
  uint16_t sport, dport;     /* ct_k ports, network-order u16 as stored */
  uint8_t l4proto, state, ip_rev, port_rev;
  uint32_t sequence;
  uint64_t ttl;
} orc_ct_entry;
int orc_ct_enable(orc_ctx *c, int on);
int orc_ct_set_time(orc_ctx *c, uint64_t ns);
int orc_ct_dump(orc_ctx *c, orc_ct_entry *out, uint32_t cap);
/* Capacity: after a batch the least recently touched live entries are deleted
 * down to max (0: unbounded; 65536 at enable, the lru_hash size).  info:
 * {live entries, evicted so far, max_entries, next batch sequence}. */
int orc_ct_set_max_entries(orc_ctx *c, uint64_t max);
int orc_ct_info(orc_ctx *c, uint64_t out[4]);
/* accept-established optimization (rule 0 == {conntrack ESTABLISHED, ACCEPT}) */
int orc_apply_accept_established(orc_ctx *c, int chain);
int orc_set_accept_established(orc_ctx *c, int chain, int on);
int orc_get_accept_established(orc_ctx *c, int chain);
int orc_read_accept_established(orc_ctx *c, int chain, uint64_t *pkts, uint64_t *bytes, int flush);

/* De Bruijn index table restated from Iptables_BitScan_dp.c:88-110. */
void orc_index64(uint16_t out[64]);

#ifdef __cplusplus
}
#endif
#endif
