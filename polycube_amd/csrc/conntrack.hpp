// conntrack.hpp — stateful connection tracking on the GPU (host-visible types).
//
// The reference labels every IPv4 packet with its connection state from the
// `connections` table (Iptables_ConntrackLabel_dp.c:190-531) and updates the
// table for every accepted packet (Iptables_ConntrackTableUpdate_dp.c:141-655),
// one packet at a time per CPU.  Here a batch runs as:
//   A. the classify kernel once per possible label (1 run when no reachable
//      chain has conntrack rules, else 4), counters off, giving each packet's
//      outcome as a function of its label;
//   B. ct_prep: stale ports (quirk Q4, by look-back), the chain, the packet's
//      conntrack key and kind, its walk record in batch order; packets that
//      need no table access are finished here;
//   C. a stable radix sort of the table-touching packets by key bucket, so
//      every key's packets form one run in batch order;
//   D. ct_heads (runs by length class) -> ct_walk: a wave per long run, a lane
//      per short one, walks its packets in order against the HBM-resident
//      table (label -> outcome -> update), so the result equals processing the
//      batch one packet at a time; outcomes go straight to batch order;
//   E. ct_count: per-rule / default / accept-established counters from the
//      final rule ids.
// Echo replies long enough to carry a quoted header (>= 70 B) may read a
// second key's state: they split the batch into segments and are run one at a
// time between the walks of the segments (ct_hard).
#pragma once
#include <cstdint>

namespace pcn {

// One table slot (32 B).  `tag`: 0 empty, 1 published, 2 being claimed.
// Slots are never freed (a deleted connection keeps its key with valid = 0),
// so linear probing stops at the first empty slot.
struct CtSlot {
  uint32_t tag;
  uint32_t src, dst;          // ct_k, ordered (network-order u32 as loaded)
  uint16_t sport, dport;      // ct_k ports, ordered
  unsigned long long ttl;     // ct_v
  uint32_t seq;
  uint8_t proto, valid, state, rev;   // rev: bit0 ipRev, bit1 portRev
};
static_assert(sizeof(CtSlot) == 32, "CtSlot is 32 bytes");

struct CtBatch {
  const uint8_t *frames;
  uint64_t frames_bytes;
  const uint32_t *offsets;
  const uint16_t *lens;
  uint32_t stride, fixed_len;
  uint32_t direction, hook;
  uint64_t n;
  const uint32_t *localip;    // sorted NBO u32
  uint32_t nlocal;
  uint32_t allow_logic, empty_mask, drop_mask;
  uint32_t fw;                // pcn-firewall dispatch: the direction's chain, labels before the chain
  uint32_t ae_mask;           // bit c: accept-established optimization on for chain c
  uint32_t nlab;              // outcomes per packet from stage A: 1 or 4
  const uint8_t *a_verdict;   // [nlab][n]
  const int32_t *a_rid;       // [nlab][n]
  uint8_t *verdicts;          // final
  int32_t *rule_ids;          // final (never null: scratch when the caller has none)
  unsigned long long *ctr[3];
  uint32_t ncounted[3];
  unsigned long long *ae_ctr; // [3][2] pkts, bytes
  unsigned long long *horus_ctr;  // [PCN_IPT_HORUS_MAX][2] (null: Horus off); Horus hits are the
                                  // packets with rule id <= PCN_IPT_RID_HORUS0 (stage A found them)
  uint32_t horus_final;       // pcn-firewall program built with conntrack off: an ACCEPT hit is RX_OK,
                              // unlabelled (Firewall_Horus_dp.c:162-164)
};

struct CtTable {
  CtSlot *slots = nullptr;
  uint32_t cap_log2 = 0;
  uint32_t *carry = nullptr;             // stale ports of the shared `packet` struct
  unsigned long long *stats = nullptr;   // [0] inserts refused because the table was full, [1] entries evicted
  unsigned long long now = 0;            // the `timestamp` the control plane sets
  // LRU at batch granularity (the lru_hash of 65536 entries,
  // Iptables_ConntrackLabel_dp.c:112): per slot, the stamp (batch seq << 32 |
  // batch index) of the last packet after which its entry was live; after a
  // batch the oldest live entries are deleted down to max_entries (0: unbounded).
  unsigned long long *touch = nullptr;
  uint32_t seq = 1;
  uint64_t max_entries = 65536;
};

struct CtScratch;   // device buffers, grown as batches need (conntrack.hip)
CtScratch *ct_scratch_new();
void ct_scratch_free(CtScratch *s);

// Stages B-E for one batch whose stage-A outcomes are in b.a_*.  Synchronises
// the stream once when the batch holds long echo replies.  Returns a hipError_t.
// prepped: stage A already wrote the walk records, key buckets and {len, cinfo}
// words (into ct_prep_buffers') and published each 64-frame group's ports word
// and the lanes whose records wait for the ports before their group, so ct_prep
// is skipped (the frames are read once per batch): ct_stale_agg / ct_stale_fix
// complete those records and advance the carry.
int ct_run(const CtBatch &b, CtTable &t, CtScratch &s, int num_cus, void *stream, bool prepped = false);

// The buffers a stage A that writes the walk records fills for an n-packet
// batch (grown as needed): 8 u32 per record, the key bucket and the {len,
// cinfo} word per packet, the bucket of packets without a key, and per 64-frame
// group the ports word and the lanes to complete (LaunchArgs::ct_pdesc / ct_fixm).
int ct_prep_buffers(CtScratch &s, uint64_t n, uint32_t **brec, uint32_t **keys, uint32_t **lcs, uint32_t *sentinel,
                    unsigned long long **pdesc, unsigned long long **fixm);

// Stateless batches (labels given per packet) on chains with accept-established
// on: move rule-0 hits to the accept-established path (rule id -3 and its
// counters), as ConntrackLabel_dp.c:580-616 takes ESTABLISHED packets there
// before the chain runs.  rule_ids may be null.
int ct_ae_fixup(const CtBatch &b, void *stream);
// walk_long's extra passes since the last reset (g_walk_passes, current device; a hipError_t)
int ct_walk_passes(uint64_t out[2], bool reset);

// Flow-affinity split (pcn_ipt_flow_owner / pcn_ipt_flow_split): the owner
// rank of every frame, from its unordered IPv4 address pair (an ICMP error's
// quoted pair); the split compacts this rank's frames, in batch order, into
// offsets/lens/in_port arrays and synchronises the stream for the count.
int ct_flow_owner(const CtBatch &b, uint32_t nranks, uint8_t *owner, int num_cus, void *stream);
int ct_flow_split(const CtBatch &b, const uint16_t *in_port, uint16_t const_in_port, uint32_t nranks, uint32_t rank,
                  uint32_t *index, uint32_t *offsets, uint16_t *lens, uint16_t *in_port_out, uint64_t *n_out,
                  int num_cus, void *stream);

// The ports the shared `packet` struct holds after a batch (Q4): *carry
// becomes the ports dword (wire bytes 34-37) of the batch's last frame the
// Parser wrote ports for, if any.  (Within a batch the classify kernel
// computes them itself, classify.hip stale_lookback.)
int ct_advance_carry(const CtBatch &b, CtScratch &s, uint32_t *carry, int num_cus, void *stream);

int ct_table_init(CtTable &t, uint32_t cap_log2);
void ct_table_free(CtTable &t);

}  // namespace pcn
