/*
 * pcn_ipt.h — C ABI of the MI355X-native pcn-iptables classification datapath.
 *
 * This is the drop-in boundary that replaces the reference's kernel layer
 * (the tail-called eBPF pipeline under src/services/pcn-iptables/src/datapaths/)
 * and the "Program wrapper + RawTable::set into BPF maps" seam of the control
 * plane.  Every entry point is extern "C", takes plain
 * pointers and sizes, never throws, and returns 0 or a negative errno value;
 * pcn_ipt_last_error() returns a thread-local message for the last failure,
 * mirroring how the reference handlers turn exceptions into
 * {kGenericError, strdup(msg)} (api/IptablesApi.cpp:72-74).
 *
 * Reference paths below are relative to /root/reference/src/.
 */
#ifndef PCN_IPT_H
#define PCN_IPT_H
#ifdef __HIPCC_RTC__
#include <cstdint>   /* the chain-program compile (hiprtc, jit.cpp) has no C headers */
#else
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define PCN_IPT_ABI_VERSION 10

/* Chains and directions (ChainNameEnum; ProgramType INGRESS/EGRESS). */
enum { PCN_IPT_INPUT = 0, PCN_IPT_FORWARD = 1, PCN_IPT_OUTPUT = 2, PCN_IPT_NCHAINS = 3 };
enum { PCN_IPT_INGRESS = 0, PCN_IPT_EGRESS = 1 };
/* Attach point of the reference cube (CubeType XDP_* / TC, polycube-base.yang:93).
 * XDP sees frames as on the wire, so an 802.1Q/802.1ad-tagged frame is not
 * IPv4 and passes unclassified (Iptables_Parser_dp.c:102-106).  At the TC hook
 * the kernel receive path has already removed the outer VLAN tag
 * (skb_vlan_untag, outside the reference), so the inner IPv4 packet is
 * classified and md->packet_len = skb->len excludes the 4 tag bytes
 * (polycubed/src/cube_tc.cpp:374-432); a tagged frame shorter than 18 bytes
 * is dropped by that untag step. */
enum { PCN_IPT_HOOK_XDP = 0, PCN_IPT_HOOK_TC = 1 };
/* Actions (ActionsInt, services/pcn-iptables/src/defines.h:79). */
enum { PCN_IPT_DROP = 0, PCN_IPT_ACCEPT = 1 };
/* Per-field module ids, same numbering as ModulesConstants (defines.h:48-56). */
enum {
  PCN_IPT_F_CONNTRACK = 0, PCN_IPT_F_IPSRC = 1, PCN_IPT_F_IPDST = 2, PCN_IPT_F_L4PROTO = 3,
  PCN_IPT_F_SPORT = 4, PCN_IPT_F_DPORT = 5, PCN_IPT_F_IFACE = 6, PCN_IPT_F_TCPFLAGS = 7,
  PCN_IPT_NFIELDS = 8
};
/* rule_ids[] output codes besides a matched rule id >= 0. */
#define PCN_IPT_RID_DEFAULT (-1)   /* chain default action taken (default counters bumped) */
#define PCN_IPT_RID_NOCHAIN (-2)   /* decided before/without a rule chain (parser, ICMP checks, PASS) */

typedef struct pcn_ipt pcn_ipt;

/* Context configuration.  Replaces the per-cube state created by
 * Iptables::Iptables (services/pcn-iptables/src/Iptables.cpp:21-133). */
typedef struct {
  int device;                 /* HIP device ordinal; -1 = control plane only (no GPU) */
  uint32_t max_counted_rules; /* 0 => 8000   (Iptables_ActionLookup_dp.c:55-56)  */
  uint32_t max_action_rules;  /* 0 => 10000  (Iptables_ActionLookup_dp.c:36)     */
  uint32_t max_rules;         /* 0 => 8192   (Iptables.h:173); hard cap 32767    */
  /* Chain programs: the classify kernel recompiled (hiprtc) with the running
   * chain's table layout as constants, like the reference recompiles each
   * datapath module with substituted macros on every chain update
   * (modules/Program.cpp:23-119).  0 = compile in the background on the first
   * launch of a new shape and use it once ready (default); 1 = that first
   * launch waits for the compile; -1 = off (generic kernel only).  Verdicts,
   * rule ids and counters are identical either way. */
  int jit;
} pcn_ipt_config;

/* One rule as received by the REST surface: ChainRuleJsonObject /
 * ChainAppendInputJsonObject (datamodel/iptables.yang:221-230, Chain.cpp:139-192).
 * NULL / negative = field not set. */
typedef struct {
  const char *src;       /* "a.b.c.d" or "a.b.c.d/n" */
  const char *dst;
  const char *l4proto;   /* "TCP"/"UDP"/"ICMP"/"GRE" (upper or lower case) */
  const char *tcpflags;  /* e.g. "SYN !ACK" */
  const char *in_iface;  /* cube port name */
  const char *out_iface;
  const char *conntrack; /* "NEW"/"ESTABLISHED"/"RELATED"/"INVALID" */
  int32_t sport;         /* -1 unset */
  int32_t dport;
  int32_t action;        /* -1 unset (=> DROP, ChainRule.cpp:76-82), 0 DROP, 1 ACCEPT */
} pcn_ipt_rule;

/* A packet batch.  All buffers are caller-owned DEVICE pointers (HBM); the
 * call is stream-ordered and asynchronous.  Replaces the per-packet entry
 * handle_rx(ctx, md) (polycubed/src/cube_xdp.cpp:403-449, extiface_xdp.cpp:178-200):
 * frames[] holds the L2 frames, lens[] is md->packet_len, in_port[] is md->in_port. */
typedef struct {
  const uint8_t *frames;     /* frame bytes */
  uint64_t frames_bytes;     /* size of the frames buffer (reads never go past it) */
  const uint32_t *offsets;   /* NULL => frame i starts at i*stride */
  const uint16_t *lens;      /* NULL => every frame is fixed_len bytes */
  uint32_t stride;
  uint32_t fixed_len;
  const uint16_t *in_port;   /* NULL => const_in_port for every frame */
  uint16_t const_in_port;
  uint16_t direction;        /* PCN_IPT_INGRESS or PCN_IPT_EGRESS */
  uint16_t hook;             /* PCN_IPT_HOOK_XDP (0) or PCN_IPT_HOOK_TC */
  uint16_t reserved;         /* 0 */
  const uint8_t *ct_status;  /* per-frame label 0..3; NULL => empty-table labels (or the
                                table, with pcn_ipt_ct_enable: then it must be NULL) */
  uint64_t n;                /* number of frames */
  uint8_t *verdicts;         /* out: 0 DROP (RX_DROP), 1 ACCEPT (RX_OK / pass / redirect) */
  int32_t *rule_ids;         /* out, nullable: matched rule, or PCN_IPT_RID_* */
} pcn_ipt_batch;

/* ---- context ---------------------------------------------------------- */
int pcn_ipt_abi_version(void);
const char *pcn_ipt_last_error(void);
int pcn_ipt_create(const pcn_ipt_config *cfg, pcn_ipt **out);
void pcn_ipt_destroy(pcn_ipt *ctx);

/* Cube ports: name -> polycube port index used by in/out-iface rules.
 * Replaces Iptables::interfaceNameToIndex (Iptables.cpp:480-484). */
int pcn_ipt_add_port(pcn_ipt *ctx, const char *name, uint16_t index);

/* Host IPs that select INPUT (ingress) / OUTPUT (egress).  Replaces the
 * `localip` BPF hash (Iptables_ChainSelector_dp.c:54) updated by
 * ChainSelector::updateLocalIps (modules/ChainSelector.cpp:72-133). */
int pcn_ipt_set_localip(pcn_ipt *ctx, const uint32_t *ips_nbo, size_t n);

/* ---- rule-level control (mirror of the REST chain verbs) -------------- */
/* Chain::append (Chain.cpp:139-192) */
int pcn_ipt_chain_append(pcn_ipt *ctx, int chain, const pcn_ipt_rule *rule);
/* Chain::insert (Chain.cpp:194-300); id <= number of rules */
int pcn_ipt_chain_insert(pcn_ipt *ctx, int chain, uint32_t id, const pcn_ipt_rule *rule);
/* Chain::delRule (Chain.cpp:1039-1064) */
int pcn_ipt_chain_delete_id(pcn_ipt *ctx, int chain, uint32_t id);
/* Chain::deletes (Chain.cpp:302-352): delete the first rule equal to *rule */
int pcn_ipt_chain_delete_match(pcn_ipt *ctx, int chain, const pcn_ipt_rule *rule);
/* Chain::delRuleList (Chain.cpp:1066-1073) */
int pcn_ipt_chain_flush(pcn_ipt *ctx, int chain);
/* Chain::setDefault (Chain.cpp:79-127) */
int pcn_ipt_chain_set_default(pcn_ipt *ctx, int chain, int action);
/* Iptables `interactive` leaf (iptables.yang:98-104, Iptables.h:181): when 0,
 * rule edits are staged until pcn_ipt_chain_apply_rules (Chain::applyRules). */
int pcn_ipt_set_interactive(pcn_ipt *ctx, int interactive);
int pcn_ipt_chain_apply_rules(pcn_ipt *ctx, int chain);
int pcn_ipt_chain_nrules(pcn_ipt *ctx, int chain);

/* ---- table-level boundary (what Chain::updateChain pushes) ------------ */
/* Replace a chain's compiled tables in one step: the per-field {key -> rule
 * bitvector} maps that Chain::updateChain (Chain.cpp:600-874) would push via
 * RawTable::set (libs/polycube/src/table.cpp:53-75), plus the action table.
 * Staged into the inactive slot of a double buffer, then flipped atomically
 * between batches (Chain.cpp:441-457,924 chainNumber).  Caller-owned, copied. */
typedef struct {
  uint32_t n;              /* entries (0 => module absent) */
  const uint32_t *keys;    /* IP: NBO u32 as the reference stores it; ports: host u16;
                              iface: port index (0xffff wildcard); proto/flags/ct: value */
  const uint8_t *plen;     /* IP prefix lengths (NULL for other fields) */
  const uint64_t *vecs;    /* n * nrw words, 63 rule bits per word (defines.h:168) */
} pcn_ipt_field_map;
typedef struct {
  uint32_t nrules;
  int default_action;
  const uint8_t *actions;                /* nrules entries (ActionLookup updateTableValue) */
  pcn_ipt_field_map maps[PCN_IPT_NFIELDS];
} pcn_ipt_tables;
int pcn_ipt_load_chain(pcn_ipt *ctx, int chain, const pcn_ipt_tables *tables);
/* Export the maps the rule compiler produced for a chain (same layout as
 * pcn_ipt_field_map, std::map order).  Returns entries, 0 if absent. */
int pcn_ipt_export_map(pcn_ipt *ctx, int chain, int field, uint32_t *keys, uint8_t *plen,
                       uint64_t *vecs, uint32_t cap, uint32_t nrw);
uint32_t pcn_ipt_chain_nrw(pcn_ipt *ctx, int chain);
/* Shape of a chain's compiled device image (diagnostics / capacity planning). */
typedef struct {
  uint32_t nrules;       /* rules in the chain */
  uint32_t nrw;          /* 63-bit words per vector after the type-group permutation */
  uint32_t nsw;          /* 64-bit summary words per vector */
  uint32_t nvec;         /* distinct vectors (classes) across all fields */
  uint32_t ngroups;      /* rule type groups */
  uint32_t present;      /* bit f set: field module f present */
  uint32_t table_bytes;  /* LDS-staged table image size */
  uint64_t part_bytes;   /* partial-word indices + distinct partial words (in the image) */
} pcn_ipt_chain_info;
int pcn_ipt_chain_get_info(pcn_ipt *ctx, int chain, pcn_ipt_chain_info *out);
/* Copy a chain's table image bytes and its scalar descriptor words (layout
 * offsets, nrw, nsw, present, all_cls) for offline inspection.  Returns the
 * image size; copies nothing when cap is too small. */
int pcn_ipt_chain_get_image(pcn_ipt *ctx, int chain, uint8_t *buf, uint32_t cap, uint32_t *desc,
                            uint32_t desc_cap);

/* ---- datapath ---------------------------------------------------------- */
/* Classify a batch (device pointers), stream = hipStream_t (NULL = default).
 * Batches may come on several streams.  A stream that has carried a batch
 * must stay valid until a batch on another stream follows it, or until
 * pcn_ipt_release_stream forgets it (or the context is destroyed): the first
 * batch on a second stream records an event on the earlier one, before it
 * launches, so a later fold of the per-workgroup counter copies can wait for
 * its work (pcn_ipt.cpp note_pack_stream).  Each batch afterwards records one
 * on its own stream; with a single stream none is recorded, since an event per
 * launch costs ~3-4 us of GPU time (profiles/r04_final2/). */
int pcn_ipt_classify(pcn_ipt *ctx, const pcn_ipt_batch *batch, void *stream);
/* Before destroying a stream that carried batches: waits for the work this
 * context queued on it and drops the context's record of it, so no later
 * batch touches the handle.  The ingest ring does this for its own streams.
 * 0 also when the stream never carried a batch. */
int pcn_ipt_release_stream(pcn_ipt *ctx, void *stream);
/* Wait for all work this context queued. */
int pcn_ipt_synchronize(pcn_ipt *ctx);

/* Launch/compile statistics of the chain programs (see pcn_ipt_config.jit). */
typedef struct {
  uint64_t launches_generic;  /* classify launches that ran the generic kernel */
  uint64_t launches_jit;      /* ... that ran a chain program                  */
  uint32_t programs_ready;    /* chain programs compiled                       */
  uint32_t programs_failed;   /* compiles or module loads that failed          */
  uint64_t launches_split;    /* chain-program launches split into a gather kernel and a rule kernel
                                 (offsets / lens batches of a chain whose image exceeds LDS) */
} pcn_ipt_jit_info;
int pcn_ipt_get_jit_info(pcn_ipt *ctx, pcn_ipt_jit_info *out);
/* Test hook: the number of guard words past the classify kernel's stale-port
 * group words (one per 64-frame group + 1, used while a Horus program keys on
 * ports) that no longer hold their pattern; 0 = no write past the groups.
 * With PCN_IPT_DEBUG_STALE_CANARY=1 in the environment every word past the
 * last batch's groups is a guard word, else only those past the largest
 * batch's.  -ENOENT before the first such batch.  Synchronises the device. */
int pcn_ipt_debug_stale_canary(pcn_ipt *ctx);
/* Test hook: how often the stateful walk went past its first pass over a key
 * bucket since the last reset (device-wide): out[0] passes over a bucket's
 * 2nd to 4th connection, out[1] walks of its remaining connections as one
 * sequence (conntrack.hip walk_long).  reset != 0 zeroes them after the read.
 * Synchronises the device. */
int pcn_ipt_debug_ct_walk_passes(pcn_ipt *ctx, uint64_t out[2], int reset);
/* Test hook: the stateful pipeline's (key bucket, batch index) sort (radix.hip)
 * on its own.  keys: n device u32 < 2^kbits (left unchanged); out: the keys
 * sorted stably and the batch index of each.  Synchronises the device. */
/* Measurement hook: with PCN_IPT_DEBUG_CLOCKS=1 in the environment each classify
 * launch records, per workgroup, s_memrealtime (100 MHz) at its start, after its
 * prologue, after its last frame and after its counter flush; this copies the
 * last launch's 4 x grid values (when cap allows) and returns the grid.
 * -ENOENT before such a launch.  Synchronises the device. */
int pcn_ipt_debug_clocks(pcn_ipt *ctx, uint64_t *out, uint32_t cap);
int pcn_ipt_debug_sort_pairs(pcn_ipt *ctx, const uint32_t *keys, uint64_t n, uint32_t kbits, uint32_t *keys_out,
                             uint32_t *idx_out);
/* Compile the chain program of `chain` for its usual launch shape (fixed
 * 64-byte stride, ingress/egress alone, image in LDS) now and wait for it —
 * the blocking compile the reference does in Chain::updateChain.  Needs no
 * device (works with device = -1).  On failure the compiler log is in
 * pcn_ipt_last_error(). */
int pcn_ipt_chain_program_compile(pcn_ipt *ctx, int chain);
/* The same for the launch shape of `shape` (fixed stride or offsets / lens,
 * side inputs, hook, direction, batch size; its buffers are never read): e.g.
 * an IMIX batch, whose chain program differs from the usual one (and, for a
 * chain whose image exceeds LDS, is a split program: a gather kernel and a
 * rule kernel).  Blocking; 0 or a negative errno. */
int pcn_ipt_chain_program_compile_for(pcn_ipt *ctx, int chain, const pcn_ipt_batch *shape);
/* Resources of the chain program a chain's launches last asked for (or, before
 * any launch, of its usual launch shape, as pcn_ipt_chain_program_compile plans
 * it), read from the code object's metadata: what a measurement of that
 * program should name.  ready: 1 compiled, 0 not compiled (yet), -1 failed;
 * the other fields are valid only when ready == 1, except dynamic_lds_bytes
 * (the last launch's, 0 before one). */
typedef struct {
  int32_t ready;
  int32_t vgpr_count, agpr_count, sgpr_count;
  int32_t vgpr_spill_count, sgpr_spill_count;
  uint32_t scratch_bytes;        /* .private_segment_fixed_size: scratch per lane */
  uint32_t static_lds_bytes;     /* .group_segment_fixed_size */
  uint32_t dynamic_lds_bytes;    /* LDS per workgroup of the chain's last launch */
  uint32_t code_bytes;           /* code object size */
  uint32_t deal_window;          /* candidates dealt per pass: 64, or 128 (two per worker lane) */
  uint32_t hdr_asm;              /* fixed-stride header loads as counted asm (classify.hip PCN_HDR_ASM) */
} pcn_ipt_program_info;
int pcn_ipt_get_program_info(pcn_ipt *ctx, int chain, pcn_ipt_program_info *out);
/* Provenance of the loaded library.  which: 0 classify.hip, 1 devchain.h,
 * 2 pcn_ipt.h, 3 image.cpp -- the text the library was built from (the first
 * three are also what chain programs compile); NULL for any other value.
 * pcn_ipt_build_sha256: sha-256 (hex) of every library source at build time. */
const char *pcn_ipt_embedded_source(int which);
const char *pcn_ipt_build_sha256(void);

/* ---- host ingest ring -------------------------------------------------- */
/* Frames that start in host memory (a NIC / AF_XDP / AF_PACKET RX ring, a
 * veth) are received into pinned slots, copied to HBM, classified and their
 * verdicts copied back, pipelined over HIP streams so PCIe traffic overlaps
 * the kernels of other slots.  Replaces the per-frame packet entry
 * (polycubed/src/extiface_xdp.cpp:178-200, cube_xdp.cpp:403-449,
 * cube_tc.cpp:374-432) for batches.  Producer: acquire -> fill -> submit;
 * consumer: complete (oldest first) -> read verdicts -> release.  The ring
 * is used by one producer and one consumer thread; classify counters are
 * bumped as by pcn_ipt_classify.  Destroy rings before their context. */
typedef struct pcn_ipt_ring pcn_ipt_ring;
#define PCN_IPT_RING_RULE_IDS 1u     /* also return matched rule ids */
/* The classify kernel reads each slot's frames (and offsets / lens / in_port)
 * where they lie, in pinned host memory, over PCIe: no copy in, and only the
 * bytes the kernel reads cross the bus (a frame's header window, not its
 * payload).  Verdicts still come back by copy.  Not with hdr_bytes. */
#define PCN_IPT_RING_ZERO_COPY 2u
/* With hdr_bytes: the host packs each frame's first hdr_bytes into a
 * contiguous pinned staging buffer (pack_threads host threads), then ONE
 * contiguous copy crosses PCIe, instead of a strided copy of hdr_bytes-byte
 * rows (which the DMA engine moves one short row per request). */
#define PCN_IPT_RING_HOST_PACK 4u
typedef struct {
  uint32_t slots;         /* pinned slots, >= 2 */
  uint32_t slot_frames;   /* frames per slot, at most */
  uint64_t slot_bytes;    /* frame bytes per slot */
  uint32_t streams;       /* HIP streams the slots rotate over (0 => one per slot) */
  uint32_t flags;         /* PCN_IPT_RING_* */
  uint32_t pack_threads;  /* PCN_IPT_RING_HOST_PACK: host threads that pack (0 => 8) */
} pcn_ipt_ring_config;
typedef struct {
  uint32_t slot;
  uint8_t *frames;        /* pinned host: slot_bytes */
  uint32_t *offsets;      /* pinned host: slot_frames entries */
  uint16_t *lens;
  uint16_t *in_port;
} pcn_ipt_ring_slot;
typedef struct {
  uint64_t n;             /* frames in the slot */
  uint64_t frames_bytes;  /* bytes to copy (0 => n * stride) */
  uint32_t stride;
  uint32_t fixed_len;
  uint8_t use_offsets, use_lens, use_in_port;
  /* With hdr_bytes: the bytes at the front of each frame that stay on the host,
   * 0 or 12 -- the Ethernet addresses, which no stage of the path reads (the
   * Parser starts at h_proto, Iptables_Parser_dp.c:94-108).  Each frame then
   * crosses PCIe as hdr_bytes - 12 bytes (36 at the XDP hook).  Not with the
   * connection table on. */
  uint8_t hdr_skip;
  uint16_t const_in_port;
  uint16_t direction;     /* PCN_IPT_INGRESS / PCN_IPT_EGRESS */
  uint16_t hook;          /* PCN_IPT_HOOK_XDP / PCN_IPT_HOOK_TC */
  /* Header-only transfer (fixed stride only): 0 copies whole frames; else only
   * the first hdr_bytes of each frame cross PCIe (a strided copy into a
   * hdr_bytes-stride device batch), fixed_len / lens still give the frames'
   * lengths.  A multiple of 16, <= stride, and at least what the classify
   * path reads: 48 at the XDP hook, 64 at the TC hook (an outer VLAN tag
   * shifts the window), 80 with the connection table on (ICMP quoted headers). */
  uint16_t hdr_bytes;
} pcn_ipt_ring_batch;
int pcn_ipt_ring_create(pcn_ipt *ctx, const pcn_ipt_ring_config *cfg, pcn_ipt_ring **out);
void pcn_ipt_ring_destroy(pcn_ipt_ring *ring);
/* A free slot to fill; -EAGAIN when every slot is in flight or unreleased. */
int pcn_ipt_ring_acquire(pcn_ipt_ring *ring, pcn_ipt_ring_slot *out);
/* Copy the filled slot in, classify it, copy its verdicts out (asynchronous). */
int pcn_ipt_ring_submit(pcn_ipt_ring *ring, uint32_t slot, const pcn_ipt_ring_batch *batch);
/* The oldest submitted slot's results (pinned host, valid until release).
 * wait = 0: -EAGAIN while it is in flight; -ENOENT: nothing submitted. */
int pcn_ipt_ring_complete(pcn_ipt_ring *ring, int wait, uint32_t *slot, uint64_t *n, const uint8_t **verdicts,
                          const int32_t **rule_ids);
int pcn_ipt_ring_release(pcn_ipt_ring *ring, uint32_t slot);
/* What the ring's submits moved and what their host side cost, since creation
 * or the last reset: the bound of an end-to-end rate (host pack threads or the
 * PCIe copy) is read from these.  No reference counterpart (the reference's
 * packets never leave the kernel's RX path); measurement only. */
typedef struct {
  uint64_t submits;       /* batches submitted */
  uint64_t frames;        /* frames submitted */
  uint64_t h2d_bytes;     /* bytes queued host -> device (frames or header rows, offsets / lens / in_port) */
  uint64_t d2h_bytes;     /* bytes queued device -> host (verdicts, rule ids) */
  uint64_t zc_bytes;      /* zero copy: header bytes the kernel reads over PCIe (the 64-byte sector of each frame) */
  uint64_t pack_ns;       /* PCN_IPT_RING_HOST_PACK: wall time of the packs (all pack threads together) */
  uint64_t submit_ns;     /* wall time inside pcn_ipt_ring_submit, pack included */
} pcn_ipt_ring_stats;
int pcn_ipt_ring_get_stats(pcn_ipt_ring *ring, pcn_ipt_ring_stats *out, int reset);

/* ---- counters ---------------------------------------------------------- */
/* Per-rule pkts/bytes (ActionLookup pkts_/bytes_<CHAIN>) and default counters
 * (pkts_/bytes_default_<CHAIN>).  flush != 0 zeroes the per-rule counters after
 * reading (read-and-flush, modules/ActionLookup.cpp:78-151).  scope 0 = this
 * GPU, 1 = summed over the communicator (after pcn_ipt_sync_counters). */
int pcn_ipt_read_counters(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n,
                          uint64_t *def_pkts, uint64_t *def_bytes, int flush, int scope);
/* Accumulated stats like Chain::getStatsList (Chain.cpp:961-976): per-rule
 * totals kept in the control plane across rule edits + the DEFAULT row. */
int pcn_ipt_chain_stats(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n,
                        uint64_t *def_pkts, uint64_t *def_bytes);
/* Chain::resetCounters (Chain.cpp:354-380) */
int pcn_ipt_chain_reset_counters(pcn_ipt *ctx, int chain);

/* ---- stateful connection tracking -------------------------------------- */
/* The `connections` table (Iptables_ConntrackLabel_dp.c:111-113, an LRU hash
 * of 65536 entries) kept in HBM, with the reference's labels
 * (ConntrackLabel_dp.c:190-531) and updates (ConntrackTableUpdate_dp.c:141-655).
 * While enabled, pcn_ipt_classify labels every IPv4 packet from the table and
 * every accepted packet updates it, with the result of running the batch one
 * packet at a time in index order (and batches in submission order).
 * Capacity: the reference's lru_hash holds 65536 entries.  Here the LRU works
 * at batch granularity: a packet touches its table key (its own, an ICMP
 * error's quoted one) when the entry is live after it; after each batch the
 * least recently touched live entries are deleted down to max_entries
 * (pcn_ipt_ct_set_max_entries: 65536 by default, 0 = unbounded), counted in
 * pcn_ipt_ct_info.evicted.  Within a batch nothing is evicted (the kernel's
 * own LRU is approximate: per-CPU lists, reference bits).  One touch per
 * packet: an echo reply that falls through to ICMP_MISS also looks up the key
 * of the header it quotes (ConntrackLabel_dp.c:450-531), and in the kernel's
 * lru_hash that lookup would refresh the quoted entry too; here (GPU and
 * oracle alike) it does not, so eviction order can differ from the kernel's
 * there.  No reference fixture covers it (parity unpinned).  Independently of
 * that, an insert that finds no free slot within 512 slots of the key's home
 * slot (a full or nearly full table: 2^capacity_log2 slots, deleted keys keep
 * theirs) is dropped and counted (inserts_lost), which bounds every lookup at
 * 512 probes.  Entries never expire in the reference either (ttl is written,
 * never compared).  batch.ct_status must be NULL while enabled. */
typedef struct {
  uint32_t src_ip, dst_ip;   /* ct_k as stored: ordered NBO u32 */
  uint16_t sport, dport;     /* ct_k ports as stored: ordered NBO u16 */
  uint8_t l4proto, state, ip_rev, port_rev;   /* state: 0 NEW .. 9 TIME_WAIT (ConntrackLabel_dp.c:70-81) */
  uint32_t sequence;
  uint64_t ttl;
} pcn_ipt_ct_entry;
typedef struct {
  uint32_t enabled, capacity_log2;
  uint64_t now;              /* timestamp used for new ttl values */
  uint64_t inserts_lost;     /* inserts refused: no free slot near the key's home (table (nearly) full) */
  uint64_t max_entries;      /* live entries kept after each batch (LRU; 0 = unbounded) */
  uint64_t evicted;          /* entries deleted by the LRU so far */
  uint64_t fused_batches;    /* stateful batches whose classify pass also built the walk records
                                (frames shorter than 70 bytes, one label: the frames read once) */
} pcn_ipt_ct_info;
/* capacity = 2^capacity_log2 slots (0 => 2^18); the table persists across enable/disable. */
int pcn_ipt_ct_enable(pcn_ipt *ctx, uint32_t capacity_log2);
int pcn_ipt_ct_disable(pcn_ipt *ctx);
int pcn_ipt_ct_clear(pcn_ipt *ctx);
/* Live entries kept after each batch (default 65536, the lru_hash size of
 * Iptables_ConntrackLabel_dp.c:112; 0 = unbounded); takes effect at the next batch. */
int pcn_ipt_ct_set_max_entries(pcn_ipt *ctx, uint64_t max_entries);
/* The `timestamp` percpu value ConntrackTableUpdate::updateTimestamp writes
 * every second (modules/ConntrackTableUpdate.cpp:108-137). */
int pcn_ipt_ct_set_time(pcn_ipt *ctx, uint64_t ns);
/* Live entries sorted by key (Iptables::getSessionTableList, Iptables.cpp:527-566);
 * copies min(count, cap), returns count. */
int pcn_ipt_ct_dump(pcn_ipt *ctx, pcn_ipt_ct_entry *out, uint32_t cap);
int pcn_ipt_ct_get_info(pcn_ipt *ctx, pcn_ipt_ct_info *out);

/* Accept-established optimization: set by the rule-level verbs exactly where
 * the reference calls ChainRule::applyAcceptEstablishedOptimization (rule 0 ==
 * {conntrack ESTABLISHED, ACCEPT}); explicit for the table-level boundary.
 * ESTABLISHED packets are then accepted before the chain (rule id -3) and
 * counted in pkts/bytes_acceptestablished_<Chain> (ConntrackLabel_dp.c:580-616),
 * which pcn_ipt_chain_stats adds to rule 0 (ChainStats.cpp:64-103). */
#define PCN_IPT_RID_ACCEPT_ESTABLISHED (-3)
int pcn_ipt_set_accept_established(pcn_ipt *ctx, int chain, int on);
int pcn_ipt_get_accept_established(pcn_ipt *ctx, int chain);
int pcn_ipt_read_accept_established(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, int flush);

/* ---- Horus (pcn-iptables `horus` leaf, iptables.yang:112-118) ----------- */
/* The exact-match prefilter of pcn-iptables, OFF by default (Iptables.h:185).
 * pcn_ipt_set_horus only sets the flag (Iptables::setHorus, Iptables.cpp:
 * 400-406).  Every chain update (verbs, apply, default change) drops the Horus
 * table and its counters, and an INPUT update with horus on, INPUT rules and
 * no FORWARD rules builds a new one (Chain::updateChain, Chain.cpp:505-592)
 * from the leading INPUT rules that set the same key fields as rule 0: a /32
 * source / destination, protocol, ports; the table ends at the first rule with
 * another pattern or a conntrack match, and a repeated key keeps its first
 * rule (Chain::horusFromRulesToMap, Utils.cpp:537-630).
 * The datapath looks every parsed ingress IPv4 packet up after the Parser and
 * before the ChainSelector (Iptables_Parser_dp.c:145-147), so forwarded
 * traffic meets INPUT rules too.  A hit bumps the Horus counters of its rule
 * and reports rule id PCN_IPT_RID_HORUS0 - <INPUT rule id>; DROP drops,
 * ACCEPT continues as PASS_LABELING (ICMP length checks, labels, conntrack
 * update, accept; Iptables_Horus_dp.c:136-161).  The key's ports are read as
 * the reference reads them, through a packed struct laid over the aligned
 * one the Parser writes: source port = [0, first source-port byte], destination
 * port = [second source-port byte, first destination-port byte]; a packet the
 * Parser writes no ports for (ICMP, GRE ...) keys on the ports the last TCP/UDP
 * packet left (Q4), tracked from the moment horus is set (or, with conntrack
 * on, by the connection table's own copy).  pcn_ipt_chain_stats adds (and
 * flushes) the Horus counters of rule id k to rule k of whichever chain is
 * read, as ChainStats::fetchCounters does (ChainStats.cpp:106-121).
 *
 * pcn-firewall has Horus on from the start, with no knob (Firewall.h:337;
 * pcn_ipt_set_horus turns it off anyway, an extension).  Each chain has its
 * own program (Chain::updateChain, pcn-firewall Chain.cpp:232-306), rebuilt by
 * every update of that chain that leaves it with rules -- not by a default
 * change, which reloads only DefaultAction (:60-82) -- with the same rule
 * (pcn-firewall Utils.cpp:483-577).  Its Parser calls it for both directions
 * (Firewall_Parser_dp.c:154-157), and there the key holds the ports as stored
 * (both sides packed).  The program keeps the conntrack setting it was built
 * with (modules/Horus.cpp:135-139): built with conntrack on, an ACCEPT hit is
 * PASS_LABELING (labels, table update, accept); built with it off, RX_OK.
 * While conntrack is off its ConntrackLabel program does not exist
 * (Firewall.cpp:163-171), so every tail call Horus makes into it fails: a miss
 * drops, and so does an ACCEPT hit of a program built with conntrack on.
 * `chain` names the program: PCN_IPT_INPUT (pcn-iptables), PCN_FW_INGRESS /
 * PCN_FW_EGRESS (pcn-firewall). */
#define PCN_IPT_RID_HORUS0 (-4096)
#define PCN_IPT_HORUS_MAX 2048                       /* HorusConst::MAX_RULE_SIZE_FOR_HORUS */
enum { PCN_IPT_HZ_SRCIP = 1, PCN_IPT_HZ_DSTIP = 2, PCN_IPT_HZ_L4PROTO = 4, PCN_IPT_HZ_SRCPORT = 8,
       PCN_IPT_HZ_DSTPORT = 16 };
typedef struct {
  uint32_t enabled;          /* the horus leaf (pcn-firewall: horus_enabled) */
  uint32_t runtime;          /* a Horus program is in place (horus_runtime_enabled_) */
  uint32_t entries;          /* keys in the table */
  uint32_t fields;           /* PCN_IPT_HZ_* set fields of the key */
  uint32_t conntrack;        /* pcn-firewall: the program was built with conntrack on */
} pcn_ipt_horus_info;
int pcn_ipt_set_horus(pcn_ipt *ctx, int on);
int pcn_ipt_get_horus_info(pcn_ipt *ctx, int chain, pcn_ipt_horus_info *out);
/* pkts_horus / bytes_horus[rule id] (Iptables_Horus_dp.c:77-90, Firewall_Horus_dp.c:82-95) */
int pcn_ipt_read_horus_counters(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n, int flush);

/* ---- pcn-firewall personality ------------------------------------------ */
/* pcn-firewall (src/services/pcn-firewall) runs the same field modules,
 * BitScan, ActionLookup and rule compiler as pcn-iptables
 * (Firewall_{IpLookup,L4ProtocolLookup,L4PortLookup,TcpFlagsLookup,
 * ConntrackMatch,BitScan,ActionLookup}_dp.c, Utils.cpp) behind a transparent
 * cube, so a context can serve it instead.  Differences, all applied by the
 * same kernel:
 *  - two chains, INGRESS and EGRESS (firewall.yang:175-176), selected by the
 *    batch direction alone (Firewall_ChainForwarder_dp.c:20-42); they live in
 *    the FORWARD and OUTPUT slots of the chain verbs, INPUT is refused;
 *  - no localip, no allow logic: an empty chain takes its default action and
 *    bumps its default counters (DefaultAction, Firewall_DefaultAction_dp.c);
 *  - no in/out-iface fields; a rule must carry an action (Chain.cpp:89-92,
 *    612-620); a conntrack field needs conntrack on (ChainRule.cpp:29-33);
 *    `deletes` without a match fails (Chain.cpp:760-771); `update` replaces
 *    the rule at id or appends at id == size (Chain::addRule, :612-644);
 *  - the ConntrackLabel stage (ICMP length checks, labels) runs only while
 *    conntrack is on (modules/Parser.cpp:41-45).  AUTOMATIC mode
 *    (accept-established ON, the default) accepts ESTABLISHED packets before
 *    the chain, uncounted, rule id PCN_IPT_RID_ACCEPT_ESTABLISHED
 *    (Firewall_ConntrackLabel_dp.c:474-478).  With the connection table
 *    (pcn_ipt_ct_enable) labels and updates are the pcn-iptables ones (the
 *    label and update code is the same, Firewall_ConntrackLabel_dp.c:116-460,
 *    Firewall_ConntrackTableUpdate_dp.c:141-650); without it they come from
 *    batch.ct_status or an empty table.  With conntrack off the label is NEW
 *    and the table is neither read nor updated.
 * Set the service on a fresh context, before any rule. */
enum { PCN_IPT_SERVICE_IPTABLES = 0, PCN_IPT_SERVICE_FIREWALL = 1 };
enum { PCN_FW_INGRESS = PCN_IPT_FORWARD, PCN_FW_EGRESS = PCN_IPT_OUTPUT };
/* ConntrackModes (pcn-firewall defines.h:56-58); a new firewall is AUTOMATIC (Firewall.h:323) */
enum { PCN_FW_CT_DISABLED = 0, PCN_FW_CT_MANUAL = 1, PCN_FW_CT_AUTOMATIC = 2 };
int pcn_ipt_set_service(pcn_ipt *ctx, int service);
int pcn_ipt_get_service(pcn_ipt *ctx);
/* Firewall::setConntrack (Firewall.cpp:151-195): off -> DISABLED; on from DISABLED -> MANUAL */
int pcn_fw_set_conntrack(pcn_ipt *ctx, int on);
/* Firewall::setAcceptEstablished (Firewall.cpp:119-142): -EINVAL while DISABLED */
int pcn_fw_set_accept_established(pcn_ipt *ctx, int on);
int pcn_fw_get_conntrack_mode(pcn_ipt *ctx);
/* Chain::addRule / replaceRule (`rule add <id>`, batch UPDATE): replace the
 * rule at id (its counters carry on), or append when id == number of rules. */
int pcn_fw_chain_update(pcn_ipt *ctx, int chain, uint32_t id, const pcn_ipt_rule *rule);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ------------------- */
/* 128-byte ncclUniqueId produced on rank 0 and shared out of band. */
int pcn_ipt_comm_unique_id(uint8_t out[128]);
int pcn_ipt_comm_init(pcn_ipt *ctx, int nranks, int rank, const uint8_t uid[128]);
/* All-gather every rank's per-rule/default counters over RCCL and sum them
 * into the scope=1 view.  Stream-ordered. */
int pcn_ipt_sync_counters(pcn_ipt *ctx, void *stream);
/* Facts about the exchange, for a scaling run's record: the RCCL that serves
 * the calls (its ncclGetVersion and the file dladdr resolves ncclCommInitRank
 * to: a process may hold more than one librccl), the context's device and PCI
 * bus id (ranks must not share one), and the summed duration of the
 * all-gather steps (all-gather + rank sum, an event pair on the communicator
 * stream per pcn_ipt_sync_counters call; waits for the ones still running).
 * ctx may be NULL: then only nccl_version and rccl_path are filled. */
typedef struct {
  int nccl_version;          /* e.g. 22606 = 2.26.6 */
  int nranks, rank;          /* 0, 0 before pcn_ipt_comm_init */
  int device;                /* HIP ordinal, -1 without a device */
  char pci_bus_id[32];
  char rccl_path[256];
  uint64_t gathers_timed;
  double gather_ms_total;
  uint64_t gathers_untimed;  /* steps not timed: their timing slot's earlier step was still
                                running (the call never waits on the device for it) */
} pcn_ipt_comm_info;
int pcn_ipt_comm_get_info(pcn_ipt *ctx, pcn_ipt_comm_info *out);
/* The two halves of pcn_ipt_sync_counters, for a caller that moves the counter
 * blocks over its own transport (gloo, MPI, a test), or reads them raw.  The
 * reference's only reduction is the control plane's sum over per-CPU counters
 * (modules/ActionLookup.cpp:78-96); here each GPU is one "CPU".
 * pcn_ipt_counter_block_words: u64 words in chain `chain`'s block,
 *   [def_pkts, def_bytes, pkts_0, bytes_0, ...] = 2 + 2 * counted rules
 *   (no device needed).
 * pcn_ipt_snapshot_counters: copy this GPU's block into `block` (device,
 *   >= block words), stream-ordered.
 * pcn_ipt_sum_counter_blocks: sum `nranks` blocks (device, rank-major, `words`
 *   u64 each, as ncclAllGather lays them out) into the scope=1 view of
 *   `chain` with the device kernel the all-gather path runs; stream-ordered.
 *   `words` must equal the chain's block words; 1 <= nranks <= 4096. */
int pcn_ipt_counter_block_words(pcn_ipt *ctx, int chain);
int pcn_ipt_snapshot_counters(pcn_ipt *ctx, int chain, uint64_t *block, void *stream);
int pcn_ipt_sum_counter_blocks(pcn_ipt *ctx, int chain, const uint64_t *blocks, uint32_t nranks, uint64_t words,
                               void *stream);

/* Flow-affinity split for stateful conntrack on N GPUs.  Replaces the NIC's
 * RSS queue choice that spreads traffic over the reference's per-CPU datapath
 * (polycubed/src/extiface_xdp.cpp:178-200 runs handle_rx on the receiving
 * CPU; the Parser's `packet` struct is per CPU, Iptables_Parser_dp.c:45).
 * The owner of a frame is a hash of its unordered IPv4 address pair (for an
 * ICMP error >= 70 B, of the quoted header's pair, whose connection it
 * labels, Iptables_ConntrackLabel_dp.c:491-529); non-IPv4 and frames the
 * Parser drops belong to rank 0.  All packets of one connection therefore
 * meet one connection table, in batch order.  Uses the batch's frames,
 * frames_bytes, offsets, lens, stride, fixed_len, in_port, const_in_port,
 * hook and n; the other fields are ignored.  1 <= nranks <= 255.
 *
 * pcn_ipt_flow_owner: owner[i] (device, n bytes) for every frame.
 * pcn_ipt_flow_split: this rank's frames in batch order: index[k] (the frame's
 * position in the batch), offsets[k], lens[k] and, if in_port_out is not
 * NULL, in_port_out[k] — device arrays of capacity n, ready to be passed as a
 * pcn_ipt_batch's offsets/lens/in_port.  *n_out (host) = the number of owned
 * frames; synchronises the stream to read it.  offsets are u32: a fixed-stride
 * batch must end below 4 GiB. */
int pcn_ipt_flow_owner(pcn_ipt *ctx, const pcn_ipt_batch *batch, uint32_t nranks, uint8_t *owner, void *stream);
int pcn_ipt_flow_split(pcn_ipt *ctx, const pcn_ipt_batch *batch, uint32_t nranks, uint32_t rank, uint32_t *index,
                       uint32_t *offsets, uint16_t *lens, uint16_t *in_port_out, uint64_t *n_out, void *stream);

#ifdef __cplusplus
}
#endif
#endif
