// devchain.h — device-side layout of one compiled chain ("chain image") and the
// classify launch arguments.  Shared by the host image builder and the HIP kernel.
//
// The reference keeps one BPF map per field module (LPM trie / hash / array of
// 1,048-byte bitvectors, Iptables_*Lookup_dp.c) and walks them with ~12 tail
// calls per packet.  Here a chain is one compact TABLE IMAGE (tens of KB at
// 1k rules) that each workgroup copies into LDS, so the per-packet path makes
// no dependent HBM/L2 access at all:
//   - IP src/dst: the kernel-LPM answer as sorted interval boundaries plus a
//     bucket index on the top address bits (2^4..2^12 buckets, sized so a
//     bucket holds few boundaries) searched in a fixed number of steps (a
//     window read of the whole bucket was measured 8% slower: the kernel is
//     bound by LDS traffic more than by dependent-read latency);
//   - sport/dport/iface: open-addressing hashes {key -> class} with the
//     wildcard class (key 0 / 0xffff) as the miss fallback;
//   - proto/tcpflags/conntrack (and sport/dport/iface while small) share one
//     META slot: each maps its value to a small index and a table holds the
//     class of the AND of their vectors;
//   - per class and 64-word block: SUMM (bit w: word w of the class vector
//     != 0), and the candidate record {PM, PBASE}: PM (bit w: word w is
//     PARTIAL, neither zero nor holding all of its rules) and the start of the
//     class's partial words in PART, stored in word order (a partial word's
//     index = PBASE + popcount(PM bits below));
//     PART holds the partial words themselves (PART_DIRECT, while the image
//     stays small enough for LDS) or u16 (u32 when PART_WIDE) indices into
//     POOL, the distinct partial words (at 1k rules ~7x fewer);
//   - PERM: bit position -> (original rule id << 1 | action).
// Images too large for LDS are read from HBM through the same accessors.
//
// Rule bits are permuted so rules that constrain the same set of fields share
// words ("type groups"); a field a word's rules do not constrain has that word
// FULL, and a field they do constrain has a sparse summary, which is what makes
// the summary AND selective.  Inside a word, bits are in ascending rule id, so
// the lowest set bit of a word is its lowest-numbered matching rule and the
// packet's rule is the minimum over its non-zero candidate words.
#pragma once
#include <cstdint>

#define PCN_CLS_MISS 0xFFFFu
#define PCN_MAX_LOCALIP 256
#define PCN_IP_BUCKET_BITS_MAX 12
#define PCN_HASH_EMPTY 0xFFFFFFFFu
#ifndef PCN_BLOCK
#define PCN_BLOCK 1024              // classify workgroup size (threads): one per CU
#endif
#define PCN_WAVE_LDS_BYTES 3072     // per-wave LDS region: header transpose buffer (64 frames x 48 B),
                                    // reused as the candidate-stage scratch
#define PCN_WAVE_SCRATCH_BYTES 1280 // the candidate-stage scratch alone: the whole region of a launch
                                    // without the fixed-stride header transpose
#define PCN_SPLIT_G_BLOCK 256       // a split launch's gather kernel: workgroup size (threads), several
                                    // workgroups per CU as its registers allow (no chain image in LDS)
#define PCN_DEAL2_WAVE_BYTES 2304   // the scratch of a 128-candidate deal window (classify.hip PCN_DEAL2):
                                    // chain programs of chains with 2+ summary blocks

#if defined(__HIPCC__) || defined(__HIPCC_RTC__)
#define PCN_HD __host__ __device__
#else
#define PCN_HD
#endif

namespace pcn {

// Horus table (pcn_ipt.h): open addressing, 16 bytes per slot
// {src, dst, ports = sk | dk << 16, meta = proto | action << 8 | 1 << 9 (used)
// | rule id << 16}; fields outside the key's set fields are 0 in both the
// slot and the packet's key.  sk / dk are the key's port bytes as the
// reference's packed horusKey holds them, read as little-endian u16.
constexpr uint32_t kHorusUsed = 1u << 9;
// LaunchArgs::horus_flags (0: pcn-iptables)
constexpr uint32_t kHzNatural = 1;       // pcn-firewall: the key holds the ports as stored (packed on both sides)
constexpr uint32_t kHzAcceptFinal = 2;   // ACCEPT hit -> RX_OK (program built with conntrack off)
constexpr uint32_t kHzAcceptDrops = 4;   // ACCEPT hit -> RX_DROP (PASS_LABELING into a deleted ConntrackLabel)
constexpr uint32_t kHzMissDrops = 8;     // miss -> RX_DROP (the tail call into a deleted ConntrackLabel)
PCN_HD inline uint32_t horus_hash(uint32_t src, uint32_t dst, uint32_t ports, uint32_t proto) {
  uint64_t h = ((uint64_t(src) << 32) | dst) * 0x9E3779B97F4A7C15ull;
  h ^= ((uint64_t(ports) << 8) | proto) * 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return static_cast<uint32_t>(h);
}

// Byte offsets inside a table image (all 16-byte aligned).
struct TableLayout {
  uint32_t bytes;
  uint32_t ip_bkt[2];      // u32[1 << (32 - ip_shift)]: (count << 16) | first boundary in the bucket
  uint32_t ip_shift[2];    // bucket = address >> ip_shift
  uint32_t ip_steps[2];    // branchless search steps: every bucket holds < 2^steps boundaries
  uint32_t ip_win[2];      // != 0: no search; every bucket holds <= ip_win boundaries and a lookup
                           // reads all ip_win of them at once (bnd is padded with 0xFFFFFFFF)
  uint32_t ip_bnd[2];      // u32[m]: interval boundaries (host-order addresses)
  uint32_t ip_cls[2];      // u16[m+1]: class of each interval
  uint32_t hash[3];        // u32[size + 1]: (key << 16) | value (sport, dport, iface); every key
                           // sits in its home slot or the next; slot size mirrors slot 0.  The
                           // value is a meta index (field joined to meta) or a class (own slot)
  uint32_t hash_mask[3];   // size - 1
  uint32_t hash_wild[3];   // value used when the key is absent (PCN_CLS_MISS: none, own slot)
  uint32_t key_skip[2];    // sport/dport value of a non-TCP/UDP packet (the module is skipped)
  uint32_t key_slot[3];    // sport/dport/iface: own slot (3..5), or 0 (joined to meta / absent)
  uint32_t nslots;         // 3 + key fields with an own slot
  uint32_t proto_idx, flags_idx, ct_idx;   // u8[256], u16[256], u8[4]: value -> meta index
  uint32_t flags_skip;     // flags index of a non-TCP packet (the module is skipped)
  uint32_t meta;           // u16[]: class of the meta slot at sum(index_f * meta_stride[f])
  uint32_t meta_stride[6]; // proto, flags, ct, sport, dport, iface (0: not a meta field)
  uint32_t sf;             // u64[nvec][nsw]: SUMM (bit w: word w of the class vector != 0)
  uint32_t pbase;          // {u64 PM, u32 PBASE, u32 0}[nvec][nsw]: PM bit w = word w partial,
                           // PBASE = first PART index of the class's block.  With indexed
                           // PART (large images) pbase and PART are the last two tables, so
                           // [0, pbase) -- every table but those -- is the LDS prefix staged
                           // when the whole image does not fit; direct images keep PART,
                           // POOL and PERM after pbase
  uint32_t part;           // u16[] (u32[] if part_wide): POOL index of each partial word
  uint32_t part_wide;
  uint32_t part_direct;    // PART holds the partial words themselves (u64), not POOL indices
  uint32_t part_dense;     // PART is dense: u16 (u32 if part_wide) POOL index of every (class,
                           // word), 0 where the word is FULL; no {PM, PBASE} records (pbase ==
                           // part).  Used when the image is too large for LDS anyway: a
                           // candidate field is then one L2 read instead of two
  uint32_t pool;           // u64[]: distinct partial words; POOL[0] is all-ones
  uint32_t zero;           // 16 zero bytes (the PART cell a FULL field reads: index 0)
  uint32_t perm;           // u16[nrw * 63]
  uint32_t wfields;        // dense PART only: u8[nrw] in the LDS prefix, bit f set when a class of
                           // slot f can be partial at word w; a candidate field whose bit is clear
                           // is FULL there and reads no PART cell from L2
};

struct DevChain {
  TableLayout lay;
  const uint8_t *image;          // table image in HBM (copied to LDS when it fits)
  unsigned long long *ctr;       // [2 + 2*ncounted]: def_pkts, def_bytes, pkts0, bytes0, ...
  uint32_t nrules, nrw, nsw, present, nvec;
  uint32_t all_cls;              // class of the all-ones vector (fields absent or skipped)
  uint32_t ncounted, max_action;
  int32_t default_action;
  uint32_t lds_image;            // byte offset of this chain's image in LDS
  uint32_t lds_limit;            // image bytes staged in LDS: all, the per-packet prefix
                                 // [0, lay.pbase) when the whole does not fit, or 0
  int32_t lds_bins;              // first LDS counter bin of this chain's rules; -1 => global atomics
  uint32_t lds_nrules;           // rule ids [0, lds_nrules) count in the LDS bins from lds_bins, the
                                 // rest with global atomics (a chain too large for a bin per rule)
};

// LDS layout of a classify workgroup: [chain images][counter bins (u32 x2)][localip][per-wave regions]
constexpr uint32_t kLdsDescBytes = 0;

struct LaunchArgs {
  DevChain ch[3];
  const uint8_t *frames;
  uint64_t frames_bytes;
  const uint32_t *offsets;
  const uint16_t *lens;
  const uint16_t *in_port;        // never null: a zero cell (mask 0) when the batch has none
  const uint8_t *ct_status;       // likewise
  uint64_t in_port_mask, ct_mask; // index masks: ~0 (per-frame arrays) or 0 (zero cell)
  uint32_t has_in_port, has_ct;
  uint8_t *verdicts;
  int32_t *rule_ids;
  const uint32_t *localip;       // sorted NBO u32
  uint64_t n;
  uint32_t stride, fixed_len;
  uint32_t nlocal;
  uint32_t nbins;                // LDS counter bins (3 default bins + rule bins)
  uint32_t bins_offset;          // byte offset of the counter bins in LDS
  uint32_t lds_images_bytes;     // bytes of chain images staged in LDS (0: read from HBM)
  uint32_t lds_localip;          // byte offset of the staged localip table in LDS
  uint32_t lds_scratch;          // byte offset of the per-wave regions (header transpose / candidate scratch)
  uint32_t wave_bytes;           // bytes per wave region
  uint32_t lds_bytes;            // dynamic LDS per workgroup
  uint16_t const_in_port;
  uint16_t direction;
  uint32_t hook;                 // PCN_IPT_HOOK_TC: strip an outer VLAN tag first (never with a fixed stride)
  uint32_t allow_logic;          // _INGRESS_ALLOWLOGIC (modules/ChainSelector.cpp:190-202)
  uint32_t empty_mask;           // bit c: chain c has no rules (ChainSelector default path)
  uint32_t drop_mask;            // bit c: chain c's default action is DROP
  uint32_t count_mask;           // bit c: packets of this launch can select chain c
  uint32_t fw;                   // 0: pcn-iptables dispatch; else pcn-firewall, PCN_FW_LAUNCH_*
  int32_t fast_chain;            // >= 0: every IPv4 TCP/UDP frame selects this chain (no localip,
                                 // allow logic or empty chain involved); -1: no wave fast path
  // Horus (the program the batch's Parser calls; horus_fields == 0: off)
  const uint32_t *horus;         // 4 u32 per slot
  uint32_t horus_flags;          // kHz*
  uint32_t horus_mask;           // slots - 1
  uint32_t horus_probes;         // longest probe sequence of a stored key
  uint32_t horus_fields;         // PCN_IPT_HZ_* set fields of the key
  uint32_t has_stale;            // the key has port fields: stale ports computed in the kernel
                                 // (classify.hip stale_lookback; chunked workgroup order)
  unsigned long long *horus_ctr; // [PCN_IPT_HORUS_MAX][2] pkts, bytes; null: not counted (stage A)
  int32_t hz_bins;               // first LDS counter bin of the Horus rule ids; -1 => wave-aggregated global atomics
  uint64_t *stale_desc;          // per 64-frame group of the batch: the published word (stale_word)
  const uint32_t *stale_carry;   // ports dword (wire bytes 34-37) the previous batches left (Q4)
  uint32_t *chunk_ctr;           // [0] workgroup start counter, [1] workgroups finished; zero before a
                                 // launch, and the launch's last workgroup zeroes both again
  uint64_t chunk_frames;         // frames per workgroup (a multiple of the block size)
  uint64_t gbase;                // batch index of this launch's frame 0 (a multiple of 64)
  uint32_t stale_epoch;          // this batch's publication epoch (24 bits, never 0)
  uint32_t *carry_out;           // non-null on a batch's last launch: its last workgroup writes the
                                 // ports the batch leaves to the next one (the carry, Q4)
  // Counter replicas: workgroup b adds each (packets, bytes) pair of its
  // counters as ONE u64, packets << kCtrPackShift | bytes, into word p (p = 0
  // default, 1 + rule id) of copy b & ctr_rep_mask at ch[c].ctr + ctr_pack_off
  // + (b & ctr_rep_mask) * ctr_rep_words.  The host folds the copies into the
  // plain block at ch[c].ctr before it reads one, and often enough that no
  // field of a copy can overflow (pcn_ipt.cpp, fold_counters / pack_bound).
  // Workgroups of a short launch finish together, and their flushes, all on
  // one block, serialised on the same few lines; the packed pair halves the
  // global atomics of the flush and of the rule ids past the LDS bins.
  // ctr_pack_off 0: plain pairs straight into ch[c].ctr (stage A's scratch).
  uint32_t ctr_rep_mask;         // copies - 1 (a power of two; 0: one copy)
  uint32_t ctr_rep_words;        // u64 words between packed copies
  uint32_t ctr_pack_off;         // u64 words from ch[c].ctr to packed copy 0; 0: unpacked
  // Deal statistics (pcn_ipt.cpp, the adaptive deal window): each workgroup
  // stores, in host-mapped memory, how many of its waves' rule stages dealt
  // more than 64 candidates -- the passes a 128-candidate window saves.  The
  // host picks the next launch's chain program from them without a sync.
  uint32_t *deal_stats;          // [grid] host-mapped u32 per workgroup; null: not counted
  uint32_t lds_stats;            // byte offset of the workgroup's u32 counter in LDS
  // Measurement only (PCN_IPT_DEBUG_CLOCKS=1, pcn_ipt_debug_clocks): thread 0 of
  // workgroup b stores s_memrealtime (100 MHz) at its start, after its prologue,
  // after its last frame and after its counter flush into dbg_clk[4 b .. 4 b + 3]
  unsigned long long *dbg_clk;   // null: not recorded
  // Split launches (classify.hip SPLIT, pcn_ipt.cpp): the gather kernel writes
  // each frame's rule-stage fields here (16 B a frame, kSplitNeed in the top
  // byte when the frame runs rules) and the rule kernel reads them back.
  uint32_t *split_rec;           // [n][4] u32; null: one fused kernel
  // Stage A of a stateful batch that also writes the walk records (pcn_ipt.cpp
  // ct_fused_prep; conntrack.hip then skips ct_prep): per frame its 32-byte
  // record (CtWalkOut::w), its key bucket and its {len, cinfo} word.  Null
  // otherwise.
  uint32_t *ct_brec;             // [n][8] u32
  uint32_t *ct_keys;             // [n]
  uint32_t *ct_lcs;              // [n]
  uint32_t ct_sentinel;          // the key bucket of packets without one (2^kbits - 1)
  // ... and its stale ports without waiting on other workgroups: every 64-frame
  // group publishes its ports word (ct_ports_word: its last TCP / UDP frame's
  // ports, or none) and a mask of the lanes whose record was built before the
  // ports the earlier groups leave are known (labelled, no ports of their own,
  // no TCP / UDP frame before them in the group); conntrack.hip ct_stale_fix
  // completes those records once every group has published.
  unsigned long long *ct_pdesc;  // [n / 64 + 1]
  unsigned long long *ct_fixm;   // [n / 64 + 1]
};
// split_rec word 3: proto | flags << 8 | ct << 16 | meta << 24, meta = chain (2 bits)
// | outer VLAN tag stripped (bit 2: the rule kernel's length is lens - 4) | kSplitNeed
constexpr uint32_t kSplitNeed = 0x80u, kSplitUntag = 0x04u;

// Packed counter pair: packets in bits 38-63, bytes in bits 0-37.
constexpr uint32_t kCtrPackShift = 38;
constexpr unsigned long long kCtrPackBytesMask = (1ull << kCtrPackShift) - 1;
constexpr unsigned long long kCtrPackPktsMax = (1ull << (64 - kCtrPackShift)) - 1;

// Host side of the packed copies (launch_classify): upper bounds of what any
// one copy holds since the last fold, and the fold to run before a launch
// that could overflow a field (it resets both bounds).
struct CopyBound {
  unsigned long long pkts, bytes;
  unsigned long long max_pkts, max_bytes;   // the fields' capacity (lower: a test hook)
  int (*fold)(void *ctx, void *stream);   // stream: a hipStream_t
  void *ctx;
};

// ---- conntrack walk records -------------------------------------------
// The record of a packet in the stateful pipeline (conntrack.hip): built by
// ct_prep, or -- in a batch whose frames are all shorter than 70 bytes, so no
// ICMP header quotes another, and with one label -- by the classify kernel's
// stage-A launch itself, which then is the batch's only pass over the frames.
// Both go through the two functions below, restated from
// Iptables_ChainSelector_dp.c:131-298 (Firewall_ChainForwarder_dp.c:20-42) and
// Iptables_ConntrackLabel_dp.c:190-531.
// Record kinds (conntrack.hip K_*): the same numbering.
constexpr uint32_t kCtKNone = 0, kCtKInv = 1, kCtKTcp = 2, kCtKUdp = 3, kCtKEcho = 4, kCtKReply = 5, kCtKErr = 6,
                   kCtKHard = 7;

// What a record is built from: the Parser's fields as conntrack.hip's parse
// reads them (multi-byte fields are little-endian loads of network-order bytes).
struct CtFrame {
  uint32_t status;               // 0 RX_DROP in the parser, 1 not IPv4 (pass), 2 IPv4 parsed
  uint32_t ports_ok;             // the Parser wrote srcPort / dstPort (TCP / UDP)
  uint32_t L, src, dst, seq, ack;
  uint32_t own, stale;           // wire bytes 34-37 of this frame; the shared struct's ports (Q4)
  uint32_t proto, flags, icmp;
  uint32_t isrc, idst, iproto, isport, idport;   // the quoted header (ICMP errors, long echo replies)
};

// ChainSelector (pcn-iptables) / ChainForwarder (pcn-firewall) as the
// conntrack labels see it: the chain a labelled packet's rules come from (3:
// none), PASS_LABELING, or no labelling at all.  horus: stage A found a Horus
// hit (DROP: final; ACCEPT: PASS_LABELING unless horus_final).
PCN_HD inline void ct_select(bool horus, bool horus_pass, bool fw, bool ingress, bool allow_logic, bool local_dst,
                             bool local_src, uint32_t empty_mask, uint32_t drop_mask, uint32_t &chain, bool &pass,
                             bool &labeled) {
  chain = 3;
  pass = false;
  labeled = true;
  if (horus) {
    if (horus_pass) pass = true;
    else labeled = false;
  } else if (fw) {
    chain = ingress ? 1u : 2u;                     // INGRESS / EGRESS in the FORWARD / OUTPUT slots
  } else if (ingress) {
    if (allow_logic) pass = true;
    else chain = local_dst ? 0u : 1u;              // INPUT / FORWARD
  } else if (local_src) {
    chain = 2u;                                    // OUTPUT
  } else {
    labeled = false;                               // egress PASS, no labelling
  }
  if (!fw && labeled && chain < 3 && ((empty_mask >> chain) & 1)) {
    if ((drop_mask >> chain) & 1) labeled = false; // DROP_NO_LABELING (default counters)
    else pass = true;                              // PASS_LABELING
  }
}

PCN_HD inline uint64_t ct_key_hash(uint32_t src, uint32_t dst, uint32_t proto, uint32_t sp, uint32_t dp) {
  uint64_t h = ((uint64_t(src) << 32) | dst) * 0x9E3779B97F4A7C15ull;
  h ^= ((uint64_t(proto) << 32) | (uint64_t(sp) << 16) | dp) * 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  return h ^ (h >> 32);
}

// The key bucket of a key hash: h % sentinel, sentinel = 2^kbits - 1 (kbits >= 8,
// conntrack.hip key_bits), by folding (2^kbits = 1 mod sentinel) instead of a
// 64-bit division.
PCN_HD inline uint32_t ct_bucket(uint64_t h, uint32_t sentinel) {
  const uint32_t k = 32 - __builtin_clz(sentinel);   // sentinel = 2^k - 1
  while (h > sentinel) h = (h & sentinel) + (h >> k);
  return h == sentinel ? 0u : static_cast<uint32_t>(h);
}

// The 32-byte walk record (conntrack.hip PackedRec: src, dst, sport | dport
// << 16, seq, ack, iports, proto | flags << 8 | kind << 16 | (rev | cinfo <<
// 2) << 24, o0), its key bucket (sentinel: no table access) and the {len,
// cinfo} word ct_count reads.  The key orders the addresses and ports
// (ConntrackLabel_dp.c:200-228); an ICMP packet's ports are the stale ones
// (Q4); an ICMP error keys on the header it quotes, a long echo reply keeps
// that header's key for its ICMP_MISS lookup (:491-529).
struct CtWalkOut {
  uint32_t w[8];
  uint32_t key, lcs;
  uint32_t kind;
};
PCN_HD inline CtWalkOut ct_walk_rec(const CtFrame &p, uint32_t chain, bool pass, bool labeled, int32_t o0,
                                    uint32_t sentinel) {
  CtWalkOut o{};
  uint32_t src = 0, dst = 0, sport = 0, dport = 0, seq = 0, ack = 0, iports = 0, proto = 0, flags = 0, rev = 0;
  uint32_t kind = kCtKNone;
  if (p.status != 2) {
    chain = 3;
    pass = false;
    labeled = false;
  }
  if (labeled) {
    const uint32_t ports = p.ports_ok ? p.own : p.stale;
    const uint32_t sp = ports & 0xffffu, dp = ports >> 16;
    uint32_t ipRev, portRev;
    if (p.src <= p.dst) { src = p.src; dst = p.dst; ipRev = 0; }
    else { src = p.dst; dst = p.src; ipRev = 1; }
    if (sp < dp) { sport = sp; dport = dp; portRev = 0; }
    else if (sp > dp) { sport = dp; dport = sp; portRev = 1; }
    else { sport = sp; dport = dp; portRev = ipRev; }
    proto = p.proto;
    rev = ipRev | (portRev << 1);
    seq = p.seq;
    ack = p.ack;
    flags = p.flags;
    if (p.proto == 6) kind = kCtKTcp;
    else if (p.proto == 17) kind = kCtKUdp;
    else if (p.proto == 1) {
      if (p.L < 42) kind = kCtKNone;                 // RX_DROP (:441-443)
      else if (p.icmp == 8) kind = kCtKEcho;
      else if (p.icmp == 0) kind = p.L >= 70 ? kCtKHard : kCtKReply;
      else if (p.icmp >= 13 && p.icmp <= 18) kind = kCtKInv;
      else if (p.L < 70) kind = kCtKNone;            // RX_DROP (:486-505)
      else kind = kCtKErr;
      if (kind == kCtKErr || kind == kCtKHard) {    // the quoted header's key
        const uint32_t qs = p.isrc <= p.idst ? p.isrc : p.idst, qd = p.isrc <= p.idst ? p.idst : p.isrc;
        const uint32_t qa = p.isport <= p.idport ? p.isport : p.idport;
        const uint32_t qb = p.isport <= p.idport ? p.idport : p.isport;
        if (kind == kCtKErr) {
          src = qs; dst = qd; sport = qa; dport = qb; proto = p.iproto;
        } else {
          seq = qs; ack = qd; flags = p.iproto; iports = qa | (qb << 16);
        }
      }
    } else {
      kind = kCtKInv;                                // :562-566
    }
  }
  const uint32_t cinfo = (chain & 3u) | (pass ? 4u : 0u);
  const bool member = kind >= kCtKTcp && kind <= kCtKErr;
  o.key = member ? ct_bucket(ct_key_hash(src, dst, proto & 0xffu, sport & 0xffffu, dport & 0xffffu), sentinel)
                 : sentinel;
  o.lcs = (p.L & 0xffffu) | cinfo << 16;
  o.w[0] = src;
  o.w[1] = dst;
  o.w[2] = (sport & 0xffffu) | (dport & 0xffffu) << 16;
  o.w[3] = seq;
  o.w[4] = ack;
  o.w[5] = iports;
  o.w[6] = (proto & 0xffu) | (flags & 0xffu) << 8 | kind << 16 | (rev | cinfo << 2) << 24;
  o.w[7] = static_cast<uint32_t>(o0);
  o.kind = kind;
  return o;
}

// The same record once the stale ports (Q4) it was built with are known to be
// `stale` (a labelled record of a frame whose Parser wrote no ports: its
// kind is not kCtKErr, which keys on the quoted header): the ports word, the
// rev bits of pfk and the key bucket, as ct_walk_rec computes them.
PCN_HD inline uint32_t ct_rec_restale(uint32_t src, uint32_t dst, uint32_t &ports, uint32_t &pfk, uint32_t stale,
                                      uint32_t sentinel) {
  const uint32_t sp = stale & 0xffffu, dp = stale >> 16;
  const uint32_t ipRev = (pfk >> 24) & 1u;
  uint32_t sport, dport, portRev;
  if (sp < dp) { sport = sp; dport = dp; portRev = 0; }
  else if (sp > dp) { sport = dp; dport = sp; portRev = 1; }
  else { sport = sp; dport = dp; portRev = ipRev; }
  ports = sport | dport << 16;
  pfk = (pfk & ~(3u << 24)) | (ipRev | portRev << 1) << 24;
  const uint32_t kind = (pfk >> 16) & 0xffu, proto = pfk & 0xffu;
  const bool member = kind >= kCtKTcp && kind <= kCtKErr;
  return member ? ct_bucket(ct_key_hash(src, dst, proto, sport, dport), sentinel) : sentinel;
}

// Ports words per 64-frame group (conntrack.hip ports_word): bit 40 published,
// bits 32-33 the state, bits 0-31 the ports of the group's last TCP / UDP frame.
constexpr unsigned long long kCtPortsLocal = 1, kCtPortsNone = 3;
PCN_HD inline unsigned long long ct_ports_word(unsigned long long st, uint32_t ports) {
  return (1ull << 40) | (st << 32) | ports;
}

// LaunchArgs::fw: pcn-firewall dispatch with its conntrack mode (defines.h:56-58)
#define PCN_FW_LAUNCH_CT_OFF 1     // DISABLED: no ConntrackLabel stage
#define PCN_FW_LAUNCH_CT_MANUAL 2  // labels + ICMP checks, then the chain
#define PCN_FW_LAUNCH_CT_AUTO 3    // MANUAL + ESTABLISHED accepted before the chain

}  // namespace pcn
