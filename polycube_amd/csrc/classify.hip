// classify.hip — the MI355X (gfx950) batch classifier for pcn-iptables.
//
// One lane per packet.  Each lane reads the 48-byte header window of its frame
// and runs the reference's Parser / ChainSelector / ConntrackLabel checks
// (Iptables_Parser_dp.c:94-153, Iptables_ChainSelector_dp.c:131-298,
// Iptables_ConntrackLabel_dp.c:436-531).  It then maps every present field to
// a class through the chain's table image (devchain.h) — staged in LDS by each
// workgroup — and ANDs the class summaries.  Only words whose summary bit
// survives are fetched from the HBM vector pool, and only for fields whose
// word is not FULL.  The lowest set bit of a word is its lowest rule id (the
// permutation keeps ids ascending inside a word), so the matched rule is the
// minimum over the non-zero candidate words — the same rule the reference's
// per-field ANDs + BitScan pick (Iptables_{IpLookup,L4ProtocolLookup,
// L4PortLookup,InterfaceLookup,TcpFlagsLookup,ConntrackMatch,BitScan,
// ActionLookup}_dp.c).  Integer work only; no MFMA.
//
// Per-rule and default pkts/bytes counters go to an LDS histogram per
// workgroup (u64 LDS atomics; default bins wave-aggregated with a ballot) that
// is flushed once per workgroup with global u64 atomics.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include <cstdint>
#ifndef __HIPCC_RTC__
#include <cstdlib>
#endif

#include "devchain.h"
#include "pcn_ipt.h"
#ifdef PCN_JIT
#include "pcn_jit_spec.h"   // generated per chain image by jit.cpp (PCN_JIT_CHAIN, PCN_JIT_FIXED, ...)
#endif

extern __shared__ __attribute__((aligned(16))) uint8_t pcn_smem[];

// Measurement-only ablation builds (tools/ablate.py; never the product .so):
// 1 parse only, 2 + field lookups, 3 + summary AND, 4 full minus counters,
// 5 full minus the end-of-launch counter flush, 6 full minus the per-rule
// counter bins, 7 per-rule bins by plain stores (wrong counts; cost of the atomic),
// 8 full minus the global atomics of the rule ids past the LDS bins,
// 9 global counter adds (flush and ids past the bins) without the byte word
// (wrong byte counts; what one packed atomic per counter pair would save).
#ifndef PCN_ABLATE
#define PCN_ABLATE 0
#endif
#ifndef PCN_HDR_LDS
#define PCN_HDR_LDS 1    // fixed stride: 1 coalesced chunks transposed through LDS, 0 per-lane strided loads
#endif
// Frames per lane in flight ahead of the one being classified.  Fixed
// stride: 2 (A/B with settled clocks, config 3: -3 % kernel time at hit rate
// 0.5, config 2: -2.5 %; profiles/r02_ab_prefetch*.log).  Offsets/lens
// batches: 1 (their 13-dword windows cost more registers; depth 2 measured
// +2 % on config 5).
#ifndef PCN_PREFETCH_FIXED
#define PCN_PREFETCH_FIXED 2
#endif
#ifndef PCN_PREFETCH_GENERIC
#define PCN_PREFETCH_GENERIC 1
#endif
#ifdef PCN_PREFETCH      // one depth for both paths (measurement builds)
#undef PCN_PREFETCH_FIXED
#undef PCN_PREFETCH_GENERIC
#define PCN_PREFETCH_FIXED PCN_PREFETCH
#define PCN_PREFETCH_GENERIC PCN_PREFETCH
#endif
#ifndef PCN_FASTPATH
#define PCN_FASTPATH 1   // wave fast path: all 64 frames plain IPv4 TCP/UDP -> straight-line parse
#endif
#ifndef PCN_PF_FAST
#define PCN_PF_FAST 1    // whole-wave frame groups: uniform base + per-lane constant offsets
#endif
#ifndef PCN_FLUSH_ROT
#define PCN_FLUSH_ROT 1  // per-workgroup rotation of the counter flush order
#endif
#ifndef PCN_CAND_PRIO
#define PCN_CAND_PRIO 1  // s_setprio of a wave in the candidate stage (-1: leave it); a wave there
                         // holds LDS state the others' memory waits do not need (A/B: -2 % / -4.5 %
                         // at hit rate 0.5 / 1, profiles/r01_ab17_cand_prio.log)
#endif
#ifndef PCN_HDR_NT
#define PCN_HDR_NT 1     // header loads with the nontemporal hint (read once, never again)
#endif
template <typename T>
__device__ __forceinline__ T hdr_load(const T *p) {
  if (PCN_HDR_NT) return __builtin_nontemporal_load(p);
  return *p;
}
// Fixed-stride header chunks as asm loads the compiler does not count
// (cdna_hip_programming.md §5.7 item 1): the compiler's own bookkeeping waited
// vmcnt(0) at the loop head, draining the other stage's chunks (issued half an
// iteration earlier) with this one's.  process() waits for a stage itself with
// a counted vmcnt: every later stage's three chunk loads are unconditional, so
// at least 3 (PF - 1) memory operations follow a stage's chunks.
// Chain programs only (checked spill-free when built, jit.cpp); the generic
// kernels keep compiler-counted loads.  A/B at config 3, hit rate 0 / 0.25 /
// 0.5 / 0.75 / 1: +2.6 / -2.0 / -1.9 / -0.7 / -1.0 % kernel time
// (profiles/r02_ab_hdr_asm.log).
#ifndef PCN_HDR_ASM
#ifdef PCN_JIT
#define PCN_HDR_ASM 1
#else
#define PCN_HDR_ASM 0
#endif
#endif
#ifndef PCN_STAGE_FAST
#define PCN_STAGE_FAST 1 // prologue: first headers in flight during the image stage, staging loads batched
#endif
// Offsets / lengths batches (IMIX): a wave's 64 scattered headers are fetched
// four lanes to a frame, one 16-byte chunk each from the frame's 16-byte
// aligned start, so one load instruction reads 16 frames' contiguous bytes
// (tools/gather_probe.hip on config 5's layout: 0.080 ms for 2^22 frames,
// against 0.132 ms one lane per frame), and the chunks are transposed through
// the wave's LDS region (16 frames a round, 80-byte rows: the 1.25 KB the
// candidate stage uses later).  0: one lane per header (load_generic).
#ifndef PCN_GEN_QUAD
#define PCN_GEN_QUAD 1
#endif
// Offsets / lengths batches of a chain program whose PART is dense (read
// from L2 in the candidate stage: config 5): the next header prefetch is
// issued after the candidate stage instead of before the parse.  vmcnt
// completes in order, so the stage's L2 reads wait for every load issued
// before them, and a prefetch issued first was forced to land there.  A/B
// on config 5 at 2^22 frames (profiles/r05_s2/ab_cfg5*.log): XDP 153-156 ->
// 148 us, TC 177.6 -> 174.4 us; at depth 2 (either issue point) no gain.
#ifndef PCN_PF_LATE
#define PCN_PF_LATE 1
#endif
// Offsets batches: a frame's offset is loaded one prefetch ahead of its
// header, so the header loads of a prefetch do not first wait on the offset
// load (two dependent memory round trips per frame otherwise).
#ifndef PCN_OFF_AHEAD
#define PCN_OFF_AHEAD 1
#endif
// Split launches (SPLIT 2, the rule kernel): records in flight per lane, and
// whether the next record is fetched after the rule stage (as the fused
// kernel does for dense PART) rather than before it.
#ifndef PCN_SPLIT_R_PF
#define PCN_SPLIT_R_PF 2
#endif
#ifndef PCN_SPLIT_R_LATE
#define PCN_SPLIT_R_LATE 0
#endif
// Tuning switches (tools/ablate.py builds experiment variants with -D...).

namespace pcn {

namespace {

constexpr int kBlock = PCN_BLOCK;
constexpr uint32_t kHashMul = 0x9E3779B1u;
constexpr uint32_t kNoRule = 0xFFFFFFFFu;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
#ifndef PCN_HDR_ASM_MEM
#define PCN_HDR_ASM_MEM 0   // 1: the asm chunk loads ordered against the compiler's memory operations (A/B: slower)
#endif
__device__ __forceinline__ void hdr_load_asm(u32x4 &dst, const u32x4 *p) {
  if (PCN_HDR_ASM_MEM) {
    if (PCN_HDR_NT) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(dst) : "v"(p) : "memory");
    else asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(p) : "memory");
  } else {
    if (PCN_HDR_NT) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(dst) : "v"(p));
    else asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(p));
  }
}

__device__ __forceinline__ uint32_t bswap16u(uint32_t x) { return ((x & 0xff) << 8) | ((x >> 8) & 0xff); }

// Table image accessor.  With LDS, the image prefix [0, limit) is staged in
// LDS (the whole image, or its per-packet tables when the whole does not fit)
// and a table at or past `limit` is read from HBM/L2.  Tables never straddle
// the limit, so the choice depends on the table's base only: a wave-uniform
// branch in the generic kernel, a constant in a chain program.
#ifndef PCN_BUF_LOADS
#define PCN_BUF_LOADS 1  // dense PART cells through buffer loads (Tab::g16 / g32)
#endif
template <bool LDS>
struct Tab {
  const uint8_t *g;
  uint32_t base;    // LDS byte offset of the image
  uint32_t limit;   // staged image bytes
  // `off` may be "negative" (a u32 wrap: the candidate stage addresses PART
  // through POOL's base), so the image offset is formed in 32 bits first.
  template <typename T>
  __device__ __forceinline__ T ld(uint32_t tbl, uint32_t off) const {
    const uint32_t at = tbl + off;
    return (LDS && tbl < limit) ? *reinterpret_cast<const T *>(pcn_smem + base + at)
                                : *reinterpret_cast<const T *>(g + at);
  }
  // A table past the LDS limit (the dense PART of a large chain) through a
  // buffer load: a 32-bit offset from the image base in SGPRs, where the
  // global form spends a 64-bit address computation (3-4 VALU) per load.
  __device__ __forceinline__ uint32_t g16(uint32_t tbl, uint32_t off) const {
    if (PCN_BUF_LOADS) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(g), 0, 0x7fffffff,
                                                                         0x00020000);
      return __builtin_amdgcn_raw_buffer_load_b16(r, tbl + off, 0, 0);
    }
    return *reinterpret_cast<const uint16_t *>(g + (tbl + off));
  }
  __device__ __forceinline__ uint32_t g32(uint32_t tbl, uint32_t off) const {
    if (PCN_BUF_LOADS) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(g), 0, 0x7fffffff,
                                                                         0x00020000);
      return __builtin_amdgcn_raw_buffer_load_b32(r, tbl + off, 0, 0);
    }
    return *reinterpret_cast<const uint32_t *>(g + (tbl + off));
  }
  __device__ __forceinline__ uint32_t u32(uint32_t tbl, uint32_t off) const { return ld<uint32_t>(tbl, off); }
  __device__ __forceinline__ uint32_t u16(uint32_t tbl, uint32_t off) const { return ld<uint16_t>(tbl, off); }
  __device__ __forceinline__ uint32_t u8(uint32_t tbl, uint32_t off) const { return ld<uint8_t>(tbl, off); }
  __device__ __forceinline__ uint64_t u64(uint32_t tbl, uint32_t off) const { return ld<uint64_t>(tbl, off); }
  __device__ __forceinline__ u32x4 u128(uint32_t tbl, uint32_t off) const { return ld<u32x4>(tbl, off); }
  __device__ __forceinline__ u32x3 u96(uint32_t tbl, uint32_t off) const { return ld<u32x3>(tbl, off); }
};

// Header window as little-endian dwords: bytes 0..47 (the fixed-stride path)
// or 0..51 (the generic path, which also serves the TC hook, where an outer
// VLAN tag shifts the IPv4 header by 4 bytes).
struct Hdr { uint32_t w[13]; };

// Fixed-stride frame: bytes 12..47 (ethertype .. TCP flags); the MAC
// addresses (w0..w2) are never read.
__device__ __forceinline__ void load_fixed(const uint8_t *frame, Hdr &h) {
  const u32x4 *p = reinterpret_cast<const u32x4 *>(frame);
  const uint32_t w3 = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(frame) + 3);
  u32x4 b = __builtin_nontemporal_load(p + 1);
  u32x4 c = __builtin_nontemporal_load(p + 2);
  h.w[0] = h.w[1] = h.w[2] = h.w[12] = 0;
  h.w[3] = w3;
  h.w[4] = b.x; h.w[5] = b.y; h.w[6] = b.z; h.w[7] = b.w;
  h.w[8] = c.x; h.w[9] = c.y; h.w[10] = c.z; h.w[11] = c.w;
}

// Unaligned frame start: 14 aligned dwords, each only if it lies inside the
// buffer, then byte-shifted into the window.
// A frame whose 16 dwords lie inside the buffer (every frame but the last
// few) is read as four 16-byte loads from its dword-aligned start: global
// loads need only dword alignment, and four requests per lane instead of
// fourteen is what an IMIX batch of scattered headers is bound by.
typedef uint32_t u32x4d __attribute__((ext_vector_type(4), aligned(4)));
#ifndef PCN_GENERIC_X4
#define PCN_GENERIC_X4 1
#endif
__device__ __forceinline__ void load_generic(const uint8_t *frames, uint64_t frames_bytes,
                                             uint64_t off, Hdr &h) {
  uint64_t base = off & ~uint64_t(3);
  uint32_t sh = static_cast<uint32_t>(off & 3);
  uint32_t d[16];
  if (PCN_GENERIC_X4 && base + 64 <= frames_bytes) {
    const u32x4d *p = reinterpret_cast<const u32x4d *>(frames + base);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4d v = __builtin_nontemporal_load(p + q);   // (a template would drop the 4-byte alignment)
      d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 14; ++k) {
      uint64_t at = base + 4u * k;
      d[k] = (at + 4 <= frames_bytes) ? *reinterpret_cast<const uint32_t *>(frames + at) : 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < 13; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

template <bool FIXED>
__device__ __forceinline__ void load_header(const LaunchArgs &a, uint64_t i, Hdr &h, uint32_t &L) {
  if (FIXED) {
    load_fixed(a.frames + i * a.stride, h);
  } else {
    uint64_t off = a.offsets ? a.offsets[i] : i * a.stride;
    load_generic(a.frames, a.frames_bytes, off, h);
    L = a.lens ? a.lens[i] : a.fixed_len;
  }
}

// localip is staged in LDS (sorted NBO u32), so the search makes no global
// load inside the loop.
__device__ __forceinline__ bool localip_has(const LaunchArgs &a, uint32_t ip) {
  const uint32_t *tab = reinterpret_cast<const uint32_t *>(pcn_smem + a.lds_localip);
  uint32_t lo = 0, hi = a.nlocal;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    uint32_t v = tab[mid];
    if (v == ip) return true;
    if (v < ip) lo = mid + 1; else hi = mid;
  }
  return false;
}

// Kernel-LPM answer for a host-order address: the bucket on the top address
// bits gives the boundaries inside it, then a branchless upper-bound search
// of `steps` (wave-uniform; unrolled in a chain program) probes finds the
// interval.
// Window mode (win != 0): the bucket's <= win boundaries are read at once
// and counted; boundaries past the bucket (the next buckets', or the
// 0xFFFFFFFF padding) exceed every address in it, except that the padding
// equals h == 0xFFFFFFFF, where all real ones are below h too -- hence min.
template <bool LDS>
__device__ __forceinline__ uint32_t ip_class(const Tab<LDS> &t, uint32_t bkt, uint32_t shift, uint32_t steps,
                                             uint32_t win, uint32_t bnd, uint32_t cls, uint32_t h) {
  const uint32_t e = t.u32(bkt, 4 * (h >> shift));
  if (win) {
    const uint32_t first = e & 0xFFFFu;
    uint32_t n = 0;
    for (uint32_t k = 0; k < win; ++k) n += t.u32(bnd, 4 * (first + k)) <= h ? 1u : 0u;
    const uint32_t count = e >> 16;
    return t.u16(cls, 2 * (first + (n < count ? n : count)));
  }
  uint32_t lo = e & 0xFFFFu;
  const uint32_t end = lo + (e >> 16);
  for (uint32_t k = steps; k-- > 0;) {
    const uint32_t probe = lo + (1u << k);          // candidate: bnd[lo .. probe) all <= h
    const uint32_t idx = (probe <= end ? probe : lo + 1) - 1;
    const bool ok = probe <= end && t.u32(bnd, 4 * idx) <= h;
    lo = ok ? probe : lo;
  }
  return t.u16(cls, 2 * lo);
}

// Port / iface hash: the key is in its home slot or the next one (the image
// builder guarantees it), so two adjacent reads decide without a loop.
template <bool LDS>
__device__ __forceinline__ uint32_t key_class(const Tab<LDS> &t, uint32_t tab, uint32_t mask, uint32_t wild,
                                              uint32_t key) {
  const uint32_t h = (key * kHashMul) >> __builtin_clz(mask);
  const uint32_t e0 = t.u32(tab, 4 * h), e1 = t.u32(tab, 4 * h + 4);
  const bool m0 = e0 != PCN_HASH_EMPTY && (e0 >> 16) == key;
  const bool m1 = e1 != PCN_HASH_EMPTY && (e1 >> 16) == key;
  return m0 ? (e0 & 0xffff) : (m1 ? (e1 & 0xffff) : wild);
}

// Horus: the key of the per-CPU packet struct.  pd = the Parser's
// srcPort/dstPort as stored (wire bytes 34-37 as a little-endian dword).
// pcn-iptables (Iptables_Horus_dp.c:112-133): the packed struct reads bytes
// 9-10 / 11-12 of the aligned one: [padding 0, first source-port byte] and
// [second source-port byte, first destination-port byte].  pcn-firewall
// (kHzNatural, Firewall_Horus_dp.c:112-133): packed on both sides, the ports
// as stored.
__device__ __forceinline__ bool horus_lookup(const LaunchArgs &a, uint32_t saddr, uint32_t daddr, uint32_t proto,
                                             uint32_t pd, uint32_t &meta) {
  const uint32_t F = a.horus_fields;
  const bool nat = a.horus_flags & kHzNatural;
  const uint32_t sk = nat ? (pd & 0xffffu) : (pd & 0xffu) << 8;
  const uint32_t dk = nat ? (pd >> 16) : ((pd >> 8) & 0xffu) | (((pd >> 16) & 0xffu) << 8);
  const uint32_t ks = (F & PCN_IPT_HZ_SRCIP) ? saddr : 0u, kd = (F & PCN_IPT_HZ_DSTIP) ? daddr : 0u;
  const uint32_t kp = (F & PCN_IPT_HZ_L4PROTO) ? proto : 0u;
  const uint32_t kports = ((F & PCN_IPT_HZ_SRCPORT) ? sk : 0u) | (((F & PCN_IPT_HZ_DSTPORT) ? dk : 0u) << 16);
  uint32_t slot = horus_hash(ks, kd, kports, kp) & a.horus_mask;
  for (uint32_t k = 0; k < a.horus_probes; ++k) {
    const u32x4 e = *reinterpret_cast<const u32x4 *>(a.horus + 4 * slot);
    if (!(e.w & kHorusUsed)) return false;
    if (e.x == ks && e.y == kd && e.z == kports && (e.w & 0xffu) == kp) { meta = e.w; return true; }
    slot = (slot + 1) & a.horus_mask;
  }
  return false;
}

// Fused stale ports: one published word per 64-frame group,
// {epoch:24 | status:2 | ports:32} (an old epoch: not published yet).
constexpr uint32_t kStaleLocal = 1;       // the group's last TCP/UDP frame's ports
constexpr uint32_t kStaleInclusive = 2;   // no TCP/UDP frame in the group: the ports before it
constexpr uint32_t kStaleNone = 3;        // no TCP/UDP frame in the group, the ports before it not known
__device__ __forceinline__ uint64_t stale_word(uint32_t epoch, uint32_t status, uint32_t ports) {
  return (static_cast<uint64_t>(epoch) << 40) | (static_cast<uint64_t>(status) << 32) | ports;
}
// The ports the last TCP/UDP frame before group g left: walk back through the
// published groups (waiting for one not yet published: it belongs to a
// workgroup that started earlier), else the carry of the previous batches.
__device__ uint32_t stale_lookback(const LaunchArgs &a, uint64_t g) {
  g = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g >> 32))) << 32) |
      __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g));
  while (g > 0) {
    --g;
    uint64_t d;
    for (;;) {
      d = __hip_atomic_load(&a.stale_desc[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((d >> 40) == a.stale_epoch) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (((d >> 32) & 3) != kStaleNone) return static_cast<uint32_t>(d);
  }
  return *a.stale_carry;
}

struct Parsed {
  uint32_t saddr, daddr;       // NBO as loaded
  uint32_t proto, sport, dport, flags;
  uint32_t ct;                 // conntrack status 0..3 (or >3: invalid input)
};

// ConntrackLabel_dp.c:436-531 (Firewall_ConntrackLabel_dp.c: the same code):
// the ICMP length checks that drop before any rule.  Sets the ICMP type
// (0xffffffff for other protocols).
__device__ __forceinline__ bool icmp_drop(const Parsed &p, const Hdr &h, uint32_t L, uint32_t &icmp_type) {
  icmp_type = 0xffffffffu;
  if (p.proto != 1) return false;
  icmp_type = (h.w[8] >> 16) & 0xff;
  if (L < 42) return true;
  return icmp_type != 8 && icmp_type != 0 && !(icmp_type >= 13 && icmp_type <= 18) && L < 70;
}

// The label an empty connection table gives (ConntrackLabel_dp.c:372-383).
__device__ __forceinline__ uint32_t empty_table_label(const Parsed &p, uint32_t icmp_type) {
  if (p.proto == 6) return (p.flags & 0x02) && ((p.flags | 0x02) == 0x02) ? 0u : 3u;
  if (p.proto == 17) return 0u;
  return icmp_type == 8 ? 0u : 3u;
}

// ---- rule-chain stage, part 1 (per lane) ----
// Maps the packet to its NS slot classes: 0 = META (proto x tcpflags x
// conntrack, plus the key fields the chain joined to it), 1/2 = IP src/dst,
// then the key fields (sport, dport, iface) that keep their own slot
// (lay.key_slot).  Returns true when the packet needs the candidate stage;
// otherwise the verdict is decided here (a field without an entry takes the
// default action, a bad conntrack label drops).  Absent or skipped fields
// contribute the all-ones vector.
template <bool LDS, int NS>
__device__ __forceinline__ bool chain_classes(const DevChain &ch, const Parsed &p, uint32_t port, uint32_t cls[NS],
                                              uint32_t &verdict, int32_t &rid) {
  const Tab<LDS> t{ch.image, ch.lds_image, ch.lds_limit};
  const TableLayout &lay = ch.lay;
  const uint32_t present = ch.present;
  const uint32_t all = ch.all_cls;
#pragma unroll
  for (int f = 1; f < NS; ++f) cls[f] = all;
  uint32_t mi = 0;   // meta index
  if (present & (1u << PCN_IPT_F_CONNTRACK)) {
    if (p.ct > 3) { rid = PCN_IPT_RID_NOCHAIN; verdict = PCN_IPT_DROP; return false; }   // array miss => RX_DROP
    mi += t.u8(lay.ct_idx, p.ct) * lay.meta_stride[2];
  }
  if (present & (1u << PCN_IPT_F_L4PROTO)) mi += t.u8(lay.proto_idx, p.proto) * lay.meta_stride[0];
  if (present & (1u << PCN_IPT_F_TCPFLAGS))                        // TcpFlagsLookup_dp.c:93-97
    mi += (p.proto == 6 ? t.u16(lay.flags_idx, 2 * p.flags) : lay.flags_skip) * lay.meta_stride[1];
  const bool l4 = p.proto == 6 || p.proto == 17;                    // L4PortLookup_dp.c:99-103
  const int key_field[3] = {PCN_IPT_F_SPORT, PCN_IPT_F_DPORT, PCN_IPT_F_IFACE};
  const uint32_t key[3] = {p.sport, p.dport, port};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (!(present & (1u << key_field[i]))) continue;
    uint32_t x = key_class(t, lay.hash[i], lay.hash_mask[i], lay.hash_wild[i], key[i]);
    if (i < 2) x = l4 ? x : lay.key_skip[i];
    const uint32_t slot = lay.key_slot[i];
    if (slot == 0) {
      mi += x * lay.meta_stride[3 + i];
    } else {
#pragma unroll
      for (int f = 3; f < NS; ++f) cls[f] = slot == static_cast<uint32_t>(f) ? x : cls[f];
    }
  }
  cls[0] = t.u16(lay.meta, 2 * mi);
  if (present & (1u << PCN_IPT_F_IPSRC))
    cls[1] = ip_class(t, lay.ip_bkt[0], lay.ip_shift[0], lay.ip_steps[0], lay.ip_win[0], lay.ip_bnd[0], lay.ip_cls[0], __builtin_bswap32(p.saddr));
  if (present & (1u << PCN_IPT_F_IPDST))
    cls[2] = ip_class(t, lay.ip_bkt[1], lay.ip_shift[1], lay.ip_steps[1], lay.ip_win[1], lay.ip_bnd[1], lay.ip_cls[1], __builtin_bswap32(p.daddr));
  bool miss = false;
#pragma unroll
  for (int f = 0; f < NS; ++f) miss |= cls[f] == PCN_CLS_MISS;
  if (miss) { rid = PCN_IPT_RID_DEFAULT; verdict = static_cast<uint32_t>(ch.default_action); return false; }
  if (PCN_ABLATE == 2) {   // keep the lookups alive: the verdict depends on them
    uint32_t x = 0;
#pragma unroll
    for (int f = 0; f < NS; ++f) x ^= cls[f];
    rid = PCN_IPT_RID_DEFAULT;
    verdict = x & 1;
    return false;
  }
  return true;
}

// Per-wave LDS scratch of the candidate stage.  It shares the wave's LDS
// region with the header transpose buffer (used earlier in the iteration).
#ifndef PCN_ITEM_CLS
#define PCN_ITEM_CLS 1   // 1: candidates carry their owner's classes; 0: owners stage class rows
#endif
#ifndef PCN_WFIELDS
#define PCN_WFIELDS 2    // dense PART: read a field's PART cell only where its slot can be partial
#endif
#ifndef PCN_REC_PIN
#define PCN_REC_PIN 0    // 1: candidate records all issued before the first is used (A/B: 1.6 % slower, profiles/r02_ab_recpin.log)
#endif
// An empty asm that takes every register of r: the loads that produce them
// are all issued before it, and each stays live until it.
template <int N>
__device__ __forceinline__ void pin_regs(u32x4 (&r)[N]) {
  static_assert(N >= 1 && N <= 6, "slot count");
  if constexpr (N == 1) asm volatile("" : "+v"(r[0]));
  else if constexpr (N == 2) asm volatile("" : "+v"(r[0]), "+v"(r[1]));
  else if constexpr (N == 3) asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]));
  else if constexpr (N == 4) asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]));
  else if constexpr (N == 5) asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]));
  else asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]));
}

// Two items per worker lane (a deal window of 128 candidates): a wave with
// more than 64 candidates (hit rate 1) pays one deal pass, not two -- the
// second item's dependent LDS chain runs in the shadow of the first's.
// 1: fixed-stride launches (their wave region is the 3 KB transpose buffer);
// 2: every launch whose wave region holds the 128 items (LaunchArgs::wave_bytes).
// Chain programs of chains with two or more summary blocks get 2 (jit.cpp:
// config 5's 10k rules deal ~200 candidates a wave), others 0 (config 3 at
// hit rate 0.5 deals fewer than 64 a wave, and the larger program cost 1.5 %).
#ifndef PCN_DEAL2
#define PCN_DEAL2 0
#endif
constexpr uint32_t kDeal2Bytes = 64 * 4 + 128 * 16;   // best[64] + item[128]
static_assert(kDeal2Bytes == PCN_DEAL2_WAVE_BYTES, "the host sizes the wave region for the 128-item window");
struct WaveScratch {
  uint32_t best[64];     // per owner lane: min (rule id << 1 | action)
  u32x4 item[64];        // (owner lane << 16 | candidate word, the owner's classes as u16 pairs)
#if !PCN_ITEM_CLS
  u32x4 cls[64];         // each owner's classes
#endif
};
static_assert(sizeof(WaveScratch) <= PCN_WAVE_SCRATCH_BYTES && PCN_WAVE_SCRATCH_BYTES <= PCN_WAVE_LDS_BYTES,
              "scratch fits the per-wave region");
static_assert(!PCN_DEAL2 || (kDeal2Bytes <= PCN_WAVE_LDS_BYTES && PCN_ITEM_CLS),
              "a 128-item window fits the fixed-stride wave region");

// ---- rule-chain stage, part 2 (whole wave, converged) ----
// Lanes with `active` AND their class summaries into a candidate-word mask,
// one 64-word block at a time.  The (lane, word) candidate pairs of the whole
// wave, over all blocks, are queued in the wave's LDS scratch and dealt out
// one per lane, 64 at a time, so a lane with many candidates does not hold
// the wave hostage and a chain of several blocks (config 5: 10k rules) pays
// one deal per 64 candidates, not one per block: each worker re-reads its
// owner's class records, ANDs the partial words of its one word and folds the
// matched entry into the owner's slot with an LDS atomic min.  Returns the
// owner's best entry.
template <int K>
struct IntK {
  static constexpr int value = K;
};

// Chains of 2-4 summary blocks in a chain program (MERGE, PCN_MERGE_BLOCKS):
// every block's summary words are read and ANDed at once (one LDS round trip),
// one queue prefix covers all of them and one divergent loop queues a lane's
// candidates of every block, instead of a summary read, a prefix and a queue
// loop per block.
#ifndef PCN_MERGE_BLOCKS
#define PCN_MERGE_BLOCKS 1
#endif
template <bool LDS, int NS, uint32_t WMAX = 64, bool MERGE = false>
__device__ __forceinline__ uint32_t chain_candidates(const DevChain &ch, bool active, const uint32_t cls[NS],
                                                     WaveScratch *ws, uint32_t wave_bytes, uint32_t &wide) {
  static_assert(WMAX == 64 || WMAX == 128, "deal window");
  // the window: 128 items when the build has the two-item workers and the
  // wave's LDS region holds them (wave-uniform), else 64
  const uint32_t W = WMAX > 64 && wave_bytes >= kDeal2Bytes ? 128u : 64u;
  const uint32_t lane = __lane_id();
  if (__ballot(active) == 0) return kNoRule;
  const Tab<LDS> t{ch.image, ch.lds_image, ch.lds_limit};
  const TableLayout &lay = ch.lay;
  const uint32_t nrw = ch.nrw, nsw = ch.nsw;
  bool staged = false;  // best slots written (only once some lane has a candidate)
  uint64_t mseen = 0;   // PCN_ABLATE == 3 only
  u32x4 *const items = ws->item;   // W entries (a 128 window runs past the struct into the wave region)
  // One worker lane's K queued items (K = 2: the second item's chain of
  // dependent LDS reads issues alongside the first's).  A lane without a
  // second item reads item 0 in its place -- the same addresses in every such
  // lane, LDS broadcasts -- and folds nothing (`two`).
  auto work = [&](auto kk, const uint32_t (&idx)[decltype(kk)::value], bool two) {
    constexpr int K = decltype(kk)::value;
    u32x4 it[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      if (PCN_ITEM_CLS) {
        it[q] = items[idx[q]];
      } else {
        const uint32_t x = reinterpret_cast<const uint32_t *>(items)[idx[q]];
#if !PCN_ITEM_CLS
        it[q] = ws->cls[x >> 16];
#endif
        it[q].x = x;
      }
    }
    uint32_t owner[K], w[K], k[K], bit[K], oc[K][NS];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      owner[q] = it[q].x >> 16;
      w[q] = it[q].x & 0xffff;
      k[q] = w[q] >> 6;
      bit[q] = w[q] & 63;
      const uint32_t packed[3] = {it[q].y, it[q].z, it[q].w};
#pragma unroll
      for (int f = 0; f < NS; ++f) oc[q][f] = (packed[f / 2] >> (16 * (f & 1))) & 0xffff;
    }
    // At a candidate word every field's summary bit is set, so a field is
    // PARTIAL there iff its PM bit is set; one 16-byte read gives PM and
    // PBASE.  Straight-line on purpose: every record read, then every word
    // read, issue back to back.  A FULL field reads POOL[0], the all-ones
    // word (indexed PART: through the zero cell, index 0).
    uint32_t at[K][NS];   // LDS/image offset of each field's u64 word
    u32x3 recs[K][NS];    // {PM lo, PM hi, PBASE} (the record's 4th dword is padding)
    uint32_t wf[K];       // dense PART: the slots that can be partial at the word (LDS)
    if (lay.part_dense) {
#pragma unroll
      for (int q = 0; q < K; ++q) wf[q] = PCN_WFIELDS && lay.wfields ? t.u8(lay.wfields, w[q]) : 0xffu;
    }
    if (!lay.part_dense) {
      // all records in flight together: one LDS round trip (left to itself
      // the compiler recycles two record registers and waits between pairs)
#pragma unroll
      for (int q = 0; q < K; ++q)
#pragma unroll
        for (int f = 0; f < NS; ++f) recs[q][f] = t.u96(lay.pbase, 16 * (oc[q][f] * nsw + k[q]));
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
      const uint64_t below = (1ull << bit[q]) - 1;
#pragma unroll
      for (int f = 0; f < NS; ++f) {
        if (lay.part_dense) {
          const uint32_t cell = oc[q][f] * nrw + w[q];
          // A slot that cannot be partial at the word reads POOL[0] (all-ones)
          // without a PART read.  PCN_WFIELDS 2: the load stays unconditional
          // (a conditional load's phi costs an immediate vmcnt(0) wait), every
          // such lane reading cell 0, one line for all of them; 1: a branch.
          const bool part = (wf[q] >> f) & 1;
          uint32_t qi = 0;   // POOL index (0: all-ones, a FULL field)
          // (dense PART is never staged in LDS: past the limit, read from L2)
          if (PCN_WFIELDS >= 2) {
            const uint32_t c = part ? cell : 0u;
            const uint32_t x = lay.part_wide ? t.g32(lay.part, 4 * c) : t.g16(lay.part, 2 * c);
            qi = part ? x : 0u;
          } else if (part) {
            qi = lay.part_wide ? t.g32(lay.part, 4 * cell) : t.g16(lay.part, 2 * cell);
          }
          at[q][f] = lay.pool + 8 * qi;
          continue;
        }
        const u32x3 r = recs[q][f];
        const uint64_t pm = static_cast<uint64_t>(r.y) << 32 | r.x;
        const uint32_t j = r.z + static_cast<uint32_t>(__builtin_popcountll(pm & below));
        const uint32_t part_mask = 0u - static_cast<uint32_t>((pm >> bit[q]) & 1);   // ~0: partial
        if (lay.part_direct) {
          at[q][f] = lay.pool + (part_mask & (lay.part + 8 * j - lay.pool));
        } else {
          const bool wide = lay.part_wide;
          const uint32_t ia = lay.zero + (part_mask & (lay.part + (wide ? 4 * j : 2 * j) - lay.zero));
          at[q][f] = lay.pool + 8 * (wide ? t.u32(lay.part, ia - lay.part) : t.u16(lay.part, ia - lay.part));
        }
      }
    }
    uint64_t acc[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
      acc[q] = ~0ull;
#pragma unroll
      for (int f = 0; f < NS; ++f) acc[q] &= t.u64(lay.pool, at[q][f] - lay.pool);   // (PART and POOL are on the same side of the limit)
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
      if (acc[q] && (q == 0 || two)) {   // an all-FULL word has acc == ~0: its lowest valid bit is bit 0
        const uint32_t e = t.u16(lay.perm, 2 * (w[q] * 63 + static_cast<uint32_t>(__builtin_ctzll(acc[q]))));
        atomicMin(&ws->best[owner[q]], e);
      }
    }
  };
  // worker side: the first `cnt` queued items
  auto drain = [&](uint32_t cnt) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (WMAX > 64 && cnt > 64) {     // wave-uniform: two items per lane
      const bool two = lane + 64 < cnt;
      const uint32_t idx[2] = {lane, two ? lane + 64 : 0u};
      work(IntK<2>{}, idx, two);
    } else if (lane < cnt) {
      const uint32_t idx[1] = {lane};
      work(IntK<1>{}, idx, false);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  u32x4 mine;   // this lane's classes ride along with each of its candidates
  {
    uint32_t pk[3] = {0u, 0u, 0u};
#pragma unroll
    for (int f = 0; f < NS; ++f) pk[f / 2] |= cls[f] << (16 * (f & 1));
    mine.y = pk[0];
    mine.z = pk[1];
    mine.w = pk[2];
  }
  if (MERGE && PCN_ABLATE != 3 && nsw >= 2 && nsw <= 4) {
    constexpr uint32_t kMaxB = 4;
    uint64_t mk[kMaxB] = {0, 0, 0, 0};
    if (active) {
      uint64_t sm[kMaxB][NS];
#pragma unroll
      for (uint32_t k = 0; k < kMaxB; ++k)
        if (k < nsw)
#pragma unroll
          for (int f = 0; f < NS; ++f) sm[k][f] = t.u64(lay.sf, 8 * (cls[f] * nsw + k));
#pragma unroll
      for (uint32_t k = 0; k < kMaxB; ++k) {
        if (k >= nsw) continue;
        const uint32_t live = nrw - k * 64;
        uint64_t m = live >= 64 ? ~0ull : ((1ull << live) - 1);
#pragma unroll
        for (int f = 0; f < NS; ++f) m &= sm[k][f];
        mk[k] = m;
      }
    }
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMaxB; ++k) c += static_cast<uint32_t>(__builtin_popcountll(mk[k]));
    uint32_t pos = 0, total = 0;
    for (uint32_t b = 0; b < 9; ++b) {   // c <= 256
      const uint64_t bm = __ballot((c >> b) & 1);
      pos += static_cast<uint32_t>(__builtin_popcountll(bm & ((1ull << lane) - 1))) << b;
      total += static_cast<uint32_t>(__builtin_popcountll(bm)) << b;
      if (__ballot(c >> (b + 1)) == 0) break;
    }
    wide += total > 64 ? 1u : 0u;
    if (total == 0) return kNoRule;
    ws->best[lane] = kNoRule;
    uint32_t p = pos, end = total;
    for (;;) {
#pragma unroll
      for (uint32_t k = 0; k < kMaxB; ++k) {
        if (k >= nsw) continue;
        while (mk[k] && p < W) {
          mine.x = (lane << 16) | (k * 64 + static_cast<uint32_t>(__builtin_ctzll(mk[k])));
          items[p] = mine;
          mk[k] &= mk[k] - 1;
          ++p;
        }
      }
      drain(end < W ? end : W);
      if (end <= W) break;
      p -= W;   // (wraps for lanes with nothing left: they write no more)
      end -= W;
    }
    return ws->best[lane];
  }
  uint32_t qn = 0;      // items queued, not yet dealt (wave-uniform, < W)
  uint32_t queued = 0;  // candidates over all blocks (wave-uniform)
  for (uint32_t k = 0; k < nsw; ++k) {
    const uint32_t live = nrw - k * 64;
    uint64_t m = 0;
    if (active) {
      m = live >= 64 ? ~0ull : ((1ull << live) - 1);
      uint64_t sm[NS];
#pragma unroll
      for (int f = 0; f < NS; ++f) sm[f] = t.u64(lay.sf, 8 * (cls[f] * nsw + k));
#pragma unroll
      for (int f = 0; f < NS; ++f) m &= sm[f];
    }
    if (PCN_ABLATE == 3) { mseen |= m; continue; }
    // exclusive prefix of the per-lane candidate counts (bit-sliced ballots,
    // as many slices as the largest count needs)
    const uint32_t c = static_cast<uint32_t>(__builtin_popcountll(m));
    uint32_t pos = 0, total = 0;
    for (uint32_t b = 0; b < 7; ++b) {
      const uint64_t bm = __ballot((c >> b) & 1);
      pos += static_cast<uint32_t>(__builtin_popcountll(bm & ((1ull << lane) - 1))) << b;
      total += static_cast<uint32_t>(__builtin_popcountll(bm)) << b;
      if (__ballot(c >> (b + 1)) == 0) break;
    }
    const bool last_block = k + 1 == nsw;
    queued += total;
    if (total == 0 && (!last_block || qn == 0)) continue;
    if (!staged) {
      staged = true;
      ws->best[lane] = kNoRule;
#if !PCN_ITEM_CLS
      ws->cls[lane] = mine;
#endif
    }
    // this block's items go to queue positions [qn, qn + total): each owner
    // writes those that fall in the current window of W, which is dealt
    // when it is full or after the last block (one call site: a chain of one
    // block runs the code of a plain per-block deal)
    uint32_t p = qn + pos, end = qn + total;
    for (;;) {
      while (m && p < W) {
        mine.x = (lane << 16) | (k * 64 + static_cast<uint32_t>(__builtin_ctzll(m)));
        if (PCN_ITEM_CLS) items[p] = mine;
        else reinterpret_cast<uint32_t *>(items)[p] = mine.x;
        m &= m - 1;
        ++p;
      }
      if (end < W && !last_block) { qn = end; break; }
      drain(end < W ? end : W);
      if (end <= W) { qn = 0; break; }
      p -= W;
      end -= W;
    }
  }
  if (PCN_ABLATE == 3) return mseen ? 0u : kNoRule;
  wide += queued > 64 ? 1u : 0u;   // a 64-candidate window needed a second pass
  return staged ? ws->best[lane] : kNoRule;
}

// ---- rule-chain stage, part 3 (per lane) ----
__device__ __forceinline__ uint32_t chain_finish(const DevChain &ch, uint32_t best, int32_t &rid) {
  if (best == kNoRule) { rid = PCN_IPT_RID_DEFAULT; return static_cast<uint32_t>(ch.default_action); }
  const uint32_t rule = best >> 1;
  if (rule >= ch.max_action) { rid = PCN_IPT_RID_NOCHAIN; return PCN_IPT_DROP; }
  rid = static_cast<int32_t>(rule);
  return (best & 1) ? PCN_IPT_ACCEPT : PCN_IPT_DROP;
}

// One chain through the three parts; `mine` = lanes whose packet runs it.
// Called with the wave converged.
template <bool LDS, int NS, uint32_t W = 64, bool MERGE = false>
__device__ __forceinline__ void run_chain(const DevChain &ch, bool mine, const Parsed &p, uint32_t port,
                                          WaveScratch *ws, uint32_t wave_bytes, uint32_t &verdict, int32_t &rid,
                                          uint32_t &wide) {
  uint32_t cls[NS];
  bool need = false;
  if (mine) need = chain_classes<LDS, NS>(ch, p, port, cls, verdict, rid);
  // the wave gets issue priority while it deals candidates through LDS
  if (PCN_CAND_PRIO >= 0) __builtin_amdgcn_s_setprio(PCN_CAND_PRIO >= 0 ? PCN_CAND_PRIO : 0);
  const uint32_t best = chain_candidates<LDS, NS, W, MERGE>(ch, need, cls, ws, wave_bytes, wide);
  if (PCN_CAND_PRIO >= 0) __builtin_amdgcn_s_setprio(0);
  if (need) verdict = chain_finish(ch, best, rid);
}

// The chain program's constants.  A JIT build (jit.cpp, the analogue of the
// reference's per-chain datapath compile with macro-substituted table sizes,
// modules/Program.cpp:23-119) bakes the running chain's layout, word counts
// and field set into the code as immediates; only its pointers stay kernargs.
#ifdef PCN_JIT
constexpr DevChain kJitChain = PCN_JIT_CHAIN;
constexpr int kJitInputs = PCN_JIT_INPUTS;   // bit 0: in_port array, bits 1-2: ct_status (array / stage-A label),
                                             // 3 stale ports, 4 Horus, 5 offsets array, 6 lens array,
                                             // 7 stage A writes the walk records (LaunchArgs::ct_brec)
#else
constexpr DevChain kJitChain{};
constexpr int kJitInputs = 7;
#endif
template <bool JIT, int CH>
__device__ __forceinline__ DevChain chain_desc(const LaunchArgs &a) {
  if constexpr (JIT) {
    DevChain c = kJitChain;
    c.image = a.ch[CH].image;
    c.ctr = a.ch[CH].ctr;
    return c;
  } else {
    return a.ch[CH < 3 ? CH : 0];
  }
}

// SPLIT (chain programs of split launches, pcn_ipt.cpp): 0 = the one fused
// kernel; 1 = the gather kernel: every step up to the rule stage (parse, TC
// untag, chain select, ICMP checks, labels), with no chain image in LDS and
// two workgroups per CU, writing the fields the rule stage reads for each
// frame that reaches it (LaunchArgs::split_rec) and finishing the others;
// 2 = the rule kernel: those fields read back coalesced, the image in LDS, the
// rule stage, verdicts and counters of those frames.  The gather's HBM latency
// is then hidden by occupancy, and the rule stage's LDS / L2 chains by a
// kernel that waits on nothing else.
template <bool FIXED, bool LDS, int CH, int NS, bool JIT, int SPLIT = 0>
__device__ __forceinline__ void classify_body(const LaunchArgs &a) {
  static_assert(SPLIT == 0 || !FIXED, "split launches are offsets / lens (IMIX) batches");
  const DevChain run_ch = chain_desc<JIT, CH>(a);   // the chain that runs rules (CH < 3)
  const unsigned long long clk0 = a.dbg_clk ? __builtin_amdgcn_s_memrealtime() : 0ull;
  unsigned long long clk1 = 0, clk2 = 0;
  constexpr uint32_t kDealW = PCN_DEAL2 >= 2 || (PCN_DEAL2 && FIXED) ? 128 : 64;   // candidate deal window (max)
  // per-workgroup histogram: u32 {pkts, bytes} per bin (the host bounds the
  // frames per workgroup so neither can wrap; the flush widens to u64)
  uint32_t *bins = reinterpret_cast<uint32_t *>(pcn_smem + a.bins_offset);
  WaveScratch *ws = reinterpret_cast<WaveScratch *>(pcn_smem + a.lds_scratch + (threadIdx.x >> 6) * a.wave_bytes);
  // stage every chain's table image in LDS and zero the counter histogram.
  // (The first frames' headers are already in flight: the prefetch below is
  // issued before this when PCN_STAGE_FAST.)  Every load of a pass is issued
  // before its stores, so a 128 KB image costs one L2 round trip, not eight.
  auto stage_images = [&]() {
    if (!LDS) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const DevChain &ch = c == CH ? run_ch : a.ch[c];
      if (!ch.lds_limit) continue;
      const u32x4 *src = reinterpret_cast<const u32x4 *>(ch.image);
      u32x4 *dst = reinterpret_cast<u32x4 *>(pcn_smem + ch.lds_image);
      const uint32_t n16 = ch.lds_limit / 16;
      if (PCN_STAGE_FAST) {
        constexpr uint32_t U = 10;   // 160 KB / (1024 threads x 16 B)
        for (uint32_t k0 = threadIdx.x; k0 < n16; k0 += U * kBlock) {
          u32x4 r[U];
#pragma unroll
          for (uint32_t u = 0; u < U; ++u)
            if (k0 + u * kBlock < n16) r[u] = src[k0 + u * kBlock];
#pragma unroll
          for (uint32_t u = 0; u < U; ++u)
            if (k0 + u * kBlock < n16) dst[k0 + u * kBlock] = r[u];
        }
      } else {
        for (uint32_t k = threadIdx.x; k < n16; k += blockDim.x) dst[k] = src[k];
      }
    }
  };
  if (!PCN_STAGE_FAST) stage_images();
  uint32_t *const byte_bins = bins + a.nbins;
  const uint32_t const_port = a.const_in_port;
#ifndef PCN_DBG_HZ
#define PCN_DBG_HZ 0     // measurement only: 1 = no stale-port tracking, 2 = no Horus lookups
#endif
  // The Parser's stale ports (Q4) for Horus keys, computed here (has_stale):
  // each workgroup takes a contiguous chunk of the batch, in the order the
  // workgroups start (a counter), and every 64-frame group publishes the
  // ports of its last TCP/UDP frame; a frame that needs the ports of an
  // earlier group looks back through the published groups.  A workgroup only
  // ever waits on groups of workgroups that started before it, so the waits
  // always resolve.
  constexpr bool kStale = (!JIT || (kJitInputs & 8)) && PCN_DBG_HZ != 1;
  constexpr bool kHorus = (!JIT || (kJitInputs & 16)) && PCN_DBG_HZ != 2;   // a Horus program is in place
  constexpr bool kCtRec = (!JIT || (kJitInputs & 128)) && SPLIT == 0;   // stage A writes the walk records
  const bool chunked = kStale && a.has_stale;
  uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t first = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint64_t n_round = (a.n + step - 1) / step * step;   // uniform trip count per wave
  if (chunked) {
    uint32_t *slot = reinterpret_cast<uint32_t *>(pcn_smem + a.bins_offset);   // zeroed after the prologue
    if (threadIdx.x == 0) *slot = atomicAdd(a.chunk_ctr, 1u);
    __syncthreads();
    const uint64_t b = *slot;
    __syncthreads();
    const uint64_t lo = b * a.chunk_frames, hi = lo + a.chunk_frames;
    const uint64_t nr = (a.n + blockDim.x - 1) / blockDim.x * blockDim.x;
    first = lo + threadIdx.x;
    step = blockDim.x;
    n_round = hi < nr ? hi : nr;
  }
  // software pipeline: the next frame's header is in flight while this one is classified
  // The prefetch is unconditional (the index is clamped to the last frame):
  // a conditional load merges into a phi the compiler can only resolve with
  // an immediate s_waitcnt vmcnt(0), which serialises load and compute.
  const uint64_t last = a.n - 1;
  // in_port / ct_status ride along with the header: when the batch has none
  // the host points them at a zero cell with a zero index mask, so the loads
  // stay unconditional too.  PF frames per lane are in flight.
  // Fixed-stride frames are fetched coalesced: a wave's 64 frames are 192
  // 16-byte chunks (bytes 0..47 of each frame), chunk t = 64q + lane is loaded
  // by instruction q of that lane, and the chunks are transposed through a
  // 3 KB per-wave LDS buffer into one header per lane.  Each instruction then
  // touches ~11 cache lines instead of 32.
  struct Stage {
    Hdr h;          // generic path (PCN_GEN_QUAD 0)
    u32x4 c[3];     // fixed path: this lane's three chunks
    u32x4 g[5];     // generic path, quad gather: the chunks this lane fetched (see prefetch)
    uint32_t sh;    // generic path: the frame start's offset in its 16-byte chunk
    bool quad;      // generic path: g[0..3] hold other frames' chunks (transpose in process)
    uint32_t offn;  // generic path, PCN_OFF_AHEAD: the offset of the frame this stage fetches next
    uint32_t L, port, ct;
  };
  const uint32_t lane = threadIdx.x & 63;
  // fixed path: frame within the wave's group, byte offset of the chunk, and
  // the chunk's byte offset from the group's first frame
  uint32_t cf[3], co[3], loff[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint32_t t = 64 * q + lane;
    cf[q] = t / 3;
    co[q] = 16 * (t - 3 * cf[q]);
    loff[q] = cf[q] * a.stride + co[q];
  }
  // per-frame side inputs a chain program knows it does not have are never loaded
  constexpr bool kLoadPort = !JIT || (kJitInputs & 1);
  constexpr bool kLoadCt = !JIT || (kJitInputs & 6);
  // offsets / lens arrays: constants of a chain program, runtime otherwise
  const bool has_off = JIT ? (kJitInputs & 32) != 0 : a.offsets != nullptr;
  const bool has_lens = JIT ? (kJitInputs & 64) != 0 : a.lens != nullptr;
  u32x4 *hbuf = reinterpret_cast<u32x4 *>(pcn_smem + a.lds_scratch + (threadIdx.x >> 6) * a.wave_bytes);
  // (a split launch's rule kernel: its 16-byte records, PCN_SPLIT_R_PF ahead)
  constexpr int PF = SPLIT == 2 ? PCN_SPLIT_R_PF : FIXED ? PCN_PREFETCH_FIXED : PCN_PREFETCH_GENERIC;
  Stage st[PF];
  auto prefetch = [&](Stage &x, uint64_t j) {   // j: this lane's frame index
    if constexpr (SPLIT == 2) {                  // the gather kernel's fields for frame j, coalesced
      const uint64_t jf = j < a.n ? j : last;
      x.g[0] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.split_rec) + jf);
      x.L = has_lens ? a.lens[jf] : a.fixed_len;
    } else if (FIXED && PCN_HDR_LDS) {
      uint64_t group = j - lane;                 // wave-uniform
      group = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(group >> 32))) << 32) |
              __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(group));
      if (PCN_PF_FAST && group + 64 <= a.n) {
        // the whole group is in the batch: scalar base + loop-invariant lane offsets
        const uint8_t *gb = a.frames + group * a.stride;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const u32x4 *src = reinterpret_cast<const u32x4 *>(gb + loff[q]);
          if (PCN_HDR_ASM) hdr_load_asm(x.c[q], src);
          else x.c[q] = hdr_load(src);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          uint64_t f = group + cf[q];
          f = f < a.n ? f : last;
          const u32x4 *src = reinterpret_cast<const u32x4 *>(a.frames + f * a.stride + co[q]);
          if (PCN_HDR_ASM) hdr_load_asm(x.c[q], src);
          else x.c[q] = hdr_load(src);
        }
      }
    } else if (FIXED) {
      const uint64_t f = j < a.n ? j : last;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        x.c[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.frames + f * a.stride) + q);
    } else if (PCN_GEN_QUAD) {
      const uint64_t jf = j < a.n ? j : last;
      uint64_t off;
      if (PCN_OFF_AHEAD && has_off) {
        off = x.offn;                                // loaded one prefetch ago
        const uint64_t jn = j + PF * step;           // the frame this stage fetches next
        x.offn = a.offsets[jn < a.n ? jn : last];
      } else {
        off = has_off ? uint64_t(a.offsets[jf]) : jf * a.stride;
      }
      const uint64_t at = reinterpret_cast<uintptr_t>(a.frames) + off;
      const uint64_t end = reinterpret_cast<uintptr_t>(a.frames) + a.frames_bytes;
      const uint64_t abase = at & ~uint64_t(15);
      x.L = has_lens ? a.lens[jf] : a.fixed_len;
      x.sh = static_cast<uint32_t>(at & 15);
      uint64_t group = j - lane;                 // wave-uniform
      group = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(group >> 32))) << 32) |
              __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(group));
      // the whole group in the batch, and every frame's 80 aligned bytes inside the buffer
      x.quad = group + 64 <= a.n && __ballot(abase + 80 > end) == 0;
      if (x.quad) {
        // instruction q: lane l fetches chunk (l & 3) of frame 16 q + (l >> 2)
        const uint32_t lo = static_cast<uint32_t>(abase), hi = static_cast<uint32_t>(abase >> 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int src = 16 * q + static_cast<int>(lane >> 2);
          const uint64_t fb = (static_cast<uint64_t>(__shfl(hi, src)) << 32) | __shfl(lo, src);
          x.g[q] = hdr_load(reinterpret_cast<const u32x4 *>(fb) + (lane & 3));
        }
        // chunk 4 (bytes 64..79) only matters when the 52-byte window crosses
        // into it; otherwise the load re-reads chunk 3's line (no new traffic)
        x.g[4] = hdr_load(reinterpret_cast<const u32x4 *>(abase) + (x.sh > 12 ? 4 : 3));
      } else {
        // one lane per frame: its own 80 bytes, each dword only if inside the buffer
        uint32_t d[20];
#pragma unroll
        for (int k = 0; k < 20; ++k) {
          const uint64_t p = abase + 4u * k;
          d[k] = p + 4 <= end ? *reinterpret_cast<const uint32_t *>(p) : 0u;
        }
#pragma unroll
        for (int q = 0; q < 5; ++q) x.g[q] = u32x4{d[4 * q], d[4 * q + 1], d[4 * q + 2], d[4 * q + 3]};
      }
    } else {
      x.L = a.fixed_len;
      load_header<FIXED>(a, j < a.n ? j : last, x.h, x.L);
    }
    const uint64_t jc = j < a.n ? j : last;
    x.port = kLoadPort ? a.in_port[jc & a.in_port_mask] : 0u;
    x.ct = kLoadCt && SPLIT != 2 ? a.ct_status[jc & a.ct_mask] : 0u;   // (the rule kernel: in the record)
  };
  if (SPLIT != 2 && !FIXED && PCN_GEN_QUAD && PCN_OFF_AHEAD && has_off) {
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      const uint64_t j = first + d * step;
      st[d].offn = a.offsets[j < a.n ? j : last];
    }
  }
#pragma unroll
  for (int d = 0; d < PF; ++d) prefetch(st[d], first + d * step);
  if (PCN_STAGE_FAST) stage_images();
  // pkts[nbins], then (variable lengths only) bytes[nbins]; with a fixed
  // length every bin's bytes are pkts * len at the flush
  for (uint32_t b = threadIdx.x; b < (FIXED ? 1u : 2u) * a.nbins; b += blockDim.x) bins[b] = 0;
  for (uint32_t k = threadIdx.x; k < a.nlocal; k += blockDim.x)
    reinterpret_cast<uint32_t *>(pcn_smem + a.lds_localip)[k] = a.localip[k];
  uint32_t *const lds_stats = reinterpret_cast<uint32_t *>(pcn_smem + a.lds_stats);
  if (threadIdx.x == 0) *lds_stats = 0;
  uint32_t wide = 0;   // this wave's rule stages that dealt more than 64 candidates (wave-uniform)
  __syncthreads();
  if (a.dbg_clk) clk1 = __builtin_amdgcn_s_memrealtime();
  // Stage d always holds the frames i with (i - first) / step == d (mod
  // PF): the loop is unrolled PF times so no stage is
  // ever copied (a register move of an in-flight load waits for it).
  auto process = [&](const uint64_t i, Stage &cur) {
    bool valid = i < a.n;
    // Pin every prefetched dword (used or not) until here, so no register the
    // load writes is recycled mid-iteration (a WAW hazard costs a vmcnt wait).
    Hdr h;
    u32x4 srec = {};   // SPLIT 2: this frame's record, taken before the stage is refilled
    if constexpr (SPLIT == 2) {
      asm volatile("" : "+v"(cur.g[0]));
      srec = cur.g[0];
    } else if (FIXED && !PCN_HDR_LDS) {
#pragma unroll
      for (int q = 0; q < 3; ++q) asm volatile("" : "+v"(cur.c[q]));
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        h.w[4 * q] = cur.c[q].x; h.w[4 * q + 1] = cur.c[q].y; h.w[4 * q + 2] = cur.c[q].z; h.w[4 * q + 3] = cur.c[q].w;
      }
    } else if (FIXED) {
      if (PCN_HDR_ASM) {
        static_assert(PF == 1 || PF == 2 || PF == 3, "counted header waits for PF 1..3");
        if constexpr (PF == 1) asm volatile("s_waitcnt vmcnt(0)" : "+v"(cur.c[0]), "+v"(cur.c[1]), "+v"(cur.c[2]));
        else if constexpr (PF == 2) asm volatile("s_waitcnt vmcnt(3)" : "+v"(cur.c[0]), "+v"(cur.c[1]), "+v"(cur.c[2]));
        else asm volatile("s_waitcnt vmcnt(6)" : "+v"(cur.c[0]), "+v"(cur.c[1]), "+v"(cur.c[2]));
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) asm volatile("" : "+v"(cur.c[q]));
      }
      asm volatile("" ::: "memory");   // the region held the last iteration's WaveScratch
#pragma unroll
      for (int q = 0; q < 3; ++q) hbuf[64 * q + lane] = cur.c[q];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const u32x4 c0 = hbuf[3 * lane], c1 = hbuf[3 * lane + 1], c2 = hbuf[3 * lane + 2];
      h.w[0] = c0.x; h.w[1] = c0.y; h.w[2] = c0.z; h.w[3] = c0.w;
      h.w[4] = c1.x; h.w[5] = c1.y; h.w[6] = c1.z; h.w[7] = c1.w;
      h.w[8] = c2.x; h.w[9] = c2.y; h.w[10] = c2.z; h.w[11] = c2.w;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else if (PCN_GEN_QUAD) {
#pragma unroll
      for (int q = 0; q < 5; ++q) asm volatile("" : "+v"(cur.g[q]));
      uint32_t d[17];
      if (cur.quad) {                              // wave-uniform
        // four rounds of 16 frames: every lane writes the chunk it fetched into
        // its frame's row, then the 16 lanes whose frames these are read their rows
        u32x4 *rows = hbuf;                        // 16 rows x 5 chunks (80 B: 4 used + padding)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          asm volatile("" ::: "memory");           // the region held the last iteration's WaveScratch
          rows[(lane >> 2) * 5 + (lane & 3)] = cur.g[q];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          if ((lane >> 4) == static_cast<uint32_t>(q)) {
            const u32x4 *row = rows + (lane & 15) * 5;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const u32x4 v = row[c];
              d[4 * c] = v.x; d[4 * c + 1] = v.y; d[4 * c + 2] = v.z; d[4 * c + 3] = v.w;
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          d[4 * c] = cur.g[c].x; d[4 * c + 1] = cur.g[c].y; d[4 * c + 2] = cur.g[c].z; d[4 * c + 3] = cur.g[c].w;
        }
      }
      d[16] = cur.g[4].x;
      // the window starts cur.sh bytes into the chunk: dword shift, then byte shift
      const uint32_t dsh = cur.sh >> 2, bsh = cur.sh & 3;
      // (the asm keeps both operands in registers: folded into d[k + dsh],
      // the window became a dynamically indexed array in scratch)
      auto sel = [](bool c, uint32_t x, uint32_t y) {
        asm volatile("" : "+v"(x), "+v"(y));
        return c ? y : x;
      };
      uint32_t f1[16], f2[14];
#pragma unroll
      for (int k = 0; k < 16; ++k) f1[k] = sel(dsh & 1, d[k], d[k + 1]);
#pragma unroll
      for (int k = 0; k < 14; ++k) f2[k] = sel(dsh & 2, f1[k], f1[k + 2]);
#pragma unroll
      for (int k = 0; k < 13; ++k) h.w[k] = __builtin_amdgcn_alignbyte(f2[k + 1], f2[k], bsh);
    } else {
#pragma unroll
      for (int k = 0; k < 13; ++k) asm volatile("" : "+v"(cur.h.w[k]));
      h = cur.h;
    }
    asm volatile("" : "+v"(cur.port), "+v"(cur.ct));
    uint32_t L = FIXED ? a.fixed_len : cur.L;
    const uint32_t cur_port = cur.port, cur_ct = cur.ct;
    constexpr bool kLate = (SPLIT == 0 || (SPLIT == 2 && PCN_SPLIT_R_LATE)) && PCN_PF_LATE && !FIXED && JIT &&
                           kJitChain.lay.part_dense;
    if (!kLate) prefetch(cur, i + PF * step);
    uint32_t verdict = PCN_IPT_DROP;
    int32_t rid = PCN_IPT_RID_NOCHAIN;
    int32_t cchain = -1;    // chain whose counters this packet bumps
    int32_t chain = -1;     // chain whose rules must run (-1: decided already)
    Parsed p{};
    uint32_t port = 0;
    uint32_t untag = 0;     // SPLIT 1: kSplitUntag once the outer VLAN tag is stripped
    uint32_t ps = 0;        // the Parser's outcome: 0 RX_DROP, 1 not IPv4, 2 parsed (walk records)
    uint32_t own_pd = 0;    // the Parser's srcPort / dstPort as stored (wire bytes 34-37)
    uint32_t stale = 0;     // ... as a packet it writes none for sees them (Q4; chunked launches)
    if constexpr (SPLIT == 2) {
      // the gather kernel's fields (SPLIT 1 below): only frames that reach the
      // rule stage are this kernel's
      const u32x4 r = srec;
      const uint32_t meta = r.w >> 24;
      valid = valid && (meta & kSplitNeed);
      p.saddr = r.x;
      p.daddr = r.y;
      p.sport = r.z & 0xffffu;
      p.dport = r.z >> 16;
      p.proto = r.w & 0xffu;
      p.flags = (r.w >> 8) & 0xffu;
      p.ct = (r.w >> 16) & 0xffu;
      port = a.has_in_port ? cur_port : const_port;
      if (meta & kSplitUntag) L -= 4;
      chain = valid ? static_cast<int32_t>(meta & 3u) : -1;
    } else {
    // Wave fast path: when every lane holds a plain IPv4 TCP/UDP frame long
    // enough for its L4 header (fixed stride: XDP, one length) and the launch
    // has a chain every such frame selects, the Parser / ChainSelector /
    // ConntrackLabel steps below reduce to straight-line field extraction.
    bool fast = false;
    bool gen = false;       // general path: the Parser ran (done: decided there)
    bool done = true;
    if (PCN_FASTPATH && FIXED && a.fast_chain >= 0) {
      const uint32_t pr = h.w[5] >> 24;
      const bool plain = valid && (h.w[3] & 0xffff) == 0x0008 &&
                         ((pr == 6 && L >= 54) || (pr == 17 && L >= 42));
      fast = __ballot(!plain) == 0;
    }
    if (fast) {
      ps = 2;
      port = a.has_in_port ? cur_port : const_port;
      p.proto = h.w[5] >> 24;
      p.saddr = (h.w[6] >> 16) | (h.w[7] << 16);
      p.daddr = (h.w[7] >> 16) | (h.w[8] << 16);
      p.flags = p.proto == 6 ? h.w[11] >> 24 : 0u;
      p.sport = bswap16u(h.w[8] >> 16);
      p.dport = bswap16u(h.w[9] & 0xffff);
      chain = a.fast_chain;
      // labels: given, or the empty-table ones (ConntrackLabel_dp.c:372-383)
      p.ct = a.has_ct ? cur_ct : empty_table_label(p, 0xffffffffu);
      if (a.fw == PCN_FW_LAUNCH_CT_OFF && !a.has_ct) p.ct = 0;
      if (a.fw == PCN_FW_LAUNCH_CT_AUTO && p.ct == 1) {   // Firewall_ConntrackLabel_dp.c:474-478
        verdict = PCN_IPT_ACCEPT; rid = PCN_IPT_RID_ACCEPT_ESTABLISHED; chain = -1;
      }
    } else if (valid) {
      port = a.has_in_port ? cur_port : const_port;
      // ---- TC hook: the outer VLAN tag is gone before the program runs ----
      bool untag_drop = false;
      if (!FIXED && a.hook == PCN_IPT_HOOK_TC && L >= 14 &&
          ((h.w[3] & 0xffff) == 0x0081 || (h.w[3] & 0xffff) == 0xA888)) {   // 0x8100 / 0x88A8
        if (L < 18) {
          untag_drop = true;
        } else {
#pragma unroll
          for (int k = 3; k < 12; ++k) h.w[k] = h.w[k + 1];
          L -= 4;
          untag = kSplitUntag;
        }
      }
      // ---- Parser_dp.c:94-153 ----
      gen = true;
      if (L < 14 || untag_drop) verdict = PCN_IPT_DROP;
      else if ((h.w[3] & 0xffff) != 0x0008) { verdict = PCN_IPT_ACCEPT; ps = 1; }   // ethertype != 0x0800
      else if (L < 34) verdict = PCN_IPT_DROP;
      else {
        p.proto = h.w[5] >> 24;
        p.saddr = (h.w[6] >> 16) | (h.w[7] << 16);
        p.daddr = (h.w[7] >> 16) | (h.w[8] << 16);
        done = false;
        ps = 2;
        if (p.proto == 6) {
          if (L < 54) { verdict = PCN_IPT_DROP; done = true; ps = 0; }
          p.flags = h.w[11] >> 24;
        } else if (p.proto == 17) {
          if (L < 42) { verdict = PCN_IPT_DROP; done = true; ps = 0; }
        }
        p.sport = bswap16u(h.w[8] >> 16);
        p.dport = bswap16u(h.w[9] & 0xffff);
      }
    }
    // ---- the Parser's srcPort/dstPort as stored (wire bytes 34-37), stale
    // for a packet it writes none for (Q4): Horus keys read them ----
    own_pd = (h.w[8] >> 16) | (h.w[9] << 16);
    if (chunked) {
      const bool wrote = fast ? valid : gen && !done && (p.proto == 6 || p.proto == 17);
      const bool need = gen && !done && p.proto != 6 && p.proto != 17;
      const uint64_t wm = __ballot(wrote);
      const uint64_t g = (a.gbase + i) >> 6;              // the wave's group (64-aligned frames)
      const uint32_t last_pd = __shfl(own_pd, wm ? 63 - __builtin_clzll(wm) : 0);
      // a wave wholly past the batch end publishes nothing: the host sizes
      // stale_desc for the batch's groups (n / 64 + 1 words), not for the grid
      if (lane == 0 && valid)
        __hip_atomic_store(&a.stale_desc[g], stale_word(a.stale_epoch, wm ? kStaleLocal : kStaleNone, last_pd),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t before = wm & ((1ull << lane) - 1);
      stale = __shfl(own_pd, before ? 63 - __builtin_clzll(before) : 0);
      if (__ballot(need && !before)) {
        const uint32_t cin = stale_lookback(a, g);
        if (!before) stale = cin;
        if (!wm && lane == 0)
          __hip_atomic_store(&a.stale_desc[g], stale_word(a.stale_epoch, kStaleInclusive, cin),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (gen) {
      if (!done && a.fw) {
        // ---- pcn-firewall: Parser -> [ConntrackLabel] -> ChainForwarder ----
        // (Firewall_Parser_dp.c:94-165, Firewall_ChainForwarder_dp.c:20-42):
        // the chain is the program's direction, INGRESS / EGRESS in the
        // FORWARD / OUTPUT slots.  The ConntrackLabel stage (the same ICMP
        // length checks and labels as pcn-iptables) runs only when conntrack
        // is on (modules/Parser.cpp:41-45); with it off the label is never
        // written (per-CPU zero: NEW).
        chain = a.direction == PCN_IPT_INGRESS ? PCN_IPT_FORWARD : PCN_IPT_OUTPUT;
        p.ct = a.has_ct ? cur_ct : 0u;
        // ---- Horus (Firewall_Parser_dp.c:154-157 -> Firewall_Horus_dp.c:97-175) ----
        bool pass = false;
        if (kHorus && a.horus_fields) {
          const uint32_t pd = (p.proto == 6 || p.proto == 17) ? own_pd : stale;
          uint32_t meta;
          if (horus_lookup(a, p.saddr, p.daddr, p.proto, pd, meta)) {   // counted with the rule bins
            rid = PCN_IPT_RID_HORUS0 - static_cast<int32_t>(meta >> 16);
            done = true;
            if (!((meta >> 8) & 1)) verdict = PCN_IPT_DROP;
            else if (a.horus_flags & kHzAcceptFinal) verdict = PCN_IPT_ACCEPT;
            else if (a.horus_flags & kHzAcceptDrops) verdict = PCN_IPT_DROP;
            else { pass = true; done = false; }           // PASS_LABELING -> ConntrackLabel
          } else if (a.horus_flags & kHzMissDrops) {
            verdict = PCN_IPT_DROP; done = true;
          }
        }
        if (!done && a.fw != PCN_FW_LAUNCH_CT_OFF) {
          uint32_t icmp_type;
          if (icmp_drop(p, h, L, icmp_type)) { verdict = PCN_IPT_DROP; done = true; }
          else if (!a.has_ct) p.ct = empty_table_label(p, icmp_type);
          // PASS_LABELING -> ConntrackTableUpdate -> RX_OK in both modes
          // (Firewall_ConntrackLabel_dp.c:463-489)
          if (!done && pass) { verdict = PCN_IPT_ACCEPT; done = true; }
          // AUTOMATIC: ESTABLISHED -> ConntrackTableUpdate -> RX_OK before the
          // chain, uncounted (Firewall_ConntrackLabel_dp.c:474-478)
          if (!done && a.fw == PCN_FW_LAUNCH_CT_AUTO && p.ct == 1) {
            verdict = PCN_IPT_ACCEPT; rid = PCN_IPT_RID_ACCEPT_ESTABLISHED; done = true;
          }
        }
        if (!done && ((a.empty_mask >> chain) & 1)) {    // DefaultAction (Firewall_DefaultAction_dp.c:37-43)
          cchain = chain; rid = PCN_IPT_RID_DEFAULT;
          verdict = ((a.drop_mask >> chain) & 1) ? PCN_IPT_DROP : PCN_IPT_ACCEPT;
          done = true;
        }
        if (done) chain = -1;
      } else if (!done) {
        bool pass = false;
        // ---- Horus (Parser_dp.c:145-147 -> Horus_dp.c:97-167), ingress ----
        if (kHorus && a.horus_fields) {
          const uint32_t pd = (p.proto == 6 || p.proto == 17) ? own_pd : stale;
          uint32_t meta;
          if (horus_lookup(a, p.saddr, p.daddr, p.proto, pd, meta)) {   // counted with the rule bins
            rid = PCN_IPT_RID_HORUS0 - static_cast<int32_t>(meta >> 16);
            if ((meta >> 8) & 1) pass = true;                 // ACCEPT: PASS_LABELING
            else { verdict = PCN_IPT_DROP; done = true; }
          }
        }
        // ---- ChainSelector_dp.c:131-298 ----
        if (!done && !pass) {
          if (a.direction == PCN_IPT_INGRESS) {
            if (a.allow_logic) pass = true;
            else chain = (a.nlocal && localip_has(a, p.daddr)) ? PCN_IPT_INPUT : PCN_IPT_FORWARD;
          } else {
            if (a.nlocal && localip_has(a, p.saddr)) chain = PCN_IPT_OUTPUT;
            else { verdict = PCN_IPT_ACCEPT; done = true; }   // egress PASS
          }
          if (!done && chain >= 0 && ((a.empty_mask >> chain) & 1)) {
            cchain = chain; rid = PCN_IPT_RID_DEFAULT;       // default counters
            if ((a.drop_mask >> chain) & 1) { verdict = PCN_IPT_DROP; done = true; }
            pass = true;
            chain = -1;
          }
        }
        // ---- ConntrackLabel_dp.c:436-531 ICMP length checks ----
        uint32_t icmp_type = 0xffffffffu;
        if (!done && icmp_drop(p, h, L, icmp_type)) { verdict = PCN_IPT_DROP; done = true; }
        if (!done) {
          p.ct = a.has_ct ? cur_ct : empty_table_label(p, icmp_type);
          if (pass) { verdict = PCN_IPT_ACCEPT; done = true; }
        }
        if (done) chain = -1;
      }
    }
    }  // SPLIT != 2
    // ---- rule chains ----
    // CH < 3: only chain CH can reach the rule stage in this launch (the host
    // picks the variant), so its descriptor is a constant-index kernarg load
    // that stays in SGPRs.  CH == 3: ingress with both INPUT and FORWARD rules.
    if (PCN_ABLATE == 1) { verdict = chain >= 0 ? 1u : verdict; chain = -1; }
    bool wr = valid;        // this kernel writes the frame's verdict (and counts it)
    if constexpr (SPLIT == 1) {
      // the rule stage runs in the rule kernel: its fields, for every frame
      // (kSplitNeed marks those it runs), one coalesced 16-byte store
      if (valid) {
        const uint32_t meta = (chain >= 0 ? kSplitNeed | static_cast<uint32_t>(chain) : 0u) | untag;
        u32x4 r;
        r.x = p.saddr;
        r.y = p.daddr;
        r.z = p.sport | (p.dport << 16);
        r.w = (p.proto & 0xffu) | (p.flags & 0xffu) << 8 | (p.ct & 0xffu) << 16 | meta << 24;
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(a.split_rec) + i);
      }
      if (chain >= 0) {
        wr = false;
        chain = -1;
      }
    } else if (CH < 3) {
      run_chain<LDS, NS, kDealW, JIT && PCN_MERGE_BLOCKS>(run_ch, chain >= 0, p, port, ws, a.wave_bytes, verdict, rid,
                                                          wide);
      if (chain >= 0) cchain = chain;
    } else {
      if (__ballot(chain == PCN_IPT_FORWARD)) {
        run_chain<LDS, NS, kDealW>(a.ch[PCN_IPT_FORWARD], chain == PCN_IPT_FORWARD, p, port, ws, a.wave_bytes, verdict, rid,
                                   wide);
        if (chain == PCN_IPT_FORWARD) cchain = PCN_IPT_FORWARD;
      }
      if (__ballot(chain == PCN_IPT_INPUT)) {
        run_chain<LDS, NS, kDealW>(a.ch[PCN_IPT_INPUT], chain == PCN_IPT_INPUT, p, port, ws, a.wave_bytes, verdict, rid,
                                   wide);
        if (chain == PCN_IPT_INPUT) cchain = PCN_IPT_INPUT;
      }
    }
    if (kLate) prefetch(cur, i + PF * step);
    if (wr) {
      a.verdicts[i] = static_cast<uint8_t>(verdict);
      if (a.rule_ids) a.rule_ids[i] = rid;
    }
    // ---- stage A of a stateful batch that writes the walk records itself ----
    // (frames shorter than 70 bytes and one label: what ct_prep would build
    // from a second read of the frames, devchain.h ct_walk_rec; the label-0
    // outcome is this launch's own)
    // Its stale ports (Q4) without waiting on another workgroup: the group's
    // ports word published, the ports of an earlier TCP / UDP frame of the
    // group taken from it, and the lanes with none before them marked for
    // conntrack.hip ct_stale_fix (uniform control flow: ballots over the wave)
    bool ct_early = false;   // no TCP / UDP frame before this one in its group
    uint64_t ct_g = 0;       // the group (uniform)
    if (kCtRec && a.ct_pdesc) {
      const bool wrote = valid && ps == 2 && (p.proto == 6 || p.proto == 17);
      const uint64_t wm = __ballot(wrote);
      const uint32_t last_pd = __shfl(own_pd, wm ? 63 - __builtin_clzll(wm) : 0);
      const uint64_t g0 = (a.gbase + i) >> 6;
      ct_g = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g0 >> 32))) << 32) |
             static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(g0)));
      if (lane == 0 && valid)
        a.ct_pdesc[ct_g] = ct_ports_word(wm ? kCtPortsLocal : kCtPortsNone, last_pd);
      const uint64_t before = wm & ((1ull << lane) - 1);
      stale = __shfl(own_pd, before ? 63 - __builtin_clzll(before) : 0);
      ct_early = !before;
    }
    bool ct_fix = false;     // this lane's record waits for the ports before its group
    if (kCtRec && a.ct_brec && valid) {
      CtFrame f{};
      const bool tcp = p.proto == 6;
      f.status = ps;
      f.ports_ok = ps == 2 && (tcp || p.proto == 17);
      f.L = L;
      f.src = p.saddr;
      f.dst = p.daddr;
      f.seq = ps == 2 && tcp ? (h.w[9] >> 16) | (h.w[10] << 16) : 0u;
      f.ack = ps == 2 && tcp ? (h.w[10] >> 16) | (h.w[11] << 16) : 0u;
      f.flags = ps == 2 && tcp ? h.w[11] >> 24 : 0u;
      f.own = own_pd;
      f.stale = stale;
      f.proto = p.proto;
      f.icmp = (h.w[8] >> 16) & 0xffu;
      uint32_t cc = 3;
      bool pass = false, labeled = false;
      if (ps == 2) {
        const bool ingress = a.direction == PCN_IPT_INGRESS;
        const bool ldst = !a.fw && ingress && !a.allow_logic && a.nlocal && localip_has(a, p.daddr);
        const bool lsrc = !a.fw && !ingress && a.nlocal && localip_has(a, p.saddr);
        ct_select(false, false, a.fw != 0, ingress, a.allow_logic != 0, ldst, lsrc, a.empty_mask, a.drop_mask, cc, pass,
                  labeled);
      }
      ct_fix = valid && labeled && ps == 2 && !f.ports_ok && ct_early;
      const CtWalkOut wo = ct_walk_rec(f, cc, pass, labeled, rid * 2 | static_cast<int32_t>(verdict), a.ct_sentinel);
      u32x4 *d = reinterpret_cast<u32x4 *>(a.ct_brec) + 2 * i;
      d[0] = u32x4{wo.w[0], wo.w[1], wo.w[2], wo.w[3]};
      d[1] = u32x4{wo.w[4], wo.w[5], wo.w[6], wo.w[7]};
      a.ct_keys[i] = wo.key;
      a.ct_lcs[i] = wo.lcs;
    }
    if (kCtRec && a.ct_pdesc) {
      const uint64_t fm = __ballot(ct_fix);
      if (lane == 0 && valid) a.ct_fixm[ct_g] = fm;
    }
    // ---- counters ----
    if (PCN_ABLATE == 4) return;
    // Horus hits (Horus_dp.c:80-90): LDS bins, or one global atomic pair per
    // distinct rule id of the wave
    if (kHorus && a.horus_ctr) {
      const bool hz = valid && rid <= PCN_IPT_RID_HORUS0;
      if (__ballot(hz)) {
        const uint32_t id = hz ? static_cast<uint32_t>(PCN_IPT_RID_HORUS0 - rid) : 0u;
        if (a.hz_bins >= 0) {
          if (hz) {
            atomicAdd(&bins[a.hz_bins + id], 1u);
            if (!FIXED) atomicAdd(&byte_bins[a.hz_bins + id], L);
          }
        } else {
          bool left = hz;
          while (__ballot(left)) {
            const uint32_t lead = static_cast<uint32_t>(__builtin_ctzll(__ballot(left)));
            const uint32_t lid = __shfl(id, lead);
            const bool mine = left && id == lid;
            const uint64_t mm = __ballot(mine);
            uint32_t by = mine ? L : 0u;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) by += __shfl_xor(by, o);
            if (lane == lead) {
              atomicAdd(&a.horus_ctr[2 * lid], static_cast<unsigned long long>(__builtin_popcountll(mm)));
              atomicAdd(&a.horus_ctr[2 * lid + 1], static_cast<unsigned long long>(by));
            }
            left = left && !mine;
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (!((a.count_mask >> c) & 1)) continue;   // chain unreachable in this launch
      // default bins: wave-aggregated per chain
      const bool mine = valid && cchain == c && rid == PCN_IPT_RID_DEFAULT;
      const uint64_t m = __ballot(mine);
      if (m) {
        uint32_t bytes = 0;
        if (!FIXED) {
          uint32_t x = mine ? L : 0u;
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
          bytes = x;
        }
        if ((threadIdx.x & 63) == 0) {
          atomicAdd(&bins[c], static_cast<uint32_t>(__builtin_popcountll(m)));
          if (!FIXED) atomicAdd(&byte_bins[c], bytes);
        }
      }
      // per-rule bins: only chains that run rules in this variant
      if (CH < 3 ? c != CH : c == PCN_IPT_OUTPUT) continue;
      const DevChain &ch = CH < 3 ? run_ch : a.ch[c];
      if (valid && cchain == c && rid >= 0 && static_cast<uint32_t>(rid) < ch.ncounted) {
        if (PCN_ABLATE == 6) {
        } else if (ch.lds_bins >= 0 && static_cast<uint32_t>(rid) < ch.lds_nrules) {
          uint32_t b = static_cast<uint32_t>(ch.lds_bins) + static_cast<uint32_t>(rid);
          if (PCN_ABLATE == 7) bins[b] = 1u;   // measurement: a plain store instead of the atomic
          else atomicAdd(&bins[b], 1u);
          if (!FIXED) atomicAdd(&byte_bins[b], L);
        } else if (PCN_ABLATE != 8) {   // (8: measurement, no global atomics for the ids past the bins)
          if (a.ctr_pack_off) {         // one packed pair into this workgroup's copy
            unsigned long long *const cp =
                ch.ctr + a.ctr_pack_off + static_cast<uint64_t>(blockIdx.x & a.ctr_rep_mask) * a.ctr_rep_words;
            atomicAdd(&cp[1 + rid], (1ull << kCtrPackShift) | L);
          } else {
            atomicAdd(&ch.ctr[2 + 2 * rid], 1ull);
            if (PCN_ABLATE != 9) atomicAdd(&ch.ctr[3 + 2 * rid], static_cast<unsigned long long>(L));
          }
        }
      }
    }
  };
  for (uint64_t i = first; i < n_round; i += PF * step) {
#pragma unroll
    for (int d = 0; d < PF; ++d)
      if (d == 0 || i + d * step < n_round) process(i + d * step, st[d]);
  }
  // the last stages' (unused) asm chunk loads land before the wave moves on
  if (PCN_HDR_ASM && FIXED && PCN_HDR_LDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.deal_stats && lane == 0 && wide) atomicAdd(lds_stats, wide);
  __syncthreads();
  if (a.dbg_clk) clk2 = __builtin_amdgcn_s_memrealtime();
  // the workgroup's deal statistics, stored into host-mapped memory (a plain
  // system-scope vector store; the host reads whatever has landed)
  if (a.deal_stats && threadIdx.x == 0)
    __hip_atomic_store(&a.deal_stats[blockIdx.x], *lds_stats, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (chunked) {
    // The launch's last workgroup to finish zeroes the start counter for the
    // next launch (no memset per launch) and, on the batch's last launch,
    // writes the carry: every group is published by then, so the look-back
    // from the end gives the ports of the batch's last frame that wrote them,
    // or the previous carry (no tail pass over the batch).
    uint32_t *slot = reinterpret_cast<uint32_t *>(pcn_smem + a.lds_scratch);   // wave 0's region, free now
    if (threadIdx.x == 0)
      *slot = __hip_atomic_fetch_add(&a.chunk_ctr[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
              gridDim.x - 1;
    __syncthreads();
    const bool last_wg = *slot != 0;
    __syncthreads();
    if (last_wg && threadIdx.x < 64) {
      if (a.carry_out) {
        const uint32_t cout = stale_lookback(a, (a.gbase + a.n + 63) >> 6);
        if (threadIdx.x == 0) *a.carry_out = cout;
      }
      if (threadIdx.x == 0) {
        __hip_atomic_store(&a.chunk_ctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.chunk_ctr[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (PCN_ABLATE == 5) return;
  // ---- flush the workgroup histogram ----
  // Workgroups finish together and all add into the same counters; each
  // starts at its own rotation of the bins so the global atomics of
  // concurrent flushes mostly land on different addresses.
  const uint32_t rot = PCN_FLUSH_ROT ? (blockIdx.x * 97u) % a.nbins : 0u;
  const uint64_t rep = a.ctr_pack_off + static_cast<uint64_t>(blockIdx.x & a.ctr_rep_mask) * a.ctr_rep_words;
  for (uint32_t b0 = threadIdx.x; b0 < a.nbins; b0 += blockDim.x) {
    const uint32_t b = b0 + rot < a.nbins ? b0 + rot : b0 + rot - a.nbins;
    const unsigned long long pk = bins[b];
    const unsigned long long by = FIXED ? pk * a.fixed_len : byte_bins[b];
    if (!pk) continue;
    unsigned long long *blk = nullptr;   // a chain's counter block, pair `pair` (0: default)
    uint32_t pair = 0;
    if (b < 3) {
      blk = a.ch[b].ctr;
    } else {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const DevChain &ch = c == CH ? run_ch : a.ch[c];
        if (ch.lds_bins >= 0 && b >= static_cast<uint32_t>(ch.lds_bins) &&
            b < static_cast<uint32_t>(ch.lds_bins) + ch.lds_nrules) {
          blk = ch.ctr;
          pair = 1 + (b - static_cast<uint32_t>(ch.lds_bins));
        }
      }
      if (a.hz_bins >= 0 && b >= static_cast<uint32_t>(a.hz_bins) && a.horus_ctr) {   // Horus: one plain block
        unsigned long long *const dst = a.horus_ctr + 2 * (b - static_cast<uint32_t>(a.hz_bins));
        atomicAdd(dst, pk);
        atomicAdd(dst + 1, by);
        continue;
      }
      if (!blk) continue;
    }
    if (a.ctr_pack_off) {
      atomicAdd(blk + rep + pair, pk << kCtrPackShift | by);
    } else {
      atomicAdd(blk + 2 * pair, pk);
      if (PCN_ABLATE != 9) atomicAdd(blk + 2 * pair + 1, by);
    }
  }
  if (a.dbg_clk) {
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long *const c = a.dbg_clk + 4ull * blockIdx.x;
      c[0] = clk0;
      c[1] = clk1;
      c[2] = clk2;
      c[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

template <bool FIXED, bool LDS, int CH, int NS>
__global__ __launch_bounds__(kBlock) void classify_kernel(const LaunchArgs a) {
  classify_body<FIXED, LDS, CH, NS, false>(a);
}

}  // namespace

#ifdef PCN_JIT
// The one kernel of a JIT chain program (looked up by name after hiprtc).
#ifndef PCN_WAVES_PER_SIMD
#define PCN_WAVES_PER_SIMD 1   // >= 8: two 1024-thread workgroups per CU (<= 64 VGPRs)
#endif
#if defined(PCN_JIT_SPLIT) && PCN_JIT_SPLIT
// A split launch's two kernels (classify_body SPLIT): the gather kernel under
// the program's usual name, in PCN_SPLIT_G_BLOCK-thread workgroups, as many
// per CU as its registers allow (no chain image in LDS: ~75 VGPRs, 6 waves
// per SIMD), then the rule kernel.
extern "C" __global__ __launch_bounds__(PCN_SPLIT_G_BLOCK) void pcn_classify_jit(const LaunchArgs a) {
  classify_body<PCN_JIT_FIXED, false, PCN_JIT_CH, PCN_JIT_NS, true, 1>(a);
}
extern "C" __global__ __launch_bounds__(kBlock, PCN_WAVES_PER_SIMD) void pcn_split_rules(const LaunchArgs a) {
  classify_body<PCN_JIT_FIXED, PCN_JIT_LDS, PCN_JIT_CH, PCN_JIT_NS, true, 2>(a);
}
#else
extern "C" __global__ __launch_bounds__(kBlock, PCN_WAVES_PER_SIMD) void pcn_classify_jit(const LaunchArgs a) {
  classify_body<PCN_JIT_FIXED, PCN_JIT_LDS, PCN_JIT_CH, PCN_JIT_NS, true>(a);
}
#endif
#else
namespace {

template <bool FIXED, bool LDS, int NS>
void launch_variant(const LaunchArgs &a, int ch, unsigned grid, size_t lds, hipStream_t stream) {
  switch (ch) {
    case 0: hipLaunchKernelGGL((classify_kernel<FIXED, LDS, 0, NS>), dim3(grid), dim3(kBlock), lds, stream, a); break;
    case 1: hipLaunchKernelGGL((classify_kernel<FIXED, LDS, 1, NS>), dim3(grid), dim3(kBlock), lds, stream, a); break;
    case 2: hipLaunchKernelGGL((classify_kernel<FIXED, LDS, 2, NS>), dim3(grid), dim3(kBlock), lds, stream, a); break;
    default: hipLaunchKernelGGL((classify_kernel<FIXED, LDS, 3, NS>), dim3(grid), dim3(kBlock), lds, stream, a); break;
  }
}

// The generic kernel always runs six slots (unused ones hold the all-ones
// class); a chain program runs exactly the chain's lay.nslots.
template <bool FIXED, bool LDS>
void launch_ns(const LaunchArgs &a, int ch, int, unsigned grid, size_t lds, hipStream_t stream) {
  launch_variant<FIXED, LDS, 6>(a, ch, grid, lds, stream);
}

}  // namespace

// Host-side launcher (called from pcn_ipt.cpp).  `ch` is the only chain that can
// reach the rule stage (0..2) or 3 for INPUT+FORWARD.  `jit` (a hipFunction_t
// or null) is the chain program compiled for exactly this launch shape
// (jit.cpp); null runs the generic variant.  Returns a hipError_t.
//
// Split launches (jit2 = the program's rule kernel, ga = the gather kernel's
// arguments: its own LDS layout, no chain image): each launch chunk runs the
// gather kernel (`jit`, ga_wg workgroups per CU) and then the rule kernel over
// the records it left in a.split_rec (indexed from the chunk's first frame).
int launch_classify(const LaunchArgs &a, bool fixed, int ch, int ns, int num_cus, void *jit, hipStream_t stream,
                    CopyBound *cb, void *jit2, const LaunchArgs *ga, unsigned ga_wg) {
  if (a.n == 0) return hipSuccess;
  const size_t lds = a.lds_bytes;
  const bool in_lds = a.lds_images_bytes > 0;
  // (PCN_IPT_DEBUG_WG_PER_CU: measurement A/B of the workgroups per CU)
  static const size_t max_per_cu = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_WG_PER_CU");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    // default one: the kernel's ~110 VGPRs allow 4 waves per SIMD, i.e. one
    // 1024-thread workgroup per CU; a second one per CU could only run after
    // the first (config 2, whose small image allowed two: 2^20 frames 28.4 ->
    // 21.7 us, 2^24 203 -> 195 us, profiles/r04_s2/)
    return v >= 1 && v <= 2 ? static_cast<size_t>(v) : size_t(1);
  }();
  size_t per_cu = lds ? (160 * 1024) / lds : max_per_cu;
  if (per_cu > max_per_cu) per_cu = max_per_cu;
  if (per_cu < 1) per_cu = 1;
  const uint64_t want = (a.n + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * per_cu;
  const unsigned grid = static_cast<unsigned>(want < cap ? want : cap);
  // u32 histogram bins: at most 2^32-1 bytes per workgroup per launch, so a
  // batch whose workgroups could exceed that is split into launches; so is
  // one that could fill more than half of a packed counter copy's fields
  // (each copy takes the flushes of `wpc` workgroups).
  const uint64_t max_len = a.lens ? 65535u : (a.fixed_len ? a.fixed_len : 1u);
  const uint64_t wpc = (grid + uint64_t(a.ctr_rep_mask)) / (uint64_t(a.ctr_rep_mask) + 1);
  const bool split = jit && jit2 && ga;
  const uint64_t gwant = (a.n + PCN_SPLIT_G_BLOCK - 1) / PCN_SPLIT_G_BLOCK;
  const unsigned ggrid = split ? static_cast<unsigned>(std::min<uint64_t>(gwant, uint64_t(num_cus) * ga_wg)) : 0u;
  // (a workgroup takes whole kBlock-frame rows of the grid stride)
  uint64_t per_block = 0xFFFFFFFFull / max_len;
  if (cb && a.ctr_pack_off) {
    per_block = std::min<uint64_t>(per_block, (cb->max_pkts / 2) / wpc);
    per_block = std::min<uint64_t>(per_block, (cb->max_bytes / 2) / (wpc * max_len));
  }
  per_block = std::max<uint64_t>(per_block / kBlock * kBlock, kBlock);
  const uint64_t chunk = per_block * grid;
  for (uint64_t base = 0; base < a.n; base += chunk) {
    LaunchArgs c = a;
    c.n = a.n - base < chunk ? a.n - base : chunk;
    if (cb && a.ctr_pack_off) {
      // the most any one copy takes from this launch; fold first if the copies
      // could overflow (cb->fold resets the bound)
      const uint64_t fw = (c.n + uint64_t(grid) * kBlock - 1) / (uint64_t(grid) * kBlock) * kBlock;
      // (a split launch's two kernels each add at most that much into a copy)
      const uint64_t pk = wpc * fw * (split ? 2 : 1), by = pk * max_len;
      if (cb->pkts + pk > cb->max_pkts || cb->bytes + by > cb->max_bytes) {
        const int e = cb->fold(cb->ctx, static_cast<void *>(stream));
        if (e != hipSuccess) return e;
      }
      cb->pkts += pk;
      cb->bytes += by;
    }
    if (a.has_stale) {   // contiguous chunks per workgroup, claimed in start order
      c.gbase = base;
      c.chunk_frames = (c.n + uint64_t(grid) * kBlock - 1) / (uint64_t(grid) * kBlock) * kBlock;
      // (the counters are zero: each launch's last workgroup resets them)
      if (base + c.n < a.n) c.carry_out = nullptr;   // only the batch's last launch writes the carry
    }
    if (base) {
      if (!a.offsets) { c.frames = a.frames + base * a.stride; c.frames_bytes = a.frames_bytes - base * a.stride; }
      else c.offsets = a.offsets + base;
      if (a.lens) c.lens = a.lens + base;
      if (a.ct_brec) {
        c.ct_brec = a.ct_brec + base * 8;
        c.ct_keys = a.ct_keys + base;
        c.ct_lcs = a.ct_lcs + base;
      }
      if (a.has_in_port) c.in_port = a.in_port + base;
      if (a.has_ct) c.ct_status = a.ct_status + base;
      c.verdicts = a.verdicts + base;
      if (a.rule_ids) c.rule_ids = a.rule_ids + base;
    }
    if (split) {
      LaunchArgs g = *ga;            // the chunk's frames, the gather kernel's LDS layout
      g.n = c.n;
      g.frames = c.frames;
      g.frames_bytes = c.frames_bytes;
      g.offsets = c.offsets;
      g.lens = c.lens;
      g.in_port = c.in_port;
      g.ct_status = c.ct_status;
      g.verdicts = c.verdicts;
      g.rule_ids = c.rule_ids;
      size_t sz = sizeof(LaunchArgs);
      void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &g, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      hipError_t e = hipModuleLaunchKernel(static_cast<hipFunction_t>(jit), ggrid, 1, 1, PCN_SPLIT_G_BLOCK, 1, 1,
                                           static_cast<unsigned>(g.lds_bytes), stream, nullptr, extra);
      if (e != hipSuccess) return static_cast<int>(e);
      void *extra2[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &c, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      e = hipModuleLaunchKernel(static_cast<hipFunction_t>(jit2), grid, 1, 1, kBlock, 1, 1, static_cast<unsigned>(lds),
                                stream, nullptr, extra2);
      if (e != hipSuccess) return static_cast<int>(e);
      continue;
    }
    if (jit) {
      size_t sz = sizeof(LaunchArgs);
      void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &c, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      const hipError_t e = hipModuleLaunchKernel(static_cast<hipFunction_t>(jit), grid, 1, 1, kBlock, 1, 1,
                                                 static_cast<unsigned>(lds), stream, nullptr, extra);
      if (e != hipSuccess) return static_cast<int>(e);
      continue;
    }
    if (fixed && in_lds) launch_ns<true, true>(c, ch, ns, grid, lds, stream);
    else if (fixed) launch_ns<true, false>(c, ch, ns, grid, lds, stream);
    else if (in_lds) launch_ns<false, true>(c, ch, ns, grid, lds, stream);
    else launch_ns<false, false>(c, ch, ns, grid, lds, stream);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return hipSuccess;
}

// Fold the packed counter copies (LaunchArgs::ctr_pack_off) into the plain
// block: pair i of every copy is taken with an atomic exchange (a classify on
// another stream may be adding meanwhile) and unpacked on its own (the sum of
// the copies could overflow a field), then added to pair i of the block.
__global__ void fold_reps_kernel(unsigned long long *ctr, uint64_t pairs, uint64_t pack_off, uint64_t stride,
                                 uint32_t reps) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= pairs) return;
  unsigned long long pk = 0, by = 0;
  for (uint32_t r = 0; r < reps; ++r) {
    unsigned long long *p = ctr + pack_off + r * stride + i;
    if (!*p) continue;
    const unsigned long long w = atomicExch(p, 0ull);
    pk += w >> kCtrPackShift;
    by += w & kCtrPackBytesMask;
  }
  if (pk) atomicAdd(&ctr[2 * i], pk);
  if (by) atomicAdd(&ctr[2 * i + 1], by);
}

int launch_fold_reps(unsigned long long *ctr, uint64_t pairs, uint64_t pack_off, uint64_t stride, uint32_t reps,
                     hipStream_t stream) {
  if (pairs == 0) return hipSuccess;
  const unsigned grid = static_cast<unsigned>((pairs + 255) / 256);
  hipLaunchKernelGGL(fold_reps_kernel, dim3(grid), dim3(256), 0, stream, ctr, pairs, pack_off, stride, reps);
  return static_cast<int>(hipGetLastError());
}

// Sum `nranks` gathered counter blocks into `out` (u64 element-wise).
__global__ void sum_ranks_kernel(const unsigned long long *in, unsigned long long *out, uint64_t count,
                                 int nranks) {
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= count) return;
  unsigned long long s = 0;
  for (int r = 0; r < nranks; ++r) s += in[static_cast<uint64_t>(r) * count + i];
  out[i] = s;
}

int launch_sum_ranks(const unsigned long long *in, unsigned long long *out, uint64_t count, int nranks,
                     hipStream_t stream) {
  if (count == 0) return hipSuccess;
  unsigned grid = static_cast<unsigned>((count + 255) / 256);
  hipLaunchKernelGGL(sum_ranks_kernel, dim3(grid), dim3(256), 0, stream, in, out, count, nranks);
  return static_cast<int>(hipGetLastError());
}
#endif  // PCN_JIT

}  // namespace pcn
