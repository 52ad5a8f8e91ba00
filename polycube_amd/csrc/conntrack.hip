// conntrack.hip — stateful connection tracking on the GPU (see conntrack.hpp).
//
// Semantics restated from the reference (paths under
// src/services/pcn-iptables/src/datapaths/):
//   key + labels      Iptables_ConntrackLabel_dp.c:190-531
//   accept-established Iptables_ConntrackLabel_dp.c:580-650
//   table update      Iptables_ConntrackTableUpdate_dp.c:141-655
//   stale ports (Q4)  Iptables_Parser_dp.c:122-143 (ports written for TCP/UDP only)
// Everything here is integer work on HBM-resident state: the parse/prep
// kernels stream the 72-byte header window once, the walk is latency-bound
// (one dependent table access per packet of a run), the sort is the
// hand-written LSD radix sort of radix.hip on a key-bucket id.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <vector>

#include "conntrack.hpp"
#include "devchain.h"
#include "radix.hpp"
#include "pcn_ipt.h"

#ifndef PCN_CT_FAST
#define PCN_CT_FAST 1   // walk: straight-line step for established TCP / live UDP connections
#endif

// llvm.amdgcn.struct.ptr.buffer.load (no clang builtin): buffer_load_dwordx4
// ... idxen, bounds-checked by record index
typedef int ct_i32x4 __attribute__((ext_vector_type(4)));
__device__ ct_i32x4 ct_struct_load_v4(__amdgpu_buffer_rsrc_t rsrc, int vindex, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");

namespace pcn {

namespace {

enum : uint8_t { K_NONE = 0, K_INV, K_TCP, K_UDP, K_ECHO, K_REPLY, K_ERR, K_HARD };
static_assert(K_INV == kCtKInv && K_TCP == kCtKTcp && K_UDP == kCtKUdp && K_ECHO == kCtKEcho &&
                  K_REPLY == kCtKReply && K_ERR == kCtKErr && K_HARD == kCtKHard,
              "record kinds as devchain.h numbers them");
enum { ST_NEW = 0, ST_EST, ST_REL, ST_INV, ST_SYN_SENT, ST_SYN_RECV, ST_FIN_WAIT_1, ST_FIN_WAIT_2, ST_LAST_ACK,
       ST_TIME_WAIT };
constexpr uint8_t FIN = 0x01, SYN = 0x02, RST = 0x04, ACK = 0x10;
constexpr uint32_t HEX_BE_ONE = 0x1000000u;
// ConntrackTableUpdate_dp.c:38-48 (ns)
constexpr unsigned long long UDP_ESTABLISHED_TIMEOUT = 180000000000ull, UDP_NEW_TIMEOUT = 30000000000ull,
                             ICMP_TIMEOUT = 30000000000ull, TCP_ESTABLISHED_T = 432000000000000ull,
                             TCP_SYN_SENT_T = 120000000000ull, TCP_SYN_RECV_T = 60000000000ull,
                             TCP_LAST_ACK_T = 30000000000ull, TCP_FIN_WAIT_T = 120000000000ull;

typedef uint32_t ct_u32x4 __attribute__((ext_vector_type(4)));

// Per-packet record written by ct_prep (32 B).
struct CtRec {
  uint32_t src, dst;       // table key: the packet's own (ordered), or the quoted header's for K_ERR
  uint16_t sport, dport;
  uint32_t seq, ack;       // TCP; for K_HARD: the quoted header's ordered src / dst
  uint16_t len;            // packet_len after a TC untag (counters)
  uint8_t proto, kind;
  uint8_t rev;             // bit0 ipRev, bit1 portRev
  uint8_t flags;           // TCP flags; for K_HARD: the quoted header's protocol
  uint8_t cinfo;           // bits 0-1: chain (3: none), bit 2: PASS_LABELING
  uint8_t icmp;
  uint32_t iports;         // K_HARD: the quoted header's ordered ports (sport | dport << 16)
};
static_assert(sizeof(CtRec) == 32, "CtRec is 32 bytes");

struct Parsed {
  uint32_t L;
  int status;              // 0 RX_DROP in the parser, 1 not IPv4 (pass), 2 IPv4 parsed
  bool ports_ok;           // the Parser wrote srcPort/dstPort
  uint32_t src, dst, seq, ack, isrc, idst;
  uint16_t sport, dport, isport, idport;
  uint8_t proto, flags, icmp, iproto;
};

// The first 72 bytes of frame i (dword-aligned loads that stay inside the buffer).
__device__ __forceinline__ void load_window(const CtBatch &b, uint64_t i, uint32_t w[18], uint32_t &L) {
  const uint64_t off = b.offsets ? b.offsets[i] : i * uint64_t(b.stride);
  L = b.lens ? b.lens[i] : b.fixed_len;
  const uint64_t base = off & ~uint64_t(3);
  const uint32_t sh = static_cast<uint32_t>(off & 3);
  uint32_t d[19];
  if (base + 76 <= b.frames_bytes) {
    // the whole window inside the buffer: unconditional loads, which the
    // compiler merges into 16-byte ones (the per-dword bound checks kept each
    // of them a separate, branch-guarded dword load)
    const uint32_t *p = reinterpret_cast<const uint32_t *>(b.frames + base);
#pragma unroll
    for (int k = 0; k < 19; ++k) d[k] = p[k];
  } else {
#pragma unroll
    for (int k = 0; k < 19; ++k) {
      const uint64_t at = base + 4u * k;
      d[k] = at + 4 <= b.frames_bytes ? *reinterpret_cast<const uint32_t *>(b.frames + at) : 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < 18; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// Iptables_Parser_dp.c:94-153 (+ the TC-hook untag, see pcn_ipt.h), reading the
// fields the conntrack modules use.  Multi-byte fields are little-endian loads
// of network-order bytes, as the eBPF reads them.
__device__ __forceinline__ Parsed parse(const uint32_t w[18], uint32_t L, uint32_t hook) {
  Parsed p{};
  int s = 0;
  if (L >= 14 && hook == PCN_IPT_HOOK_TC) {
    const uint32_t et = ((w[3] & 0xff) << 8) | ((w[3] >> 8) & 0xff);
    if (et == 0x8100 || et == 0x88A8) {
      if (L < 18) { p.status = 0; return p; }
      s = 1;
      L -= 4;
    }
  }
  p.L = L;
  // bytes >= 12 move by one dword.  The asm keeps both words in registers:
  // folded into w[k + s], the window became a dynamically indexed array the
  // compiler placed in LDS (72 KB a workgroup: two workgroups per CU).
  auto W = [&](int k) {
    uint32_t a = w[k], b = w[k + 1];
    asm volatile("" : "+v"(a), "+v"(b));
    return s ? b : a;
  };
  if (L < 14) { p.status = 0; return p; }
  const uint32_t et = ((W(3) & 0xff) << 8) | ((W(3) >> 8) & 0xff);
  if (et != 0x0800) { p.status = 1; return p; }
  if (L < 34) { p.status = 0; return p; }
  p.proto = static_cast<uint8_t>(W(5) >> 24);
  p.src = (W(6) >> 16) | (W(7) << 16);
  p.dst = (W(7) >> 16) | (W(8) << 16);
  if (p.proto == 6) {
    if (L < 54) { p.status = 0; return p; }
    p.seq = (W(9) >> 16) | (W(10) << 16);
    p.ack = (W(10) >> 16) | (W(11) << 16);
    p.flags = static_cast<uint8_t>(W(11) >> 24);
    p.ports_ok = true;
  } else if (p.proto == 17) {
    if (L < 42) { p.status = 0; return p; }
    p.ports_ok = true;
  }
  p.sport = static_cast<uint16_t>(W(8) >> 16);
  p.dport = static_cast<uint16_t>(W(9) & 0xffff);
  p.icmp = static_cast<uint8_t>((W(8) >> 16) & 0xff);
  p.iproto = static_cast<uint8_t>(W(12) >> 24);
  p.isrc = (W(13) >> 16) | (W(14) << 16);
  p.idst = (W(14) >> 16) | (W(15) << 16);
  p.isport = static_cast<uint16_t>(W(15) >> 16);
  p.idport = static_cast<uint16_t>(W(16) & 0xffff);
  p.status = 2;
  return p;
}

__device__ __forceinline__ bool localip_has(const CtBatch &b, uint32_t ip) {
  uint32_t lo = 0, hi = b.nlocal;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint32_t v = b.localip[mid];
    if (v == ip) return true;
    if (v < ip) lo = mid + 1; else hi = mid;
  }
  return false;
}

__device__ __forceinline__ uint64_t key_hash(uint32_t src, uint32_t dst, uint8_t proto, uint16_t sp, uint16_t dp) {
  return ct_key_hash(src, dst, proto, sp, dp);     // devchain.h (the classify kernel's stage A uses it too)
}

// A packet's walk record in HBM (32 B), written by ct_prep in batch order and
// read by the walk through the sorted index: the fields the label / update
// code reads and the stage-A outcome of label 0 (rule id << 1 | verdict).
// The key bucket and batch index come from the sorted arrays, the outcomes of
// labels 1-3 (only when a chain has conntrack rules) from a side array.  (A
// 64-byte record held all of them: twice the bytes for ct_prep to write and
// for the walk's random gathers to read.)
struct alignas(16) PackedRec {
  uint32_t src, dst;
  uint32_t ports;          // sport | dport << 16
  uint32_t seq, ack, iports;
  uint32_t pfk;            // proto | flags << 8 | kind << 16 | (rev | cinfo << 2) << 24
  int32_t o0;
};
static_assert(sizeof(PackedRec) == 32, "PackedRec is 32 bytes");

// The walk's working copy of a record, in registers.
struct WalkRec {
  CtRec r;
  uint32_t key, idx;
  int32_t o0, o1, o2, o3;
};

__device__ __forceinline__ PackedRec pack_rec(const CtRec &r, int32_t o0) {
  PackedRec p;
  p.src = r.src;
  p.dst = r.dst;
  p.ports = uint32_t(r.sport) | uint32_t(r.dport) << 16;
  p.seq = r.seq;
  p.ack = r.ack;
  p.iports = r.iports;
  p.pfk = uint32_t(r.proto) | uint32_t(r.flags) << 8 | uint32_t(r.kind) << 16 | uint32_t(r.rev | r.cinfo << 2) << 24;
  p.o0 = o0;
  return p;
}

__device__ __forceinline__ CtRec ct_rec(const PackedRec &p) {
  CtRec r{};
  r.src = p.src;
  r.dst = p.dst;
  r.sport = static_cast<uint16_t>(p.ports);
  r.dport = static_cast<uint16_t>(p.ports >> 16);
  r.seq = p.seq;
  r.ack = p.ack;
  r.iports = p.iports;
  r.proto = static_cast<uint8_t>(p.pfk);
  r.flags = static_cast<uint8_t>(p.pfk >> 8);
  r.kind = static_cast<uint8_t>(p.pfk >> 16);
  r.rev = static_cast<uint8_t>((p.pfk >> 24) & 3);
  r.cinfo = static_cast<uint8_t>(p.pfk >> 26);
  return r;
}

// One record as two 16-byte loads (a field-by-field copy of the packed
// struct issues narrow loads on the walk's critical path).
__device__ __forceinline__ PackedRec load_prec(const PackedRec *p) {
  const ct_u32x4 *s = reinterpret_cast<const ct_u32x4 *>(p);
  union {
    ct_u32x4 v[2];
    PackedRec r;
  } u;
  u.v[0] = s[0];
  u.v[1] = s[1];
  return u.r;
}

__device__ __forceinline__ void store_prec(PackedRec *p, const PackedRec &r) {
  union {
    ct_u32x4 v[2];
    PackedRec r;
  } u;
  u.r = r;
  ct_u32x4 *d = reinterpret_cast<ct_u32x4 *>(p);
  d[0] = u.v[0];
  d[1] = u.v[1];
}

__device__ __forceinline__ int32_t pack_outcome(const CtBatch &b, uint32_t l, uint64_t i) {
  return l < b.nlab ? (b.a_rid[l * b.n + i] * 2) | b.a_verdict[l * b.n + i] : 0;
}

// The Parser's stale ports (Q4) inside ct_prep, without a pass of its own:
// workgroups claim contiguous chunks of the batch in start order, every
// 64-frame group publishes the ports of its last TCP/UDP frame (or that it
// has none), and a frame that needs the ports of an earlier group looks back
// through the published words, {1:24 | status:2 | ports:32} (0: not yet).
// A group only waits on lower groups, whose waves are running or done, so the
// waits resolve.  (Was ct_parse + a max-scan + ct_carry: 0.32 ms a batch.)
// Frames per claimed chunk: 4096, or fewer (a multiple of 64, at least 512)
// when the batch would otherwise not give every CU eight workgroups -- a
// 2 M-frame batch (one rank's share of a flow split) ran 508 workgroups of
// 256 threads, 8 waves per CU, on its dependent header reads.
constexpr uint32_t kPrepChunk = 4096;
__host__ __device__ inline uint32_t prep_chunk(uint64_t n, int num_cus) {
  uint64_t c = (n / (uint64_t(num_cus) * 8) + 63) / 64 * 64;
  return static_cast<uint32_t>(c < 512 ? 512 : c > kPrepChunk ? kPrepChunk : c);
}
constexpr unsigned long long kStLocal = 1, kStIncl = 2, kStNone = 3;
static_assert(kStLocal == kCtPortsLocal && kStNone == kCtPortsNone, "devchain.h ct_ports_word: the same states");
// ct_stale_agg / ct_stale_fix: 1024 groups a workgroup, 4 a thread
constexpr uint32_t kStaleScanBlock = 256, kStaleScanPer = 4;
constexpr uint64_t kStaleScanGroups = uint64_t(kStaleScanBlock) * kStaleScanPer;

__device__ __forceinline__ unsigned long long ports_word(unsigned long long st, uint32_t ports) {
  return (1ull << 40) | (st << 32) | ports;
}
__device__ uint32_t ports_lookback(const unsigned long long *desc, uint64_t g, const uint32_t *carry) {
  while (g > 0) {
    --g;
    unsigned long long d;
    for (;;) {
      d = __hip_atomic_load(&desc[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d >> 40) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (((d >> 32) & 3) != kStNone) return static_cast<uint32_t>(d);
  }
  return *carry;
}

// Chain selection (ChainSelector_dp.c:131-298), the conntrack key and kind;
// packets that need no table access get their final outcome here.
// PCN_CT_PREP_LDS: a wave whose 64 frames sit at a 64-byte stride (the
// fixed-stride batch) loads them as coalesced 16-byte chunks and transposes
// them through LDS into per-lane windows, and writes its 64 walk records back
// the same way, instead of one lane per 76-byte window / 64-byte record (every
// wave instruction then touching 64 lines).
#ifndef PCN_CT_PREP_LDS
#define PCN_CT_PREP_LDS 1
#endif
#ifndef PCN_CT_PREP_PF
#define PCN_CT_PREP_PF 1     // the next group's loads in flight (fixed-stride path)
#endif
constexpr uint32_t kPrepBlock = 256;
constexpr uint32_t kPrepRow = 5;                 // 16-byte chunks per frame row in LDS (4 + 1 of padding)
#ifdef PCN_CT_PREP_WAVES
#define PCN_CT_PREP_ATTR __attribute__((amdgpu_waves_per_eu(PCN_CT_PREP_WAVES)))
#else
#define PCN_CT_PREP_ATTR
#endif
__global__ __launch_bounds__(kPrepBlock) PCN_CT_PREP_ATTR void ct_prep_kernel(CtBatch b, const uint32_t *carry, PackedRec *brec,
                               ct_u32x4 *ox, uint32_t *lcs, uint32_t *keys, uint32_t kbits, uint32_t *hard_cnt, uint32_t *hard_list, unsigned long long *desc,
                               uint32_t *chunk_ctr, uint32_t chunk_frames) {
  const uint32_t sentinel = (1u << kbits) - 1;
  const uint32_t lane = __lane_id();
  const bool a0_final = b.nlab == 1 && b.a_rid == b.rule_ids && b.a_verdict == b.verdicts;
  __shared__ uint32_t chunk;
#if PCN_CT_PREP_LDS
  __shared__ ct_u32x4 prep_stage[(kPrepBlock / 64) * 65 * kPrepRow];
  ct_u32x4 *const stage = prep_stage + (threadIdx.x >> 6) * 65 * kPrepRow;
  const bool stride64 = !b.offsets && b.stride == 64 && (reinterpret_cast<uintptr_t>(b.frames) & 15) == 0;
#endif
  for (;;) {
    if (threadIdx.x == 0) chunk = atomicAdd(chunk_ctr, 1u);
    __syncthreads();
    const uint64_t lo = uint64_t(chunk) * chunk_frames;
    __syncthreads();                                      // everyone has read `chunk`
    if (lo >= b.n) return;
    const uint64_t hi = lo + chunk_frames < b.n ? lo + chunk_frames : b.n;
#if PCN_CT_PREP_LDS && PCN_CT_PREP_PF
    // The next group's frames and label-0 outcome are in flight while a wave
    // works on its group (one group's loads at a time left the waves waiting
    // on memory three quarters of their life).
    ct_u32x4 pc[4] = {}, pex = {};
    int32_t prid = 0;
    uint8_t pver = 0;
    auto fetch = [&](uint64_t g0) {
      if (stride64 && (g0 + 64) * 64 + 16 <= b.frames_bytes) {
        const ct_u32x4 *src = reinterpret_cast<const ct_u32x4 *>(b.frames + g0 * 64);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) pc[q] = src[q * 64 + lane];
        pex = src[256];
      }
      const uint64_t j = g0 + lane < hi ? g0 + lane : hi - 1;
      prid = b.a_rid[j];
      pver = b.a_verdict[j];
    };
    if (lo + (threadIdx.x & ~63u) < hi) fetch(lo + (threadIdx.x & ~63u));
#endif
  for (uint64_t i0 = lo + (threadIdx.x & ~63u); i0 < hi; i0 += blockDim.x) {   // one 64-frame group per wave
    const uint64_t i = i0 + lane;
    const bool valid = i < hi;
    uint32_t w[18], L;
#if PCN_CT_PREP_LDS && PCN_CT_PREP_PF
    const int32_t rid0 = prid;
    const uint8_t ver0 = pver;
#else
    const int32_t rid0 = b.a_rid[valid ? i : hi - 1];
    const uint8_t ver0 = b.a_verdict[valid ? i : hi - 1];
#endif
#if PCN_CT_PREP_LDS
    // the group's 64 frames and the next frame's first chunk inside the buffer (wave-uniform)
    const bool fast = stride64 && (i0 + 64) * 64 + 16 <= b.frames_bytes;
#if PCN_CT_PREP_PF
    const ct_u32x4 c[4] = {pc[0], pc[1], pc[2], pc[3]};
    const ct_u32x4 extra = pex;
#endif
    if (fast) {
#if !PCN_CT_PREP_PF
      const ct_u32x4 *src = reinterpret_cast<const ct_u32x4 *>(b.frames + i0 * 64);
      ct_u32x4 c[4];
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) c[q] = src[q * 64 + lane];   // chunk t = 64 q + lane: frame t / 4
      const ct_u32x4 extra = src[256];                               // the next frame's bytes 0-15
#endif
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t t = q * 64 + lane;
        stage[(t >> 2) * kPrepRow + (t & 3)] = c[q];
      }
      if (lane == 0) stage[64 * kPrepRow] = extra;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const ct_u32x4 *row = stage + lane * kPrepRow;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        const ct_u32x4 v = row[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
      }
      const ct_u32x4 nx = row[kPrepRow];
      w[16] = nx.x;
      w[17] = nx.y;
      L = b.lens ? b.lens[valid ? i : hi - 1] : b.fixed_len;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      load_window(b, valid ? i : hi - 1, w, L);
    }
#if PCN_CT_PREP_PF
    if (i0 + blockDim.x < hi) fetch(i0 + blockDim.x);   // after the group's chunks went to LDS
#endif
#else
    load_window(b, valid ? i : hi - 1, w, L);
#endif
    const Parsed p = parse(w, L, b.hook);
    // ---- the shared `packet` struct's ports as this frame sees them ----
    const uint32_t own = uint32_t(p.sport) | (uint32_t(p.dport) << 16);
    const bool wrote = valid && p.status == 2 && p.ports_ok;
    const uint64_t wm = __ballot(wrote);
    const uint64_t g = i0 >> 6;
    const uint32_t last_pd = __shfl(own, wm ? 63 - __builtin_clzll(wm) : 0);
    if (lane == 0)
      __hip_atomic_store(&desc[g], ports_word(wm ? kStLocal : kStNone, last_pd), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t before = wm & ((1ull << lane) - 1);
    uint32_t stale = __shfl(own, before ? 63 - __builtin_clzll(before) : 0);
    if (__ballot(valid && p.status == 2 && !p.ports_ok && !before)) {
      const uint32_t cin = ports_lookback(desc, g, carry);
      if (!before) stale = cin;
      if (!wm && lane == 0)
        __hip_atomic_store(&desc[g], ports_word(kStIncl, cin), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PackedRec pr;
    if (valid) {
      // the record (devchain.h ct_walk_rec: the classify kernel's stage A
      // builds the same one when it writes the records itself)
      uint32_t chain = 3;
      bool pass = false, labeled = false;
      if (p.status == 2) {
        // a Horus hit (stage A found it: the same for every label) skips the
        // ChainSelector / ChainForwarder: DROP is final, ACCEPT is PASS_LABELING
        // (Horus_dp.c:150-160; Firewall_Horus_dp.c:151-161), or final for a
        // pcn-firewall program built with conntrack off (:162-164).
        // pcn-firewall: Parser -> ConntrackLabel -> ChainForwarder; an empty
        // chain goes to DefaultAction after labelling, which stage A resolved.
        const bool horus = rid0 <= PCN_IPT_RID_HORUS0;
        const bool ingress = b.direction == PCN_IPT_INGRESS;
        const bool local_dst = !b.fw && ingress && !b.allow_logic && b.nlocal && localip_has(b, p.dst);
        const bool local_src = !b.fw && !ingress && b.nlocal && localip_has(b, p.src);
        ct_select(horus, ver0 == PCN_IPT_ACCEPT && !b.horus_final, b.fw, ingress, b.allow_logic, local_dst, local_src,
                  b.empty_mask, b.drop_mask, chain, pass, labeled);
      }
      CtFrame f;
      f.status = static_cast<uint32_t>(p.status);
      f.ports_ok = p.ports_ok;
      f.L = p.L;
      f.src = p.src;
      f.dst = p.dst;
      f.seq = p.seq;
      f.ack = p.ack;
      f.own = own;
      f.stale = stale;
      f.proto = p.proto;
      f.flags = p.flags;
      f.icmp = p.icmp;
      f.isrc = p.isrc;
      f.idst = p.idst;
      f.iproto = p.iproto;
      f.isport = p.isport;
      f.idport = p.idport;
      const int32_t o0 = b.nlab ? (rid0 * 2) | ver0 : 0;   // pack_outcome(b, 0, i)
      const CtWalkOut wo = ct_walk_rec(f, chain, pass, labeled, o0, sentinel);
      const bool member = wo.kind >= K_TCP && wo.kind <= K_ERR;
      keys[i] = wo.key;
      lcs[i] = wo.lcs;                                  // what ct_count reads (not the 64-byte record)
      if (b.nlab == 4)
        ox[i] = ct_u32x4{static_cast<uint32_t>(o0), static_cast<uint32_t>(pack_outcome(b, 1, i)),
                         static_cast<uint32_t>(pack_outcome(b, 2, i)), static_cast<uint32_t>(pack_outcome(b, 3, i))};
      static_assert(sizeof(PackedRec) == sizeof(wo.w), "the walk record is 8 words");
      __builtin_memcpy(&pr, wo.w, sizeof(pr));
#if PCN_CT_PREP_LDS
      if (fast) {                                       // this lane's record into its LDS row
        union {
          ct_u32x4 v[2];
          PackedRec rec;
        } u;
        u.rec = pr;
        stage[lane * kPrepRow] = u.v[0];
        stage[lane * kPrepRow + 1] = u.v[1];
      } else {
        store_prec(&brec[i], pr);
      }
#else
      store_prec(&brec[i], pr);
#endif
      if (wo.kind == K_HARD) hard_list[atomicAdd(hard_cnt, 1u)] = static_cast<uint32_t>(i);
      // every packet's outcome as far as it is known here, coalesced: final for
      // those with no table access (label INVALID for K_INV, else any label);
      // the label-0 one for the rest, which the walk overwrites only where it
      // differs (put_outcome)
      // (one label: stage A wrote its outcomes into the final arrays themselves)
      const bool l3 = !member && wo.kind == K_INV && !pass && b.nlab == 4;
      if (!a0_final) {
        b.verdicts[i] = l3 ? b.a_verdict[3 * b.n + i] : ver0;
        b.rule_ids[i] = l3 ? b.a_rid[3 * b.n + i] : rid0;
      }
    }
#if PCN_CT_PREP_LDS
    if (fast) {                                         // the wave's records as coalesced chunks
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      ct_u32x4 *dst = reinterpret_cast<ct_u32x4 *>(brec + i0);
#pragma unroll
      for (uint32_t q = 0; q < 2; ++q) {
        const uint32_t t = q * 64 + lane;
        if (i0 + (t >> 1) < hi) dst[t] = stage[(t >> 1) * kPrepRow + (t & 1)];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#endif
  }
  }
}


// ---- the table ----------------------------------------------------------
struct Key {
  uint32_t src, dst;
  uint16_t sport, dport;
  uint8_t proto;
};

// A connection's value (ct_v) while a walking lane owns it, in registers.
// Everything below passes values, never addresses of locals, so the lane's
// state stays in VGPRs (an address-taken local would live in scratch).
struct Ent {
  unsigned long long ttl;
  uint32_t seq;
  uint8_t state, rev, live;
};

// A slot is two 16-byte halves: {tag, src, dst, sport | dport << 16} and
// {ttl, seq, proto | valid << 8 | state << 16 | rev << 24}; each is read or
// written with one access (field-by-field accesses were six dependent loads
// per probe).
__device__ __forceinline__ ct_u32x4 slot_half(const CtSlot *e, int h) {
  return reinterpret_cast<const ct_u32x4 *>(e)[h];
}
__device__ __forceinline__ Ent slot_value(const ct_u32x4 hi) {
  return Ent{static_cast<unsigned long long>(hi.y) << 32 | hi.x, hi.z, static_cast<uint8_t>(hi.w >> 16),
             static_cast<uint8_t>(hi.w >> 24), static_cast<uint8_t>((hi.w >> 8) & 0xff)};
}

__device__ __forceinline__ bool same(const Key &a, const Key &b) {
  return a.src == b.src && a.dst == b.dst && a.sport == b.sport && a.dport == b.dport && a.proto == b.proto;
}

// The slot holding `k` (live or deleted), or null; with claim, an empty slot
// is taken for it.  One lane owns each key in a launch, so a slot another
// lane is claiming (tag 2) never holds ours.  Also returns the slot's value
// (a claimed slot: not live), by value so the caller's copy stays in registers.
//
// The tag loads are relaxed: an agent-scope acquire on gfx950 invalidates the
// CU's L1 and the XCD's L2 after every probe (buffer_inv sc1), which cost the
// whole walk dearly under lookup-heavy traffic (millions of one-packet keys).
// Nothing here needs it: within a launch, a slot another lane publishes holds
// another key, and a slot's key half only ever goes from zeros to its key, so
// a stale read of it is zeros and can only mismatch -- except for the all-zero
// key (an ICMP error quoting proto 0 between 0.0.0.0 and itself), which takes
// the acquire and a re-read before it may match.  For the same reason the
// publishing store is relaxed (a release is an L2 write-back per insert).
// Earlier launches' slots are visible through the kernel boundary.
struct SlotRef {
  CtSlot *e;
  Ent v;
};
//
// A key lives within kMaxProbe slots of its home slot: an insert that finds
// no empty slot that close is refused (counted in stats[0], as for a full
// table), so a lookup stops there too.  Without the bound a nearly full
// table made every miss and insert scan up to the whole table, ~1 us per
// dependent probe.
#ifndef PCN_CT_SLOT1
#define PCN_CT_SLOT1 1
#endif
constexpr uint64_t kMaxProbe = 512;
__device__ SlotRef table_slot(const CtTable &t, const Key &k, bool claim) {
  const uint64_t mask = (uint64_t(1) << t.cap_log2) - 1;
  const uint64_t probes = mask < kMaxProbe ? mask + 1 : kMaxProbe;
  const bool zero_key = (k.src | k.dst | k.sport | k.dport | k.proto) == 0;
  uint64_t s = key_hash(k.src, k.dst, k.proto, k.sport, k.dport) >> 7;
  for (uint64_t probe = 0; probe < probes; ++probe, ++s) {
    CtSlot *e = &t.slots[s & mask];
#if PCN_CT_SLOT1
    // the whole slot in one round trip: the tag is the key half's first word
    // (a tag load, then the halves, was two dependent loads per probe -- the
    // head of every walking wave's and lane's first lookup)
    ct_u32x4 lo = slot_half(e, 0), hi = slot_half(e, 1);
    uint32_t tag = lo.x;
#else
    uint32_t tag = __hip_atomic_load(&e->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    if (tag == 0) {
      if (!claim) return SlotRef{nullptr, Ent{}};
      if (atomicCAS(&e->tag, 0u, 2u) == 0u) {
        e->src = k.src; e->dst = k.dst; e->sport = k.sport; e->dport = k.dport; e->proto = k.proto;
        e->valid = 0;
        __hip_atomic_store(&e->tag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return SlotRef{e, Ent{}};
      }
      tag = __hip_atomic_load(&e->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if PCN_CT_SLOT1
      if (tag == 1) { lo = slot_half(e, 0); hi = slot_half(e, 1); }   // published under us: read it again
#endif
    }
    if (tag != 1) continue;
#if PCN_CT_SLOT1
    if (zero_key) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      lo = slot_half(e, 0);
      hi = slot_half(e, 1);
    }
#else
    if (zero_key) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const ct_u32x4 lo = slot_half(e, 0), hi = slot_half(e, 1);
#endif
    if (lo.y == k.src && lo.z == k.dst && lo.w == (uint32_t(k.sport) | uint32_t(k.dport) << 16) &&
        (hi.w & 0xff) == k.proto)
      return SlotRef{e, slot_value(hi)};
  }
  if (claim) atomicAdd(&t.stats[0], 1ull);          // no free slot near home: the insert is lost
  return SlotRef{nullptr, Ent{}};
}

struct Cache {              // the key a walking lane last touched, its slot and value
  Key k;
  CtSlot *e;                // slot holding k (live or deleted), or null
  Ent v;
  bool valid, dirty;
  uint32_t touch;           // 1 + the batch index of the last packet after which k was live (0: none)
};

__device__ __forceinline__ void flush(const CtTable &t, Cache &c) {
  if (c.dirty && c.e) {     // the value half in one store (proto is the key's)
    ct_u32x4 hi;
    hi.x = static_cast<uint32_t>(c.v.ttl);
    hi.y = static_cast<uint32_t>(c.v.ttl >> 32);
    hi.z = c.v.seq;
    hi.w = uint32_t(c.k.proto) | uint32_t(c.v.live) << 8 | uint32_t(c.v.state) << 16 | uint32_t(c.v.rev) << 24;
    reinterpret_cast<ct_u32x4 *>(c.e)[1] = hi;
  }
  // the LRU stamp: this batch's last touch, or ~0 once the entry is gone
  // (touch[] holds a stamp exactly for the live entries: the eviction reads nothing else)
  if (c.e) {
    if (c.v.live && c.touch) t.touch[c.e - t.slots] = static_cast<unsigned long long>(t.seq) << 32 | (c.touch - 1);
    else if (!c.v.live && c.dirty) t.touch[c.e - t.slots] = ~0ull;
  }
  c.dirty = false;
  c.touch = 0;
}

// connections.lookup: makes k the cached key; returns whether it is live (value in c.v).
__device__ __forceinline__ bool lookup(const CtTable &t, Cache &c, const Key &k) {
  if (!c.valid || !same(c.k, k)) {
    flush(t, c);
    c.k = k;
    const SlotRef r = table_slot(t, k, false);
    c.e = r.e;
    c.v = r.v;
    c.valid = true;
  }
  return c.v.live;
}

// connections.update (noexist = false) / .insert (BPF_NOEXIST) of the cached key
// kSpec: a wave's lane evaluating a record against a broadcast copy of the
// connection (walk_long): a put that would claim a slot clears c.valid instead.
template <bool kSpec = false>
__device__ __forceinline__ void put(const CtTable &t, Cache &c, unsigned long long ttl, uint8_t state, uint32_t seq,
                                   uint8_t rev, bool noexist) {
  if (c.v.live && noexist) return;
  if (!c.e) {
    if (kSpec) { c.valid = false; return; }
    c.e = table_slot(t, c.k, true).e;
    if (!c.e) return;
  }
  c.v = Ent{ttl, seq, state, rev, 1};
  c.dirty = true;
}

__device__ __forceinline__ bool syn_only(uint8_t f) { return (f & SYN) && (f | SYN) == SYN; }
__device__ __forceinline__ bool ack_only(uint8_t f) { return (f & ACK) && (f | ACK) == ACK; }
__device__ __forceinline__ bool synack_only(uint8_t f) {
  return (f & ACK) && (f & SYN) && (f | (SYN | ACK)) == (SYN | ACK);
}

// A long echo reply's quoted header (ConntrackLabel_dp.c:491-529), read
// without touching the walking lane's cache.  Only K_HARD records whose
// quoted key bucket holds no packet of the batch are walked (ct_hard_split),
// so nothing in this launch writes that key: the read is exact wherever in
// the walk it happens.
__device__ __forceinline__ bool quoted_live(const CtTable &t, const CtRec &r) {
  const Key q{r.seq, r.ack, static_cast<uint16_t>(r.iports & 0xffff), static_cast<uint16_t>(r.iports >> 16), r.flags};
  return table_slot(t, q, false).v.live;
}

// ConntrackLabel_dp.c:230-433 for TCP/UDP/echo/echo-replies/errors against the
// entry e (live or not); -1 = RX_DROP.
__device__ int label_of(const CtTable &t, const CtRec &r, bool live, const Ent &e) {
  const bool fwd = live && e.rev == r.rev;
  const bool rev = live && ((e.rev ^ r.rev) == 3);
  switch (r.kind) {
  case K_TCP:
    if (fwd || rev) {
      if (r.flags & RST) return ST_EST;
      const uint8_t s = e.state;
      if (s == ST_SYN_SENT)
        return fwd ? (syn_only(r.flags) ? ST_NEW : ST_INV) : (synack_only(r.flags) && r.ack == e.seq ? ST_EST : ST_INV);
      if (s == ST_SYN_RECV)
        return fwd ? (ack_only(r.flags) && r.ack == e.seq ? ST_EST : ST_INV)
                   : (synack_only(r.flags) && r.ack == e.seq ? ST_EST : ST_INV);
      if (s == ST_EST || s == ST_FIN_WAIT_1 || s == ST_FIN_WAIT_2 || s == ST_LAST_ACK) return ST_EST;
      if (s == ST_TIME_WAIT && syn_only(r.flags)) return ST_NEW;
      return ST_INV;
    }
    return syn_only(r.flags) ? ST_NEW : ST_INV;
  case K_UDP:
    if (fwd) return e.state == ST_NEW ? ST_NEW : ST_EST;
    if (rev) return ST_EST;
    return ST_NEW;
  case K_ECHO:
    return ST_NEW;
  case K_REPLY:                                   // < 70 bytes: the miss path drops
    if (!live) return ST_INV;
    return rev ? ST_EST : -1;
  case K_HARD:                                    // >= 70 bytes: ICMP_MISS reads the quoted header
    if (!live) return ST_INV;
    return rev ? ST_EST : quoted_live(t, r) ? ST_REL : ST_INV;
  case K_ERR:
    return live ? ST_REL : ST_INV;
  default:
    return ST_INV;
  }
}

// ConntrackTableUpdate_dp.c:141-655 for an accepted packet with label l; the
// cached key is the packet's own.
template <bool kSpec = false>
__device__ __forceinline__ void update(const CtTable &t, Cache &c, const CtRec &r, int l) {
  if (l == ST_INV) return;
  const unsigned long long now = t.now;
  const bool live = c.v.live;
  Ent &e = c.v;
  if (live) c.dirty = true;
  if (r.kind == K_TCP) {
    if (r.flags & RST) return;
    const int dir = !live ? 0 : e.rev == r.rev ? 1 : ((e.rev ^ r.rev) == 3) ? 2 : 0;
    if (dir) {
      const uint8_t s = e.state;
      if (s == ST_SYN_SENT) {
        if (dir == 1) { if (syn_only(r.flags)) e.ttl = now + TCP_SYN_SENT_T; return; }
        if (synack_only(r.flags) && r.ack == e.seq) {
          e.state = ST_SYN_RECV; e.ttl = now + TCP_SYN_RECV_T; e.seq = r.seq + HEX_BE_ONE;
        }
        return;
      }
      if (s == ST_SYN_RECV) {
        if (dir == 1) {
          if (ack_only(r.flags) && r.ack == e.seq) { e.state = ST_EST; e.ttl = now + TCP_ESTABLISHED_T; }
        } else if (synack_only(r.flags) && r.ack == e.seq) {
          e.ttl = now + TCP_SYN_RECV_T;
        }
        return;
      }
      if (s == ST_EST) {
        if (r.flags & FIN) { e.state = ST_FIN_WAIT_1; e.ttl = now + TCP_FIN_WAIT_T; e.seq = r.ack; }
        else e.ttl = now + TCP_ESTABLISHED_T;
        return;
      }
      if (s == ST_FIN_WAIT_1 || s == ST_FIN_WAIT_2) {
        if (s == ST_FIN_WAIT_1) {
          if (!((r.flags & ACK) && r.seq == e.seq)) return;
          e.state = ST_FIN_WAIT_2;                 // no goto: falls into FIN_WAIT_2
        }
        if (r.flags & FIN) { e.state = ST_LAST_ACK; e.ttl = now + TCP_LAST_ACK_T; e.seq = r.ack; }
        else e.ttl = now + TCP_FIN_WAIT_T;
        return;
      }
      if (s == ST_LAST_ACK) {
        if ((r.flags & ACK) && r.seq == e.seq) e.state = ST_TIME_WAIT;
        e.ttl = now + TCP_LAST_ACK_T;
        return;
      }
      if (s != ST_TIME_WAIT || l != ST_NEW) return;   // TIME_WAIT + NEW: goto TCP_MISS
    }
    if (syn_only(r.flags)) put<kSpec>(t, c, now + TCP_SYN_SENT_T, ST_SYN_SENT, r.seq + HEX_BE_ONE, r.rev, false);
    return;
  }
  if (r.kind == K_UDP) {
    if (live && e.rev == r.rev) { e.ttl = now + (e.state == ST_NEW ? UDP_NEW_TIMEOUT : UDP_ESTABLISHED_TIMEOUT); return; }
    if (live && (e.rev ^ r.rev) == 3) {
      if (e.state == ST_NEW) { e.ttl = now + UDP_NEW_TIMEOUT; e.state = ST_EST; }
      else e.ttl = now + UDP_ESTABLISHED_TIMEOUT;
      return;
    }
    put<kSpec>(t, c, now + UDP_NEW_TIMEOUT, ST_NEW, 0, r.rev, true);
    return;
  }
  if (r.kind == K_ECHO) { put<kSpec>(t, c, now + ICMP_TIMEOUT, ST_NEW, 0, r.rev, true); return; }
  if (r.kind == K_REPLY || r.kind == K_HARD) {
    if (live) e.live = 0;                          // connections.delete
  }
}

// Outcome (rule id << 1 | verdict) of a labelled packet with label l (-1:
// dropped by ConntrackLabel), from its stage-A outcomes o0..o3 (per label).
__device__ __forceinline__ int32_t outcome(const CtBatch &b, int32_t o0, int32_t o1, int32_t o2, int32_t o3,
                                           const CtRec &r, int l) {
  const bool pass = r.cinfo & 4;
  const uint32_t chain = r.cinfo & 3;
  if (l < 0) return pass ? (o0 & ~1) : int32_t(PCN_IPT_RID_NOCHAIN) * 2;   // RX_DROP
  if (pass) return o0;
  if (((b.ae_mask >> chain) & 1) && l == ST_EST) return -3 * 2 + PCN_IPT_ACCEPT;
  if (b.nlab != 4) return o0;
  return l == 0 ? o0 : l == 1 ? o1 : l == 2 ? o2 : o3;
}

__device__ __forceinline__ int32_t process(const CtBatch &b, const CtTable &t, Cache &c, const WalkRec &w) {
  const CtRec &r = w.r;
  const bool live = lookup(t, c, Key{r.src, r.dst, r.sport, r.dport, r.proto});
  const int l = label_of(t, r, live, c.v);
  const int32_t o = outcome(b, w.o0, w.o1, w.o2, w.o3, r, l);
  if ((o & 1) == PCN_IPT_ACCEPT && l >= 0 && r.kind != K_ERR) update(t, c, r, l);
  return o;
}

// The common step of a long run, without the general label/update code: a
// TCP or UDP packet of the cached live connection, in its forward or reverse
// direction.  TCP only while ESTABLISHED and without FIN: label ESTABLISHED
// (label_of: RST or an established state), and an accepted packet refreshes
// the ttl unless it carries RST (update's ST_EST branch).  UDP: label_of's
// UDP_FORWARD / UDP_REVERSE and update's two live branches.  Returns false
// (nothing done) for anything else, which then takes process().
__device__ __forceinline__ bool fast_step(const CtBatch &b, const CtTable &t, Cache &c, const WalkRec &w,
                                          int32_t &o) {
  const CtRec &r = w.r;
  if (!c.valid || !c.v.live || (r.kind != K_TCP && r.kind != K_UDP)) return false;
  const bool fwd = c.v.rev == r.rev, rev = (c.v.rev ^ r.rev) == 3;
  if (!(fwd || rev) || !same(c.k, Key{r.src, r.dst, r.sport, r.dport, r.proto})) return false;
  if (r.kind == K_TCP) {
    if (c.v.state != ST_EST || (r.flags & FIN)) return false;
    o = outcome(b, w.o0, w.o1, w.o2, w.o3, r, ST_EST);
    if ((o & 1) == PCN_IPT_ACCEPT) {
      c.dirty = true;
      if (!(r.flags & RST)) c.v.ttl = t.now + TCP_ESTABLISHED_T;
    }
    return true;
  }
  const bool nw = c.v.state == ST_NEW;
  o = outcome(b, w.o0, w.o1, w.o2, w.o3, r, fwd && nw ? ST_NEW : ST_EST);
  if ((o & 1) == PCN_IPT_ACCEPT) {
    c.dirty = true;
    c.v.ttl = t.now + (nw ? UDP_NEW_TIMEOUT : UDP_ESTABLISHED_TIMEOUT);
    if (rev && nw) c.v.state = ST_EST;
  }
  return true;
}

__device__ __forceinline__ int32_t step(const CtBatch &b, const CtTable &t, Cache &c, const WalkRec &w) {
  int32_t o;
  if (!(PCN_CT_FAST && fast_step(b, t, c, w, o))) o = process(b, t, c, w);
  if (c.v.live && c.e) c.touch = w.idx + 1;        // the LRU touch (the cached key is the record's)
  return o;
}

// After the sort: walk records in sorted order (each walking lane then reads
// consecutive lines) and the list of run heads.
#ifndef PCN_CT_DBG_T
#define PCN_CT_DBG_T 0 // measurement builds only: per walk block, its entry / run start / first chunk / end clocks
#endif
#if PCN_CT_DBG_T
constexpr uint32_t kDbgWaves = 1u << 17;
__device__ unsigned long long g_walk_t[4 * kDbgWaves];
#endif
#ifndef PCN_CT_DBG
#define PCN_CT_DBG 0   // measurement builds only: walk_long prints its round counts for long runs
#endif
#ifndef PCN_CT_LONG_RUN
#define PCN_CT_LONG_RUN 128
#endif
constexpr uint64_t kLongRun = PCN_CT_LONG_RUN;   // a run at least this long gets a whole wave

// Run heads by length class, so a wave's lanes walk runs of about the same
// length (a wave takes as long as its longest run: with a million one-packet
// keys mixed in, 2^16 flows of ~256 packets were spread over 30 K waves
// instead of 1 K).  Class 0: >= kLongRun packets (one wave each); classes
// 1-4: [64, kLongRun), [8, 64), [2, 8), 1 (one lane each).  A class whose runs
// have at least L packets has at most n / L heads, which fixes its region of
// `heads` (kHeadsCap(n) entries in all).
constexpr uint32_t kRunClasses = 5;
__host__ __device__ constexpr uint64_t class_cap(uint64_t n, uint32_t c) {
  return c == 0 ? n / kLongRun + 1 : c == 1 ? n / 64 + 1 : c == 2 ? n / 8 + 1 : c == 3 ? n / 2 + 1 : n;
}
__host__ __device__ constexpr uint64_t class_off(uint64_t n, uint32_t c) {
  uint64_t off = 0;
  for (uint32_t k = 0; k < c; ++k) off += class_cap(n, k);
  return off;
}
__host__ __device__ constexpr uint64_t heads_cap(uint64_t n) { return class_off(n, kRunClasses); }


// The run heads of each class.  A workgroup stages a contiguous tile of
// `per` x kHeadsBlock sorted keys (plus the key before it and kLongRun
// after it) in LDS with coalesced loads, counts its heads per class,
// reserves its places with one global atomic per class, then classifies again
// from LDS and writes the heads (LDS atomics per wave and class).  Per-wave
// global atomics on the five counters serialised (2-6 ms a batch); reading
// the six keys of a classification from L2, twice, cost 95 us a 2^24 batch.
// Keys per thread: 16, or fewer (a multiple of 4) so that a smaller batch
// still gives every CU two workgroups.
#ifndef PCN_CT_SEG
#define PCN_CT_SEG 512   // records per segment (a power of two >= kLongRun); 0: no segments
#endif
constexpr uint64_t kSeg = PCN_CT_SEG;
static_assert(kSeg == 0 || (kSeg >= kLongRun && (kSeg & (kSeg - 1)) == 0), "PCN_CT_SEG");
// 1024 threads: every workgroup reserves its heads with one global atomic per
// class, and those land on five addresses (~12 ns apiece, serialised): 4,096
// workgroups of 256 threads a 2^24 batch spent most of ct_heads' 67 us there.
#ifndef PCN_CT_HEADS_BLOCK
#define PCN_CT_HEADS_BLOCK 1024
#endif
constexpr uint32_t kHeadsBlock = PCN_CT_HEADS_BLOCK;
static_assert(kSeg == 0 || (4 * uint64_t(kHeadsBlock)) % (kSeg ? kSeg : 1) == 0, "a heads tile starts at a cut");
#ifndef PCN_CT_HEADS_PER
#define PCN_CT_HEADS_PER 16
#endif
constexpr uint32_t kHeadsPer = PCN_CT_HEADS_PER;
inline uint32_t heads_per(uint64_t n, int num_cus) {
  const uint64_t p = (n / (uint64_t(kHeadsBlock) * 2 * num_cus) + 3) / 4 * 4;
  return static_cast<uint32_t>(p < 4 ? 4 : p > kHeadsPer ? kHeadsPer : p);
}
// Workgroup 0 also advances the carry (the ports the batch leaves to the
// next one, Q4): ct_prep's groups are all published by now, so a look-back
// from the batch end gives the ports of its last frame the Parser wrote them
// for, or the old carry.  (Two tail kernels and a memset did this, ~27 us a
// batch; ct_prep itself doing it put its parse window in scratch.)
__global__ __launch_bounds__(kHeadsBlock) void ct_heads_kernel(uint64_t n, const uint32_t *skeys, uint32_t *heads,
                                                               uint32_t *nheads, uint32_t sentinel, uint32_t per,
                                                               const unsigned long long *desc, uint32_t *carry,
                                                               uint32_t *cuts, uint32_t *ncuts, const uint32_t *nhard,
                                                               uint32_t *bm, uint64_t bm_words) {
  // the key-bucket bitmap of the long echo replies (ct_hbits_set,
  // ct_hard_split: both done) left zeroed for the next batch
  if (*nhard)
    for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w < bm_words;
         w += uint64_t(gridDim.x) * blockDim.x)
      bm[w] = 0;
  __shared__ uint32_t cnt[kRunClasses], base[kRunClasses];
  if (desc && blockIdx.x == 0 && threadIdx.x < 64) {   // (null: stage A advanced it)
    const uint32_t c = ports_lookback(desc, (n + 63) / 64, carry);
    if (threadIdx.x == 0) *carry = c;
  }
  __shared__ uint32_t tile[kHeadsPer * kHeadsBlock + kLongRun + 1];   // keys [lo - 1, lo + T + kLongRun)
  const uint32_t T = per * kHeadsBlock;
  const uint64_t lo = uint64_t(blockIdx.x) * T;
  if (threadIdx.x < kRunClasses) cnt[threadIdx.x] = 0;
  // tile[j] = key at q - 1 (never a key past the ends).  Every load of the
  // tile is issued before the first is used: unconditional (the index clamped
  // into the batch, the value masked after), where a conditional load per
  // iteration waited a memory round trip each (17 a workgroup).
  constexpr uint32_t kTileIt = (kHeadsPer * kHeadsBlock + kLongRun + 1 + kHeadsBlock - 1) / kHeadsBlock;
  uint32_t tv[kTileIt];
#pragma unroll
  for (uint32_t k = 0; k < kTileIt; ++k) {
    const uint64_t q = lo + threadIdx.x + k * kHeadsBlock;
    const uint64_t src = q >= 1 ? (q - 1 < n ? q - 1 : n - 1) : 0;
    tv[k] = skeys[src];
  }
#pragma unroll
  for (uint32_t k = 0; k < kTileIt; ++k) {
    const uint32_t j = threadIdx.x + k * kHeadsBlock;
    const uint64_t q = lo + j;
    if (j < T + kLongRun + 1) tile[j] = q >= 1 && q - 1 < n ? tv[k] : 0xffffffffu;
  }
  __syncthreads();
  // The tile's active cuts (the walk's cut_active: the run holds B - 1 and kSeg
  // records from B on) for the segment waves: rare, one atomic each.
  if (kSeg != 0 && threadIdx.x < T / (kSeg ? kSeg : 1)) {
    const uint64_t B = lo + uint64_t(threadIdx.x) * kSeg;
    if (B >= 1 && B + kSeg <= n) {
      const uint32_t r = static_cast<uint32_t>(B - lo);
      const uint32_t k = tile[r + 1];
      if (k != sentinel && tile[r] == k && skeys[B + kSeg - 1] == k)
        cuts[atomicAdd(ncuts, 1u)] = static_cast<uint32_t>(B / (kSeg ? kSeg : 1));
    }
  }
  // the class of tile position r (sorted position lo + r); kRunClasses: not a run head
  auto run_class_lds = [&](uint32_t r) -> uint32_t {
    const uint32_t k = tile[r + 1], km = tile[r];
    const uint32_t k1 = tile[r + 2], k7 = tile[r + 8], k63 = tile[r + 64], kl = tile[r + 1 + kLongRun];
    if (lo + r >= n || k == sentinel || km == k) return kRunClasses;
    return kl == k ? 0 : k63 == k ? 1 : k7 == k ? 2 : k1 == k ? 3 : 4;   // more than kLongRun / 63 / 7 / 1 packets
  };
  // each position's class (3 bits) kept for the second pass, which re-read
  // the six keys of every position from LDS
  uint32_t mine[kRunClasses] = {};
  uint64_t cls = 0;
#pragma unroll
  for (uint32_t j = 0; j < kHeadsPer; ++j) {
    if (j >= per) break;
    const uint32_t c = run_class_lds(j * kHeadsBlock + threadIdx.x);
    cls |= uint64_t(c) << (3 * j);
#pragma unroll
    for (uint32_t k = 0; k < kRunClasses; ++k) mine[k] += c == k;
  }
#pragma unroll
  for (uint32_t k = 0; k < kRunClasses; ++k)
    if (mine[k]) atomicAdd(&cnt[k], mine[k]);
  __syncthreads();
  if (threadIdx.x < kRunClasses) {
    base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(&nheads[threadIdx.x], cnt[threadIdx.x]) : 0u;
    cnt[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint32_t lane = __lane_id();
#pragma unroll
  for (uint32_t it = 0; it < kHeadsPer; ++it) {
    if (it >= per) break;                            // (per: uniform)
    const uint32_t r = it * kHeadsBlock + threadIdx.x;
    const uint64_t q = lo + r;
    const uint32_t c = static_cast<uint32_t>(cls >> (3 * it)) & 7u;
#pragma unroll
    for (uint32_t k = 0; k < kRunClasses; ++k) {
      const uint64_t m = __ballot(c == k);
      if (!m) continue;
      const uint32_t leader = static_cast<uint32_t>(__builtin_ctzll(m));
      uint32_t at = 0;
      if (lane == leader) at = atomicAdd(&cnt[k], static_cast<uint32_t>(__popcll(m)));
      at = __shfl(at, static_cast<int>(leader));
      if (c == k) heads[class_off(n, k) + base[k] + at + __popcll(m & ((1ull << lane) - 1))] = static_cast<uint32_t>(q);
    }
  }
}

// One lane per run of equal key buckets, in batch order, over the packets with
// index < hi it has not done yet.  The lane keeps its connection in registers
// and its next two records in flight.  The walk's time is the longest run
// (the heaviest flow of the batch) times the per-packet cost of one lane
// (~0.9 us measured: instruction-bound, the wave executes the union of its
// lanes' paths); 4 records in flight measured the same.
// A long run (one wave): the wave stages the run's next 64 records in LDS
// with one coalesced load while it walks the previous 64.  The walk of a
// chunk is parallel where the reference's order cannot matter: in a round,
// every lane takes its record's full label -> outcome -> update against the
// connection as it stands (lane 0's cache, broadcast).  The leading records
// that leave the connection as it is (an established flow's data, packets of
// a half-closed or deleted flow that change nothing, a ttl already set to the
// value they would set) all have their outcome at once.  The first record
// that changes the connection is also right (it saw the state before it) and
// its result becomes the cache; only a record that needs the table itself (a
// slot to claim, another key of the bucket) takes step() on lane 0.  The next
// round starts after that record, so a chunk costs one round per change.
// (The walk reads each record from batch order through the sorted index: a
// dependent load, but no gather pass into sorted order, which cost 0.4-0.6 ms
// a batch more than the walk saved.)
// A walked packet's outcome, by batch index.  ct_prep has already written
// every packet's label-0 outcome (coalesced), so a walk stores only the
// outcomes that differ from it (sparse): the scattered one-byte and four-byte
// stores by batch index cost the walk as much as its record gathers, and with
// rules that do not match on conntrack state nearly every outcome is the
// label-0 one.  A re-walk over a speculative segment stores them all (dense),
// since the speculation may have stored others.  (Writing sorted-order
// outcomes and scattering them in a pass of their own cost 0.3-0.4 ms more.)
__device__ __forceinline__ void put_outcome(const CtBatch &b, const WalkRec &w, int32_t o, bool dense) {
  if (dense || o != w.o0) {
    b.verdicts[w.idx] = static_cast<uint8_t>(o & 1);
    b.rule_ids[w.idx] = o >> 1;
  }
}

struct RecSrc {
  const PackedRec *rec;   // batch order
  const uint32_t *sidx;   // sorted position -> batch index
  const uint32_t *skeys;  // sorted position -> key bucket
  const ct_u32x4 *ox;     // the four stage-A outcomes per packet (lab4 only)
  uint32_t lab4;          // the batch has four labels (a chain with conntrack rules)
  // the record of batch index i at sorted position q
  __device__ __forceinline__ WalkRec load(uint32_t i, uint64_t q) const {
    WalkRec w;
    const PackedRec p = load_prec(&rec[i]);
    w.r = ct_rec(p);
    w.key = skeys[q];
    w.idx = i;
    w.o0 = p.o0;
    w.o1 = w.o2 = w.o3 = 0;
    if (lab4) {
      const ct_u32x4 v = ox[i];
      w.o1 = static_cast<int32_t>(v.y);
      w.o2 = static_cast<int32_t>(v.z);
      w.o3 = static_cast<int32_t>(v.w);
    }
    return w;
  }
  __device__ __forceinline__ WalkRec at(uint64_t q) const { return load(sidx[q], q); }
  __device__ __forceinline__ uint32_t key(uint64_t q) const { return skeys[q]; }
  // the batch index / key bucket at sorted position q, clamped into the batch (n >= 1)
  __device__ __forceinline__ uint32_t idx_at(uint64_t q, uint64_t n) const { return sidx[q < n ? q : n - 1]; }
  __device__ __forceinline__ uint32_t key_at(uint64_t q, uint64_t n) const { return skeys[q < n ? q : n - 1]; }
  // The record of batch index i at sorted position q (< n, key bucket kq) if
  // that is the run's key k; zeros, and no memory request, otherwise: the
  // index of a structured buffer load (stride 32, n records) is out of range
  // for the lanes past a run's end.  (Every run's last chunk, and the chunk
  // prefetched after it, fetched a 128-byte line per lane there: ~70 of the
  // ~250 records of a bench flow's run, a quarter of the walk's fills.)
  __device__ __forceinline__ WalkRec load_run(uint32_t i, uint32_t kq, uint32_t k, uint64_t q, uint64_t n) const {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<PackedRec *>(rec), 32, static_cast<uint32_t>(n), 0x00020000);
    const uint32_t vi = kq == k && q < n ? i : 0xFFFFFFFFu;
    union {
      ct_u32x4 v[2];
      PackedRec p;
    } u;
    u.v[0] = __builtin_bit_cast(ct_u32x4, ct_struct_load_v4(rs, static_cast<int>(vi), 0, 0, 0));
    u.v[1] = __builtin_bit_cast(ct_u32x4, ct_struct_load_v4(rs, static_cast<int>(vi), 16, 0, 0));
    WalkRec w;
    w.r = ct_rec(u.p);
    w.key = kq;
    w.idx = i;
    w.o0 = u.p.o0;
    w.o1 = w.o2 = w.o3 = 0;
    if (lab4) {
      const ct_u32x4 v = ox[i];
      w.o1 = static_cast<int32_t>(v.y);
      w.o2 = static_cast<int32_t>(v.z);
      w.o3 = static_cast<int32_t>(v.w);
    }
    return w;
  }
};

// The walk of one long run's records in chunks of 64, from sorted position q0
// up to `bound` (or the run's end, or the first record at batch index >= hi),
// with lane 0's cache `c` as the connection's state on entry and on return.
// Returns the sorted position where it stopped.  kSpec: a speculative segment
// (walk_seg): it may not touch the table, so where a record needs it (cls 2)
// the walk stops there and sets `aborted`.
// A lane's record, to every lane (one record of a chunk: the rare table step).
__device__ __forceinline__ WalkRec shfl_rec(const WalkRec &w, uint32_t from) {
  const int f = static_cast<int>(from);
  union {
    ct_u32x4 v[2];
    PackedRec p;
  } u;
  u.p = pack_rec(w.r, w.o0);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    u.v[q].x = __shfl(u.v[q].x, f);
    u.v[q].y = __shfl(u.v[q].y, f);
    u.v[q].z = __shfl(u.v[q].z, f);
    u.v[q].w = __shfl(u.v[q].w, f);
  }
  WalkRec x;
  x.r = ct_rec(u.p);
  x.key = __shfl(w.key, f);
  x.idx = __shfl(w.idx, f);
  x.o0 = u.p.o0;
  x.o1 = __shfl(w.o1, f);
  x.o2 = __shfl(w.o2, f);
  x.o3 = __shfl(w.o3, f);
  return x;
}

// The chunk a lane walks is its own record in registers, and the next chunk's
// record is in flight meanwhile (one load per lane).  (The first version staged
// chunks in LDS behind two workgroup barriers each, whose release waited for
// the chunk's scattered outcome stores.)
// A run is one key *bucket*, and a bucket can hold several connections (25-bit
// buckets: ~64 colliding pairs among 2^16 flows).  Walked as one sequence, two
// interleaved connections made every other record a table step on lane 0
// (flush, probe, ~1.5 us each): a 500-record run of two flows took up to 0.8
// ms, the whole walk's tail.  The connections of a bucket are independent, so
// the head wave walks them one after the other instead: pass j takes the
// records of the j-th connection to appear in the run (its key in `PassKeys`,
// LDS) and skips the others, noting the first record of a connection it has
// not seen; past kPassKeys connections the last pass takes all the rest as one
// sequence (the old way).  kAllKeys: every record (segments, and the runs
// whose walk a segment continues).
constexpr int kPassKeys = 4;
constexpr int kAllKeys = -2, kOtherKeys = -1;
// How often walk_long went past its first pass: [0] passes for a bucket's 2nd..
// kPassKeys-th connection, [1] "the rest as one sequence" walks.  Only bucket
// collisions get there (a global atomic each, ~64 a batch on the bench
// traffic); read by the tests through pcn_ipt_debug_ct_walk_passes to see that
// the path they mean to cover ran.  One pair per DEVICE, not per context: two
// contexts on one device add into the same counters (a test reads them with a
// single context).
__device__ unsigned long long g_walk_passes[2];
struct PassKeys {
  uint32_t n;
  uint32_t k[kPassKeys][4];   // src, dst, sport | dport << 16, proto
};
__device__ __forceinline__ void pass_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// i0, k0, i1, k1: the batch indices and key buckets of the first two chunks
// (sorted positions q0 + lane and q0 + 64 + lane, clamped), loaded by the
// caller: a long run's head wave issues them with the run's key and cut
// probes, one round trip for all.  Each chunk's indices and keys are loaded a
// chunk ahead of its records, so that only the run's lanes fetch a record.
template <bool kSpec>
__device__ __forceinline__ uint64_t walk_chunks(const CtBatch &b, const CtTable &t, const RecSrc &wrec,
                                                uint32_t k, uint64_t q0, uint32_t i0, uint32_t k0, uint32_t i1,
                                                uint32_t k1, uint64_t hi,
                                                uint64_t bound, Cache &c, bool &aborted, bool dense = false,
                                                uint64_t *tfirst = nullptr, PassKeys *pk = nullptr,
                                                int pass = kAllKeys, uint64_t *unk = nullptr) {
  (void)tfirst;                                     // (measurement builds only)
  const uint32_t lane = threadIdx.x;
  const uint64_t lim = bound < b.n ? bound : b.n;
  uint64_t base = q0;
  aborted = false;
  WalkRec w = wrec.load_run(i0, k0, k, base + lane, b.n);
  uint32_t nidx = i1, nkey = k1;                    // the next chunk's indices and keys, a chunk ahead
#if PCN_CT_DBG
  uint32_t dbg_chunks = 0, dbg_rounds = 0, dbg_changes = 0, dbg_steps = 0, dbg_recs = 0;
  const uint64_t dbg_t0 = wall_clock64();
#endif
  for (;;) {
    const WalkRec nx = wrec.load_run(nidx, nkey, k, base + 64 + lane, b.n);
    nidx = wrec.idx_at(base + 128 + lane, b.n);
    nkey = wrec.key_at(base + 128 + lane, b.n);
    const CtRec &r = w.r;
    const bool inrun = base + lane < lim && w.key == k && w.idx < hi;
    const uint64_t rm = __ballot(inrun);           // the run's records: a prefix of the chunk
    const uint32_t m = rm == ~0ull ? 64u : static_cast<uint32_t>(__builtin_ctzll(~rm));
    uint32_t u0 = 0;
    bool part = true;                               // this lane's record belongs to the pass
    if (pass != kAllKeys) {
      const uint32_t rp = uint32_t(r.sport) | uint32_t(r.dport) << 16;
      if (pk->n == 0) {                             // the pass-0 connection: the run's first record
        if (lane == 0) {
          pk->k[0][0] = r.src;
          pk->k[0][1] = r.dst;
          pk->k[0][2] = rp;
          pk->k[0][3] = r.proto;
          pk->n = 1;
        }
        pass_fence();
      }
      const uint32_t nk = pk->n;
      int kid = -1;
#pragma unroll
      for (int j = 0; j < kPassKeys; ++j)
        if (j < static_cast<int>(nk) && r.src == pk->k[j][0] && r.dst == pk->k[j][1] && rp == pk->k[j][2] &&
            r.proto == pk->k[j][3])
          kid = j;
      part = pass >= 0 ? kid == pass : kid < 0;
      if (pass >= 0 && *unk == ~0ull) {
        const uint64_t um = __ballot(lane < m && kid < 0);
        if (um) *unk = base + __builtin_ctzll(um);
      }
    }
#if PCN_CT_DBG
    ++dbg_chunks;
    dbg_recs += m;
#endif
    while (u0 < m) {
#if PCN_CT_DBG
      ++dbg_rounds;
#endif
      // lane 0's cached connection, to every lane
      const uint32_t sv = __shfl(c.valid ? 1u | (c.v.live ? 2u : 0u) | (c.e ? 4u : 0u) : 0u, 0);
      const uint32_t ks = __shfl(c.k.src, 0), kd = __shfl(c.k.dst, 0);
      const uint32_t kp = __shfl(uint32_t(c.k.sport) | uint32_t(c.k.dport) << 16, 0);
      const uint32_t kx = __shfl(uint32_t(c.k.proto) | uint32_t(c.v.state) << 8 | uint32_t(c.v.rev) << 16, 0);
      const uint32_t tl = __shfl(static_cast<uint32_t>(c.v.ttl), 0), th = __shfl(static_cast<uint32_t>(c.v.ttl >> 32), 0);
      const uint32_t sq = __shfl(c.v.seq, 0);
      // every lane of the round: the full label -> outcome -> update of its
      // record against that state, on a private copy.  cls 0: leaves the
      // connection as it is (the ttl it sets is the one it has); 1: changes it
      // (the round's last record: the next round starts from its result);
      // 2: needs the table itself (another key of the bucket, a slot to claim,
      // no cached key yet) and takes step() on lane 0.
      int cls = part ? 2 : 0;                      // another connection's record: nothing to do here
      int32_t o = 0;
      Cache cc{};
      if (part && lane >= u0 && lane < m && (sv & 1) && r.src == ks && r.dst == kd &&
          (uint32_t(r.sport) | uint32_t(r.dport) << 16) == kp && r.proto == (kx & 0xff)) {
        cc.k = Key{ks, kd, static_cast<uint16_t>(kp), static_cast<uint16_t>(kp >> 16), static_cast<uint8_t>(kx)};
        cc.e = (sv & 4) ? t.slots : nullptr;          // never dereferenced under kSpec
        cc.v = Ent{uint64_t(th) << 32 | tl, sq, static_cast<uint8_t>(kx >> 8), static_cast<uint8_t>(kx >> 16),
                   static_cast<uint8_t>((sv >> 1) & 1)};
        cc.valid = true;
        cc.dirty = false;
        const int l = label_of(t, r, cc.v.live, cc.v);
        o = outcome(b, w.o0, w.o1, w.o2, w.o3, r, l);
        if ((o & 1) == PCN_IPT_ACCEPT && l >= 0 && r.kind != K_ERR) update<true>(t, cc, r, l);
        cls = !cc.valid ? 2
              : (cc.v.ttl == (uint64_t(th) << 32 | tl) && cc.v.seq == sq && cc.v.state == ((kx >> 8) & 0xff) &&
                 cc.v.rev == ((kx >> 16) & 0xff) && cc.v.live == ((sv >> 1) & 1))
                  ? 0 : 1;
      }
      const uint64_t em = __ballot(cls == 0) >> u0;
      const uint32_t cnt = em == ~0ull >> u0 ? 64u - u0 : static_cast<uint32_t>(__builtin_ctzll(~em));
      const uint32_t end = u0 + cnt < m ? u0 + cnt : m;
      const bool mine = lane >= u0 && lane < end;
      if (mine && part) put_outcome(b, w, o, dense);
      const bool anyd = __ballot(mine && cls == 0 && cc.dirty) != 0;
      if (lane == 0 && anyd) c.dirty = true;
      // the LRU touch: records that leave the connection as it is touch it if it is live
      const uint64_t rng = end > u0 ? (end == 64 ? ~0ull : (1ull << end) - 1) & ~((1ull << u0) - 1) : 0ull;
      const uint64_t pm = __ballot(part) & rng;      // the last of them that is the pass's
      const uint32_t lidx = __shfl(w.idx, pm ? 63 - __builtin_clzll(pm) : u0);
      if (lane == 0 && pm && (sv & 2)) c.touch = lidx + 1;
      u0 = end;
      if (u0 < m) {
        const int ecls = __shfl(cls, u0);
#if PCN_CT_DBG
        if (ecls == 1) ++dbg_changes; else ++dbg_steps;
#endif
        if (ecls == 1) {                              // the changing record: its result is the new state
          if (lane == u0) put_outcome(b, w, o, dense);
          const uint32_t nl = __shfl(static_cast<uint32_t>(cc.v.ttl), u0);
          const uint32_t nh = __shfl(static_cast<uint32_t>(cc.v.ttl >> 32), u0);
          const uint32_t ns = __shfl(cc.v.seq, u0);
          const uint32_t nf = __shfl(uint32_t(cc.v.state) | uint32_t(cc.v.rev) << 8 | uint32_t(cc.v.live) << 16 |
                                         uint32_t(cc.dirty) << 24, u0);
          const uint32_t cidx = __shfl(w.idx, u0);
          if (lane == 0) {
            c.v = Ent{uint64_t(nh) << 32 | nl, ns, static_cast<uint8_t>(nf), static_cast<uint8_t>(nf >> 8),
                      static_cast<uint8_t>(nf >> 16)};
            if (nf >> 24) c.dirty = true;
            if (c.v.live && c.e) c.touch = cidx + 1;
          }
        } else if (kSpec) {                           // the table is not ours to touch: give up here
          aborted = true;
          return base + u0;
        } else {                                      // the record that needs the table: the full step
          const WalkRec x = shfl_rec(w, u0);
          if (lane == 0) put_outcome(b, x, step(b, t, c, x), dense);
        }
        ++u0;
      }
    }
#if PCN_CT_DBG_T
    if (tfirst && !*tfirst) *tfirst = wall_clock64();
#endif
    if (m < 64) {                                     // the run (or this part of it) ends here
#if PCN_CT_DBG
      if (lane == 0 && (dbg_chunks >= 40 || (q0 & 4095) < 64))   // the long ones, and a sample
        printf("walk_long run: %u records, %u chunks, %u rounds, %u changes, %u table steps, %llu us\n", dbg_recs,
               dbg_chunks, dbg_rounds, dbg_changes, dbg_steps, (unsigned long long)((wall_clock64() - dbg_t0) / 100));
#endif
      return base + m;
    }
    base += 64;
    w = nx;
  }
}

// ---- speculative segments of long runs --------------------------------------
// The walk of a long run is sequential in its records, ~14 us per chunk of
// 64: the heaviest run of a batch (thousands of packets of one key) bounded
// the whole walk.  So a run is cut at the sorted positions B that are
// multiples of kSeg and have at least kSeg of its records from B on ("active"
// cuts: a run's active cuts are consecutive from its first cut, and its last
// segment holds kSeg to 2 kSeg - 1 records).  Runs of ordinary flows (a few
// hundred packets) are never cut.  The head wave walks up to the first active
// cut; every later segment is walked at the same time by a wave of its own
// (walk_seg) that takes as its entry state the key's entry as the table holds
// it at the start of the batch (nothing else writes that key in this launch),
// with the ttl unknown (kTtlUnset: a ttl, once set, is now + a constant,
// never read).  It writes its outcomes and its exit state but nothing to the
// table, and stops (aborted) at the first record that would need the table.
// ct_seg_fix then chains the segments in order: a segment whose entry guess
// equals the state its predecessor actually left is right as walked (the walk
// reads nothing else: the ttl is never compared, a long echo reply's quoted
// key is not written in the batch), and its exit becomes the state; any other
// segment is walked again from the true state, its outcomes overwritten.  A
// key that keeps its state through the batch has every guess hold; a
// connection opened or closed mid-run costs re-walked segments from there on.
// (kSeg, the records per speculative segment: below, with walk_seg)
constexpr unsigned long long kTtlUnset = ~0ull;
__host__ __device__ constexpr uint64_t seg_count(uint64_t n) { return kSeg ? n / (kSeg ? kSeg : 1) + 1 : 0; }
// Waves for the active cuts (walk_seg, ct_seg_fix), each taking every
// seg_waves-th: a wave per cut, active or not (32 K at 2^24, nearly all with
// nothing to do), cost the walk 12 us a batch.  The count is fixed before
// ct_heads has counted the active cuts (no read-back), so it is sized for the
// worst case the device can run at once, PCN_CT_SEG_WAVES_PER_CU per CU (a
// batch of one long connection has a cut every kSeg records: 32 K at 2^24),
// and waves without a cut return at once.
#ifndef PCN_CT_SEG_WAVES_PER_CU
#define PCN_CT_SEG_WAVES_PER_CU 4
#endif
__host__ __device__ constexpr uint32_t seg_waves(uint64_t n, int num_cus) {
  return static_cast<uint32_t>(seg_count(n) < uint64_t(num_cus) * PCN_CT_SEG_WAVES_PER_CU
                                   ? seg_count(n) : uint64_t(num_cus) * PCN_CT_SEG_WAVES_PER_CU);
}

struct alignas(16) SegRec {       // 64 bytes, one per cut j (sorted position j * kSeg)
  uint32_t src, dst, ports, gx;   // the guess: key, proto | state << 8 | rev << 16 | live << 24
  uint32_t gseq, gslot;           //            seq, slot index (~0: none)
  uint32_t ttl_lo, ttl_hi;        // the exit: ttl (kTtlUnset: none set), seq,
  uint32_t xseq, xx;              //           state | rev << 8 | live << 16 | dirty << 24
  uint32_t touch, stop, status;   // LRU touch, where the walk stopped, 0 none / 1 walked / 2 aborted
  uint32_t pad[3];
};
struct alignas(16) HeadExit {     // the head wave's state at its run's first cut
  uint32_t src, dst, ports, px;   // px: proto | state << 8 | rev << 16 | live << 24
  uint32_t ttl_lo, ttl_hi, seq, slot;
  uint32_t flags, touch, vb;      // flags: valid | dirty << 1
  uint32_t pad[5];
};

// Cut B is active for the run of key bucket k: the run holds B - 1 and at
// least kSeg records from B on (sorted keys are contiguous, so two probes).
__device__ __forceinline__ bool cut_active(const uint32_t *skeys, uint64_t n, uint64_t B, uint32_t k) {
  return B >= 1 && B + kSeg <= n && skeys[B - 1] == k && skeys[B + kSeg - 1] == k;
}

__device__ __forceinline__ uint32_t cache_px(const Cache &c) {
  return uint32_t(c.k.proto) | uint32_t(c.v.state) << 8 | uint32_t(c.v.rev) << 16 | uint32_t(c.v.live) << 24;
}

// A long run's head wave: from its head (first) or its cursor up to hi.  With
// segments, the first pass stops at the run's first cut if that is active; if
// the walk gets there, the state is left to ct_seg_fix (no flush, no cursor).
__device__ void walk_long(const CtBatch &b, const CtTable &t, const RecSrc &wrec,
                          uint32_t p, uint32_t *cursor, uint32_t vb, uint64_t hi, int first, HeadExit *hx) {
  // One round trip for the run's key, its first cut's two probes and the
  // first two chunks' batch indices: every load unconditional (indices
  // clamped), where the cut's short-circuit test and the key before the
  // indices made four dependent ones ahead of the first record.
  const uint32_t lane = threadIdx.x;
  const uint64_t last = b.n - 1;
  const uint64_t q0 = first ? p : cursor[vb];
  const uint32_t k = wrec.key(p);
  const uint64_t B1 = kSeg ? (p / (kSeg ? kSeg : 1) + 1) * kSeg : 0;
  // (wrec's sorted keys: ct_tail passes no skeys)
  const uint32_t kb = wrec.key(B1 - 1 < last ? B1 - 1 : last), ke = wrec.key(B1 + kSeg - 1 < last ? B1 + kSeg - 1 : last);
  uint32_t i0 = wrec.idx_at(q0 + lane, b.n), i1 = wrec.idx_at(q0 + 64 + lane, b.n);
  uint32_t k0 = wrec.key_at(q0 + lane, b.n), k1 = wrec.key_at(q0 + 64 + lane, b.n);
  // cut B1 is active (cut_active): the run holds B1 - 1 and kSeg records from B1 on
  const uint64_t bound = first != 0 && kSeg != 0 && B1 + kSeg <= b.n && kb == k && ke == k ? B1 : ~0ull;
  Cache c{};
  bool ab;
  __shared__ PassKeys pk;
  const bool passes = bound == ~0ull;               // no segment continues this walk
  if (passes) {
    if (threadIdx.x == 0) pk.n = 0;
    pass_fence();
  }
  uint64_t unk = ~0ull;
  // pass 0, then the bucket's other connections, one pass each from their
  // first record (one call site: each inlined copy of the walk costs registers)
  uint64_t stop = 0, from = q0;
  int pass = passes ? 0 : kAllKeys;
#if PCN_CT_DBG_T
  const uint64_t dt0 = wall_clock64();
  uint64_t dt1 = 0;
#endif
  for (;;) {
#if PCN_CT_DBG_T
    const uint64_t st = walk_chunks<false>(b, t, wrec, k, from, i0, k0, i1, k1, hi, bound, c, ab, false, &dt1, &pk, pass,
                                           &unk);
#else
    const uint64_t st = walk_chunks<false>(b, t, wrec, k, from, i0, k0, i1, k1, hi, bound, c, ab, false, nullptr, &pk,
                                           pass, &unk);
#endif
    if (from == q0) stop = st;                       // every pass stops there (the run's end, or hi)
    if (unk == ~0ull) break;
    from = unk;
    unk = ~0ull;
    i0 = wrec.idx_at(from + lane, b.n);
    i1 = wrec.idx_at(from + 64 + lane, b.n);
    k0 = wrec.key_at(from + lane, b.n);
    k1 = wrec.key_at(from + 64 + lane, b.n);
    if (++pass < kPassKeys) {
      const WalkRec x = wrec.at(from);
      if (threadIdx.x == 0) {
        atomicAdd(&g_walk_passes[0], 1ull);
        pk.k[pass][0] = x.r.src;
        pk.k[pass][1] = x.r.dst;
        pk.k[pass][2] = uint32_t(x.r.sport) | uint32_t(x.r.dport) << 16;
        pk.k[pass][3] = x.r.proto;
        pk.n = pass + 1;
      }
      pass_fence();
    } else {
      pass = kOtherKeys;                            // the rest as one sequence (sets no unk)
      if (threadIdx.x == 0) atomicAdd(&g_walk_passes[1], 1ull);
    }
  }
#if PCN_CT_DBG_T
  if (threadIdx.x == 0 && vb < kDbgWaves) {
    g_walk_t[4 * vb + 1] = dt0;
    g_walk_t[4 * vb + 2] = dt1;
    g_walk_t[4 * vb + 3] = wall_clock64() | (stop - q0) << 48;
  }
#endif
  bool cont = false;
  if (stop == bound) {                           // (an active cut: the key goes on there)
    cont = wrec.sidx[bound] < hi;
  }
  if (threadIdx.x != 0) return;
  if (cont) {
    HeadExit h{};
    h.src = c.k.src;
    h.dst = c.k.dst;
    h.ports = uint32_t(c.k.sport) | uint32_t(c.k.dport) << 16;
    h.px = cache_px(c);
    h.ttl_lo = static_cast<uint32_t>(c.v.ttl);
    h.ttl_hi = static_cast<uint32_t>(c.v.ttl >> 32);
    h.seq = c.v.seq;
    h.slot = c.e ? static_cast<uint32_t>(c.e - t.slots) : ~0u;
    h.flags = uint32_t(c.valid) | uint32_t(c.dirty) << 1;
    h.touch = c.touch;
    h.vb = vb;
    hx[bound / kSeg] = h;
  } else {
    flush(t, c);
    cursor[vb] = static_cast<uint32_t>(stop);
  }
}

// Cut j: if it is active for the run across sorted position B = j * kSeg,
// walk that run's records from B speculatively, up to the next cut if that is
// active too, else to the run's end.  Every cut writes its status.
__device__ __forceinline__ void walk_seg(const CtBatch &b, const CtTable &t, const RecSrc &wrec,
                                         const uint32_t *skeys, uint32_t sentinel, SegRec *seg,
                                         uint32_t j, uint64_t hi) {
  const uint32_t lane = threadIdx.x;
  const uint64_t B = uint64_t(j) * kSeg;
  const uint32_t k = B < b.n ? skeys[B] : sentinel;
  bool ok = k != sentinel && cut_active(skeys, b.n, B, k);
  const WalkRec x = wrec.at(ok ? B : 0);
  ok = ok && x.idx < hi;
  if (!ok) {
    if (lane == 0) seg[j].status = 0;
    return;
  }
  const Key gk{x.r.src, x.r.dst, x.r.sport, x.r.dport, x.r.proto};
  const SlotRef g = table_slot(t, gk, false);     // the key's entry as the batch found it
  Cache c{};
  c.k = gk;
  c.e = g.e;
  c.v = g.v;
  c.v.ttl = kTtlUnset;
  c.valid = true;
  bool ab;
  const uint64_t bound = cut_active(skeys, b.n, B + kSeg, k) ? B + kSeg : ~0ull;
  const uint64_t stop = walk_chunks<true>(b, t, wrec, k, B, wrec.idx_at(B + lane, b.n), wrec.key_at(B + lane, b.n),
                                          wrec.idx_at(B + 64 + lane, b.n), wrec.key_at(B + 64 + lane, b.n), hi, bound, c,
                                          ab);
  if (lane != 0) return;
  SegRec s{};
  s.src = gk.src;
  s.dst = gk.dst;
  s.ports = uint32_t(gk.sport) | uint32_t(gk.dport) << 16;
  s.gx = uint32_t(gk.proto) | uint32_t(g.v.state) << 8 | uint32_t(g.v.rev) << 16 | uint32_t(g.v.live) << 24;
  s.gseq = g.v.seq;
  s.gslot = g.e ? static_cast<uint32_t>(g.e - t.slots) : ~0u;
  s.ttl_lo = static_cast<uint32_t>(c.v.ttl);
  s.ttl_hi = static_cast<uint32_t>(c.v.ttl >> 32);
  s.xseq = c.v.seq;
  s.xx = uint32_t(c.v.state) | uint32_t(c.v.rev) << 8 | uint32_t(c.v.live) << 16 | uint32_t(c.dirty) << 24;
  s.touch = c.touch;
  s.stop = static_cast<uint32_t>(stop);
  s.status = ab ? 2u : 1u;
  seg[j] = s;
}

struct WalkPlan {
  uint32_t cnt[kRunClasses];       // runs per class
  uint32_t blk0[kRunClasses + 1];  // first virtual block of each class
};

// The batch's control words (CtScratch::ctl, u32), all on the device: the walk
// is planned and sized there, so ct_run never reads anything back (the stream
// stays asynchronous).
constexpr uint32_t kCtlHard = 0;      // long echo replies (K_HARD) in hard_list
constexpr uint32_t kCtlClass = 1;     // [1..5] runs per length class (ct_heads)
constexpr uint32_t kCtlSegN = 6;      // active cuts in CtScratch::cuts (ct_heads)
constexpr uint32_t kCtlChunk = 8;     // ct_prep's chunk counter
constexpr uint32_t kCtlTh = 9;        // K_HARD records the walk cannot take (th_list)
constexpr uint32_t kCtlThFirst = 10;  // 0xFFFFFFFF - the first of them (0: none)
constexpr uint32_t kCtlLive = 12;     // LRU: live entries after the batch (ct_ev_pass 0)
constexpr uint32_t kCtlEvict = 13;    //      1 when more than max_entries are live
constexpr uint32_t kCtlEvK = 14;      //      rank (1-based) of the newest stamp to evict, within the prefix
constexpr uint32_t kCtlEvDone = 15;   //      workgroups done with the current pass
constexpr uint32_t kCtlEvPrefix = 28; // u64: the stamp digits chosen so far
constexpr uint32_t kCtlEvLow = 30;    //      the stamp bits below this one are still to choose
constexpr uint32_t kCtlEvNotMin = 32; //      u64: ~(the oldest live stamp) (a max, so zero-initialised)
constexpr uint32_t kCtlEvMax = 34;    //      u64: the newest live stamp
constexpr uint32_t kCtlZero = 36;     // words zeroed per batch
constexpr uint32_t kCtlWords = 64;

// The walk plan from ct_heads' class counts, computed where it is used (a
// kernel of its own, ct_plan, was a launch of ~5 us a batch): in registers,
// indexed only by constants (a local copy indexed by class went to scratch).
__device__ __forceinline__ WalkPlan plan_of(const uint32_t *ctl) {
  WalkPlan plan;
  uint32_t b0 = 0;
#pragma unroll
  for (uint32_t c = 0; c < kRunClasses; ++c) {
    const uint32_t cnt = ctl[kCtlClass + c];
    plan.cnt[c] = cnt;
    plan.blk0[c] = b0;
    b0 += c == 0 ? cnt : (cnt + 63) / 64;      // one wave per long run, one lane per shorter run
  }
  plan.blk0[kRunClasses] = b0;
  return plan;
}

__device__ __forceinline__ uint64_t walk_hi(const CtBatch &b, const uint32_t *ctl) {
  const uint32_t th = ctl[kCtlThFirst];
  return th ? uint64_t(0xFFFFFFFFu - th) : b.n;
}

// Virtual block vb of the plan (one 64-lane wave): a long run, or up to 64
// shorter runs of one class, one per lane, each from its head (first) or its
// cursor up to batch index hi.  Every lane returns here (no early exit), so a
// persistent wave can take the next block.
// head: heads[vb] (class 0's heads come first), loaded by the caller ahead of
// the plan's words.
__device__ void walk_vb(const CtBatch &b, const CtTable &t, const RecSrc &wrec,
                        const uint32_t *heads, const WalkPlan &plan, uint32_t *cursor, uint64_t hi, int first,
                        uint32_t vb, uint32_t head, HeadExit *hx) {
  const uint32_t b1 = plan.blk0[1];
  if (vb < b1) {                                  // one wave per long run
    walk_long(b, t, wrec, head, cursor, vb, hi, first, hx);
    return;
  }
  // the block's class, its first block and run count from the plan's words
  // read at once (a search reading one word a step was a round trip each)
  static_assert(kRunClasses == 5, "walk_vb's class selection");
  const uint32_t b2 = plan.blk0[2], b3 = plan.blk0[3], b4 = plan.blk0[4];
  const uint32_t c1 = plan.cnt[1], c2 = plan.cnt[2], c3 = plan.cnt[3], c4 = plan.cnt[4];
  const uint32_t cls = 1u + (vb >= b2 ? 1u : 0u) + (vb >= b3 ? 1u : 0u) + (vb >= b4 ? 1u : 0u);
  const uint32_t blk = cls == 1 ? b1 : cls == 2 ? b2 : cls == 3 ? b3 : b4;
  const uint32_t cnt = cls == 1 ? c1 : cls == 2 ? c2 : cls == 3 ? c3 : c4;
  const uint32_t jj = (vb - blk) * 64 + threadIdx.x;
  if (jj < cnt) {
    const uint64_t j = class_off(b.n, cls) + jj;
    const uint32_t p = heads[j];
    uint64_t q = first ? p : cursor[j];
    const uint64_t last = b.n - 1;
    Cache c{};
    // two records in flight in named registers, A/B alternating (a register
    // move of an in-flight load would wait for it), and the batch indices of
    // the two after them (the record loads never wait on an index load).
    // The key and all four indices are issued before any record: a record
    // issued between two index loads made the second one's wait cover it.
    auto cl = [&](uint64_t r) -> uint64_t { return r < last ? r : last; };
    const uint32_t k = wrec.key(p);
    const uint32_t iA = wrec.idx_at(q, b.n), iB = wrec.idx_at(q + 1, b.n);
    uint32_t IA = wrec.idx_at(q + 2, b.n), IB = wrec.idx_at(q + 3, b.n);
    WalkRec A = wrec.load(iA, cl(q));
    WalkRec B = wrec.load(iB, cl(q + 1));
    for (;;) {
      if (q >= b.n || A.key != k || A.idx >= hi) break;
      put_outcome(b, A, step(b, t, c, A), false);
      A = wrec.load(IA, cl(q + 2));
      IA = wrec.sidx[cl(q + 4)];
      ++q;
      if (q >= b.n || B.key != k || B.idx >= hi) break;
      put_outcome(b, B, step(b, t, c, B), false);
      B = wrec.load(IB, cl(q + 2));
      IB = wrec.sidx[cl(q + 4)];
      ++q;
    }
    flush(t, c);
    cursor[j] = static_cast<uint32_t>(q);
  }
}

// The walk: one 64-lane workgroup per virtual block of the device-side plan
// (long runs first), up to the first long echo reply it cannot take (or the
// batch end).  The host launches the plan's upper bound, n / 64 + 6 blocks
// (a run of class 0 has >= 64 packets, a lane of the others >= 1), and the
// blocks past the plan return at once: a workgroup that returns costs the
// dispatcher next to nothing, where a persistent grid taking blocks from one
// counter serialised ~10^5 atomics on one address (7.1 vs 2.9 ms a batch).
// With segments, the first nseg = seg_waves(n) workgroups walk the active cuts
// that ct_heads listed (walk_seg), each taking every nseg-th of them.
__global__ __launch_bounds__(64) void ct_walk_kernel(CtBatch b, CtTable t, const RecSrc wrec,
                                                     const uint32_t *heads, const uint32_t *ctl, uint32_t *cursor,
                                                     const uint32_t *skeys, uint32_t sentinel, SegRec *seg,
                                                     HeadExit *hx, const uint32_t *cuts, uint32_t nseg) {
  if (blockIdx.x < nseg) {
    const uint32_t na = ctl[kCtlSegN];
    for (uint32_t i = blockIdx.x; i < na; i += nseg) {
#if PCN_CT_DBG
      const uint64_t dbg_t0 = wall_clock64();
#endif
      const uint32_t j = cuts[i];
      walk_seg(b, t, wrec, skeys, sentinel, seg, j, walk_hi(b, ctl));
#if PCN_CT_DBG
      const uint64_t dt = wall_clock64() - dbg_t0;
      if (threadIdx.x == 0 && seg[j].status)
        printf("seg %u: status %u, walked %u, %llu us\n", j, seg[j].status, seg[j].stop - j * uint32_t(kSeg),
               (unsigned long long)(dt / 100));
#endif
    }
    return;
  }
  // (the plan is read in place: a local copy indexed by class went to scratch)
#if PCN_CT_DBG_T
  if (threadIdx.x == 0 && blockIdx.x >= nseg && blockIdx.x - nseg < kDbgWaves) g_walk_t[4 * (blockIdx.x - nseg)] = wall_clock64();
#endif
  const WalkPlan plan = plan_of(ctl);
  const uint32_t vb = blockIdx.x - nseg;
  // the head of a long run in flight with the plan's words (the index
  // clamped into the buffer; a block past the plan returns without using it)
  const uint64_t hcap = heads_cap(b.n);
  const uint32_t head = heads[vb < hcap ? vb : 0];
  if (vb >= plan.blk0[kRunClasses]) return;
  walk_vb(b, t, wrec, heads, plan, cursor, walk_hi(b, ctl), 1, vb, head, hx);
}

// For a cut j that is its run's first (the head stopped there): chain
// the run's segments in order from the head's state, re-walking those whose
// guess does not hold, then flush the connection and set the run's cursor.
__device__ void seg_fix_cut(const CtBatch &b, const CtTable &t, const RecSrc &wrec, const uint32_t *skeys,
                            const SegRec *seg, const HeadExit *hx, uint32_t *cursor, const uint32_t *ctl, uint32_t j) {
  const uint64_t B = uint64_t(j) * kSeg;
  if (j == 0 || B >= b.n || seg[j].status == 0) return;
  const uint32_t k = skeys[B];
  if (j > 1 && skeys[B - kSeg - 1] == k) return;   // the run holds cut j - 1 too: not its first cut
  const uint64_t hi = walk_hi(b, ctl);
  const HeadExit h = hx[j];
  Cache c{};
  c.k = Key{h.src, h.dst, static_cast<uint16_t>(h.ports), static_cast<uint16_t>(h.ports >> 16),
            static_cast<uint8_t>(h.px)};
  c.e = h.slot != ~0u ? &t.slots[h.slot] : nullptr;
  c.v = Ent{uint64_t(h.ttl_hi) << 32 | h.ttl_lo, h.seq, static_cast<uint8_t>(h.px >> 8),
            static_cast<uint8_t>(h.px >> 16), static_cast<uint8_t>(h.px >> 24)};
  c.valid = h.flags & 1;
  c.dirty = (h.flags >> 1) & 1;
  c.touch = h.touch;
  uint64_t stop = B;
  const uint32_t lane = threadIdx.x;
  // Up to 64 segments at a time (lane L: segment j0 + L).  The longest prefix
  // of them whose guesses hold and whose run goes on past them takes their
  // exits at once, with no walk: each lane compares its guess with its
  // predecessor's exit (lane 0 with the state as it stands), which is the
  // state it walked from exactly when every earlier one held.  The first
  // other segment is then taken as before -- left to its exit, or walked again
  // from the true state -- and the next 64 start after it.  One at a time, a
  // batch of one long connection (32 K cuts at 2^24) chained its cuts for
  // ~30 ms in this one wave.
  for (uint64_t j0 = j;;) {
    const uint64_t jl = j0 + lane, cl = jl * kSeg;
    SegRec sl{};
    bool more_l = false;
    if (cl < b.n) {
      sl = seg[jl];
      more_l = cut_active(skeys, b.n, cl + kSeg, k);
    }
    const uint32_t c_ports = uint32_t(c.k.sport) | uint32_t(c.k.dport) << 16;
    const uint32_t c_slot = c.e ? static_cast<uint32_t>(c.e - t.slots) : ~0u;
    // the predecessor's exit: its key and slot are its guess's (a held
    // speculative walk claims no slot and meets no other key), its value the exit
    const uint32_t c_src = __shfl(c.k.src, 0), c_dst = __shfl(c.k.dst, 0), c_pp = __shfl(c_ports, 0);
    const uint32_t c_sl = __shfl(c_slot, 0), c_seq = __shfl(c.v.seq, 0), c_px = __shfl(cache_px(c), 0);
    const bool c_ok = __shfl(c.valid ? 1 : 0, 0) != 0;
    const uint32_t u_src = __shfl_up(sl.src, 1), u_dst = __shfl_up(sl.dst, 1), u_ports = __shfl_up(sl.ports, 1);
    const uint32_t u_slot = __shfl_up(sl.gslot, 1), u_seq = __shfl_up(sl.xseq, 1);
    const uint32_t u_px = (__shfl_up(sl.gx, 1) & 0xffu) | (__shfl_up(sl.xx, 1) & 0xffffffu) << 8;
    const bool u_ok = __shfl_up(sl.status, 1) == 1u;
    const uint32_t p_src = lane ? u_src : c_src, p_dst = lane ? u_dst : c_dst, p_ports = lane ? u_ports : c_pp;
    const uint32_t p_slot = lane ? u_slot : c_sl, p_seq = lane ? u_seq : c_seq, p_px = lane ? u_px : c_px;
    const bool p_ok = lane ? u_ok : c_ok;
    const bool held_l = sl.status == 1 && p_ok && p_src == sl.src && p_dst == sl.dst && p_ports == sl.ports &&
                        p_slot == sl.gslot && p_px == sl.gx && p_seq == sl.gseq;
    const bool fast = held_l && more_l && sl.stop >= cl + kSeg;
    const uint64_t ends = __ballot(!fast);
    const uint32_t pfx = ends ? static_cast<uint32_t>(__builtin_ctzll(ends)) : 64u;
    if (pfx) {                                      // segments [j0, j0 + pfx): their exits at once
      const uint64_t in = pfx == 64 ? ~0ull : (1ull << pfx) - 1;
      const uint64_t ttl_m = __ballot((uint64_t(sl.ttl_hi) << 32 | sl.ttl_lo) != kTtlUnset) & in;
      const uint64_t touch_m = __ballot(sl.touch != 0) & in;
      const bool dirty = (__ballot((sl.xx >> 24) != 0) & in) != 0;
      const int last = static_cast<int>(pfx - 1);
      const uint32_t x_seq = __shfl(sl.xseq, last), x_xx = __shfl(sl.xx, last), x_stop = __shfl(sl.stop, last);
      const int tl = ttl_m ? 63 - __builtin_clzll(ttl_m) : 0, hl = touch_m ? 63 - __builtin_clzll(touch_m) : 0;
      const uint32_t t_lo = __shfl(sl.ttl_lo, tl), t_hi = __shfl(sl.ttl_hi, tl), tch = __shfl(sl.touch, hl);
      if (lane == 0) {
        if (ttl_m) c.v.ttl = uint64_t(t_hi) << 32 | t_lo;
        c.v.seq = x_seq;
        c.v.state = static_cast<uint8_t>(x_xx);
        c.v.rev = static_cast<uint8_t>(x_xx >> 8);
        c.v.live = static_cast<uint8_t>(x_xx >> 16);
        if (dirty) c.dirty = true;
        if (touch_m) c.touch = tch;
      }
      stop = x_stop;
    }
    if (pfx == 64) {
      j0 += 64;
      continue;
    }
    // segment jj = j0 + pfx, one at a time as before
    const uint64_t jj = j0 + pfx;
    const uint64_t cut = jj * kSeg;
    const bool held = __shfl(held_l ? 1 : 0, static_cast<int>(pfx)) != 0;
    const bool more = __shfl(more_l ? 1 : 0, static_cast<int>(pfx)) != 0;
    if (cut >= b.n || __shfl(sl.status, static_cast<int>(pfx)) == 0) {   // hi cuts the run at this (active) cut
      stop = cut;
      break;
    }
    if (held) {                                    // the segment as walked: its exit is the state
      const SegRec sp = seg[jj];
      if (lane == 0) {
        const unsigned long long ttl = uint64_t(sp.ttl_hi) << 32 | sp.ttl_lo;
        if (ttl != kTtlUnset) c.v.ttl = ttl;
        c.v.seq = sp.xseq;
        c.v.state = static_cast<uint8_t>(sp.xx);
        c.v.rev = static_cast<uint8_t>(sp.xx >> 8);
        c.v.live = static_cast<uint8_t>(sp.xx >> 16);
        if (sp.xx >> 24) c.dirty = true;
        if (sp.touch) c.touch = sp.touch;
      }
      stop = sp.stop;
    } else {
      bool ab;
      stop = walk_chunks<false>(b, t, wrec, k, cut, wrec.idx_at(cut + threadIdx.x, b.n), wrec.key_at(cut + threadIdx.x, b.n),
                                wrec.idx_at(cut + 64 + threadIdx.x, b.n), wrec.key_at(cut + 64 + threadIdx.x, b.n), hi,
                                more ? cut + kSeg : ~0ull, c, ab, true);
    }
#if PCN_CT_DBG
    if (threadIdx.x == 0)
      printf("fix %u: cut %u %s (after %u held at once)\n", j, static_cast<uint32_t>(jj), held ? "held" : "re-walked", pfx);
#endif
    if (!more || stop < cut + kSeg) break;         // the run ended in this segment (or hi cut it)
    j0 = jj + 1;
  }
  if (threadIdx.x == 0) {
    flush(t, c);
    cursor[h.vb] = static_cast<uint32_t>(stop);
  }
}

// One wave per seg_waves(n)-th active cut (only a run's first cut does work;
// the bench traffic has such runs: their fixes in ct_tail, one after the other
// in one wave, took 80 us against this kernel's 22).
__global__ __launch_bounds__(64) void ct_seg_fix_kernel(CtBatch b, CtTable t, const RecSrc wrec,
                                                        const uint32_t *skeys, const SegRec *seg, const HeadExit *hx,
                                                        uint32_t *cursor, const uint32_t *ctl, const uint32_t *cuts) {
  const uint32_t na = ctl[kCtlSegN];
  for (uint32_t i = blockIdx.x; i < na; i += gridDim.x) seg_fix_cut(b, t, wrec, skeys, seg, hx, cursor, ctl, cuts[i]);
}

// An echo reply long enough to quote a header (ConntrackLabel_dp.c:450-531)
// whose quoted key bucket also has packets in the batch, so that key's state
// at its position is only known once everything before it has been walked:
// its own key decides ESTABLISHED; otherwise ICMP_MISS reads the quoted key.
__device__ void hard_step(const CtBatch &b, const CtTable &t, const PackedRec *brec, uint32_t i) {
  const CtRec r = ct_rec(load_prec(&brec[i]));
  Cache c2{};
  const Key q{r.seq, r.ack, static_cast<uint16_t>(r.iports & 0xffff), static_cast<uint16_t>(r.iports >> 16), r.flags};
  const bool quoted = lookup(t, c2, q);            // read-only
  Cache c{};
  const bool live = lookup(t, c, Key{r.src, r.dst, r.sport, r.dport, r.proto});
  const int l = !live ? ST_INV : ((c.v.rev ^ r.rev) == 3) ? ST_EST : quoted ? ST_REL : ST_INV;
  const int32_t o = outcome(b, pack_outcome(b, 0, i), pack_outcome(b, 1, i), pack_outcome(b, 2, i),
                            pack_outcome(b, 3, i), r, l);
  if ((o & 1) == PCN_IPT_ACCEPT && l >= 0) update(t, c, r, l);
  if (c.v.live && c.e) c.touch = i + 1;
  flush(t, c);
  b.verdicts[i] = static_cast<uint8_t>(o & 1);
  b.rule_ids[i] = o >> 1;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t u = __shfl_xor(v, o);
    v = u < v ? u : v;
  }
  return v;
}

// The rest of the batch from the first long echo reply the walk could not
// take, in one wave: that reply (its own and its quoted key read from the
// table, everything before it being done), then every run walked on from its
// cursor up to the next such reply, and so on to the batch end.  A batch
// without them returns at once.  (These need an echo-reply payload that reads
// as a header of a connection with packets in the same batch: rare, and slow
// here, but exact.)
__global__ __launch_bounds__(64) void ct_tail_kernel(CtBatch b, CtTable t, const RecSrc wrec, const PackedRec *brec,
                                                     const uint32_t *heads, const uint32_t *ctl,
                                                     const uint32_t *th_list, uint32_t *cursor) {
  const uint32_t th = ctl[kCtlThFirst];
  if (!th) return;
  const uint32_t nth = ctl[kCtlTh];
  const WalkPlan plan = plan_of(ctl);
  const uint32_t total = plan.blk0[kRunClasses];
  uint32_t cur = 0xFFFFFFFFu - th;
  for (;;) {
    if (threadIdx.x == 0) hard_step(b, t, brec, cur);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // its table writes before any lane reads on
    __syncthreads();
    uint32_t nxt = 0xFFFFFFFFu;
    for (uint32_t k = threadIdx.x; k < nth; k += 64) {
      const uint32_t v = th_list[k];
      if (v > cur && v < nxt) nxt = v;
    }
    nxt = wave_min(nxt);
    const uint64_t hi = nxt == 0xFFFFFFFFu ? b.n : nxt;
    for (uint32_t vb = 0; vb < total; ++vb) {
      walk_vb(b, t, wrec, heads, plan, cursor, hi, 0, vb, heads[vb], nullptr);   // (no cuts)
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __syncthreads();
    }
    if (nxt == 0xFFFFFFFFu) return;
    cur = nxt;
  }
}

// ---- LRU at batch granularity (Iptables_ConntrackLabel_dp.c:112: lru_hash of
// 65536) ----
// After the walk, if more than max_entries entries are live, the live entries
// with the oldest touch stamps (batch seq << 32 | batch index of the last
// packet after which each was live; distinct, since a packet touches one key)
// are deleted down to max_entries.  touch[] holds the stamp of every live
// entry and ~0 for every other slot, so the cut reads 8 bytes a slot and
// nothing else: a radix select, each pass a histogram of the stamps that
// match the digits chosen so far.
// Pass 0 counts the live entries and finds the oldest and newest live
// stamp: every stamp shares the bits above their highest difference, so the
// digit passes start there (a batch's stamps differ in the batch index and a
// few low bits of the batch sequence: four passes instead of six).  Pass p > 0
// takes the next kEvDigit bits (fewer at the bottom) below the chosen prefix and
// returns at once when nothing is left to choose.  Every workgroup merges its
// LDS histogram into the global one with one atomic per non-empty bin, and
// the pass's last workgroup picks the digit with a block-wide scan.  (Six
// fixed 11-bit passes of 64 workgroups took 26 us each, 0.19 ms a batch:
// profiles/r03_s24_ev_ab.log.)
#ifndef PCN_CT_EV_DIGIT
#define PCN_CT_EV_DIGIT 11   // A/B 14: six launches of 17.8 us against seven of 15.4 (profiles/r04_s14/)
#endif
constexpr uint32_t kEvDigit = PCN_CT_EV_DIGIT;
constexpr uint32_t kEvBins = 1u << kEvDigit;
constexpr int kEvPasses = 1 + (64 + kEvDigit - 1) / kEvDigit;   // pass 0 + the digits of 64 bits
static_assert(kEvBins % 1024 == 0, "the final scan gives each of the 1024 threads a run of bins");
constexpr uint32_t kEvBlock = 1024;

__global__ __launch_bounds__(kEvBlock) void ct_ev_pass_kernel(CtTable t, uint32_t *ctl, uint32_t *hist, int p) {
  __shared__ uint32_t h[kEvBins];
  __shared__ uint32_t scan[kEvBlock];
  __shared__ uint32_t live_s;
  __shared__ unsigned long long lo_s, hi_s;
  __shared__ bool last;
  uint32_t low = 0;
  if (p > 0) {
    if (!ctl[kCtlEvict]) return;
    low = ctl[kCtlEvLow];
    if (low == 0) return;                              // every bit chosen
  }
  const uint32_t width = low < kEvDigit ? low : kEvDigit, shift = low - width;
  for (uint32_t k = threadIdx.x; k < kEvBins; k += blockDim.x) h[k] = 0;
  if (threadIdx.x == 0) {
    live_s = 0;
    lo_s = 0;
    hi_s = 0;
  }
  __syncthreads();
  const uint64_t prefix = *reinterpret_cast<const unsigned long long *>(ctl + kCtlEvPrefix);
  const uint64_t above = low >= 64 ? 0ull : ~((uint64_t(1) << low) - 1);
  const uint64_t cap = uint64_t(1) << t.cap_log2;
  const uint64_t stp = uint64_t(gridDim.x) * blockDim.x;
  uint32_t live = 0;
  unsigned long long nmin = 0, mx = 0;                 // ~oldest, newest
  // 16 stamps a thread in flight together: unconditional loads (index clamped,
  // the lanes past the table masked) -- a conditional load merges into a phi
  // the compiler resolves with an immediate vmcnt(0), one round trip per load
  constexpr int U = 16;
  for (uint64_t i0 = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i0 < cap; i0 += U * stp) {
    unsigned long long key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) key[u] = t.touch[i0 + u * stp < cap ? i0 + u * stp : cap - 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool in = i0 + u * stp < cap && key[u] != ~0ull && (p == 0 || (key[u] & above) == prefix);
      if (p == 0) {
        if (in) {
          ++live;
          nmin = ~key[u] > nmin ? ~key[u] : nmin;
          mx = key[u] > mx ? key[u] : mx;
        }
        continue;
      }
      // LDS atomics on one address serialise (~20 ns each), and a digit's
      // stamps fall into a few bins (a batch's stamps differ in the batch
      // index's high bits and the sequence's low ones): the lanes of a digit
      // find each other by one ballot per digit bit and add once.  (Only the
      // lanes sharing the first lane's digit added together before; the
      // rest, most of a wave, added one by one: ~24 us a pass.)
      // The first two lanes' digits add once each (a pass over few bins: most
      // of the wave); then, when the second digit was rare (the first digit
      // pass, its stamps spread over the bins), the rest lane by lane, else the
      // bit-ballot match.  (The match for every slot: the first digit pass
      // took 35 us of 32 workgroups' ballots.)
      const uint64_t im = __ballot(in);
      if (!im) continue;
      const uint32_t lane = threadIdx.x & 63;
      const uint32_t d = static_cast<uint32_t>(key[u] >> shift) & ((1u << width) - 1);
      const uint32_t l0 = static_cast<uint32_t>(__builtin_ctzll(im));
      const uint32_t d0 = static_cast<uint32_t>(__shfl(static_cast<int>(d), static_cast<int>(l0)));
      const uint64_t m0 = __ballot(in && d == d0);
      if (lane == l0) atomicAdd(&h[d0], static_cast<uint32_t>(__builtin_popcountll(m0)));
      uint64_t rest = im & ~m0;
      if (!rest) continue;
      const uint32_t l1 = static_cast<uint32_t>(__builtin_ctzll(rest));
      const uint32_t d1 = static_cast<uint32_t>(__shfl(static_cast<int>(d), static_cast<int>(l1)));
      const uint64_t m1 = __ballot(in && d == d1);
      if (lane == l1) atomicAdd(&h[d1], static_cast<uint32_t>(__builtin_popcountll(m1)));
      rest &= ~m1;
      if (!rest) continue;
      const bool mine = (rest >> lane) & 1;
      if (__builtin_popcountll(m1) <= 2) {
        if (mine) atomicAdd(&h[d], 1u);
        continue;
      }
      uint64_t peers = rest;
      for (uint32_t bit = 0; bit < width; ++bit) {
        const uint64_t bb = __ballot((d >> bit) & 1);
        peers &= ((d >> bit) & 1) ? bb : ~bb;
      }
      if (mine && lane == __builtin_ctzll(peers))
        atomicAdd(&h[d], static_cast<uint32_t>(__builtin_popcountll(peers)));
    }
  }
  uint32_t *hp = hist + p * kEvBins;
  // The merges are device-scope atomics, which every workgroup's reads of
  // them (atomic loads) see once they have completed: each wave waits for its
  // own (returning atomics, the results consumed) before the workgroup
  // arrives.  No fence: a __threadfence() in all 16 waves (an L2 write-back
  // and invalidate each) cost ~15 us a pass.
  uint64_t dep = 0;
  if (p == 0) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {              // one LDS atomic per wave
      live += __shfl_xor(live, o);
      const unsigned long long a = __shfl_xor(nmin, o), b = __shfl_xor(mx, o);
      nmin = a > nmin ? a : nmin;
      mx = b > mx ? b : mx;
    }
    if ((threadIdx.x & 63) == 0 && live) {
      atomicAdd(&live_s, live);
      atomicMax(&lo_s, nmin);
      atomicMax(&hi_s, mx);
    }
    __syncthreads();
    if (threadIdx.x == 0 && live_s) {
      dep += atomicAdd(&ctl[kCtlLive], live_s);
      dep += atomicMax(reinterpret_cast<unsigned long long *>(ctl + kCtlEvNotMin), lo_s);
      dep += atomicMax(reinterpret_cast<unsigned long long *>(ctl + kCtlEvMax), hi_s);
    }
  } else {
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kEvBins; k += blockDim.x)
      if (h[k]) dep += atomicAdd(&hp[k], h[k]);
  }
  asm volatile("" ::"v"(dep));
  __syncthreads();
  // the arrival orders this workgroup's histogram merges before it and the last
  // arriver's reads after it (acquire-release at agent scope: one ordering
  // operation per workgroup, where a __threadfence in every wave cost 9-23 us a
  // pass; returning device atomics completing at L2 alone is a gfx950 property,
  // not a guarantee of the memory model)
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&ctl[kCtlEvDone], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  if (p == 0) {                                        // the last workgroup: evict at all, and from which bit
    if (threadIdx.x == 0) {
      ctl[kCtlEvDone] = 0;
      const uint32_t lv = __hip_atomic_load(&ctl[kCtlLive], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t.max_entries && lv > t.max_entries) {
        const uint64_t oldest = ~__hip_atomic_load(reinterpret_cast<unsigned long long *>(ctl + kCtlEvNotMin),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t newest = __hip_atomic_load(reinterpret_cast<unsigned long long *>(ctl + kCtlEvMax),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // bits above the highest one where the oldest and newest differ are common to all
        const uint32_t top = oldest == newest ? 0u : 64u - static_cast<uint32_t>(__builtin_clzll(oldest ^ newest));
        ctl[kCtlEvK] = lv - static_cast<uint32_t>(t.max_entries);
        *reinterpret_cast<unsigned long long *>(ctl + kCtlEvPrefix) =
            top >= 64 ? 0ull : oldest & ~((uint64_t(1) << top) - 1);
        ctl[kCtlEvLow] = top;
        ctl[kCtlEvict] = 1;
      }                                                // (else kCtlEvict stays 0)
    }
    return;
  }
  // the digit whose bin holds the k-th smallest matching stamp, by a block-wide
  // scan of each thread's run of `per` bins
  const uint32_t k = ctl[kCtlEvK];
  constexpr uint32_t per = kEvBins / kEvBlock;
  const uint32_t b0 = per * threadIdx.x;               // this thread's bins
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t j = 0; j < per; ++j) mine += __hip_atomic_load(&hp[b0 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  scan[threadIdx.x] = mine;
  __syncthreads();
  for (uint32_t o = 1; o < kEvBlock; o <<= 1) {        // inclusive scan
    const uint32_t v = threadIdx.x >= o ? scan[threadIdx.x - o] : 0u;
    __syncthreads();
    scan[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t incl = scan[threadIdx.x], excl = incl - mine;
  if (excl < k && k <= incl) {                         // exactly one thread
    uint32_t below = excl, d = b0;
    for (;;) {
      const uint32_t c = __hip_atomic_load(&hp[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (below + c >= k) break;
      below += c;
      ++d;
    }
    ctl[kCtlEvK] = k - below;
    *reinterpret_cast<unsigned long long *>(ctl + kCtlEvPrefix) = prefix | (uint64_t(d) << shift);
    ctl[kCtlEvLow] = shift;
  }
  if (threadIdx.x == 0) ctl[kCtlEvDone] = 0;          // for the next pass
}

// Delete the live entries whose stamp is at most the chosen one (exactly the
// oldest live - max_entries), count them, and clear the histograms.
constexpr uint32_t kEvictBlock = 1024;
__global__ __launch_bounds__(kEvictBlock) void ct_ev_evict_kernel(CtTable t, const uint32_t *ctl, uint32_t *hist) {
  const uint64_t stp = uint64_t(gridDim.x) * blockDim.x;
  const uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (uint64_t k = g; k < uint64_t(kEvPasses) * kEvBins; k += stp) hist[k] = 0;
  if (!ctl[kCtlEvict]) return;                       // (uniform: every thread returns)
  const uint64_t cut = *reinterpret_cast<const unsigned long long *>(ctl + kCtlEvPrefix);
  const uint64_t cap = uint64_t(1) << t.cap_log2;
  uint32_t n = 0;
  constexpr int U = 4;                                 // stamps in flight together (unconditional loads)
  for (uint64_t i0 = g; i0 < cap; i0 += U * stp) {
    unsigned long long key[U];
#pragma unroll
    for (int u = 0; u < U; ++u) key[u] = t.touch[i0 + u * stp < cap ? i0 + u * stp : cap - 1];
    uint32_t del = 0;                                  // (all decided before any store: one wait)
#pragma unroll
    for (int u = 0; u < U; ++u) del |= (i0 + u * stp < cap && key[u] <= cut ? 1u : 0u) << u;   // newer / not live: kept
    asm volatile("" : "+v"(del));                      // (opaque: the compares are not sunk into the stores' branches)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!((del >> u) & 1)) continue;
      const uint64_t i = i0 + u * stp;
      // valid = 0 (connections.delete): the byte alone -- no read of the
      // slot (a load per deletion, each waited for before its store)
      t.slots[i].valid = 0;
      t.touch[i] = ~0ull;
      ++n;
    }
  }
  // one atomic per workgroup on the one counter: device-scope atomics on one
  // address serialise (~7 ns apiece), and one per wave -- 4,096 waves of a
  // 2^20-slot table, nearly all deleting on the bench traffic -- was 30 us of
  // the kernel's 30 (one per thread with a deletion: ~200 K of them)
  __shared__ uint32_t wn[kEvictBlock / 64];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0) wn[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kEvictBlock / 64; ++w) tot += wn[w];
    if (tot) atomicAdd(&t.stats[1], static_cast<unsigned long long>(tot));
  }
}

// Long echo replies (K_HARD) into the walk: a reply joins its own key's run
// unless its quoted key's bucket holds a packet of the batch (or another
// reply's own key), which only the tail can order.  Three passes over a
// bitmap of the batch's key buckets; each returns at once without replies.
// The bitmap is zero when a batch starts: from its allocation, then cleared
// by ct_heads after any batch that set bits (a clearing kernel of its own was
// a launch a batch).

__device__ __forceinline__ void set_bit(uint32_t *bm, uint32_t k) {
  const uint32_t m = 1u << (k & 31);
  if (!(bm[k >> 5] & m)) atomicOr(&bm[k >> 5], m);   // hot keys: most of their packets find it set
}

__device__ __forceinline__ uint32_t own_bucket(const CtRec &r, uint32_t sentinel) {
  return ct_bucket(key_hash(r.src, r.dst, r.proto, r.sport, r.dport), sentinel);
}

__global__ void ct_hbits_set_kernel(uint64_t n, const uint32_t *ctl, const uint32_t *keys, const uint32_t *hard_list,
                                    const PackedRec *brec, uint32_t *bm, uint32_t sentinel) {
  const uint32_t nh = ctl[kCtlHard];
  if (!nh) return;
  const uint64_t stp = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stp) {
    const uint32_t k = keys[i];
    if (k != sentinel) set_bit(bm, k);
  }
  for (uint64_t h = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; h < nh; h += stp)
    set_bit(bm, own_bucket(ct_rec(load_prec(&brec[hard_list[h]])), sentinel));
}

__global__ void ct_hard_split_kernel(uint32_t *ctl, const uint32_t *hard_list, const PackedRec *brec, uint32_t *keys,
                                     const uint32_t *bm, uint32_t sentinel, uint32_t *th_list) {
  const uint32_t nh = ctl[kCtlHard];
  const uint64_t stp = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t h = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; h < nh; h += stp) {
    const uint32_t i = hard_list[h];
    const CtRec r = ct_rec(load_prec(&brec[i]));
    const uint32_t qb = ct_bucket(
        key_hash(r.seq, r.ack, r.flags, static_cast<uint16_t>(r.iports & 0xffff), static_cast<uint16_t>(r.iports >> 16)),
        sentinel);
    if ((bm[qb >> 5] >> (qb & 31)) & 1) {
      th_list[atomicAdd(&ctl[kCtlTh], 1u)] = i;
      atomicMax(&ctl[kCtlThFirst], 0xFFFFFFFFu - i);
    } else {
      const uint32_t k = own_bucket(r, sentinel);
      keys[i] = k;
    }
  }
}

// Counters from the final rule ids: per-rule and default (ActionLookup_dp.c:96-111,
// Parser_dp.c:47-58) and accept-established (ConntrackLabel_dp.c:137-188).
constexpr uint32_t kCountBlock = 1024;
constexpr uint32_t kLdsRules = 1024;          // LDS bins per chain; rules above use global atomics
constexpr uint64_t kCountChunk = 65536;       // packets per workgroup at most: packed bins cannot carry
static_assert(kCountChunk * 65535 < (1ull << 40) && kCountChunk < (1ull << 24), "ct_count packed bins");
// Packets per workgroup: kCountChunk, or fewer (a multiple of 4 x kCountBlock)
// so that every CU gets a workgroup (a 2 M-frame batch ran 32 workgroups,
// 93 us; 256 of them 29 us).
inline uint64_t count_chunk(uint64_t n, int num_cus) {
  constexpr uint64_t q = 4 * kCountBlock;
  const uint64_t c = (n / uint64_t(num_cus) + q - 1) / q * q;   // (two per CU measured slower: 29 -> 36 us; 33 -> 38 in r06_s19)
  return c < q ? q : c > kCountChunk ? kCountChunk : c;
}

// bin k of ct_count's 4 x (2 + kLdsRules): per chain c < 3 the default (0),
// accept-established (1) and rule bins (2..); group 3 the Horus rule ids
__device__ __forceinline__ void ct_count_add(const CtBatch &b, uint32_t k, unsigned long long pk,
                                             unsigned long long by) {
  constexpr uint32_t per = 2 + kLdsRules;
  const uint32_t c = k / per, bin = k % per;
  unsigned long long *dp, *db;
  if (c == 3) { dp = &b.horus_ctr[2 * (bin - 2)]; db = &b.horus_ctr[2 * (bin - 2) + 1]; }
  else if (bin == 0) { dp = &b.ctr[c][0]; db = &b.ctr[c][1]; }
  else if (bin == 1) { dp = &b.ae_ctr[2 * c]; db = &b.ae_ctr[2 * c + 1]; }
  else { dp = &b.ctr[c][2 + 2 * (bin - 2)]; db = &b.ctr[c][3 + 2 * (bin - 2)]; }
  atomicAdd(dp, pk);
  atomicAdd(db, by);
}

#ifndef PCN_CT_COUNT_U
#define PCN_CT_COUNT_U 8   // (16: 37.0 us a 2^24 batch against 33.4, profiles/r06_s19/)
#endif
template <class T>
__device__ __forceinline__ T sel3(uint32_t c, T a, T b, T d) {
  return c == 0 ? a : c == 1 ? b : d;
}
// It also leaves the next batch's control words and ports descriptors zeroed
// (ctl[0, kCtlZero), pdesc[0, ngroups)): two memsets a batch were a launch each.
// The workgroup's bins go out as one row of `part` (ct_count_reduce_kernel sums
// the rows and adds each counter once): adding them to the counters here, two
// device-scope atomics per non-zero bin from every workgroup, landed ~500 K
// atomics a 2^24 batch on ~2 K addresses, serialised where they meet.  (part
// null: the atomics, PCN_IPT_DEBUG_CT_COUNT_ATOMIC=1, for the A/B.)
// VEC: rule ids and {len, cinfo} words read 16 bytes (four packets) a load
// (both arrays 16-byte aligned; a chunk is a multiple of 4096 packets).
template <bool VEC>
__global__ __launch_bounds__(kCountBlock) void ct_count_kernel(CtBatch b, const uint32_t *lcs, uint64_t chunk,
                                                               uint32_t *ctl, unsigned long long *pdesc,
                                                               uint64_t ngroups, unsigned long long *part) {
  constexpr uint32_t per = 2 + kLdsRules;
  for (uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < ngroups; g += uint64_t(gridDim.x) * blockDim.x)
    pdesc[g] = 0;
  if (blockIdx.x == 0 && threadIdx.x < kCtlZero) ctl[threadIdx.x] = 0;
  // groups 0-2: the chains; group 3: Horus rule ids (bins 2..).  One u64 LDS
  // atomic per packet: pkts in bits 40-63, bytes in bits 0-39 (a workgroup's
  // <= 2^16 packets of <= 65535 bytes cannot carry out of either field).
  __shared__ unsigned long long bins[4 * per];
  for (uint32_t k = threadIdx.x; k < 4 * per; k += blockDim.x) bins[k] = 0;
  __syncthreads();
  const uint64_t lo = uint64_t(blockIdx.x) * chunk;
  const uint64_t hi = lo + chunk < b.n ? lo + chunk : b.n;
  // The default rule's packets (half of them on the bench traffic) go to one
  // bin per chain: as LDS atomics, 32 lanes of an instruction on one address
  // serialised.  A lane sums them in registers instead (packed as the bins).
  unsigned long long dflt0 = 0, dflt1 = 0, dflt2 = 0;
  // (b.ncounted[c] or b.ctr[c] indexed by a lane's chain is a vector load from
  // the kernel arguments, or from a private copy of them, whose wait, vmcnt(0),
  // drained every load in flight: they are kept in scalars, made opaque so the
  // compiler cannot fold the selects back into an indexed load)
  auto sreg = [](auto x) {
    asm volatile("" : "+s"(x));
    return x;
  };
  const uint32_t nc0 = sreg(b.ncounted[0]), nc1 = sreg(b.ncounted[1]), nc2 = sreg(b.ncounted[2]);
  unsigned long long *const ctr0 = sreg(b.ctr[0]), *const ctr1 = sreg(b.ctr[1]), *const ctr2 = sreg(b.ctr[2]);
  unsigned long long *const hctr = b.horus_ctr;
  // One packet's bin by selects, one branch for the LDS atomic and one for the
  // rare global counters (rule or Horus ids >= kLdsRules): the branch per case
  // made the kernel instruction-bound (63 us a 2^24 batch, 31 of them the loads).
  // Horus ids: Horus_dp.c:80-90, counted at the lookup, whatever the chain.
  // (values selected by sel3: `c == 0 ? x : ...` of lvalues is a select between
  // their addresses, which put them in scratch)
  auto count1 = [&](int32_t rid, uint32_t lc) {
    const uint32_t len = lc & 0xffff, c = (lc >> 16) & 3;
    const unsigned long long v = (1ull << 40) | len;
    const bool hor = rid <= PCN_IPT_RID_HORUS0;
    const uint32_t hid = static_cast<uint32_t>(PCN_IPT_RID_HORUS0 - rid);
    const bool chain = !hor && c != 3;
    const bool rule = chain && rid >= 0 && static_cast<uint32_t>(rid) < sel3(c, nc0, nc1, nc2);
    const bool hc = hor && hctr != nullptr;
    const bool dfl = chain && rid == PCN_IPT_RID_DEFAULT;
    dflt0 += dfl && c == 0 ? v : 0ull;
    dflt1 += dfl && c == 1 ? v : 0ull;
    dflt2 += dfl && c == 2 ? v : 0ull;
    const uint32_t id = hc ? hid : static_cast<uint32_t>(rid);
    if ((hc || rule) && id >= kLdsRules) {
      unsigned long long *const cr =
          hc ? hctr + 2 * uint64_t(id) : sel3(c, ctr0, ctr1, ctr2) + 2 + 2 * uint64_t(id);
      atomicAdd(cr, 1ull);
      atomicAdd(cr + 1, static_cast<unsigned long long>(len));
    }
    const bool lds = (hc || rule) ? id < kLdsRules : chain && rid == -3;
    const uint32_t bin = hc ? 3 * per + 2 + id : rule ? c * per + 2 + id : c * per + 1;
    if (lds) atomicAdd(&bins[bin], v);
  };
  // U packets per thread whose loads are in flight together (4: a thread's 64
  // packets of a 2^24 batch took 16 dependent round trips): unconditional, the
  // index clamped to the chunk's last (a conditional load merges into a phi the
  // compiler resolves with an immediate wait); lanes past it are masked where
  // the packets are counted.  (The next round's loads issued before a round is
  // counted measured slower, 35.1 against 33.4 us: r06_s19.)
  constexpr uint32_t U = PCN_CT_COUNT_U;
  if constexpr (VEC) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    constexpr uint32_t V = U / 4;
    const u32x4 *const rv = reinterpret_cast<const u32x4 *>(b.rule_ids);
    const u32x4 *const lv = reinterpret_cast<const u32x4 *>(lcs);
    const uint64_t lo4 = lo / 4, hi4 = hi / 4;          // lo is a multiple of 4
    const uint64_t step = uint64_t(V) * blockDim.x;
    auto load = [&](u32x4 *r, u32x4 *l, uint64_t q0) {
#pragma unroll
      for (uint32_t u = 0; u < V; ++u) {
        const uint64_t q = q0 + u * blockDim.x;
        const uint64_t j = q < hi4 ? q : hi4 - 1;
        r[u] = rv[j];
        l[u] = lv[j];
      }
    };
    for (uint64_t q0 = lo4 + threadIdx.x; q0 < hi4; q0 += step) {
      u32x4 r[V], l[V];
      load(r, l, q0);
#pragma unroll
      for (uint32_t u = 0; u < V; ++u) {
        if (q0 + u * blockDim.x >= hi4) continue;
        count1(static_cast<int32_t>(r[u].x), l[u].x);
        count1(static_cast<int32_t>(r[u].y), l[u].y);
        count1(static_cast<int32_t>(r[u].z), l[u].z);
        count1(static_cast<int32_t>(r[u].w), l[u].w);
      }
    }
    if (threadIdx.x < hi - hi4 * 4) {                   // the last 0-3 packets of an unaligned end
      const uint64_t i = hi4 * 4 + threadIdx.x;
      count1(b.rule_ids[i], lcs[i]);
    }
  } else {
    const uint64_t step = uint64_t(U) * blockDim.x;
    auto load = [&](int32_t *r, uint32_t *l, uint64_t i0) {
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint64_t i = i0 + u * blockDim.x;
        const uint64_t j = i < hi ? i : hi - 1;
        r[u] = b.rule_ids[j];
        l[u] = lcs[j];
      }
    };
    for (uint64_t i0 = lo + threadIdx.x; i0 < hi; i0 += step) {
      int32_t rids[U];
      uint32_t lcv[U];
      load(rids, lcv, i0);
#pragma unroll
      for (uint32_t u = 0; u < U; ++u)
        if (i0 + u * blockDim.x < hi) count1(rids[u], lcv[u]);
    }
  }
  const unsigned long long dflt[3] = {dflt0, dflt1, dflt2};
  // the default bins, summed over the wave: one LDS atomic per wave and chain
#pragma unroll
  for (uint32_t c = 0; c < 3; ++c) {
    unsigned long long v = dflt[c];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&bins[c * per], v);
  }
  __syncthreads();
  if (part) {
    unsigned long long *const row = part + uint64_t(blockIdx.x) * (4 * per);
    for (uint32_t k = threadIdx.x; k < 4 * per; k += blockDim.x) row[k] = bins[k];
    return;
  }
  for (uint32_t k = threadIdx.x; k < 4 * per; k += blockDim.x) {
    const unsigned long long v = bins[k];
    if (v) ct_count_add(b, k, v >> 40, v & ((1ull << 40) - 1));
  }
}

// Per bin (64 a workgroup, lane = bin) the sum of the ct_count rows: 16 waves
// take every 16th row, their sums meet in LDS, and each non-zero bin is added
// to its counters once.
constexpr uint32_t kCountRedWaves = 16;
__global__ __launch_bounds__(64 * kCountRedWaves) void ct_count_reduce_kernel(CtBatch b,
                                                                               const unsigned long long *part,
                                                                               uint32_t rows) {
  constexpr uint32_t per = 2 + kLdsRules, nbins = 4 * per;
  constexpr uint32_t R = 8;   // rows whose loads are in flight together
  __shared__ unsigned long long sp[kCountRedWaves][64], sb[kCountRedWaves][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t k = blockIdx.x * 64 + lane;
  unsigned long long p = 0, by = 0;
  if (k < nbins) {
    for (uint32_t r0 = w; r0 < rows; r0 += R * kCountRedWaves) {
      unsigned long long v[R];
#pragma unroll
      for (uint32_t j = 0; j < R; ++j) {
        const uint32_t r = r0 + j * kCountRedWaves;
        v[j] = part[uint64_t(r < rows ? r : w) * nbins + k];
      }
#pragma unroll
      for (uint32_t j = 0; j < R; ++j) {
        if (r0 + j * kCountRedWaves >= rows) continue;
        p += v[j] >> 40;
        by += v[j] & ((1ull << 40) - 1);
      }
    }
  }
  sp[w][lane] = p;
  sb[w][lane] = by;
  __syncthreads();
  if (w || k >= nbins) return;
#pragma unroll
  for (uint32_t x = 1; x < kCountRedWaves; ++x) {
    p += sp[x][lane];
    by += sb[x][lane];
  }
  if (p) ct_count_add(b, k, p, by);
}

// Stateless accept-established: rule 0 of an AE chain is exactly
// {conntrack ESTABLISHED, ACCEPT}, so its hits are the packets the reference
// accepts before the chain (ConntrackLabel_dp.c:580-616).
__global__ void ae_move_kernel(CtBatch b) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int c = 0; c < 3; ++c) {
    if (!((b.ae_mask >> c) & 1) || !b.ncounted[c]) continue;
    // atomic: a classify on another stream may be adding to rule 0 meanwhile
    atomicAdd(&b.ae_ctr[2 * c], atomicExch(&b.ctr[c][2], 0ull));
    atomicAdd(&b.ae_ctr[2 * c + 1], atomicExch(&b.ctr[c][3], 0ull));
  }
}

__global__ void ae_rid_kernel(CtBatch b) {
  const uint64_t step = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < b.n; i += step) {
    if (b.rule_ids[i] != 0) continue;
    uint32_t w[18], L;
    load_window(b, i, w, L);
    const Parsed p = parse(w, L, b.hook);
    const uint32_t chain = b.direction == PCN_IPT_EGRESS ? PCN_IPT_OUTPUT
                           : (b.nlocal && localip_has(b, p.dst)) ? PCN_IPT_INPUT : PCN_IPT_FORWARD;
    if ((b.ae_mask >> chain) & 1) b.rule_ids[i] = -3;
  }
}

unsigned grid_for(uint64_t n, unsigned block, int num_cus) {
  const uint64_t want = (n + block - 1) / block;
  const uint64_t cap = uint64_t(num_cus) * 16;
  return static_cast<unsigned>(want < cap ? (want ? want : 1) : cap);
}

}  // namespace

struct CtScratch {
  uint64_t cap = 0;
  bool dirty = false;                     // a batch returned early: ctl / pdesc need zeroing
  unsigned long long *pdesc = nullptr;   // ct_prep: the ports word of every 64-frame group
  uint32_t *keys = nullptr, *keys2 = nullptr;
  uint32_t *lcs = nullptr;                // per packet: len | cinfo << 16 (ct_count)
  uint32_t *idx2 = nullptr, *cursor = nullptr, *hard_list = nullptr, *ctl = nullptr;
  uint32_t *th_list = nullptr;            // long echo replies left to ct_tail
  uint32_t *bm = nullptr;                 // key-bucket bitmap (ct_hbits_*)
  uint32_t *evh = nullptr;                // LRU radix-select histograms (kEvPasses x kEvBins, kept zeroed)
  uint64_t bm_bytes = 0;
  uint32_t *heads = nullptr;
  SegRec *seg = nullptr;                  // speculative segments of long runs (walk_seg, seg_fix_cut)
  HeadExit *hx = nullptr;
  uint32_t *cuts = nullptr;               // the batch's active cuts (ct_heads; ctl[kCtlSegN] of them)
  PackedRec *brec = nullptr;  // walk records, batch order
  ct_u32x4 *ox = nullptr;     // the four stage-A outcomes per packet (batches with four labels)
  uint64_t ox_cap = 0;
  RadixScratch rx;            // the (key bucket, index) sort (radix.hip)
  // ct_advance_carry: 1 + the batch's last port-writing frame
  unsigned long long *zfound = nullptr;
  // a stage A that wrote the walk records: per group the lanes to complete
  // (ct_stale_fix), per 1024 groups the last ports word (ct_stale_agg)
  unsigned long long *fixm = nullptr;
  unsigned long long *sagg = nullptr;
  unsigned long long *cpart = nullptr;    // ct_count: a row of bins per workgroup
  uint64_t cpart_rows = 0;
};

CtScratch *ct_scratch_new() { return new CtScratch(); }

void ct_scratch_free(CtScratch *s) {
  if (!s) return;
  for (void *p : {static_cast<void *>(s->pdesc), static_cast<void *>(s->lcs),
                  static_cast<void *>(s->keys), static_cast<void *>(s->keys2),
                  static_cast<void *>(s->idx2), static_cast<void *>(s->cursor), static_cast<void *>(s->hard_list),
                  static_cast<void *>(s->ctl), static_cast<void *>(s->brec), static_cast<void *>(s->ox),
                  static_cast<void *>(s->heads),
                  static_cast<void *>(s->zfound), static_cast<void *>(s->th_list), static_cast<void *>(s->bm),
                  static_cast<void *>(s->evh), static_cast<void *>(s->seg), static_cast<void *>(s->hx),
                  static_cast<void *>(s->cuts), static_cast<void *>(s->fixm), static_cast<void *>(s->sagg),
                  static_cast<void *>(s->cpart)})
    if (p) (void)hipFree(p);
  radix_free(s->rx);
  delete s;
}

int ct_table_init(CtTable &t, uint32_t cap_log2) {
  ct_table_free(t);
  const uint64_t n = uint64_t(1) << cap_log2;
  hipError_t e = hipMalloc(&t.slots, n * sizeof(CtSlot));
  if (e == hipSuccess) e = hipMemset(t.slots, 0, n * sizeof(CtSlot));
  if (e == hipSuccess) e = hipMalloc(&t.carry, 64);
  if (e == hipSuccess) e = hipMemset(t.carry, 0, 64);
  if (e == hipSuccess) t.stats = reinterpret_cast<unsigned long long *>(t.carry + 2);
  if (e == hipSuccess) e = hipMalloc(&t.touch, n * 8);
  if (e == hipSuccess) e = hipMemset(t.touch, 0xff, n * 8);     // ~0: no live entry
  t.cap_log2 = cap_log2;
  t.seq = 1;
  return e;
}

void ct_table_free(CtTable &t) {
  if (t.slots) (void)hipFree(t.slots);
  if (t.carry) (void)hipFree(t.carry);
  if (t.touch) (void)hipFree(t.touch);
  t.slots = nullptr;
  t.carry = nullptr;
  t.stats = nullptr;
  t.touch = nullptr;
}

#define CT_CHECK(x)                         \
  do {                                      \
    const int e_ = int(x);                  \
    if (e_ != hipSuccess) return int(e_);   \
  } while (0)

// PCN_IPT_DEBUG_CT_KBITS=b (16..30): key buckets of at most b bits, whatever
// the batch size (A/B of fewer sort passes against more bucket collisions)
static uint32_t debug_key_bits() {
  static const uint32_t v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_CT_KBITS");
    const long b = e ? std::strtol(e, nullptr, 10) : 0;
    return b >= 16 && b <= 30 ? static_cast<uint32_t>(b) : 30u;
  }();
  return v;
}

static int grow(CtScratch &s, uint64_t n, uint32_t kbits, bool lab4) {
  if (lab4 && s.ox_cap < n) {                  // only batches with four labels read it
    if (s.ox) CT_CHECK(hipFree(s.ox));
    CT_CHECK(hipMalloc(&s.ox, n * sizeof(ct_u32x4)));
    s.ox_cap = n;
  }
  if (s.cap < n) {
    for (uint32_t **p : {&s.keys, &s.keys2, &s.idx2, &s.hard_list, &s.th_list, &s.lcs}) {
      if (*p) CT_CHECK(hipFree(*p));
      CT_CHECK(hipMalloc(p, n * 4));
    }
    for (uint32_t **p : {&s.cursor, &s.heads}) {
      if (*p) CT_CHECK(hipFree(*p));
      CT_CHECK(hipMalloc(p, heads_cap(n) * 4));
    }
    if (s.pdesc) CT_CHECK(hipFree(s.pdesc));
    CT_CHECK(hipMalloc(&s.pdesc, (n / 64 + 2) * 8));
    CT_CHECK(hipMemset(s.pdesc, 0, (n / 64 + 2) * 8));
    if (s.brec) CT_CHECK(hipFree(s.brec));
    CT_CHECK(hipMalloc(&s.brec, n * sizeof(PackedRec)));
    if (s.fixm) CT_CHECK(hipFree(s.fixm));
    if (s.sagg) CT_CHECK(hipFree(s.sagg));
    CT_CHECK(hipMalloc(&s.fixm, (n / 64 + 2) * 8));
    CT_CHECK(hipMalloc(&s.sagg, (n / 64 / kStaleScanGroups + 3) * 8));
    if (kSeg) {
      if (s.seg) CT_CHECK(hipFree(s.seg));
      if (s.hx) CT_CHECK(hipFree(s.hx));
      if (s.cuts) CT_CHECK(hipFree(s.cuts));
      CT_CHECK(hipMalloc(&s.seg, (seg_count(n) + 1) * sizeof(SegRec)));
      CT_CHECK(hipMalloc(&s.hx, (seg_count(n) + 1) * sizeof(HeadExit)));
      CT_CHECK(hipMalloc(&s.cuts, (seg_count(n) + 1) * 4));
    }
    if (!s.ctl) {
      CT_CHECK(hipMalloc(&s.ctl, kCtlWords * 4));   // the kCtl* words + the walk plan
      CT_CHECK(hipMemset(s.ctl, 0, kCtlWords * 4));
    }
    if (!s.evh) {
      CT_CHECK(hipMalloc(&s.evh, kEvPasses * kEvBins * 4));
      CT_CHECK(hipMemset(s.evh, 0, kEvPasses * kEvBins * 4));
    }
    s.cap = n;
  }
  const uint64_t bmb = (uint64_t(1) << kbits) / 8;
  if (s.bm_bytes < bmb) {
    if (s.bm) CT_CHECK(hipFree(s.bm));
    CT_CHECK(hipMalloc(&s.bm, bmb));
    CT_CHECK(hipMemset(s.bm, 0, bmb));          // zero from here on: ct_heads clears what a batch set
    s.bm_bytes = bmb;
  }
  return hipSuccess;
}

// The stale ports of a stage A that wrote the walk records (LaunchArgs::ct_pdesc):
// each 64-frame group published its ports word, Local (the ports of its last
// TCP / UDP frame) or None, and the lanes whose records were built without the
// ports the groups before it leave (fixm).  ct_stale_agg gives every run of
// kStaleScanGroups groups the last Local word in it; ct_stale_fix scans each run
// (the last Local word before it from the aggregates, else the batch's carry),
// completes the marked records (devchain.h ct_rec_restale) and advances the
// carry.  No workgroup waits on another, and an all-ICMP batch costs one pass.

__global__ __launch_bounds__(kStaleScanBlock) void ct_stale_agg_kernel(const unsigned long long *pdesc, uint64_t ngroups,
                                                                      unsigned long long *agg, const uint32_t *carry,
                                                                      uint32_t nblk) {
  __shared__ int best;
  if (threadIdx.x == 0) best = -1;
  __syncthreads();
  const uint64_t g0 = blockIdx.x * kStaleScanGroups + uint64_t(threadIdx.x) * kStaleScanPer;
  unsigned long long d[kStaleScanPer];
#pragma unroll
  for (uint32_t k = 0; k < kStaleScanPer; ++k) d[k] = g0 + k < ngroups ? pdesc[g0 + k] : 0ull;
  int pos = -1;
  uint32_t ports = 0;
#pragma unroll
  for (uint32_t k = 0; k < kStaleScanPer; ++k)
    if (((d[k] >> 32) & 3) == kStLocal) {
      pos = static_cast<int>(threadIdx.x * kStaleScanPer + k);
      ports = static_cast<uint32_t>(d[k]);
    }
  if (pos >= 0) atomicMax(&best, pos);
  __syncthreads();
  if (pos >= 0 && pos == best) agg[blockIdx.x] = ct_ports_word(kCtPortsLocal, ports);
  if (threadIdx.x == 0 && best < 0) agg[blockIdx.x] = ct_ports_word(kCtPortsNone, 0);
  if (blockIdx.x == 0 && threadIdx.x == 0) agg[nblk] = *carry;   // ct_stale_fix writes the new carry
}

__global__ __launch_bounds__(kStaleScanBlock) void ct_stale_fix_kernel(const unsigned long long *pdesc,
                                                                      const unsigned long long *fixm, uint64_t ngroups,
                                                                      const unsigned long long *agg, uint32_t nblk,
                                                                      uint32_t *carry, PackedRec *brec, uint32_t *keys,
                                                                      uint32_t sentinel, uint64_t n) {
  __shared__ unsigned long long sv[kStaleScanBlock];
  __shared__ uint32_t cin;
  const uint32_t t = threadIdx.x, lane = t & 63;
  if (t < 64) {   // the ports before this run: the last Local aggregate before it, else the carry
    uint32_t c = static_cast<uint32_t>(agg[nblk]);
    for (int64_t j0 = static_cast<int64_t>(blockIdx.x) - 1; j0 >= 0; j0 -= 64) {
      const int64_t j = j0 - static_cast<int64_t>(lane);
      const unsigned long long a = j >= 0 ? agg[j] : 0ull;
      const uint64_t m = __ballot(j >= 0 && ((a >> 32) & 3) == kStLocal);
      if (m) {   // the lowest lane is the latest run
        c = __shfl(static_cast<uint32_t>(a), __builtin_ctzll(m));
        break;
      }
    }
    if (t == 0) cin = c;
  }
  const uint64_t g0 = blockIdx.x * kStaleScanGroups + uint64_t(t) * kStaleScanPer;
  unsigned long long d[kStaleScanPer];
#pragma unroll
  for (uint32_t k = 0; k < kStaleScanPer; ++k) d[k] = g0 + k < ngroups ? pdesc[g0 + k] : 0ull;
  unsigned long long last = 0;   // this thread's last Local word (0: none)
#pragma unroll
  for (uint32_t k = 0; k < kStaleScanPer; ++k)
    if (((d[k] >> 32) & 3) == kStLocal) last = d[k];
  sv[t] = last;
  __syncthreads();
  // inclusive scan over the threads, the latest Local word winning
  for (uint32_t off = 1; off < kStaleScanBlock; off <<= 1) {
    const unsigned long long v = sv[t], u = t >= off ? sv[t - off] : 0ull;
    __syncthreads();
    if (!v && u) sv[t] = u;
    __syncthreads();
  }
  const unsigned long long pre = t ? sv[t - 1] : 0ull;
  uint32_t run = pre ? static_cast<uint32_t>(pre) : cin;
  unsigned long long fm[kStaleScanPer];   // (all loaded before the first is used)
#pragma unroll
  for (uint32_t k = 0; k < kStaleScanPer; ++k) fm[k] = g0 + k < ngroups ? fixm[g0 + k] : 0ull;
#pragma unroll
  for (uint32_t k = 0; k < kStaleScanPer; ++k) {
    const uint64_t g = g0 + k;
    for (unsigned long long m = fm[k]; m; m &= m - 1) {
      const uint64_t f = g * 64 + static_cast<uint64_t>(__builtin_ctzll(m));
      if (f >= n) break;
      PackedRec r = load_prec(&brec[f]);
      if (((r.pfk >> 16) & 0xffu) == kCtKErr) continue;   // keys on the quoted header (no stale ports)
      keys[f] = ct_rec_restale(r.src, r.dst, r.ports, r.pfk, run, sentinel);
      brec[f].ports = r.ports;
      brec[f].pfk = r.pfk;
    }
    if (((d[k] >> 32) & 3) == kStLocal) run = static_cast<uint32_t>(d[k]);
  }
  if (blockIdx.x == nblk - 1 && t == kStaleScanBlock - 1) *carry = run;   // the ports the batch leaves
}

// The carry alone: the ports of the batch's last frame that wrote them.
// Workgroup g takes the g-th block of frames counting from the end and stops
// once a later block has found one, so a batch that ends in TCP/UDP costs one
// wave of blocks, not a pass over the batch.  found = 1 + that frame's index.
__global__ void tail_ports_kernel(CtBatch b, unsigned long long *found) {
  __shared__ uint32_t best;
  __shared__ int stop;
  const uint64_t B = blockDim.x;
  for (uint64_t blk = blockIdx.x; blk * B < b.n; blk += gridDim.x) {
    const uint64_t hi = b.n - blk * B;                     // this block: frames [hi - B, hi)
    if (threadIdx.x == 0) {
      best = 0;
      stop = __hip_atomic_load(found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > hi;
    }
    __syncthreads();
    if (stop) return;                                      // uniform: a later frame has them
    if (threadIdx.x < hi) {
      const uint64_t i = hi - 1 - threadIdx.x;
      uint32_t w[18], L;
      load_window(b, i, w, L);
      const Parsed p = parse(w, L, b.hook);
      if (p.status == 2 && p.ports_ok) atomicMax(&best, static_cast<uint32_t>(B - threadIdx.x));
    }
    __syncthreads();
    const uint32_t got = best;                             // B - t of the latest frame t
    if (got) {
      if (threadIdx.x == 0) atomicMax(found, static_cast<unsigned long long>(hi - (B - got)));
      return;
    }
    __syncthreads();                                       // best / stop are rewritten next round
  }
}

__global__ void tail_carry_kernel(CtBatch b, const unsigned long long *found, uint32_t *carry) {
  if (threadIdx.x != 0 || blockIdx.x != 0 || !*found) return;
  uint32_t w[18], L;
  load_window(b, *found - 1, w, L);
  const Parsed p = parse(w, L, b.hook);
  *carry = uint32_t(p.sport) | (uint32_t(p.dport) << 16);
}

int ct_advance_carry(const CtBatch &b, CtScratch &s, uint32_t *carry, int num_cus, void *stream) {
  if (b.n == 0) return hipSuccess;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!s.zfound) CT_CHECK(hipMalloc(&s.zfound, 64));
  CT_CHECK(hipMemsetAsync(s.zfound, 0, 8, st));
  const unsigned blk = 256;
  const unsigned grid = static_cast<unsigned>(std::min<uint64_t>((b.n + blk - 1) / blk, uint64_t(num_cus) * 4));
  hipLaunchKernelGGL(tail_ports_kernel, dim3(grid), dim3(blk), 0, st, b, s.zfound);
  CT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(tail_carry_kernel, dim3(1), dim3(64), 0, st, b, s.zfound, carry);
  CT_CHECK(hipGetLastError());
  return hipSuccess;
}

// key buckets: 2^kbits >= n (a 2^24 batch sorts 24-bit keys in three 8-bit
// passes; 2^kbits >= 2n gave 25 bits and a 9-bit first pass, +20 us, for half
// the bucket collisions between connections, which the walk takes in passes)
#ifndef PCN_CT_KEY_SLACK
#define PCN_CT_KEY_SLACK 1
#endif
static uint32_t key_bits(uint64_t n) {
  uint32_t kbits = 8;
  while (kbits < 30 && (uint64_t(1) << kbits) < PCN_CT_KEY_SLACK * n) ++kbits;
  return std::min(kbits, debug_key_bits());
}

int ct_prep_buffers(CtScratch &s, uint64_t n, uint32_t **brec, uint32_t **keys, uint32_t **lcs, uint32_t *sentinel,
                    unsigned long long **pdesc, unsigned long long **fixm) {
  if (n == 0 || n >= 0x7FFFFFFFull) return int(hipErrorInvalidValue);
  const uint32_t kbits = key_bits(n);
  CT_CHECK(grow(s, n, kbits, false));
  *brec = reinterpret_cast<uint32_t *>(s.brec);
  *keys = s.keys;
  *lcs = s.lcs;
  *sentinel = (1u << kbits) - 1;
  *pdesc = s.pdesc;
  *fixm = s.fixm;
  return hipSuccess;
}

int ct_run(const CtBatch &b, CtTable &t, CtScratch &s, int num_cus, void *stream, bool prepped) {
  if (b.n == 0) return hipSuccess;
  if (b.n >= 0x7FFFFFFFull) return int(hipErrorInvalidValue);   // 32-bit item indices (radix.hip)
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t kbits = key_bits(b.n);
  const uint32_t sentinel = (1u << kbits) - 1;
  CT_CHECK(grow(s, b.n, kbits, b.nlab == 4));
  const unsigned blk = 256, grid = grid_for(b.n, blk, num_cus);
  // one memset for the control words (long echo replies, run counts per
  // class, ct_prep's chunk counter, ...; kCtl*): each memset is a launch of
  // its own (~5 us between kernels)
  // ctl's first kCtlZero words and the ports descriptors are zero: from their
  // allocation, then from the previous batch's ct_count; only a batch that
  // returned early with an error leaves them to memsets here
  // (a prepped batch's stage A has written every group's ports word already)
  if (s.dirty) {
    CT_CHECK(hipMemsetAsync(s.ctl, 0, kCtlZero * 4, st));
    if (!prepped) CT_CHECK(hipMemsetAsync(s.pdesc, 0, (s.cap / 64 + 2) * 8, st));
    CT_CHECK(hipMemsetAsync(s.bm, 0, s.bm_bytes, st));
  }
  s.dirty = true;
  if (prepped) {
    // the records stage A built before the ports the earlier groups leave were
    // known, completed; the carry advanced
    const uint64_t ngroups = (b.n + 63) / 64;
    const uint32_t nblk = static_cast<uint32_t>((ngroups + kStaleScanGroups - 1) / kStaleScanGroups);
    hipLaunchKernelGGL(ct_stale_agg_kernel, dim3(nblk), dim3(kStaleScanBlock), 0, st, s.pdesc, ngroups, s.sagg, t.carry,
                       nblk);
    CT_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ct_stale_fix_kernel, dim3(nblk), dim3(kStaleScanBlock), 0, st, s.pdesc, s.fixm, ngroups, s.sagg,
                       nblk, t.carry, s.brec, s.keys, sentinel, b.n);
    CT_CHECK(hipGetLastError());
  }
  if (!prepped) {
    const uint32_t pchunk = prep_chunk(b.n, num_cus);
    const unsigned pgrid = static_cast<unsigned>(std::min<uint64_t>(uint64_t(num_cus) * 8, (b.n + pchunk - 1) / pchunk));
    hipLaunchKernelGGL(ct_prep_kernel, dim3(pgrid), dim3(kPrepBlock), 0, st, b, t.carry, s.brec, s.ox, s.lcs, s.keys,
                       kbits, s.ctl + kCtlHard, s.hard_list, s.pdesc, s.ctl + kCtlChunk, pchunk);
    CT_CHECK(hipGetLastError());
  }
  // long echo replies join their own key's run unless their quoted key's
  // bucket is in the batch (each kernel returns at once without replies)
  // (a prepped batch has none: its frames are shorter than 70 bytes, and
  // neither these two kernels nor ct_tail are launched for it)
  const uint64_t bm_words = (uint64_t(1) << kbits) / 32;
  if (!prepped) {
    hipLaunchKernelGGL(ct_hbits_set_kernel, dim3(grid), dim3(blk), 0, st, b.n, s.ctl, s.keys, s.hard_list, s.brec, s.bm,
                       sentinel);
    CT_CHECK(hipGetLastError());
    hipLaunchKernelGGL(ct_hard_split_kernel, dim3(grid), dim3(blk), 0, st, s.ctl, s.hard_list, s.brec, s.keys, s.bm,
                       sentinel, s.th_list);
    CT_CHECK(hipGetLastError());
  }
  // (ct_heads advances the carry from ct_prep's published groups)
  // the sort (radix.hip; s.keys is its ping-pong buffer from here on)
  CT_CHECK(radix_sort_pairs(s.rx, s.keys, s.keys2, s.idx2, b.n, kbits, num_cus, st));
  const RecSrc src{s.brec, s.idx2, s.keys2, s.ox, b.nlab == 4 ? 1u : 0u};
  const uint32_t hper = heads_per(b.n, num_cus);
  const uint64_t htile = uint64_t(hper) * kHeadsBlock;
  hipLaunchKernelGGL(ct_heads_kernel, dim3(static_cast<unsigned>((b.n + htile - 1) / htile)), dim3(kHeadsBlock), 0, st,
                     b.n, s.keys2, s.heads, s.ctl + kCtlClass, sentinel, hper, prepped ? nullptr : s.pdesc, t.carry, s.cuts,
                     s.ctl + kCtlSegN, s.ctl + kCtlHard, s.bm, bm_words);
  CT_CHECK(hipGetLastError());
  // (the walk plan is computed on the device from ct_heads' counts, in the walk
  // itself: no read-back, the stream stays asynchronous)
  // the cuts of long runs, then the plan's upper bound
  const uint32_t nseg = seg_waves(b.n, num_cus);
  const unsigned wgrid = static_cast<unsigned>(nseg + b.n / 64 + kRunClasses + 1);
  hipLaunchKernelGGL(ct_walk_kernel, dim3(wgrid), dim3(64), 0, st, b, t, src, s.heads, s.ctl, s.cursor,
                     s.keys2, sentinel, s.seg, s.hx, s.cuts, nseg);
  CT_CHECK(hipGetLastError());
  if (kSeg) {
    hipLaunchKernelGGL(ct_seg_fix_kernel, dim3(nseg), dim3(64), 0, st, b, t, src, s.keys2, s.seg, s.hx,
                       s.cursor, s.ctl, s.cuts);
    CT_CHECK(hipGetLastError());
  }
  if (!prepped) {   // (the long echo replies the walk cannot take: none in a prepped batch)
    hipLaunchKernelGGL(ct_tail_kernel, dim3(1), dim3(64), 0, st, b, t, src, s.brec, s.heads, s.ctl, s.th_list,
                       s.cursor);
    CT_CHECK(hipGetLastError());
  }
  if (t.max_entries) {                         // LRU down to max_entries (no read-back either)
    const uint64_t cap = uint64_t(1) << t.cap_log2;
    // few workgroups: each one's merge and finish atomics land on the same few
    // addresses, which serialise at ~0.1 us apiece (256 workgroups: 69 us a pass)
    const unsigned pgrid2 = static_cast<unsigned>(std::min<uint64_t>(cap / (4 * kEvBlock) + 1, 32));
    for (int p = 0; p < kEvPasses; ++p) {
      hipLaunchKernelGGL(ct_ev_pass_kernel, dim3(pgrid2), dim3(kEvBlock), 0, st, t, s.ctl, s.evh, p);
      CT_CHECK(hipGetLastError());
    }
    // one workgroup per CU (a 2^20-slot table: 4 stamps a thread, one round)
    const unsigned egrid = static_cast<unsigned>(std::min<uint64_t>(cap / kEvictBlock + 1, uint64_t(num_cus)));
    hipLaunchKernelGGL(ct_ev_evict_kernel, dim3(egrid), dim3(kEvictBlock), 0, st, t, s.ctl, s.evh);
    CT_CHECK(hipGetLastError());
  }
  ++t.seq;                                     // the next batch's touch stamps are newer
  const uint64_t cchunk = count_chunk(b.n, num_cus);
  const unsigned cgrid = static_cast<unsigned>((b.n + cchunk - 1) / cchunk);
  static const bool count_atomic = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_CT_COUNT_ATOMIC");
    return e && e[0] == '1';
  }();
  constexpr uint32_t kCountBins = 4 * (2 + kLdsRules);
  if (!count_atomic && s.cpart_rows < cgrid) {
    if (s.cpart) CT_CHECK(hipFree(s.cpart));
    s.cpart = nullptr;
    s.cpart_rows = 0;
    CT_CHECK(hipMalloc(&s.cpart, uint64_t(cgrid) * kCountBins * 8));
    s.cpart_rows = cgrid;
  }
  const bool cvec = (reinterpret_cast<uintptr_t>(b.rule_ids) | reinterpret_cast<uintptr_t>(s.lcs)) % 16 == 0;
  hipLaunchKernelGGL(cvec ? ct_count_kernel<true> : ct_count_kernel<false>, dim3(cgrid), dim3(kCountBlock), 0, st, b,
                     s.lcs, cchunk, s.ctl, s.pdesc, b.n / 64 + 1, count_atomic ? nullptr : s.cpart);
  CT_CHECK(hipGetLastError());
  if (!count_atomic) {
    hipLaunchKernelGGL(ct_count_reduce_kernel, dim3((kCountBins + 63) / 64), dim3(64 * kCountRedWaves), 0, st, b,
                       s.cpart, cgrid);
    CT_CHECK(hipGetLastError());
  }
  s.dirty = false;
  return hipSuccess;
}

int ct_walk_passes(uint64_t out[2], bool reset) {
  unsigned long long v[2];
  hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_walk_passes), sizeof(v), 0, hipMemcpyDeviceToHost);
  if (e == hipSuccess && reset) {
    const unsigned long long z[2] = {0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_walk_passes), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
  out[0] = v[0];
  out[1] = v[1];
  return static_cast<int>(e);
}

int ct_ae_fixup(const CtBatch &b, void *stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (b.rule_ids && b.n) {
    hipLaunchKernelGGL(ae_rid_kernel, dim3(grid_for(b.n, 256, 256)), dim3(256), 0, st, b);
    CT_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(ae_move_kernel, dim3(1), dim3(64), 0, st, b);
  return int(hipGetLastError());
}

// ---- flow-affinity split (pcn_ipt_flow_owner / pcn_ipt_flow_split) ---------
// The GPU analogue of the NIC's RSS queue choice in front of the reference's
// per-CPU datapath: every packet of a connection goes to one owner, so each
// owner's connection table and Parser state (the per-CPU `packet` struct,
// Iptables_Parser_dp.c:27-37, quirk Q4) see that connection's packets in
// batch order.  The owner hashes the *unordered* IPv4 address pair, which is
// the part of the conntrack key (ConntrackLabel_dp.c:200-228) that is the
// packet's own for every kind: an ICMP error is owned by the connection it
// quotes (its key, :491-529), so RELATED finds the table that holds it.
namespace {

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// Reads only the dwords the owner needs (bytes 12-35, and 52-63 of an ICMP
// error), not parse()'s 72-byte window.  Same field rules as parse()
// (Iptables_Parser_dp.c:94-153, the TC untag).  `vec`: the launch is a
// 16-byte aligned fixed-stride batch whose first 48 bytes of every frame lie
// inside the buffer, read as three 16-byte loads per lane (the scattered
// dword loads run at ~2.4 TB/s on 64-byte frames, limited by requests).
// vec: frame i's first 48 bytes as three 16-byte loads
__device__ __forceinline__ void flow_h12(const CtBatch &b, uint64_t i, uint32_t (&h12)[12]) {
  const uint4 *q = reinterpret_cast<const uint4 *>(b.frames + i * uint64_t(b.stride));
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const uint4 v = q[k];
    h12[4 * k] = v.x; h12[4 * k + 1] = v.y; h12[4 * k + 2] = v.z; h12[4 * k + 3] = v.w;
  }
}
// The owner from frame i's words; vec: h12 holds its first 48 bytes (the
// caller loaded them, so several frames' loads can be in flight together).
__device__ __forceinline__ uint32_t flow_owner_core(const CtBatch &b, uint64_t i, uint32_t nranks, bool vec,
                                                    const uint32_t (&h12)[12]) {
  const uint64_t off = b.offsets ? b.offsets[i] : i * uint64_t(b.stride);
  uint32_t L = b.lens ? b.lens[i] : b.fixed_len;
  const uint64_t base = off & ~uint64_t(3);
  const uint32_t sh = static_cast<uint32_t>(off & 3);
  auto D = [&](uint32_t k) {
    const uint64_t at = base + 4u * k;
    return at + 4 <= b.frames_bytes ? *reinterpret_cast<const uint32_t *>(b.frames + at) : 0u;
  };
  uint32_t s = 0;
  // (vec: word k or k + 1 of h12 chosen by value -- h12[k + s] indexed by the
  // run-time shift, or a select of the two elements as lvalues, put the whole
  // array in scratch: 400 bytes a lane in flow_count)
  auto W = [&](uint32_t k) {
    if (vec && k + 1 < 12) return sel3(s, h12[k], h12[k + 1], h12[k + 1]);
    if (vec && k + s < 12) return h12[11];
    return __builtin_amdgcn_alignbyte(D(k + s + 1), D(k + s), sh);
  };
  if (L < 14) return 0;
  uint32_t et = ((W(3) & 0xff) << 8) | ((W(3) >> 8) & 0xff);
  if (b.hook == PCN_IPT_HOOK_TC && (et == 0x8100 || et == 0x88A8)) {
    if (L < 18) return 0;
    s = 1;
    L -= 4;
    et = ((W(3) & 0xff) << 8) | ((W(3) >> 8) & 0xff);
  }
  if (et != 0x0800 || L < 34) return 0;            // not IPv4, or dropped by the Parser: no state
  const uint32_t w5 = W(5), w7 = W(7);
  const uint8_t proto = static_cast<uint8_t>(w5 >> 24);
  if ((proto == 6 && L < 54) || (proto == 17 && L < 42)) return 0;
  uint32_t a = (W(6) >> 16) | (w7 << 16), c = (w7 >> 16) | (W(8) << 16);
  if (proto == 1 && L >= 70) {
    const uint8_t icmp = static_cast<uint8_t>((W(8) >> 16) & 0xff);
    if (icmp != 0 && icmp != 8 && !(icmp >= 13 && icmp <= 18)) {   // an error: its quoted pair
      const uint32_t w14 = W(14);
      a = (W(13) >> 16) | (w14 << 16);
      c = (w14 >> 16) | (W(15) << 16);
    }
  }
  const uint32_t lo = a < c ? a : c, hi = a < c ? c : a;
  const uint32_t h = fmix32(fmix32(lo ^ 0x9e3779b9u) ^ hi);
  return static_cast<uint32_t>((uint64_t(h) * nranks) >> 32);
}
__device__ __forceinline__ uint32_t flow_owner_of(const CtBatch &b, uint64_t i, uint32_t nranks, bool vec) {
  uint32_t h12[12] = {};
  if (vec) flow_h12(b, i, h12);
  return flow_owner_core(b, i, nranks, vec, h12);
}

__global__ void flow_owner_kernel(CtBatch b, uint32_t nranks, bool vec, uint8_t *owner) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < b.n; i += uint64_t(gridDim.x) * blockDim.x)
    owner[i] = static_cast<uint8_t>(flow_owner_of(b, i, nranks, vec));
}

// Stable compaction of this rank's frames in three passes (a hipCUB
// DeviceSelect over the flags measured 161 us per 2^24 frames; these passes
// touch the flags once more and the outputs once).  A tile is 2048 frames:
// 8 coalesced rounds of 256; order inside a tile comes from wave ballots.
constexpr uint32_t kSplitBlock = 256, kSplitItems = 8, kSplitTile = kSplitBlock * kSplitItems;

__global__ __launch_bounds__(256) void flow_count_kernel(CtBatch b, uint32_t nranks, uint32_t rank, bool vec,
                                                         uint8_t *flag, uint32_t *bcount) {
  __shared__ uint32_t wsum[kSplitBlock / 64];
  const uint64_t tile = uint64_t(blockIdx.x) * kSplitTile;
  uint32_t c = 0;
  // vec: every item's 48 bytes loaded before the first owner is computed
  // (the index clamped into the batch): behind `if (i < n)` and the owner's
  // own branches each item's loads waited for the previous item's owner
  uint32_t h12[kSplitItems][12] = {};
  if (vec) {
#pragma unroll
    for (uint32_t k = 0; k < kSplitItems; ++k) {
      const uint64_t i = tile + k * kSplitBlock + threadIdx.x;
      flow_h12(b, i < b.n ? i : b.n - 1, h12[k]);
    }
  }
#pragma unroll
  for (uint32_t k = 0; k < kSplitItems; ++k) {
    const uint64_t i = tile + k * kSplitBlock + threadIdx.x;
    bool f = false;
    if (i < b.n) {
      f = flow_owner_core(b, i, nranks, vec, h12[k]) == rank;
      flag[i] = f;
    }
    c += __popcll(__ballot(f));
  }
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kSplitBlock / 64; ++w) t += wsum[w];
    bcount[blockIdx.x] = t;
  }
}

// In place: bcount[] -> exclusive prefix; *total = the owned count.  One block.
__global__ __launch_bounds__(1024) void flow_scan_kernel(uint32_t *bcount, uint32_t nb, uint32_t *total) {
  __shared__ uint32_t sm[1024];
  const uint32_t per = (nb + 1023) / 1024, lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint32_t sum = 0;
  for (uint32_t j = lo; j < hi; ++j) sum += bcount[j];
  sm[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint32_t v = threadIdx.x >= d ? sm[threadIdx.x - d] : 0u;
    __syncthreads();
    sm[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = sm[threadIdx.x] - sum;
  for (uint32_t j = lo; j < hi; ++j) {
    const uint32_t c = bcount[j];
    bcount[j] = run;
    run += c;
  }
  if (threadIdx.x == 1023) *total = sm[1023];
}

// Owned frames as an offsets/lens/in_port batch, in batch order.
__global__ __launch_bounds__(256) void flow_write_kernel(CtBatch b, const uint8_t *flag, const uint32_t *bstart,
                                                         const uint16_t *in_port, uint16_t const_in_port,
                                                         uint32_t *index, uint32_t *offsets, uint16_t *lens,
                                                         uint16_t *in_port_out) {
  __shared__ uint32_t wsum[kSplitBlock / 64];
  const uint64_t tile = uint64_t(blockIdx.x) * kSplitTile;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t base = bstart[blockIdx.x];
  uint8_t fl[kSplitItems];   // every round's flag loaded at once (index clamped, masked below)
#pragma unroll
  for (uint32_t k = 0; k < kSplitItems; ++k) {
    const uint64_t i = tile + k * kSplitBlock + threadIdx.x;
    fl[k] = flag[i < b.n ? i : b.n - 1];
  }
#pragma unroll
  for (uint32_t k = 0; k < kSplitItems; ++k) {
    const uint64_t i = tile + k * kSplitBlock + threadIdx.x;
    const bool f = i < b.n && fl[k];
    const uint64_t m = __ballot(f);
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    uint32_t pre = base, tot = 0;
    for (uint32_t w = 0; w < kSplitBlock / 64; ++w) {
      if (w < wave) pre += wsum[w];
      tot += wsum[w];
    }
    if (f) {
      const uint32_t at = pre + __popcll(m & ((uint64_t(1) << lane) - 1));
      index[at] = static_cast<uint32_t>(i);
      offsets[at] = b.offsets ? b.offsets[i] : static_cast<uint32_t>(i * b.stride);
      lens[at] = b.lens ? b.lens[i] : static_cast<uint16_t>(b.fixed_len);
      if (in_port_out) in_port_out[at] = in_port ? in_port[i] : const_in_port;
    }
    base += tot;
    __syncthreads();
  }
}

bool flow_vec(const CtBatch &b) {
  return !b.offsets && b.stride % 16 == 0 && b.stride >= 48 && (reinterpret_cast<uintptr_t>(b.frames) % 16) == 0 &&
         (b.n - 1) * uint64_t(b.stride) + 48 <= b.frames_bytes;
}

}  // namespace

int ct_flow_owner(const CtBatch &b, uint32_t nranks, uint8_t *owner, int num_cus, void *stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!b.n) return 0;
  hipLaunchKernelGGL(flow_owner_kernel, dim3(grid_for(b.n, 256, num_cus)), dim3(256), 0, st, b, nranks, flow_vec(b), owner);
  return int(hipGetLastError());
}

int ct_flow_split(const CtBatch &b, const uint16_t *in_port, uint16_t const_in_port, uint32_t nranks, uint32_t rank,
                  uint32_t *index, uint32_t *offsets, uint16_t *lens, uint16_t *in_port_out, uint64_t *n_out,
                  int num_cus, void *stream) {
  (void)num_cus;
  hipStream_t st = static_cast<hipStream_t>(stream);
  *n_out = 0;
  if (!b.n) return 0;
  const uint64_t nb = (b.n + kSplitTile - 1) / kSplitTile;
  const size_t head = (b.n + 255) / 256 * 256;      // flags, then the tile counts, then the total
  uint8_t *buf = nullptr;
  CT_CHECK(hipMallocAsync(reinterpret_cast<void **>(&buf), head + nb * 4 + 256, st));
  uint8_t *flag = buf;
  uint32_t *bcount = reinterpret_cast<uint32_t *>(buf + head);
  uint32_t *total = bcount + nb;
  const bool vec = flow_vec(b);
  hipLaunchKernelGGL(flow_count_kernel, dim3(unsigned(nb)), dim3(kSplitBlock), 0, st, b, nranks, rank, vec, flag,
                     bcount);
  int e = int(hipGetLastError());
  if (e == hipSuccess) {
    hipLaunchKernelGGL(flow_scan_kernel, dim3(1), dim3(1024), 0, st, bcount, uint32_t(nb), total);
    e = int(hipGetLastError());
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(flow_write_kernel, dim3(unsigned(nb)), dim3(kSplitBlock), 0, st, b, flag, bcount, in_port,
                       const_in_port, index, offsets, lens, in_port_out);
    e = int(hipGetLastError());
  }
  uint32_t m = 0;
  if (e == hipSuccess) e = int(hipMemcpyAsync(&m, total, 4, hipMemcpyDeviceToHost, st));
  const int f = int(hipFreeAsync(buf, st));
  if (e == hipSuccess) e = int(hipStreamSynchronize(st));
  if (e == hipSuccess) e = f;
  if (e == hipSuccess) *n_out = m;
  return e;
}

}  // namespace pcn

#if PCN_CT_DBG_T
// measurement builds only (tools/walk_times.py): the walk's per-block clocks
extern "C" int pcn_ipt_dbg_walk_times(unsigned long long *out, size_t words) {
  if (words > 4 * size_t(pcn::kDbgWaves)) words = 4 * size_t(pcn::kDbgWaves);
  return int(hipMemcpyFromSymbol(out, HIP_SYMBOL(pcn::g_walk_t), words * 8));
}
extern "C" int pcn_ipt_dbg_walk_clear() {
  static unsigned long long zero[4 * pcn::kDbgWaves];
  return int(hipMemcpyToSymbol(HIP_SYMBOL(pcn::g_walk_t), zero, sizeof(zero)));
}
#endif
