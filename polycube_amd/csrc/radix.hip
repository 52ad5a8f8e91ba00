// radix.hip — the stateful pipeline's sort (radix.hpp): stable LSD radix sort
// of (key bucket, batch index) pairs, hand-written for gfx950, reduce-then-scan.
//
// Each digit pass (8 / 8 / 8 bits of a 2^24 batch's 24-bit key; up to 9 bits a
// pass) splits its input into one contiguous super-tile per CU (a whole
// number of 8192-item sub-tiles), and runs three kernels over the same split:
// 1. radix_up_kernel: each half super-tile's count of every digit (two
//    workgroups a super-tile, two per CU, so one's loads overlap the other's
//    LDS adds: 31 -> 26 us a pass; the all-ones digit -- the batch's "no
//    table" bucket, often most keys -- wave-aggregated), cnt[row][512];
// 2. radix_colscan_kernel: per digit the exclusive prefix over super-tiles,
//    pre[b][d], and the digit's total, tot[d] (16 digits a workgroup, the rows
//    in 64 slices: 5 us at 512 rows);
// 3. radix_pass_kernel: the digits' global starts (an exclusive scan of tot),
//    then the super-tile's sub-tiles in order: each ranked wave by wave and
//    slot by slot in input order (lanes of one digit matched with `bits`
//    ballots, each digit's leader adding the slot's count to the wave's LDS
//    counter with one returning atomic), ordered by digit in LDS and written
//    out (consecutive items of a digit to consecutive addresses), the running
//    per-digit bases advanced in LDS.  The first pass makes the values (batch
//    indices) itself.
// No workgroup waits on another (no look-back, tile claims or spin), and the
// digit totals come from the counts, so there is no histogram kernel.
// Stability: a sub-tile's items keep input order within a digit (wave, slot,
// lane order is input order), sub-tiles and super-tiles are placed in order.
//
// A onesweep version (one histogram kernel, then per digit one kernel whose
// tiles summed their predecessors' counts by decoupled look-back) measured
// 161 us a pass against this one's 136 (up 30 + scan 6 + pass 100): its
// look-back chains cost 52 us a pass (profiles/r05_s7, r05_s8, r05_s11).
#include "radix.hpp"

#include <algorithm>
#include <cstdlib>

namespace pcn {
namespace {

constexpr uint32_t kRBlock = 1024;                 // workgroups: one per CU (100 KB of LDS, ~128 VGPRs)
constexpr uint32_t kRItems = 8;
constexpr uint32_t kRTile = kRBlock * kRItems;     // 8192 pairs a sub-tile
constexpr uint32_t kRWaves = kRBlock / 64;         // 16
constexpr uint32_t kRMaxBits = 9;
constexpr uint32_t kRMaxBins = 1u << kRMaxBits;    // 512 (<= kRBlock: one thread per digit)
// dynamic LDS of a pass: per-wave digit counts, digit starts and bases, scan
// scratch, the sub-tile's keys and values ordered by digit
constexpr uint32_t kPassLds = kRWaves * kRMaxBins * 4 + (2 * kRMaxBins + kRWaves) * 4 + 2 * kRTile * 4;
static_assert(kRMaxBins <= kRBlock, "one thread per digit");

constexpr uint32_t kRMaxPass = 4;                  // keys of up to 36 bits
#ifndef PCN_RADIX_UNI_ROUNDS
#define PCN_RADIX_UNI_ROUNDS 4   // the up-sweep's last pass: equal-digit vectors aggregated (0: off, A/B)
#endif

struct Digits {
  uint32_t npass;
  uint32_t shift[kRMaxPass], bits[kRMaxPass];
};

Digits digits_for(uint32_t kbits) {
  Digits d{};
  if (kbits == 0) kbits = 1;
  d.npass = (kbits + kRMaxBits - 1) / kRMaxBits;
  uint32_t left = kbits, sh = 0;
  for (uint32_t p = 0; p < d.npass; ++p) {
    const uint32_t b = (left + (d.npass - p) - 1) / (d.npass - p);
    d.shift[p] = sh;
    d.bits[p] = b;
    sh += b;
    left -= b;
  }
  return d;
}

// Exclusive prefix over the block's threads (one value each); waves scan their
// 64 values with lane shuffles, then the wave totals.  Two barriers.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t *wtot) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= static_cast<uint32_t>(o)) inc += y;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (uint32_t k = 0; k < kRWaves; ++k) before += k < w ? wtot[k] : 0u;
  __syncthreads();
  return before + inc - x;
}

// SUB workgroups share a super-tile, each counting 1 / SUB of it into a row of
// its own (cnt[b * SUB + part]; the column scan sums them): two per CU overlap
// one's loads with the other's LDS atomics.
template <uint32_t U, uint32_t SUB>
__global__ __launch_bounds__(kRBlock) void radix_up_kernel(const uint32_t *kin, uint64_t n, uint32_t shift,
                                                               uint32_t bits, uint64_t per, uint32_t *cnt,
                                                               uint32_t runs) {
  __shared__ uint32_t h[kRMaxBins];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t dmask = (1u << bits) - 1;
  if (tid < kRMaxBins) h[tid] = 0;
  __syncthreads();
  const uint64_t sper = per / SUB;   // (per: a multiple of 8192)
  const uint64_t lo = uint64_t(blockIdx.x / SUB) * per + (blockIdx.x % SUB) * sper;
  const uint64_t hi = lo + sper < n ? lo + sper : n > lo ? n : lo;   // (a part past the end: empty)
  // Lanes of one digit add together, by their leader: the all-ones digit (the
  // "no table" bucket) and, in the last pass (`runs`), the first other lane's
  // digit; the rest lane by lane.  The last pass reads keys sorted by every
  // lower bit, where each connection's packets are one run of equal keys:
  // lane by lane, a wave's 64 adds went to one or two bins (45 us against
  // 21-24 for the other passes, where the extra ballots cost 7 us a pass).
  auto add = [&](uint32_t k, bool v) {
    const uint32_t dk = (k >> shift) & dmask;
    const uint64_t hm = __ballot(v && dk == dmask);
    if (hm && lane == static_cast<uint32_t>(__builtin_ctzll(hm)))
      atomicAdd(&h[dmask], static_cast<uint32_t>(__builtin_popcountll(hm)));
    if (!runs) {
      if (v && dk != dmask) atomicAdd(&h[dk], 1u);
      return;
    }
    const uint64_t rest = __ballot(v && dk != dmask);
    if (!rest) return;
    const uint32_t l0 = static_cast<uint32_t>(__builtin_ctzll(rest));
    const uint32_t d0 = static_cast<uint32_t>(__shfl(static_cast<int>(dk), static_cast<int>(l0)));
    const uint64_t m0 = __ballot(v && dk == d0);
    if (lane == l0) atomicAdd(&h[d0], static_cast<uint32_t>(__builtin_popcountll(m0)));
    if (v && dk != dmask && dk != d0) atomicAdd(&h[dk], 1u);
  };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // U 16-byte loads in flight per thread; lo is a multiple of 4096: 16-byte aligned.  The whole 16-byte vectors
  // [lo, hi4) are read with unconditional loads (the index clamped, the lanes
  // past the range masked): a conditional load merges into a phi the compiler
  // resolves with an immediate vmcnt(0), one round trip per load.  The last
  // 0-3 keys of an unaligned end are added by the first lanes.
  const uint64_t lo4 = lo / 4, hi4 = hi / 4;
  constexpr uint64_t kStep = uint64_t(kRBlock) * U;
  const u32x4 *const kv = reinterpret_cast<const u32x4 *>(kin);
  auto load = [&](u32x4 *k4, uint64_t base) {
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t q = base + u * kRBlock + tid;
      k4[u] = kv[q < hi4 ? q : hi4 - 1];
    }
  };
  // The last pass (`runs`): a lane's four keys are mostly one digit (a run),
  // and so are most lanes of a wave: the lanes whose four digits are equal add
  // 4 x their count once per distinct digit (up to kUniRounds digits a vector
  // slot; lanes left over, and the others, key by key as before).
  constexpr int kUniRounds = PCN_RADIX_UNI_ROUNDS;
  auto count = [&](const u32x4 *k4, uint64_t base) {
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      bool v = base + u * kRBlock + tid < hi4;
      if (kUniRounds > 0 && runs) {
        const uint32_t dx = (k4[u].x >> shift) & dmask;
        const bool uni = v && dx == ((k4[u].y >> shift) & dmask) && dx == ((k4[u].z >> shift) & dmask) &&
                         dx == ((k4[u].w >> shift) & dmask);
        uint64_t left = __ballot(uni);
        for (int it = 0; it < kUniRounds && left; ++it) {   // (wave-uniform)
          const uint32_t l0 = static_cast<uint32_t>(__builtin_ctzll(left));
          const uint32_t d0 = static_cast<uint32_t>(__shfl(static_cast<int>(dx), static_cast<int>(l0)));
          const uint64_t m0 = __ballot(uni && dx == d0);
          if (lane == l0) atomicAdd(&h[d0], 4u * static_cast<uint32_t>(__builtin_popcountll(m0)));
          left &= ~m0;
        }
        v = v && (!uni || ((left >> lane) & 1));
      }
      add(k4[u].x, v);
      add(k4[u].y, v);
      add(k4[u].z, v);
      add(k4[u].w, v);
    }
  };
  // A round is U loads per thread, all in flight together (256 KB a CU:
  // a 2^24-key batch is one round per workgroup).  Double-buffered rounds
  // measured no better: the compiler drains the loads a loop carries at the
  // loop head anyway.
  for (uint64_t base = lo4; base < hi4; base += kStep) {   // uniform per workgroup
    u32x4 k4[U];
    load(k4, base);
    count(k4, base);
  }
  {
    const uint64_t i = hi4 * 4 + tid;   // (uniform call: add() ballots)
    const bool v = tid < 64 && i < hi;
    add(v ? kin[v ? i : lo] : 0u, v);
  }
  __syncthreads();
  if (tid < kRMaxBins) cnt[uint64_t(blockIdx.x) * kRMaxBins + tid] = h[tid];
}

static uint32_t up_sub() {   // PCN_IPT_DEBUG_RADIX_UP_SUB=1|2: workgroups per super-tile in the up-sweep (A/B)
  static const uint32_t v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_RADIX_UP_SUB");
    return e && e[0] == '1' ? 1u : 2u;
  }();
  return v;
}

// 16 digits a workgroup; the rows (sub per super-tile) in 64 slices, lane l of
// wave w taking digit l % 16 of slice 4w + l / 16: each slice's sum, their
// exclusive prefix in LDS, then each slice's rows again with the running
// prefix (pre is written per super-tile, at its first row).  The rows of a
// slice are read R at a time, their loads in flight together (unconditional,
// the row clamped and masked).  (64 digits a workgroup over 16 wave-slices,
// one round trip per row: 7.5 us a scan at 256 rows, 12.4 at 512.)
constexpr uint32_t kScanDigits = 16, kScanSlices = kRBlock / kScanDigits;   // 64
__global__ __launch_bounds__(kRBlock) void radix_colscan_kernel(const uint32_t *cnt, uint32_t *pre, uint32_t *tot,
                                                                 uint32_t groups, uint32_t nb, uint32_t sub) {
  __shared__ uint32_t part[kScanSlices][kScanDigits];
  const uint32_t dl = threadIdx.x % kScanDigits, sl = threadIdx.x / kScanDigits;
  const uint32_t d = blockIdx.x * kScanDigits + dl;
  const uint32_t rps = (groups + kScanSlices - 1) / kScanSlices;
  const uint32_t lo = sl * rps < groups ? sl * rps : groups, hi = lo + rps < groups ? lo + rps : groups;
  constexpr uint32_t R = 8;
  const uint32_t dd = d < nb ? d : 0;
  auto chunk = [&](uint32_t *x, uint32_t b0) {
#pragma unroll
    for (uint32_t j = 0; j < R; ++j) {
      const uint32_t b = b0 + j < hi ? b0 + j : hi - 1;
      x[j] = cnt[uint64_t(b) * kRMaxBins + dd];
    }
  };
  uint32_t sum = 0;
  for (uint32_t b0 = lo; b0 < hi; b0 += R) {
    uint32_t x[R];
    chunk(x, b0);
#pragma unroll
    for (uint32_t j = 0; j < R; ++j) sum += b0 + j < hi ? x[j] : 0u;
  }
  part[sl][dl] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t k = 0; k < sl; ++k) run += part[k][dl];
  if (d < nb && sl == kScanSlices - 1) tot[d] = run + sum;
  for (uint32_t b0 = lo; b0 < hi; b0 += R) {
    uint32_t x[R];
    chunk(x, b0);
#pragma unroll
    for (uint32_t j = 0; j < R; ++j) {
      const uint32_t b = b0 + j;
      if (b >= hi) break;
      if (d < nb && b % sub == 0) pre[uint64_t(b / sub) * kRMaxBins + d] = run;
      run += x[j];
    }
  }
}

// 4 waves per SIMD.  A sub-tile's values and the next sub-tile's keys are
// loaded after its ranking, in flight through its scan; keys and values go
// out in one loop.  On gfx950 vmcnt retires loads and stores in issue order.
// VIN: the values are read (every pass but the first, whose values are the
// indices themselves) -- a template parameter, not a branch: loads on one side
// of a branch and computed values on the other merge into a phi the compiler
// resolves by waiting for the loads at once.
template <bool VIN>
__global__ __launch_bounds__(kRBlock) void radix_pass_kernel(const uint32_t *kin, const uint32_t *vin,
                                                            uint32_t *kout, uint32_t *vout, uint64_t n,
                                                            uint32_t shift, uint32_t bits, uint64_t per,
                                                            const uint32_t *pre, const uint32_t *tot) {
  constexpr uint32_t kW = kRWaves, kTile = kRTile, SB = kRBlock;
  extern __shared__ __attribute__((aligned(16))) uint8_t rsm[];
  uint32_t *const wcnt = reinterpret_cast<uint32_t *>(rsm);   // [wave][digit]
  uint32_t *const dstart = wcnt + kW * kRMaxBins;              // digit's first place in the sub-tile
  uint32_t *const dbase = dstart + kRMaxBins;                  // digit's next place in the output
  uint32_t *const wtot = dbase + kRMaxBins;
  uint32_t *const bufk = wtot + kRWaves;                       // the sub-tile's keys by digit
  uint32_t *const bufv = bufk + kTile;                         // and its values
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nb = 1u << bits, dmask = nb - 1;
  const uint32_t d = tid;
  {
    const uint32_t t = d < nb ? tot[d] : 0u;
    const uint32_t off = block_excl_scan(t, wtot);
    if (d < nb) dbase[d] = off + pre[uint64_t(blockIdx.x) * kRMaxBins + d];
  }
  const uint64_t lo = uint64_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
  uint32_t *const wc = wcnt + w * kRMaxBins;
  // item k of lane l in wave w is the sub-tile's item w * 512 + k * 64 + l
  // (input order)
  const uint32_t li = w * (kRItems * 64) + lane;
  // Buffer loads bounded by the sub-tile (a lane past it reads 0 and is masked
  // everywhere after): no branch, no clamp, the slot in the instruction's
  // offset.  (A conditional load merges into a phi the compiler resolves with
  // an immediate vmcnt(0): a round trip per load.)
  auto load = [&](const uint32_t *src, uint32_t *dst, uint64_t at) {
    // (the descriptor's fields made scalar explicitly, else a waterfall loop per load)
    const uint32_t m = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(hi - at < kTile ? hi - at : kTile));
    const uint64_t base = reinterpret_cast<uintptr_t>(src + at);
    // (readfirstlane returns int: widen through uint32_t, or the low word's
    // sign extends into the high one)
    const uint32_t bhi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base >> 32)));
    const uint32_t blo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base)));
    const uint64_t ub = (static_cast<uint64_t>(bhi) << 32) | blo;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(ub), 0, 4 * m, 0x00020000);
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) dst[k] = __builtin_amdgcn_raw_buffer_load_b32(r, 4 * (li + k * 64), 0, 0);
  };
  uint32_t key[kRItems], nkey[kRItems];
  if (lo < hi) load(kin, key, lo);
  for (uint64_t t0 = lo; t0 < hi; t0 += kTile) {   // uniform per workgroup
    const uint32_t items = static_cast<uint32_t>(hi - t0 < kTile ? hi - t0 : kTile);
    reinterpret_cast<uint4 *>(wcnt)[tid] = uint4{0u, 0u, 0u, 0u};   // kW * 2 KB: 32 bytes a thread
    reinterpret_cast<uint4 *>(wcnt)[tid + SB] = uint4{0u, 0u, 0u, 0u};
    __syncthreads();
    // ranks within the wave, slot by slot in input order: the lanes of one
    // digit matched with `bits` ballots (no LDS), then each digit's leader lane
    // adds the slot's count to the wave's counter with ONE returning LDS
    // atomic per slot, all eight issued back to back (LDS executes a wave's
    // operations in order, so slot k sees slot k - 1's adds), then the bases
    // broadcast from the leaders
    uint32_t pos[kRItems], add[kRItems];   // pos: rank in the slot | leader << 16 until the atomics
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      const bool v = li + k * 64 < items;
      const uint32_t dk = (key[k] >> shift) & dmask;
      uint64_t m = __ballot(v);
      for (uint32_t b = 0; b < bits; ++b) {
        const uint64_t bb = __ballot((dk >> b) & 1);
        m &= ((dk >> b) & 1) ? bb : ~bb;
      }
      const uint32_t leader = m ? static_cast<uint32_t>(__builtin_ctzll(m)) : lane;
      add[k] = v && lane == leader ? static_cast<uint32_t>(__builtin_popcountll(m)) : 0u;
      pos[k] = static_cast<uint32_t>(__builtin_popcountll(m & ((1ull << lane) - 1))) | (leader << 16);
    }
    uint32_t old[kRItems];
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      old[k] = 0;
      if (add[k]) old[k] = atomicAdd(&wc[(key[k] >> shift) & dmask], add[k]);
    }
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k)
      pos[k] = (pos[k] & 0xffffu) + static_cast<uint32_t>(__shfl(old[k], static_cast<int>(pos[k] >> 16)));
    // this sub-tile's values, then the next sub-tile's keys: both in flight
    // through the scan (issued after the ranking, so the wait for this
    // sub-tile's keys above never counts them)
    uint32_t val[kRItems];   // the first pass's values are the indices themselves
    if constexpr (VIN) {
      load(vin, val, t0);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < kRItems; ++k) val[k] = static_cast<uint32_t>(t0) + li + k * 64;   // (n < 2^30)
    }
    if (t0 + kTile < hi) load(kin, nkey, t0 + kTile);
    __syncthreads();
    uint32_t c = 0;   // the sub-tile's count of digit d
    if (d < nb) {
#pragma unroll
      for (uint32_t ww = 0; ww < kW; ++ww) {
        const uint32_t x = wcnt[ww * kRMaxBins + d];
        wcnt[ww * kRMaxBins + d] = c;
        c += x;
      }
    }
    const uint32_t ds = block_excl_scan(c, wtot);
    if (d < nb) dstart[d] = ds;
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      if (li + k * 64 < items) {
        const uint32_t dk = (key[k] >> shift) & dmask;
        const uint32_t p = pos[k] + dstart[dk] + wc[dk];
        bufk[p] = key[k];
        bufv[p] = val[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      const uint32_t j = tid + k * SB;
      if (j < items) {
        const uint32_t kk = bufk[j];
        const uint32_t dk = (kk >> shift) & dmask;
        const uint32_t g = dbase[dk] + (j - dstart[dk]);
        kout[g] = kk;
        vout[g] = bufv[j];
      }
    }
    __syncthreads();                 // every read of dbase / dstart / the buffers done
    if (d < nb) dbase[d] += c;
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) key[k] = nkey[k];
  }
}
}  // namespace

void radix_free(RadixScratch &s) {
  for (void *p : {static_cast<void *>(s.tk), static_cast<void *>(s.tv), static_cast<void *>(s.tv2),
                  static_cast<void *>(s.seg)})
    if (p) (void)hipFree(p);
  s = RadixScratch{};
}

#define RX_CHECK(x)                         \
  do {                                      \
    const hipError_t e_ = (x);              \
    if (e_ != hipSuccess) return int(e_);   \
  } while (0)

int radix_sort_pairs(RadixScratch &s, uint32_t *keys_in, uint32_t *keys_out, uint32_t *vals_out, uint64_t n,
                     uint32_t kbits, int num_cus, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n >= (uint64_t(1) << 30) || kbits > kRMaxPass * kRMaxBits) return int(hipErrorInvalidValue);
  if (s.cap < n) {
    for (uint32_t **p : {&s.tk, &s.tv, &s.tv2}) {
      if (*p) RX_CHECK(hipFree(*p));
      *p = nullptr;
      RX_CHECK(hipMalloc(p, n * 4));
    }
    s.cap = n;
  }
  const Digits dg = digits_for(kbits);
  // ping-pong: the last pass writes the outputs; keys_in doubles as a key buffer
  // pass p reads what pass p - 1 wrote: (tk, tv) and (keys_in, tv2) alternate,
  // the first pass reads keys_in (its values are the indices), the last
  // writes the outputs
  const uint32_t *kin[kRMaxPass], *vin[kRMaxPass];
  uint32_t *kout[kRMaxPass], *vout[kRMaxPass];
  for (uint32_t p = 0; p < dg.npass; ++p) {
    kin[p] = p == 0 ? keys_in : kout[p - 1];
    vin[p] = p == 0 ? nullptr : vout[p - 1];
    const bool last = p + 1 == dg.npass;
    kout[p] = last ? keys_out : (p % 2 == 0 ? s.tk : keys_in);
    vout[p] = last ? vals_out : (p % 2 == 0 ? s.tv : s.tv2);
  }
  // super-tiles of whole sub-tiles, one workgroup per CU
  const uint64_t g0 = std::max<uint64_t>(1, uint64_t(num_cus > 0 ? num_cus : 1));
  const uint64_t subs = (n + kRTile - 1) / kRTile;
  const uint64_t per = (subs + g0 - 1) / g0 * kRTile;
  const uint32_t groups = static_cast<uint32_t>((n + per - 1) / per);
  constexpr uint32_t kMaxSub = 2;
  const uint32_t sub = up_sub();
  if (s.seg_groups < groups) {
    if (s.seg) RX_CHECK(hipFree(s.seg));
    s.seg = nullptr;
    RX_CHECK(hipMalloc(&s.seg, ((kMaxSub + 1) * uint64_t(groups) + 1) * kRMaxBins * 4));
    s.seg_groups = groups;
  }
  uint32_t *const cnt = s.seg, *const pre = cnt + uint64_t(groups) * kMaxSub * kRMaxBins;
  uint32_t *const tot = pre + uint64_t(groups) * kRMaxBins;
  for (uint32_t p = 0; p < dg.npass; ++p) {
    const uint32_t nb = 1u << dg.bits[p];
    const uint32_t runs = p > 0 && p + 1 == dg.npass ? 1u : 0u;
    if (sub == 2)
      hipLaunchKernelGGL((radix_up_kernel<8, 2>), dim3(2 * groups), dim3(kRBlock), 0, st, kin[p], n, dg.shift[p],
                         dg.bits[p], per, cnt, runs);
    else
      hipLaunchKernelGGL((radix_up_kernel<16, 1>), dim3(groups), dim3(kRBlock), 0, st, kin[p], n, dg.shift[p],
                         dg.bits[p], per, cnt, runs);
    RX_CHECK(hipGetLastError());
    hipLaunchKernelGGL(radix_colscan_kernel, dim3((nb + kScanDigits - 1) / kScanDigits), dim3(kRBlock), 0, st, cnt,
                       pre, tot, sub * groups, nb, sub);
    RX_CHECK(hipGetLastError());
    if (vin[p])
      hipLaunchKernelGGL(radix_pass_kernel<true>, dim3(groups), dim3(kRBlock), kPassLds, st, kin[p], vin[p], kout[p],
                         vout[p], n, dg.shift[p], dg.bits[p], per, pre, tot);
    else
      hipLaunchKernelGGL(radix_pass_kernel<false>, dim3(groups), dim3(kRBlock), kPassLds, st, kin[p], vin[p], kout[p],
                         vout[p], n, dg.shift[p], dg.bits[p], per, pre, tot);
    RX_CHECK(hipGetLastError());
  }
  return hipSuccess;
}

}  // namespace pcn
