// radix.hip — the stateful pipeline's sort (radix.hpp): stable LSD radix sort
// of (key bucket, batch index) pairs, hand-written for gfx950.
//
// 1. radix_hist_kernel: one read of the keys, every pass's digit histogram at
//    once (LDS histograms, one global add per non-empty bin and workgroup into
//    one of 16 copies; the keys of packets that need no table -- one "hot"
//    bucket, often most of a batch -- wave-aggregated).
// 2. radix_scan_kernel: the global exclusive prefix of each digit's bins (the
//    copies summed), and the histograms zeroed for the next sort.
// 3. radix_pass_kernel, once per digit (9 / 8 / 8 bits of a 25-bit key): a
//    tile of 8192 pairs per 1024-thread workgroup (one per CU), claimed in
//    start order.  Its items are ranked wave by wave and slot by
//    slot in input order (lanes of one digit matched with `bits` ballots, a
//    per-wave running count in LDS), the tile's digit counts -- counted
//    first, before the ranking -- are published and the counts of the tiles
//    before it summed by decoupled look-back (one u64
//    per tile and digit: epoch, aggregate / inclusive flag, count; 16 earlier
//    tiles read at once -- read one by one, the chain of dependent reads of
//    the first tiles, which all start together, was the pass's time), then
//    the tile is ordered by digit in LDS and written
//    out: consecutive items of a digit go to consecutive addresses.  The first
//    pass makes the values (batch indices) itself.
// Stability: a tile's items keep input order within a digit (wave, slot, lane
// order is input order), and tiles are placed in tile order.
#include "radix.hpp"

#include <algorithm>
#include <cstdlib>
#include <string>

namespace pcn {
namespace {

constexpr uint32_t kRBlock = 1024;                 // pass workgroups: one per CU (88 KB of LDS)
constexpr uint32_t kRItems = 8;
constexpr uint32_t kRTile = kRBlock * kRItems;     // 8192 pairs a tile
constexpr uint32_t kRWaves = kRBlock / 64;         // 16
constexpr uint32_t kRMaxBits = 9;
constexpr uint32_t kRMaxBins = 1u << kRMaxBits;    // 512 (<= kRBlock: one thread per digit)
constexpr unsigned long long kFlagAgg = 1ull << 30, kFlagInc = 2ull << 30;
constexpr uint32_t kCountMask = (1u << 30) - 1;
constexpr uint32_t kLookWin = 16;                  // earlier tiles read at once in the look-back
constexpr uint32_t kHistBlock = 1024, kHistCopies = 16;   // histogram workgroups add into copy b % 16
// dynamic LDS of a pass: per-wave digit counts (u16), tile counts, tile starts,
// global bases, wave totals, the tile's keys and values ordered by digit, the
// claimed tile id
constexpr uint32_t kPassLds = kRWaves * kRMaxBins * 2 + (3 * kRMaxBins + kRWaves + 2 * kRTile + 4) * 4;
static_assert(kRMaxBins <= kRBlock, "one thread per digit");

constexpr uint32_t kRMaxPass = 4;                  // keys of up to 36 bits

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

__global__ __launch_bounds__(kHistBlock) void radix_hist_kernel(const uint32_t *keys, uint64_t n, Digits dg,
                                                                uint32_t hot, uint32_t *hist) {
  __shared__ uint32_t h[kRMaxPass * kRMaxBins];
  for (uint32_t i = threadIdx.x; i < kRMaxPass * kRMaxBins; i += kHistBlock) h[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  auto add = [&](uint32_t key, bool valid) {
    const bool is_hot = valid && key == hot;
    const uint64_t hm = __ballot(is_hot);
    if (hm && lane == static_cast<uint32_t>(__builtin_ctzll(hm))) {
      const uint32_t c = static_cast<uint32_t>(__builtin_popcountll(hm));
      for (uint32_t p = 0; p < dg.npass; ++p) atomicAdd(&h[p * kRMaxBins + ((hot >> dg.shift[p]) & ((1u << dg.bits[p]) - 1))], c);
    }
    if (valid && !is_hot)
      for (uint32_t p = 0; p < dg.npass; ++p) atomicAdd(&h[p * kRMaxBins + ((key >> dg.shift[p]) & ((1u << dg.bits[p]) - 1))], 1u);
  };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  // four 16-byte loads in flight per thread (one at a time, the kernel waited
  // a memory round trip per 4 keys)
  constexpr uint32_t U = 4;
  const uint64_t n4 = n / 4, stride = uint64_t(gridDim.x) * kHistBlock * U;
  for (uint64_t base = uint64_t(blockIdx.x) * kHistBlock * U; base < n4; base += stride) {   // uniform per workgroup
    u32x4 k4[U];
    bool v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t q = base + u * kHistBlock + threadIdx.x;
      v[u] = q < n4;
      k4[u] = v[u] ? reinterpret_cast<const u32x4 *>(keys)[q] : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      add(k4[u].x, v[u]);
      add(k4[u].y, v[u]);
      add(k4[u].z, v[u]);
      add(k4[u].w, v[u]);
    }
  }
  if (blockIdx.x == 0) {                   // the last n % 4 keys
    const uint64_t q = n4 * 4 + threadIdx.x;
    const bool v = threadIdx.x < (n & 3);
    add(v ? keys[q] : 0u, v);
  }
  __syncthreads();
  // into copy b % 16: the adds of all workgroups to one bin serialised at the
  // memory side (53 us a sort with one copy and 512 workgroups)
  uint32_t *const hc = hist + (blockIdx.x % kHistCopies) * (kRMaxPass * kRMaxBins);
  for (uint32_t i = threadIdx.x; i < kRMaxPass * kRMaxBins; i += kHistBlock)
    if (h[i]) atomicAdd(&hc[i], h[i]);
}

__global__ __launch_bounds__(kRMaxBins) void radix_scan_kernel(uint32_t *hist, uint32_t *offs, uint32_t npass) {
  __shared__ uint32_t s[kRMaxBins];
  const uint32_t t = threadIdx.x;
  for (uint32_t p = 0; p < npass; ++p) {
    uint32_t x = 0;
    for (uint32_t c = 0; c < kHistCopies; ++c) {
      uint32_t *const h = hist + c * (kRMaxPass * kRMaxBins) + p * kRMaxBins + t;
      x += *h;
      *h = 0;                              // zero for the next sort
    }
    s[t] = x;
    __syncthreads();
    for (uint32_t off = 1; off < kRMaxBins; off <<= 1) {
      const uint32_t y = t >= off ? s[t - off] : 0u;
      __syncthreads();
      s[t] += y;
      __syncthreads();
    }
    offs[p * kRMaxBins + t] = s[t] - x;
    __syncthreads();
  }
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

__global__ __launch_bounds__(kRBlock) void radix_pass_kernel(const uint32_t *kin, const uint32_t *vin, uint32_t *kout,
                                                             uint32_t *vout, uint64_t n, uint32_t shift, uint32_t bits,
                                                             const uint32_t *offs, unsigned long long *look,
                                                             unsigned long long *tile_ctr,
                                                             unsigned long long tile_base, uint32_t epoch) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rsm[];
  uint16_t *const wcnt = reinterpret_cast<uint16_t *>(rsm);   // [wave][digit]
  uint32_t *const tcnt = reinterpret_cast<uint32_t *>(wcnt + kRWaves * kRMaxBins);   // the tile's count per digit
  uint32_t *const dstart = tcnt + kRMaxBins;                   // its digit's first place in the tile
  uint32_t *const dbase = dstart + kRMaxBins;                  // its digit's first place in the output
  uint32_t *const wtot = dbase + kRMaxBins;                    // [kRWaves] scan scratch
  uint32_t *const lk = wtot + kRWaves;
  uint32_t *const lv = lk + kRTile;
  uint32_t *const s_tile = lv + kRTile;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nb = 1u << bits, dmask = nb - 1;
  for (uint32_t i = tid; i < kRWaves * kRMaxBins / 2; i += kRBlock) reinterpret_cast<uint32_t *>(wcnt)[i] = 0;
  if (tid < kRMaxBins) tcnt[tid] = 0;
  if (tid == 0) *s_tile = static_cast<uint32_t>(atomicAdd(tile_ctr, 1ull) - tile_base);
  __syncthreads();
  const uint32_t tile = *s_tile;
  const uint64_t t0 = uint64_t(tile) * kRTile;
  // item k of lane l in wave w is the tile's item w * 512 + k * 64 + l (input order)
  uint32_t key[kRItems], val[kRItems], rnk[kRItems];
#pragma unroll
  for (uint32_t k = 0; k < kRItems; ++k) {
    const uint64_t i = t0 + w * (kRItems * 64) + k * 64 + lane;
    const bool v = i < n;
    key[k] = v ? kin[i] : 0u;
    val[k] = v ? (vin ? vin[i] : static_cast<uint32_t>(i)) : 0u;
  }
  const uint32_t d = tid;
  // The tile's digit counts first (LDS adds; the all-ones digit -- the
  // batch's "no table" bucket, often most keys -- wave-aggregated), so the
  // tile publishes its aggregate before it ranks: the tiles after it, which
  // all start together in the first round, find it early in their look-back.
#pragma unroll
  for (uint32_t k = 0; k < kRItems; ++k) {
    const bool v = t0 + w * (kRItems * 64) + k * 64 + lane < n;
    const uint32_t d = (key[k] >> shift) & dmask;
    const uint64_t hm = __ballot(v && d == dmask);
    if (hm && lane == static_cast<uint32_t>(__builtin_ctzll(hm)))
      atomicAdd(&tcnt[dmask], static_cast<uint32_t>(__builtin_popcountll(hm)));
    if (v && d != dmask) atomicAdd(&tcnt[d], 1u);
  }
  __syncthreads();
  const uint32_t c = d < nb ? tcnt[d] : 0u;
  if (d < nb) {
    // decoupled look-back: the counts of digit d in every earlier tile, kLookWin
    // earlier tiles read at once (a tile's predecessors publish while it reads);
    // the waves without a digit rank their items meanwhile
    const unsigned long long tag = static_cast<unsigned long long>(epoch) << 32;
    unsigned long long *const mine = look + uint64_t(tile) * kRMaxBins + d;
    uint32_t prefix = 0;
    if (tile == 0) {
      __hip_atomic_store(mine, tag | kFlagInc | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(mine, tag | kFlagAgg | c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t t = tile;        // tiles [0, t) are still to sum
      bool done = false;
      while (!done) {
        unsigned long long x[kLookWin];
#pragma unroll
        for (uint32_t j = 0; j < kLookWin; ++j)
          x[j] = j < t ? __hip_atomic_load(look + uint64_t(t - 1 - j) * kRMaxBins + d, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                       : 0ull;
        uint32_t used = 0;
        bool stall = false;
#pragma unroll
        for (uint32_t j = 0; j < kLookWin; ++j) {
          if (done || stall || j >= t) continue;
          if ((x[j] >> 32) != epoch) {   // not yet published (an earlier tile: claimed and running)
            stall = true;
            continue;
          }
          prefix += static_cast<uint32_t>(x[j]) & kCountMask;
          ++used;
          if (x[j] & kFlagInc) done = true;
        }
        t -= used;
        if (!done && stall) __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(mine, tag | kFlagInc | (prefix + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    dbase[d] = offs[d] + prefix;
  }
  // ranks within the wave's items of one digit, slot by slot
  uint16_t *const wc = wcnt + w * kRMaxBins;
#pragma unroll
  for (uint32_t k = 0; k < kRItems; ++k) {
    const bool v = t0 + w * (kRItems * 64) + k * 64 + lane < n;
    const uint32_t dk = (key[k] >> shift) & dmask;
    uint64_t m = __ballot(v);
    for (uint32_t b = 0; b < bits; ++b) {
      const uint64_t bb = __ballot((dk >> b) & 1);
      m &= ((dk >> b) & 1) ? bb : ~bb;
    }
    const uint32_t leader = m ? static_cast<uint32_t>(__builtin_ctzll(m)) : lane;
    uint32_t old = 0;
    if (v && lane == leader) {
      old = wc[dk];
      wc[dk] = static_cast<uint16_t>(old + static_cast<uint32_t>(__builtin_popcountll(m)));
    }
    old = __shfl(old, static_cast<int>(leader));
    rnk[k] = old + static_cast<uint32_t>(__builtin_popcountll(m & ((1ull << lane) - 1)));
  }
  __syncthreads();
  // thread d: the waves' exclusive prefix of digit d (in place)
  if (d < nb) {
    uint32_t run = 0;
#pragma unroll
    for (uint32_t ww = 0; ww < kRWaves; ++ww) {
      const uint32_t x = wcnt[ww * kRMaxBins + d];
      wcnt[ww * kRMaxBins + d] = static_cast<uint16_t>(run);
      run += x;
    }
  }
  // the digits' starts inside the tile
  const uint32_t ds = block_excl_scan(c, wtot);
  if (d < nb) dstart[d] = ds;
  __syncthreads();
  // the tile ordered by digit in LDS, then written out run by run
#pragma unroll
  for (uint32_t k = 0; k < kRItems; ++k) {
    if (t0 + w * (kRItems * 64) + k * 64 + lane < n) {
      const uint32_t dk = (key[k] >> shift) & dmask;
      const uint32_t pos = dstart[dk] + wc[dk] + rnk[k];
      lk[pos] = key[k];
      lv[pos] = val[k];
    }
  }
  __syncthreads();
  const uint32_t items = static_cast<uint32_t>(n - t0 < kRTile ? n - t0 : kRTile);
  for (uint32_t j = tid; j < items; j += kRBlock) {
    const uint32_t kk = lk[j];
    const uint32_t dk = (kk >> shift) & dmask;
    const uint64_t g = uint64_t(dbase[dk]) + (j - dstart[dk]);
    kout[g] = kk;
    vout[g] = lv[j];
  }
}


// ---- reduce-then-scan over super-tiles (PCN_IPT_DEBUG_RADIX=rts) ----------
// Workgroup b of a pass owns the contiguous super-tile [b * per, (b + 1) * per)
// of its input (per = a whole number of 8192-item sub-tiles; one workgroup per
// CU), the same range in all three kernels of the pass:
//   radix_seg_up_kernel:   the super-tile's count of every digit, cnt[b][512];
//   radix_seg_scan_kernel: per digit, the exclusive prefix over super-tiles
//                          (pre[b][d]) and the digit's total (tot[d]);
//   radix_seg_pass_kernel: the digits' global starts (exclusive scan of tot),
//                          then the super-tile's sub-tiles in order, each
//                          ranked, ordered by digit in LDS and written out,
//                          the running per-digit bases advanced in LDS.
// No look-back, no tile claims, no spin: a workgroup waits on nothing but its
// own loads.  The digit totals come from the counts, so no histogram kernel.
constexpr uint32_t seg_lds(uint32_t sb) { return sb / 64 * kRMaxBins * 2 + (2 * kRMaxBins + kRWaves) * 4 + sb * kRItems * 4; }

__global__ __launch_bounds__(kRBlock) void radix_seg_up_kernel(const uint32_t *kin, uint64_t n, uint32_t shift,
                                                               uint32_t bits, uint64_t per, uint32_t *cnt) {
  __shared__ uint32_t h[kRMaxBins];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t dmask = (1u << bits) - 1;
  if (tid < kRMaxBins) h[tid] = 0;
  __syncthreads();
  const uint64_t lo = uint64_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
  auto add = [&](uint32_t k, bool v) {
    const uint32_t dk = (k >> shift) & dmask;
    const uint64_t hm = __ballot(v && dk == dmask);   // the all-ones digit: the "no table" bucket
    if (hm && lane == static_cast<uint32_t>(__builtin_ctzll(hm)))
      atomicAdd(&h[dmask], static_cast<uint32_t>(__builtin_popcountll(hm)));
    if (v && dk != dmask) atomicAdd(&h[dk], 1u);
  };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  constexpr uint32_t U = 4;   // 16-byte loads in flight per thread
  // lo is a multiple of 8192: 16-byte aligned
  for (uint64_t base = lo; base < hi; base += uint64_t(kRBlock) * 4 * U) {   // uniform per workgroup
    u32x4 k4[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t i = base + 4 * (u * kRBlock + tid);
      k4[u] = i + 4 <= hi ? *reinterpret_cast<const u32x4 *>(kin + i)
                          : u32x4{i < hi ? kin[i] : 0u, i + 1 < hi ? kin[i + 1] : 0u, i + 2 < hi ? kin[i + 2] : 0u, 0u};
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t i = base + 4 * (u * kRBlock + tid);
      add(k4[u].x, i < hi);
      add(k4[u].y, i + 1 < hi);
      add(k4[u].z, i + 2 < hi);
      add(k4[u].w, i + 3 < hi);
    }
  }
  __syncthreads();
  if (tid < kRMaxBins) cnt[uint64_t(blockIdx.x) * kRMaxBins + tid] = h[tid];
}

// 64 digits a workgroup (lane = digit), wave w a contiguous range of super-tiles
__global__ __launch_bounds__(kRBlock) void radix_seg_scan_kernel(const uint32_t *cnt, uint32_t *pre, uint32_t *tot,
                                                                 uint32_t groups, uint32_t nb) {
  __shared__ uint32_t part[kRWaves][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t d = blockIdx.x * 64 + lane;
  const uint32_t per = (groups + kRWaves - 1) / kRWaves;
  const uint32_t lo = w * per, hi = lo + per < groups ? lo + per : groups;
  uint32_t sum = 0;
  if (d < nb)
    for (uint32_t b = lo; b < hi; ++b) sum += cnt[uint64_t(b) * kRMaxBins + d];
  part[w][lane] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t k = 0; k < w; ++k) run += part[k][lane];
  if (d < nb && w == kRWaves - 1) tot[d] = run + sum;
  if (d < nb)
    for (uint32_t b = lo; b < hi; ++b) {
      const uint32_t x = cnt[uint64_t(b) * kRMaxBins + d];
      pre[uint64_t(b) * kRMaxBins + d] = run;
      run += x;
    }
}

// SB threads a workgroup, 1024 / SB workgroups per CU (~116 VGPRs: 4 waves per
// SIMD); the next sub-tile's keys are loaded while this one is ordered and written.
template <uint32_t SB>
__global__ __launch_bounds__(SB) void radix_seg_pass_kernel(const uint32_t *kin, const uint32_t *vin,
                                                                    uint32_t *kout, uint32_t *vout, uint64_t n,
                                                                    uint32_t shift, uint32_t bits, uint64_t per,
                                                                    const uint32_t *pre, const uint32_t *tot) {
  constexpr uint32_t kW = SB / 64, kTile = SB * kRItems;
  extern __shared__ __attribute__((aligned(16))) uint8_t rsm[];
  uint16_t *const wcnt = reinterpret_cast<uint16_t *>(rsm);   // [wave][digit]
  uint32_t *const dstart = reinterpret_cast<uint32_t *>(wcnt + kW * kRMaxBins);   // digit's first place in the sub-tile
  uint32_t *const dbase = dstart + kRMaxBins;                  // digit's next place in the output
  uint32_t *const wtot = dbase + kRMaxBins;
  uint32_t *const buf = wtot + kW;                        // the sub-tile's keys, then values, by digit
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t nb = 1u << bits, dmask = nb - 1;
  const uint32_t d = tid;
  {
    const uint32_t t = d < nb ? tot[d] : 0u;
    const uint32_t off = block_excl_scan(t, wtot);
    if (d < nb) dbase[d] = off + pre[uint64_t(blockIdx.x) * kRMaxBins + d];
  }
  const uint64_t lo = uint64_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
  uint16_t *const wc = wcnt + w * kRMaxBins;
  // item k of lane l in wave w is the sub-tile's item w * 512 + k * 64 + l
  // (input order); 32-bit offsets from the sub-tile's uniform base
  const uint32_t li = w * (kRItems * 64) + lane;
  uint32_t key[kRItems], nkey[kRItems];
  auto load_keys = [&](uint32_t *dst, uint64_t at) {
    const uint32_t m = static_cast<uint32_t>(hi - at < kTile ? hi - at : kTile);
    const uint32_t *const kt = kin + at;
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) dst[k] = li + k * 64 < m ? kt[li + k * 64] : 0u;
  };
  if (lo < hi) load_keys(key, lo);
  for (uint64_t t0 = lo; t0 < hi; t0 += kTile) {   // uniform per workgroup
    reinterpret_cast<uint2 *>(wcnt)[tid] = uint2{0u, 0u};   // 16 KB: 16 bytes a thread
    reinterpret_cast<uint2 *>(wcnt)[tid + SB] = uint2{0u, 0u};
    __syncthreads();
    const uint32_t items = static_cast<uint32_t>(hi - t0 < kTile ? hi - t0 : kTile);
    const uint32_t *const vt = vin ? vin + t0 : nullptr;
    uint32_t pos[kRItems];
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
      uint32_t old = 0;
      if (v && lane == leader) {
        old = wc[dk];
        wc[dk] = static_cast<uint16_t>(old + static_cast<uint32_t>(__builtin_popcountll(m)));
      }
      old = __shfl(old, static_cast<int>(leader));
      pos[k] = old + static_cast<uint32_t>(__builtin_popcountll(m & ((1ull << lane) - 1)));
    }
    if (t0 + kTile < hi) load_keys(nkey, t0 + kTile);   // in flight through the rest of this sub-tile
    __syncthreads();
    uint32_t c = 0;   // the sub-tile's count of digit d
    if (d < nb) {
#pragma unroll
      for (uint32_t ww = 0; ww < kW; ++ww) {
        const uint32_t x = wcnt[ww * kRMaxBins + d];
        wcnt[ww * kRMaxBins + d] = static_cast<uint16_t>(c);
        c += x;
      }
    }
    const uint32_t ds = block_excl_scan(c, wtot);
    if (d < nb) dstart[d] = ds;
    __syncthreads();
    uint32_t val[kRItems];
    const uint32_t ib = static_cast<uint32_t>(t0);   // (n < 2^30)
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      const uint32_t j = li + k * 64;
      val[k] = j < items ? (vt ? vt[j] : ib + j) : 0u;
      if (j < items) {
        const uint32_t dk = (key[k] >> shift) & dmask;
        pos[k] += dstart[dk] + wc[dk];
        buf[pos[k]] = key[k];
      }
    }
    __syncthreads();
    uint32_t g[kRItems];
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      const uint32_t j = tid + k * SB;
      if (j < items) {
        const uint32_t kk = buf[j];
        const uint32_t dk = (kk >> shift) & dmask;
        g[k] = dbase[dk] + (j - dstart[dk]);
        kout[g[k]] = kk;
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k)
      if (li + k * 64 < items) buf[pos[k]] = val[k];
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) {
      const uint32_t j = tid + k * SB;
      if (j < items) vout[g[k]] = buf[j];
    }
    if (d < nb) dbase[d] += c;   // (read above, before the last barrier)
#pragma unroll
    for (uint32_t k = 0; k < kRItems; ++k) key[k] = nkey[k];
  }
}
}  // namespace

// PCN_IPT_DEBUG_RADIX=rts / rts512: reduce-then-scan passes over super-tiles
// with 1024- / 512-thread workgroups instead of the onesweep look-back (A/B);
// read per sort, so a test can flip it (one getenv per batch).  0 = onesweep.
static uint32_t radix_seg_block() {
  const char *e = std::getenv("PCN_IPT_DEBUG_RADIX");
  if (!e) return 0;
  const std::string v(e);
  return v == "rts" ? 1024u : v == "rts512" ? 512u : 0u;
}

void radix_free(RadixScratch &s) {
  for (void *p : {static_cast<void *>(s.tk), static_cast<void *>(s.tv), static_cast<void *>(s.tv2),
                  static_cast<void *>(s.seg),
                  static_cast<void *>(s.look), static_cast<void *>(s.hist), static_cast<void *>(s.offs),
                  static_cast<void *>(s.tile_ctr)})
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
  const uint64_t tiles = (n + kRTile - 1) / kRTile;
  if (s.cap < n) {
    for (uint32_t **p : {&s.tk, &s.tv, &s.tv2}) {
      if (*p) RX_CHECK(hipFree(*p));
      *p = nullptr;
      RX_CHECK(hipMalloc(p, n * 4));
    }
    s.cap = n;
  }
  if (s.look_tiles < tiles) {
    if (s.look) RX_CHECK(hipFree(s.look));
    s.look = nullptr;
    RX_CHECK(hipMalloc(&s.look, tiles * kRMaxBins * 8));
    RX_CHECK(hipMemsetAsync(s.look, 0, tiles * kRMaxBins * 8, st));   // epoch 0: never a pass's
    s.look_tiles = tiles;
  }
  if (!s.hist) {
    RX_CHECK(hipMalloc(&s.hist, kHistCopies * kRMaxPass * kRMaxBins * 4));
    RX_CHECK(hipMalloc(&s.offs, kRMaxPass * kRMaxBins * 4));
    RX_CHECK(hipMalloc(&s.tile_ctr, 64));
    RX_CHECK(hipMemsetAsync(s.hist, 0, kHistCopies * kRMaxPass * kRMaxBins * 4, st));
    RX_CHECK(hipMemsetAsync(s.tile_ctr, 0, 64, st));
    s.tiles_issued = 0;
  }
  const Digits dg = digits_for(kbits);
  const uint32_t hot = kbits >= 32 ? ~0u : (1u << kbits) - 1;   // the sentinel bucket (conntrack.hip)
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
  if (const uint32_t sb = radix_seg_block()) {
    // super-tiles of whole sub-tiles (sb * 8 items), 1024 / sb workgroups per CU
    const uint64_t sub = uint64_t(sb) * kRItems;
    const uint64_t g0 = std::max<uint64_t>(1, uint64_t(num_cus > 0 ? num_cus : 1) * (kRBlock / sb));
    const uint64_t subs = (n + sub - 1) / sub;
    const uint64_t per = (subs + g0 - 1) / g0 * sub;
    const uint32_t groups = static_cast<uint32_t>((n + per - 1) / per);
    if (s.seg_groups < groups) {
      if (s.seg) RX_CHECK(hipFree(s.seg));
      s.seg = nullptr;
      RX_CHECK(hipMalloc(&s.seg, (2 * uint64_t(groups) + 1) * kRMaxBins * 4));
      s.seg_groups = groups;
    }
    uint32_t *const cnt = s.seg, *const pre = s.seg + uint64_t(groups) * kRMaxBins, *const tot = pre + uint64_t(groups) * kRMaxBins;
    for (uint32_t p = 0; p < dg.npass; ++p) {
      const uint32_t nb = 1u << dg.bits[p];
      hipLaunchKernelGGL(radix_seg_up_kernel, dim3(groups), dim3(kRBlock), 0, st, kin[p], n, dg.shift[p], dg.bits[p],
                         per, cnt);
      RX_CHECK(hipGetLastError());
      hipLaunchKernelGGL(radix_seg_scan_kernel, dim3((nb + 63) / 64), dim3(kRBlock), 0, st, cnt, pre, tot, groups, nb);
      RX_CHECK(hipGetLastError());
      if (sb == 512)
        hipLaunchKernelGGL(radix_seg_pass_kernel<512>, dim3(groups), dim3(512), seg_lds(512), st, kin[p], vin[p],
                           kout[p], vout[p], n, dg.shift[p], dg.bits[p], per, pre, tot);
      else
        hipLaunchKernelGGL(radix_seg_pass_kernel<1024>, dim3(groups), dim3(1024), seg_lds(1024), st, kin[p], vin[p],
                           kout[p], vout[p], n, dg.shift[p], dg.bits[p], per, pre, tot);
      RX_CHECK(hipGetLastError());
    }
    return hipSuccess;
  }
  const uint64_t hwant = (n / 16 + kHistBlock - 1) / kHistBlock;
  const unsigned hgrid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(hwant, uint64_t(num_cus))));
  hipLaunchKernelGGL(radix_hist_kernel, dim3(hgrid), dim3(kHistBlock), 0, st, keys_in, n, dg, hot, s.hist);
  RX_CHECK(hipGetLastError());
  hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(kRMaxBins), 0, st, s.hist, s.offs, dg.npass);
  RX_CHECK(hipGetLastError());
  for (uint32_t p = 0; p < dg.npass; ++p) {
    if (++s.epoch == 0) s.epoch = 1;   // (2^32 passes: the words of epoch 0 are the zeroed ones)
    hipLaunchKernelGGL(radix_pass_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kRBlock), kPassLds, st, kin[p],
                       vin[p], kout[p], vout[p], n, dg.shift[p], dg.bits[p], s.offs + p * kRMaxBins, s.look,
                       s.tile_ctr, s.tiles_issued, s.epoch);
    RX_CHECK(hipGetLastError());
    s.tiles_issued += tiles;
  }
  return hipSuccess;
}

}  // namespace pcn
