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

// Reduce-then-scan, up-sweep: tile t's count of every digit into cnt[t][512].
__global__ __launch_bounds__(kRBlock) void radix_up_kernel(const uint32_t *kin, uint64_t n, uint32_t shift,
                                                           uint32_t bits, uint32_t *cnt) {
  __shared__ uint32_t h[kRMaxBins];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t dmask = (1u << bits) - 1;
  if (tid < kRMaxBins) h[tid] = 0;
  __syncthreads();
  const uint64_t t0 = uint64_t(blockIdx.x) * kRTile;
#pragma unroll
  for (uint32_t k = 0; k < kRItems; ++k) {
    const uint64_t i = t0 + k * kRBlock + tid;
    const bool v = i < n;
    const uint32_t dk = v ? (kin[i] >> shift) & dmask : 0u;
    const uint64_t hm = __ballot(v && dk == dmask);
    if (hm && lane == static_cast<uint32_t>(__builtin_ctzll(hm))) atomicAdd(&h[dmask], static_cast<uint32_t>(__builtin_popcountll(hm)));
    if (v && dk != dmask) atomicAdd(&h[dk], 1u);
  }
  __syncthreads();
  if (tid < kRMaxBins) cnt[uint64_t(blockIdx.x) * kRMaxBins + tid] = h[tid];
}

// Reduce-then-scan, scan: for 64 digits per workgroup (lane = digit), the
// exclusive prefix over tiles of cnt[t][d], plus the digit's global base, into
// pre[t][d].  Wave w takes a contiguous range of tiles.
__global__ __launch_bounds__(kRBlock) void radix_tscan_kernel(const uint32_t *cnt, uint32_t *pre, uint64_t tiles,
                                                              uint32_t nb, const uint32_t *offs) {
  __shared__ uint32_t part[kRWaves][64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t d = blockIdx.x * 64 + lane;
  const uint64_t per = (tiles + kRWaves - 1) / kRWaves;
  const uint64_t lo = w * per, hi = lo + per < tiles ? lo + per : tiles;
  uint32_t sum = 0;
  if (d < nb)
    for (uint64_t t = lo; t < hi; ++t) sum += cnt[t * kRMaxBins + d];
  part[w][lane] = sum;
  __syncthreads();
  uint32_t run = d < nb ? offs[d] : 0u;
  for (uint32_t k = 0; k < w; ++k) run += part[k][lane];
  if (d < nb)
    for (uint64_t t = lo; t < hi; ++t) {
      const uint32_t x = cnt[t * kRMaxBins + d];
      pre[t * kRMaxBins + d] = run;
      run += x;
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
                                                             unsigned long long tile_base, uint32_t epoch,
                                                             const uint32_t *pre) {
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
  // Reduce-then-scan mode (pre != null, PCN_IPT_DEBUG_RADIX=rts): the tile's
  // digit bases come from radix_up_kernel + radix_tscan_kernel; no look-back.
  const uint32_t d = tid;
  uint32_t c = 0;
  if (pre) {
    if (d < nb) dbase[d] = pre[uint64_t(tile) * kRMaxBins + d];
  } else {
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
  c = d < nb ? tcnt[d] : 0u;
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
  }   // (pre)
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
  // thread d: the waves' exclusive prefix of digit d (in place); the tile's
  // count of it (reduce-then-scan: not counted before)
  if (d < nb) {
    uint32_t run = 0;
#pragma unroll
    for (uint32_t ww = 0; ww < kRWaves; ++ww) {
      const uint32_t x = wcnt[ww * kRMaxBins + d];
      wcnt[ww * kRMaxBins + d] = static_cast<uint16_t>(run);
      run += x;
    }
    if (pre) c = run;
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

}  // namespace

// PCN_IPT_DEBUG_RADIX=rts: reduce-then-scan passes (up-sweep, tile scan,
// down-sweep) instead of the onesweep look-back (A/B)
// (read per sort, so a test can flip it; one getenv per batch)
static bool radix_rts() {
  const char *e = std::getenv("PCN_IPT_DEBUG_RADIX");
  return e && std::string(e) == "rts";
}

void radix_free(RadixScratch &s) {
  for (void *p : {static_cast<void *>(s.tk), static_cast<void *>(s.tv), static_cast<void *>(s.tv2),
                  static_cast<void *>(s.rts),
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
  const uint64_t hwant = (n / 16 + kHistBlock - 1) / kHistBlock;
  const unsigned hgrid = static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(hwant, uint64_t(num_cus))));
  hipLaunchKernelGGL(radix_hist_kernel, dim3(hgrid), dim3(kHistBlock), 0, st, keys_in, n, dg, hot, s.hist);
  RX_CHECK(hipGetLastError());
  hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(kRMaxBins), 0, st, s.hist, s.offs, dg.npass);
  RX_CHECK(hipGetLastError());
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
  const bool rts = radix_rts();
  if (rts && s.rts_tiles < tiles) {
    if (s.rts) RX_CHECK(hipFree(s.rts));
    s.rts = nullptr;
    RX_CHECK(hipMalloc(&s.rts, 2 * tiles * kRMaxBins * 4));
    s.rts_tiles = tiles;
  }
  for (uint32_t p = 0; p < dg.npass; ++p) {
    if (++s.epoch == 0) s.epoch = 1;   // (2^32 passes: the words of epoch 0 are the zeroed ones)
    uint32_t *pre = nullptr;
    if (rts) {
      uint32_t *const cnt = s.rts;
      pre = s.rts + tiles * kRMaxBins;
      hipLaunchKernelGGL(radix_up_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kRBlock), 0, st, kin[p], n,
                         dg.shift[p], dg.bits[p], cnt);
      RX_CHECK(hipGetLastError());
      const uint32_t nb = 1u << dg.bits[p];
      hipLaunchKernelGGL(radix_tscan_kernel, dim3((nb + 63) / 64), dim3(kRBlock), 0, st, cnt, pre, tiles, nb,
                         s.offs + p * kRMaxBins);
      RX_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(radix_pass_kernel, dim3(static_cast<unsigned>(tiles)), dim3(kRBlock), kPassLds, st, kin[p],
                       vin[p], kout[p], vout[p], n, dg.shift[p], dg.bits[p], s.offs + p * kRMaxBins, s.look,
                       s.tile_ctr, s.tiles_issued, s.epoch, pre);
    RX_CHECK(hipGetLastError());
    s.tiles_issued += tiles;
  }
  return hipSuccess;
}

}  // namespace pcn
