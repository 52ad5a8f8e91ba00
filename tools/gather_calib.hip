// gather_calib.hip -- calibration of rocprofv3's HBM traffic counters for the
// access patterns of this datapath (measurement only, never linked into the
// product).  MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide streaming
// reads (FETCH_SIZE = TCC_EA0_RDREQ x 64 B, half the bytes of 128-byte requests)
// and asks for a calibration on a known byte count in one's own pattern before
// quoting an absolute.  Each pattern below reads a byte set whose 128-byte line
// and 64-byte sector footprint the host computes exactly; rocprofv3 --pmc passes
// over this program then give FETCH_SIZE and the TCC_EA0_RDREQ_{32B,64B,128B}
// split per dispatch, to be set against those footprints (tools/gather_calib.py).
//
// Patterns (one kernel name each, so the PMC rows separate by name):
//   calib_stream     1 GiB, 16 B per lane, coalesced (the guide's calibrated case)
//   calib_stride_S   48-byte windows at a fixed stride S (64..1536; the frame-size
//                    sweep), three 16-byte loads per lane, one lane per frame
//   calib_imix       52-byte windows at config 5's IMIX offsets (7:4:1 of 64 / 576
//                    / 1500-byte frames packed back to back), four lanes per frame
//                    + the offset (4 B) and length (2 B) arrays: the gather ceiling
//   calib_rec32      32-byte records read once each in a random order (ct_walk's
//                    record gather through the sorted index, 2^24 records)
// Every buffer is 2 GiB or more past any earlier one's use and the Infinity
// Cache holds 256 MiB: each dispatch is timed and counted from HBM (the first of
// each pattern aside).  Usage: ./gather_calib <pattern> [log2n] [reps]
//   pattern: stream | stride:<S> | imix | rec32 ; prints one JSON line with the
//   host-side footprints and the HIP-event time per dispatch.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_calib.hip -o tools/gather_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ __launch_bounds__(256) void calib_stream(const u32x4 *p, uint64_t n16, uint32_t *out) {
  uint32_t x = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9e3779b9u) out[0] = x;     // keeps the loads; never true for the buffers here
}

// the Infinity Cache scrub between dispatches (a kernel of its own name: not counted)
__global__ __launch_bounds__(256) void calib_scrub(const u32x4 *p, uint64_t n16, uint32_t *out) {
  uint32_t x = 0;
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x9e3779b9u) out[0] = x;
}

__global__ __launch_bounds__(256) void calib_stride(const uint8_t *f, uint64_t n, uint32_t stride, uint8_t *v) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint8_t *b = f + i * stride;
    uint32_t x = 0;
    if ((stride & 15) == 0) {
      const u32x4 *q = reinterpret_cast<const u32x4 *>(b);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const u32x4 c = __builtin_nontemporal_load(q + k);
        x ^= c.x ^ c.y ^ c.z ^ c.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 12; ++k) x ^= *reinterpret_cast<const uint32_t *>(b + 4 * k);   // stride % 4 == 0
    }
    v[i] = static_cast<uint8_t>(x);
  }
}

__global__ __launch_bounds__(256) void calib_imix(const uint8_t *f, const uint32_t *off, const uint16_t *len,
                                                  uint8_t *v, uint64_t n) {
  const uint32_t q = threadIdx.x & 3;
  const uint64_t step = uint64_t(gridDim.x) * blockDim.x / 4;
  for (uint64_t g = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 4; g < n; g += step) {
    const uint32_t o = off[g];
    const uint8_t *base = f + (o & ~15u);
    uint32_t x = q == 0 ? len[g] : 0u;
    const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base) + q);
    x ^= a.x ^ a.y ^ a.z ^ a.w;
    if (q == 0 && (o & 15) > 12) {
      const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base) + 4);
      x ^= b.x;
    }
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if (q == 0) v[g] = static_cast<uint8_t>(x & 1);
  }
}

__global__ __launch_bounds__(256) void calib_rec32(const u32x4 *rec, const uint32_t *idx, uint64_t n, uint8_t *v) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t j = idx[i];
    const u32x4 a = rec[2 * uint64_t(j)], b = rec[2 * uint64_t(j) + 1];
    v[i] = static_cast<uint8_t>(a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w);
  }
}

// distinct `unit`-byte blocks covered by the byte ranges [s, s + len) (s ascending)
static uint64_t blocks(const std::vector<uint64_t> &s, uint32_t len, uint32_t unit) {
  uint64_t cnt = 0, last = ~0ull;
  for (uint64_t a : s) {
    for (uint64_t bl = a / unit; bl <= (a + len - 1) / unit; ++bl)
      if (bl != last) { ++cnt; last = bl; }
  }
  return cnt;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s stream|stride:<S>|imix|rec32 [log2n] [reps]\n", argv[0]);
    return 2;
  }
  const std::string pat = argv[1];
  const unsigned log2n = argc > 2 ? std::atoi(argv[2]) : 24;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 10;
  const uint64_t n = uint64_t(1) << log2n;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const unsigned grid = static_cast<unsigned>(cus * 8);
  // a 2 GiB scrub buffer read between dispatches keeps the Infinity Cache cold
  const uint64_t scrub_bytes = uint64_t(2) << 30;
  u32x4 *scrub;
  CK(hipMalloc(&scrub, scrub_bytes));
  CK(hipMemset(scrub, 1, scrub_bytes));
  uint32_t *sink;
  CK(hipMalloc(&sink, 64));
  uint8_t *v;
  CK(hipMalloc(&v, n));
  double alg = 0, lines = 0, sectors = 0;     // bytes the pattern reads; 128 B lines; 64 B sectors
  std::string what;
  std::function<void()> launch;
  uint8_t *f = nullptr;
  uint32_t *off = nullptr, *idx = nullptr;
  uint16_t *len = nullptr;
  if (pat == "stream") {
    const uint64_t bytes = uint64_t(1) << 30;
    CK(hipMalloc(&f, bytes));
    CK(hipMemset(f, 3, bytes));
    alg = lines = sectors = double(bytes);
    lines /= 128;
    sectors /= 64;
    what = "1 GiB read once, 16 B per lane, coalesced";
    launch = [&, bytes] { hipLaunchKernelGGL(calib_stream, dim3(grid), dim3(256), 0, 0, reinterpret_cast<u32x4 *>(f), bytes / 16, sink); };
  } else if (pat.rfind("stride:", 0) == 0) {
    const uint32_t stride = static_cast<uint32_t>(std::atoi(pat.c_str() + 7));
    if (stride < 48 || stride % 4) { std::fprintf(stderr, "stride must be >= 48 and a multiple of 4\n"); return 2; }
    const uint64_t bytes = n * stride;
    // CALIB_ALLOC=uc / fg: the frames in uncached / fine-grained device memory (whether the
    // L2 then fetches less than a 128-byte line for a 48-byte window)
    const char *al = std::getenv("CALIB_ALLOC");
    if (al && std::string(al) == "uc") CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&f), bytes + 64, hipDeviceMallocUncached));
    else if (al && std::string(al) == "fg") CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&f), bytes + 64, hipDeviceMallocFinegrained));
    else CK(hipMalloc(&f, bytes + 64));
    CK(hipMemset(f, 5, bytes + 64));
    std::vector<uint64_t> s(n);
    for (uint64_t i = 0; i < n; ++i) s[i] = i * stride;
    alg = double(n) * 48;
    lines = double(blocks(s, 48, 128));
    sectors = double(blocks(s, 48, 64));
    what = "48-byte windows at a fixed stride of " + std::to_string(stride) + " B, one lane per frame";
    launch = [&, stride] { hipLaunchKernelGGL(calib_stride, dim3(grid), dim3(256), 0, 0, f, n, stride, v); };
  } else if (pat == "imix") {
    std::mt19937_64 rng(5);
    std::vector<uint32_t> ho(n);
    std::vector<uint16_t> hl(n);
    uint64_t at = 0;
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t r = rng() % 12;
      const uint16_t sz = r < 7 ? 64 : r < 11 ? 576 : 1500;
      ho[i] = static_cast<uint32_t>(at);
      hl[i] = sz;
      at += sz;
    }
    CK(hipMalloc(&f, at + 128));
    CK(hipMemset(f, 7, at + 128));
    CK(hipMalloc(&off, n * 4));
    CK(hipMalloc(&len, n * 2));
    CK(hipMemcpy(off, ho.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(len, hl.data(), n * 2, hipMemcpyHostToDevice));
    // what the kernel touches: [o & ~15, (o & ~15) + 64) and, when o & 15 > 12, the next 16 B
    uint64_t ln = 0, sc = 0;
    {
      uint64_t lastl = ~0ull, lasts = ~0ull;
      for (uint64_t i = 0; i < n; ++i) {
        const uint64_t a = ho[i] & ~15ull, e = a + ((ho[i] & 15) > 12 ? 80 : 64);
        for (uint64_t b = a / 128; b <= (e - 1) / 128; ++b) if (b != lastl) { ++ln; lastl = b; }
        for (uint64_t b = a / 64; b <= (e - 1) / 64; ++b) if (b != lasts) { ++sc; lasts = b; }
      }
    }
    alg = double(n) * (52 + 4 + 2);
    lines = double(ln) + double(n) * 6 / 128;
    sectors = double(sc) + double(n) * 6 / 64;
    what = "IMIX 7:4:1 of 64/576/1500-byte frames packed back to back: a 52-byte window per frame (4 lanes x 16 B "
           "from its 16-byte-aligned start, a fifth chunk when the window crosses it) + offset + length";
    launch = [&] { hipLaunchKernelGGL(calib_imix, dim3(grid), dim3(256), 0, 0, f, off, len, v, n); };
  } else if (pat == "rec32") {
    CK(hipMalloc(&f, n * 32));
    CK(hipMemset(f, 9, n * 32));
    std::vector<uint32_t> hi(n);
    for (uint64_t i = 0; i < n; ++i) hi[i] = static_cast<uint32_t>(i);
    std::mt19937_64 rng(7);
    for (uint64_t i = n - 1; i > 0; --i) std::swap(hi[i], hi[rng() % (i + 1)]);
    CK(hipMalloc(&idx, n * 4));
    CK(hipMemcpy(idx, hi.data(), n * 4, hipMemcpyHostToDevice));
    alg = double(n) * (32 + 4);
    lines = double(n) * 32 / 128 + double(n) * 4 / 128;
    sectors = double(n) * 32 / 64 + double(n) * 4 / 64;
    what = "32-byte records each read once, in a random permutation order (+ the 4-byte index array, coalesced)";
    launch = [&] { hipLaunchKernelGGL(calib_rec32, dim3(grid), dim3(256), 0, 0, reinterpret_cast<u32x4 *>(f), idx, n, v); };
  } else {
    std::fprintf(stderr, "unknown pattern %s\n", pat.c_str());
    return 2;
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float total = 0;
  for (int r = 0; r < reps + 1; ++r) {
    hipLaunchKernelGGL(calib_scrub, dim3(grid), dim3(256), 0, 0, scrub, scrub_bytes / 16, sink);
    CK(hipEventRecord(a, 0));
    launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r) total += ms;               // the first dispatch is a warmup
  }
  CK(hipGetLastError());
  const double ms = total / reps;
  std::printf("{\"pattern\": \"%s\", \"n\": %llu, \"what\": \"%s\", \"alg_bytes\": %.0f, \"lines_128b\": %.0f, "
              "\"sectors_64b\": %.0f, \"ms\": %.5f, \"alg_gb_s\": %.1f, \"line_gb_s\": %.1f, \"sector_gb_s\": %.1f}\n",
              pat.c_str(), static_cast<unsigned long long>(pat == "stream" ? 0 : n), what.c_str(), alg, lines, sectors,
              ms, alg / ms / 1e6, lines * 128 / ms / 1e6, sectors * 64 / ms / 1e6);
  return 0;
}
