// gather_probe.hip — the read ceiling of config 5's access pattern (no
// classification work): 2^22 IMIX frames (64 / 576 / 1500 B, 7:4:1) packed
// back to back, as synth.imix_frames lays them out, or each frame at a 64-byte
// boundary ("aligned", how NIC RX buffers place them).  Every kernel reads the
// frame's offset (4 B), length (2 B) and the header window the classify kernel
// needs (bytes 0..51), and writes one verdict byte:
//   lane   : one lane per frame, four 16-byte loads from the dword-aligned start
//            (the classify kernel's generic path, load_generic)
//   quad   : four lanes per frame, one 16-byte load each from the frame's
//            16-byte-aligned start (+ a fifth chunk when the window crosses it),
//            so one load instruction covers 16 frames' contiguous bytes
// Reports kernel time, Gpkt/s and GB/s at the algorithmic 70 B/pkt.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/gather_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4d __attribute__((ext_vector_type(4), aligned(4)));

__global__ void lane_k(const uint8_t *f, const uint32_t *off, const uint16_t *len, uint8_t *v, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t base = off[i] & ~3u;
    const u32x4d *p = reinterpret_cast<const u32x4d *>(f + base);
    uint32_t x = len[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4d a = __builtin_nontemporal_load(p + q);
      x ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    v[i] = static_cast<uint8_t>(x & 1);
  }
}

__global__ void quad_k(const uint8_t *f, const uint32_t *off, const uint16_t *len, uint8_t *v, uint32_t n) {
  const uint32_t lane = threadIdx.x & 63, q = lane & 3;
  const uint32_t step = gridDim.x * blockDim.x / 4;
  for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) / 4; g < n + 0u; g += step) {
    // frame g: lanes 4k..4k+3 of the wave hold the 16 frames of one instruction
    const uint32_t o = off[g];
    const uint64_t base = o & ~15u;
    uint32_t x = q == 0 ? len[g] : 0u;
    const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(f + base) + q);
    x ^= a.x ^ a.y ^ a.z ^ a.w;
    if (q == 0 && (o & 15) > 12) {              // the window [o, o + 52) runs into a fifth chunk
      const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(f + base) + 4);
      x ^= b.x;
    }
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if (q == 0) v[g] = static_cast<uint8_t>(x & 1);
  }
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? static_cast<uint32_t>(atoi(argv[1])) : (1u << 22);
  const int iters = 50;
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  std::mt19937_64 rng(0x1111);
  std::discrete_distribution<int> pick({7.0, 4.0, 1.0});
  const uint32_t sz[3] = {64, 576, 1500};
  for (int layout = 0; layout < 2; ++layout) {
    std::vector<uint32_t> off(n);
    std::vector<uint16_t> len(n);
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t s = sz[pick(rng)];
      off[i] = static_cast<uint32_t>(at);
      len[i] = static_cast<uint16_t>(s);
      at += layout ? (s + 63) / 64 * 64 : s;
    }
    const uint64_t bytes = at + 128;
    uint8_t *df;
    uint32_t *doff;
    uint16_t *dlen;
    uint8_t *dv;
    CK(hipMalloc(&df, bytes));
    CK(hipMemset(df, 0x5a, bytes));
    CK(hipMalloc(&doff, n * 4ull));
    CK(hipMalloc(&dlen, n * 2ull));
    CK(hipMalloc(&dv, n));
    CK(hipMemcpy(doff, off.data(), n * 4ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, len.data(), n * 2ull, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int kind = 0; kind < 2; ++kind) {
      for (int occ : {4, 8, 16}) {
        const unsigned grid = static_cast<unsigned>(cus * occ);
        auto launch = [&]() {
          if (kind == 0) hipLaunchKernelGGL(lane_k, dim3(grid), dim3(256), 0, 0, df, doff, dlen, dv, n);
          else hipLaunchKernelGGL(quad_k, dim3(grid), dim3(256), 0, 0, df, doff, dlen, dv, n);
        };
        const auto t0 = std::chrono::steady_clock::now();          // settle the clocks for 1 s
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 1.0) {
          for (int k = 0; k < 16; ++k) launch();
          CK(hipDeviceSynchronize());
        }
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < iters; ++k) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= iters;
        printf("%-8s %-5s grid %5u: %.4f ms  %.2f Gpkt/s  %.0f GB/s at 70 B/pkt\n", layout ? "aligned" : "packed",
               kind ? "quad" : "lane", grid, ms, n / (ms * 1e-3) / 1e9, 70.0 * n / (ms * 1e-3) / 1e9);
      }
    }
    CK(hipFree(df));
    CK(hipFree(doff));
    CK(hipFree(dlen));
    CK(hipFree(dv));
  }
  return 0;
}
