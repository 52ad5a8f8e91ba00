// stream_probe2.hip — header-streaming ceilings of the fixed-stride classify
// access pattern with settled clocks (1 s of untimed launches first), at the
// classify kernel's geometry (one 1024-thread workgroup per CU, persistent
// grid-stride loop, 64 frames of 64 B per wave iteration):
//   all64     : every 16-byte chunk of every frame (4 per frame), coalesced
//   hdr48     : chunks 0..2 of each frame (bytes 0..47), chunk t = 64q + lane
//   hdr48_lds : hdr48 + the transpose through LDS (3 ds_write_b128, 3 ds_read_b128)
//   hdr48_pf2 : hdr48_lds with two frame groups per lane in flight
//   glds      : chunks 0..2 by global_load_lds_dwordx4 straight into LDS, then
//               3 ds_read_b128 (one group in flight)
//   glds_pf2  : glds with two LDS landing buffers per wave (two groups in flight)
// Each writes one verdict byte per frame.  Measurement tool (GPU box only).
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe2.hip -o tools/stream_probe2
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

__device__ __forceinline__ unsigned fold(u32x4 a, u32x4 b, u32x4 c) { return a.w ^ b.y ^ c.x ^ c.w; }

__global__ __launch_bounds__(1024) void all64_k(const u32x4 *in, unsigned char *v, size_t npkt) {
  const size_t nvec = npkt * 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 a = __builtin_nontemporal_load(in + i);
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if ((threadIdx.x & 3) == 0) v[i >> 2] = (unsigned char)(x & 1);
  }
}

// MODE 0: registers only, 1: LDS transpose, 2: LDS transpose + depth 2
template <int MODE>
__global__ __launch_bounds__(1024) void hdr48_k(const unsigned char *f, unsigned char *v, size_t npkt) {
  const unsigned lane = threadIdx.x & 63;
  u32x4 *hb = reinterpret_cast<u32x4 *>(smem + (threadIdx.x >> 6) * 3072);
  unsigned loff[3];
  for (int q = 0; q < 3; ++q) {
    const unsigned t = 64 * q + lane, fr = t / 3;
    loff[q] = fr * 64 + 16 * (t - 3 * fr);
  }
  const size_t step = (size_t)gridDim.x * blockDim.x;
  constexpr int D = MODE == 2 ? 2 : 1;
  u32x4 c[D][3];
  auto issue = [&](int d, size_t i) {
    size_t g = i - lane;
    if (g + 64 > npkt) g = npkt - 64;
    const unsigned char *gb = f + g * 64;
    for (int q = 0; q < 3; ++q) c[d][q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(gb + loff[q]));
  };
  const size_t first = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (int d = 0; d < D; ++d) issue(d, first + d * step);
  for (size_t i = first; i < npkt; i += D * step) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const size_t j = i + d * step;
      if (d && j >= npkt) break;
      u32x4 a, b, cc;
      if (MODE == 0) {
        a = c[d][0]; b = c[d][1]; cc = c[d][2];
      } else {
        for (int q = 0; q < 3; ++q) asm volatile("" : "+v"(c[d][q]));
        for (int q = 0; q < 3; ++q) hb[64 * q + lane] = c[d][q];
        __builtin_amdgcn_wave_barrier();
        a = hb[3 * lane]; b = hb[3 * lane + 1]; cc = hb[3 * lane + 2];
        __builtin_amdgcn_wave_barrier();
      }
      issue(d, j + D * step);
      v[j] = (unsigned char)(fold(a, b, cc) & 1);
    }
  }
}

// glds: chunk t = 64q + lane lands at hb + 16 * (64q + lane) (base + lane x 16)
template <int D>
__global__ __launch_bounds__(1024) void glds_k(const unsigned char *f, unsigned char *v, size_t npkt) {
  const unsigned lane = threadIdx.x & 63;
  unsigned char *wave = smem + (threadIdx.x >> 6) * (3072 * D);
  unsigned loff[3];
  for (int q = 0; q < 3; ++q) {
    const unsigned t = 64 * q + lane, fr = t / 3;
    loff[q] = fr * 64 + 16 * (t - 3 * fr);
  }
  const size_t step = (size_t)gridDim.x * blockDim.x;
  auto issue = [&](int d, size_t i) {
    size_t g = i - lane;
    if (g + 64 > npkt) g = npkt - 64;
    const unsigned char *gb = f + g * 64;
    for (int q = 0; q < 3; ++q)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(gb + loff[q]),
                                       (__attribute__((address_space(3))) void *)(wave + 3072 * d + 1024 * q),
                                       16, 0, 2);
  };
  const size_t first = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (int d = 0; d < D; ++d) issue(d, first + d * step);
  for (size_t i = first; i < npkt; i += D * step) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const size_t j = i + d * step;
      if (d && j >= npkt) break;
      // a glds is a pending VM op until it lands: wait until only younger ones
      // (the other buffer's three, and the verdict stores) may be outstanding
      if (D == 2 && d == 0) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if (D == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const u32x4 *hb = reinterpret_cast<const u32x4 *>(wave + 3072 * d);
      const u32x4 a = hb[3 * lane], b = hb[3 * lane + 1], cc = hb[3 * lane + 2];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(d, j + D * step);
      v[j] = (unsigned char)(fold(a, b, cc) & 1);
    }
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const size_t npkt = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 24);
  const size_t bytes = npkt * 64;
  unsigned char *f, *v;
  CK(hipMalloc(&f, bytes)); CK(hipMalloc(&v, npkt));
  CK(hipMemset(f, 1, bytes));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  auto all64 = [&] { hipLaunchKernelGGL(all64_k, dim3(cus), dim3(1024), 0, 0, (const u32x4 *)f, v, npkt); };
  auto h0 = [&] { hipLaunchKernelGGL(hdr48_k<0>, dim3(cus), dim3(1024), 0, 0, f, v, npkt); };
  auto h1 = [&] { hipLaunchKernelGGL(hdr48_k<1>, dim3(cus), dim3(1024), 16 * 3072, 0, f, v, npkt); };
  auto h2 = [&] { hipLaunchKernelGGL(hdr48_k<2>, dim3(cus), dim3(1024), 16 * 3072, 0, f, v, npkt); };
  auto g1 = [&] { hipLaunchKernelGGL(glds_k<1>, dim3(cus), dim3(1024), 16 * 3072, 0, f, v, npkt); };
  auto g2 = [&] { hipLaunchKernelGGL(glds_k<2>, dim3(cus), dim3(1024), 16 * 6144, 0, f, v, npkt); };
  // settle the clocks
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 1.0) {
    for (int k = 0; k < 32; ++k) all64();
    CK(hipDeviceSynchronize());
  }
  for (int rep = 0; rep < 2; ++rep) {
    struct { const char *name; float ms; } r[] = {
        {"all64", timeit(all64, 50)}, {"hdr48", timeit(h0, 50)}, {"hdr48_lds", timeit(h1, 50)},
        {"hdr48_pf2", timeit(h2, 50)}, {"glds", timeit(g1, 50)}, {"glds_pf2", timeit(g2, 50)}};
    for (auto &x : r)
      printf("%-10s %.4f ms  %6.0f GB/s (64 B/pkt)  %.1f Gpkt/s\n", x.name, x.ms, bytes / x.ms / 1e6, npkt / x.ms / 1e6);
  }
  return 0;
}
