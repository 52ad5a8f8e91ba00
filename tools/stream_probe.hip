// stream_probe.hip — measures the header-streaming ceiling of the classify
// access pattern on MI355X (no classification work):
//   copy     : float4 grid-stride copy (reference HBM rate)
//   read1k   : coalesced 16 B/lane reads of the whole frame buffer, 1 B/pkt store
//   stride64 : one lane per 64-byte frame, 3 x 16 B nt loads, 1 B verdict store
//   stride64x: as stride64 but 4 frames per lane (ILP 4)
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy_k(const u32x4 *in, u32x4 *out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = __builtin_nontemporal_load(in + i);
}

__global__ void read1k_k(const u32x4 *in, unsigned char *v, size_t npkt) {
  // 4 lanes per frame: lane reads 16 B; the frame's verdict from a 4-lane reduction
  size_t nvec = npkt * 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 a = __builtin_nontemporal_load(in + i);
    unsigned x = a.x ^ a.y ^ a.z ^ a.w;
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if ((threadIdx.x & 3) == 0) v[i >> 2] = (unsigned char)(x & 1);
  }
}

__global__ void stride64_k(const unsigned char *f, unsigned char *v, size_t npkt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < npkt; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 *p = (const u32x4 *)(f + i * 64);
    u32x4 a = __builtin_nontemporal_load(p), b = __builtin_nontemporal_load(p + 1), c = __builtin_nontemporal_load(p + 2);
    unsigned x = a.w ^ b.y ^ c.x ^ c.w;
    v[i] = (unsigned char)(x & 1);
  }
}

template <int ILP>
__global__ void stride64x_k(const unsigned char *f, unsigned char *v, size_t npkt) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i0 < npkt; i0 += stride * ILP) {
    u32x4 a[ILP], b[ILP], c[ILP];
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      size_t i = i0 + k * stride;
      if (i < npkt) {
        const u32x4 *p = (const u32x4 *)(f + i * 64);
        a[k] = __builtin_nontemporal_load(p); b[k] = __builtin_nontemporal_load(p + 1); c[k] = __builtin_nontemporal_load(p + 2);
      }
    }
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      size_t i = i0 + k * stride;
      if (i < npkt) v[i] = (unsigned char)((a[k].w ^ b[k].y ^ c[k].x ^ c[k].w) & 1);
    }
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char **argv) {
  size_t npkt = (size_t)1 << (argc > 1 ? atoi(argv[1]) : 24);
  size_t bytes = npkt * 64;
  unsigned char *f, *out, *v;
  CK(hipMalloc(&f, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&v, npkt));
  CK(hipMemset(f, 1, bytes));
  int cus = 256;
  for (int g : {1024, 2048, 4096}) {
    float ms = timeit([&] { hipLaunchKernelGGL(copy_k, dim3(g), dim3(256), 0, 0, (const u32x4 *)f, (u32x4 *)out, bytes / 16); }, 20);
    printf("copy      grid %5d: %.3f ms  %.0f GB/s (read+write)\n", g, ms, 2.0 * bytes / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(read1k_k, dim3(g), dim3(256), 0, 0, (const u32x4 *)f, v, npkt); }, 20);
    printf("read1k    grid %5d: %.3f ms  %.0f GB/s  %.1f Gpkt/s\n", g, ms, bytes / ms / 1e6, npkt / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(stride64_k, dim3(g), dim3(256), 0, 0, f, v, npkt); }, 20);
    printf("stride64  grid %5d: %.3f ms  %.0f GB/s  %.1f Gpkt/s\n", g, ms, bytes / ms / 1e6, npkt / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(stride64x_k<4>, dim3(g), dim3(256), 0, 0, f, v, npkt); }, 20);
    printf("stride64x4 grid %5d: %.3f ms  %.0f GB/s  %.1f Gpkt/s\n", g, ms, bytes / ms / 1e6, npkt / ms / 1e6);
  }
  (void)cus;
  return 0;
}
