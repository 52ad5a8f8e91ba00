// gather_rand.hip -- the read floor of the stateful walk's access pattern:
// 2^24 records of 32 (or 16) bytes read in the order of a random permutation
// (what the walk does through the sorted index: rec[sidx[q]]), against the
// same records read in order.  Each lane reads its index, then its record as
// 16-byte loads, and folds it into one output word.  Measurement only.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_rand.hip -o tools/gather_rand
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int Q>   // 16-byte chunks per record
__global__ __launch_bounds__(256) void gather_k(const u32x4 *rec, const uint32_t *idx, uint32_t *out, uint32_t n) {
  const uint32_t stp = gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += stp) {
    const uint32_t i = idx[q];
#pragma unroll
    for (int c = 0; c < Q; ++c) {
      const u32x4 v = rec[uint64_t(i) * Q + c];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int Q>
float run(const u32x4 *rec, const uint32_t *idx, uint32_t *out, uint32_t n, int grid) {
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(gather_k<Q>, dim3(grid), dim3(256), 0, 0, rec, idx, out, n);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  const int it = 20;
  for (int k = 0; k < it; ++k) hipLaunchKernelGGL(gather_k<Q>, dim3(grid), dim3(256), 0, 0, rec, idx, out, n);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / it;
}

int main() {
  const uint32_t n = 1u << 24;
  std::vector<uint32_t> perm(n);
  std::iota(perm.begin(), perm.end(), 0u);
  std::vector<uint32_t> ident = perm;
  std::shuffle(perm.begin(), perm.end(), std::mt19937(7));
  u32x4 *rec;
  uint32_t *dperm, *dident, *out;
  CK(hipMalloc(&rec, size_t(n) * 32));
  CK(hipMemset(rec, 1, size_t(n) * 32));
  CK(hipMalloc(&dperm, size_t(n) * 4));
  CK(hipMalloc(&dident, size_t(n) * 4));
  CK(hipMemcpy(dperm, perm.data(), size_t(n) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dident, ident.data(), size_t(n) * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int wpc : {8, 32}) {
    const int grid = cus * wpc;
    CK(hipMalloc(&out, size_t(grid) * 256 * 4));
    printf("grid %d x 256: 32 B random %.3f ms, in order %.3f ms; 16 B random %.3f ms, in order %.3f ms\n", grid,
           run<2>(rec, dperm, out, n, grid), run<2>(rec, dident, out, n, grid), run<1>(rec, dperm, out, n, grid),
           run<1>(rec, dident, out, n, grid));
    CK(hipFree(out));
  }
  return 0;
}
