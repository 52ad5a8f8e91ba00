// gather_ceiling.hip -- the read ceiling of a scattered-header batch (config 5's
// IMIX offsets), measured on the bench's own device buffers: per frame, its
// offset (4 B) and length (2 B), the header window the classify kernel needs
// (bytes 0..51 from the frame start), and one verdict byte out -- no
// classification at all.  Four lanes per frame, one 16-byte load each from the
// frame's 16-byte-aligned start (a fifth chunk when the window crosses it),
// so one load instruction covers the contiguous bytes of 16 frames: the
// fastest of the gather shapes tools/gather_probe.hip compares.
//
// Measurement infrastructure, not product: bench.py loads it (ctypes) to put
// the ceiling next to the classify kernel's time in the config-5 line.
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/gather_ceiling.hip -o tools/libgather_ceiling.so
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void gather_quad_kernel(const uint8_t *f, const uint32_t *off, const uint16_t *len,
                                                          uint8_t *v, uint64_t n) {
  const uint32_t q = threadIdx.x & 3;
  const uint64_t step = uint64_t(gridDim.x) * blockDim.x / 4;
  for (uint64_t g = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 4; g < n; g += step) {
    const uint32_t o = off[g];
    const uint8_t *base = f + (o & ~15u);
    uint32_t x = q == 0 ? len[g] : 0u;
    const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base) + q);
    x ^= a.x ^ a.y ^ a.z ^ a.w;
    if (q == 0 && (o & 15) > 12) {             // the window [o, o + 52) runs into a fifth chunk
      const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base) + 4);
      x ^= b.x;
    }
    x ^= __shfl_xor(x, 1);
    x ^= __shfl_xor(x, 2);
    if (q == 0) v[g] = static_cast<uint8_t>(x & 1);
  }
}

// Average ms per launch over `iters` launches on `stream` (HIP events on that
// stream), after `warm` untimed ones; grid = 8 workgroups per CU.  Returns a
// hipError_t.  The caller guarantees 80 readable bytes past every frame's
// 16-byte-aligned start (the bench's buffers carry 64 bytes of tail padding
// and every IMIX frame is at least 64 bytes).
extern "C" int gather_ceiling_ms(const uint8_t *frames, const uint32_t *offsets, const uint16_t *lens, uint8_t *out,
                                 uint64_t n, int warm, int iters, void *stream, float *ms) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return int(e);
  const unsigned grid = static_cast<unsigned>(cus * 8);
  for (int k = 0; k < warm; ++k) hipLaunchKernelGGL(gather_quad_kernel, dim3(grid), dim3(256), 0, st, frames, offsets, lens, out, n);
  hipEvent_t a, b;
  if ((e = hipEventCreate(&a)) != hipSuccess) return int(e);
  if ((e = hipEventCreate(&b)) != hipSuccess) return int(e);
  (void)hipEventRecord(a, st);
  for (int k = 0; k < iters; ++k) hipLaunchKernelGGL(gather_quad_kernel, dim3(grid), dim3(256), 0, st, frames, offsets, lens, out, n);
  (void)hipEventRecord(b, st);
  e = hipEventSynchronize(b);
  float t = 0;
  if (e == hipSuccess) e = hipEventElapsedTime(&t, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  if (e == hipSuccess) *ms = t / static_cast<float>(iters);
  return int(e);
}
