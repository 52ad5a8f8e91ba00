// tools/rocprim_sort_ab.hip -- measurement only, never linked into the product.
// The rocPRIM onesweep radix sort of round 4, on the stateful pipeline's sort
// shape ((key bucket, index) pairs, kbits-bit keys, values a counting
// iterator), timed with HIP events, for an A/B against polycube_amd/csrc/radix.hip
// (the product sort; `tools/ct_probe.py` times it in the pipeline).  Moved out of
// conntrack.hip in round 6.
//   hipcc --offload-arch=gfx950 -O3 tools/rocprim_sort_ab.hip -o tools/rocprim_sort_ab
//   ./tools/rocprim_sort_ab [log2n=24] [kbits=24] [reps=20]
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

int main(int argc, char **argv) {
  const unsigned log2n = argc > 1 ? std::atoi(argv[1]) : 24, kbits = argc > 2 ? std::atoi(argv[2]) : 24;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
  const unsigned n = 1u << log2n;
  std::vector<uint32_t> h(n);
  uint32_t x = 0x9e3779b9u;
  for (auto &k : h) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    k = x & ((1u << kbits) - 1);
  }
  uint32_t *keys, *keys2, *vals;
  CK(hipMalloc(&keys, n * 4));
  CK(hipMalloc(&keys2, n * 4));
  CK(hipMalloc(&vals, n * 4));
  CK(hipMemcpy(keys, h.data(), n * 4, hipMemcpyHostToDevice));
  using Cfg = rocprim::radix_sort_config<
      rocprim::default_config, rocprim::default_config,
      rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, 9,
                                          rocprim::block_radix_rank_algorithm::match>>;
  size_t bytes = 0;
  void *tmp = nullptr;
  auto sort = [&](void *t, size_t &b) {
    return rocprim::radix_sort_pairs<Cfg>(t, b, keys, keys2, rocprim::counting_iterator<uint32_t>(0u), vals, n, 0u,
                                          kbits, hipStream_t(0));
  };
  CK(sort(nullptr, bytes));
  CK(hipMalloc(&tmp, bytes));
  for (int i = 0; i < 3; ++i) CK(sort(tmp, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) CK(sort(tmp, bytes));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("{\"sort\": \"rocprim onesweep 1024x8, 9-bit digits\", \"n\": %u, \"kbits\": %u, \"us_per_sort\": %.1f}\n",
              n, kbits, ms * 1e3 / reps);
  return 0;
}
