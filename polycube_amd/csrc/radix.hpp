// radix.hpp — stable LSD radix sort of (key, batch index) pairs for the
// stateful pipeline (conntrack.hip): the key buckets of a batch sorted so each
// connection's packets form a run in batch order.  Hand-written for gfx950
// (radix.hip): one histogram pass over the keys for every digit, then one
// onesweep pass per digit (decoupled look-back between 8192-key tiles).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pcn {

struct RadixScratch {
  uint64_t cap = 0;                      // keys the buffers hold
  uint32_t *tk = nullptr, *tv = nullptr, *tv2 = nullptr;   // ping-pong keys / values
  unsigned long long *look = nullptr;    // look-back words: [tile][512] {epoch:32 | flag:2 | count:30}
  uint64_t look_tiles = 0;
  uint32_t *hist = nullptr;              // [4][512] digit counts (zero between sorts)
  uint32_t *offs = nullptr;              // [4][512] exclusive prefix of hist
  unsigned long long *tile_ctr = nullptr;   // tiles claimed so far (monotonic)
  unsigned long long tiles_issued = 0;   // host mirror: the counter's value before a pass
  uint32_t epoch = 0;                    // look-back words of older passes never match
  uint32_t *seg = nullptr;               // reduce-then-scan: super-tile counts, prefixes [2][group][512], totals [512]
  uint32_t seg_groups = 0;
};

// Sort keys_in[0..n) (every key < 2^kbits, kbits <= 36, n < 2^30) stably; the batch
// indices 0..n-1 ride along.  keys_in is clobbered (a ping-pong buffer).
// Stream-ordered, no host read-back.  Returns a hipError_t.
int radix_sort_pairs(RadixScratch &s, uint32_t *keys_in, uint32_t *keys_out, uint32_t *vals_out, uint64_t n,
                     uint32_t kbits, int num_cus, hipStream_t st);
void radix_free(RadixScratch &s);

}  // namespace pcn
