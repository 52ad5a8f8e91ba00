// radix.hpp — stable LSD radix sort of (key, batch index) pairs for the
// stateful pipeline (conntrack.hip): the key buckets of a batch sorted so each
// connection's packets form a run in batch order.  Hand-written for gfx950
// (radix.hip): per digit an up-sweep of per-super-tile counts, a column scan and
// a down-sweep that ranks and places 8192-key sub-tiles in order.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pcn {

struct RadixScratch {
  uint64_t cap = 0;                      // keys the buffers hold
  uint32_t *tk = nullptr, *tv = nullptr, *tv2 = nullptr;   // ping-pong keys / values
  uint32_t *seg = nullptr;               // super-tile counts and prefixes [2][group][512], digit totals [512]
  uint32_t seg_groups = 0;
};

// Sort keys_in[0..n) (every key < 2^kbits, kbits <= 36, n < 2^30) stably; the batch
// indices 0..n-1 ride along.  keys_in is clobbered (a ping-pong buffer).
// Stream-ordered, no host read-back.  Returns a hipError_t.
int radix_sort_pairs(RadixScratch &s, uint32_t *keys_in, uint32_t *keys_out, uint32_t *vals_out, uint64_t n,
                     uint32_t kbits, int num_cus, hipStream_t st);
void radix_free(RadixScratch &s);

}  // namespace pcn
