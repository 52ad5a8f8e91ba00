// classify.hip — the MI355X (gfx950) batch classifier for pcn-iptables.
//
// One lane per packet.  Each lane reads the 48-byte header window of its frame,
// runs the reference's Parser / ChainSelector / ConntrackLabel checks
// (Iptables_Parser_dp.c:94-153, Iptables_ChainSelector_dp.c:131-298,
// Iptables_ConntrackLabel_dp.c:436-531), maps every present field to a class id
// through the chain image (devchain.h), then finds the lowest rule whose bit
// survives the AND of all field vectors (the IpLookup/L4*/InterfaceLookup/
// TcpFlagsLookup/ConntrackMatch ANDs + BitScan + ActionLookup of
// Iptables_*_dp.c).  Instead of ANDing every word of every vector, the lane
// ANDs the per-vector word summaries first and only visits candidate words in
// ascending order: the first non-zero word of the full AND is the same word,
// so the rule id is identical.  Integer work only; no MFMA.
//
// Per-rule and default pkts/bytes counters are accumulated in an LDS histogram
// per workgroup (u64 LDS atomics; default bins are wave-aggregated with a
// ballot) and flushed once per workgroup with global u64 atomics.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "devchain.h"
#include "pcn_ipt.h"

namespace pcn {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t bswap16u(uint32_t x) { return ((x & 0xff) << 8) | ((x >> 8) & 0xff); }

// 48-byte header window as 12 little-endian dwords.
struct Hdr { uint32_t w[12]; };
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void load_fixed(const uint8_t *frame, Hdr &h) {
  const u32x4 *p = reinterpret_cast<const u32x4 *>(frame);
  u32x4 a = __builtin_nontemporal_load(p + 0);
  u32x4 b = __builtin_nontemporal_load(p + 1);
  u32x4 c = __builtin_nontemporal_load(p + 2);
  h.w[0] = a.x; h.w[1] = a.y; h.w[2] = a.z; h.w[3] = a.w;
  h.w[4] = b.x; h.w[5] = b.y; h.w[6] = b.z; h.w[7] = b.w;
  h.w[8] = c.x; h.w[9] = c.y; h.w[10] = c.z; h.w[11] = c.w;
}

// Unaligned frame start: 13 aligned dwords, each only if it lies inside the
// buffer, then byte-shifted into the window.
__device__ __forceinline__ void load_generic(const uint8_t *frames, uint64_t frames_bytes,
                                             uint64_t off, Hdr &h) {
  uint64_t base = off & ~uint64_t(3);
  uint32_t sh = static_cast<uint32_t>(off & 3);
  uint32_t d[13];
#pragma unroll
  for (int k = 0; k < 13; ++k) {
    uint64_t at = base + 4u * k;
    d[k] = (at + 4 <= frames_bytes) ? *reinterpret_cast<const uint32_t *>(frames + at) : 0u;
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) h.w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

__device__ __forceinline__ bool localip_has(const LaunchArgs &a, uint32_t ip) {
  uint32_t lo = 0, hi = a.nlocal;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    uint32_t v = a.localip[mid];
    if (v == ip) return true;
    if (v < ip) lo = mid + 1; else hi = mid;
  }
  return false;
}

__device__ __forceinline__ uint32_t lpm(const uint32_t *l1, const uint32_t *blk, uint32_t h) {
  uint32_t e = l1[h >> 16];
  if (e & PCN_IP_PTR) {
    e = blk[((e & ~PCN_IP_PTR) << 8) | ((h >> 8) & 0xff)];
    if (e & PCN_IP_PTR) e = blk[((e & ~PCN_IP_PTR) << 8) | (h & 0xff)];
  }
  return e;
}

struct Parsed {
  uint32_t saddr, daddr;       // NBO as loaded
  uint32_t proto, sport, dport, flags;
  uint32_t ct;                 // conntrack status 0..3 (or >3: invalid input)
};

// Rule-chain stage for lanes of one chain (ch is wave-uniform).
// Returns verdict; sets rid (>=0 rule, -1 default, -2 no-chain drop).
__device__ __forceinline__ uint32_t run_chain(const DevChain &ch, const Parsed &p, uint32_t port,
                                              int32_t &rid) {
  uint32_t cls[8];
  uint32_t nf = 0;
  bool miss = false;
  const uint32_t present = ch.present;
  if (present & (1u << PCN_IPT_F_CONNTRACK)) {
    if (p.ct > 3) { rid = PCN_IPT_RID_NOCHAIN; return PCN_IPT_DROP; }   // array miss => RX_DROP
    uint32_t c = ch.ct_cls[p.ct];
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if (present & (1u << PCN_IPT_F_IPSRC)) {
    uint32_t c = lpm(ch.ip_l1[0], ch.ip_blk[0], __builtin_bswap32(p.saddr));
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if (present & (1u << PCN_IPT_F_IPDST)) {
    uint32_t c = lpm(ch.ip_l1[1], ch.ip_blk[1], __builtin_bswap32(p.daddr));
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if (present & (1u << PCN_IPT_F_L4PROTO)) {
    uint32_t c = ch.proto_cls[p.proto];
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  const bool l4 = p.proto == 6 || p.proto == 17;   // L4PortLookup_dp.c:99-103
  if ((present & (1u << PCN_IPT_F_SPORT)) && l4) {
    uint32_t c = ch.key_cls[0][p.sport];
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if ((present & (1u << PCN_IPT_F_DPORT)) && l4) {
    uint32_t c = ch.key_cls[1][p.dport];
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if (present & (1u << PCN_IPT_F_IFACE)) {
    uint32_t c = ch.key_cls[2][port];
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if ((present & (1u << PCN_IPT_F_TCPFLAGS)) && p.proto == 6) {   // TcpFlagsLookup_dp.c:93-97
    uint32_t c = ch.flags_cls[p.flags];
    miss |= c == PCN_CLS_MISS; cls[nf] = c; nf += c != PCN_CLS_MISS;
  }
  if (miss) { rid = PCN_IPT_RID_DEFAULT; return static_cast<uint32_t>(ch.default_action); }

  const uint32_t nrw = ch.nrw, nsw = ch.nsw;
  int32_t rule = -1;
  for (uint32_t k = 0; k < nsw && rule < 0; ++k) {
    uint32_t live = nrw - k * 64;
    uint64_t m = live >= 64 ? ~0ull : ((1ull << live) - 1);
#pragma unroll
    for (int f = 0; f < 8; ++f)
      if (f < static_cast<int>(nf)) m &= ch.summ[cls[f] * nsw + k];
    while (m) {
      uint32_t w = k * 64 + static_cast<uint32_t>(__builtin_ctzll(m));
      uint64_t acc = 0x7FFFFFFFFFFFFFFFull;   // ChainSelector_dp.c:205-218 init
#pragma unroll
      for (int f = 0; f < 8; ++f)
        if (f < static_cast<int>(nf)) acc &= ch.pool[cls[f] * nrw + w];
      if (acc) { rule = static_cast<int32_t>(w * 63 + __builtin_ctzll(acc)); break; }
      m &= m - 1;
    }
  }
  if (rule < 0) { rid = PCN_IPT_RID_DEFAULT; return static_cast<uint32_t>(ch.default_action); }
  if (static_cast<uint32_t>(rule) >= ch.max_action) { rid = PCN_IPT_RID_NOCHAIN; return PCN_IPT_DROP; }
  rid = rule;
  return ch.actions[rule] ? PCN_IPT_ACCEPT : PCN_IPT_DROP;
}

template <bool FIXED>
__global__ __launch_bounds__(kBlock) void classify_kernel(const LaunchArgs a) {
  extern __shared__ unsigned long long bins[];   // [nbins][2]: pkts, bytes
  for (uint32_t b = threadIdx.x; b < 2 * a.nbins; b += blockDim.x) bins[b] = 0;
  __syncthreads();

  const uint64_t step = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t n_round = (a.n + step - 1) / step * step;   // uniform trip count per wave
  for (uint64_t i = first; i < n_round; i += step) {
    const bool valid = i < a.n;
    uint32_t verdict = PCN_IPT_DROP;
    int32_t rid = PCN_IPT_RID_NOCHAIN;
    int32_t cchain = -1;    // chain whose counters this packet bumps
    uint32_t L = 0;
    int32_t chain = -1;     // chain whose rules must run (-1: decided already)
    Parsed p{};
    uint32_t port = 0;
    if (valid) {
      Hdr h;
      if (FIXED) {
        load_fixed(a.frames + i * a.stride, h);
        L = a.fixed_len;
      } else {
        uint64_t off = a.offsets ? a.offsets[i] : i * a.stride;
        load_generic(a.frames, a.frames_bytes, off, h);
        L = a.lens ? a.lens[i] : a.fixed_len;
      }
      port = a.in_port ? a.in_port[i] : a.const_in_port;
      // ---- Parser_dp.c:94-153 ----
      bool done = true;
      if (L < 14) verdict = PCN_IPT_DROP;
      else if ((h.w[3] & 0xffff) != 0x0008) verdict = PCN_IPT_ACCEPT;   // ethertype != 0x0800
      else if (L < 34) verdict = PCN_IPT_DROP;
      else {
        p.proto = h.w[5] >> 24;
        p.saddr = (h.w[6] >> 16) | (h.w[7] << 16);
        p.daddr = (h.w[7] >> 16) | (h.w[8] << 16);
        done = false;
        if (p.proto == 6) {
          if (L < 54) { verdict = PCN_IPT_DROP; done = true; }
          p.flags = h.w[11] >> 24;
        } else if (p.proto == 17) {
          if (L < 42) { verdict = PCN_IPT_DROP; done = true; }
        }
        p.sport = bswap16u(h.w[8] >> 16);
        p.dport = bswap16u(h.w[9] & 0xffff);
      }
      if (!done) {
        // ---- ChainSelector_dp.c:131-298 ----
        bool pass = false;
        if (a.direction == PCN_IPT_INGRESS) {
          if (a.allow_logic) pass = true;
          else chain = (a.nlocal && localip_has(a, p.daddr)) ? PCN_IPT_INPUT : PCN_IPT_FORWARD;
        } else {
          if (a.nlocal && localip_has(a, p.saddr)) chain = PCN_IPT_OUTPUT;
          else { verdict = PCN_IPT_ACCEPT; done = true; }   // egress PASS
        }
        if (!done && chain >= 0 && a.ch[chain].nrules == 0) {
          cchain = chain; rid = PCN_IPT_RID_DEFAULT;       // default counters
          if (a.ch[chain].default_action == PCN_IPT_DROP) { verdict = PCN_IPT_DROP; done = true; }
          pass = true;
          chain = -1;
        }
        // ---- ConntrackLabel_dp.c:436-531 ICMP length checks ----
        uint32_t icmp_type = 0xffffffffu;
        if (!done && p.proto == 1) {
          icmp_type = (h.w[8] >> 16) & 0xff;
          if (L < 42) { verdict = PCN_IPT_DROP; done = true; }
          else if (icmp_type != 8 && icmp_type != 0 && !(icmp_type >= 13 && icmp_type <= 18) && L < 70) {
            verdict = PCN_IPT_DROP; done = true;
          }
        }
        if (!done) {
          if (a.ct_status) {
            p.ct = a.ct_status[i];
          } else if (p.proto == 6) {      // empty-table labels, ConntrackLabel_dp.c:372-383
            p.ct = (p.flags & 0x02) && ((p.flags | 0x02) == 0x02) ? 0u : 3u;
          } else if (p.proto == 17) {
            p.ct = 0;
          } else {
            p.ct = icmp_type == 8 ? 0u : 3u;
          }
          if (pass) { verdict = PCN_IPT_ACCEPT; done = true; }
        }
        if (done) chain = -1;
      }
    }
    // ---- rule chains: one wave-uniform chain at a time ----
    while (true) {
      uint64_t pending = __ballot(chain >= 0);
      if (!pending) break;
      int32_t c = __builtin_amdgcn_readfirstlane(__shfl(chain, __builtin_ctzll(pending)));
      if (chain == c) {
        verdict = run_chain(a.ch[c], p, port, rid);
        cchain = c;
        chain = -1;
      }
    }
    if (valid) {
      a.verdicts[i] = static_cast<uint8_t>(verdict);
      if (a.rule_ids) a.rule_ids[i] = rid;
    }
    // ---- counters ----
    // default bins: wave-aggregated per chain
    for (int c = 0; c < 3; ++c) {
      bool mine = valid && cchain == c && rid == PCN_IPT_RID_DEFAULT;
      uint64_t m = __ballot(mine);
      if (!m) continue;
      uint32_t bytes = mine ? L : 0u;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) bytes += __shfl_xor(bytes, o);
      if ((threadIdx.x & 63) == 0) {
        atomicAdd(&bins[2 * c], static_cast<unsigned long long>(__builtin_popcountll(m)));
        atomicAdd(&bins[2 * c + 1], static_cast<unsigned long long>(bytes));
      }
    }
    if (valid && cchain >= 0 && rid >= 0) {
      const DevChain &ch = a.ch[cchain];
      if (static_cast<uint32_t>(rid) < ch.ncounted) {
        if (ch.lds_base >= 0) {
          uint32_t b = static_cast<uint32_t>(ch.lds_base) + static_cast<uint32_t>(rid);
          atomicAdd(&bins[2 * b], 1ull);
          atomicAdd(&bins[2 * b + 1], static_cast<unsigned long long>(L));
        } else {
          atomicAdd(&ch.ctr[2 + 2 * rid], 1ull);
          atomicAdd(&ch.ctr[3 + 2 * rid], static_cast<unsigned long long>(L));
        }
      }
    }
  }
  __syncthreads();
  // ---- flush the workgroup histogram ----
  for (uint32_t b = threadIdx.x; b < a.nbins; b += blockDim.x) {
    unsigned long long pk = bins[2 * b], by = bins[2 * b + 1];
    if (!pk) continue;
    unsigned long long *dst;
    if (b < 3) {
      dst = a.ch[b].ctr;
    } else {
      int c = 0;
      for (; c < 3; ++c) {
        const DevChain &ch = a.ch[c];
        if (ch.lds_base >= 0 && b >= static_cast<uint32_t>(ch.lds_base) &&
            b < static_cast<uint32_t>(ch.lds_base) + ch.ncounted) break;
      }
      if (c == 3) continue;
      dst = a.ch[c].ctr + 2 + 2 * (b - static_cast<uint32_t>(a.ch[c].lds_base));
    }
    atomicAdd(dst, pk);
    atomicAdd(dst + 1, by);
  }
}

}  // namespace

// Host-side launcher (called from pcn_ipt.cpp).  Returns a hipError_t value.
int launch_classify(const LaunchArgs &a, bool fixed, int num_cus, hipStream_t stream) {
  if (a.n == 0) return hipSuccess;
  const uint64_t want = (a.n + kBlock - 1) / kBlock;
  const uint64_t cap = static_cast<uint64_t>(num_cus) * 8;
  const unsigned grid = static_cast<unsigned>(want < cap ? want : cap);
  const size_t lds = static_cast<size_t>(a.nbins) * 2 * sizeof(unsigned long long);
  if (fixed)
    hipLaunchKernelGGL(classify_kernel<true>, dim3(grid), dim3(kBlock), lds, stream, a);
  else
    hipLaunchKernelGGL(classify_kernel<false>, dim3(grid), dim3(kBlock), lds, stream, a);
  return static_cast<int>(hipGetLastError());
}

// Sum `nranks` gathered counter blocks into `out` (u64 element-wise).
__global__ void sum_ranks_kernel(const unsigned long long *in, unsigned long long *out, uint64_t count,
                                 int nranks) {
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= count) return;
  unsigned long long s = 0;
  for (int r = 0; r < nranks; ++r) s += in[static_cast<uint64_t>(r) * count + i];
  out[i] = s;
}

int launch_sum_ranks(const unsigned long long *in, unsigned long long *out, uint64_t count, int nranks,
                     hipStream_t stream) {
  if (count == 0) return hipSuccess;
  unsigned grid = static_cast<unsigned>((count + 255) / 256);
  hipLaunchKernelGGL(sum_ranks_kernel, dim3(grid), dim3(256), 0, stream, in, out, count, nranks);
  return static_cast<int>(hipGetLastError());
}

}  // namespace pcn
