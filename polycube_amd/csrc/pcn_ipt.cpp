// pcn_ipt.cpp — context, control plane mirror and C ABI (include/pcn_ipt.h).
//
// The control-plane half mirrors the reference's Chain / ChainRule / ChainStats
// objects (services/pcn-iptables/src/Chain.cpp, ChainRule.cpp, ChainStats.cpp):
// rule edits, interactive vs staged apply, read-and-flush counter accumulation.
// The datapath half owns the chain images in HBM (double-buffered per chain),
// the counters, and launches the HIP classify kernel (classify.hip).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "conntrack.hpp"
#include "radix.hpp"
#include "devchain.h"
#include "image.hpp"
#include "jit.hpp"
#include "pcn_ipt.h"
#include "ruleset.hpp"

namespace pcn {
int launch_classify(const LaunchArgs &a, bool fixed, int ch, int ns, int num_cus, void *jit, hipStream_t stream,
                    CopyBound *cb, void *jit2 = nullptr, const LaunchArgs *ga = nullptr, unsigned ga_wg = 0);
int launch_sum_ranks(const unsigned long long *in, unsigned long long *out, uint64_t count, int nranks,
                     hipStream_t stream);
int launch_fold_reps(unsigned long long *ctr, uint64_t pairs, uint64_t pack_off, uint64_t stride, uint32_t reps,
                     hipStream_t stream);
}  // namespace pcn

namespace pcn {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

}  // namespace pcn

namespace {

using namespace pcn;

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

#ifndef PCN_DEBUG_MAX_RULE_BINS
#define PCN_DEBUG_MAX_RULE_BINS 2048
#endif
#ifndef PCN_DEBUG_LDS_BUDGET
#define PCN_DEBUG_LDS_BUDGET (160 * 1024)
#endif
constexpr uint32_t kMaxLdsRuleBins = PCN_DEBUG_MAX_RULE_BINS;   // per-workgroup LDS histogram budget (16 KB of u32 pairs)
constexpr uint32_t kLdsBudget = PCN_DEBUG_LDS_BUDGET;  // gfx950 LDS per CU (one workgroup may take it all)

// Measurement knob (tools/ablate.py experiments): bytes per wave region
// (default PCN_WAVE_LDS_BYTES; a kernel built without the header transpose
// needs only its candidate scratch).
// LDS counter bins for the lowest rule ids of a chain too large for a bin
// per rule, in what is left of the LDS budget after `used` bytes (the bins
// round up to 16 bytes): first-match traffic falls on low rule ids more
// often than on high ones (an earlier rule shadows later ones).  0: too few
// to bother.
uint32_t partial_rule_bins(uint32_t used, uint32_t per_bin, uint32_t ncounted) {
  constexpr uint32_t kMinBins = 256;
  if (used + 16 + kMinBins * per_bin > kLdsBudget) return 0;
  const uint32_t nb = (kLdsBudget - used - 16) / per_bin;
  return nb < ncounted ? nb : ncounted;
}

// PCN_IPT_DEBUG_CLOCKS=1: classify launches record per-workgroup clocks
// (LaunchArgs::dbg_clk; pcn_ipt_debug_clocks reads the last launch's)
bool debug_clocks() {
  static const bool v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_CLOCKS");
    return e && *e == '1';
  }();
  return v;
}
constexpr uint32_t kDbgClkGrid = 4096;

// PCN_IPT_DEBUG_STAGE_A_COUNTS=1: stage A counts into its scratch block again (A/B)
bool debug_stage_a_counts() {
  static const bool v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_STAGE_A_COUNTS");
    return e && e[0] == '1';
  }();
  return v;
}

// PCN_IPT_DEBUG_DEAL2_MULTI=0: chains of 2+ summary blocks deal 64 candidates a
// pass too (no 128-item wave region: that LDS goes to counter bins); A/B
bool multi_block_deal2() {
  static const bool v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_DEAL2_MULTI");
    return !(e && *e == '0');
  }();
  return v;
}

// Split launches (classify.hip SPLIT): offsets / lens batches of a chain whose
// image does not fit LDS (dense PART: config 5) may run a gather kernel of
// PCN_SPLIT_G_BLOCK-thread workgroups, several per CU, and then the rule
// kernel over its records.  Built, bit-exact and measured slower than the one
// fused kernel (config 5 XDP 134 -> 201-213 us: gather 123 + rules 85 us,
// profiles/r06_s2/), so off unless a context is created with
// PCN_IPT_DEBUG_SPLIT=1 in the environment (read per context, for the tests'
// and the A/B's sake).  PCN_IPT_DEBUG_SPLIT_WG: the gather kernel's
// workgroups per CU (default 6: its ~75 VGPRs allow 6 waves per SIMD).
// PCN_IPT_DEBUG_CT_FUSED=0: stateful batches always run ct_prep (A/B of the
// stage A that writes the walk records)
bool ct_fused_prep() {
  static const bool v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_CT_FUSED");
    return !(e && *e == '0');
  }();
  return v;
}

bool split_env() {
  const char *e = std::getenv("PCN_IPT_DEBUG_SPLIT");
  return e && std::atoi(e) == 1;
}
unsigned split_gather_wg() {
  static const unsigned v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_SPLIT_WG");
    const long x = e ? std::strtol(e, nullptr, 10) : 6;
    return x >= 1 && x <= 32 ? static_cast<unsigned>(x) : 6u;
  }();
  return v;
}

// PCN_IPT_DEBUG_FIXED_ALIGN=16: fixed-stride batches only at 16-byte strides (A/B of the
// dword-aligned fixed path; 4 otherwise)
uint32_t fixed_align() {
  static const uint32_t v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_FIXED_ALIGN");
    return e && std::strtol(e, nullptr, 10) == 16 ? 16u : 4u;
  }();
  return v;
}

// PCN_IPT_DEBUG_SHALLOW=0: keep prefetch depth 2 for launches of few frames
// per lane (A/B of JitShape::shallow)
bool shallow_prefetch() {
  static const bool v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_SHALLOW");
    return !(e && *e == '0');
  }();
  return v;
}

// Adaptive deal window (launch_batch): 1 on (default), 0 off (the 64-candidate
// chain program always), 2 the 128 one always (A/B): PCN_IPT_DEBUG_DEAL_ADAPT.
int deal_adapt() {
  static const int v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_DEAL_ADAPT");
    return e ? std::atoi(e) : 1;
  }();
  return v;
}
constexpr uint32_t kDealStatsSlots = 1024;   // workgroups a counted launch may have

uint32_t wave_region_bytes(bool fixed, bool deal2) {
  static const uint32_t v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_WAVE_BYTES");
    return e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : uint32_t(PCN_WAVE_LDS_BYTES);
  }();
  // only the fixed-stride path transposes headers through the region
  // (PCN_IPT_DEBUG_WAVE_BYTES_GENERIC: a larger candidate scratch elsewhere, A/B)
  static const uint32_t g = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_WAVE_BYTES_GENERIC");
    return e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : uint32_t(PCN_WAVE_SCRATCH_BYTES);
  }();
  // a chain program with the 128-candidate deal window (jit.cpp) needs its scratch
  return fixed ? v : deal2 ? std::max<uint32_t>(g, PCN_DEAL2_WAVE_BYTES) : g;
}

struct ImageSlot {
  void *tables = nullptr;
  size_t tables_cap = 0;
};

void ensure(void *&buf, size_t &cap, size_t need) {
  if (cap >= need && buf) return;
  if (buf) hip_check(hipFree(buf), "hipFree");
  buf = nullptr;
  cap = std::max<size_t>(need, 4096);
  hip_check(hipMalloc(&buf, cap), "hipMalloc(chain image)");
}

struct ChainState {
  // control plane (Chain)
  std::vector<Rule> rules;
  int default_action = PCN_IPT_ACCEPT;        // Iptables.cpp:33-38
  std::vector<std::pair<uint64_t, uint64_t>> stats;   // ChainStats totals (counters_)
  ChainTables tables;                          // last applied compile
  pcn_ipt_chain_info info{};                   // shape of the last built image
  std::vector<uint8_t> image_copy;             // host copy of the last built table image
  std::vector<uint32_t> desc_words;            // TableLayout words + nrw, nsw, present, all_cls
  // datapath
  ImageSlot slot[2];
  int active = -1;
  DevChain desc{};                             // descriptor of the active slot
  unsigned long long *ctr = nullptr;           // [2 + 2*max_counted]
  unsigned long long *ctr_global = nullptr;    // summed over ranks
  unsigned long long *gather = nullptr;        // [nranks][2 + 2*max_counted]
  unsigned long long *stage = nullptr;         // snapshot of ctr the all-gather sends
  // chain program of the last launch shape (jit.hpp): descriptor + shape it was made for
  DevChain jit_desc{};
  JitShape jit_shape{};
  std::string jit_spec;
  uint32_t last_lds_bytes = 0;                 // dynamic LDS of the last launch that ran this chain's rules
  bool deal_wide = false;                      // adaptive deal window: the 128-candidate program in use
  std::string last_spec;                       // the chain program the last launch ran (empty: generic)
};

// One Horus program (pcn_ipt.h): pcn-iptables has one (ingress, built from
// INPUT); pcn-firewall one per chain (Firewall.h:333-340).
struct HorusProg {
  bool runtime = false;                        // horus_runtime_enabled_
  bool ct = false;                             // pcn-firewall: _CONNTRACK_ENABLED when built
  uint32_t fields = 0, entries = 0, mask = 0, probes = 0;
  uint32_t nids = 0;                           // 1 + the largest rule id in the table
  uint32_t *d_tab = nullptr;                   // 4 u32 per slot
  size_t cap = 0;
  unsigned long long *d_ctr = nullptr;         // [PCN_IPT_HORUS_MAX][2]
};

}  // namespace

struct pcn_ipt {
  pcn_ipt_config cfg{};
  std::mutex mu;
  PortTable ports;
  ChainState chains[PCN_IPT_NCHAINS];
  std::vector<uint32_t> localip;
  uint32_t *d_localip = nullptr;
  uint8_t *d_zero = nullptr;                   // 64 zero bytes: stand-in in_port / ct_status
  bool interactive = true;                     // Iptables.h:181
  int service = PCN_IPT_SERVICE_IPTABLES;      // pcn_ipt_set_service
  int fw_ct_mode = PCN_FW_CT_AUTOMATIC;        // pcn-firewall conntrackMode (Firewall.h:323)
  bool has_device = false;
  int num_cus = 256;
  size_t ctr_words = 0;
  uint32_t ctr_reps = 1;                       // counter copies per chain (LaunchArgs::ctr_rep_mask)
  // Packed copies (LaunchArgs::ctr_pack_off): the most any copy can hold since
  // the last full fold, the streams that launched into them since then, and
  // the event a full fold uses to wait for those streams' work.
  // With more than one stream in play each launch records an event on its
  // stream, and the fold waits on those (no stream handle is used later).
  CopyBound pack{};
  std::vector<std::pair<hipStream_t, hipEvent_t>> pack_streams;
  // per chain: device work that can add to its counters was queued since
  // fetch_stats last read them (else they are all zero and the read, a device
  // sync, a fold and a copy per rule append, is skipped)
  bool ctr_dirty[PCN_IPT_NCHAINS] = {false, false, false};
  ncclComm_t comm = nullptr;
  // the counter all-gather runs on its own stream, off the classify stream's
  // critical path: the classify stream only snapshots the counters
  hipStream_t comm_stream = nullptr;
  hipEvent_t ev_staged = nullptr, ev_gathered = nullptr;
  bool gather_pending = false;
  int nranks = 1, rank = 0;
  // timing of the all-gather steps on the communicator stream: a ring of
  // event pairs, folded into the sum once complete (pcn_ipt_comm_get_info)
  static constexpr int kGatherEv = 8;
  hipEvent_t ev_g0[kGatherEv] = {}, ev_g1[kGatherEv] = {};
  bool ev_g_live[kGatherEv] = {};
  int ev_g_next = 0;
  uint64_t gathers_timed = 0, gathers_untimed = 0;
  double gather_ms = 0.0;
  JitCache jit;                                // chain programs (per launch shape)
  uint64_t launches_generic = 0, launches_jit = 0;
  // accept-established optimization per chain (Iptables.h accept_established_enabled_*)
  bool ae[PCN_IPT_NCHAINS] = {false, false, false};
  unsigned long long *d_ae = nullptr;          // [3][2] pkts/bytes_acceptestablished_<Chain>
  // stateful conntrack (conntrack.hpp)
  bool ct_on = false;
  CtTable ct;
  CtScratch *cts = nullptr;
  uint8_t *d_labels = nullptr;                 // {0, 1, 2, 3}: constant labels of the stage-A runs
  unsigned long long *ctr_scratch = nullptr;   // [3][ctr_words]: stage-A counters (discarded)
  void *ct_buf = nullptr;                      // stage-A outcomes + a rule-id array
  size_t ct_buf_cap = 0;
  // Stateful batches share ct_buf, the CtScratch buffers and the table, so
  // they run one after another in submission order whatever stream each
  // comes on: the next one's stage A waits for this event, recorded after
  // the previous one's last conntrack kernel.
  hipEvent_t ev_ct = nullptr;
  bool ct_pending = false;
  // Horus (pcn_ipt.h): the flag and the programs in place with their counters:
  // [0] pcn-iptables INPUT / pcn-firewall INGRESS, [1] pcn-firewall EGRESS
  bool hz_enabled = false;
  HorusProg hz[2];
  uint32_t *d_hz_carry = nullptr;              // the Parser's stale ports while conntrack is off
  // the classify kernel's stale-port groups (classify.hip stale_lookback)
  uint64_t *d_stale_desc = nullptr;            // one word per 64-frame group
  size_t stale_groups = 0;
  size_t stale_guard_from = 0;                 // first guard word (pcn_ipt_debug_stale_canary)
  uint32_t stale_epoch = 0;                    // bumped per launch (24 bits)
  uint32_t *d_chunk_ctr = nullptr;
  // adaptive deal window (launch_batch): per workgroup of the last launch that
  // counted, its waves that dealt more than 64 candidates (host-mapped, written
  // by the kernel); that launch's grid and frames (0: nothing counted since)
  uint32_t *h_deal_stats = nullptr;
  uint32_t deal_grid = 0;
  uint64_t deal_frames = 0;
  // PCN_IPT_DEBUG_CLOCKS=1: per-workgroup clocks of the last classify launch
  unsigned long long *d_dbg_clk = nullptr;
  uint32_t dbg_grid = 0;
  // split launches: the gather kernel's records (16 B a frame), grown to the largest batch
  uint32_t *d_split_rec = nullptr;
  uint64_t split_cap = 0;
  bool split = false;                      // split launches allowed (PCN_IPT_DEBUG_SPLIT=1 at creation)
  uint64_t ct_fused_batches = 0;           // stateful batches whose stage A wrote the walk records
  uint64_t launches_split = 0;
};

namespace pcn {
// HIP device of a context, or -1 for a control-plane-only context (ring.cpp).
int device_of(const pcn_ipt *ctx) { return ctx && ctx->has_device ? ctx->cfg.device : -1; }
}  // namespace pcn

namespace {

void device_guard(pcn_ipt *ctx) {
  if (ctx->has_device) hip_check(hipSetDevice(ctx->cfg.device), "hipSetDevice");
}

// Guard words past the stale-port groups: a kernel that published a group
// past its batch would overwrite one (pcn_ipt_debug_stale_canary).
constexpr size_t kStaleCanary = 16;
constexpr int kStaleCanaryByte = 0xA5;
// PCN_IPT_DEBUG_STALE_CANARY=1: guard every word past each batch's groups
// (a memset per launch that is smaller than the largest; tests only, read at
// every launch so a test can set it)
bool debug_stale_canary() {
  const char *e = std::getenv("PCN_IPT_DEBUG_STALE_CANARY");
  return e && *e == '1';
}

// Measurement knob (tools/ablate.py): PCN_IPT_DEBUG_GRID_CUS=k sizes the
// classify grid as if the device had k CUs (the grid is min(frames / 1024,
// CUs x workgroups per CU)).
int classify_grid_cus(int num_cus) {
  static const int v = [] {
    const char *e = std::getenv("PCN_IPT_DEBUG_GRID_CUS");
    return e ? std::atoi(e) : 0;
  }();
  return v > 0 ? v : num_cus;
}

// Add the duration of all-gather step k (its event pair on the communicator
// stream) to the context's total; waits for it if it is still running.
void fold_gather_time(pcn_ipt *ctx, int k) {
  hip_check(hipEventSynchronize(ctx->ev_g1[k]), "hipEventSynchronize");
  float ms = 0.f;
  hip_check(hipEventElapsedTime(&ms, ctx->ev_g0[k], ctx->ev_g1[k]), "hipEventElapsedTime");
  ctx->gather_ms += ms;
  ++ctx->gathers_timed;
  ctx->ev_g_live[k] = false;
}

uint32_t counted(const pcn_ipt *ctx, uint32_t nrules) {
  return std::min(nrules, ctx->cfg.max_counted_rules);
}

// Packed counter copies per chain block (LaunchArgs::ctr_rep_mask): 64, or
// PCN_IPT_DEBUG_CTR_REPS (a power of two, measurement A/B).  A/B on config 2 at
// 2^20 frames, 1 / 16 / 64 copies: 43.5 / 28.4 / 27.4 us a launch; config 3:
// 213 / 209 / 207 us; config 5: 166 / 162 us (profiles/r04_s2/).
uint32_t ctr_reps_default() {
  const char *e = std::getenv("PCN_IPT_DEBUG_CTR_REPS");
  const long v = e ? std::strtol(e, nullptr, 10) : 64;
  return v >= 1 && v <= 256 && (v & (v - 1)) == 0 ? static_cast<uint32_t>(v) : 64u;
}

// Fold a chain's packed counter copies into its plain block (cs.ctr, the
// first ctr_words words; the copies follow it), the pairs of the block's
// first `words` words, stream-ordered; every read, snapshot or clear of a
// block does this first.
void fold_counters(pcn_ipt *ctx, const ChainState &cs, size_t words, hipStream_t s) {
  if (!cs.ctr) return;
  const int rc = launch_fold_reps(cs.ctr, (words + 1) / 2, ctx->ctr_words, ctx->ctr_words / 2, ctx->ctr_reps, s);
  if (rc != hipSuccess) throw HipError(std::string("counter fold: ") + hipGetErrorString(hipError_t(rc)));
}

// Every chain's copies folded on `stream` once the work queued so far on the
// other streams that launched into them has run: the launches queued before
// this fold are then all in it, so the copies hold at most what launches
// queued after it add, which is what pcn_ipt::pack counts from zero again.
// launch_classify calls it before a launch that could overflow a field of a
// copy (every ~60 launches of 2^22 IMIX frames, ~250 of 2^24 64-byte frames).
int fold_all_copies(void *c, void *stream) {
  pcn_ipt *ctx = static_cast<pcn_ipt *>(c);
  const hipStream_t s = static_cast<hipStream_t>(stream);
  try {
    for (const auto &se : ctx->pack_streams)
      if (se.first != s && se.second) hip_check(hipStreamWaitEvent(s, se.second, 0), "hipStreamWaitEvent(fold)");
    for (const ChainState &cs : ctx->chains) fold_counters(ctx, cs, ctx->ctr_words, s);
  } catch (const HipError &) {
    return static_cast<int>(hipErrorUnknown);
  }
  // the streams stay known (their events are reused); only the bound restarts
  ctx->pack.pkts = ctx->pack.bytes = 0;
  return hipSuccess;
}

// Bookkeeping of the launches into the packed copies, in two halves around a
// launch on stream s.  Before it (register_pack_stream): s joins the known
// streams, and when that makes two or more, every other known stream records
// its event now, at the end of what it has queued (an event recorded earlier
// may predate batches queued while it was the only stream: once the other
// streams are released, note_pack_stream records nothing) -- so a fold inside
// this very launch (launch_classify, cb->fold) waits for all their work, and no
// stream handle is ever used after the launch that introduced it.
// After it (note_pack_stream): once two streams are known, the launch leaves
// an event behind on s.  With one stream neither records anything.
void register_pack_stream(pcn_ipt *ctx, hipStream_t s) {
  auto &v = ctx->pack_streams;
  if (std::find_if(v.begin(), v.end(), [&](const auto &se) { return se.first == s; }) != v.end()) return;
  v.emplace_back(s, nullptr);
  if (v.size() < 2) return;
  for (auto &se : v) {
    if (se.first == s) continue;
    if (!se.second) hip_check(hipEventCreateWithFlags(&se.second, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(se.second, se.first), "hipEventRecord(pack)");
  }
}

void note_pack_stream(pcn_ipt *ctx, hipStream_t s) {
  auto &v = ctx->pack_streams;
  if (v.size() < 2) return;
  for (auto &se : v) {
    if (se.first != s) continue;
    if (!se.second) hip_check(hipEventCreateWithFlags(&se.second, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(se.second, se.first), "hipEventRecord(pack)");
  }
}

// Upload a compiled chain into the inactive slot, then flip (Chain.cpp:441-457,924).
void load_tables(pcn_ipt *ctx, int chain, ChainTables tables) {
  ChainState &cs = ctx->chains[chain];
  HostImage img = build_image(tables);       // may throw (trie capacity etc.)
  cs.image_copy = img.tables;
  cs.desc_words.assign(reinterpret_cast<const uint32_t *>(&img.lay),
                       reinterpret_cast<const uint32_t *>(&img.lay) + sizeof(TableLayout) / 4);
  cs.desc_words.insert(cs.desc_words.end(), {img.nrw, img.nsw, img.present, img.all_cls});
  cs.info = pcn_ipt_chain_info{img.nrules, img.nrw, img.nsw, img.nvec, img.ngroups, img.present,
                               img.lay.bytes, img.part_bytes};
  DevChain d{};
  d.lay = img.lay;
  d.nrules = img.nrules;
  d.nrw = img.nrw;
  d.nsw = img.nsw;
  d.present = img.present;
  d.nvec = img.nvec;
  d.all_cls = img.all_cls;
  d.ncounted = counted(ctx, img.nrules);
  d.max_action = ctx->cfg.max_action_rules;
  d.default_action = img.default_action;
  d.lds_image = 0;
  d.lds_bins = -1;
  d.lds_nrules = 0;
  if (ctx->has_device) {
    device_guard(ctx);
    // every batch queued before this call must not see a half-written slot
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    int next = cs.active < 0 ? 0 : 1 - cs.active;
    ImageSlot &s = cs.slot[next];
    ensure(s.tables, s.tables_cap, img.tables.size());
    hip_check(hipMemcpy(s.tables, img.tables.data(), img.tables.size(), hipMemcpyHostToDevice),
              "hipMemcpy(chain tables)");
    // a new ActionLookup program starts with zeroed per-rule counters; the
    // default counters live in shared maps and persist (Iptables_Parser_dp.c:47-58)
    fold_counters(ctx, cs, ctx->ctr_words, nullptr);
    hip_check(hipMemset(cs.ctr + 2, 0, (ctx->ctr_words - 2) * sizeof(unsigned long long)),
              "hipMemset(counters)");
    d.image = static_cast<const uint8_t *>(s.tables);
    d.ctr = cs.ctr;
    cs.active = next;
  }
  // (without a device the descriptor still describes the chain: a chain
  // program can be planned and compiled, pcn_ipt_chain_program_compile)
  cs.desc = d;
  cs.tables = std::move(tables);
}

// The Horus program a chain's updates rebuild: pcn-iptables INPUT -> [0];
// pcn-firewall INGRESS (FORWARD slot) -> [0], EGRESS (OUTPUT slot) -> [1].
int horus_slot(const pcn_ipt *ctx, int chain) {
  if (ctx->service == PCN_IPT_SERVICE_FIREWALL) return chain == PCN_IPT_FORWARD ? 0 : chain == PCN_IPT_OUTPUT ? 1 : -1;
  return chain == PCN_IPT_INPUT ? 0 : -1;
}

// The program whose counters a chain's stats take.
HorusProg *horus_stats_prog(pcn_ipt *ctx, int chain) {
  if (ctx->service != PCN_IPT_SERVICE_FIREWALL) return &ctx->hz[0];
  const int k = horus_slot(ctx, chain);
  return k < 0 ? nullptr : &ctx->hz[k];
}

// The program a batch's Parser calls, if one is in place: pcn-iptables
// ingress only (the egress Parser's tail call lands on an empty slot);
// pcn-firewall the direction's own.
const HorusProg *horus_of_batch(const pcn_ipt *ctx, int direction) {
  const HorusProg *h = ctx->service == PCN_IPT_SERVICE_FIREWALL ? &ctx->hz[direction == PCN_IPT_INGRESS ? 0 : 1]
                       : direction == PCN_IPT_INGRESS ? &ctx->hz[0] : nullptr;
  return h && h->runtime ? h : nullptr;
}

// ChainStats::fetchCounters for every rule (read-and-flush into host totals),
// i.e. Chain::getStatsList (Chain.cpp:961-976) without the DEFAULT row.
void fetch_stats(pcn_ipt *ctx, int chain) {
  ChainState &cs = ctx->chains[chain];
  cs.stats.resize(cs.rules.size());
  if (!ctx->has_device || cs.active < 0 || !ctx->ctr_dirty[chain]) return;
  device_guard(ctx);
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  ctx->ctr_dirty[chain] = false;
  uint32_t n = counted(ctx, cs.desc.nrules);
  std::vector<unsigned long long> buf(2 + 2 * size_t(n));
  fold_counters(ctx, cs, buf.size(), nullptr);
  hip_check(hipMemcpy(buf.data(), cs.ctr, buf.size() * 8, hipMemcpyDeviceToHost), "hipMemcpy(counters)");
  for (uint32_t id = 0; id < n && id < cs.stats.size(); ++id) {
    cs.stats[id].first += buf[2 + 2 * id];
    cs.stats[id].second += buf[3 + 2 * id];
  }
  hip_check(hipMemset(cs.ctr + 2, 0, 2 * size_t(n) * 8), "hipMemset(counters)");
  // while a Horus program is in place, rule k of the chain read also takes
  // (and flushes) its counters of rule id k: pcn-iptables' one program
  // whichever chain is read (ChainStats.cpp:106-121), pcn-firewall's the
  // chain's own (pcn-firewall ChainStats.cpp:127-143)
  const HorusProg *hp = horus_stats_prog(ctx, chain);
  if (hp && hp->runtime && !cs.stats.empty()) {
    const size_t m = std::min<size_t>(cs.stats.size(), PCN_IPT_HORUS_MAX);
    std::vector<unsigned long long> hz(2 * m);
    hip_check(hipMemcpy(hz.data(), hp->d_ctr, hz.size() * 8, hipMemcpyDeviceToHost), "hipMemcpy(horus counters)");
    for (size_t id = 0; id < m; ++id) {
      cs.stats[id].first += hz[2 * id];
      cs.stats[id].second += hz[2 * id + 1];
    }
    hip_check(hipMemset(hp->d_ctr, 0, hz.size() * 8), "hipMemset(horus counters)");
  }
  // rule 0 of an accept-established chain also takes (and flushes) the
  // accept-established counters (ChainStats.cpp:64-103)
  if (ctx->ae[chain] && !cs.stats.empty()) {
    unsigned long long ae[2];
    hip_check(hipMemcpy(ae, ctx->d_ae + 2 * chain, 16, hipMemcpyDeviceToHost), "hipMemcpy(ae counters)");
    cs.stats[0].first += ae[0];
    cs.stats[0].second += ae[1];
    hip_check(hipMemset(ctx->d_ae + 2 * chain, 0, 16), "hipMemset(ae counters)");
  }
}

// ChainRule::applyAcceptEstablishedOptimization (ChainRule.cpp:211-238) ->
// Iptables::enable/disableAcceptEstablished (Iptables.cpp:351-449): rule 0 is
// exactly {conntrack ESTABLISHED, action ACCEPT}.  The disable switch has no
// `break`, so disabling INPUT also disables FORWARD and OUTPUT.
void apply_ae(pcn_ipt *ctx, int chain) {
  if (ctx->service == PCN_IPT_SERVICE_FIREWALL) return;   // pcn-firewall has no per-chain optimization
  const auto &rules = ctx->chains[chain].rules;
  bool found = false;
  if (!rules.empty()) {
    const Rule &r = rules[0];
    found = r.conntrack && *r.conntrack == 1 && r.action == PCN_IPT_ACCEPT && !r.src && !r.dst && !r.l4proto &&
            !r.sport && !r.dport && !r.tcpflags && !r.in_iface && !r.out_iface;
  }
  if (found) ctx->ae[chain] = true;
  else for (int c = chain; c < PCN_IPT_NCHAINS; ++c) ctx->ae[c] = false;
}

// Chain::fromRuleToHorusKeyValue + horusFromRulesToMap (pcn-iptables
// Utils.cpp:537-630, pcn-firewall Utils.cpp:483-577): the leading rules that
// set the same key fields as rule 0 (a /32 address, protocol, ports), up to
// the first conntrack rule; a repeated key keeps its first rule
// (std::map::insert).
struct HorusEntry {
  uint32_t src, dst, ports, meta;   // devchain.h slot layout
};
std::vector<HorusEntry> horus_entries(const std::vector<Rule> &rules, uint32_t &fields) {
  std::vector<HorusEntry> out;
  uint32_t set_fields = 0;
  HorusEntry key{0, 0, 0, 0};
  uint8_t proto = 0;
  for (size_t i = 0; i < rules.size() && i < PCN_IPT_HORUS_MAX; ++i) {
    const Rule &r = rules[i];
    if (r.conntrack) break;
    uint32_t f = 0;
    if (r.src && r.src->len == 32) { f |= PCN_IPT_HZ_SRCIP; key.src = r.src->ip; }
    if (r.dst && r.dst->len == 32) { f |= PCN_IPT_HZ_DSTIP; key.dst = r.dst->ip; }
    if (r.l4proto) { f |= PCN_IPT_HZ_L4PROTO; proto = *r.l4proto; }
    // ports: htons(port) as the packed key holds it (modules/Horus.cpp:44-51), read as a LE u16
    auto be = [](uint16_t x) { return static_cast<uint32_t>(((x & 0xff) << 8) | (x >> 8)); };
    if (r.sport) { f |= PCN_IPT_HZ_SRCPORT; key.ports = (key.ports & 0xffff0000u) | be(*r.sport); }
    if (r.dport) { f |= PCN_IPT_HZ_DSTPORT; key.ports = (key.ports & 0xffffu) | (be(*r.dport) << 16); }
    if (i == 0) {
      if (!f) break;
      set_fields = f;
    }
    if (f != set_fields) break;
    HorusEntry e{(f & PCN_IPT_HZ_SRCIP) ? key.src : 0u, (f & PCN_IPT_HZ_DSTIP) ? key.dst : 0u,
                 ((f & PCN_IPT_HZ_SRCPORT) ? (key.ports & 0xffffu) : 0u) |
                     ((f & PCN_IPT_HZ_DSTPORT) ? (key.ports & 0xffff0000u) : 0u),
                 ((f & PCN_IPT_HZ_L4PROTO) ? proto : 0u) | (r.action == PCN_IPT_ACCEPT ? 0x100u : 0u) |
                     kHorusUsed | (static_cast<uint32_t>(i) << 16)};
    bool dup = false;
    for (const HorusEntry &x : out)
      dup = dup || (x.src == e.src && x.dst == e.dst && x.ports == e.ports && (x.meta & 0xff) == (e.meta & 0xff));
    if (!dup) out.push_back(e);
  }
  fields = set_fields;
  return out;
}

// Drop a program (and its counters), then, with entries, build its table:
// open addressing at load <= 1/2, linear probing; the kernel probes at most
// `probes` slots.
void horus_set(pcn_ipt *ctx, HorusProg &h, const std::vector<HorusEntry> &ents, uint32_t fields) {
  h.runtime = false;
  h.entries = h.fields = h.nids = 0;
  if (ctx->has_device) {
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipMemset(h.d_ctr, 0, PCN_IPT_HORUS_MAX * 16), "hipMemset(horus counters)");
  }
  if (ents.empty()) return;
  uint32_t size = 16;
  while (size < 2 * ents.size()) size <<= 1;
  std::vector<HorusEntry> tab(size, HorusEntry{0, 0, 0, 0});
  uint32_t probes = 1;
  for (const HorusEntry &e : ents) {
    h.nids = std::max(h.nids, (e.meta >> 16) + 1);
    uint32_t slot = horus_hash(e.src, e.dst, e.ports, e.meta & 0xff) & (size - 1), k = 1;
    while (tab[slot].meta & kHorusUsed) { slot = (slot + 1) & (size - 1); ++k; }
    tab[slot] = e;
    probes = std::max(probes, k);
  }
  if (ctx->has_device) {
    const size_t bytes = size_t(size) * sizeof(HorusEntry);
    if (h.cap < bytes) {
      if (h.d_tab) hip_check(hipFree(h.d_tab), "hipFree");
      h.d_tab = nullptr;
      hip_check(hipMalloc(&h.d_tab, bytes), "hipMalloc(horus table)");
      h.cap = bytes;
    }
    hip_check(hipMemcpy(h.d_tab, tab.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy(horus table)");
  }
  h.fields = fields;
  h.entries = static_cast<uint32_t>(ents.size());
  h.mask = size - 1;
  h.probes = probes;
  h.runtime = true;
}

// Chain::updateChain's Horus part, after every update of `chain` (build =
// false: the chain's rules are not known, pcn_ipt_load_chain).
// pcn-iptables (Chain.cpp:505-592): any update drops the program; an INPUT
// update with horus on, INPUT rules and an empty FORWARD rule list builds a
// new one.  pcn-firewall (Chain.cpp:232-306): an INGRESS / EGRESS update
// rebuilds that chain's own program when horus is on and the chain has rules;
// the program keeps the conntrack setting it was compiled with
// (modules/Horus.cpp:135-139; setConntrack does not reload it).
void horus_update(pcn_ipt *ctx, int chain, bool build = true) {
  const bool firewall = ctx->service == PCN_IPT_SERVICE_FIREWALL;
  const int k = firewall ? horus_slot(ctx, chain) : 0;
  if (k < 0) return;
  HorusProg &h = ctx->hz[k];
  uint32_t fields = 0;
  std::vector<HorusEntry> ents;
  const bool want = build && ctx->hz_enabled &&
                    (firewall ? !ctx->chains[chain].rules.empty()
                              : chain == PCN_IPT_INPUT && !ctx->chains[PCN_IPT_INPUT].rules.empty() &&
                                    ctx->chains[PCN_IPT_FORWARD].rules.empty());
  if (want) ents = horus_entries(ctx->chains[chain].rules, fields);
  horus_set(ctx, h, ents, fields);
  h.ct = firewall && ctx->fw_ct_mode != PCN_FW_CT_DISABLED;
}

void update_chain(pcn_ipt *ctx, int chain, bool horus = true) {   // Chain::updateChain
  ChainState &cs = ctx->chains[chain];
  load_tables(ctx, chain, compile_chain(cs.rules, chain, cs.default_action, ctx->ports));
  if (horus) horus_update(ctx, chain);
}

bool valid_chain(int c) { return c >= 0 && c < PCN_IPT_NCHAINS; }

// A chain verb's chain: pcn-firewall has only INGRESS / EGRESS (the FORWARD /
// OUTPUT slots).
bool valid_chain(const pcn_ipt *ctx, int c) {
  return valid_chain(c) && (ctx->service != PCN_IPT_SERVICE_FIREWALL || c != PCN_IPT_INPUT);
}

// ChainRule::update for the context's service.  pcn-firewall: no interface
// fields; the action must be set (Chain.cpp:89-92, 612-620); a conntrack
// match needs conntrack on (ChainRule.cpp:29-33).
Rule rule_from_c(const pcn_ipt *ctx, const pcn_ipt_rule &r) {
  if (ctx->service == PCN_IPT_SERVICE_FIREWALL) {
    if (r.in_iface || r.out_iface) throw std::runtime_error("pcn-firewall rules have no in-iface/out-iface");
    if (r.action < 0) throw std::runtime_error("action not specified for the rule");
    if (r.conntrack && ctx->fw_ct_mode == PCN_FW_CT_DISABLED)
      throw std::runtime_error("Please enable the connection tracking module.");
  }
  return Rule::from_c(r, ctx->ports);
}

template <typename F>
int guarded(pcn_ipt *ctx, F &&f) {
  if (!ctx) return fail(-EINVAL, "null context");
  std::lock_guard<std::mutex> lock(ctx->mu);
  try {
    return f();
  } catch (const HipError &e) {
    return fail(-EIO, e.what());
  } catch (const TableFull &e) {
    return fail(-ENOSPC, e.what());
  } catch (const std::exception &e) {
    return fail(-EINVAL, e.what());
  }
}

}  // namespace

extern "C" {

int pcn_ipt_abi_version(void) { return PCN_IPT_ABI_VERSION; }

const char *pcn_ipt_last_error(void) { return g_last_error.c_str(); }

int pcn_ipt_create(const pcn_ipt_config *cfg, pcn_ipt **out) {
  if (!cfg || !out) return fail(-EINVAL, "null argument");
  *out = nullptr;
  auto ctx = std::make_unique<pcn_ipt>();
  ctx->cfg = *cfg;
  if (!ctx->cfg.max_counted_rules) ctx->cfg.max_counted_rules = 8000;
  if (!ctx->cfg.max_action_rules) ctx->cfg.max_action_rules = 10000;
  if (!ctx->cfg.max_rules) ctx->cfg.max_rules = 8192;
  if (ctx->cfg.max_rules > 32767) return fail(-EINVAL, "max_rules > 32767");
  if (ctx->cfg.jit < -1 || ctx->cfg.jit > 1) return fail(-EINVAL, "jit must be -1, 0 or 1");
  ctx->ctr_words = 2 + 2 * size_t(ctx->cfg.max_counted_rules);
  ctx->ctr_reps = ctr_reps_default();
  ctx->split = split_env();
  ctx->pack.fold = fold_all_copies;
  ctx->pack.ctx = ctx.get();
  ctx->pack.max_pkts = kCtrPackPktsMax;
  ctx->pack.max_bytes = kCtrPackBytesMask;
  if (const char *e = std::getenv("PCN_IPT_DEBUG_PACK_MAX_PKTS")) {   // test hook: fold every few launches
    const unsigned long long v = std::strtoull(e, nullptr, 10);
    if (v >= 4096 && v < kCtrPackPktsMax) {
      ctx->pack.max_pkts = v;
      ctx->pack.max_bytes = v * 64;
    }
  }
  if (cfg->device >= 0) {
    try {
      int ndev = 0;
      hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
      if (cfg->device >= ndev) return fail(-ENODEV, "no such HIP device");
      ctx->has_device = true;
      device_guard(ctx.get());
      hipDeviceProp_t prop;
      hip_check(hipGetDeviceProperties(&prop, cfg->device), "hipGetDeviceProperties");
      ctx->num_cus = prop.multiProcessorCount;
      hip_check(hipMalloc(&ctx->d_localip, PCN_MAX_LOCALIP * 4), "hipMalloc(localip)");
      hip_check(hipMalloc(&ctx->d_zero, 64), "hipMalloc(zero cell)");
      hip_check(hipMemset(ctx->d_zero, 0, 64), "hipMemset(zero cell)");
      hip_check(hipMalloc(&ctx->d_ae, 64), "hipMalloc(ae counters)");
      hip_check(hipMemset(ctx->d_ae, 0, 64), "hipMemset(ae counters)");
      hip_check(hipMalloc(&ctx->d_labels, 64), "hipMalloc(labels)");
      const uint8_t labels[4] = {0, 1, 2, 3};
      hip_check(hipMemcpy(ctx->d_labels, labels, 4, hipMemcpyHostToDevice), "hipMemcpy(labels)");
      hip_check(hipMalloc(&ctx->ctr_scratch, 3 * ctx->ctr_words * 8), "hipMalloc(scratch counters)");
      for (HorusProg &h : ctx->hz) {
        hip_check(hipMalloc(&h.d_ctr, PCN_IPT_HORUS_MAX * 16), "hipMalloc(horus counters)");
        hip_check(hipMemset(h.d_ctr, 0, PCN_IPT_HORUS_MAX * 16), "hipMemset(horus counters)");
      }
      hip_check(hipHostMalloc(reinterpret_cast<void **>(&ctx->h_deal_stats), kDealStatsSlots * 4, hipHostMallocDefault),
                "hipHostMalloc(deal statistics)");
      std::memset(ctx->h_deal_stats, 0, kDealStatsSlots * 4);
      hip_check(hipMalloc(&ctx->d_hz_carry, 64), "hipMalloc(horus carry)");
      hip_check(hipMemset(ctx->d_hz_carry, 0, 64), "hipMemset(horus carry)");
      for (auto &cs : ctx->chains) {
        // the plain block, then ctr_reps packed copies of ctr_words / 2 pairs
        const size_t words = ctx->ctr_words + size_t(ctx->ctr_reps) * (ctx->ctr_words / 2);
        hip_check(hipMalloc(&cs.ctr, words * 8), "hipMalloc(counters)");
        hip_check(hipMemset(cs.ctr, 0, words * 8), "hipMemset(counters)");
        hip_check(hipMalloc(&cs.ctr_global, ctx->ctr_words * 8), "hipMalloc(counters)");
        hip_check(hipMemset(cs.ctr_global, 0, ctx->ctr_words * 8), "hipMemset(counters)");
      }
      for (int c = 0; c < PCN_IPT_NCHAINS; ++c) update_chain(ctx.get(), c);
    } catch (const std::exception &e) {
      return fail(-EIO, e.what());
    }
  } else {
    for (int c = 0; c < PCN_IPT_NCHAINS; ++c) update_chain(ctx.get(), c);
  }
  *out = ctx.release();
  return 0;
}

void pcn_ipt_destroy(pcn_ipt *ctx) {
  if (!ctx) return;
  if (ctx->has_device) {
    (void)hipSetDevice(ctx->cfg.device);
    (void)hipDeviceSynchronize();
    for (auto &cs : ctx->chains) {
      for (auto &s : cs.slot) {
        if (s.tables) (void)hipFree(s.tables);
      }
      if (cs.ctr) (void)hipFree(cs.ctr);
      if (cs.ctr_global) (void)hipFree(cs.ctr_global);
      if (cs.gather) (void)hipFree(cs.gather);
      if (cs.stage) (void)hipFree(cs.stage);
    }
    if (ctx->d_localip) (void)hipFree(ctx->d_localip);
    if (ctx->d_zero) (void)hipFree(ctx->d_zero);
    if (ctx->d_ae) (void)hipFree(ctx->d_ae);
    if (ctx->d_labels) (void)hipFree(ctx->d_labels);
    if (ctx->ctr_scratch) (void)hipFree(ctx->ctr_scratch);
    if (ctx->ct_buf) (void)hipFree(ctx->ct_buf);
    ct_table_free(ctx->ct);
    ct_scratch_free(ctx->cts);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    if (ctx->comm_stream) (void)hipStreamDestroy(ctx->comm_stream);
    if (ctx->ev_staged) (void)hipEventDestroy(ctx->ev_staged);
    if (ctx->ev_gathered) (void)hipEventDestroy(ctx->ev_gathered);
    for (int k = 0; k < pcn_ipt::kGatherEv; ++k) {
      if (ctx->ev_g0[k]) (void)hipEventDestroy(ctx->ev_g0[k]);
      if (ctx->ev_g1[k]) (void)hipEventDestroy(ctx->ev_g1[k]);
    }
    if (ctx->ev_ct) (void)hipEventDestroy(ctx->ev_ct);
    if (ctx->h_deal_stats) (void)hipHostFree(ctx->h_deal_stats);
    if (ctx->d_dbg_clk) (void)hipFree(ctx->d_dbg_clk);
    if (ctx->d_split_rec) (void)hipFree(ctx->d_split_rec);
    for (auto &se : ctx->pack_streams)
      if (se.second) (void)hipEventDestroy(se.second);
    for (void *p : {static_cast<void *>(ctx->hz[0].d_tab), static_cast<void *>(ctx->hz[0].d_ctr),
                    static_cast<void *>(ctx->hz[1].d_tab), static_cast<void *>(ctx->hz[1].d_ctr),
                    static_cast<void *>(ctx->d_hz_carry), static_cast<void *>(ctx->d_stale_desc),
                    static_cast<void *>(ctx->d_chunk_ctr)})
      if (p) (void)hipFree(p);
  }
  delete ctx;
}

int pcn_ipt_add_port(pcn_ipt *ctx, const char *name, uint16_t index) {
  return guarded(ctx, [&] {
    if (!name || !*name) return fail(-EINVAL, "empty port name");
    ctx->ports.add(name, index);
    return 0;
  });
}

int pcn_ipt_set_localip(pcn_ipt *ctx, const uint32_t *ips, size_t n) {
  return guarded(ctx, [&] {
    if (n > PCN_MAX_LOCALIP) return fail(-ENOSPC, "localip holds at most 256 addresses");
    std::vector<uint32_t> v(ips, ips + n);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    if (ctx->has_device) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      if (!v.empty())
        hip_check(hipMemcpy(ctx->d_localip, v.data(), v.size() * 4, hipMemcpyHostToDevice), "hipMemcpy(localip)");
    }
    ctx->localip = std::move(v);
    return 0;
  });
}

int pcn_ipt_chain_append(pcn_ipt *ctx, int chain, const pcn_ipt_rule *rule) {
  return guarded(ctx, [&] {
    if (!valid_chain(ctx, chain) || !rule) return fail(-EINVAL, "bad chain or rule");
    ChainState &cs = ctx->chains[chain];
    Rule r = rule_from_c(ctx, *rule);
    if (cs.rules.size() >= ctx->cfg.max_rules) return fail(-ENOSPC, "too many rules");
    fetch_stats(ctx, chain);                          // Chain::addRule -> getStatsList
    cs.rules.push_back(std::move(r));
    cs.stats.resize(cs.rules.size());
    if (ctx->interactive) {
      update_chain(ctx, chain);
      apply_ae(ctx, chain);                           // Chain.cpp:186-188
    }
    return 0;
  });
}

int pcn_ipt_chain_insert(pcn_ipt *ctx, int chain, uint32_t id, const pcn_ipt_rule *rule) {
  return guarded(ctx, [&] {
    if (!valid_chain(ctx, chain) || !rule) return fail(-EINVAL, "bad chain or rule");
    ChainState &cs = ctx->chains[chain];
    if (id > cs.rules.size()) return fail(-EINVAL, "id not allowed");   // Chain.cpp:238-240
    Rule r = rule_from_c(ctx, *rule);
    if (cs.rules.size() >= ctx->cfg.max_rules) return fail(-ENOSPC, "too many rules");
    fetch_stats(ctx, chain);
    cs.rules.insert(cs.rules.begin() + id, std::move(r));
    cs.stats.insert(cs.stats.begin() + id, {0, 0});
    if (ctx->interactive) {
      update_chain(ctx, chain);
      apply_ae(ctx, chain);                           // Chain.cpp:306-308
    }
    return 0;
  });
}

int pcn_ipt_chain_delete_id(pcn_ipt *ctx, int chain, uint32_t id) {
  return guarded(ctx, [&] {
    if (!valid_chain(ctx, chain)) return fail(-EINVAL, "bad chain");
    ChainState &cs = ctx->chains[chain];
    if (id >= cs.rules.size()) return fail(-ENOENT, "There is no rule " + std::to_string(id));
    fetch_stats(ctx, chain);
    cs.rules.erase(cs.rules.begin() + id);
    cs.stats.erase(cs.stats.begin() + id);
    if (ctx->interactive) update_chain(ctx, chain);
    return 0;
  });
}

int pcn_ipt_chain_delete_match(pcn_ipt *ctx, int chain, const pcn_ipt_rule *rule) {
  return guarded(ctx, [&] {
    if (!valid_chain(ctx, chain) || !rule) return fail(-EINVAL, "bad chain or rule");
    ChainState &cs = ctx->chains[chain];
    Rule r;
    try {
      r = Rule::from_c(*rule, ctx->ports);
    } catch (const std::exception &) {
      return fail(-EINVAL, "No matching rule to delete");    // Chain.cpp:344-346
    }
    for (size_t i = 0; i < cs.rules.size(); ++i) {
      if (cs.rules[i] == r) {
        fetch_stats(ctx, chain);
        cs.rules.erase(cs.rules.begin() + i);
        cs.stats.erase(cs.stats.begin() + i);
        if (ctx->interactive) update_chain(ctx, chain);
        return 0;                                     // delRule(i); return; (Chain.cpp:358-361)
      }
    }
    if (ctx->service == PCN_IPT_SERVICE_FIREWALL)
      return fail(-ENOENT, "no matching rule to delete");   // pcn-firewall Chain.cpp:760-771
    apply_ae(ctx, chain);                             // only reached without a match (Chain.cpp:368)
    return 0;   // no match: the reference returns without error
  });
}

int pcn_ipt_chain_flush(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(ctx, chain)) return fail(-EINVAL, "bad chain");
    ChainState &cs = ctx->chains[chain];
    cs.rules.clear();
    cs.stats.clear();
    if (ctx->interactive) update_chain(ctx, chain);
    return 0;
  });
}

int pcn_ipt_chain_set_default(pcn_ipt *ctx, int chain, int action) {
  return guarded(ctx, [&] {
    if (!valid_chain(ctx, chain) || (action != PCN_IPT_DROP && action != PCN_IPT_ACCEPT))
      return fail(-EINVAL, "bad chain or action");
    ChainState &cs = ctx->chains[chain];
    if (cs.default_action == action) return 0;
    cs.default_action = action;
    // Chain::setDefault -> reloadChain: the programs are rebuilt from the
    // current rule list with the new default action.  pcn-firewall reloads only
    // its DefaultAction program (pcn-firewall Chain.cpp:60-82): no chain
    // update, so its Horus program stays in place.
    fetch_stats(ctx, chain);
    try {
      update_chain(ctx, chain, ctx->service != PCN_IPT_SERVICE_FIREWALL);
    } catch (const TableFull &e) {
      // the reference catches the reload's runtime_error, logs "Can't reload
      // the code for default action" and returns normally (Chain.cpp:123-129);
      // the chain keeps its last image, the next update reports the overflow
      g_last_error = std::string("Can't reload the code for default action. Error: ") + e.what();
    }
    return 0;
  });
}

int pcn_ipt_set_interactive(pcn_ipt *ctx, int interactive) {
  return guarded(ctx, [&] {
    ctx->interactive = interactive != 0;
    return 0;
  });
}

int pcn_ipt_chain_apply_rules(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    fetch_stats(ctx, chain);
    update_chain(ctx, chain);
    apply_ae(ctx, chain);                             // Chain.cpp:408
    return 0;
  });
}

int pcn_ipt_chain_nrules(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    return static_cast<int>(ctx->chains[chain].rules.size());
  });
}

int pcn_ipt_load_chain(pcn_ipt *ctx, int chain, const pcn_ipt_tables *t) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain) || !t) return fail(-EINVAL, "bad chain or tables");
    if (t->default_action != PCN_IPT_DROP && t->default_action != PCN_IPT_ACCEPT)
      return fail(-EINVAL, "bad default action");
    ChainTables ct;
    ct.nrules = t->nrules;
    ct.nrw = words_for_rules(t->nrules);
    ct.default_action = t->default_action;
    if (t->nrules && !t->actions) return fail(-EINVAL, "actions required");
    ct.actions.assign(t->actions, t->actions + t->nrules);
    for (int f = 0; f < PCN_IPT_NFIELDS; ++f) {
      const pcn_ipt_field_map &m = t->maps[f];
      if (!m.n) continue;
      if (!m.keys || !m.vecs) return fail(-EINVAL, "field map without keys/vecs");
      bool ip = f == PCN_IPT_F_IPSRC || f == PCN_IPT_F_IPDST;
      if (ip && !m.plen) return fail(-EINVAL, "IP map without prefix lengths");
      FieldMap &fm = ct.maps[f];
      for (uint32_t k = 0; k < m.n; ++k) {
        fm.keys.push_back(m.keys[k]);
        if (ip) {
          if (m.plen[k] > 32) return fail(-EINVAL, "prefix length > 32");
          fm.plen.push_back(m.plen[k]);
        }
        fm.vecs.emplace_back(m.vecs + size_t(k) * ct.nrw, m.vecs + size_t(k + 1) * ct.nrw);
      }
    }
    load_tables(ctx, chain, std::move(ct));
    horus_update(ctx, chain, false);   // an update without rules: no Horus program (Chain.cpp:505)
    return 0;
  });
}

int pcn_ipt_export_map(pcn_ipt *ctx, int chain, int field, uint32_t *keys, uint8_t *plen, uint64_t *vecs,
                       uint32_t cap, uint32_t nrw) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain) || field < 0 || field >= PCN_IPT_NFIELDS) return fail(-EINVAL, "bad chain/field");
    const ChainTables &t = ctx->chains[chain].tables;
    const FieldMap &m = t.maps[field];
    if (m.keys.size() > cap) return fail(-ENOSPC, "export buffer too small");
    for (size_t k = 0; k < m.keys.size(); ++k) {
      if (keys) keys[k] = m.keys[k];
      if (plen) plen[k] = m.plen.empty() ? 0 : m.plen[k];
      if (vecs)
        for (uint32_t w = 0; w < nrw; ++w) vecs[k * nrw + w] = w < t.nrw ? m.vecs[k][w] : 0;
    }
    return static_cast<int>(m.keys.size());
  });
}

uint32_t pcn_ipt_chain_nrw(pcn_ipt *ctx, int chain) {
  if (!ctx || !valid_chain(chain)) return 0;
  std::lock_guard<std::mutex> lock(ctx->mu);
  return ctx->chains[chain].tables.nrw;
}

}  // extern "C"

namespace {

// Overrides of one stage-A launch of a stateful batch (conntrack.hpp): a
// constant label for every packet, outcomes into scratch, counters discarded.
struct StageA {
  const uint8_t *ct;
  uint8_t *verdicts;
  int32_t *rule_ids;
  // non-null: this stage A also writes the walk records (conntrack.hpp
  // ct_prep_buffers), so ct_run skips ct_prep
  uint32_t *brec = nullptr, *keys = nullptr, *lcs = nullptr;
  uint32_t sentinel = 0;
  unsigned long long *pdesc = nullptr, *fixm = nullptr;   // the stale ports, completed by ct_stale_fix
};

// carry_out (stateless batches that track the stale ports): when the kernel
// computes them itself (has_stale), its last workgroup writes the carry there
// and *carried becomes true; otherwise the caller advances the carry.
// plan (pcn_ipt_chain_program_compile): compute the launch as usual, then set
// *plan to the chain program's spec ("" when no chain program would run) and
// return before anything is allocated, requested or launched.
int launch_batch(pcn_ipt *ctx, const pcn_ipt_batch *b, void *stream, const StageA *sa, const uint32_t *carry,
                 uint32_t *carry_out = nullptr, bool *carried = nullptr, std::string *plan = nullptr) {
  {
    if (!b) return fail(-EINVAL, "null batch");
    if (!ctx->has_device && !plan) return fail(-ENODEV, "context has no HIP device (created with device=-1)");
    if (b->n == 0) return 0;
    if (!b->frames || !b->verdicts) return fail(-EINVAL, "frames and verdicts are required");
    if (b->direction != PCN_IPT_INGRESS && b->direction != PCN_IPT_EGRESS) return fail(-EINVAL, "bad direction");
    if (b->hook != PCN_IPT_HOOK_XDP && b->hook != PCN_IPT_HOOK_TC) return fail(-EINVAL, "bad hook");
    device_guard(ctx);
    LaunchArgs a{};
    for (int c = 0; c < PCN_IPT_NCHAINS; ++c) {
      a.ch[c] = ctx->chains[c].desc;
      if (!a.ch[c].nrules) a.empty_mask |= 1u << c;
      if (a.ch[c].default_action == PCN_IPT_DROP) a.drop_mask |= 1u << c;
    }
    const ChainState &in = ctx->chains[PCN_IPT_INPUT], &fw = ctx->chains[PCN_IPT_FORWARD];
    const bool firewall = ctx->service == PCN_IPT_SERVICE_FIREWALL;
    a.allow_logic = !firewall && in.default_action == PCN_IPT_ACCEPT && fw.default_action == PCN_IPT_ACCEPT &&
                    in.rules.size() == 0 && fw.rules.size() == 0 && in.desc.nrules == 0 &&
                    fw.desc.nrules == 0;
    if (firewall)
      a.fw = ctx->fw_ct_mode == PCN_FW_CT_DISABLED ? PCN_FW_LAUNCH_CT_OFF
             : ctx->fw_ct_mode == PCN_FW_CT_MANUAL ? PCN_FW_LAUNCH_CT_MANUAL : PCN_FW_LAUNCH_CT_AUTO;
    // which chains can reach the rule stage (ChainSelector_dp.c:157-168, 243-260;
    // pcn-firewall: the direction's chain, Firewall_ChainForwarder_dp.c:20-42)
    const bool has_local = firewall || !ctx->localip.empty();
    const bool reach_fw = b->direction == PCN_IPT_INGRESS && !a.allow_logic && a.ch[PCN_IPT_FORWARD].nrules;
    const bool reach_in = !firewall && b->direction == PCN_IPT_INGRESS && !a.allow_logic && has_local &&
                          a.ch[PCN_IPT_INPUT].nrules;
    const bool reach_out = b->direction == PCN_IPT_EGRESS && has_local && a.ch[PCN_IPT_OUTPUT].nrules;
    int ch = PCN_IPT_FORWARD;
    if (reach_fw && reach_in) ch = 3;
    else if (reach_in) ch = PCN_IPT_INPUT;
    else if (reach_out) ch = PCN_IPT_OUTPUT;
    // LDS: the table images of the chains that run rules in this launch (the
    // one chain first, at offset 0), then the counter histogram: 3 default
    // bins + rule bins (that chain first, then FORWARD, INPUT, OUTPUT), then
    // localip and the per-wave regions.
    int order[3] = {PCN_IPT_FORWARD, PCN_IPT_INPUT, PCN_IPT_OUTPUT};
    if (ch < 3) {
      int k = 1;
      order[0] = ch;
      for (int c : {PCN_IPT_FORWARD, PCN_IPT_INPUT, PCN_IPT_OUTPUT})
        if (c != ch) order[k++] = c;
    }
    const bool any_rules = reach_fw || reach_in || reach_out;
    auto runs = [&](int c) {
      return any_rules && (ch < 3 ? c == ch : (c == PCN_IPT_FORWARD || c == PCN_IPT_INPUT));
    };
    // fixed-stride fast path: 48-byte header windows inside the buffer, each read as
    // three 16-byte loads from the frame's start, which need dword alignment only
    // (a 1500-byte stride: 172 B of lines a frame, against the generic gather's 16-byte
    // aligned 64-byte span; PCN_IPT_DEBUG_FIXED_ALIGN=16 restores the 16-byte rule, A/B)
    // (TC frames may carry a VLAN tag: the 52-byte window of the generic path)
    const uint32_t falign = fixed_align();
    bool fixed = b->hook == PCN_IPT_HOOK_XDP && !b->offsets && !b->lens && b->stride % falign == 0 && b->stride >= 48 &&
                 (reinterpret_cast<uintptr_t>(b->frames) % falign) == 0 &&
                 (b->n - 1) * uint64_t(b->stride) + 48 <= b->frames_bytes;
    // LDS plan (every field below): a chain program of a chain with 2+ summary
    // blocks deals 128 candidates a pass (jit.cpp) and needs the larger wave
    // region; the plan is made for it, and made again without it when the
    // launch falls back to the generic kernel (program still compiling, or
    // failed), so the generic kernel keeps that LDS for images and bins.
    auto plan_lds = [&](bool deal2) {
      uint32_t base = 3;
      for (int c : order) {
        uint32_t nc = a.ch[c].ncounted;
        if (nc && base - 3 + nc <= kMaxLdsRuleBins) {
          a.ch[c].lds_bins = static_cast<int32_t>(base);
          a.ch[c].lds_nrules = nc;
          base += nc;
        } else {
          a.ch[c].lds_bins = -1;
          a.ch[c].lds_nrules = 0;
        }
      }
      // Horus hits count into the same workgroup histogram (a hot key would
      // otherwise serialize on one global address)
      const HorusProg *hzb = horus_of_batch(ctx, b->direction);
      a.hz_bins = -1;
      if (hzb && !sa && base - 3 + hzb->nids <= kMaxLdsRuleBins) {
        a.hz_bins = static_cast<int32_t>(base);
        base += hzb->nids;
      }
      a.nbins = base;
      a.nlocal = static_cast<uint32_t>(ctx->localip.size());
      // counter bins: u32 pkts, plus u32 bytes unless every frame has the same length
      const uint32_t bin_bytes = (fixed ? 4 : 8) * a.nbins;
      const uint32_t tail = (bin_bytes + 15) / 16 * 16 + (a.nlocal * 4 + 15) / 16 * 16 +
                            (PCN_BLOCK / 64) * wave_region_bytes(fixed, deal2);
      // whole images if they fit, else their per-packet prefix [0, pbase) (the
      // candidate-stage tables are then read from L2/HBM), else nothing
      uint32_t img_bytes = 0;
      for (int mode = 0; mode < 3; ++mode) {
        img_bytes = 0;
        for (int c : order) {
          a.ch[c].lds_image = 0;
          a.ch[c].lds_limit = 0;
          if (!runs(c) || mode == 2) continue;
          a.ch[c].lds_image = kLdsDescBytes + img_bytes;
          a.ch[c].lds_limit = mode == 0 ? a.ch[c].lay.bytes : a.ch[c].lay.pbase;
          img_bytes += a.ch[c].lds_limit;
        }
        if (mode == 2 || kLdsDescBytes + img_bytes + tail <= kLdsBudget) break;
      }
      // A chain that runs rules here but got no bin per rule (more rules than
      // the histogram budget): bins for its lowest rule ids in the LDS the
      // images leave over, the rest counted with global atomics.  Placed after
      // the choice above, so no image loses its place in LDS to them.
      for (int c : order) {
        if (!runs(c) || a.ch[c].lds_bins >= 0 || !a.ch[c].ncounted) continue;
        const uint32_t nb = partial_rule_bins(kLdsDescBytes + img_bytes + tail, fixed ? 4 : 8, a.ch[c].ncounted);
        if (nb) {                    // before the Horus bins, which the flush takes to run to the end
          a.ch[c].lds_bins = a.hz_bins >= 0 ? a.hz_bins : static_cast<int32_t>(base);
          a.ch[c].lds_nrules = nb;
          if (a.hz_bins >= 0) a.hz_bins += static_cast<int32_t>(nb);
          base += nb;
          a.nbins = base;
        }
        break;
      }
      const uint32_t all_bin_bytes = (fixed ? 4 : 8) * a.nbins;
      a.lds_images_bytes = img_bytes;
      a.bins_offset = kLdsDescBytes + img_bytes;
      a.lds_localip = a.bins_offset + (all_bin_bytes + 15) / 16 * 16;
      a.lds_stats = (a.lds_localip + a.nlocal * 4 + 15) / 16 * 16;   // the deal statistics' counter
      a.lds_scratch = a.lds_stats + 16;
      a.wave_bytes = wave_region_bytes(fixed, deal2);
      a.lds_bytes = a.lds_scratch + (PCN_BLOCK / 64) * a.wave_bytes;
    };
    bool deal2 = ch < 3 && any_rules && a.ch[ch].nsw >= 2 && ctx->cfg.jit >= 0 && multi_block_deal2();
    plan_lds(deal2);
    a.frames = b->frames;
    a.frames_bytes = b->frames_bytes;
    a.offsets = b->offsets;
    a.lens = b->lens;
    a.has_in_port = b->in_port != nullptr;
    a.has_ct = sa || b->ct_status != nullptr;
    a.in_port = a.has_in_port ? b->in_port : reinterpret_cast<const uint16_t *>(ctx->d_zero);
    a.ct_status = sa ? sa->ct : a.has_ct ? b->ct_status : ctx->d_zero;
    a.in_port_mask = a.has_in_port ? ~uint64_t(0) : 0;
    a.ct_mask = a.has_ct && !sa ? ~uint64_t(0) : 0;
    a.verdicts = sa ? sa->verdicts : b->verdicts;
    a.rule_ids = sa ? sa->rule_ids : b->rule_ids;
    if (sa)
      for (int c = 0; c < PCN_IPT_NCHAINS; ++c) a.ch[c].ctr = ctx->ctr_scratch + c * ctx->ctr_words;
    // packed copies after each chain's plain block (stage A's scratch counters: plain adds)
    a.ctr_rep_mask = sa ? 0u : ctx->ctr_reps - 1;
    a.ctr_rep_words = static_cast<uint32_t>(ctx->ctr_words / 2);
    a.ctr_pack_off = sa ? 0u : static_cast<uint32_t>(ctx->ctr_words);
    a.localip = ctx->d_localip;
    a.n = b->n;
    a.stride = b->stride;
    a.fixed_len = b->fixed_len;
    a.const_in_port = b->const_in_port;
    a.direction = b->direction;
    a.hook = b->hook;
    if (!b->offsets) {
      uint64_t last = (b->n - 1) * uint64_t(b->stride);
      if (last >= b->frames_bytes) return fail(-EINVAL, "frames_bytes smaller than n*stride");
    }
    // chains a packet of this launch can select (ChainSelector_dp.c:157-168, 243-260)
    // wave fast path (classify.hip): the chain every IPv4 TCP/UDP frame of the
    // launch selects, when that needs no per-packet choice
    a.fast_chain = -1;
    if (firewall) {
      const int c = b->direction == PCN_IPT_INGRESS ? PCN_IPT_FORWARD : PCN_IPT_OUTPUT;
      if (a.ch[c].nrules) a.fast_chain = c;
    } else if (b->direction == PCN_IPT_INGRESS && !a.allow_logic && ctx->localip.empty() &&
               a.ch[PCN_IPT_FORWARD].nrules) {
      a.fast_chain = PCN_IPT_FORWARD;
    }
    a.count_mask = b->direction == PCN_IPT_INGRESS
                       ? (1u << PCN_IPT_FORWARD) | (has_local && !firewall ? 1u << PCN_IPT_INPUT : 0u)
                       : (has_local ? 1u << PCN_IPT_OUTPUT : 0u);
    // stage A counts nothing: ct_count counts every packet from its final
    // outcome, and stage A's counters went to discarded scratch (their LDS adds,
    // ballots and the flush into one block were pure cost)
    if (sa && !debug_stage_a_counts()) a.count_mask = 0;
    // The Parser's stale ports (Q4) computed in the kernel (has_stale): one
    // word per 64-frame group of the batch, a start counter, the carry in and
    // (on the batch's last launch) out.
    auto track_stale = [&]() {
      if (plan) {
        a.has_stale = 1;
        return;
      }
      // the key reads ports: stale ones (Q4) computed in the kernel
      // one word per 64-frame group of the batch (+1 for the look-back from
      // the end); the kernel publishes only groups that hold frames
      const size_t groups = b->n / 64 + 1;
      if (ctx->stale_groups < groups) {
        if (ctx->d_stale_desc) hip_check(hipFree(ctx->d_stale_desc), "hipFree");
        ctx->d_stale_desc = nullptr;
        // + kStaleCanary guard words past the groups (pcn_ipt_debug_stale_canary)
        hip_check(hipMalloc(&ctx->d_stale_desc, (groups + kStaleCanary) * 8), "hipMalloc(stale groups)");
        hip_check(hipMemset(ctx->d_stale_desc, 0, groups * 8), "hipMemset(stale groups)");
        hip_check(hipMemset(ctx->d_stale_desc + groups, kStaleCanaryByte, kStaleCanary * 8), "hipMemset(canary)");
        ctx->stale_groups = groups;
        ctx->stale_epoch = 0;
      }
      if (debug_stale_canary() && groups < ctx->stale_groups)
        // test hook: guard every word past this batch's groups, not only those
        // past the largest batch so far
        hip_check(hipMemsetAsync(ctx->d_stale_desc + groups, kStaleCanaryByte, (ctx->stale_groups - groups) * 8,
                                 static_cast<hipStream_t>(stream)), "hipMemset(canary)");
      ctx->stale_guard_from = debug_stale_canary() ? groups : ctx->stale_groups;
      if (!ctx->d_chunk_ctr) {   // zero from here on: each launch's last workgroup resets it
        hip_check(hipMalloc(&ctx->d_chunk_ctr, 64), "hipMalloc(chunk counter)");
        hip_check(hipMemset(ctx->d_chunk_ctr, 0, 64), "hipMemset(chunk counter)");
      }
      if (++ctx->stale_epoch >= (1u << 24)) {       // words of an old epoch must never match
        hip_check(hipMemsetAsync(ctx->d_stale_desc, 0, ctx->stale_groups * 8, static_cast<hipStream_t>(stream)),
                  "hipMemset(stale groups)");
        ctx->stale_epoch = 1;
      }
      a.has_stale = 1;
      a.stale_desc = ctx->d_stale_desc;
      a.stale_carry = carry;
      a.chunk_ctr = ctx->d_chunk_ctr;
      a.stale_epoch = ctx->stale_epoch;
      a.carry_out = carry_out;
      if (carried) *carried = carry_out != nullptr;
    };
    // Horus: the program the batch's Parser calls, while one is in place
    if (const HorusProg *hz = horus_of_batch(ctx, b->direction)) {
      a.horus = hz->d_tab;
      a.horus_mask = hz->mask;
      a.horus_probes = hz->probes;
      a.horus_fields = hz->fields;
      a.horus_ctr = sa ? nullptr : hz->d_ctr;         // stage A: ct_count counts the final outcome
      if (firewall) {
        a.horus_flags = kHzNatural;
        if (!hz->ct) a.horus_flags |= kHzAcceptFinal;                        // Firewall_Horus_dp.c:162-164
        else if (ctx->fw_ct_mode == PCN_FW_CT_DISABLED) a.horus_flags |= kHzAcceptDrops;
        if (ctx->fw_ct_mode == PCN_FW_CT_DISABLED) a.horus_flags |= kHzMissDrops;   // :170-174
      }
      a.fast_chain = -1;                               // the lookup lives in the general path
      if (carry && (hz->fields & (PCN_IPT_HZ_SRCPORT | PCN_IPT_HZ_DSTPORT))) track_stale();
    }
    // stage A of a stateful batch that writes the walk records (ct_fused_prep):
    // its records need every frame's stale ports too -- published per group and
    // completed after the launch (conntrack.hip ct_stale_fix), so no workgroup
    // waits on another's groups
    if (sa && sa->brec) {
      a.ct_brec = sa->brec;
      a.ct_keys = sa->keys;
      a.ct_lcs = sa->lcs;
      a.ct_sentinel = sa->sentinel;
      a.ct_pdesc = sa->pdesc;
      a.ct_fixm = sa->fixm;
    }
    // slot count of the chain program (the generic kernel always runs 6)
    const int ns = ch < 3 ? static_cast<int>(a.ch[ch].lay.nslots) : 6;
    // chain program for this launch shape (jit.hpp), when enabled and ready
    void *fn = nullptr, *fn2 = nullptr;
    if (plan) plan->clear();
    if (ch < 3 && (reach_fw || reach_in || reach_out) && (ctx->cfg.jit >= 0 || plan)) {
      ChainState &cs = ctx->chains[ch];
      JitShape shape;
      shape.fixed = fixed;
      shape.lds = a.lds_images_bytes > 0;
      shape.ch = ch;
      shape.ns = ns;
      shape.inputs = (a.has_in_port ? 1 : 0) | (a.has_ct && !sa ? 2 : 0) | (sa ? 4 : 0) | (a.has_stale ? 8 : 0) |
                     (a.horus_fields ? 16 : 0) | (a.offsets ? 32 : 0) | (a.lens ? 64 : 0) | (a.ct_brec ? 128 : 0);
      shape.deal2 = deal2;
      shape.split = !fixed && !sa && !a.has_stale && !a.horus_fields && a.ch[ch].lay.part_dense && ctx->split &&
                    !debug_clocks();
      {
        const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((b->n + PCN_BLOCK - 1) / PCN_BLOCK,
                                                                       uint64_t(classify_grid_cus(ctx->num_cus))));
        shape.shallow = fixed && !plan && (b->n + grid * PCN_BLOCK - 1) / (grid * PCN_BLOCK) <= 8 &&
                        shallow_prefetch();
      }
      DevChain key = a.ch[ch];
      key.image = nullptr;
      key.ctr = nullptr;
      if (cs.jit_spec.empty() || std::memcmp(&key, &cs.jit_desc, sizeof(DevChain)) != 0 ||
          shape.fixed != cs.jit_shape.fixed ||
          shape.lds != cs.jit_shape.lds || shape.ch != cs.jit_shape.ch || shape.ns != cs.jit_shape.ns ||
          shape.inputs != cs.jit_shape.inputs || shape.shallow != cs.jit_shape.shallow ||
          shape.deal2 != cs.jit_shape.deal2 || shape.split != cs.jit_shape.split) {
        cs.jit_desc = key;
        cs.jit_shape = shape;
        cs.jit_spec = jit_spec(key, shape);
      }
      if (plan) {
        *plan = cs.jit_spec;
        return 0;
      }
      ctx->jit.request(cs.jit_spec, ctx->cfg.jit == 1);
      fn = ctx->jit.function(cs.jit_spec, ctx->cfg.device);
      if (fn && shape.split) {
        // a split program's first kernel is its gather kernel: it never runs alone
        fn2 = ctx->jit.function(cs.jit_spec, ctx->cfg.device, 1);
        if (!fn2) fn = nullptr;
      }
      cs.last_spec = fn ? cs.jit_spec : std::string();
      // the generic kernel deals 64 a pass: give the 128-item region back
      if (!fn && deal2) {
        deal2 = false;
        plan_lds(false);
      }
      cs.last_lds_bytes = a.lds_bytes;
      // Adaptive deal window (fixed-stride chains of one summary block, whose
      // chain program deals 64 candidates a pass): with the previous launch's
      // waves mostly holding more than 64 candidates (hit rate near 1: two
      // passes each) the program with the 128-candidate window (classify.hip
      // PCN_DEAL2 = 1, the same 3 KB wave region) runs instead; where no wave
      // needs a second pass the 64 one stays (its smaller program is ~1.5 %
      // faster).  The counts come from the kernel itself through
      // host-mapped memory, read without a sync: whatever has landed.
      const int adapt = deal_adapt();
      // (stage A too: the stateful traffic is often mostly rule hits)
      if (fn && fixed && a.ch[ch].nsw == 1 && adapt && ctx->h_deal_stats) {
        const std::string spec128 = cs.jit_spec + "#ifndef PCN_DEAL2\n#define PCN_DEAL2 1\n#endif\n";
        ctx->jit.request(spec128, false);
        bool wide = adapt == 2 || cs.deal_wide;
        if (adapt == 1 && ctx->deal_frames) {
          uint64_t sum = 0;
          for (uint32_t k = 0; k < ctx->deal_grid; ++k) sum += reinterpret_cast<volatile uint32_t *>(ctx->h_deal_stats)[k];
          const uint64_t waves = (ctx->deal_frames + 63) / 64;
          if (!wide && sum * 8 > waves) wide = true;          // more than 1/8 of the waves: switch to 128
          else if (wide && sum * 32 < waves) wide = false;    // fewer than 1/32: back to 64
        }
        cs.deal_wide = wide;
        if (void *f128 = wide ? ctx->jit.function(spec128, ctx->cfg.device) : nullptr) {
          fn = f128;
          cs.last_spec = spec128;
        }
        const uint64_t grid = std::min<uint64_t>((b->n + PCN_BLOCK - 1) / PCN_BLOCK,
                                                 uint64_t(classify_grid_cus(ctx->num_cus)));
        if (grid <= kDealStatsSlots) {
          a.deal_stats = ctx->h_deal_stats;
          ctx->deal_grid = static_cast<uint32_t>(grid);
          ctx->deal_frames = b->n;
        }
      }
    }
    if (!a.deal_stats && !plan) ctx->deal_frames = 0;   // this launch counts nothing: forget the old counts
    if (plan) return 0;
    ++(fn ? ctx->launches_jit : ctx->launches_generic);
    const hipStream_t hs = static_cast<hipStream_t>(stream);
    for (bool &d : ctx->ctr_dirty) d = true;        // (fetch_stats reads them again)
    if (debug_clocks() && !sa) {
      if (!ctx->d_dbg_clk) hip_check(hipMalloc(&ctx->d_dbg_clk, kDbgClkGrid * 32), "hipMalloc(debug clocks)");
      a.dbg_clk = ctx->d_dbg_clk;
      ctx->dbg_grid = static_cast<uint32_t>(std::min<uint64_t>((b->n + PCN_BLOCK - 1) / PCN_BLOCK,
                                                               uint64_t(classify_grid_cus(ctx->num_cus))));
      if (ctx->dbg_grid > kDbgClkGrid) a.dbg_clk = nullptr;
    }
    LaunchArgs ga{};
    if (fn2) {
      // the gather kernel's records, and its own LDS layout: the default bins
      // (it counts the frames it finishes), localip and the per-wave regions
      // of the quad gather; no chain image, no rule bins
      if (ctx->split_cap < b->n) {
        if (ctx->d_split_rec) hip_check(hipFree(ctx->d_split_rec), "hipFree(split records)");
        ctx->d_split_rec = nullptr;
        ctx->split_cap = 0;
        hip_check(hipMalloc(&ctx->d_split_rec, b->n * 16), "hipMalloc(split records)");
        ctx->split_cap = b->n;
      }
      a.split_rec = ctx->d_split_rec;
      ga = a;
      ga.nbins = 3;
      ga.hz_bins = -1;
      for (int c = 0; c < 3; ++c) {
        ga.ch[c].lds_bins = -1;
        ga.ch[c].lds_nrules = 0;
        ga.ch[c].lds_image = 0;
        ga.ch[c].lds_limit = 0;
      }
      ga.lds_images_bytes = 0;
      ga.bins_offset = kLdsDescBytes;
      ga.lds_localip = ga.bins_offset + (8 * ga.nbins + 15) / 16 * 16;
      ga.lds_stats = (ga.lds_localip + ga.nlocal * 4 + 15) / 16 * 16;
      ga.lds_scratch = ga.lds_stats + 16;
      ga.wave_bytes = wave_region_bytes(false, false);
      ga.lds_bytes = ga.lds_scratch + (PCN_SPLIT_G_BLOCK / 64) * ga.wave_bytes;
      ga.deal_stats = nullptr;
      ga.dbg_clk = nullptr;
      ++ctx->launches_split;
    }
    if (!sa) register_pack_stream(ctx, hs);
    int rc = launch_classify(a, fixed, ch, ns, classify_grid_cus(ctx->num_cus), fn, hs, sa ? nullptr : &ctx->pack,
                             fn2, fn2 ? &ga : nullptr, split_gather_wg());
    if (!rc && !sa) note_pack_stream(ctx, hs);
    if (rc != hipSuccess) return fail(-EIO, std::string("classify launch: ") + hipGetErrorString(hipError_t(rc)));
    return 0;
  }
}

// The conntrack kernels' view of a batch (conntrack.hpp).
CtBatch ct_batch(pcn_ipt *ctx, const pcn_ipt_batch *b, uint32_t ae_mask) {
  CtBatch cb{};
  cb.frames = b->frames;
  cb.frames_bytes = b->frames_bytes;
  cb.offsets = b->offsets;
  cb.lens = b->lens;
  cb.stride = b->stride;
  cb.fixed_len = b->fixed_len;
  cb.direction = b->direction;
  cb.hook = b->hook;
  cb.n = b->n;
  cb.localip = ctx->d_localip;
  cb.nlocal = static_cast<uint32_t>(ctx->localip.size());
  const ChainState &in = ctx->chains[PCN_IPT_INPUT], &fw = ctx->chains[PCN_IPT_FORWARD];
  cb.fw = ctx->service == PCN_IPT_SERVICE_FIREWALL;
  cb.allow_logic = !cb.fw && in.default_action == PCN_IPT_ACCEPT && fw.default_action == PCN_IPT_ACCEPT &&
                   in.rules.size() == 0 && fw.rules.size() == 0 && in.desc.nrules == 0 && fw.desc.nrules == 0;
  for (int c = 0; c < PCN_IPT_NCHAINS; ++c) {
    const ChainState &cs = ctx->chains[c];
    if (!cs.desc.nrules) cb.empty_mask |= 1u << c;
    if (cs.desc.default_action == PCN_IPT_DROP) cb.drop_mask |= 1u << c;
    cb.ctr[c] = cs.ctr;
    cb.ncounted[c] = cs.desc.ncounted;
  }
  cb.ae_mask = ae_mask;
  cb.ae_ctr = ctx->d_ae;
  const HorusProg *hz = horus_of_batch(ctx, b->direction);
  cb.horus_ctr = hz ? hz->d_ctr : nullptr;
  cb.horus_final = hz && cb.fw && !hz->ct;          // pcn-firewall built with conntrack off: ACCEPT is RX_OK
  cb.verdicts = b->verdicts;
  cb.rule_ids = b->rule_ids;
  return cb;
}

}  // namespace

extern "C" {

int pcn_ipt_classify(pcn_ipt *ctx, const pcn_ipt_batch *b, void *stream) {
  return guarded(ctx, [&]() -> int {
    if (!b) return fail(-EINVAL, "null batch");
    if (!ctx->has_device) return fail(-ENODEV, "context has no HIP device (created with device=-1)");
    if (b->n == 0) return 0;
    // chains this batch can reach, and which of them run accept-established
    const uint32_t reach = b->direction == PCN_IPT_EGRESS ? 1u << PCN_IPT_OUTPUT
                                                          : (1u << PCN_IPT_INPUT) | (1u << PCN_IPT_FORWARD);
    uint32_t ae_mask = 0, ct_rules = 0;
    for (int c = 0; c < PCN_IPT_NCHAINS; ++c) {
      if (!((reach >> c) & 1)) continue;
      if (ctx->ae[c] && ctx->chains[c].desc.nrules && ctx->service == PCN_IPT_SERVICE_IPTABLES) ae_mask |= 1u << c;
      if (ctx->chains[c].desc.nrules && (ctx->chains[c].desc.present & (1u << PCN_IPT_F_CONNTRACK))) ct_rules = 1;
    }
    hipStream_t st = static_cast<hipStream_t>(stream);
    const bool firewall = ctx->service == PCN_IPT_SERVICE_FIREWALL;
    const bool stateful = ctx->ct_on && !(firewall && ctx->fw_ct_mode == PCN_FW_CT_DISABLED);
    // Horus keys read the Parser's stale ports (Q4): tracked from batch to
    // batch while horus is set, in the connection table's own copy while it is
    // on (advanced by ct_run in stateful batches, here otherwise: pcn-firewall
    // with conntrack DISABLED still parses into the same struct)
    const bool track = ctx->hz_enabled || (ctx->ct_on && !stateful);
    const HorusProg *hz = horus_of_batch(ctx, b->direction);
    const bool want_stale = hz && (hz->fields & (PCN_IPT_HZ_SRCPORT | PCN_IPT_HZ_DSTPORT));
    const bool serial = stateful || track;
    if (serial && (!b->frames || !b->verdicts)) return fail(-EINVAL, "frames and verdicts are required");
    device_guard(ctx);
    // batches that share the context's conntrack / stale-port state run one
    // after another in submission order, whatever stream each comes on
    if (serial && ctx->ct_pending) hip_check(hipStreamWaitEvent(st, ctx->ev_ct, 0), "hipStreamWaitEvent(serial)");
    // with the connection table on, its own copy (advanced by ct_run when stateful)
    uint32_t *carry = ctx->ct_on ? ctx->ct.carry : ctx->d_hz_carry;
    // A Horus program still in place after horus was turned off keys on the
    // stale ports too: the table's copy while conntrack is on (the oracle's
    // st->sport/dport), as the reference's one per-CPU struct would give.
    const uint32_t *stale = want_stale && (track || ctx->ct_on) ? carry : nullptr;
    // the carry after this batch: the ports its last TCP/UDP frame left
    auto advance_carry = [&]() -> int {
      if (!track || stateful) return 0;
      if (!ctx->cts) ctx->cts = ct_scratch_new();
      const int e = ct_advance_carry(ct_batch(ctx, b, 0), *ctx->cts, carry, ctx->num_cus, st);
      if (e != hipSuccess) return fail(-EIO, std::string("stale ports: ") + hipGetErrorString(hipError_t(e)));
      return 0;
    };
    if (!ctx->ev_ct && serial) hip_check(hipEventCreateWithFlags(&ctx->ev_ct, hipEventDisableTiming), "hipEventCreate");
    auto mark = [&]() {
      if (!serial) return 0;
      hip_check(hipEventRecord(ctx->ev_ct, st), "hipEventRecord(serial)");
      ctx->ct_pending = true;
      return 0;
    };
    // pcn-firewall with conntrack DISABLED: no labels and no table updates
    // (Firewall_ConntrackTableUpdate_dp.c:136-138), whatever the table holds
    if (!stateful) {
      bool carried = false;
      int rc = launch_batch(ctx, b, stream, nullptr, stale, track ? carry : nullptr, &carried);
      if (!rc && !carried) rc = advance_carry();
      if (rc) return rc;
      if (!ae_mask) return mark();
      // Not serialised with other streams' batches (ae_mask is not in
      // `serial`): the accept-established counter move is an atomic exchange
      // and add on d_ae, so interleaved batches neither lose nor double counts.
      device_guard(ctx);
      for (int c = 0; c < PCN_IPT_NCHAINS; ++c)   // rule 0's counts, wherever the flushes put them
        if ((ae_mask >> c) & 1) fold_counters(ctx, ctx->chains[c], 4, st);
      const int e = ct_ae_fixup(ct_batch(ctx, b, ae_mask), st);
      if (e != hipSuccess) return fail(-EIO, std::string("accept-established fixup: ") + hipGetErrorString(hipError_t(e)));
      return mark();
    }
    // stateful: stage A (one classify run per label that can change the outcome), then conntrack.hpp B-E
    if (b->ct_status) return fail(-EINVAL, "stateful conntrack labels packets from its table: ct_status must be NULL");
    const uint32_t nlab = ct_rules ? 4 : 1;
    const size_t n = b->n;
    const size_t need = nlab * n * 5 + (b->rule_ids ? 0 : n * 4) + 64;
    if (ctx->ct_buf_cap < need) {
      if (ctx->ct_buf) hip_check(hipFree(ctx->ct_buf), "hipFree");
      ctx->ct_buf = nullptr;
      hip_check(hipMalloc(&ctx->ct_buf, need), "hipMalloc(conntrack outcomes)");
      ctx->ct_buf_cap = need;
    }
    int32_t *a_rid = static_cast<int32_t *>(ctx->ct_buf);
    int32_t *rids = b->rule_ids ? b->rule_ids : a_rid + nlab * n;
    uint8_t *a_v = reinterpret_cast<uint8_t *>(a_rid + nlab * n + (b->rule_ids ? 0 : n));
    if (nlab == 1) {
      // one label: stage A writes straight into the final outcome arrays (every
      // packet's label-0 outcome is its outcome unless the walk changes it), and
      // ct_prep, seeing them aliased, does not copy them there (2^24 packets:
      // 80 MB of writes)
      a_rid = rids;
      a_v = b->verdicts;
    }
    // Frames shorter than 70 bytes (no ICMP header can quote another) with
    // one label and no Horus program: stage A builds the walk records, key
    // buckets and {len, cinfo} words itself (devchain.h ct_walk_rec), and ct_run
    // skips ct_prep (its ct_stale_fix completes the stale ports and advances the
    // carry) -- the batch's frames are read once instead of twice
    // (PCN_IPT_DEBUG_CT_FUSED=0: ct_prep, A/B).
    const bool fused = nlab == 1 && !hz && !b->offsets && !b->lens && b->fixed_len < 70 &&
                       b->hook == PCN_IPT_HOOK_XDP && n < 0x7FFFFFFFull && ct_fused_prep();
    if (!ctx->cts) ctx->cts = ct_scratch_new();
    for (uint32_t l = 0; l < nlab; ++l) {
      StageA sa{ctx->d_labels + l, a_v + l * n, a_rid + l * n};
      if (fused) {
        const int e = ct_prep_buffers(*ctx->cts, n, &sa.brec, &sa.keys, &sa.lcs, &sa.sentinel, &sa.pdesc, &sa.fixm);
        if (e != hipSuccess) return fail(-EIO, std::string("conntrack buffers: ") + hipGetErrorString(hipError_t(e)));
      }
      int rc = launch_batch(ctx, b, stream, &sa, fused ? nullptr : stale);
      if (rc) return rc;
    }
    // pcn-firewall AUTOMATIC: ESTABLISHED packets are accepted before the chain
    // (Firewall_ConntrackLabel_dp.c:474-478); uncounted -- the firewall has no
    // accept-established counters, so what ct_count puts there is never read
    if (firewall && ctx->fw_ct_mode == PCN_FW_CT_AUTOMATIC)
      ae_mask = b->direction == PCN_IPT_EGRESS ? 1u << PCN_IPT_OUTPUT : 1u << PCN_IPT_FORWARD;
    CtBatch cb = ct_batch(ctx, b, ae_mask);
    cb.nlab = nlab;
    cb.a_verdict = a_v;
    cb.a_rid = a_rid;
    cb.rule_ids = rids;
    const int e = ct_run(cb, ctx->ct, *ctx->cts, ctx->num_cus, st, fused);
    if (e != hipSuccess) return fail(-EIO, std::string("conntrack: ") + hipGetErrorString(hipError_t(e)));
    if (fused) ++ctx->ct_fused_batches;
    return mark();
  });
}

int pcn_ipt_get_jit_info(pcn_ipt *ctx, pcn_ipt_jit_info *out) {
  return guarded(ctx, [&] {
    if (!out) return fail(-EINVAL, "null output");
    out->launches_generic = ctx->launches_generic;
    out->launches_jit = ctx->launches_jit;
    out->programs_ready = static_cast<uint32_t>(ctx->jit.compiled());
    out->programs_failed = static_cast<uint32_t>(ctx->jit.failed());
    out->launches_split = ctx->launches_split;
    return 0;
  });
}

namespace {
// The chain program spec of a chain's usual launch shape: a stateless
// fixed-stride batch of 64-byte frames in the chain's direction, planned by
// the launch code itself (so the descriptor has the same LDS placement,
// counter bins -- Horus bins included -- and side inputs as the launches it is
// compiled for).  0, or a negative errno (with the error set).
int usual_spec(pcn_ipt *ctx, int chain, std::string &spec) {
    pcn_ipt_batch b{};
    uint8_t *const never_read = reinterpret_cast<uint8_t *>(uintptr_t(1) << 12);   // a plan reads no buffer
    b.frames = never_read;
    b.n = uint64_t(1) << 20;
    b.stride = 64;
    b.fixed_len = 64;
    b.frames_bytes = b.n * b.stride;
    b.verdicts = never_read;
    b.direction = chain == PCN_IPT_OUTPUT ? PCN_IPT_EGRESS : PCN_IPT_INGRESS;
    const HorusProg *hz = horus_of_batch(ctx, b.direction);
    const bool track = ctx->hz_enabled || ctx->ct_on;
    const bool want_stale = hz && (hz->fields & (PCN_IPT_HZ_SRCPORT | PCN_IPT_HZ_DSTPORT));
    const uint32_t *stale = want_stale && track ? (ctx->ct_on ? ctx->ct.carry : ctx->d_hz_carry) : nullptr;
    int rc = launch_batch(ctx, &b, nullptr, nullptr, stale, nullptr, nullptr, &spec);
    if (rc) return rc;
    if (spec.empty()) return fail(-ENOENT, "no chain program runs this chain's rules in its usual launch");
    return 0;
}
}  // namespace

int pcn_ipt_chain_program_compile_for(pcn_ipt *ctx, int chain, const pcn_ipt_batch *shape) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    if (!shape) return fail(-EINVAL, "null shape");
    if (ctx->chains[chain].info.nrules == 0) return fail(-ENOENT, "chain has no rules");
    // a plan reads no buffer: any non-null address stands in for the batch's own
    pcn_ipt_batch b = *shape;
    uint8_t *const never_read = reinterpret_cast<uint8_t *>(uintptr_t(1) << 12);
    if (!b.frames) b.frames = never_read;
    if (!b.verdicts) b.verdicts = never_read;
    if (!b.n) b.n = uint64_t(1) << 20;
    if (!b.offsets && !b.frames_bytes) b.frames_bytes = b.n * uint64_t(b.stride ? b.stride : 64);
    std::string spec;
    if (int rc = launch_batch(ctx, &b, nullptr, nullptr, nullptr, nullptr, nullptr, &spec)) return rc;
    if (spec.empty()) return fail(-ENOENT, "no chain program runs this chain's rules in that launch");
    ctx->jit.request(spec, true);
    if (!ctx->jit.ready(spec)) return fail(-EIO, "chain program compile failed: " + ctx->jit.last_log());
    return 0;
  });
}

int pcn_ipt_chain_program_compile(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    if (ctx->chains[chain].info.nrules == 0) return fail(-ENOENT, "chain has no rules");
    std::string spec;
    if (int rc = usual_spec(ctx, chain, spec)) return rc;
    ctx->jit.request(spec, true);
    if (!ctx->jit.ready(spec)) return fail(-EIO, "chain program compile failed: " + ctx->jit.last_log());
    return 0;
  });
}

int pcn_ipt_get_program_info(pcn_ipt *ctx, int chain, pcn_ipt_program_info *out) {
  if (!out) return fail(-EINVAL, "null out");
  std::memset(out, 0, sizeof(*out));
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    const ChainState &cs = ctx->chains[chain];
    out->dynamic_lds_bytes = cs.last_lds_bytes;
    std::string spec = !cs.last_spec.empty() ? cs.last_spec : cs.jit_spec;
    if (spec.empty()) {
      if (cs.info.nrules == 0) return 0;
      if (int rc = usual_spec(ctx, chain, spec)) return rc;
    }
    ProgramMeta m;
    out->ready = ctx->jit.meta(spec, &m);
    if (out->ready != 1) return 0;
    out->vgpr_count = m.vgpr;
    out->agpr_count = m.agpr;
    out->sgpr_count = m.sgpr;
    out->vgpr_spill_count = m.vgpr_spill;
    out->sgpr_spill_count = m.sgpr_spill;
    out->scratch_bytes = m.scratch < 0 ? 0u : static_cast<uint32_t>(m.scratch);
    out->static_lds_bytes = m.static_lds < 0 ? 0u : static_cast<uint32_t>(m.static_lds);
    out->code_bytes = m.code_bytes;
    out->deal_window = spec.find("#define PCN_DEAL2 2") != std::string::npos ||
                               (spec.find("#define PCN_DEAL2 1") != std::string::npos && cs.jit_shape.fixed)
                           ? 128u : 64u;
    out->hdr_asm = m.hdr_asm;
    return 0;
  });
}

int pcn_ipt_debug_sort_pairs(pcn_ipt *ctx, const uint32_t *keys, uint64_t n, uint32_t kbits, uint32_t *keys_out,
                             uint32_t *idx_out) {
  return guarded(ctx, [&] {
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (!keys || !keys_out || !idx_out || kbits == 0 || kbits > 32) return fail(-EINVAL, "bad argument");
    device_guard(ctx);
    RadixScratch rx;
    uint32_t *tmp = nullptr;
    hip_check(hipMalloc(&tmp, std::max<uint64_t>(n, 1) * 4), "hipMalloc(sort keys)");
    hip_check(hipMemcpy(tmp, keys, n * 4, hipMemcpyDeviceToDevice), "hipMemcpy(sort keys)");
    const int rc = radix_sort_pairs(rx, tmp, keys_out, idx_out, n, kbits, ctx->num_cus, nullptr);
    const hipError_t e = hipDeviceSynchronize();
    (void)hipFree(tmp);
    radix_free(rx);
    if (rc != hipSuccess) return fail(-EINVAL, std::string("radix sort: ") + hipGetErrorString(hipError_t(rc)));
    hip_check(e, "hipDeviceSynchronize");
    return 0;
  });
}

int pcn_ipt_debug_clocks(pcn_ipt *ctx, uint64_t *out, uint32_t cap) {
  return guarded(ctx, [&] {
    if (!ctx->d_dbg_clk || !ctx->dbg_grid) return fail(-ENOENT, "no launch recorded (PCN_IPT_DEBUG_CLOCKS=1)");
    if (!out || cap < 4 * ctx->dbg_grid) return static_cast<int>(ctx->dbg_grid);
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipMemcpy(out, ctx->d_dbg_clk, size_t(ctx->dbg_grid) * 32, hipMemcpyDeviceToHost), "hipMemcpy(clocks)");
    return static_cast<int>(ctx->dbg_grid);
  });
}

int pcn_ipt_release_stream(pcn_ipt *ctx, void *stream) {
  return guarded(ctx, [&] {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    auto &v = ctx->pack_streams;
    auto it = std::find_if(v.begin(), v.end(), [&](const auto &se) { return se.first == s; });
    if (it == v.end()) return 0;
    device_guard(ctx);
    hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    if (it->second) hip_check(hipEventDestroy(it->second), "hipEventDestroy");
    v.erase(it);
    // a lone stream records no events (note_pack_stream): drop the one it
    // holds, so no later fold trusts an event older than its last batches
    if (v.size() == 1 && v[0].second) {
      hip_check(hipEventDestroy(v[0].second), "hipEventDestroy");
      v[0].second = nullptr;
    }
    return 0;
  });
}

extern const char pcn_jit_src_classify[];
extern const char pcn_jit_src_devchain[];
extern const char pcn_jit_src_pcn_ipt[];
extern const char pcn_src_image[];
extern const char pcn_build_src_sha256[];

const char *pcn_ipt_embedded_source(int which) {
  switch (which) {
    case 0: return pcn_jit_src_classify;
    case 1: return pcn_jit_src_devchain;
    case 2: return pcn_jit_src_pcn_ipt;
    case 3: return pcn_src_image;
    default: return nullptr;
  }
}

const char *pcn_ipt_build_sha256(void) { return pcn_build_src_sha256; }

int pcn_ipt_chain_get_info(pcn_ipt *ctx, int chain, pcn_ipt_chain_info *out) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain) || !out) return fail(-EINVAL, "bad chain or output");
    *out = ctx->chains[chain].info;
    return 0;
  });
}

int pcn_ipt_chain_get_image(pcn_ipt *ctx, int chain, uint8_t *buf, uint32_t cap, uint32_t *desc,
                            uint32_t desc_cap) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    const ChainState &cs = ctx->chains[chain];
    if (buf && cap >= cs.image_copy.size()) std::memcpy(buf, cs.image_copy.data(), cs.image_copy.size());
    if (desc && desc_cap >= cs.desc_words.size())
      std::memcpy(desc, cs.desc_words.data(), cs.desc_words.size() * 4);
    return static_cast<int>(cs.image_copy.size());
  });
}

int pcn_ipt_synchronize(pcn_ipt *ctx) {
  return guarded(ctx, [&] {
    if (ctx->has_device) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    }
    return 0;
  });
}

int pcn_ipt_read_counters(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n,
                          uint64_t *def_pkts, uint64_t *def_bytes, int flush, int scope) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    ChainState &cs = ctx->chains[chain];
    std::vector<unsigned long long> buf(ctx->ctr_words, 0);
    if (ctx->has_device) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      fold_counters(ctx, cs, ctx->ctr_words, nullptr);
      hip_check(hipMemcpy(buf.data(), scope ? cs.ctr_global : cs.ctr, buf.size() * 8, hipMemcpyDeviceToHost),
                "hipMemcpy(counters)");
    }
    uint32_t nc = ctx->cfg.max_counted_rules;
    for (uint32_t i = 0; i < n; ++i) {
      if (pkts) pkts[i] = i < nc ? buf[2 + 2 * size_t(i)] : 0;
      if (bytes) bytes[i] = i < nc ? buf[3 + 2 * size_t(i)] : 0;
    }
    if (def_pkts) *def_pkts = buf[0];
    if (def_bytes) *def_bytes = buf[1];
    if (flush && ctx->has_device) {
      hip_check(hipMemset(cs.ctr + 2, 0, (ctx->ctr_words - 2) * 8), "hipMemset(counters)");
      hip_check(hipMemset(cs.ctr_global + 2, 0, (ctx->ctr_words - 2) * 8), "hipMemset(counters)");
    }
    return 0;
  });
}

int pcn_ipt_chain_stats(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n,
                        uint64_t *def_pkts, uint64_t *def_bytes) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    ChainState &cs = ctx->chains[chain];
    fetch_stats(ctx, chain);
    for (uint32_t i = 0; i < n; ++i) {
      if (pkts) pkts[i] = i < cs.stats.size() ? cs.stats[i].first : 0;
      if (bytes) bytes[i] = i < cs.stats.size() ? cs.stats[i].second : 0;
    }
    unsigned long long d[2] = {0, 0};
    if (ctx->has_device) hip_check(hipMemcpy(d, cs.ctr, 16, hipMemcpyDeviceToHost), "hipMemcpy(counters)");
    if (def_pkts) *def_pkts = d[0];
    if (def_bytes) *def_bytes = d[1];
    return static_cast<int>(cs.stats.size());
  });
}

int pcn_ipt_chain_reset_counters(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    ChainState &cs = ctx->chains[chain];
    if (ctx->has_device) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      // pcn-firewall also flushes the DefaultAction counters (pcn-firewall Chain.cpp:154-155)
      const size_t from = ctx->service == PCN_IPT_SERVICE_FIREWALL ? 0 : 2;
      fold_counters(ctx, cs, ctx->ctr_words, nullptr);
      hip_check(hipMemset(cs.ctr + from, 0, (ctx->ctr_words - from) * 8), "hipMemset(counters)");
      // ... and the chain's Horus counters of its rule ids (pcn-firewall Chain.cpp:139-152)
      const int k = horus_slot(ctx, chain);
      if (ctx->service == PCN_IPT_SERVICE_FIREWALL && k >= 0 && ctx->hz[k].runtime)
        hip_check(hipMemset(ctx->hz[k].d_ctr, 0,
                            std::min<size_t>(cs.rules.size(), PCN_IPT_HORUS_MAX) * 16), "hipMemset(horus counters)");
    }
    cs.stats.assign(cs.rules.size(), {0, 0});     // counters_.clear()
    return 0;
  });
}

int pcn_ipt_comm_unique_id(uint8_t out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(-EIO, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out, &id, 128);
  return 0;
}

int pcn_ipt_comm_init(pcn_ipt *ctx, int nranks, int rank, const uint8_t uid[128]) {
  return guarded(ctx, [&] {
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(-EINVAL, "bad rank/nranks");
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");   // no gather in flight
    if (ctx->comm) { ncclCommDestroy(ctx->comm); ctx->comm = nullptr; }
    ncclUniqueId id;
    std::memcpy(&id, uid, 128);
    ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, id, rank);
    if (r != ncclSuccess) return fail(-EIO, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    ctx->nranks = nranks;
    ctx->rank = rank;
    for (auto &cs : ctx->chains) {
      if (cs.gather) hip_check(hipFree(cs.gather), "hipFree");
      hip_check(hipMalloc(&cs.gather, ctx->ctr_words * 8 * size_t(nranks)), "hipMalloc(gather)");
      if (!cs.stage) hip_check(hipMalloc(&cs.stage, ctx->ctr_words * 8), "hipMalloc(stage)");
    }
    if (!ctx->comm_stream) hip_check(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking), "hipStreamCreate");
    if (!ctx->ev_staged) hip_check(hipEventCreateWithFlags(&ctx->ev_staged, hipEventDisableTiming), "hipEventCreate");
    if (!ctx->ev_gathered) hip_check(hipEventCreateWithFlags(&ctx->ev_gathered, hipEventDisableTiming), "hipEventCreate");
    ctx->gather_pending = false;
    return 0;
  });
}

int pcn_ipt_sync_counters(pcn_ipt *ctx, void *stream) {
  return guarded(ctx, [&] {
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    device_guard(ctx);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!ctx->comm) {
      for (auto &cs : ctx->chains) {
        fold_counters(ctx, cs, ctx->ctr_words, s);
        hip_check(hipMemcpyAsync(cs.ctr_global, cs.ctr, ctx->ctr_words * 8, hipMemcpyDeviceToDevice, s),
                  "hipMemcpyAsync(counters)");
      }
      return 0;
    }
    // The classify stream snapshots each chain's live prefix (defaults +
    // counted rules) once the previous all-gather has sent its snapshot; the
    // all-gather and the rank sum then run on the communicator's stream while
    // the classify stream goes on with the next batch.
    if (ctx->gather_pending) hip_check(hipStreamWaitEvent(s, ctx->ev_gathered, 0), "hipStreamWaitEvent");
    size_t count[PCN_IPT_NCHAINS];
    for (int c = 0; c < PCN_IPT_NCHAINS; ++c) {
      ChainState &cs = ctx->chains[c];
      count[c] = 2 + 2 * size_t(cs.desc.ncounted);
      fold_counters(ctx, cs, count[c], s);
      hip_check(hipMemcpyAsync(cs.stage, cs.ctr, count[c] * 8, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync(stage)");
    }
    hip_check(hipEventRecord(ctx->ev_staged, s), "hipEventRecord");
    hipStream_t cs_ = ctx->comm_stream;
    hip_check(hipStreamWaitEvent(cs_, ctx->ev_staged, 0), "hipStreamWaitEvent");
    // time the exchange on the communicator stream (all-gather + rank sum):
    // reuse the oldest pair of the ring, folding its duration in first
    // reuse the oldest pair of the ring once its step has run, folding its
    // duration in first; while it still runs this step goes untimed (the call
    // never waits on the device)
    const int ge = ctx->ev_g_next;
    bool timed = true;
    if (ctx->ev_g_live[ge]) {
      const hipError_t q = hipEventQuery(ctx->ev_g1[ge]);
      if (q == hipSuccess) {
        fold_gather_time(ctx, ge);
      } else if (q == hipErrorNotReady) {
        timed = false;
        ++ctx->gathers_untimed;
      } else {
        hip_check(q, "hipEventQuery");
      }
    }
    if (timed) {
      ctx->ev_g_next = (ge + 1) % pcn_ipt::kGatherEv;
      if (!ctx->ev_g0[ge]) hip_check(hipEventCreate(&ctx->ev_g0[ge]), "hipEventCreate");
      if (!ctx->ev_g1[ge]) hip_check(hipEventCreate(&ctx->ev_g1[ge]), "hipEventCreate");
      hip_check(hipEventRecord(ctx->ev_g0[ge], cs_), "hipEventRecord");
    }
    ncclResult_t r = ncclGroupStart();
    for (int c = 0; c < PCN_IPT_NCHAINS && r == ncclSuccess; ++c)
      r = ncclAllGather(ctx->chains[c].stage, ctx->chains[c].gather, count[c], ncclUint64, ctx->comm, cs_);
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(-EIO, std::string("ncclAllGather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    for (int c = 0; c < PCN_IPT_NCHAINS; ++c) {
      ChainState &cs = ctx->chains[c];
      int rc = launch_sum_ranks(cs.gather, cs.ctr_global, count[c], ctx->nranks, cs_);
      if (rc != hipSuccess) return fail(-EIO, "sum_ranks launch failed");
    }
    if (timed) {
      hip_check(hipEventRecord(ctx->ev_g1[ge], cs_), "hipEventRecord");
      ctx->ev_g_live[ge] = true;
    }
    hip_check(hipEventRecord(ctx->ev_gathered, cs_), "hipEventRecord");
    ctx->gather_pending = true;
    return 0;
  });
}

int pcn_ipt_debug_ct_walk_passes(pcn_ipt *ctx, uint64_t out[2], int reset) {
  return guarded(ctx, [&] {
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (!out) return fail(-EINVAL, "null out");
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(static_cast<hipError_t>(ct_walk_passes(out, reset != 0)), "ct_walk_passes");
    return 0;
  });
}

int pcn_ipt_debug_stale_canary(pcn_ipt *ctx) {
  return guarded(ctx, [&] {
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (!ctx->d_stale_desc) return fail(-ENOENT, "no stale-port groups allocated");
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    const size_t from = ctx->stale_guard_from, words = ctx->stale_groups + kStaleCanary - from;
    std::vector<uint64_t> w(words);
    hip_check(hipMemcpy(w.data(), ctx->d_stale_desc + from, words * 8, hipMemcpyDeviceToHost), "hipMemcpy(canary)");
    uint64_t pat;
    std::memset(&pat, kStaleCanaryByte, 8);
    int bad = 0;
    for (uint64_t x : w) bad += x != pat;
    return bad;
  });
}

int pcn_ipt_comm_get_info(pcn_ipt *ctx, pcn_ipt_comm_info *out) {
  if (!out) return fail(-EINVAL, "null out");
  std::memset(out, 0, sizeof(*out));
  int v = 0;
  if (ncclGetVersion(&v) == ncclSuccess) out->nccl_version = v;
  Dl_info di{};
  if (dladdr(reinterpret_cast<void *>(&ncclCommInitRank), &di) && di.dli_fname)
    std::snprintf(out->rccl_path, sizeof(out->rccl_path), "%s", di.dli_fname);
  out->device = -1;
  if (!ctx) return 0;
  return guarded(ctx, [&] {
    out->nranks = ctx->comm ? ctx->nranks : 0;
    out->rank = ctx->comm ? ctx->rank : 0;
    if (!ctx->has_device) return 0;
    device_guard(ctx);
    out->device = ctx->cfg.device;
    hip_check(hipDeviceGetPCIBusId(out->pci_bus_id, sizeof(out->pci_bus_id), ctx->cfg.device),
              "hipDeviceGetPCIBusId");
    for (int k = 0; k < pcn_ipt::kGatherEv; ++k)
      if (ctx->ev_g_live[k]) fold_gather_time(ctx, k);
    out->gathers_timed = ctx->gathers_timed;
    out->gather_ms_total = ctx->gather_ms;
    out->gathers_untimed = ctx->gathers_untimed;
    return 0;
  });
}

int pcn_ipt_counter_block_words(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    return static_cast<int>(2 + 2 * size_t(counted(ctx, ctx->chains[chain].info.nrules)));   // the applied chain
  });
}

int pcn_ipt_snapshot_counters(pcn_ipt *ctx, int chain, uint64_t *block, void *stream) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (!block) return fail(-EINVAL, "null block");
    device_guard(ctx);
    ChainState &cs = ctx->chains[chain];
    const size_t words = 2 + 2 * size_t(cs.desc.ncounted);
    fold_counters(ctx, cs, words, static_cast<hipStream_t>(stream));
    hip_check(hipMemcpyAsync(block, cs.ctr, words * 8, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)),
              "hipMemcpyAsync(snapshot)");
    return 0;
  });
}

int pcn_ipt_sum_counter_blocks(pcn_ipt *ctx, int chain, const uint64_t *blocks, uint32_t nranks, uint64_t words,
                               void *stream) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (!blocks) return fail(-EINVAL, "null blocks");
    if (nranks < 1 || nranks > 4096) return fail(-EINVAL, "nranks must be 1..4096");
    ChainState &cs = ctx->chains[chain];
    if (words != 2 + 2 * uint64_t(cs.desc.ncounted) || words > ctx->ctr_words)
      return fail(-EINVAL, "words != the chain's counter block words");
    device_guard(ctx);
    int rc = launch_sum_ranks(reinterpret_cast<const unsigned long long *>(blocks), cs.ctr_global, words,
                              static_cast<int>(nranks), static_cast<hipStream_t>(stream));
    if (rc != hipSuccess) return fail(-EIO, "sum_ranks launch failed");
    return 0;
  });
}

// ---- stateful conntrack ---------------------------------------------------

int pcn_ipt_ct_enable(pcn_ipt *ctx, uint32_t capacity_log2) {
  return guarded(ctx, [&] {
    if (!ctx->has_device) return fail(-ENODEV, "no device");
    if (capacity_log2 == 0) capacity_log2 = 18;
    if (capacity_log2 < 10 || capacity_log2 > 30) return fail(-EINVAL, "capacity_log2 must be 10..30");
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    if (!ctx->ct.slots || ctx->ct.cap_log2 != capacity_log2) {
      const unsigned long long now = ctx->ct.now;
      hip_check(hipError_t(ct_table_init(ctx->ct, capacity_log2)), "conntrack table");
      ctx->ct.now = now;
    }
    if (!ctx->cts) ctx->cts = ct_scratch_new();
    ctx->ct_on = true;
    return 0;
  });
}

int pcn_ipt_ct_disable(pcn_ipt *ctx) {
  return guarded(ctx, [&] {
    ctx->ct_on = false;
    return 0;
  });
}

int pcn_ipt_ct_clear(pcn_ipt *ctx) {
  return guarded(ctx, [&] {
    if (!ctx->ct.slots) return 0;
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    hip_check(hipMemset(ctx->ct.slots, 0, (size_t(1) << ctx->ct.cap_log2) * sizeof(CtSlot)), "hipMemset(conntrack)");
    hip_check(hipMemset(ctx->ct.carry, 0, 64), "hipMemset(conntrack)");
    hip_check(hipMemset(ctx->ct.touch, 0xff, (size_t(1) << ctx->ct.cap_log2) * 8), "hipMemset(conntrack)");
    ctx->ct.seq = 1;
    return 0;
  });
}

int pcn_ipt_ct_set_max_entries(pcn_ipt *ctx, uint64_t max_entries) {
  return guarded(ctx, [&] {
    if (max_entries > (uint64_t(1) << 32) - 1) return fail(-EINVAL, "max_entries must be below 2^32");
    ctx->ct.max_entries = max_entries;
    return 0;
  });
}

int pcn_ipt_ct_set_time(pcn_ipt *ctx, uint64_t ns) {
  return guarded(ctx, [&] {
    ctx->ct.now = ns;
    return 0;
  });
}

int pcn_ipt_ct_dump(pcn_ipt *ctx, pcn_ipt_ct_entry *out, uint32_t cap) {
  return guarded(ctx, [&] {
    if (!ctx->ct.slots) return fail(-EINVAL, "conntrack is not enabled");
    device_guard(ctx);
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    std::vector<CtSlot> slots(size_t(1) << ctx->ct.cap_log2);
    hip_check(hipMemcpy(slots.data(), ctx->ct.slots, slots.size() * sizeof(CtSlot), hipMemcpyDeviceToHost),
              "hipMemcpy(conntrack)");
    std::vector<pcn_ipt_ct_entry> v;
    for (const CtSlot &e : slots) {
      if (e.tag != 1 || !e.valid) continue;
      pcn_ipt_ct_entry x{};
      x.src_ip = e.src; x.dst_ip = e.dst; x.sport = e.sport; x.dport = e.dport; x.l4proto = e.proto;
      x.state = e.state; x.ip_rev = e.rev & 1; x.port_rev = (e.rev >> 1) & 1; x.sequence = e.seq; x.ttl = e.ttl;
      v.push_back(x);
    }
    std::sort(v.begin(), v.end(), [](const pcn_ipt_ct_entry &a, const pcn_ipt_ct_entry &b) {
      if (a.src_ip != b.src_ip) return a.src_ip < b.src_ip;
      if (a.dst_ip != b.dst_ip) return a.dst_ip < b.dst_ip;
      if (a.l4proto != b.l4proto) return a.l4proto < b.l4proto;
      if (a.sport != b.sport) return a.sport < b.sport;
      return a.dport < b.dport;
    });
    if (out) std::memcpy(out, v.data(), std::min<size_t>(v.size(), cap) * sizeof(pcn_ipt_ct_entry));
    return static_cast<int>(v.size());
  });
}

int pcn_ipt_ct_get_info(pcn_ipt *ctx, pcn_ipt_ct_info *out) {
  return guarded(ctx, [&] {
    if (!out) return fail(-EINVAL, "null output");
    *out = pcn_ipt_ct_info{};
    out->enabled = ctx->ct_on;
    out->capacity_log2 = ctx->ct.cap_log2;
    out->now = ctx->ct.now;
    if (ctx->ct.carry) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      unsigned long long st[2] = {0, 0};
      hip_check(hipMemcpy(st, ctx->ct.stats, 16, hipMemcpyDeviceToHost), "hipMemcpy(conntrack stats)");
      out->inserts_lost = st[0];
      out->evicted = st[1];
      out->fused_batches = ctx->ct_fused_batches;
    }
    out->max_entries = ctx->ct.max_entries;
    return 0;
  });
}

int pcn_ipt_set_accept_established(pcn_ipt *ctx, int chain, int on) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    if (ctx->service == PCN_IPT_SERVICE_FIREWALL)
      return fail(-EINVAL, "pcn-firewall: use pcn_fw_set_accept_established");
    ctx->ae[chain] = on != 0;
    return 0;
  });
}

int pcn_ipt_get_accept_established(pcn_ipt *ctx, int chain) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    return ctx->ae[chain] ? 1 : 0;
  });
}

int pcn_ipt_read_accept_established(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, int flush) {
  return guarded(ctx, [&] {
    if (!valid_chain(chain)) return fail(-EINVAL, "bad chain");
    unsigned long long v[2] = {0, 0};
    if (ctx->has_device) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      hip_check(hipMemcpy(v, ctx->d_ae + 2 * chain, 16, hipMemcpyDeviceToHost), "hipMemcpy(ae counters)");
      if (flush) hip_check(hipMemset(ctx->d_ae + 2 * chain, 0, 16), "hipMemset(ae counters)");
    }
    if (pkts) *pkts = v[0];
    if (bytes) *bytes = v[1];
    return 0;
  });
}

// ---- Horus ---------------------------------------------------------------

int pcn_ipt_set_horus(pcn_ipt *ctx, int on) {
  return guarded(ctx, [&] {
    // Iptables::setHorus (Iptables.cpp:400-406): the flag; the next chain
    // update acts on it.  (pcn-firewall has no such knob: on from the start.)
    ctx->hz_enabled = on != 0;
    return 0;
  });
}

int pcn_ipt_get_horus_info(pcn_ipt *ctx, int chain, pcn_ipt_horus_info *out) {
  return guarded(ctx, [&] {
    if (!out) return fail(-EINVAL, "null output");
    const int k = horus_slot(ctx, chain);
    if (k < 0) return fail(-EINVAL, "no Horus program for this chain");
    const HorusProg &h = ctx->hz[k];
    out->enabled = ctx->hz_enabled;
    out->runtime = h.runtime;
    out->entries = h.entries;
    out->fields = h.fields;
    out->conntrack = h.runtime && h.ct;
    return 0;
  });
}

int pcn_ipt_read_horus_counters(pcn_ipt *ctx, int chain, uint64_t *pkts, uint64_t *bytes, uint32_t n, int flush) {
  return guarded(ctx, [&] {
    const int k = horus_slot(ctx, chain);
    if (k < 0) return fail(-EINVAL, "no Horus program for this chain");
    std::vector<unsigned long long> v(2 * size_t(PCN_IPT_HORUS_MAX), 0);
    if (ctx->has_device) {
      device_guard(ctx);
      hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
      hip_check(hipMemcpy(v.data(), ctx->hz[k].d_ctr, v.size() * 8, hipMemcpyDeviceToHost), "hipMemcpy(horus counters)");
      if (flush) hip_check(hipMemset(ctx->hz[k].d_ctr, 0, v.size() * 8), "hipMemset(horus counters)");
    }
    for (uint32_t i = 0; i < n; ++i) {
      if (pkts) pkts[i] = i < PCN_IPT_HORUS_MAX ? v[2 * size_t(i)] : 0;
      if (bytes) bytes[i] = i < PCN_IPT_HORUS_MAX ? v[2 * size_t(i) + 1] : 0;
    }
    return 0;
  });
}

// ---- pcn-firewall personality -------------------------------------------

int pcn_ipt_set_service(pcn_ipt *ctx, int service) {
  return guarded(ctx, [&] {
    if (service != PCN_IPT_SERVICE_IPTABLES && service != PCN_IPT_SERVICE_FIREWALL)
      return fail(-EINVAL, "unknown service");
    for (const ChainState &cs : ctx->chains)
      if (!cs.rules.empty() || cs.desc.nrules) return fail(-EBUSY, "set the service before adding rules");
    if (ctx->ct_on) return fail(-EBUSY, "disable the connection table first");
    ctx->service = service;
    ctx->fw_ct_mode = PCN_FW_CT_AUTOMATIC;            // Firewall.h:323
    for (bool &on : ctx->ae) on = false;
    // pcn-firewall's horus_enabled is true from the start (Firewall.h:337);
    // pcn-iptables' leaf is OFF by default (Iptables.h:185)
    ctx->hz_enabled = service == PCN_IPT_SERVICE_FIREWALL;
    for (HorusProg &h : ctx->hz) horus_set(ctx, h, {}, 0);
    return 0;
  });
}

int pcn_ipt_get_service(pcn_ipt *ctx) {
  return guarded(ctx, [&] { return ctx->service; });
}

int pcn_fw_set_conntrack(pcn_ipt *ctx, int on) {
  return guarded(ctx, [&] {
    if (ctx->service != PCN_IPT_SERVICE_FIREWALL) return fail(-EINVAL, "not a pcn-firewall context");
    if (!on) ctx->fw_ct_mode = PCN_FW_CT_DISABLED;                       // Firewall.cpp:152-174
    else if (ctx->fw_ct_mode == PCN_FW_CT_DISABLED) ctx->fw_ct_mode = PCN_FW_CT_MANUAL;   // :176-193
    return 0;
  });
}

int pcn_fw_set_accept_established(pcn_ipt *ctx, int on) {
  return guarded(ctx, [&] {
    if (ctx->service != PCN_IPT_SERVICE_FIREWALL) return fail(-EINVAL, "not a pcn-firewall context");
    if (ctx->fw_ct_mode == PCN_FW_CT_DISABLED) return fail(-EINVAL, "Please enable conntrack first.");
    ctx->fw_ct_mode = on ? PCN_FW_CT_AUTOMATIC : PCN_FW_CT_MANUAL;   // Firewall.cpp:119-142
    return 0;
  });
}

int pcn_fw_get_conntrack_mode(pcn_ipt *ctx) {
  return guarded(ctx, [&] {
    if (ctx->service != PCN_IPT_SERVICE_FIREWALL) return fail(-EINVAL, "not a pcn-firewall context");
    return ctx->fw_ct_mode;
  });
}

int pcn_fw_chain_update(pcn_ipt *ctx, int chain, uint32_t id, const pcn_ipt_rule *rule) {
  return guarded(ctx, [&] {
    if (ctx->service != PCN_IPT_SERVICE_FIREWALL) return fail(-EINVAL, "not a pcn-firewall context");
    if (!valid_chain(ctx, chain) || !rule) return fail(-EINVAL, "bad chain or rule");
    ChainState &cs = ctx->chains[chain];
    if (id > cs.rules.size()) return fail(-EINVAL, "rule id not allowed");   // Chain.cpp:614-616
    Rule r = rule_from_c(ctx, *rule);
    if (id == cs.rules.size() && cs.rules.size() >= ctx->cfg.max_rules) return fail(-ENOSPC, "too many rules");
    fetch_stats(ctx, chain);                          // "Forcing counters update" (Chain.cpp:624-625)
    if (id == cs.rules.size()) {
      cs.rules.push_back(std::move(r));
      cs.stats.resize(cs.rules.size());
    } else {
      cs.rules[id] = std::move(r);                    // the rule's counters carry on (counters_[id] kept)
    }
    if (ctx->interactive) update_chain(ctx, chain);
    return 0;
  });
}


static int flow_args(pcn_ipt *ctx, const pcn_ipt_batch *b, uint32_t nranks) {
  if (!b) return fail(-EINVAL, "null batch");
  if (!ctx->has_device) return fail(-ENODEV, "context has no HIP device (created with device=-1)");
  if (nranks < 1 || nranks > 255) return fail(-EINVAL, "nranks must be 1..255");
  if (b->n && !b->frames) return fail(-EINVAL, "frames are required");
  if (b->n > 0xffffffffull) return fail(-EINVAL, "at most 2^32-1 frames per batch");
  if (b->hook != PCN_IPT_HOOK_XDP && b->hook != PCN_IPT_HOOK_TC) return fail(-EINVAL, "unknown hook");
  return 0;
}

int pcn_ipt_flow_owner(pcn_ipt *ctx, const pcn_ipt_batch *b, uint32_t nranks, uint8_t *owner, void *stream) {
  return guarded(ctx, [&] {
    if (int rc = flow_args(ctx, b, nranks)) return rc;
    if (b->n && !owner) return fail(-EINVAL, "owner is required");
    device_guard(ctx);
    const int e = ct_flow_owner(ct_batch(ctx, b, 0), nranks, owner, ctx->num_cus, stream);
    if (e != hipSuccess) return fail(-EIO, std::string("flow owner: ") + hipGetErrorString(hipError_t(e)));
    return 0;
  });
}

int pcn_ipt_flow_split(pcn_ipt *ctx, const pcn_ipt_batch *b, uint32_t nranks, uint32_t rank, uint32_t *index,
                       uint32_t *offsets, uint16_t *lens, uint16_t *in_port_out, uint64_t *n_out, void *stream) {
  return guarded(ctx, [&] {
    if (int rc = flow_args(ctx, b, nranks)) return rc;
    if (rank >= nranks) return fail(-EINVAL, "rank must be < nranks");
    if (!n_out) return fail(-EINVAL, "n_out is required");
    *n_out = 0;
    if (!b->n) return 0;
    if (!index || !offsets || !lens) return fail(-EINVAL, "index, offsets and lens are required");
    if (!b->offsets && (b->n - 1) * uint64_t(b->stride) > 0xffffffffull)
      return fail(-EINVAL, "a fixed-stride batch must end below 4 GiB (offsets are u32)");
    if (!b->lens && b->fixed_len > 0xffff) return fail(-EINVAL, "fixed_len must fit u16");
    device_guard(ctx);
    const int e = ct_flow_split(ct_batch(ctx, b, 0), b->in_port, b->const_in_port, nranks, rank, index, offsets,
                                lens, in_port_out, n_out, ctx->num_cus, stream);
    if (e != hipSuccess) return fail(-EIO, std::string("flow split: ") + hipGetErrorString(hipError_t(e)));
    return 0;
  });
}

}  // extern "C"

