// ring.cpp — host ingest ring: frames that start in host memory (a NIC or
// AF_XDP/AF_PACKET RX ring, a veth) go through pinned slots to HBM, are
// classified there, and their verdicts come back to pinned host memory.
//
// This is the MI355X counterpart of the reference's packet entry, where the
// kernel hands each received frame to the cube's first program
// (extiface_xdp.cpp:178-200 -> cube_xdp.cpp:403-449 handle_rx_xdp_wrapper,
// cube_tc.cpp:374-432 for TC): instead of one frame per call, a slot of frames
// per submit, pipelined over HIP streams so the PCIe copies in and out overlap
// the classify kernels of other slots.
#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <algorithm>
#include <condition_variable>
#include <cerrno>
#include <cstring>
#include <chrono>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pcn_ipt.h"

namespace {

enum SlotState { kFree, kFilling, kInFlight, kReturned };

struct Slot {
  SlotState state = kFree;
  // pinned host memory
  uint8_t *h_frames = nullptr;
  uint32_t *h_offsets = nullptr;
  uint16_t *h_lens = nullptr;
  uint16_t *h_in_port = nullptr;
  uint8_t *h_verdicts = nullptr;
  int32_t *h_rule_ids = nullptr;
  // device memory
  uint8_t *d_frames = nullptr;
  uint32_t *d_offsets = nullptr;
  uint16_t *d_lens = nullptr;
  uint16_t *d_in_port = nullptr;
  uint8_t *d_verdicts = nullptr;
  int32_t *d_rule_ids = nullptr;
  hipEvent_t done = nullptr;
  uint64_t n = 0;
  // PCN_IPT_RING_HOST_PACK: the packed header windows (pinned host), bytes held
  uint8_t *h_pack = nullptr;
  size_t pack_cap = 0;
  // PCN_IPT_RING_ZERO_COPY: device addresses of the pinned buffers (not owned)
  uint8_t *z_frames = nullptr;
  uint32_t *z_offsets = nullptr;
  uint16_t *z_lens = nullptr, *z_in_port = nullptr;
};

// Host threads that pack header windows (PCN_IPT_RING_HOST_PACK): run(fn, k)
// calls fn(0..k-1) on the pool (and the caller) and returns when all are done.
class PackPool {
 public:
  explicit PackPool(unsigned n) {
    for (unsigned i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~PackPool() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : workers_) t.join();
  }
  void run(const std::function<void(unsigned)> &fn, unsigned parts) {
    std::unique_lock<std::mutex> l(mu_);
    fn_ = &fn;
    parts_ = parts;
    next_ = 0;
    left_ = parts;
    ++gen_;
    cv_.notify_all();
    l.unlock();
    work();                                    // the caller takes parts too
    l.lock();
    done_.wait(l, [&] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      unsigned k;
      const std::function<void(unsigned)> *fn;
      {
        std::lock_guard<std::mutex> l(mu_);
        if (!fn_ || next_ >= parts_) return;
        k = next_++;
        fn = fn_;
      }
      (*fn)(k);
      std::lock_guard<std::mutex> l(mu_);
      if (--left_ == 0) done_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(unsigned)> *fn_ = nullptr;
  unsigned parts_ = 0, next_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

namespace pcn {
int fail(int code, const std::string &msg);   // pcn_ipt.cpp: sets pcn_ipt_last_error()
int device_of(const pcn_ipt *ctx);
}  // namespace pcn

namespace {
int ring_fail(int code, const std::string &msg) { return pcn::fail(code, msg); }
}  // namespace

namespace {
// Copy `rows` rows of hb bytes from a stride-byte source into contiguous rows
// (the host pack).  The common widths copy with a compile-time size, so each
// row is a few 16-byte moves instead of a memcpy call (a 48-byte call per
// frame held 16 threads at ~3.7 GB/s each, 74 % of the e2e leg's wall time).
// The rows go out with streaming stores: the packed buffer is read only by
// the DMA engine, so its lines need not be fetched into the cache first (a
// plain store reads each destination line before writing it).
template <size_t W>
void pack_fixed(uint8_t *dst, const uint8_t *src, size_t rows, size_t stride) {
  static_assert(W % 16 == 0, "16-byte rows");
  if (reinterpret_cast<uintptr_t>(dst) % 16) {
    for (size_t i = 0; i < rows; ++i) std::memcpy(dst + i * W, src + i * stride, W);
    return;
  }
  for (size_t i = 0; i < rows; ++i) {
    const __m128i *s = reinterpret_cast<const __m128i *>(src + i * stride);
    __m128i *d = reinterpret_cast<__m128i *>(dst + i * W);
    for (size_t q = 0; q < W / 16; ++q) _mm_stream_si128(d + q, _mm_loadu_si128(s + q));
  }
  _mm_sfence();
}
// Rows of W bytes, W a multiple of 4 but not of 16 (the windows without their
// 12 Ethernet-address bytes, hdr_skip): four rows are a whole number of 16-byte
// stores, assembled in registers (compile-time copies) and streamed out.
template <size_t W>
void pack_fixed4(uint8_t *dst, const uint8_t *src, size_t rows, size_t stride) {
  static_assert(W % 4 == 0 && (4 * W) % 16 == 0, "four rows: whole 16-byte stores");
  size_t i = 0;
  if (reinterpret_cast<uintptr_t>(dst) % 16 == 0) {
    alignas(16) uint8_t buf[4 * W];
    for (; i + 4 <= rows; i += 4) {
      for (size_t r = 0; r < 4; ++r) std::memcpy(buf + r * W, src + (i + r) * stride, W);
      __m128i *d = reinterpret_cast<__m128i *>(dst + i * W);
      for (size_t q = 0; q < 4 * W / 16; ++q) _mm_stream_si128(d + q, _mm_load_si128(reinterpret_cast<const __m128i *>(buf) + q));
    }
    _mm_sfence();
  }
  for (; i < rows; ++i) std::memcpy(dst + i * W, src + i * stride, W);
}
void pack_rows(uint8_t *dst, const uint8_t *src, size_t rows, size_t hb, size_t stride) {
  switch (hb) {
    case 48: pack_fixed<48>(dst, src, rows, stride); return;
    case 64: pack_fixed<64>(dst, src, rows, stride); return;
    case 80: pack_fixed<80>(dst, src, rows, stride); return;
    case 36: pack_fixed4<36>(dst, src, rows, stride); return;
    case 52: pack_fixed4<52>(dst, src, rows, stride); return;
    default:
      for (size_t i = 0; i < rows; ++i) std::memcpy(dst + i * hb, src + i * stride, hb);
  }
}
// hdr_skip: the device rows start kSkipPad bytes into the slot's frame buffer, so
// frame i's (unused) first bytes, read by the classify kernel's header window
// from before row i, stay inside the buffer (and a generic-path gather's 16-byte
// aligned start, up to 15 bytes earlier still)
constexpr size_t kSkipPad = 32;
}  // namespace

struct pcn_ipt_ring {
  pcn_ipt *ctx = nullptr;
  int device = 0;
  pcn_ipt_ring_config cfg{};
  std::vector<Slot> slots;
  std::vector<hipStream_t> streams;
  std::deque<uint32_t> inflight;   // submission order
  std::mutex mu;
  std::unique_ptr<PackPool> pack;  // PCN_IPT_RING_HOST_PACK
  pcn_ipt_ring_stats stats{};      // under mu
};

namespace {

void free_slot(Slot &s) {
  if (s.h_frames) (void)hipHostFree(s.h_frames);
  if (s.h_offsets) (void)hipHostFree(s.h_offsets);
  if (s.h_lens) (void)hipHostFree(s.h_lens);
  if (s.h_in_port) (void)hipHostFree(s.h_in_port);
  if (s.h_verdicts) (void)hipHostFree(s.h_verdicts);
  if (s.h_rule_ids) (void)hipHostFree(s.h_rule_ids);
  if (s.h_pack) (void)hipHostFree(s.h_pack);
  if (s.d_frames) (void)hipFree(s.d_frames);
  if (s.d_offsets) (void)hipFree(s.d_offsets);
  if (s.d_lens) (void)hipFree(s.d_lens);
  if (s.d_in_port) (void)hipFree(s.d_in_port);
  if (s.d_verdicts) (void)hipFree(s.d_verdicts);
  if (s.d_rule_ids) (void)hipFree(s.d_rule_ids);
  if (s.done) (void)hipEventDestroy(s.done);
  s = Slot{};
}

bool alloc_slot(Slot &s, const pcn_ipt_ring_config &c) {
  const size_t f = c.slot_frames;
  bool ok = hipHostMalloc(reinterpret_cast<void **>(&s.h_frames), c.slot_bytes, hipHostMallocDefault) == hipSuccess &&
            hipHostMalloc(reinterpret_cast<void **>(&s.h_offsets), 4 * f, hipHostMallocDefault) == hipSuccess &&
            hipHostMalloc(reinterpret_cast<void **>(&s.h_lens), 2 * f, hipHostMallocDefault) == hipSuccess &&
            hipHostMalloc(reinterpret_cast<void **>(&s.h_in_port), 2 * f, hipHostMallocDefault) == hipSuccess &&
            hipHostMalloc(reinterpret_cast<void **>(&s.h_verdicts), f, hipHostMallocDefault) == hipSuccess &&
            hipMalloc(reinterpret_cast<void **>(&s.d_verdicts), f) == hipSuccess &&
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
  if (ok && (c.flags & PCN_IPT_RING_ZERO_COPY)) {
    // the kernel reads the pinned buffers themselves, through their device addresses
    ok = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.z_frames), s.h_frames, 0) == hipSuccess &&
         hipHostGetDevicePointer(reinterpret_cast<void **>(&s.z_offsets), s.h_offsets, 0) == hipSuccess &&
         hipHostGetDevicePointer(reinterpret_cast<void **>(&s.z_lens), s.h_lens, 0) == hipSuccess &&
         hipHostGetDevicePointer(reinterpret_cast<void **>(&s.z_in_port), s.h_in_port, 0) == hipSuccess;
  } else if (ok) {
    ok = hipMalloc(reinterpret_cast<void **>(&s.d_frames), c.slot_bytes) == hipSuccess &&
         hipMalloc(reinterpret_cast<void **>(&s.d_offsets), 4 * f) == hipSuccess &&
         hipMalloc(reinterpret_cast<void **>(&s.d_lens), 2 * f) == hipSuccess &&
         hipMalloc(reinterpret_cast<void **>(&s.d_in_port), 2 * f) == hipSuccess;
  }
  if (ok && (c.flags & PCN_IPT_RING_RULE_IDS))
    ok = hipHostMalloc(reinterpret_cast<void **>(&s.h_rule_ids), 4 * f, hipHostMallocDefault) == hipSuccess &&
         hipMalloc(reinterpret_cast<void **>(&s.d_rule_ids), 4 * f) == hipSuccess;
  return ok;
}

}  // namespace

extern "C" {

int pcn_ipt_ring_create(pcn_ipt *ctx, const pcn_ipt_ring_config *cfg, pcn_ipt_ring **out) {
  if (!ctx || !cfg || !out) return ring_fail(-EINVAL, "null argument");
  *out = nullptr;
  const int device = pcn::device_of(ctx);
  if (device < 0) return ring_fail(-ENODEV, "context has no HIP device (created with device=-1)");
  if (cfg->slots < 2 || cfg->slot_frames == 0 || cfg->slot_bytes == 0)
    return ring_fail(-EINVAL, "need >= 2 slots of >= 1 frame and >= 1 byte");
  if (cfg->flags & ~uint32_t(PCN_IPT_RING_RULE_IDS | PCN_IPT_RING_ZERO_COPY | PCN_IPT_RING_HOST_PACK))
    return ring_fail(-EINVAL, "unknown ring flags");
  if ((cfg->flags & PCN_IPT_RING_ZERO_COPY) && (cfg->flags & PCN_IPT_RING_HOST_PACK))
    return ring_fail(-EINVAL, "PCN_IPT_RING_HOST_PACK packs for a copy: not with PCN_IPT_RING_ZERO_COPY");
  if (cfg->pack_threads > 64) return ring_fail(-EINVAL, "pack_threads > 64");
  if (hipSetDevice(device) != hipSuccess) return ring_fail(-ENODEV, "hipSetDevice failed");
  auto *r = new pcn_ipt_ring();
  r->ctx = ctx;
  r->device = device;
  r->cfg = *cfg;
  if (!r->cfg.streams || r->cfg.streams > r->cfg.slots) r->cfg.streams = r->cfg.slots;
  r->slots.resize(r->cfg.slots);
  bool ok = true;
  for (auto &s : r->slots) ok = ok && alloc_slot(s, r->cfg);
  for (uint32_t k = 0; ok && k < r->cfg.streams; ++k) {
    hipStream_t st = nullptr;
    ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
    if (ok) r->streams.push_back(st);
  }
  if (!ok) {
    (void)hipGetLastError();
    pcn_ipt_ring_destroy(r);
    return ring_fail(-ENOMEM, "ring allocation failed (pinned host or device memory)");
  }
  if (r->cfg.flags & PCN_IPT_RING_HOST_PACK) {
    if (!r->cfg.pack_threads) r->cfg.pack_threads = 8;
    r->pack = std::make_unique<PackPool>(r->cfg.pack_threads - 1);   // + the submitting thread
  }
  *out = r;
  return 0;
}

void pcn_ipt_ring_destroy(pcn_ipt_ring *r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  for (hipStream_t st : r->streams) (void)hipStreamSynchronize(st);
  for (auto &s : r->slots) free_slot(s);
  // the context keeps a record of every stream that carried a batch (its
  // counter-copy bookkeeping): drop ours before the handles die
  for (hipStream_t st : r->streams) (void)pcn_ipt_release_stream(r->ctx, st);
  for (hipStream_t st : r->streams) (void)hipStreamDestroy(st);
  delete r;
}

int pcn_ipt_ring_acquire(pcn_ipt_ring *r, pcn_ipt_ring_slot *out) {
  if (!r || !out) return ring_fail(-EINVAL, "null argument");
  std::lock_guard<std::mutex> l(r->mu);
  for (uint32_t k = 0; k < r->slots.size(); ++k) {
    Slot &s = r->slots[k];
    if (s.state != kFree) continue;
    s.state = kFilling;
    out->slot = k;
    out->frames = s.h_frames;
    out->offsets = s.h_offsets;
    out->lens = s.h_lens;
    out->in_port = s.h_in_port;
    return 0;
  }
  return ring_fail(-EAGAIN, "every slot is in flight or not yet released");
}

int pcn_ipt_ring_submit(pcn_ipt_ring *r, uint32_t slot, const pcn_ipt_ring_batch *b) {
  if (!r || !b) return ring_fail(-EINVAL, "null argument");
  std::unique_lock<std::mutex> l(r->mu);
  if (slot >= r->slots.size() || r->slots[slot].state != kFilling) return ring_fail(-EINVAL, "slot not acquired");
  Slot &s = r->slots[slot];
  if (b->n > r->cfg.slot_frames) return ring_fail(-EINVAL, "more frames than the slot holds");
  const uint64_t bytes = b->frames_bytes ? b->frames_bytes : b->n * uint64_t(b->stride);
  if (bytes > r->cfg.slot_bytes) return ring_fail(-EINVAL, "frame bytes exceed the slot");
  const uint32_t hb = b->hdr_bytes;
  const uint32_t skip = b->hdr_skip;
  const bool zc = r->cfg.flags & PCN_IPT_RING_ZERO_COPY;
  if (hb && zc) return ring_fail(-EINVAL, "hdr_bytes with a zero-copy ring (the kernel reads only the headers anyway)");
  if (skip && !hb) return ring_fail(-EINVAL, "hdr_skip needs a header-only transfer (hdr_bytes)");
  if (skip != 0 && skip != 12) return ring_fail(-EINVAL, "hdr_skip must be 0 or 12 (the Ethernet addresses)");
  if (hb) {
    pcn_ipt_ct_info ci{};
    const bool ct = pcn_ipt_ct_get_info(r->ctx, &ci) == 0 && ci.enabled;
    const uint32_t need = ct ? 80u : b->hook == PCN_IPT_HOOK_TC ? 64u : 48u;
    if (b->use_offsets) return ring_fail(-EINVAL, "a header-only transfer needs a fixed stride");
    if (hb % 16 || hb > b->stride || hb < need)
      return ring_fail(-EINVAL, "hdr_bytes must be a multiple of 16, <= stride and >= " + std::to_string(need));
    if (skip && ct) return ring_fail(-EINVAL, "hdr_skip with the connection table on");
    if (skip && kSkipPad + b->n * uint64_t(hb - skip) > r->cfg.slot_bytes)
      return ring_fail(-EINVAL, "hdr_skip: the packed rows exceed the slot");
  }
  const uint32_t rw = hb - skip;   // bytes of a frame that cross PCIe (header-only transfers)
  uint8_t *const d_rows = s.d_frames + (skip ? kSkipPad : 0);
  if (hipSetDevice(r->device) != hipSuccess) return ring_fail(-ENODEV, "hipSetDevice failed");
  const auto t_submit = std::chrono::steady_clock::now();
  uint64_t pack_ns = 0;
  hipStream_t st = r->streams[slot % r->streams.size()];
  const size_t n = b->n;
  // PCIe in: frames (or their first hb bytes: a strided copy, hb-byte rows
  // packed on the device) and the per-frame arrays the batch uses
  bool ok = true;
  if (hb && r->pack && n) {
    // host pack: the windows into contiguous pinned rows (the slot's last
    // copy out of them was queued on this slot's stream: wait for it first)
    if (s.pack_cap < n * rw) {
      if (hipStreamSynchronize(st) != hipSuccess) return ring_fail(-EIO, "hipStreamSynchronize failed");
      if (s.h_pack) (void)hipHostFree(s.h_pack);
      s.h_pack = nullptr;
      s.pack_cap = 0;
      if (hipHostMalloc(reinterpret_cast<void **>(&s.h_pack), size_t(r->cfg.slot_frames) * hb, hipHostMallocDefault) !=
          hipSuccess)
        return ring_fail(-ENOMEM, "pinned pack buffer");
      s.pack_cap = size_t(r->cfg.slot_frames) * hb;
    } else if (hipEventSynchronize(s.done) != hipSuccess) {   // (a released slot: its copies are done already)
      return ring_fail(-EIO, "hipEventSynchronize failed");
    }
    const uint8_t *src = s.h_frames + skip;
    uint8_t *dst = s.h_pack;
    const uint32_t stride = b->stride;
    const unsigned parts = r->cfg.pack_threads * 4;
    const size_t per = ((n + parts - 1) / parts + 3) / 4 * 4;   // (whole groups of four rows)
    // the slot is the producer's (kFilling): the consumer's complete / release
    // need not wait for the pack
    l.unlock();
    const auto t_pack = std::chrono::steady_clock::now();
    r->pack->run([&](unsigned k) {
      const size_t lo = std::min<size_t>(n, k * per), hi = std::min<size_t>(n, lo + per);
      pack_rows(dst + lo * rw, src + lo * stride, hi - lo, rw, stride);
    }, parts);
    pack_ns = static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_pack).count());
    l.lock();
    ok = hipMemcpyAsync(d_rows, s.h_pack, n * rw, hipMemcpyHostToDevice, st) == hipSuccess;
  } else if (!zc) {
    ok = hb ? hipMemcpy2DAsync(d_rows, rw, s.h_frames + skip, b->stride, rw, n, hipMemcpyHostToDevice, st) == hipSuccess
            : hipMemcpyAsync(s.d_frames, s.h_frames, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
  }
  if (!zc) {   // the per-frame arrays the batch uses
    if (ok && b->use_offsets) ok = hipMemcpyAsync(s.d_offsets, s.h_offsets, 4 * n, hipMemcpyHostToDevice, st) == hipSuccess;
    if (ok && b->use_lens) ok = hipMemcpyAsync(s.d_lens, s.h_lens, 2 * n, hipMemcpyHostToDevice, st) == hipSuccess;
    if (ok && b->use_in_port) ok = hipMemcpyAsync(s.d_in_port, s.h_in_port, 2 * n, hipMemcpyHostToDevice, st) == hipSuccess;
  }
  // a failed submit leaves the slot kFilling (the caller may release and
  // refill it): wait until nothing queued on the stream still reads it
  auto quiesce = [&](int code, const std::string &msg) {
    (void)hipStreamSynchronize(st);
    (void)hipGetLastError();
    return ring_fail(code, msg);
  };
  if (!ok) return quiesce(-EIO, "hipMemcpyAsync (H2D) failed");
  pcn_ipt_batch batch{};
  // (hdr_skip: frame i starts 12 bytes before its row, in the previous row or the pad)
  batch.frames = zc ? s.z_frames : d_rows - skip;
  batch.frames_bytes = hb ? skip + n * rw : bytes;
  batch.offsets = b->use_offsets ? (zc ? s.z_offsets : s.d_offsets) : nullptr;
  batch.lens = b->use_lens ? (zc ? s.z_lens : s.d_lens) : nullptr;
  batch.stride = hb ? rw : b->stride;
  batch.fixed_len = b->fixed_len;
  batch.in_port = b->use_in_port ? (zc ? s.z_in_port : s.d_in_port) : nullptr;
  batch.const_in_port = b->const_in_port;
  batch.direction = b->direction;
  batch.hook = b->hook;
  batch.n = n;
  batch.verdicts = s.d_verdicts;
  batch.rule_ids = s.d_rule_ids;
  if (n) {
    const int rc = pcn_ipt_classify(r->ctx, &batch, st);
    if (rc) return quiesce(rc, std::string("classify: ") + pcn_ipt_last_error());
  }
  // PCIe out: verdicts (and rule ids)
  ok = hipMemcpyAsync(s.h_verdicts, s.d_verdicts, n, hipMemcpyDeviceToHost, st) == hipSuccess;
  if (ok && s.d_rule_ids) ok = hipMemcpyAsync(s.h_rule_ids, s.d_rule_ids, 4 * n, hipMemcpyDeviceToHost, st) == hipSuccess;
  if (ok) ok = hipEventRecord(s.done, st) == hipSuccess;
  if (!ok) return quiesce(-EIO, "hipMemcpyAsync (D2H) / hipEventRecord failed");
  s.n = n;
  s.state = kInFlight;
  r->inflight.push_back(slot);
  pcn_ipt_ring_stats &rs = r->stats;
  rs.submits += 1;
  rs.frames += n;
  const uint64_t arrays = (b->use_offsets ? 4 : 0) + (b->use_lens ? 2 : 0) + (b->use_in_port ? 2 : 0);
  if (zc) rs.zc_bytes += n * (64 + arrays);
  else rs.h2d_bytes += (hb ? n * rw : bytes) + n * arrays;
  rs.d2h_bytes += n * (s.d_rule_ids ? 5 : 1);
  rs.pack_ns += pack_ns;
  rs.submit_ns += static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_submit).count());
  return 0;
}

int pcn_ipt_ring_get_stats(pcn_ipt_ring *r, pcn_ipt_ring_stats *out, int reset) {
  if (!r || !out) return ring_fail(-EINVAL, "null argument");
  std::lock_guard<std::mutex> l(r->mu);
  *out = r->stats;
  if (reset) r->stats = pcn_ipt_ring_stats{};
  return 0;
}

int pcn_ipt_ring_complete(pcn_ipt_ring *r, int wait, uint32_t *slot, uint64_t *n, const uint8_t **verdicts,
                          const int32_t **rule_ids) {
  if (!r) return ring_fail(-EINVAL, "null ring");
  uint32_t k;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> l(r->mu);
    if (r->inflight.empty()) return ring_fail(-ENOENT, "nothing in flight");
    k = r->inflight.front();
    ev = r->slots[k].done;
  }
  if (hipSetDevice(r->device) != hipSuccess) return ring_fail(-ENODEV, "hipSetDevice failed");
  if (wait) {
    if (hipEventSynchronize(ev) != hipSuccess) return ring_fail(-EIO, "hipEventSynchronize failed");
  } else {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipErrorNotReady) return ring_fail(-EAGAIN, "oldest slot still in flight");
    if (q != hipSuccess) return ring_fail(-EIO, "hipEventQuery failed");
  }
  std::lock_guard<std::mutex> l(r->mu);
  r->inflight.pop_front();
  Slot &s = r->slots[k];
  s.state = kReturned;
  if (slot) *slot = k;
  if (n) *n = s.n;
  if (verdicts) *verdicts = s.h_verdicts;
  if (rule_ids) *rule_ids = s.h_rule_ids;
  return 0;
}

int pcn_ipt_ring_release(pcn_ipt_ring *r, uint32_t slot) {
  if (!r) return ring_fail(-EINVAL, "null ring");
  std::lock_guard<std::mutex> l(r->mu);
  if (slot >= r->slots.size() || (r->slots[slot].state != kReturned && r->slots[slot].state != kFilling))
    return ring_fail(-EINVAL, "slot is not held by the caller");
  r->slots[slot].state = kFree;
  return 0;
}

}  // extern "C"
