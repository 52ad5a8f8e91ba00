// jit.hpp — per-chain "chain programs": the classify kernel recompiled with one
// chain's table-image layout baked in as constants.
//
// The reference builds every datapath module from C text in which the control
// plane has substituted the chain's sizes and constants (_NR_ELEMENTS,
// _DEFAULTACTION, _WILDCARD_*, next-hop indices; modules/Program.cpp:23-119,
// modules/L4PortLookup.cpp:62-105) and compiles it with bcc on every chain
// update (Chain.cpp:431-929).  Here the same idea targets gfx950: the chain
// image's offsets, word counts, field set and search depths become immediates
// of classify.hip compiled by hiprtc, so the kernel needs no SGPRs (and no SGPR
// spills) for them and its loops over words and search steps fully unroll.
// Compiles run on a background thread; until a program is ready (or if the
// compile fails) the generic variant of the same kernel runs.
#pragma once
#include <cstdint>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "devchain.h"

namespace pcn {

// The launch shape a chain program is specialised for.
struct JitShape {
  bool fixed = true;   // fixed-stride 16-B-aligned frames
  bool lds = true;     // chain images staged in LDS
  int ch = 1;          // the one chain that runs rules (0..2)
  int ns = 5;          // class slots
  int inputs = 0;      // bit 0: per-frame in_port array, bit 1: per-frame ct_status array
  bool shallow = false;   // fixed stride, at most 8 frames per lane: header prefetch depth 1
  bool deal2 = false;     // two candidates per worker lane (a chain of 2+ summary blocks; the launch
                          // sized the wave region for the 128-candidate window)
  bool split = false;     // a split launch: gather kernel + rule kernel (classify.hip SPLIT)
};

// Source of the generated "pcn_jit_spec.h" for one chain descriptor (its
// pointers are ignored); doubles as the cache key.
std::string jit_spec(const DevChain &d, const JitShape &s);

// Resources of a compiled chain program, from its code object's metadata.
struct ProgramMeta {
  int vgpr = -1, agpr = -1, sgpr = -1, vgpr_spill = -1, sgpr_spill = -1;
  int scratch = -1;       // .private_segment_fixed_size (bytes per lane)
  int static_lds = -1;    // .group_segment_fixed_size
  uint32_t code_bytes = 0;
  bool hdr_asm = true;    // built with the counted asm header loads (else rebuilt without, jit.cpp compile)
};

class JitCache {
 public:
  JitCache() = default;
  ~JitCache();
  JitCache(const JitCache &) = delete;
  JitCache &operator=(const JitCache &) = delete;

  // Start compiling `spec` unless it is known; blocking waits for the result.
  void request(const std::string &spec, bool blocking);
  // The kernel (hipFunction_t) for `spec` on the current device, or null when
  // it is absent, still compiling or failed.  Loads the module on first use.
  // which = 1: a split program's second kernel (pcn_split_rules), null otherwise.
  void *function(const std::string &spec, int device, int which = 0);
  // Compiled successfully (false while compiling or after a failure).
  bool ready(const std::string &spec) const;
  // 1 and *out filled when compiled, 0 while compiling or never requested, -1 failed.
  int meta(const std::string &spec, ProgramMeta *out) const;
  // Programs compiled / failed so far (diagnostics).
  int compiled() const;
  int failed() const;
  std::string last_log() const;

 private:
  struct Entry {
    // empty vector: compile failed; the last byte says whether the counted asm
    // header loads were kept (1) or the program was rebuilt without (0)
    std::shared_future<std::vector<char>> code;
    struct Loaded {
      void *mod = nullptr, *fn = nullptr, *fn2 = nullptr;   // hipModule_t, pcn_classify_jit, pcn_split_rules
    };
    std::map<int, Loaded> loaded;   // by device
    bool bad = false;
  };
  mutable std::mutex mu_;
  std::map<std::string, std::shared_ptr<Entry>> entries_;
  std::string last_log_;
};

}  // namespace pcn
