// npow_internal.h -- structures shared by the gfx950 kernels and the host engine.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "npow_blake2b.h"
#include "npow_hash_asm.inc"

namespace npow {

constexpr int kBlock = 256;  // lanes per workgroup (4 waves of 64)

enum class Mode : int { kSearch = 0, kSweep = 1, kValues = 2 };

// Kernel arguments, passed by value: the kernarg segment lands in SGPRs, so the
// root-derived uniforms and the threshold cost no memory traffic per nonce
// (SURVEY.md §7 "Uniform data in SGPRs").
struct LaunchArgs {
  uint64_t u[NPOW_ASM_N_UNIFORMS];  // nonce-independent intermediates (npow_asm_uniforms)
  uint64_t threshold;  // valid iff value >= threshold
  uint64_t base;       // first nonce of this launch (wraps mod 2^64)
  uint64_t count;      // nonces in this launch (lane index i < count)
  uint32_t poll_mask;  // a wave polls the host abort word when (iter & poll_mask) == 0
  uint32_t cap;        // sweep: capacity of the hit buffer
};

// Device-resident per-task state (hipMalloc; reset by hipMemsetAsync per task).
// The nonces-hashed counter is sharded over 256 cache lines: every wave adds its
// count once at exit, and 8,192 waves adding to ONE word serialise at the memory
// side (~12 ns each, MI355X_MICROARCH.md "fanin") -- a ~100 us tail on every launch.
constexpr int kDoneShards = 256;
struct DevState {
  union {
    struct {
      uint32_t found;       // first-win slot: 0 -> 1 by atomicCAS (search)
      uint32_t abort;       // host abort relayed by the wave that saw it
    };
    uint64_t stop;          // both, read by every wave with one 8-byte load
  };
  uint32_t n_hits;          // sweep: hits appended (may exceed cap)
  uint32_t pad0;
  uint64_t nonce;           // winning nonce (search)
  uint64_t value;           // winning value (search)
  uint32_t zero;            // always 0: the non-polling iterations' load target
  uint8_t pad1[64 - 36];
  unsigned long long done_shard[kDoneShards * 8];  // nonces hashed, one counter per 64-byte line
  uint64_t done() const {
    uint64_t s = 0;
    for (int i = 0; i < kDoneShards; ++i) s += done_shard[i * 8];
    return s;
  }
};

// Host-coherent pinned mailbox (hipHostMalloc coherent + mapped).  The winning
// wave publishes here with system-scope stores so the host thread sees a win
// without waiting for the launch to drain; the host raises `abort` to stop
// every wave of every in-flight launch (polled every poll_mask+1 iterations).
struct alignas(64) HostMailbox {
  uint32_t found;
  uint32_t pad0;
  uint64_t nonce;
  uint64_t value;
  uint8_t pad1[64 - 24];
  uint32_t abort;  // on its own cache line
  uint8_t pad2[60];
};

// Launchers (defined in npow_kernel.hip).
hipError_t launch_task(Mode mode, int grid, hipStream_t stream, const LaunchArgs& a, DevState* st,
                       HostMailbox* mb, uint64_t* out);
// Fill a.u[] for one root (host).
inline void fill_uniforms(LaunchArgs& a, const RootPrecomp& pre) { npow_asm_uniforms(pre.m, a.u); }

hipError_t launch_pairs(int grid, hipStream_t stream, const uint64_t* roots_words, const uint64_t* nonces,
                        uint32_t n, uint64_t* out);

}  // namespace npow
