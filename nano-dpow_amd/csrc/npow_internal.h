// npow_internal.h -- structures shared by the gfx950 kernels and the host engine.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "npow_blake2b.h"

namespace npow {

constexpr int kBlock = 256;  // lanes per workgroup (4 waves of 64)

enum class Mode : int { kSearch = 0, kSweep = 1, kValues = 2 };

// Kernel arguments, passed by value: the kernarg segment lands in SGPRs, so the
// root words, the round-1 constants and the threshold cost no memory traffic
// per nonce (SURVEY.md §7 "Uniform data in SGPRs").
struct LaunchArgs {
  RootPrecomp pre;     // 128 B: root words + nonce-independent round-1 state
  uint64_t threshold;  // valid iff value >= threshold
  uint64_t base;       // first nonce of this launch (wraps mod 2^64)
  uint64_t count;      // nonces in this launch (lane index i < count)
  uint32_t poll_mask;  // a wave polls the host abort word when (iter & poll_mask) == 0
  uint32_t cap;        // sweep: capacity of the hit buffer
};

// Device-resident per-task state (hipMalloc; reset by hipMemsetAsync per task).
struct DevState {
  uint32_t found;           // first-win slot: 0 -> 1 by atomicCAS (search)
  uint32_t n_hits;          // sweep: hits appended (may exceed cap)
  uint64_t nonce;           // winning nonce (search)
  uint64_t value;           // winning value (search)
  unsigned long long done;  // nonces hashed (all launches of the task)
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
hipError_t launch_pairs(int grid, hipStream_t stream, const uint64_t* roots_words, const uint64_t* nonces,
                        uint32_t n, uint64_t* out);

}  // namespace npow
