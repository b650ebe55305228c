// kernel_direct_bench.cpp -- launch the search kernels directly (no engine / pool host logic)
// with a never-hit threshold and time them with HIP events on their stream, interleaved:
//   task  = npow_task_kernel<kSweep> (kernel-argument uniforms, one root; no hits)
//   pool1 = npow_pool_kernel<false> with one unbounded entry
//   pool8 = npow_pool_kernel<false> with eight unbounded entries
// Build: hipcc -O3 --offload-arch=gfx950 -Inano-dpow_amd/csrc -Iinclude -x hip tools/experiments/kernel_direct_bench.cpp
//        -x none nano-dpow_amd/csrc/npow_kernel.o -o build/kernel_direct_bench
// Run:   ./build/kernel_direct_bench [reps] [iters] [poll_mask] [gap_us] [blocks_per_cu]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>

#include "npow_internal.h"

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

using namespace npow;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 256;
  const uint32_t pmask = argc > 3 ? (uint32_t)atoi(argv[3]) : 1023;  // host-word poll mask
  const int gap_us = argc > 4 ? atoi(argv[4]) : 0;                      // host sleep between launches
  const int bpc = argc > 5 ? atoi(argv[5]) : 8;                          // workgroups per CU
  CK(hipSetDevice(0));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount * bpc;
  const uint64_t W = (uint64_t)grid * (kBlock / 64);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  DevState* st;
  CK(hipMalloc(&st, sizeof(DevState)));
  CK(hipMemset(st, 0, sizeof(DevState)));
  HostMailbox* mb;
  CK(hipHostMalloc((void**)&mb, sizeof(HostMailbox), hipHostMallocCoherent | hipHostMallocMapped));
  memset(mb, 0, sizeof(HostMailbox));
  HostMailbox* mbd;
  CK(hipHostGetDevicePointer((void**)&mbd, mb, 0));
  PoolDevState* pst;
  CK(hipMalloc(&pst, sizeof(PoolDevState)));
  CK(hipMemset(pst, 0, sizeof(PoolDevState)));
  PoolMailbox* pmb;
  CK(hipHostMalloc((void**)&pmb, sizeof(PoolMailbox), hipHostMallocCoherent | hipHostMallocMapped));
  memset(pmb, 0, sizeof(PoolMailbox));
  PoolMailbox* pmbd;
  CK(hipHostGetDevicePointer((void**)&pmbd, pmb, 0));

  uint8_t root[32];
  for (int i = 0; i < 32; ++i) root[i] = (uint8_t)(i * 7 + 1);
  const RootPrecomp pre = host_precompute(root);
  LaunchArgs a{};
  fill_uniforms(a, pre);
  a.threshold = ~0ull;
  a.poll_mask = pmask;
  a.count = W * 64 * iters;
  a.max_claim = 64;

  PoolTable* tabs[2];
  for (int k = 0; k < 2; ++k) {
    PoolTable h{};
    const uint32_t n = k == 0 ? 1 : 8;
    h.n = n;
    h.poll_mask = pmask;
    h.iters = iters;
    for (uint32_t e = 0; e < n; ++e) {
      npow_asm_uniforms(pre.m, h.e[e].u);
      h.e[e].threshold = ~0ull;
      h.e[e].base = (uint64_t)e << 50;
      h.e[e].count = W * 64 * iters;
      h.e[e].gen = 1;
      h.e[e].slot = e;
      h.e[e].bounded = 0;
    }
    CK(hipMalloc(&tabs[k], sizeof(PoolTable)));
    CK(hipMemcpy(tabs[k], &h, sizeof(PoolTable), hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"task", "pool1", "pool8"};
  double tot[3] = {0, 0, 0};
  for (int r = 0; r < reps; ++r) {
    for (int v = 0; v < 3; ++v) {
      CK(hipEventRecord(e0, s));
      if (v == 0) {
        a.claim_slot = (uint32_t)r & 1;
        CK(launch_task(Mode::kSweep, grid, s, a, st, mbd, nullptr));
      } else {
        CK(launch_pool(grid, s, tabs[v - 1], false, pst, pmbd));
      }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      if (gap_us > 0) usleep(gap_us);
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) tot[v] += ms;
    }
  }
  const double nonces = (double)W * 64 * iters;
  for (int v = 0; v < 3; ++v) {
    const double ms = tot[v] / (reps - 1);
    printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"gnps\": %.4f}\n", names[v], ms, nonces / (ms * 1e-3) / 1e9);
  }
  return 0;
}
