// Diagnostic: throughput AND in-kernel shader clock of the generated hash stream
// (nano-dpow_amd/csrc/npow_hash_asm.inc) in a bare grid-stride loop, to tell an
// issue-bound kernel from a clock-limited one (MI355X_MICROARCH.md "DVFS give-back" item 6:
// clock = d(s_memtime) / d(s_memrealtime) x 100 MHz, median over workgroups).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../nano-dpow_amd/csrc -o hash_clock hash_clock.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "npow_hash_asm.inc"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

struct Args { uint64_t u[NPOW_ASM_N_UNIFORMS]; uint64_t base; int iters; };

__global__ __launch_bounds__(256) void hash_loop(const Args a, uint64_t* out, unsigned long long* stamps) {
  uint64_t u[NPOW_ASM_N_UNIFORMS];
#pragma unroll
  for (int i = 0; i < NPOW_ASM_N_UNIFORMS; ++i) u[i] = a.u[i];
  const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t nonce = a.base + gid, acc = 0;
  unsigned long long t0 = 0, r0 = 0;
  if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < a.iters; ++it) {
    acc ^= npow_asm_work_value(nonce, u);
    nonce += stride;
  }
  out[gid] = acc;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 256;
  const int bpc = argc > 2 ? atoi(argv[2]) : 8;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount * bpc;
  Args a{};
  const uint64_t m[4] = {0x0706050403020100ull, 0x0f0e0d0c0b0a0908ull, 0x1716151413121110ull, 0x1f1e1d1c1b1a1918ull};
  npow_asm_uniforms(m, a.u);
  a.base = 1ull << 50;
  a.iters = iters;
  uint64_t* d_out; unsigned long long* d_st;
  CHECK(hipMalloc(&d_out, (size_t)grid * 256 * 8));
  CHECK(hipMalloc(&d_st, (size_t)grid * 16));
  for (int w = 0; w < 5; ++w) hash_loop<<<grid, 256>>>(a, d_out, d_st);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hash_loop<<<grid, 256>>>(a, d_out, d_st);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> st((size_t)grid * 2);
  CHECK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> ghz;
  for (int b = 0; b < grid; ++b) ghz.push_back((double)st[2 * b] / (double)st[2 * b + 1] * 0.1);
  std::sort(ghz.begin(), ghz.end());
  const double nonces = (double)grid * 256 * iters * reps;
  const double gnps = nonces / (ms * 1e-3) / 1e9;
  const double clk = ghz[ghz.size() / 2];
  // SIMD cycles per wave iteration (64 nonces) implied by throughput at the measured clock
  const double cyc = p.multiProcessorCount * 4.0 * clk * 1e9 * 64.0 / (gnps * 1e9);
  printf("{\"iters\": %d, \"blocks_per_cu\": %d, \"gnps\": %.3f, \"clock_ghz_median\": %.3f, \"clock_ghz_min\": %.3f, "
         "\"clock_ghz_max\": %.3f, \"simd_cycles_per_wave_iter\": %.0f, \"ms_per_launch\": %.3f}\n",
         iters, bpc, gnps, clk, ghz.front(), ghz.back(), cyc, ms / reps);
  return 0;
}
