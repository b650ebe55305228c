// wave_probe.cpp -- diagnostic: per-wave timing of one npow_pool_kernel launch (kernel built with
// -DNPOW_WAVE_PROBE).  Prints the spread of wave start / end times and of iteration rates per XCD
// and per SIMD, to see whether a full launch ends with a slow tail.
// Build: hipcc -O3 --offload-arch=gfx950 -Inano-dpow_amd/csrc -Iinclude -x hip tools/experiments/wave_probe.cpp
//        -o build/wave_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#define NPOW_WAVE_PROBE 1
#include "npow_kernel.hip"  // one translation unit: the probe array is a device global of the kernel

using namespace npow;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
  const uint32_t iters = argc > 1 ? atoi(argv[1]) : 256;
  const uint32_t budget_us = argc > 2 ? atoi(argv[2]) : 0;
  const int bpc = argc > 3 ? atoi(argv[3]) : 8;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int grid = p.multiProcessorCount * bpc;
  const uint32_t W = grid * 4;
  PoolDevState* pst; CK(hipMalloc(&pst, sizeof(PoolDevState))); CK(hipMemset(pst, 0, sizeof(PoolDevState)));
  PoolMailbox* pmb; CK(hipHostMalloc((void**)&pmb, sizeof(PoolMailbox), hipHostMallocCoherent | hipHostMallocMapped));
  memset(pmb, 0, sizeof(PoolMailbox));
  PoolMailbox* pmbd; CK(hipHostGetDevicePointer((void**)&pmbd, pmb, 0));
  uint8_t root[32]; for (int i = 0; i < 32; ++i) root[i] = i;
  PoolTable h{}; h.n = 1; h.poll_mask = 1023; h.iters = iters; h.budget = budget_us * 100;
  npow_asm_uniforms(host_precompute(root).m, h.e[0].u);
  h.e[0].threshold = ~0ull; h.e[0].count = (uint64_t)W * 64 * iters; h.e[0].gen = 1;
  PoolTable* t; CK(hipMalloc(&t, sizeof(PoolTable))); CK(hipMemcpy(t, &h, sizeof(h), hipMemcpyHostToDevice));
  std::vector<uint64_t> pr((size_t)W * 4);
  for (int rep = 0; rep < 3; ++rep) {
    CK(launch_pool(grid, 0, t, false, pst, pmbd));
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(npow_wave_probe), pr.size() * 8));
  uint64_t s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
  std::map<int, std::vector<double>> rate_xcc, rate_simd;
  std::vector<double> rates, ends;
  for (uint32_t w = 0; w < W; ++w) {
    const uint64_t st = pr[w * 4], en = pr[w * 4 + 1], it = pr[w * 4 + 2], id = pr[w * 4 + 3];
    s0 = std::min(s0, st); s1 = std::max(s1, st); e0 = std::min(e0, en); e1 = std::max(e1, en);
    const double r = (double)it / ((en - st) * 1e-8);  // iterations per second (realtime 100 MHz)
    rates.push_back(r);
    rate_xcc[(int)(id >> 32) & 0xf].push_back(r);
    rate_simd[(int)((uint32_t)id >> 4) & 3].push_back(r);
  }
  for (uint32_t w = 0; w < W; ++w) ends.push_back((pr[w * 4 + 1] - s0) * 1e-2);  // us after first start
  std::sort(rates.begin(), rates.end()); std::sort(ends.begin(), ends.end());
  printf("{\"blocks_per_cu\": %d, \"iters\": %u, \"budget_us\": %u, \"start_spread_us\": %.1f, \"end_spread_us\": %.1f, "
         "\"launch_us\": %.1f, \"end_p01_us\": %.1f, \"end_p50_us\": %.1f, \"end_p99_us\": %.1f, "
         "\"rate_min\": %.1f, \"rate_p50\": %.1f, \"rate_max\": %.1f",
         bpc, iters, budget_us, (s1 - s0) * 1e-2, (e1 - e0) * 1e-2, (e1 - s0) * 1e-2, ends[W / 100], ends[W / 2],
         ends[W * 99 / 100], rates.front(), rates[W / 2], rates.back());
  printf(", \"rate_by_xcc\": {");
  for (auto& kv : rate_xcc) {
    double m = 0; for (double x : kv.second) m += x;
    printf("\"%d\": %.1f, ", kv.first, m / kv.second.size());
  }
  printf("\"n\": %zu}, \"rate_by_simd\": {", rate_xcc.size());
  for (auto& kv : rate_simd) {
    double m = 0; for (double x : kv.second) m += x;
    printf("\"%d\": %.1f, ", kv.first, m / kv.second.size());
  }
  printf("\"n\": %zu}", rate_simd.size());
  // placement: waves per (xcc, se, sh, cu) and how many started late (> 500 us after the first)
  std::map<uint64_t, int> per_cu, late_cu;
  for (uint32_t w = 0; w < W; ++w) {
    const uint64_t id = pr[w * 4 + 3];
    const uint32_t hw = (uint32_t)id;
    const uint64_t key = ((id >> 32) & 0xf) << 16 | ((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 0xf);
    per_cu[key]++;
    if (pr[w * 4] - s0 > 50000) late_cu[key]++;
  }
  std::map<int, int> hist;
  for (auto& kv : per_cu) hist[kv.second]++;
  printf(", \"cus_seen\": %zu, \"waves_per_cu_hist\": {", per_cu.size());
  for (auto& kv : hist) printf("\"%d\": %d, ", kv.first, kv.second);
  int late = 0; for (auto& kv : late_cu) late += kv.second;
  printf("\"x\": 0}, \"late_waves\": %d, \"cus_with_late\": %zu}\n", late, late_cu.size());
  return 0;
}
