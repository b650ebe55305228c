// cu_mask_probe.hip -- where do the workgroups of a CU-masked stream (hipExtStreamCreateWithCUMask) run
// on the MI355X?  For each mask layout, 4 masked streams (one per quarter of the CUs) each launch
// 4 x popcount(mask) 512-lane workgroups that spin for a fixed wall time; every workgroup records its
// XCC_ID, HW_ID (SE / SH / CU) and start / end s_memrealtime.  Prints, per stream: the distinct
// (xcc, se, sh, cu) it ran on, per-XCD CU counts, and whether its workgroups were all resident at once;
// then whether the 4 streams' CU sets are disjoint and whether their kernels overlapped in time.
// Build: hipcc --offload-arch=gfx950 -O2 -o build/cu_mask_probe tools/experiments/cu_mask_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

struct Rec {
  uint32_t xcc, hwid;
  uint64_t t0, t1;
};

__global__ __launch_bounds__(512) void probe(Rec* out, uint64_t spin_ticks) {
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  uint64_t t = t0;
  while (t - t0 < spin_ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[blockIdx.x].xcc = xcc;
    out[blockIdx.x].hwid = hwid;
    out[blockIdx.x].t0 = t0;
    out[blockIdx.x].t1 = t;
  }
}

int main(int argc, char** argv) {
  const int ndev = argc > 1 ? atoi(argv[1]) : 4;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("CUs %d, logical devices %d\n", cus, ndev);
  // layouts: "block" = CUs [d*cus/ndev, (d+1)*cus/ndev); "stride" = CU i where i % ndev == d
  for (int layout = 0; layout < 2; ++layout) {
    const char* lname = layout == 0 ? "block" : "stride";
    std::vector<hipStream_t> st(ndev);
    std::vector<int> pop(ndev, 0);
    for (int d = 0; d < ndev; ++d) {
      std::vector<uint32_t> mask((cus + 31) / 32, 0);
      for (int i = 0; i < cus; ++i) {
        const bool on = layout == 0 ? (i * ndev / cus == d) : (i % ndev == d);
        if (on) {
          mask[i / 32] |= 1u << (i % 32);
          ++pop[d];
        }
      }
      CHECK(hipExtStreamCreateWithCUMask(&st[d], (uint32_t)mask.size(), mask.data()));
    }
    std::vector<Rec*> dbuf(ndev);
    std::vector<int> grid(ndev);
    for (int d = 0; d < ndev; ++d) {
      grid[d] = 4 * pop[d];
      CHECK(hipMalloc(&dbuf[d], grid[d] * sizeof(Rec)));
      CHECK(hipMemset(dbuf[d], 0, grid[d] * sizeof(Rec)));
    }
    CHECK(hipDeviceSynchronize());
    for (int d = 0; d < ndev; ++d) hipLaunchKernelGGL(probe, dim3(grid[d]), dim3(512), 0, st[d], dbuf[d], 200000ull);  // 2 ms
    CHECK(hipDeviceSynchronize());
    std::vector<std::set<std::tuple<int, int, int, int>>> sets(ndev);
    std::vector<uint64_t> first(ndev, ~0ull), last(ndev, 0), last_start(ndev, 0);
    for (int d = 0; d < ndev; ++d) {
      std::vector<Rec> h(grid[d]);
      CHECK(hipMemcpy(h.data(), dbuf[d], grid[d] * sizeof(Rec), hipMemcpyDeviceToHost));
      std::map<int, std::set<std::tuple<int, int, int>>> per_xcc;
      std::map<int, int> wg_per_xcc;
      for (const Rec& r : h) {
        const int cu = (r.hwid >> 8) & 15, sh = (r.hwid >> 12) & 1, se = (r.hwid >> 13) & 7;
        sets[d].insert({(int)r.xcc & 15, se, sh, cu});
        per_xcc[r.xcc & 15].insert({se, sh, cu});
        wg_per_xcc[r.xcc & 15]++;
        first[d] = std::min(first[d], r.t0);
        last[d] = std::max(last[d], r.t1);
        last_start[d] = std::max(last_start[d], r.t0);
      }
      printf("%s d%d mask CUs %d grid %d: distinct CUs %zu; per XCD (CUs/wgs):", lname, d, pop[d], grid[d], sets[d].size());
      for (auto& kv : per_xcc) printf(" x%d:%zu/%d", kv.first, kv.second.size(), wg_per_xcc[kv.first]);
      printf("; start spread %.1f us, span %.1f us\n", (last_start[d] - first[d]) / 100.0, (last[d] - first[d]) / 100.0);
    }
    bool disjoint = true;
    for (int a = 0; a < ndev; ++a)
      for (int b = a + 1; b < ndev; ++b)
        for (auto& x : sets[a])
          if (sets[b].count(x)) disjoint = false;
    const uint64_t f0 = *std::min_element(first.begin(), first.end());
    printf("%s: disjoint %s; kernel starts relative to the first (us):", lname, disjoint ? "yes" : "NO");
    for (int d = 0; d < ndev; ++d) printf(" %.1f", (first[d] - f0) / 100.0);
    printf("; ends:");
    for (int d = 0; d < ndev; ++d) printf(" %.1f", (last[d] - f0) / 100.0);
    printf("\n");
    for (int d = 0; d < ndev; ++d) {
      CHECK(hipFree(dbuf[d]));
      CHECK(hipStreamDestroy(st[d]));
    }
  }
  return 0;
}
