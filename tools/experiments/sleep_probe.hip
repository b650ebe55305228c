// Round-5 probe: how long s_sleep N takes on gfx950 (s_memrealtime, 100 MHz) for a few N, one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int N>
__global__ void k(unsigned long long* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 100; ++i) __builtin_amdgcn_s_sleep(N);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}
template <int N>
void run(unsigned long long* d) {
  unsigned long long h = 0;
  hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
  printf("s_sleep %3d: %.3f us each\n", N, h / 10000.0);
}
int main() {
  unsigned long long* d = nullptr;
  if (hipMalloc(&d, 8) != hipSuccess) return 1;
  run<1>(d); run<1>(d); run<8>(d); run<16>(d); run<32>(d); run<64>(d); run<127>(d);
  return 0;
}
