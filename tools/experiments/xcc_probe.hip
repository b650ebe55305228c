// Round-5 probe: the hardware XCC id (s_getreg HW_REG_XCC_ID) of each workgroup of a 1,024-workgroup launch --
// its histogram and how often it equals blockIdx.x % 8 (the round-robin dealing the pool's shards assume).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) o[blockIdx.x] = x;
}
int main() {
  unsigned* d = nullptr;
  unsigned h[1024];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1024), dim3(512), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  int hist[16] = {0}, same = 0;
  for (int i = 0; i < 1024; ++i) {
    hist[h[i] & 15]++;
    same += (int)((h[i] & 7) == (unsigned)(i % 8));
  }
  printf("raw[0..9]: ");
  for (int i = 0; i < 10; ++i) printf("%#x ", h[i]);
  printf("\nhistogram (low 4 bits):");
  for (int i = 0; i < 16; ++i) printf(" %d", hist[i]);
  printf("\nxcc == block %% 8: %d of 1024\n", same);
  return 0;
}
