// Second VALU microbenchmark round (gfx950): candidate rotation sequences for the hash stream,
// plus an exhaustive bit-exactness check of v_pack_b32_f16 used as a 16-bit half shuffle.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_ubench2 valu_ubench2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

// Each op body updates r[i], r[i+1] (32-bit) and may use z (a zero VGPR) and k.
#define OPS(X) \
  X(XOR, 2, "v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2") \
  X(PACK_F16, 2, "v_pack_b32_f16 %0, %0, %2 op_sel:[1,0]\n\tv_pack_b32_f16 %1, %1, %2 op_sel:[1,0]") \
  X(MOV_SDWA, 2, "v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n\tv_mov_b32_sdwa %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0") \
  X(LSHL32_7, 2, "v_lshlrev_b32 %0, 7, %0\n\tv_lshlrev_b32 %1, 7, %1") \
  X(LSHL32_E64, 2, "v_lshlrev_b32_e64 %0, 7, %0\n\tv_lshlrev_b32_e64 %1, 7, %1") \
  X(LSHR32, 2, "v_lshrrev_b32 %0, 7, %0\n\tv_lshrrev_b32 %1, 7, %1") \
  X(AND_OR, 2, "v_and_or_b32 %0, %0, %2, %1\n\tv_and_or_b32 %1, %1, %2, %0") \
  X(PK_LSHL16, 2, "v_pk_lshlrev_b16 %0, 8, %0\n\tv_pk_lshlrev_b16 %1, 8, %1") \
  X(CVT_PK_U16, 2, "v_cvt_pk_u16_u32 %0, %0, %2\n\tv_cvt_pk_u16_u32 %1, %1, %2") \
  X(ALIGNBIT, 2, "v_alignbit_b32 %0, %0, %2, 24\n\tv_alignbit_b32 %1, %1, %2, 16") \
  X(SWAP, 1, "v_swap_b32 %0, %1") \
  X(MOV, 2, "v_mov_b32 %0, %1\n\tv_mov_b32 %1, %2")

enum Op {
#define E(name, n, s) name,
  OPS(E)
#undef E
  ROTL1_LSHLADD, ROTL1_ALIGN, ROT16_PACK, ROT16_ALIGN, N_OPS
};
static const char* kNames[N_OPS] = {
#define E(name, n, s) #name,
  OPS(E)
#undef E
  "ROTL1 via lshrrev+lshl_add_u64 {t,0} (2 ins)", "ROTL1 via 2 alignbit (2 ins)",
  "ROT16 via 2 v_pack_b32_f16 (2 ins)", "ROT16 via 2 alignbit (2 ins)"};
static const int kIns[N_OPS] = {
#define E(name, n, s) n,
  OPS(E)
#undef E
  2, 2, 2, 2};

template <int OP>
__global__ __launch_bounds__(256, 8) void ub(uint32_t* out, int iters, uint32_t k, unsigned long long* clk) {
  uint32_t r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i + blockIdx.x;
  if constexpr (OP == ROTL1_LSHLADD) asm volatile("v_mov_b32 v61, 0" ::: "v61");
  uint64_t t0 = 0, rt0 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); rt0 = __builtin_amdgcn_s_memrealtime(); }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
#define E(name, n, s) if constexpr (OP == name) { asm volatile(s : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k)); }
      OPS(E)
#undef E
      if constexpr (OP == ROTL1_LSHLADD) {
        // x = {r[i], r[i+1]}; t = hi >> 31 into the low half of a {t, 0} pair; x' = (x << 1) + {t,0}
        uint64_t x = ((uint64_t)r[i + 1] << 32) | r[i];
        // v61 holds 0 (set before the loop); t goes to v60 so {v60, v61} = x >> 63
        asm volatile("v_lshrrev_b32 v60, 31, %1\n\tv_lshl_add_u64 %0, %0, 1, v[60:61]" : "+v"(x) : "v"(r[i + 1]) : "v60");
        r[i] = (uint32_t)x; r[i + 1] = (uint32_t)(x >> 32);
      } else if constexpr (OP == ROTL1_ALIGN) {
        uint32_t a, b;
        asm volatile("v_alignbit_b32 %2, %0, %1, 31\n\tv_alignbit_b32 %3, %1, %0, 31" : "+v"(r[i]), "+v"(r[i + 1]), "=&v"(a), "=&v"(b));
        r[i] = a; r[i + 1] = b;
      } else if constexpr (OP == ROT16_PACK) {
        uint32_t a, b;
        asm volatile("v_pack_b32_f16 %2, %0, %1 op_sel:[1,0]\n\tv_pack_b32_f16 %3, %1, %0 op_sel:[1,0]" : "+v"(r[i]), "+v"(r[i + 1]), "=&v"(a), "=&v"(b));
        r[i] = a; r[i + 1] = b;
      } else if constexpr (OP == ROT16_ALIGN) {
        uint32_t a, b;
        asm volatile("v_alignbit_b32 %2, %1, %0, 16\n\tv_alignbit_b32 %3, %0, %1, 16" : "+v"(r[i]), "+v"(r[i + 1]), "=&v"(a), "=&v"(b));
        r[i] = a; r[i + 1] = b;
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - rt0; }
}

template <int OP>
static void run(int cus, uint32_t* d_out, unsigned long long* d_clk, int iters) {
  const int blocks = cus * 8, threads = 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) ub<OP><<<blocks, threads>>>(d_out, iters, 0x9e3779b9u, d_clk);
  CHECK(hipDeviceSynchronize());
  const int reps = 5;
  CHECK(hipEventRecord(a));
  for (int w = 0; w < reps; ++w) ub<OP><<<blocks, threads>>>(d_out, iters, 0x9e3779b9u, d_clk);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  unsigned long long clk[2];
  CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
  double ghz = (double)clk[0] / (double)clk[1] * 0.1;
  double wave_ins = (double)blocks * (threads / 64) * iters * 8.0 * kIns[OP] * reps;
  double lane_ops_per_clk_cu = wave_ins * 64.0 / (ms * 1e-3) / (ghz * 1e9) / cus;
  printf("{\"op\": \"%s\", \"clock_ghz\": %.3f, \"cycles_per_wave_ins_per_simd\": %.3f, \"ms\": %.3f}\n",
         kNames[OP], ghz, 256.0 / lane_ops_per_clk_cu, ms / reps);
}

// exhaustive: v_pack_b32_f16 D, S0, S1 op_sel:[1,0] == (S1.lo16 << 16) | S0.hi16 for every 16-bit pattern
__global__ void pack_check(unsigned int* bad, uint32_t salt) {
  const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;  // 0 .. 2^32-1 over the grid-stride loop
  for (uint64_t v = x; v < (1ull << 32); v += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t s0 = ((uint32_t)v & 0xffff0000u) | ((salt * 2654435761u + (uint32_t)v) & 0xffffu);
    const uint32_t s1 = ((uint32_t)v & 0x0000ffffu) | (((salt ^ (uint32_t)v) * 40503u) << 16);
    uint32_t d;
    asm volatile("v_pack_b32_f16 %0, %1, %2 op_sel:[1,0]" : "=v"(d) : "v"(s0), "v"(s1));
    const uint32_t want = (s1 << 16) | (s0 >> 16);
    if (d != want) atomicAdd(bad, 1u);
  }
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 32768;
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  uint32_t* d_out; unsigned long long* d_clk; unsigned int* d_bad;
  CHECK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4));
  CHECK(hipMalloc(&d_clk, 16));
  CHECK(hipMalloc(&d_bad, 4));
  CHECK(hipMemset(d_bad, 0, 4));
  pack_check<<<cus * 16, 256>>>(d_bad, 12345u);
  unsigned int bad = 0;
  CHECK(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
  printf("{\"pack_b32_f16_exhaustive_2^32_mismatches\": %u}\n", bad);
#define R(name, n, s) run<name>(cus, d_out, d_clk, iters);
  OPS(R)
#undef R
  run<ROTL1_LSHLADD>(cus, d_out, d_clk, iters);
  run<ROTL1_ALIGN>(cus, d_out, d_clk, iters);
  run<ROT16_PACK>(cus, d_out, d_clk, iters);
  run<ROT16_ALIGN>(cus, d_out, d_clk, iters);
  return 0;
}
