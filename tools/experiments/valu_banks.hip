// valu_banks.hip -- does the VGPR bank of an instruction's operands change its issue cost on
// gfx950?  Streams of 16 independent instructions per iteration with explicit registers:
// each variant fixes the (dst, src0, src1) register numbers mod 4 (the bank, if banks are
// index mod 4).  8 waves/SIMD (256 CUs x 8 blocks x 256 lanes), in-kernel clock.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/valu_banks tools/experiments/valu_banks.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#define CHECK(x)                                                                                     \
  do {                                                                                               \
    hipError_t e = (x);                                                                              \
    if (e != hipSuccess) {                                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);          \
      exit(1);                                                                                       \
    }                                                                                                \
  } while (0)

// Registers v8..v63 are ours (clobbered).  Variant strings are generated at compile time by
// macros below: 16 instructions per iteration.
#define CLOB                                                                                          \
  "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", \
      "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36",  \
      "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50",  \
      "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"

template <int V>
__device__ __forceinline__ void body();

// xor, dst == src0 (in place), src1 from another register: d/s0 bank 0, s1 bank b
#define X4(a, b) "v_xor_b32_e64 v" #a ", v" #a ", v" #b "\n"
// V0: s1 same bank (reg+32)
template <> __device__ __forceinline__ void body<0>() {
  asm volatile(X4(8, 40) X4(12, 44) X4(16, 48) X4(20, 52) X4(24, 56) X4(28, 60) X4(32, 40) X4(36, 44)
               X4(8, 48) X4(12, 52) X4(16, 56) X4(20, 60) X4(24, 40) X4(28, 44) X4(32, 48) X4(36, 52) ::: CLOB);
}
// V1: s1 next bank
template <> __device__ __forceinline__ void body<1>() {
  asm volatile(X4(8, 41) X4(12, 45) X4(16, 49) X4(20, 53) X4(24, 57) X4(28, 61) X4(32, 41) X4(36, 45)
               X4(8, 49) X4(12, 53) X4(16, 57) X4(20, 61) X4(24, 41) X4(28, 45) X4(32, 49) X4(36, 53) ::: CLOB);
}
// V2: three distinct banks: d bank 0, s0 bank 1, s1 bank 2 (not in place)
#define X3(d, a, b) "v_xor_b32_e64 v" #d ", v" #a ", v" #b "\n"
template <> __device__ __forceinline__ void body<2>() {
  asm volatile(X3(8, 41, 42) X3(12, 45, 46) X3(16, 49, 50) X3(20, 53, 54) X3(24, 57, 58) X3(28, 61, 62)
               X3(32, 41, 46) X3(36, 45, 50) X3(8, 49, 54) X3(12, 53, 58) X3(16, 57, 62) X3(20, 61, 42)
               X3(24, 41, 50) X3(28, 45, 54) X3(32, 49, 58) X3(36, 53, 62) ::: CLOB);
}
// V3: all three in the same bank (not in place)
template <> __device__ __forceinline__ void body<3>() {
  asm volatile(X3(8, 40, 44) X3(12, 48, 52) X3(16, 56, 60) X3(20, 40, 48) X3(24, 44, 52) X3(28, 48, 56)
               X3(32, 52, 60) X3(36, 40, 56) X3(8, 44, 60) X3(12, 40, 52) X3(16, 44, 56) X3(20, 48, 60)
               X3(24, 40, 44) X3(28, 48, 52) X3(32, 56, 60) X3(36, 44, 48) ::: CLOB);
}
// lshl_add_u64 d = s0 + s2 (64-bit pairs): V4 pairs in the same banks (s0 v[8+4k], s2 v[40+4k]);
// V5 s2 in the other bank pair (v[42+4k])
#define L(d, a, b) "v_lshl_add_u64 v[" #d ":" #d "+1], v[" #a ":" #a "+1], 0, v[" #b ":" #b "+1]\n"
template <> __device__ __forceinline__ void body<4>() {
  asm volatile(L(8, 8, 40) L(12, 12, 44) L(16, 16, 48) L(20, 20, 52) L(24, 24, 56) L(28, 28, 60)
               L(32, 32, 40) L(36, 36, 44) L(8, 8, 48) L(12, 12, 52) L(16, 16, 56) L(20, 20, 60)
               L(24, 24, 40) L(28, 28, 44) L(32, 32, 48) L(36, 36, 52) ::: CLOB);
}
template <> __device__ __forceinline__ void body<5>() {
  asm volatile(L(8, 8, 42) L(12, 12, 46) L(16, 16, 50) L(20, 20, 54) L(24, 24, 58) L(28, 28, 62)
               L(32, 32, 42) L(36, 36, 46) L(8, 8, 50) L(12, 12, 54) L(16, 16, 58) L(20, 20, 62)
               L(24, 24, 42) L(28, 28, 46) L(32, 32, 50) L(36, 36, 54) ::: CLOB);
}
// alignbit d = align(s0, s1, 24): V6 s0,s1 same bank; V7 different banks; V8 d,s0,s1 3 banks
#define A(d, a, b) "v_alignbit_b32 v" #d ", v" #a ", v" #b ", 24\n"
template <> __device__ __forceinline__ void body<6>() {
  asm volatile(A(8, 40, 44) A(12, 48, 52) A(16, 56, 60) A(20, 40, 48) A(24, 44, 52) A(28, 48, 56)
               A(32, 52, 60) A(36, 40, 56) A(9, 44, 60) A(13, 40, 52) A(17, 44, 56) A(21, 48, 60)
               A(25, 40, 44) A(29, 48, 52) A(33, 56, 60) A(37, 44, 48) ::: CLOB);
}
template <> __device__ __forceinline__ void body<7>() {
  asm volatile(A(8, 41, 42) A(12, 45, 46) A(16, 49, 50) A(20, 53, 54) A(24, 57, 58) A(28, 61, 62)
               A(32, 41, 46) A(36, 45, 50) A(9, 49, 54) A(13, 53, 58) A(17, 57, 62) A(21, 61, 42)
               A(25, 41, 50) A(29, 45, 54) A(33, 49, 58) A(37, 53, 62) ::: CLOB);
}
// V8: mixed realistic G fragment: 2 xor + 2 alignbit + 1 lshl_add, banks arbitrary (as the
// generator allocates today) vs V9: same ops with every instruction's operands in distinct banks
template <> __device__ __forceinline__ void body<8>() {
  asm volatile(X3(10, 40, 44) X3(11, 41, 45) A(12, 11, 10) A(13, 10, 11) L(8, 8, 12)
               X3(14, 48, 52) X3(15, 49, 53) A(16, 15, 14) A(17, 14, 15) L(20, 20, 16)
               X3(22, 56, 60) X3(23, 57, 61) A(24, 23, 22) A(25, 22, 23) L(28, 28, 24)
               X3(30, 40, 48) ::: CLOB);
}
template <> __device__ __forceinline__ void body<9>() {
  asm volatile(X3(10, 41, 46) X3(11, 43, 44) A(12, 11, 10) A(13, 10, 11) L(8, 8, 14)
               X3(18, 49, 54) X3(19, 51, 52) A(16, 19, 18) A(17, 18, 19) L(20, 20, 26)
               X3(30, 57, 62) X3(31, 59, 60) A(32, 31, 30) A(33, 30, 31) L(36, 36, 34)
               X3(38, 41, 50) ::: CLOB);
}

static const char* kNames[] = {
    "xor in-place, s1 same bank", "xor in-place, s1 next bank", "xor d/s0/s1 three banks",
    "xor d/s0/s1 one bank", "lshl_add_u64 pairs same bank pair", "lshl_add_u64 pairs other bank pair",
    "alignbit s0/s1 same bank", "alignbit s0/s1 different banks", "G fragment, banks as allocated",
    "G fragment, operands in distinct banks"};
static const int kNins[] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16};

template <int V>
__global__ __launch_bounds__(256) void ub(int iters, unsigned long long* clk) {
  // seed the registers (values do not matter for issue cost)
  asm volatile(
      "v_mov_b32 v8, v0\n v_mov_b32 v9, v0\n v_mov_b32 v10, v0\n v_mov_b32 v11, v0\n"
      "v_mov_b32 v40, v0\n v_mov_b32 v41, v0\n v_mov_b32 v42, v0\n v_mov_b32 v43, v0\n" ::: CLOB);
  uint64_t t0 = 0, rt0 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
    body<V>();
    body<V>();
    body<V>();
    body<V>();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - rt0;
  }
}

template <int V>
static void run(int cus, unsigned long long* d_clk, int iters) {
  const int blocks = cus * 8, threads = 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  ub<V><<<blocks, threads>>>(iters, d_clk);
  CHECK(hipDeviceSynchronize());
  const int reps = 5;
  CHECK(hipEventRecord(a));
  for (int w = 0; w < reps; ++w) ub<V><<<blocks, threads>>>(iters, d_clk);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  unsigned long long clk[2];
  CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
  const double ghz = (double)clk[0] / (double)clk[1] * 0.1;
  const double wave_ins = (double)blocks * (threads / 64) * iters * 4.0 * kNins[V] * reps;
  const double simd_cycles = (ms * 1e-3) * (ghz * 1e9) * cus * 4;  // SIMD-cycles available
  printf("{\"variant\": \"%s\", \"clock_ghz\": %.3f, \"cycles_per_wave_ins_per_simd\": %.3f}\n", kNames[V], ghz,
         simd_cycles / wave_ins);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 8192;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  unsigned long long* d_clk;
  CHECK(hipMalloc(&d_clk, 16));
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(p.multiProcessorCount, d_clk, iters);
    run<1>(p.multiProcessorCount, d_clk, iters);
    run<2>(p.multiProcessorCount, d_clk, iters);
    run<3>(p.multiProcessorCount, d_clk, iters);
    run<4>(p.multiProcessorCount, d_clk, iters);
    run<5>(p.multiProcessorCount, d_clk, iters);
    run<6>(p.multiProcessorCount, d_clk, iters);
    run<7>(p.multiProcessorCount, d_clk, iters);
    run<8>(p.multiProcessorCount, d_clk, iters);
    run<9>(p.multiProcessorCount, d_clk, iters);
  }
  return 0;
}
