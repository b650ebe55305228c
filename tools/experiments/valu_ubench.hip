// VALU issue-rate microbenchmark for gfx950 (MI355X).
//
// Measures wave64 instruction throughput of the integer ops a BLAKE2b round
// can be built from, at full occupancy (8 waves/SIMD), each thread running
// 16 independent dependency chains so issue rate, not latency, is measured.
// Reports lane-ops per clock per CU (at the in-kernel clock, from
// s_memtime / s_memrealtime) and chip-wide Gops/s.  Used to pin the VALU
// roofline peak in DESIGN.md (SURVEY.md §8(d) "confirm lanes/clk with a
// v_xor_b32 throughput microbenchmark on the box").
//
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_ubench valu_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

enum Op { XOR32, ALIGNBIT, ADDCO_PAIR, LSHL_ADD_U64, BITOP3, PERM, ADD3, LSHR_B64, ADD_U32, FMA_F32, PK_FMA_F32, XOR_SDWA, LSHR_B32, LSHL_OR, ALIGNBYTE, PK_MOV, XOR_SGPR, XAD, BFI, DPP, LSHL_ADD_U32, MIX_ALIGN_XOR, XOR_ADD_ALT, XOR_DEP, OR32, LSHL32, XOR_LSHR_ALT, XOR_LIT, XOR_INLINE, AL2_XOR2, XOR_E64, XOR_SGPR_SRC1, CNDMASK, SUB32, XOR4_SAME, BITOP3_OR, ADD64_XOR2, N_OPS };
static const char* kNames[N_OPS] = {"v_xor_b32", "v_alignbit_b32", "v_add_co_u32+v_addc_co_u32", "v_lshl_add_u64", "v_bitop3_b32", "v_perm_b32", "v_add3_u32", "v_lshrrev_b64", "v_add_u32", "v_fma_f32", "v_pk_fma_f32 (64-bit)", "v_xor_b32_sdwa WORD preserve", "v_lshrrev_b32", "v_lshl_or_b32", "v_alignbyte_b32", "v_pk_mov_b32 swap", "v_xor_b32 (sgpr src)", "v_xad_u32", "v_bfi_b32", "v_mov_b32_dpp", "v_lshl_add_u32", "alignbit+xor alternating", "xor,add_u32 alternating", "xor dependent pair", "v_or_b32", "v_lshlrev_b32", "xor,lshrrev alternating", "v_xor_b32 literal", "v_xor_b32 inline const", "2 alignbit + 2 xor", "v_xor_b32_e64 vgprs", "v_xor_b32_e64 v, v, s", "v_cndmask_b32", "v_sub_u32", "4 xor same reg pair chain-free", "bitop3 or-of-shifted? (0xfe)", "lshl_add_u64 + 2 xor"};
// instructions issued per asm unit (one unit per i step of 2)
static const int kInsPerUnit[N_OPS] = {2, 2, 2, 1, 2, 2, 2, 1, 2, 2, 1, 2, 2, 2, 2, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 4, 2, 2, 2, 2, 4, 2, 3};

template <int OP>
__global__ __launch_bounds__(256, 8) void ubench(uint32_t* out, int iters, uint32_t k, uint32_t ks,
                                                 unsigned long long* clk) {
  uint32_t r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i + blockIdx.x;
  uint64_t t0 = 0, rt0 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      if constexpr (OP == XOR32) {
        asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == ALIGNBIT) {
        asm volatile("v_alignbit_b32 %0, %0, %2, 24\n\tv_alignbit_b32 %1, %1, %2, 16" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == ADDCO_PAIR) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k) : "vcc");
      } else if constexpr (OP == LSHL_ADD_U64) {
        uint64_t a = ((uint64_t)r[i + 1] << 32) | r[i]; uint64_t b = ((uint64_t)k << 32) | k; asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a) : "v"(b)); r[i] = (uint32_t)a; r[i + 1] = (uint32_t)(a >> 32);
      } else if constexpr (OP == BITOP3) {
        asm volatile("v_bitop3_b32 %0, %0, %2, %1 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %0 bitop3:0x96" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == PERM) {
        asm volatile("v_perm_b32 %0, %0, %2, %2\n\tv_perm_b32 %1, %1, %2, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == ADD3) {
        asm volatile("v_add3_u32 %0, %0, %2, %2\n\tv_add3_u32 %1, %1, %2, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == LSHR_B64) {
        uint64_t a = ((uint64_t)r[i + 1] << 32) | r[i]; asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(a)); r[i] = (uint32_t)a; r[i + 1] = (uint32_t)(a >> 32);
      } else if constexpr (OP == ADD_U32) {
        asm volatile("v_add_u32 %0, %0, %2\n\tv_add_u32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == FMA_F32) {
        asm volatile("v_fma_f32 %0, %0, %2, %2\n\tv_fma_f32 %1, %1, %2, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == PK_FMA_F32) {
        uint64_t a = ((uint64_t)r[i + 1] << 32) | r[i]; uint64_t b = ((uint64_t)k << 32) | k; asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(b)); r[i] = (uint32_t)a; r[i + 1] = (uint32_t)(a >> 32);
      } else if constexpr (OP == XOR_SDWA) {
        asm volatile("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n\tv_xor_b32_sdwa %1, %0, %2 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == LSHR_B32) {
        asm volatile("v_lshrrev_b32 %0, 3, %0\n\tv_lshrrev_b32 %1, 5, %1" : "+v"(r[i]), "+v"(r[i + 1]) :);
      } else if constexpr (OP == LSHL_OR) {
        asm volatile("v_lshl_or_b32 %0, %0, 8, %2\n\tv_lshl_or_b32 %1, %1, 8, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == ALIGNBYTE) {
        asm volatile("v_alignbyte_b32 %0, %0, %2, 3\n\tv_alignbyte_b32 %1, %1, %2, 2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == PK_MOV) {
        uint64_t a = ((uint64_t)r[i + 1] << 32) | r[i]; asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(a)); r[i] = (uint32_t)a; r[i + 1] = (uint32_t)(a >> 32);
      } else if constexpr (OP == XOR_SGPR) {
        asm volatile("v_xor_b32 %0, %2, %0\n\tv_xor_b32 %1, %2, %1" : "+v"(r[i]), "+v"(r[i + 1]) : "s"(ks));
      } else if constexpr (OP == XAD) {
        asm volatile("v_xad_u32 %0, %0, %2, %1\n\tv_xad_u32 %1, %1, %2, %0" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == BFI) {
        asm volatile("v_bfi_b32 %0, %0, %2, %1\n\tv_bfi_b32 %1, %1, %2, %0" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == DPP) {
        asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r[i]), "+v"(r[i + 1]) :);
      } else if constexpr (OP == LSHL_ADD_U32) {
        asm volatile("v_lshl_add_u32 %0, %0, 1, %2\n\tv_lshl_add_u32 %1, %1, 1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == MIX_ALIGN_XOR) {
        asm volatile("v_alignbit_b32 %0, %0, %2, 24\n\tv_xor_b32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == XOR_ADD_ALT) {
        asm volatile("v_xor_b32 %0, %0, %2\n\tv_add_u32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == XOR_DEP) {
        asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == OR32) {
        asm volatile("v_or_b32 %0, %0, %2\n\tv_or_b32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == LSHL32) {
        asm volatile("v_lshlrev_b32 %0, 3, %0\n\tv_lshlrev_b32 %1, 5, %1" : "+v"(r[i]), "+v"(r[i + 1]) :);
      } else if constexpr (OP == XOR_LSHR_ALT) {
        asm volatile("v_xor_b32 %0, %0, %2\n\tv_lshrrev_b32 %1, 5, %1" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == XOR_LIT) {
        asm volatile("v_xor_b32 %0, 0x12345678, %0\n\tv_xor_b32 %1, 0x9abcdef1, %1" : "+v"(r[i]), "+v"(r[i + 1]) :);
      } else if constexpr (OP == XOR_INLINE) {
        asm volatile("v_xor_b32 %0, 7, %0\n\tv_xor_b32 %1, -3, %1" : "+v"(r[i]), "+v"(r[i + 1]) :);
      } else if constexpr (OP == AL2_XOR2) {
        asm volatile("v_alignbit_b32 %0, %0, %2, 24\n\tv_alignbit_b32 %1, %1, %2, 24\n\tv_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == XOR_E64) {
        asm volatile("v_xor_b32_e64 %0, %0, %2\n\tv_xor_b32_e64 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == XOR_SGPR_SRC1) {
        asm volatile("v_xor_b32_e64 %0, %0, %2\n\tv_xor_b32_e64 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "s"(ks));
      } else if constexpr (OP == CNDMASK) {
        asm volatile("v_cndmask_b32 %0, %0, %2, vcc\n\tv_cndmask_b32 %1, %1, %2, vcc" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == SUB32) {
        asm volatile("v_sub_u32 %0, %0, %2\n\tv_sub_u32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == XOR4_SAME) {
        asm volatile("v_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2\n\tv_xor_b32 %0, %0, %1\n\tv_xor_b32 %1, %1, %2" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == BITOP3_OR) {
        asm volatile("v_bitop3_b32 %0, %0, %2, %1 bitop3:0xfe\n\tv_bitop3_b32 %1, %1, %2, %0 bitop3:0xfe" : "+v"(r[i]), "+v"(r[i + 1]) : "v"(k));
      } else if constexpr (OP == ADD64_XOR2) {
        uint64_t a = ((uint64_t)r[i + 1] << 32) | r[i]; uint64_t b = ((uint64_t)k << 32) | k; uint32_t x0 = r[(i + 2) & 15], x1 = r[(i + 3) & 15]; asm volatile("v_lshl_add_u64 %0, %0, 0, %3\n\tv_xor_b32 %1, %1, %4\n\tv_xor_b32 %2, %2, %4" : "+v"(a), "+v"(x0), "+v"(x1) : "v"(b), "v"(k)); r[i] = (uint32_t)a; r[i + 1] = (uint32_t)(a >> 32); r[(i + 2) & 15] = x0; r[(i + 3) & 15] = x1;
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - rt0;
  }
}

template <int OP>
static void run(int cus, uint32_t* d_out, unsigned long long* d_clk, int iters) {
  const int blocks = cus * 8, threads = 256;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  // warmup (also lets the clock settle)
  for (int w = 0; w < 3; ++w) ubench<OP><<<blocks, threads>>>(d_out, iters, 0x9e3779b9u, 0x7f4a7c15u, d_clk);
  CHECK(hipDeviceSynchronize());
  const int reps = 5;
  CHECK(hipEventRecord(a));
  for (int w = 0; w < reps; ++w) ubench<OP><<<blocks, threads>>>(d_out, iters, 0x9e3779b9u, 0x7f4a7c15u, d_clk);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms, a, b));
  unsigned long long clk[2];
  CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
  double ghz = (double)clk[0] / (double)clk[1] * 0.1;  // s_memrealtime ticks at 100 MHz
  double wave_ins = (double)blocks * (threads / 64) * iters * 8.0 * kInsPerUnit[OP] * reps;
  double lane_ops = wave_ins * 64.0;
  double s = ms * 1e-3;
  double lane_ops_per_clk_cu = lane_ops / s / (ghz * 1e9) / cus;
  printf("{\"op\": \"%s\", \"gops_per_s\": %.1f, \"clock_ghz\": %.3f, \"lane_ops_per_clk_per_cu\": %.2f, "
         "\"cycles_per_wave_ins_per_simd\": %.3f, \"ms\": %.3f}\n",
         kNames[OP], lane_ops / s * 1e-9, ghz, lane_ops_per_clk_cu, 4.0 * 64.0 / lane_ops_per_clk_cu, ms / reps);
  CHECK(hipEventDestroy(a)); CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 4096;
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  printf("{\"device\": \"%s\", \"gcn_arch\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.name, p.gcnArchName, cus, p.clockRate);
  uint32_t* d_out; unsigned long long* d_clk;
  CHECK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4));
  CHECK(hipMalloc(&d_clk, 16));
  run<XOR32>(cus, d_out, d_clk, iters);
  run<ALIGNBIT>(cus, d_out, d_clk, iters);
  run<ADDCO_PAIR>(cus, d_out, d_clk, iters);
  run<LSHL_ADD_U64>(cus, d_out, d_clk, iters);
  run<BITOP3>(cus, d_out, d_clk, iters);
  run<PERM>(cus, d_out, d_clk, iters);
  run<ADD3>(cus, d_out, d_clk, iters);
  run<LSHR_B64>(cus, d_out, d_clk, iters);
  run<ADD_U32>(cus, d_out, d_clk, iters);
  run<FMA_F32>(cus, d_out, d_clk, iters);
  run<PK_FMA_F32>(cus, d_out, d_clk, iters);
  run<XOR_SDWA>(cus, d_out, d_clk, iters);
  run<LSHR_B32>(cus, d_out, d_clk, iters);
  run<LSHL_OR>(cus, d_out, d_clk, iters);
  run<ALIGNBYTE>(cus, d_out, d_clk, iters);
  run<PK_MOV>(cus, d_out, d_clk, iters);
  run<XOR_SGPR>(cus, d_out, d_clk, iters);
  run<XAD>(cus, d_out, d_clk, iters);
  run<BFI>(cus, d_out, d_clk, iters);
  run<DPP>(cus, d_out, d_clk, iters);
  run<LSHL_ADD_U32>(cus, d_out, d_clk, iters);
  run<MIX_ALIGN_XOR>(cus, d_out, d_clk, iters);
  run<XOR_ADD_ALT>(cus, d_out, d_clk, iters);
  run<XOR_DEP>(cus, d_out, d_clk, iters);
  run<OR32>(cus, d_out, d_clk, iters);
  run<LSHL32>(cus, d_out, d_clk, iters);
  run<XOR_LSHR_ALT>(cus, d_out, d_clk, iters);
  run<XOR_LIT>(cus, d_out, d_clk, iters);
  run<XOR_INLINE>(cus, d_out, d_clk, iters);
  run<AL2_XOR2>(cus, d_out, d_clk, iters);
  run<XOR_E64>(cus, d_out, d_clk, iters);
  run<XOR_SGPR_SRC1>(cus, d_out, d_clk, iters);
  run<CNDMASK>(cus, d_out, d_clk, iters);
  run<SUB32>(cus, d_out, d_clk, iters);
  run<XOR4_SAME>(cus, d_out, d_clk, iters);
  run<BITOP3_OR>(cus, d_out, d_clk, iters);
  run<ADD64_XOR2>(cus, d_out, d_clk, iters);
  run<XOR32>(cus, d_out, d_clk, iters);
  CHECK(hipFree(d_out)); CHECK(hipFree(d_clk));
  return 0;
}
