// npow_kernel.hip -- gfx950 (MI355X / CDNA4) kernels of the Nano proof-of-work engine.
//
// Replaces the OpenCL kernel `nano_work` + inline `blake2b()` embedded in the
// reference work server (client/bin/windows/nano-work-server.exe @1657474..1661900).
// Written from the BLAKE2b definition for the gfx950 VALU, not translated:
//
//  * The per-nonce hash is a generated instruction stream (tools/gen_hash_asm.py): one nonce per
//    lane, the 16-word state in a fixed VGPR window, 12 rounds unrolled with the message schedule
//    resolved at generation time (11 of 16 message words are zero).  Every nonce-independent
//    intermediate (round 1's three column steps and more) is computed once per root on the host.
//    Round 12's dead half is removed.
//  * 64-bit adds are single `v_lshl_add_u64` instructions (half rate, 4 SIMD cycles for the whole
//    add; the v_add_co/v_addc carry pair serialises the wave on VCC -- DESIGN.md section 4).
//  * Rotations are split into 32-bit halves: rotr32 is a free register swap folded into the xor
//    that feeds it, rotr24 / rotr16 / rotr63 are two `v_alignbit_b32` each.
//  * The shipped stream, npow_hash_asm_lockstep_ld.inc, is scheduled in intervals (the full-rate
//    part of one G step -- xors --, then the half-rate part of the next -- its alignbits, then its 64-bit
//    adds: adds last runs the same cycles at a ~1 % higher power-limited clock)
//    and loads the root's uniforms into SGPRs itself.  A gfx950 SIMD issues a full-rate
//    instruction of one wave in the shadow of another wave's v_alignbit_b32, but only when the
//    alignbit's wave wins arbitration first: the stream raises its wave's priority (s_setprio 1)
//    for each half-rate run and drops it for each full-rate run, so the 8 waves of a SIMD interleave
//    their runs (round 3, DESIGN.md section 4: -9 % SIMD cycles per hash).  Every kernel that runs it
//    (search, sweep, values) has four 512-lane workgroups per CU (8 waves per SIMD), and every
//    loop decision is a workgroup decision.
//  * First-win search (npow_pool_kernel_ls2*): every live job of the device's work pool in one
//    launch; first win per job by atomicMax on its slot's dead word, published to a host-coherent
//    mailbox with system-scope stores; the host kill / yield words are polled by one wave in
//    poll_mask+1 per iteration; a launch ends on a wall-clock budget read from s_memrealtime.
//  * Sweep (npow_sweep_kernel_ls2): workgroups claim rows of blocks from 8 per-XCD counters; every
//    hit appended through an atomic counter (order-free; the host sorts).
//  * Values (npow_values_kernel_ls2): every value of a range through the same stream (parity); a
//    second, independently scheduled stream (npow_hash_asm.inc, no barriers) backs
//    npow_values_kernel_seq, and npow_pairs_kernel is plain C++ (per-lane roots).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "npow_internal.h"

namespace npow {

// ---- 64-bit rotations on 32-bit halves --------------------------------------------------
__device__ __forceinline__ uint64_t pack(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

__device__ __forceinline__ uint64_t rotr32(uint64_t x) {  // register swap, no instruction
  return pack((uint32_t)(x >> 32), (uint32_t)x);
}
template <int N>  // 0 < N < 32
__device__ __forceinline__ uint64_t rotr_lt32(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_alignbit(hi, lo, N), __builtin_amdgcn_alignbit(lo, hi, N));
}
__device__ __forceinline__ uint64_t rotr63(uint64_t x) {  // = rotl 1
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return pack(__builtin_amdgcn_alignbit(lo, hi, 31), __builtin_amdgcn_alignbit(hi, lo, 31));
}

// ---- message words: m0 = nonce, m1..m4 = root, the rest zero (resolved at compile time) --
template <int I>
__device__ __forceinline__ uint64_t add_msg(uint64_t a, uint64_t nonce, const uint64_t (&m)[4]) {
  if constexpr (I == 0) return a + nonce;
  else if constexpr (I <= 4) return a + m[I - 1];
  else return a;
}

template <int X, int Y>
__device__ __forceinline__ void G(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, uint64_t n,
                                  const uint64_t (&m)[4]) {
  a = add_msg<X>(a, n, m) + b;
  d = rotr32(d ^ a);
  c = c + d;
  b = rotr_lt32<24>(b ^ c);
  a = add_msg<Y>(a, n, m) + b;
  d = rotr_lt32<16>(d ^ a);
  c = c + d;
  b = rotr63(b ^ c);
}

template <int R>
__device__ __forceinline__ void columns(uint64_t (&v)[16], uint64_t n, const uint64_t (&m)[4]) {
  G<kSigma[R][0], kSigma[R][1]>(v[0], v[4], v[8], v[12], n, m);
  G<kSigma[R][2], kSigma[R][3]>(v[1], v[5], v[9], v[13], n, m);
  G<kSigma[R][4], kSigma[R][5]>(v[2], v[6], v[10], v[14], n, m);
  G<kSigma[R][6], kSigma[R][7]>(v[3], v[7], v[11], v[15], n, m);
}
template <int R>
__device__ __forceinline__ void diagonals(uint64_t (&v)[16], uint64_t n, const uint64_t (&m)[4]) {
  G<kSigma[R][8], kSigma[R][9]>(v[0], v[5], v[10], v[15], n, m);
  G<kSigma[R][10], kSigma[R][11]>(v[1], v[6], v[11], v[12], n, m);
  G<kSigma[R][12], kSigma[R][13]>(v[2], v[7], v[8], v[13], n, m);
  G<kSigma[R][14], kSigma[R][15]>(v[3], v[4], v[9], v[14], n, m);
}

template <int R>
__device__ __forceinline__ void rounds_from(uint64_t (&v)[16], uint64_t n, const uint64_t (&m)[4]) {
  if constexpr (R < 12) {
    columns<R>(v, n, m);
    diagonals<R>(v, n, m);
    rounds_from<R + 1>(v, n, m);
  }
}

// Generic work value (per-lane root): all 12 rounds on the GPU.
__device__ __forceinline__ uint64_t work_value_full(uint64_t nonce, const uint64_t (&m)[4]) {
  uint64_t v[16] = {kH0, kIV1, kIV2, kIV3, kIV4, kIV5, kIV6, kIV7,
                    kIV0, kIV1, kIV2, kIV3, kV12, kIV5, kV14, kIV7};
  rounds_from<0>(v, nonce, m);
  return kH0 ^ v[0] ^ v[8];
}

__device__ __forceinline__ uint64_t uni64(uint64_t x) {  // a wave-uniform value, in SGPRs
  return pack(__builtin_amdgcn_readfirstlane((uint32_t)x), __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)));
}
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)x, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
  return pack(lo, hi);
}

// ---- Values through the seq stream (npow_values_kernel_seq) ---------------------------------
// The second hash path: npow_hash_asm.inc (the same DAG, list-scheduled without barriers, uniforms
// as asm operands), 256-lane workgroups, static grid-stride mapping.
__global__ __launch_bounds__(kBlock) void npow_values_kernel_seq(const LaunchArgs a, DevState* __restrict__ st,
                                                                 uint64_t* __restrict__ out) {
  uint64_t u[NPOW_ASM_N_UNIFORMS];  // the compiler keeps kernel arguments in SGPRs
#pragma unroll
  for (int i = 0; i < NPOW_ASM_N_UNIFORMS; ++i) u[i] = a.u[i];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave0 = (uint64_t)__builtin_amdgcn_readfirstlane(blockIdx.x * kBlock + (threadIdx.x & ~63u));
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  uint64_t done = 0;
  for (uint64_t ib = wave0; ib < a.count; ib += stride) {
    const uint64_t i = ib + lane;
    const uint64_t value = npow_asm_work_value(a.base + i, u);
    if (i < a.count) out[i] = value;
    const uint64_t rem = a.count - ib;
    done += rem < 64 ? rem : 64;
  }
  if (lane == 0 && done) atomicAdd(&st->done_shard[(blockIdx.x % kDoneShards) * 8], (unsigned long long)done);
}

// ---- Sweep (npow_sweep_kernel_ls2) -----------------------------------------------------------
// Every hit of [base, base + count): four 512-lane workgroups per CU.  The unit of work is a row of
// kLsWaves (8) consecutive 64-nonce blocks, one per wave (block = row * kLsWaves + wave); workgroups claim runs of
// rows from 8 per-XCD counters (thread 0 claims and LDS broadcasts the claim: two barriers per claim
// of <= max_claim rows), and the stop words (the device abort word, and the pinned host abort word on
// one claim in poll_mask + 1) are read with the claim, so a cancel lands within one claim (<= 64
// rows, ~0.15 ms).  Blocks past the range's end are masked off.
//
// Why claims: VALU issue favours a SIMD's oldest wave, so with fixed shares the
// young workgroups finish late and the launch ends in a tail; claiming keeps every SIMD full until
// the range is used up.  The launch's rows are split into 8 sub-ranges with one counter each on its
// own cache line (atomics on ONE address serialise at ~18 ns); a workgroup starts on its XCD's
// sub-range (workgroups are dealt to XCDs round-robin) and then helps the others.  Claim size =
// remaining / (2 x workgroups per sub-range), between 1 and max_claim.  The counters alternate by
// launch parity: launch k claims from claim[k & 1][*] and zeroes claim[(k + 1) & 1][*].
__global__ __launch_bounds__(kLsBlock, 8) void npow_sweep_kernel_ls2(const LaunchArgs a, DevState* __restrict__ st,
                                                                    HostMailbox* __restrict__ mb,
                                                                    uint64_t* __restrict__ out) {
  __shared__ uint32_t s_claim[3];  // first row, end row (within the sub-range), stop
  const uint64_t* up = ((const LaunchArgs*)__builtin_amdgcn_kernarg_segment_ptr())->u;  // loaded by the stream
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t g = blockIdx.x;
  const uint32_t slot = a.claim_slot & 1;
  if (g == 0 && threadIdx.x < kClaimRanges)
    __hip_atomic_store(&st->claim[((1 - slot) * kClaimRanges + threadIdx.x) * 8], 0ull, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t T = (uint32_t)((a.count + 63) >> 6);                          // 64-nonce blocks
  const uint32_t last_lanes = (uint32_t)(a.count - ((uint64_t)(T - 1) << 6));  // 1..64 in block T-1
  const uint32_t R = (T + kLsWaves - 1) / kLsWaves;                            // rows
  const uint64_t W2 = 2ull * gridDim.x / kClaimRanges;                         // 2 x workgroups per sub-range
  const uint64_t lane_nonce = a.base + lane;                                   // + block * 64
  const uint32_t home = g % kClaimRanges;
  uint64_t done = 0;
  uint32_t claims = 0;
  bool go = true;
  for (uint32_t k = 0; k < kClaimRanges && go; ++k) {
    const uint32_t x = (home + k) % kClaimRanges;
    const uint32_t lo = (uint32_t)((uint64_t)R * x / kClaimRanges);
    const uint32_t Rx = (uint32_t)((uint64_t)R * (x + 1) / kClaimRanges) - lo;
    unsigned long long* ctr = &st->claim[(slot * kClaimRanges + x) * 8];
    uint64_t seen = 0;  // thread 0: the counter as last seen (helping: read before the first claim)
    if (k && threadIdx.x == 0) seen = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if (threadIdx.x == 0) {
        uint32_t c = Rx, end = Rx;
        if (seen < Rx) {
          uint64_t n = (Rx - seen) / W2;
          n = n < 1 ? 1 : (n > a.max_claim ? a.max_claim : n);
          const uint64_t c64 = atomicAdd(ctr, (unsigned long long)n);
          seen = c64 + n;
          if (c64 < Rx) {
            c = (uint32_t)c64;
            end = (uint32_t)(seen < Rx ? seen : Rx);
          }
        }
        uint32_t stop = __hip_atomic_load(&st->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (((claims + g) & a.poll_mask) == 0 &&
            __hip_atomic_load(&mb->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
          __hip_atomic_store(&st->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          stop = 1;
        }
        s_claim[0] = c;
        s_claim[1] = end;
        s_claim[2] = stop;
      }
      ++claims;
      __syncthreads();
      const uint32_t c = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&s_claim[0]);
      const uint32_t end = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&s_claim[1]);
      const uint32_t stop = __builtin_amdgcn_readfirstlane(*(volatile uint32_t*)&s_claim[2]);
      __syncthreads();  // thread 0 rewrites s_claim only after every wave has read it
      if (stop) {
        go = false;
        break;
      }
      if (c >= Rx) break;
      for (uint32_t row = lo + c; row < lo + end; ++row) {
        const uint32_t b = row * kLsWaves + wv;
        const uint64_t nonce = lane_nonce + ((uint64_t)b << 6);
        const uint64_t value = npow_asm_work_value_lockstep_ld(nonce, up);
        uint64_t hits = __ballot(value >= a.threshold);
        if (__builtin_expect(b >= T - 1, 0)) {  // the last block may be partial; blocks past it are empty
          const uint32_t nl = b == T - 1 ? last_lanes : 0u;
          hits &= nl == 64 ? ~0ull : (1ull << nl) - 1;
          done += nl;
        } else {
          done += 64;
        }
        if (__builtin_expect(hits != 0, 0) && ((hits >> lane) & 1)) {  // append every hit
          const uint32_t hs = atomicAdd(&st->n_hits, 1u);
          if (hs < a.cap) out[hs] = nonce;
        }
      }
    }
  }
  if (lane == 0 && done)
    atomicAdd(&st->done_shard[((g * kLsWaves + wv) % kDoneShards) * 8], (unsigned long long)done);
}

// ---- Values through the shipped stream (npow_values_kernel_ls2) ----------------------------------
// Every value of [base, base + count), hashed by exactly the instruction stream the search and sweep
// kernels run (npow_hash_asm_lockstep_ld.inc: the same uniform loads, the same priority runs, the
// same shape of four 512-lane workgroups per CU), so the parity tests compare that stream's 64-bit values with the
// oracle -- not only its hit / no-hit decisions.  Rows of kLsWaves blocks (one per wave) go to workgroups
// round-robin; every wave of a workgroup runs the same number of rows (workgroup-uniform control
// flow, as the search kernel's), and lanes past the range's end hash but do not store.
// 8 bytes per nonce written (the only kernel with algorithmic HBM traffic), coalesced: a wave stores
// 512 contiguous bytes per row.
__global__ __launch_bounds__(kLsBlock, 8) void npow_values_kernel_ls2(const LaunchArgs a, DevState* __restrict__ st,
                                                                     uint64_t* __restrict__ out) {
  const uint64_t* up = ((const LaunchArgs*)__builtin_amdgcn_kernarg_segment_ptr())->u;  // loaded by the stream
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t T = (uint32_t)((a.count + 63) >> 6);   // 64-nonce blocks (count <= 2^31 per launch)
  const uint32_t R = (T + kLsWaves - 1) / kLsWaves;     // rows
  uint64_t done = 0;
  for (uint32_t row = blockIdx.x; row < R; row += gridDim.x) {  // workgroup-uniform
    const uint32_t b = row * kLsWaves + wv;
    const uint64_t i = ((uint64_t)b << 6) + lane;
    const uint64_t value = npow_asm_work_value_lockstep_ld(a.base + i, up);
    if (i < a.count) out[i] = value;
    const uint64_t first = (uint64_t)b << 6;
    done += first >= a.count ? 0 : (a.count - first < 64 ? a.count - first : 64);
  }
  if (lane == 0 && done)
    atomicAdd(&st->done_shard[((blockIdx.x * kLsWaves + wv) % kDoneShards) * 8], (unsigned long long)done);
}

// ---- Work pool: many roots per launch (npow_pool_kernel_ls2*) ----------------------------------
// One launch searches every live entry of the device's table (up to kMaxSlots jobs: the DPoW
// burst, many work_generate requests in flight) plus the dynamic entries published while it runs.
// Index mapping: PoolEntry comment in npow_internal.h.  With one entry this is the plain first-win
// search.
struct PoolCursor {
  const uint64_t* up;  // the entry's uniforms in memory (the stream loads them itself)
  uint64_t threshold, base, gen;
  uint32_t slot;
  uint32_t K, j;      // block index b = it * K + j; nonce = base + b * 64 + lane
  uint32_t it_end;    // the wave runs the entry while it < it_end
  uint32_t last_b;    // bounded: index of the entry's last block ...
  uint32_t tail;      // ... and its lanes in range (64 = full)
  uint32_t bounded;   // exact dense coverage: ignores the launch's time budget
};

__device__ __forceinline__ uint64_t load_dead(PoolDevState* st, uint32_t slot) {
  return __hip_atomic_load(&st->slot[slot].dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Load entry `pe` into the cursor of wave wv of workgroup g (G workgroups, n table entries, e =
// this entry's index).  Bounded entries are dense over their own workgroups (g % n == e, rank
// g / n); unbounded ones map (it, workgroup, wave) to distinct blocks, so a workgroup that moves
// here from a dead entry hashes fresh nonces.
__device__ __forceinline__ void pool_load_ls(const PoolEntry* __restrict__ pe, PoolCursor& c, uint32_t g, uint32_t wv,
                                             uint32_t G, uint32_t n, uint32_t e, uint32_t iters) {
  c.up = pe->u;
  c.threshold = pe->threshold;
  c.base = pe->base;
  c.gen = pe->gen;
  c.slot = pe->slot;
  c.bounded = pe->bounded;
  if (pe->bounded) {
    // own workgroups only: rank r = g / n of cnt; count <= K * iters * 64 (host: launch())
    const uint32_t cnt = G / n + (e < G % n ? 1u : 0u);
    const uint32_t j0 = (g / n) * kLsWaves;
    c.K = kLsWaves * cnt;
    c.j = j0 + wv;
    const uint32_t blocks = (uint32_t)((pe->count + 63) / 64);
    c.it_end = blocks > j0 ? (blocks - j0 + c.K - 1) / c.K : 0u;  // the workgroup's first wave's count
    c.last_b = blocks - 1u;
    c.tail = (uint32_t)(pe->count - (uint64_t)(blocks - 1u) * 64);
  } else {
    c.K = G * kLsWaves;
    c.j = g * kLsWaves + wv;
    c.it_end = iters;
    c.last_b = 0xffffffffu;
    c.tail = 64;
  }
}

__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Live in-kernel clock (PoolClk): the first wave of workgroups 0..kClkWaves-1 -- one per XCD,
// workgroups are dealt to XCDs round-robin -- reads s_memtime after its first instruction and
// both counters after its last; 2 scalar reads and one 24-byte store per 4,096 waves.
__device__ __forceinline__ bool clk_wave() { return blockIdx.x < (unsigned)kClkWaves && threadIdx.x < 64; }
// The search kernels keep the start in LDS: a register live across the whole kernel was spilled to
// scratch by every wave (8 bytes per lane: ~4 MB written and read back per launch, in PMC).
__shared__ uint64_t s_clk_start;
__device__ __forceinline__ void clk_begin_lds() {
  if (clk_wave() && threadIdx.x == 0) s_clk_start = __builtin_amdgcn_s_memtime();
}
__device__ __forceinline__ void clk_end_ls2(const PoolTable* tab, PoolMailbox* mb, uint64_t t_start, uint32_t wv) {
  // wave 0 of workgroups 0..kClkWaves-1; the work-item id is not kept to the end (it was spilled)
  if (wv != 0 || blockIdx.x >= (unsigned)kClkWaves) return;
  const uint64_t c_end = __builtin_amdgcn_s_memtime();
  const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
  if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0) {
    PoolClk* r = &mb->clk[tab->ring & 3][blockIdx.x];
    __hip_atomic_store(&r->cycles, c_end - s_clk_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->ref, t_end - t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->t0, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->t1, t_end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&r->seq, tab->seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
// The search body (npow_pool_kernel_ls2*): four 512-lane workgroups per CU put 8 waves on every
// SIMD.  Each iteration ends with an s_barrier (round 2 also had one after every interval of the
// stream; round 3's stream has none, its waves' priority runs interleave them instead -- DESIGN.md
// section 4), so every wave of a workgroup hashes the same number of times and everything that ends a
// wave's loop is decided per workgroup:
//  * a workgroup works on one entry at a time (its own entry g % n first; bounded entries are dense
//    over their own workgroups' waves, PoolEntry comment with unit = workgroup);
//  * a wave that wants its workgroup to stop (a win, a dead / killed / yielded entry, the time
//    budget) files a request in LDS, s_stop[segment % 3] = min((it + 1) << 2 | kind) with kind 0 =
//    end the launch, 1-3 = leave the entry (why: see the loop), drained before the iteration's closing s_barrier; every
//    wave reads the word at the top of an iteration, so all waves see the same set of requests and
//    leave together, before the next hash (round 4; one hash after it, ~16 us, until round 3);
//  * leaving an entry: wave 0 picks the next entry and broadcasts it through LDS (one
//    __syncthreads); each entry segment has its own request word (3 rotate: the word of segment
//    s + 1 is reset at the end of segment s, after its last reader).
// The register budget at 8 waves per SIMD is 64 VGPRs and 80 SGPRs, of which the stream takes 38 for
// the uniforms it loads itself.  The loop keeps only what every iteration needs in registers: the
// nonce advances in a VGPR by K * 64, the block index by K; the entry's fields, the table and the
// mailbox are re-read inside the rare branches (a win, a poll, leaving an entry).
//
// Early finish: a won or killed entry usually shares its launch with live ones, which keep the
// launch running for the rest of its budget; the job's nonce count would only be read back after
// that.  Instead wave 0 of a workgroup joins an entry (adds 1 to its shard of the slot's wgs counters) before its
// waves hash it, and leaves it (subtracts 1) after all its waves have added their done counts.  An
// entry is over once its dead word holds its generation (a win, a kill relay, a yield); a joiner
// that then finds it dead leaves at once without hashing.  Whoever sees wgs at 0 after seeing the
// entry dead -- the last leaver, or the marker itself -- sums the slot's done shards and publishes
// the total (PoolMailbox::fin).  The protocol's operations are agent-scope atomics, performed at the
// device's point of coherence, and each one completes before the next is issued (s_waitcnt), so
// they are sequentially consistent among themselves: a workgroup that joins after that wgs read
// also finds the entry dead, and every hashing workgroup's done add precedes its leave, so every
// published total is the final one (and equal, if two publish).  The host then finishes the job at
// once.  (Sequentially consistent C++ atomics would also order every other memory access: an L2
// write-back and invalidate around each operation, which quadrupled the search kernel's fetches --
// 12.3 MB per launch against 2.8.  A compare-and-swap join was measured too: 512 workgroups
// retrying on one word at every launch start cost 40 % of throughput.)
__device__ __forceinline__ void ls2_complete() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ bool ls2_over(PoolDevState* st, uint32_t slot, uint64_t gen) {
  const bool over = __hip_atomic_load(&st->slot[slot].dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= gen;
  ls2_complete();
  return over;
}
// Every shard at 0, read one after another after the entry was seen dead: a shard read as 0 means a
// later joiner on that shard will find the entry dead.
__device__ __forceinline__ bool ls2_empty(PoolDevState* st, uint32_t slot) {
  for (int k = 0; k < kWgsShards; ++k) {
    const bool zero = __hip_atomic_load(&st->count[slot][k].wgs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    ls2_complete();
    if (!zero) return false;
  }
  return true;
}
__device__ __forceinline__ uint32_t ls2_shard() { return blockIdx.x % kWgsShards; }

__device__ __forceinline__ void ls2_publish_fin(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen) {
  unsigned long long total = 0, late = 0;
#pragma unroll 1
  for (int i = 0; i < kPoolDoneShards; ++i) {  // (unrolled, the two sums spilled to scratch: this is inlined into
                                               // the poll branch of the search loop, where SGPRs are all taken)
    total += __hip_atomic_load(&st->done[slot][i * 8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    late += __hip_atomic_load(&st->done[slot][i * 8 + kLateWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __hip_atomic_store(&mb->fin[slot].total, (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&mb->fin[slot].late, (uint64_t)late, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&mb->fin[slot].gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Leave the entry (after the workgroup's done adds); the last one out of a dead entry publishes.
__device__ __forceinline__ void ls2_leave(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen) {
  ls2_complete();  // the workgroup's done add first
  const unsigned long long old =
      __hip_atomic_fetch_add(&st->count[slot][ls2_shard()].wgs, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ls2_complete();
  if (old == 1ull && ls2_over(st, slot, gen) && ls2_empty(st, slot)) ls2_publish_fin(st, mb, slot, gen);
}

// Mark it dead (a win, a kill relay, a yield); with no workgroup on it, publish now.
__device__ __forceinline__ void ls2_kill(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen, bool counted) {
  __hip_atomic_fetch_max(&st->slot[slot].dead, (unsigned long long)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ls2_complete();
  if (counted && ls2_empty(st, slot)) ls2_publish_fin(st, mb, slot, gen);
}

// Join it unless it is over (then leave again at once, without hashing).  Uncounted launches
// (PoolTable::counted) only check that it is live.  (The pinned kill word is not read here: the extra
// load in ls2_pick, a call, made the search loop reload 3 more spilled SGPRs with v_readlane every
// iteration; the polls see a kill within an iteration anyway.)
__device__ __forceinline__ bool ls2_join(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen, bool counted) {
  if (!counted) return load_dead(st, slot) < gen;
  __hip_atomic_fetch_add(&st->count[slot][ls2_shard()].wgs, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ls2_complete();
  if (!ls2_over(st, slot, gen)) return true;
  ls2_leave(st, mb, slot, gen);
  return false;
}

// Wave 0, every lane: sum the slot's done shards and late words and publish the final count (PoolMailbox::fin).
// Lanes 0..31 load the done shards, lanes 32..63 the late words of the same lines, in parallel (one lane per
// shard) instead of ~40 round trips one after another -- the publish is on the path of a won job's reply.
__device__ __forceinline__ void ls2_fin_wave(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen,
                                             uint32_t lane) {
  static_assert(kPoolDoneShards == 32, "one half-wave per counter");
  unsigned long long t = __hip_atomic_load(&st->done[slot][(lane & 31) * 8 + (lane < 32 ? 0 : kLateWord)],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) t += __shfl_xor(t, m);
  const unsigned long long t_late = readlane64(t, 32);
  if (lane == 0) {
    __hip_atomic_store(&mb->fin[slot].total, (uint64_t)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mb->fin[slot].late, (uint64_t)t_late, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mb->fin[slot].t_fin, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&mb->fin[slot].gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The same leave by all 64 lanes of wave 0, with the workgroup's count: the checks load in parallel, and the last
// leaver of a dead entry publishes its final count (ls2_fin_wave).  An uncounted launch only adds the counts (its
// end is counted by ls2_exit instead).
__device__ __forceinline__ void ls2_leave_wave(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen,
                                               uint32_t sum, uint32_t late, bool counted) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  unsigned long long* const shard = &st->done[slot][(blockIdx.x % kPoolDoneShards) * 8];
  unsigned long long old = 0;
  if (!counted) {
    if (lane == 0 && sum) atomicAdd(shard, (unsigned long long)sum);
    if (lane == 0 && late) atomicAdd(shard + kLateWord, (unsigned long long)late);
    return;
  }
  if (lane == 0) {
    if (sum) atomicAdd(shard, (unsigned long long)sum);
    if (late) atomicAdd(shard + kLateWord, (unsigned long long)late);
    ls2_complete();  // the counts first
    old = __hip_atomic_fetch_add(&st->count[slot][ls2_shard()].wgs, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ls2_complete();
  }
  if (__builtin_amdgcn_readfirstlane((uint32_t)old) != 1u || (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(old >> 32)) != 0u)
    return;
  const bool over = load_dead(st, slot) >= gen;  // every lane, same word
  ls2_complete();
  if (!__builtin_amdgcn_readfirstlane(over ? 1u : 0u)) return;
  const bool busy = lane < kWgsShards &&
                    __hip_atomic_load(&st->count[slot][lane].wgs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  ls2_complete();
  if (__ballot(busy) != 0) return;
  ls2_fin_wave(st, mb, slot, gen, lane);
}

// Wave 0 of every workgroup of an uncounted (one-entry) launch, at its end (round 5): leave the
// launch's exit count (PoolExit: per XCD shard, then over the shards) after the workgroup's done add; the last
// workgroup out publishes the entry's final count if the entry is over (a win, a kill relayed into its dead word)
// -- every workgroup of the launch has added its count by then, and no later launch hashes a dead entry (its
// workgroups check the dead word before their first hash), so the total is final.  The host then finishes the job
// from that record (Worker::early_finish), instead of waiting for the launch's stop event and the read-back of the
// done counts queued behind it (~0.2-0.35 ms over CU-masked streams).  An entry that is still
// live (the time budget ended the launch) publishes nothing: the next launch goes on with it.  Two levels keep the
// fan-in per word at 1 / 8 of the grid (one address takes ~18 ns per atomic: 1,024 exits on one word ~18 us).
__device__ __noinline__ void ls2_exit(const PoolTable* tab, PoolDevState* st, PoolMailbox* mb, uint32_t G, uint32_t g) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t x = g % kWgsShards;
  const uint32_t in_shard = G / kWgsShards + (x < G % kWgsShards ? 1u : 0u);
  const uint32_t shards = G < (uint32_t)kWgsShards ? G : (uint32_t)kWgsShards;
  PoolExit* ex = &st->exits[tab->ring & (kPoolRing - 1)];
  uint32_t last = 0;
  if (lane == 0) {
    ls2_complete();  // the workgroup's done add first
    unsigned long long* sc = &ex->shard[x][0];
    const unsigned long long o = __hip_atomic_fetch_add(sc, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ls2_complete();
    if (o + 1 == in_shard) {
      __hip_atomic_store(sc, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the ring's next launch
      const unsigned long long t = __hip_atomic_fetch_add(&ex->top, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ls2_complete();
      if (t + 1 == shards) {
        __hip_atomic_store(&ex->top, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 1;
      }
    }
  }
  if (!__builtin_amdgcn_readfirstlane(last)) return;
  const PoolEntry* pe = &tab->e[0];  // the launch's only entry
  const uint32_t slot = pe->slot;
  const uint64_t gen = pe->gen;
  const bool over = load_dead(st, slot) >= gen;
  ls2_complete();
  if (!__builtin_amdgcn_readfirstlane(over ? 1u : 0u)) return;
  ls2_fin_wave(st, mb, slot, gen, lane);
}

__device__ __forceinline__ void ls2_publish_win(PoolDevState* st, PoolMailbox* mb, uint32_t slot, uint64_t gen,
                                             uint64_t wn, uint64_t wv) {
  if (__hip_atomic_fetch_max(&st->slot[slot].dead, (unsigned long long)gen, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT) < gen) {  // first win (the result waits for it)
    PoolWin* pw = &mb->win[slot];
    __hip_atomic_store(&pw->nonce, wn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&pw->value, wv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&pw->t, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&pw->gen, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    // the winner's own workgroup is on the entry: its leave publishes, after the win record
  }
}

// The launch's entries: the table's n, then the dynamic entries the host has published since the
// table was built (PoolMailbox::dyn, at most kDynEntries; n + their count <= kMaxSlots, one slot
// each).  kNoEntry: none.
constexpr uint32_t kNoEntry = 0xffffffffu;
// Through the constant address space: the launch's entries do not change while it can read them,
// and the table's and the ring's fields then load with scalar loads into SGPRs alike.
typedef const __attribute__((address_space(4))) PoolEntry ConstEntry;
__device__ __forceinline__ ConstEntry* ls2_entry(const PoolTable* tab, const PoolMailbox* mb, uint32_t e) {
  const PoolEntry* p = e < tab->n ? &tab->e[e] : &mb->dyn[(tab->dyn_base + (e - tab->n)) % kDynRing].e;
  return (ConstEntry*)(uintptr_t)p;
}
// An entry's slot, generation and bounded flag for a poll's scans of the launch's other entries (kill relays, yields,
// balancing).  A dynamic entry's are read past the caches (system-scope loads of host memory), so a poll needs no
// acquire of newly published entries first (ls2_fresh: an L2 invalidation, one per XCD, the others waiting for it --
// a poll that waited there held up its workgroup's stop when a search was won); a workgroup that picks an entry to
// hash does acquire (ls2_choose).
struct EntryHdr {
  uint64_t gen;
  uint32_t slot, bounded;
};
__device__ __forceinline__ EntryHdr ls2_hdr(const PoolTable* tab, PoolMailbox* mb, uint32_t e) {
  if (e < tab->n) {
    ConstEntry* q = (ConstEntry*)(uintptr_t)&tab->e[e];
    return EntryHdr{q->gen, q->slot, q->bounded};
  }
  PoolEntry* q = &mb->dyn[(tab->dyn_base + (e - tab->n)) % kDynRing].e;
  return EntryHdr{__hip_atomic_load(&q->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                  __hip_atomic_load(&q->slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                  __hip_atomic_load(&q->bounded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)};
}
// Relaxed: an acquire at system scope invalidates the L2, which at every poll cost 4x the search
// kernel's fetches.  But a ring position's lines may still sit in an XCD's L2 from an earlier launch
// (measured: wrong uniforms, invalid work), so a workgroup acquires once after it first sees a newly
// published entry (ls2_fresh; *seen is its LDS count of the entries it has acquired for).
__device__ __forceinline__ uint64_t ls2_ctl(PoolMailbox* mb) {
  return __hip_atomic_load(&mb->ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Each workgroup acquires for itself (round 5 tried one L2 invalidation per XCD with the others waiting for it, and an
// L1 invalidation each: the waits and the L1s made the joins as slow, and a skipped L1 invalidation let picks read
// stale generations -- tools/gpu_r05ac.sh, r05ad).  Only picks acquire: polls read other entries past the caches
// (ls2_hdr).
__device__ __forceinline__ void ls2_fresh(const PoolTable* tab, PoolDevState* st, uint32_t nd, uint32_t* seen) {
  (void)tab;
  (void)st;
  if (nd > *seen) {
#ifndef NPOW_DIAG_NO_FRESH_FENCE
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope: the host wrote the entries
#endif
    *seen = nd;
  }
}
__device__ __forceinline__ uint32_t ls2_dyn_count(const PoolTable* tab, uint64_t ctl) {
  const uint32_t d = (uint32_t)ctl - tab->dyn_base;
  return d < (uint32_t)kDynEntries ? d : (uint32_t)kDynEntries;
}
// The same for a value that may predate the launch's table (PoolDevState::ctl_mirror): none then.
__device__ __forceinline__ uint32_t ls2_dyn_count_since(const PoolTable* tab, uint64_t ctl) {
  const int32_t d = (int32_t)((uint32_t)ctl - tab->dyn_base);
  return d <= 0 ? 0u : (d < kDynEntries ? (uint32_t)d : (uint32_t)kDynEntries);
}

// The launch's entries this workgroup knows to be over (bit k: entry k -- dead, or bounded, which no workgroup moves
// to): an entry's header (slot, generation) is read from the table or from the pinned dynamic ring, uncached over PCIe
// for every lane that looks at it, so a lingering launch, whose ring fills with the serial client's finished
// searches, would otherwise re-read every one of them at each pick and at each balancing poll (round 5).  An entry
// once dead stays dead (its slot's dead word only grows), so the mask is exact.  Wave 0 picks; any wave's poll may
// add bits (an LDS atomic or).
__shared__ unsigned long long s_over;
__device__ __forceinline__ void ls2_mark_over(unsigned long long bits) {
  if (bits) __hip_atomic_fetch_or(&s_over, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Occupancy for balancing: this XCD shard's workgroups on the entry (workgroups are dealt to the XCDs
// round-robin, so balancing each shard balances the whole).
__device__ __forceinline__ unsigned long long ls2_wgs(PoolDevState* st, uint32_t slot) {
  return __hip_atomic_load(&st->count[slot][ls2_shard()].wgs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A polling wave (lane 0 only): the host words of the entry.  Returns bit 0 set when the wave's
// workgroup must leave the entry, and bit 1 too when the reason is the pinned kill word: new jobs wait and the entry is unbounded (a yield), it was
// killed, or it is unbounded and a dynamic entry has at least two workgroups fewer than it (the
// workgroup moves there: a job that joined the running launch collects its share a workgroup at a
// time, each from the most crowded entry among the pollers).
__device__ __forceinline__ uint32_t ls2_poll(const PoolTable* tab, PoolDevState* st, PoolMailbox* mb, uint32_t e,
                                         uint32_t* seen) {
  const ConstEntry* pe = ls2_entry(tab, mb, e);
  const uint64_t ctl = ls2_ctl(mb);
  // a lingering launch keeps the device-memory mirror of ctl fresh from its polls too: a workgroup leaving an entry
  // picks its next one from the mirror (ls2_pick), and the mirror is otherwise raised only by lingering workgroups
  if (tab->linger)
    __hip_atomic_fetch_max(&st->ctl_mirror[0], (unsigned long long)ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // (a one-entry launch -- uncounted -- holds only the entry whose kill word this poll reads below: no read of
  // the counter there, whose uncached read at every poll was 0.76 MB per 10-ms launch of PMC traffic)
  // (nor in a launch of one entry so far: a lingering launch is counted from its first entry on)
  const uint32_t nd = ls2_dyn_count(tab, ctl);
  const uint32_t kills = tab->counted && tab->n + nd > 1
                             ? (uint32_t)__hip_atomic_load(&mb->kills, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                             : tab->kill_base;
  (void)seen;  // (the entries it looks at here are read past the caches: ls2_hdr)
  bool leave = false;
  // A job of this launch was killed since it was built, and no wave has relayed that kill yet: relay every such
  // entry (its dead word first, a device read; the kill word, uncached, only for live entries), then record the
  // counter value so that the other polls skip the scan (round 4: scanning at every poll after a kill cost a
  // 512-request burst 10 % of its kernel rate -- 64 serial uncached reads stalled each polling workgroup).
  // The scan's key is this launch's (seq, kills) (keyed by the count alone, a launch could skip the
  // scan because another launch, holding other entries, had relayed up to the same count).  The kill words are
  // read only after `kills` was compared (a control dependency: the loads are issued after its value returned,
  // and they bypass the caches), so every kill the counter stands for is seen: the host raises a kill word
  // before it bumps the counter (release).  The compiler barrier keeps them from being hoisted above it.
  unsigned long long* const kd = &st->kills_done[tab->ring & (kPoolRing - 1)][0];
  const unsigned long long key = ((unsigned long long)tab->seq << 32) | kills;
  if (kills != tab->kill_base && __hip_atomic_load(kd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != key) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const unsigned long long over = __hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (uint32_t k = 0; k < tab->n + nd; ++k) {
      if ((over >> k) & 1) continue;
      const EntryHdr q = ls2_hdr(tab, mb, k);
      if (load_dead(st, q.slot) < q.gen &&
          __hip_atomic_load(&mb->kill[q.slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == q.gen)
        ls2_kill(st, mb, q.slot, q.gen, tab->counted != 0);
    }
    __hip_atomic_store(kd, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if ((ctl >> 32) != (tab->yield_base >> 32)) {
    // (only the entries still live: each kill is an atomic and, counted, 8 serial loads -- over a lingering launch's
    // ring of 33 mostly finished entries ~0.35 ms, which held up a losing search's stop when the host ended the
    // launch under it)
    const unsigned long long over = __hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (uint32_t k = 0; k < tab->n + nd; ++k) {
      if ((over >> k) & 1) continue;
      const EntryHdr q = ls2_hdr(tab, mb, k);
      if (!q.bounded && load_dead(st, q.slot) < q.gen) ls2_kill(st, mb, q.slot, q.gen, tab->counted != 0);
    }
    leave = !pe->bounded;
  }
  bool killed = false;
  if (__hip_atomic_load(&mb->kill[pe->slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == pe->gen) {
#ifdef NPOW_DIAG_TIMES
    __hip_atomic_store(&mb->fin[pe->slot].t_relay, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    ls2_kill(st, mb, pe->slot, pe->gen, tab->counted != 0);  // relay
    leave = killed = true;
  }
  if (!leave && !pe->bounded && nd > 0) {
    const unsigned long long mine = ls2_wgs(st, pe->slot);
    const unsigned long long over = __hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    unsigned long long found = 0;
    for (uint32_t k = tab->n; k < tab->n + nd && !leave; ++k) {
      if (k == e || ((over >> k) & 1)) continue;
      const EntryHdr q = ls2_hdr(tab, mb, k);
      if (q.bounded || load_dead(st, q.slot) >= q.gen) {
        found |= 1ull << k;
        continue;
      }
      leave = ls2_wgs(st, q.slot) + 2 <= mine;
    }
    ls2_mark_over(found);
  }
  return (leave ? 1u : 0u) | (killed ? 2u : 0u);
}

// Wave 0 (every lane): of the launch's first nd dynamic entries and its table's, the live unbounded entry other than e
// with the fewest workgroups, joined, ties broken by a hash of the workgroup index so that the workgroups leaving one
// entry spread over the others; kNoEntry if none can be.  Each lane looks at one entry.
__device__ __forceinline__ uint32_t ls2_choose(const PoolTable* tab, PoolDevState* st, PoolMailbox* mb, uint32_t e,
                                               uint32_t nd, uint32_t* seen, uint32_t lane, uint32_t g) {
  const uint32_t N = tab->n + nd;  // <= kMaxSlots = 64: one lane each
  ls2_fresh(tab, st, nd, seen);
  for (int attempt = 0; attempt < 4; ++attempt) {
    unsigned long long key = ~0ull;
    bool over = false;
    const unsigned long long known = __hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (lane < N && lane != e && !((known >> lane) & 1)) {
      ConstEntry* q = ls2_entry(tab, mb, lane);
      if (!q->bounded && load_dead(st, q->slot) < q->gen) {
        const uint32_t tie = ((lane + 1u) * 0x9e3779b1u) ^ (g * 0x85ebca6bu);
        key = (ls2_wgs(st, q->slot) << 32) | (tie & ~63u) | lane;
      } else {
        over = true;
      }
    }
    const unsigned long long now_over = __ballot(over);
    if (lane == 0) ls2_mark_over(now_over);
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const unsigned long long o = __shfl_xor(key, m);
      key = o < key ? o : key;
    }
    if (key == ~0ull) return kNoEntry;
    const uint32_t pick = (uint32_t)key & 63u;
    uint32_t ok = 0;
    if (lane == 0) {
      ConstEntry* q = ls2_entry(tab, mb, pick);
      ok = ls2_join(st, mb, q->slot, q->gen, tab->counted != 0) ? 1u : 0u;
    }
    if (__builtin_amdgcn_readfirstlane(ok)) return pick;
  }
  return kNoEntry;  // entries died under every attempt
}

// Wave 0 (every lane) of a workgroup of a lingering launch (PoolTable::linger, round 5) that found no live entry to
// move to: wait in the launch for the host's next dynamic entry instead of leaving it, so that a serial client's next
// search starts without a launch (its dispatch, the stream's events, the host's launch call and the cold start: the
// GPU's gap between two searches was ~35 us on one device and ~110 us on each of 8 CU partitions,
// tools/experiments/launch_spans.py).  Returns the entry joined, or kNoEntry once the host raised a yield (it ends a
// lingering launch that a new launch must follow: a bounded job, a sweep, shutdown, the launch's time budget over --
// Worker::end_linger) or after a budget's worth of lingering (a host that stopped looking).
// The pinned word is read by ~2 lingering workgroups per look period grid-wide (phase (k + g) mod P, P ~ G / 2), each
// of which raises PoolDevState::ctl_mirror to it; the others look at the mirror in device memory.  Between looks the
// wave sleeps ~1.8 us (s_sleep 64: 64 x 64 clocks); the other waves of the workgroup wait at the barrier after it.
// Round 6: lingering waves poll no kill word, so an entry whose hashing workgroups had all left it
// while it was live -- the launch's time budget ends a hashing workgroup (kind 0) while others linger on, up to a
// budget past their own entry into ls2_linger -- had nobody to relay its kill: its final count was not published until
// the host gave up on it (1 ms) and ended the launch, and until then nobody hashed it either.  Now the lingering
// workgroup that reads the pinned words (about two per look grid-wide) also relays every kill raised since the
// launch's last relay (the same scan, keyed by (seq, kills), as ls2_poll's: a dead entry with no workgroup on it is
// published at once by ls2_kill) and looks at all of the launch's live entries again, not only new ones (such an entry
// is joined and hashed again; past the launch's budget its joiners leave within 4 iterations, ending the launch).
// Lane 0.  (Inlined: the search loop keeps its register allocation, tools/kernel_loop_census.py, and no call frame.)
__device__ __forceinline__ void ls2_linger_relay(const PoolTable* tab, PoolDevState* st, PoolMailbox* mb, uint32_t nd) {
  const uint32_t kills = (uint32_t)__hip_atomic_load(&mb->kills, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned long long* const kd = &st->kills_done[tab->ring & (kPoolRing - 1)][0];
  const unsigned long long key = ((unsigned long long)tab->seq << 32) | kills;
  if (kills == tab->kill_base || __hip_atomic_load(kd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key) return;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the kill words after the counter (ls2_poll)
  const unsigned long long over = __hip_atomic_load(&s_over, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (uint32_t k = 0; k < tab->n + nd; ++k) {
    if ((over >> k) & 1) continue;
    const EntryHdr q = ls2_hdr(tab, mb, k);
    if (load_dead(st, q.slot) < q.gen &&
        __hip_atomic_load(&mb->kill[q.slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == q.gen) {
      // (marked before the kill, whose publish releases the final count: the host reads it with the record)
      __hip_atomic_store(&mb->fin[q.slot].linger_gen, q.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ls2_kill(st, mb, q.slot, q.gen, true);  // (a lingering launch is counted)
    }
  }
  __hip_atomic_store(kd, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t ls2_linger(const PoolTable* tab, PoolDevState* st, PoolMailbox* mb, uint32_t* seen,
                                            uint32_t looked) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const uint32_t g = blockIdx.x;
  const uint32_t P = tab->linger;  // a power of two (Worker::launch)
  unsigned long long* const mirror = &st->ctl_mirror[0];
  const uint32_t base_hi = (uint32_t)(tab->yield_base >> 32);
  const uint32_t t_enter = (uint32_t)__builtin_amdgcn_s_memrealtime();
  for (uint32_t k = 0;; ++k) {
    if ((uint32_t)__builtin_amdgcn_s_memrealtime() - t_enter >= tab->budget) return kNoEntry;
    uint64_t ctl;
    const bool pinned = ((k + g) & (P - 1)) == 0;
    if (pinned) {
      ctl = ls2_ctl(mb);
      __hip_atomic_fetch_max(mirror, (unsigned long long)ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      ctl = __hip_atomic_load(mirror, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t hi = (uint32_t)(ctl >> 32);
    if ((int32_t)(hi - base_hi) > 0) return kNoEntry;  // a yield since the table was built
    if (hi == base_hi) {                               // (an older mirror value: no news)
      const uint32_t nd = ls2_dyn_count_since(tab, ctl);
      if (pinned) {
        if (lane == 0) ls2_linger_relay(tab, st, mb, nd);
        looked = 0;  // every live entry again (above)
      }
      if (nd > looked || (pinned && tab->n > 0)) {
        const uint32_t p = ls2_choose(tab, st, mb, kNoEntry, nd, seen, lane, g);
        if (p != kNoEntry) return p;
        looked = nd;  // (joined by others and over already, or cancelled)
      }
    }
    __builtin_amdgcn_s_sleep(64);
  }
}

// Wave 0 (every lane): the entry the workgroup works on next, joined; kNoEntry if none can be.  At
// the launch's start (first) its own entry e, bounded or not, if it can be joined; otherwise another
// live unbounded entry (ls2_choose).
__device__ __noinline__ uint32_t ls2_pick(const PoolTable* tab, PoolDevState* st, PoolMailbox* mb, uint32_t e,
                                          bool first, uint32_t* seen) {
  // the lane from mbcnt, not threadIdx: a callee that reads the work-item id makes every wave keep
  // (and spill) the register the ABI passes it in
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)), g = blockIdx.x;
  if (first) {
    uint32_t ok = 0;
    if (lane == 0) {
      ConstEntry* pe = ls2_entry(tab, mb, e);
      ok = ls2_join(st, mb, pe->slot, pe->gen, tab->counted != 0) ? 1u : 0u;  // (the join checks dead itself)
    }
    if (__builtin_amdgcn_readfirstlane(ok)) return e;
  }
  // the dynamic entries published so far: the pinned word -- or in a lingering launch leaving an entry the mirror
  // (all its workgroups leave a won entry at once: ~G uncached reads of the pinned word together otherwise), which
  // may be older: ls2_linger then learns of the newer ones
  const bool lg = !first && tab->linger;
  const uint32_t nd = lg ? ls2_dyn_count_since(tab, __hip_atomic_load(&st->ctl_mirror[0], __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT))
                         : ls2_dyn_count(tab, ls2_ctl(mb));
  return ls2_choose(tab, st, mb, e, nd, seen, lane, g);
}

// Odd, so that it0 -> -it0 * kPollStride is a bijection modulo every power of two; its residues mod 2^10..2^13 step
// by 0.43, 0.22, 0.11 and 0.80 of the range (the fractional part of the golden ratio in 32 bits).
constexpr uint32_t kPollStride = 0x9E3779B9u;

template <bool BOUNDED>
__device__ __forceinline__ void pool_body_ls2(const PoolTable* __restrict__ tab, PoolDevState* __restrict__ st,
                                              PoolMailbox* __restrict__ mb, const uint64_t t_start) {
  __shared__ uint32_t s_stop[3];         // per entry segment (mod 3): the earliest stop request
  __shared__ uint32_t s_flag[kLsWaves];  // lane 0 of a polling wave -> its wave: leave the entry (one word
                                         // per wave: with a poll interval below 16, several waves poll at once)
  __shared__ uint32_t s_next;
  __shared__ uint32_t s_done[kLsWaves];  // each wave's nonces on the entry it is leaving
  __shared__ uint32_t s_seen;            // dynamic entries this workgroup has acquired for (ls2_fresh)
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t g = blockIdx.x, G = gridDim.x;
  const uint32_t w = g * kLsWaves + wv;
  const uint32_t n = tab->n, iters = tab->iters;
  if (threadIdx.x < 3) s_stop[threadIdx.x] = ~0u;
  const bool counted = tab->counted != 0;
  if (wv == 0) {
    if (lane == 0) {
      s_seen = 0;
      s_over = 0;
    }
    // its own entry first.  An uncounted (one-entry) launch only checks that it is live: it may follow
    // a counted launch that held the same entry and has published its final count, after which no
    // nonce may be hashed for it (tests/test_gpu_configs.py caught one launch doing so).
    uint32_t first;
    if (n == 0) {
      first = kNoEntry;  // an empty lingering launch (Worker::relaunch_linger): straight to ls2_linger
    } else if (counted) {
      first = ls2_pick(tab, st, mb, g % n, true, &s_seen);
    } else {
      // only the device-side dead word: reading the pinned kill word here too (512 workgroups' PCIe reads
      // at once) delayed every launch's first hash by 30-60 us -- receive-difficulty searches p50 0.29-0.33
      // against 0.26 ms (profiles/r03_ab_latency.jsonl); a kill is seen by the first polls instead
      ConstEntry* pe = ls2_entry(tab, mb, g % n);
      first = load_dead(st, pe->slot) < pe->gen ? g % n : kNoEntry;
    }
    if (lane == 0) s_next = first;
  }
  __syncthreads();

  uint32_t e = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
  uint32_t seg = 0, it = 0;
  uint32_t pc = w;  // the poll phase, (iterations on the entry) * kPollStride + w: carried through the loop (the
                    // invariant w, beside it, was spilled and reloaded with a v_readlane every iteration once
                    // ls2_linger was called)
  bool end = false;
  for (;;) {  // a lingering launch: rounds of entries, each after the workgroup waited for the next one (ls2_linger)
  for (;;) {
    if (e == kNoEntry) break;
    const PoolEntry* pe = (const PoolEntry*)ls2_entry(tab, mb, e);
    PoolCursor c;
    pool_load_ls(pe, c, g, wv, G, n, e, iters);
#ifdef NPOW_DIAG_TIMES
    if (wv == 0 && lane == 0) {
      const uint64_t tj = __builtin_amdgcn_s_memrealtime();
      __hip_atomic_store(&mb->fin[c.slot].t_join, tj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&mb->diag_join[g & 1023], tj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#endif
    // the poll phase restarts with each entry: the workgroups that join one together (a launch's start, a lingering
    // launch's next search) then hash it in step, so exactly one wave in poll_mask + 1 polls per iteration; carried
    // on from the launch's start instead, the phases of workgroups that had lingered apart drifted and the polls
    // came at random (a tail on the losers' stop span over CU partitions)
    pc = w;
    const uint32_t sw = seg % 3;
    const uint32_t poll_mask = tab->poll_mask, budget = tab->budget;
    unsigned long long* const dead_p = &st->slot[c.slot].dead;
    uint32_t b = it * c.K + c.j;
    uint64_t nonce = c.base + ((uint64_t)b << 6) + lane;
    const uint64_t step = (uint64_t)c.K << 6;
    uint32_t done = 0;
    while (it < c.it_end) {
      const uint32_t verdict = __hip_atomic_load(&s_stop[sw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint64_t dead = __hip_atomic_load(dead_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // The verdict holds every request filed after the previous hashes: each was drained before the
      // s_barrier closing its iteration, which every wave passed before this read.  So all waves see the same
      // set here and leave together, before this hash (round 4; rounds 2-3 acted on it after the hash: one
      // more hash per stop).  A request of this iteration from a wave already past its hash (value > it) is
      // left for the next read, which every wave makes.
      const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane(verdict);
      if (v != ~0u && (v >> 2) <= it) {
        end = (v & 3u) == 0;
        break;
      }
      const uint32_t it0 = it;
      const uint32_t pc0 = pc;  // the poll phase of iteration it0
      const uint64_t thr = c.threshold, gen = c.gen;
      const uint64_t value = npow_asm_work_value_lockstep_ld(nonce, c.up);
      ++it;
      pc += kPollStride;
      bool hit = value >= thr;
      if constexpr (BOUNDED) {
        const uint32_t in_lanes = b < c.last_b ? 64u : (b == c.last_b ? c.tail : 0u);
        hit = hit && lane < in_lanes;
        done += in_lanes;
      } else {
        done += 64;
      }
      const uint64_t hits = __ballot(hit);
      // why the workgroup must leave the entry, as a stop-request kind (0 = not at all; the time budget files
      // kind 0 = end the launch): 1 = the entry was over before this hash started (its dead word), 2 = it is
      // over since this hash (a win; a kill read by this wave's poll), 3 = leave for another reason (a yield,
      // a move to a new entry).  The smallest kind of the earliest iteration wins, so the exit knows how many
      // of the workgroup's last hashes started after it knew the entry was over: 2 for kind 1, 1 for kind 2.
      uint32_t why = hits != 0 ? 2u : 0u;
      if (__builtin_expect(hits != 0, 0)) {
        const int wl = __builtin_ctzll(hits);
        const uint64_t wn = readlane64(nonce, wl), wval = readlane64(value, wl);
        if (lane == 0) {
          // the entry's slot and generation re-read from it (c.up points at the entry): kept live for
          // this rare branch they were spilled to scratch by every wave at every entry it joined
          ConstEntry* ce = (ConstEntry*)(uintptr_t)c.up;
          asm volatile("" : "+s"(ce));
          ls2_publish_win(st, mb, ce->slot, ce->gen, wn, wval);
        }
      }
      // which wave polls at iteration it0: the one with w = -it0 * kPollStride (mod poll_mask + 1) -- consecutive
      // iterations' pollers spread over the grid (round 5).  With w = -it0 a launch's first ~100 polls all fell to its
      // last-dispatched workgroups, the youngest and slowest on their SIMDs (VALU issue favours the oldest wave): on a
      // grid of 1,024 waves (one 32-CU partition) a host kill then waited ~200 us for a poll instead of ~15
      // (profiles/r05f_over_g8.err: relay p50 207 us after the win against 37 us on 64-CU partitions)
      if (__builtin_expect((pc0 & poll_mask) == 0, 0)) {
        if (lane == 0) s_flag[wv] = ls2_poll(tab, st, mb, e, &s_seen);  // the wave's own word
        lds_drain();
        const uint32_t p = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&s_flag[wv], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT));
        why = (p & 2u) ? 2u : (why ? why : (p ? 3u : 0u));
      }
      // the dead word in one v_cmp (readlane64 took two v_readlane and their SALU hazards), and the time budget
      // at every fourth iteration: the launch's start clock lives in lanes of a VGPR (an SGPR spill) whose two
      // v_readlane per iteration, with their s_nop hazards, cost 15 SIMD cycles per hash (-0.36 %,
      // tools/experiments/loop_ab.py, profiles/r04_ab_loop.jsonl); a launch now ends up to ~45 us past its budget
      if (__ballot(dead == gen) != 0) why = 1u;
      const bool late = budget && !c.bounded && (it0 & 3u) == 0 &&
                        (uint32_t)__builtin_amdgcn_s_memrealtime() - (uint32_t)t_start >= budget;
      if (__builtin_expect(why != 0 || late, 0)) {
        if (lane == 0)
          __hip_atomic_fetch_min(&s_stop[sw], (it << 2) | (late ? 0u : why), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
        lds_drain();
      }
      nonce += step;
      b += c.K;
      __builtin_amdgcn_s_barrier();
    }
    // the workgroup's count, added by wave 0 before it leaves the entry (early finish, ls2_leave):
    // one atomic and no fence per wave
    if (lane == 0) s_done[wv] = done;
    __syncthreads();
    if (wv == 0) {
      uint32_t sum = lane < kLsWaves ? s_done[lane] : 0u;
#pragma unroll
      for (int m = kLsWaves / 2; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
      // device-side overshoot: the workgroup's hashes of this entry that started after one of its waves knew
      // the entry was over -- a request filed after hash i ends the loop before hash i + 1, so one such hash
      // per wave when the dead word was already up before hash i (kind 1; its value is read after the hash
      // that its load's latency hides behind), none when hash i itself revealed it (kind 2: a win, a kill read
      // by a poll).  Every wave of the workgroup leaves at the same iteration; capped by the workgroup's count.
      // (read back from LDS after the barrier above rather than kept in a register through the loop: one more
      // value live across the loop spilled to scratch)
      const uint32_t v = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&s_stop[sw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      const uint32_t kind = v != ~0u && (v >> 2) == it ? (v & 3u) : 0u;  // the loop ended on this request
      uint32_t late_n = kind == 1u ? 64u * kLsWaves : 0u;
      late_n = late_n < sum ? late_n : sum;
      ls2_leave_wave(st, mb, c.slot, c.gen, sum, late_n, counted);
    }
    if (it >= iters || end || !counted) break;  // an uncounted launch has no other entry
    if (wv == 0) {
      const uint32_t next = ls2_pick(tab, st, mb, e, false, &s_seen);
      if (lane == 0) {
        s_next = next;
        s_stop[(seg + 1) % 3] = ~0u;
      }
    }
    __syncthreads();
    e = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    ++seg;
  }
  // no entry to move to (the loop ended on kNoEntry, not on the budget or the iteration cap): a lingering launch's
  // workgroup waits for the host's next one.  (Called here, after the entry loop, and not from ls2_pick: a callee
  // there clobbering more registers made the search loop reload 4 more spilled SGPRs every iteration.)
  if constexpr (BOUNDED) break;  // (the host sets linger only for launches of unbounded entries)
  if (e != kNoEntry || !tab->linger) break;
  __syncthreads();  // every wave has read s_next before wave 0 writes it again
  if (wv == 0) {
    const uint32_t next = ls2_linger(tab, st, mb, &s_seen, 0);
    if (lane == 0) s_next = next;
  }
  __syncthreads();
  e = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
  if (e == kNoEntry) break;
  }
  if (!counted && wv == 0) ls2_exit(tab, st, mb, G, g);  // the one-entry launch's end record (round 5)
  clk_end_ls2(tab, mb, t_start, wv);
}

template <bool BOUNDED>
__global__ __launch_bounds__(kLsBlock, 8) void npow_pool_kernel_ls2(const PoolTable* __restrict__ tab,
                                                                   PoolDevState* __restrict__ st,
                                                                   PoolMailbox* __restrict__ mb) {
  uint64_t t_start;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_start) :: "memory");
  clk_begin_lds();
  pool_body_ls2<BOUNDED>(tab, st, mb, t_start);  // records the clock at its end (clk_end_ls2)
}

template <bool BOUNDED>
__global__ __launch_bounds__(kLsBlock, 8) void npow_pool_kernel_ls2_arg(const PoolTableArg targ,
                                                                       PoolDevState* __restrict__ st,
                                                                       PoolMailbox* __restrict__ mb) {
  uint64_t t_start;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_start) :: "memory");
  (void)targ;
  const PoolTable* tab = (const PoolTable*)__builtin_amdgcn_kernarg_segment_ptr();
  clk_begin_lds();
  pool_body_ls2<BOUNDED>(tab, st, mb, t_start);  // records the clock at its end (clk_end_ls2)
}

hipError_t launch_pool(hipStream_t stream, int grid, const PoolTable* tab, bool bounded, PoolDevState* st,
                       PoolMailbox* mb) {
  if (bounded)
    npow_pool_kernel_ls2<true><<<grid, kLsBlock, 0, stream>>>(tab, st, mb);
  else
    npow_pool_kernel_ls2<false><<<grid, kLsBlock, 0, stream>>>(tab, st, mb);
  return hipGetLastError();
}

hipError_t launch_pool_arg(hipStream_t stream, int grid, const PoolTable& host_tab, bool bounded, PoolDevState* st,
                           PoolMailbox* mb) {
  if (host_tab.n > (uint32_t)kArgEntries) return hipErrorInvalidValue;
  PoolTableArg a;
  memcpy(&a, &host_tab, pool_table_bytes(host_tab.n));
  if (bounded)
    npow_pool_kernel_ls2_arg<true><<<grid, kLsBlock, 0, stream>>>(a, st, mb);
  else
    npow_pool_kernel_ls2_arg<false><<<grid, kLsBlock, 0, stream>>>(a, st, mb);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void npow_pairs_kernel(const uint64_t* __restrict__ roots_words,
                                                            const uint64_t* __restrict__ nonces, uint32_t n,
                                                            uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint64_t m[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = roots_words[4 * (size_t)i + k];
  out[i] = work_value_full(nonces[i], m);
}

hipError_t launch_task(Mode mode, int grid, hipStream_t stream, const LaunchArgs& a, DevState* st,
                       HostMailbox* mb, uint64_t* out) {
  switch (mode) {
    case Mode::kSweep:
      npow_sweep_kernel_ls2<<<grid, kLsBlock, 0, stream>>>(a, st, mb, out);
      break;
    case Mode::kValues:
      npow_values_kernel_ls2<<<grid, kLsBlock, 0, stream>>>(a, st, out);
      break;
    case Mode::kValuesSeq:
      npow_values_kernel_seq<<<grid, kBlock, 0, stream>>>(a, st, out);
      break;
  }
  return hipGetLastError();
}

hipError_t launch_pairs(int grid, hipStream_t stream, const uint64_t* roots_words, const uint64_t* nonces,
                        uint32_t n, uint64_t* out) {
  npow_pairs_kernel<<<grid, kBlock, 0, stream>>>(roots_words, nonces, n, out);
  return hipGetLastError();
}

}  // namespace npow
