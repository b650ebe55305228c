// npow_internal.h -- structures shared by the gfx950 kernels and the host engine.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "npow_blake2b.h"
#include "npow_hash_asm.inc"
#include "npow_hash_asm_lockstep_ld.inc"

namespace npow {

constexpr int kBlock = 256;               // npow_values_kernel_seq / npow_pairs_kernel: lanes per workgroup
// Search, sweep and values kernels of the shipped stream: 8 waves per SIMD in four 512-lane
// workgroups per CU (round 3: against two 1,024-lane ones, -0.65 % SIMD cycles per hash in searches
// and +1.2 % sweep rate, profiles/r03_ab_wgsize*.jsonl; 256-lane ones are slower).
constexpr int kLsWaves = 8;                // waves per workgroup (2 per SIMD) ...
constexpr int kLsBlock = kLsWaves * 64;    // ... 512 lanes
constexpr int kLsGroups = 4;               // ... four workgroups per CU: 8 waves per SIMD, 64 VGPRs each

// One-root tasks (launch_task): npow_sweep_kernel_ls2 (kSweep), npow_values_kernel_ls2 (kValues, the
// shipped stream), npow_values_kernel_seq (kValuesSeq, the second stream); first-win searches are
// the pool's (npow_pool_kernel_ls2*).
enum class Mode : int { kSweep = 1, kValues = 2, kValuesSeq = 3 };

// Kernel arguments, passed by value: the kernarg segment lands in SGPRs, so the
// root-derived uniforms and the threshold cost no memory traffic per nonce
// (SURVEY.md §7 "Uniform data in SGPRs").
struct LaunchArgs {
  uint64_t u[NPOW_ASM_N_UNIFORMS];  // nonce-independent intermediates (npow_asm_uniforms)
  uint64_t threshold;  // valid iff value >= threshold
  uint64_t base;       // first nonce of this launch (wraps mod 2^64)
  uint64_t count;      // nonces in this launch (lane index i < count)
  uint32_t poll_mask;  // a wave polls the host abort word when (iter & poll_mask) == 0
  uint32_t cap;        // sweep: capacity of the hit buffer
  uint32_t claim_slot; // sweep: DevState::claim[claim_slot] is this launch's work counter
  uint32_t max_claim;  // sweep: most 64-nonce wave iterations one claim takes
};

// Device-resident per-task state (hipMalloc; reset by hipMemsetAsync per task).
// The nonces-hashed counter is sharded over 256 cache lines: every wave adds its
// count once at exit, and 8,192 waves adding to ONE word serialise at the memory
// side (~12 ns each, MI355X_MICROARCH.md "fanin") -- a ~100 us tail on every launch.
constexpr int kDoneShards = 256;
constexpr int kClaimRanges = 8;  // sweep sub-ranges per launch (one per XCD), npow_sweep_kernel_ls2
struct DevState {
  union {
    struct {
      uint32_t found;       // unused (first-win search lives in the pool); always 0
      uint32_t abort;       // host abort relayed by the wave that saw it
    };
    uint64_t stop;          // both, read by every wave with one 8-byte load
  };
  uint32_t n_hits;          // sweep: hits appended (may exceed cap)
  uint32_t pad0;
  uint64_t nonce;           // winning nonce (search)
  uint64_t value;           // winning value (search)
  uint32_t zero;            // always 0: the non-polling iterations' load target
  uint8_t pad1[64 - 36];
  // Sweep work counters (rows of kLsWaves blocks claimed so far) of the launch's 8 sub-ranges
  // (one per XCD), for each launch parity: launch k claims from claim[k & 1][*] and zeroes
  // claim[(k + 1) & 1][*] for launch k + 1 (same stream, so launch k - 1, their previous
  // user, has finished).  One cache line each: atomics on one address serialise (~18 ns
  // each), and every wave polls `stop` above each iteration.
  unsigned long long claim[2 * kClaimRanges * 8];
  unsigned long long done_shard[kDoneShards * 8];  // nonces hashed, one counter per 64-byte line
  uint64_t done() const {
    uint64_t s = 0;
    for (int i = 0; i < kDoneShards; ++i) s += done_shard[i * 8];
    return s;
  }
};

// Host-coherent pinned mailbox (hipHostMalloc coherent + mapped).  The winning
// wave publishes here with system-scope stores so the host thread sees a win
// without waiting for the launch to drain; the host raises `abort` to stop
// every wave of every in-flight launch (polled every poll_mask+1 iterations).
struct alignas(64) HostMailbox {
  uint32_t found;
  uint32_t pad0;
  uint64_t nonce;
  uint64_t value;
  uint8_t pad1[64 - 24];
  uint32_t abort;  // on its own cache line
  uint8_t pad2[60];
};

// ---- Work pool: many roots searched by one launch (npow_pool_kernel_ls2*) -------------------
// Each device keeps up to kMaxSlots live jobs in "slots".  Every launch reads a table of
// the live entries (its kernel arguments, or device memory past kArgEntries entries);
// workgroup g starts on entry g % n.  A slot is identified per job by a generation number `gen` (unique, > 0): a slot
// is dead for generation g once PoolDevState::slot[s].dead >= g (set by its winner with
// atomicMax, or relayed from the host kill word), so a slot can be reused for a new job
// with a larger gen without clearing any device memory.
constexpr int kMaxSlots = 64;
constexpr int kPoolDoneShards = 32;

// Nonce-index mapping of one entry (the launch's region is [base, base + count)); w = g * kLsWaves + wave:
//  * unbounded (search until won/cancelled): index = (it * W + w) * 64 + lane, W = grid
//    waves -- every (iteration, wave) pair is distinct, so workgroups that move here from a
//    dead entry hash fresh nonces; the region spans W * iters * 64 nonces (holes allowed);
//  * bounded (max_nonces set; must cover its range exactly once): only the entry's own
//    workgroups (g % n == e, rank r = g / n, k_e of them) run it, index = (it * 8 k_e + 8 r +
//    wave) * 64 + lane (8 = kLsWaves), dense over [0, count) with count <= 8 k_e * iters * 64; others never
//    enter it.
struct PoolEntry {
  uint64_t u[NPOW_ASM_N_UNIFORMS];  // nonce-independent intermediates of the root
  uint64_t threshold;
  uint64_t base;
  uint64_t count;
  uint64_t gen;
  uint32_t slot;     // device slot index (PoolDevState / PoolMailbox arrays)
  uint32_t bounded;  // 1: dense mapping over the entry's own workgroups, no migrants
};
static_assert(offsetof(PoolEntry, u) == 0, "the search kernel finds an entry from its uniforms' address");
struct PoolTable {
  uint32_t n;          // entries in use (1..kMaxSlots)
  uint32_t poll_mask;  // a wave reads the host kill word when ((it + w) & poll_mask) == 0
  uint32_t iters;      // wave iterations of this launch (the cap; bounded entries' dense span)
  uint32_t budget;     // > 0: a wave on an unbounded entry stops once this many 100-MHz
                       // s_memrealtime ticks have passed since it started (all waves stop
                       // together); 0 = iteration count only
  uint64_t yield_base;    // PoolMailbox::ctl when the table was built: a polling wave that reads
                          // a different high half ends the launch's unbounded entries
  uint32_t ring;          // PoolMailbox::clk[ring]: this launch's clock records ...
  uint32_t seq;           // ... tagged with the launch's sequence number (low 32 bits)
  uint32_t dyn_base;      // search kernels: the low half of PoolMailbox::ctl when the table was built -- the
                          // launch may also search the entries the host publishes after it
  uint32_t counted;       // search kernels: workgroups are counted on their entries (early finish,
                          // dynamic entries).  The host sets it for tables of 2 or more entries: a
                          // launch with one entry ends with it, and counting only slows its end.
  uint32_t kill_base;     // the low half of PoolMailbox::kills when the table was built: a polling wave that
                          // reads another value relays the kill words of every entry, not only its own
  uint32_t linger;        // search kernels (counted launches, round 5), > 0: a workgroup that finds no live entry
                          // waits in the launch for the host's next dynamic entry (ls2_linger) until a yield,
                          // instead of leaving -- the next search needs no launch; the value (a power of two) is
                          // the lingering workgroups' period, in looks, of reading the pinned ctl word
  uint32_t pad[4];
  PoolEntry e[kMaxSlots];
};
inline size_t pool_table_bytes(uint32_t n) { return offsetof(PoolTable, e) + (size_t)n * sizeof(PoolEntry); }

// The same table with at most kArgEntries entries, passed by value as the launch's kernel
// arguments (npow_pool_kernel_arg): its bytes are a prefix of PoolTable's.
constexpr int kArgEntries = 16;
struct PoolTableArg {
  uint8_t header[offsetof(PoolTable, e)];
  PoolEntry e[kArgEntries];
};
static_assert(offsetof(PoolTableArg, e) == offsetof(PoolTable, e), "PoolTableArg must be a prefix of PoolTable");
static_assert(sizeof(PoolTableArg) + 2 * sizeof(void*) <= 4096, "kernel arguments are limited to 4 KiB");

struct PoolSlotWord {
  unsigned long long dead;  // highest generation known dead in this slot
  uint8_t pad[56];
};
// Two-group kernels: workgroups on the slot's entry (npow_pool_kernel_ls2*; joins and leaves
// balance within every launch, so they are 0 between launches), one counter per XCD shard
// (workgroup index mod kWgsShards: 64 joins per word at a launch's start instead of 512).  Once the
// entry is dead, whoever sees every shard at 0 publishes the slot's final nonce count
// (PoolMailbox::fin).  Lines of their own: beside `dead`, which every wave loads every iteration,
// each join / leave atomic would evict that line.
constexpr int kWgsShards = 8;
struct PoolSlotCount {
  unsigned long long wgs;
  uint8_t pad[56];
};
// Word kLateWord of each done shard's line: the device-side overshoot -- nonces a workgroup hashed for the
// entry in iterations that started after one of its waves knew the entry was over (its dead word, a win, or a
// kill read by its poll), added when it leaves the entry.  Cumulative per slot like the done counts.
constexpr int kLateWord = 1;
// Workgroups that have left an uncounted (one-entry) launch, per launch ring (round 5): one counter per XCD
// shard (workgroup index mod kWgsShards), then one over the shards, each on its own line -- the last one out
// of a shard bumps `top`, the last one out of the launch publishes the entry's final count when the entry is
// over (PoolMailbox::fin, as the counted launches' last leaver does), so a won or killed one-entry job
// finishes without waiting for its launch's event and the done-count read-back behind it.  Every counter is
// back at 0 when its launch ends (the last one out resets it), ready for the ring's next launch.
struct PoolExit {
  unsigned long long shard[kWgsShards][8];
  unsigned long long top;
  uint8_t pad[56];
};
constexpr int kPoolRing = 4;  // launch ring of the pool kernels (host: kEventRing)
struct PoolDevState {
  PoolSlotWord slot[kMaxSlots];
  PoolSlotCount count[kMaxSlots][kWgsShards];
  unsigned long long done[kMaxSlots][kPoolDoneShards * 8];  // nonces hashed (word 0) and late ones (word
                                                            // kLateWord), sharded over 64-B lines
  // Per launch ring: (the launch's seq << 32) | the low half of PoolMailbox::kills up to which a wave of THAT
  // launch has relayed every kill word of its entries into the dead words (ls2_poll): one scan per kill and
  // launch, not one per poll (a 64-entry scan is 64 uncached reads).  Keyed by launch: a launch
  // holding other entries must not skip the scan because another launch relayed up to the same count.
  alignas(64) unsigned long long kills_done[kPoolRing][8];
  PoolExit exits[kPoolRing];
  // The latest PoolMailbox::ctl a lingering workgroup read from the pinned word (ls2_linger), for the other
  // lingering workgroups to read from device memory: one uncached host read per 64 lingering workgroups' looks
  // instead of one each.  Monotonic like ctl; a value older than a launch's table reads as no news (ls2_mirror_ok).
  alignas(64) unsigned long long ctl_mirror[8];
};

// Pinned host-coherent mailbox of the pool: one win record per slot (the winner stores
// nonce and value, then releases gen) and one kill word per slot the host raises.
struct alignas(64) PoolWin {
  uint64_t gen;
  uint64_t nonce;
  uint64_t value;
  uint64_t t;  // s_memrealtime (100 MHz) when the winning wave published (NANOPOW_TRACE_LATENCY timelines)
  uint8_t pad[32];
};
// In-kernel clock of a search launch: the first wave of workgroups 0..7 (one per XCD) records
// its s_memtime span (shader cycles) and s_memrealtime span (100 MHz) from its first to its
// last instruction; clock = cycles / ref * 100 MHz.  Written only here, read only by the host.
constexpr int kClkWaves = 8;
struct PoolClk {
  uint64_t cycles, ref;
  uint32_t seq, pad;
  uint64_t t0, t1;  // the recording wave's s_memrealtime at its first and last instruction (absolute, 100 MHz)
};
// Final nonce count of a closed entry (search kernels): the sum of the slot's done shards once
// no workgroup is left on it and none can join, so a won or killed job finishes without waiting
// for its launch to end (the other entries may keep it running for the rest of its budget).
struct alignas(64) PoolFin {
  uint64_t gen;    // released after total and late
  uint64_t total;  // the slot's done shards, summed (cumulative over its generations)
  uint64_t late;   // the slot's late words, summed (kLateWord; cumulative)
  uint64_t t_fin;    // s_memrealtime of the publication (NANOPOW_TRACE_LATENCY GPU timelines)
  uint64_t t_relay;  // diagnostic builds (-DNPOW_DIAG_TIMES): s_memrealtime when a poll read the slot's kill word
  uint64_t t_join;   // ... and when a workgroup last started hashing the slot's entry
  uint64_t linger_gen;  // round 6: the generation whose kill a lingering workgroup relayed (ls2_linger_relay) --
                        // an entry left live with no workgroup on it; the host counts them (stats linger_relays)
  uint8_t pad[8];
};
static_assert(sizeof(PoolFin) == 64, "one line per slot");
// An unbounded job adopted while a search launch runs joins that launch instead of ending it
// (a yield): the host writes its entry at ring position p (dyn[p % kDynRing]) and then releases
// the low half of PoolMailbox::ctl = p + 1; the launch's entries are its table's n entries followed by positions
// dyn_base.. of the ring, at most kDynEntries of them, and workgroups move to a new entry as they rebalance
// (npow_kernel.hip).  Each entry has cache lines of its own, and a position is written at most once while a launch
// that can read it runs, so no scalar-cache line can hold an older entry there.  The ring holds two launches' worth
// (round 5): a lingering launch whose kDynEntries are used up is replaced by an empty one queued behind it, and the
// next search's entry goes to positions the ending launch cannot read (Worker::dyn_add).
constexpr int kDynEntries = 32;
constexpr int kDynRing = 2 * kDynEntries;
struct alignas(64) PoolDynEntry {
  PoolEntry e;
  uint8_t pad[192 - sizeof(PoolEntry)];
};
static_assert(sizeof(PoolDynEntry) == 192, "3 cache lines per dynamic entry");
struct PoolMailbox {
  PoolWin win[kMaxSlots];
  PoolFin fin[kMaxSlots];
  PoolDynEntry dyn[kDynRing];
  uint64_t kill[kMaxSlots];  // kill[s] = gen: the job in slot s (that generation) must stop
  // High half: bumped by the host when new jobs wait for the next launch (a yield); low half: the
  // dynamic entries published (ring positions, see PoolDynEntry).  One word, so a poll reads both
  // with one uncached read.
  alignas(64) uint64_t ctl;
  // Bumped by the host after it raises any kill word of this device (round 4): a poll lands on one entry,
  // and with n live entries a kill of another entry would wait ~n polls for a wave on that entry.
  alignas(64) uint64_t kills;
  alignas(64) PoolClk clk[kPoolRing][kClkWaves];  // [launch ring][XCD] (host: kEventRing == kPoolRing)
#ifdef NPOW_DIAG_TIMES
  uint64_t diag_join[1024];  // diagnostic builds: s_memrealtime when workgroup g last started an entry
#endif
};

// Grid of a search launch: kLsGroups 512-lane workgroups per CU.  A "unit" is what an entry's share
// is counted in: a workgroup of kLsWaves waves (workgroups work on one entry at a time).
struct PoolShape {
  int grid;  // workgroups
  uint32_t units() const { return (uint32_t)grid; }
  // nonces a bounded entry e of n can cover in one launch of `iters` wave iterations
  uint64_t own(uint32_t e, uint32_t n, uint32_t iters) const {
    const uint32_t U = units();
    return (uint64_t)(U / n + (e < U % n ? 1u : 0u)) * kLsWaves * iters * 64;
  }
  uint64_t full(uint32_t iters) const { return (uint64_t)units() * kLsWaves * iters * 64; }
  // The iteration cap of a launch: with 8 waves per SIMD a wave iteration takes as long
  // as two hashes of its SIMD's other group, so half of g_iters keeps a launch's longest duration
  // (and its nonce span) where the round-1 tuning put it.
  uint32_t launch_iters(uint32_t iters) const { return iters > 1 ? iters / 2 : 1u; }
};

// Launchers (defined in npow_kernel.hip).
hipError_t launch_task(Mode mode, int grid, hipStream_t stream, const LaunchArgs& a, DevState* st,
                       HostMailbox* mb, uint64_t* out);
// bounded: the table holds a bounded entry (selects the kernel variant with per-lane range tests);
// the table in device memory (more than kArgEntries entries, uploaded in stream order before it)
hipError_t launch_pool(hipStream_t stream, int grid, const PoolTable* tab, bool bounded, PoolDevState* st,
                       PoolMailbox* mb);
// The same with the table (n <= kArgEntries) passed in the kernel arguments: no upload.
hipError_t launch_pool_arg(hipStream_t stream, int grid, const PoolTable& host_tab, bool bounded, PoolDevState* st,
                           PoolMailbox* mb);
// Fill a.u[] for one root (host).
inline void fill_uniforms(LaunchArgs& a, const RootPrecomp& pre) { npow_asm_uniforms(pre.m, a.u); }

hipError_t launch_pairs(int grid, hipStream_t stream, const uint64_t* roots_words, const uint64_t* nonces,
                        uint32_t n, uint64_t* out);

}  // namespace npow
