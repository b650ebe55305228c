/*
 * nanopow.h -- C ABI of libnanopow.so, the MI355X (gfx950) Nano proof-of-work engine.
 *
 * This library replaces the compute core of the reference's work server,
 * client/bin/windows/nano-work-server.exe (Rust + OpenCL; source not vendored,
 * upstream nanocurrency/nano-work-server v1.0).  The DPoW client never calls
 * this ABI directly: client/work_handler.py:53,75-78,104-108 talks HTTP JSON
 * to a work server, and this repository's work server
 * (nano-dpow_amd/nanopow/server.py) binds these symbols through ctypes.
 *
 * Conventions
 *   - Every function is exception-free and returns int status unless noted:
 *       NPOW_OK (0) found / done, NPOW_CANCELLED (1), NPOW_EXHAUSTED (2),
 *       negative = error; npow_last_error() then returns a thread-local message.
 *   - A root (block hash) is 32 raw bytes in the order of its hex string.
 *   - Nonces, thresholds and work values are host-endian uint64_t.  The work
 *     string a client sees is the big-endian hex of the nonce ("%016llx"),
 *     while the bytes hashed are the nonce little-endian (dpow_server.py:130).
 *   - work value = LE_u64(BLAKE2b-64(LE64(nonce) || root)); work is valid iff
 *     value >= threshold (nano-work-server.exe @1661643 `nano_work`:
 *     `if (blake2b(attempt_l, item_a) >= difficulty)`).
 *   - Buffers are caller-owned; the library keeps no pointer past a call
 *     (the `cancel` word is read only while the call runs).
 *   - A cancel word is raised from another thread with a release store
 *     (`__atomic_store_n(w, 1, __ATOMIC_RELEASE)`; an aligned 32-bit store, as
 *     ctypes makes, is one on x86-64); the library load-acquires it.
 *   - device_mask bit d selects logical device d (HIP device d, or d mod the HIP
 *     devices under NANOPOW_VIRTUAL_DEVICES, a test setting); 0 means "all devices".
 *   - Calls that use disjoint device sets may run concurrently from
 *     different threads; calls that share a device serialise on it.
 */
#ifndef NANOPOW_H
#define NANOPOW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NPOW_OK 0
#define NPOW_CANCELLED 1
#define NPOW_EXHAUSTED 2
#define NPOW_PENDING 3             /* npow_wait: timeout elapsed, the ticket is still valid */
#define NPOW_ERR_NOT_INITIALISED (-1)
#define NPOW_ERR_NO_DEVICE (-2)
#define NPOW_ERR_BAD_ARGUMENT (-3)
#define NPOW_ERR_HIP (-4)
#define NPOW_ERR_INVALID_WORK (-5) /* a job's last device was dropped for 3 invalid results in a row */
#define NPOW_ERR_CAPACITY (-6)     /* sweep found more hits than `cap` (n_out still exact) */
#define NPOW_ERR_INTERNAL (-7)     /* host-side failure (out of memory, thread creation); no C++
                                      exception ever crosses this ABI */

/* ABI revision (npow_abi_version()).  3: npow_values runs the search kernels' stream;
 * npow_values_path, npow_wait_info, npow_device_stats_get_sized added;
 * npow_device_stats_get writes only the revision-2 prefix of npow_device_stats.
 * 4: npow_config_cpu_threads (CPU workers, --cpu-threads), npow_wait_result (the outcome at the decision);
 * npow_device_stats gains late_nonces,
 * hip_device, cu_first; npow_search_info gains late_nonces_losers / late_nonces_winner (both structs
 * are written up to the size the caller passes, so revision-3 callers are unaffected).
 * 5: npow_search_info gains the search's host timeline (adopt_us, launch_us, launch_all_us, win_seen_us);
 * npow_device_stats gains idle_ms / idle_gaps (the GPU idle between the device's search launches) and
 * affinity_checks / affinity_failures (NANOPOW_TEST_HOOKS=1, since npow_init: the calling thread's HIP device checked
 * at every HIP call site of the device) and watcher_decisions.  Both structs are still written up to the size the caller passes.
 * 6: npow_device_stats gains stale_drains / stale_late / stale_missing / stale_gpu_delay_us (won or killed jobs of a
 * lingering launch whose final count had not come 1 ms after their stop; of those, the ones whose count came later and
 * the ones whose count never came -- a protocol check: 0), linger_ms (the device's lingering launches waiting with
 * nothing to hash, inside kernel_ms) and linger_relays (kills relayed by a lingering workgroup). */
#define NPOW_ABI_VERSION 6

/* Hash paths of npow_values_path. */
#define NPOW_PATH_SEARCH 0  /* the instruction stream the search and sweep kernels execute
                               (npow_hash_asm_lockstep_ld.inc, four 512-lane workgroups per CU) */
#define NPOW_PATH_SEQ 1     /* a second generated stream, scheduled without barriers (npow_hash_asm.inc) */
#define NPOW_PATH_GENERIC 2 /* plain HIP C++ of the 12 rounds, one (root, nonce) per lane */

/* Per-device counters; kernel_ms is measured with HIP events recorded on the
 * stream each kernel is launched on (bench.py's roofline leg reads these). */
typedef struct npow_device_stats {
  uint64_t launches;      /* kernel launches (search + sweep + values) */
  uint64_t nonces;        /* nonces whose hash the kernels computed */
  double kernel_ms;       /* sum of per-launch event-timed durations */
  uint64_t invalid_work;  /* GPU winners rejected by CPU re-validation */
  int32_t cus;            /* compute units */
  int32_t grid;           /* workgroups per search/sweep launch */
  double clock_mhz;       /* in-kernel shader clock of the search launches since the last reset:
                             s_memtime / s_memrealtime spans of one wave per XCD (0 = none yet) */
  double host_cpu_ms;     /* CPU time of the device's pool worker thread since the last reset */
  double host_wall_ms;    /* wall time since the last reset (host_cpu_ms / host_wall_ms = the
                             worker's share of one core) */
  int32_t dead;           /* 1 once the device has been dropped: 3 invalid results in a row
                             (nano-work-server.exe @1669144) or a failed HIP call; searches then
                             skip it and its jobs' remaining ranges move to the other devices */
  int32_t pool_groups;    /* workgroups per CU of the search kernel (npow_pool_kernel_ls2*): 4
                             512-lane ones -- 8 waves per SIMD either way; earlier ABI-3 libraries
                             ran 2 of 1,024 lanes, revisions before ABI 3 also had 0 = seq, 1 */
  uint64_t early_finishes;  /* jobs finished from the kernel's published final count (search
                               kernels): a won or killed entry's count once no workgroup is left on
                               it, before the launch that held it ends */
  uint64_t early_mismatches; /* of those, counts that the read-back after the launch contradicted
                               (always 0: a protocol check) */
  uint64_t yields;          /* running launches ended early so that new jobs could start */
  uint64_t dyn_entries;     /* jobs that joined a running launch instead (no yield) */
  /* ---- ABI 3 (npow_device_stats_get_sized only) ---- */
  uint64_t kills_relayed;   /* losing jobs of this device stopped by another device's win: the deciding
                               thread raised this device's kill word directly (no wait for its worker) */
  /* ---- ABI 4 ---- */
  uint64_t late_nonces;     /* device-side overshoot of the search kernels: nonces hashed by workgroups in
                               iterations that started after one of their waves knew the job was over (its
                               dead word, a win, a kill read by a poll) -- counted in the kernel */
  int32_t hip_device;       /* HIP device this logical device runs on (-1: the CPU workers) */
  int32_t cu_first;         /* -1: the whole GPU; else the first CU of its partition (NANOPOW_VIRTUAL_DEVICES:
                               a CU-masked stream over CUs [cu_first, cu_first + cus)) */
  /* ---- ABI 5 ---- */
  double idle_ms;           /* GPU idle on the device's stream between consecutive search launches: from one
                               launch's stop event to the next one's start event (HIP events), summed */
  uint64_t idle_gaps;       /* ... over this many pairs of consecutive launches */
  uint64_t affinity_checks; /* NANOPOW_TEST_HOOKS=1: HIP call sites of this device at which the calling thread's
                               current HIP device was checked (hipGetDevice == hip_device) ... */
  uint64_t affinity_failures; /* ... and found wrong (the call then fails: NPOW_ERR_INTERNAL) */
  uint64_t watcher_decisions; /* jobs decided by the process's win watcher from this device's win records (it spins
                                 over every live slot's record; NANOPOW_WATCHER=0 leaves them to the device's worker) */
  /* ---- ABI 6 ---- */
  uint64_t stale_drains;    /* won or killed jobs of a lingering launch whose final count the kernel had not published
                               1 ms after the stop (the worker then ended the launch and read the count back) */
  double linger_ms;         /* of kernel_ms, the time this device's lingering launches waited with nothing to hash
                               (host-timed): (kernel_ms - linger_ms) is the time the device hashed */
  uint64_t linger_relays;   /* final counts published after a lingering workgroup relayed the kill of an entry that
                               no workgroup was hashing (ls2_linger_relay; without it the count never came) */
  uint64_t stale_late;      /* of stale_drains: the count was published later after all (the GPU was late) ... */
  uint64_t stale_missing;   /* ... or never, though every launch that held the job ended: a protocol hole, 0 */
  double stale_gpu_delay_us; /* the latest such late count's publish after the job's deciding win, on the GPU's clock
                                (s_memrealtime; one clock over CU partitions of one GPU, not across GPUs) */
} npow_device_stats;

/* Outcome of one search (npow_wait_info).  Times are host steady-clock microseconds since
 * npow_submit.  For a job split over several devices, the other devices keep hashing from the
 * moment the host accepts the winner until their waves have left the job: stop_after_decide_us is
 * the longest such span among them as the host observed it (the device's worker saw the job's
 * final count or the launch that held it complete -- so an upper bound of the device time), and
 * overshoot_nonces the sum over them of that span times the device's kernel rate (likewise an
 * upper bound of the nonces hashed after the decision).  Both are 0 for a one-device job. */
typedef struct npow_search_info {
  uint32_t size;            /* set by the caller: sizeof(npow_search_info) it was compiled with */
  int32_t status;           /* as npow_wait returns it */
  uint64_t nonce, value;    /* valid when status == NPOW_OK */
  uint64_t nonces_done;     /* every device, including the rest of a launch after the win */
  int32_t winner_device;    /* logical device whose result decided the job; -1 if none */
  int32_t n_devices;        /* devices the job was split over */
  double decide_us;         /* the winner accepted (CPU re-validated) */
  double finish_us;         /* every device done with the job */
  double stop_after_decide_us;
  uint64_t overshoot_nonces;
  /* ---- ABI 4: counted on the devices (npow_device_stats.late_nonces, per job) ---- */
  uint64_t late_nonces_losers;  /* nonces the other devices' waves hashed for the job after they knew it was
                                   over (the kill relayed into their dead word); the host-side bound above
                                   adds the kill's way there and the worker's observation */
  uint64_t late_nonces_winner;  /* the same on the deciding device after its own win */
  /* ---- ABI 5: the search's host timeline (us since npow_submit; 0 = it did not happen) ---- */
  double adopt_us;          /* the first device's pool worker took the job */
  double launch_us;         /* the first launch holding it was issued (any device) */
  double launch_all_us;     /* every device of the job had issued a launch holding it */
  double win_seen_us;       /* the deciding device's winner record was read by the host (decide_us follows its CPU
                               re-validation) */
} npow_search_info;

/* CPU workers (nano-work-server.exe @1681064 `--cpu-threads N`): before npow_init, ask it to add
 * `threads` host threads (0 = none, the default; at most 1024) as one more logical device after the
 * GPUs.  Searches whose device_mask selects it (mask 0 = all devices does) give it a stride of
 * their own like a GPU; its threads hash with the library's own CPU work value (the function that
 * re-validates GPU winners), one job at a time, and the first valid result from any device decides
 * the job.  Sweeps and values run on GPUs only.  npow_init still fails without a GPU: the CPU workers
 * run beside GPUs, never instead of them.  Its npow_device_stats has hip_device = -1, cus = threads.
 * NPOW_ERR_BAD_ARGUMENT after npow_init. */
int npow_config_cpu_threads(uint32_t threads);

/* Open every visible HIP device, create its stream and buffers.
 * Replaces the work server's OpenCL device set-up for `--gpu P:D[:THREADS]`
 * (nano-work-server.exe @1681064).  Idempotent. */
int npow_init(int* n_devices);

/* Release every device resource.  Safe to call more than once. */
void npow_shutdown(void);

/* Thread-local description of the last error on this thread ("" if none). */
const char* npow_last_error(void);

/* CPU work value of one (root, nonce): the CPU re-validation the work server
 * applies to every GPU result ("GPU returned invalid work", nano-work-server.exe
 * @1669040) and the `work_validate` action (@1680400..1680528). */
uint64_t npow_work_value(const uint8_t root[32], uint64_t nonce);

/* First-win search: scan the nonce space from `start` on every device in
 * `device_mask` (device k of G starts at start + k*2^64/G, disjoint strides) until one
 * value >= threshold is found (NPOW_OK), `*cancel` becomes non-zero
 * (NPOW_CANCELLED), or every device's range [start_k, start_k + max_nonces_per_device)
 * (0 = unbounded) has been hashed without a hit (NPOW_EXHAUSTED).
 * Replaces the kernel `nano_work` (nano-work-server.exe @1661643) and the work
 * server's GPU loop behind `work_generate` (@1673856 reply fields work /
 * difficulty / multiplier, "Cancelled" @1673856).  Every GPU winner is
 * re-validated on the CPU before it is returned.
 * The search is a job of the engine's work pool (= npow_submit + npow_wait): it runs
 * in the same kernel launches as every other job in flight on those devices.
 * `cancel` may be NULL.  `nonces_done` (may be NULL) receives the number of
 * nonces hashed by all devices, including the rest of a chunk after the win. */
int npow_search(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t device_mask,
                uint64_t max_nonces_per_device, const volatile uint32_t* cancel,
                uint64_t* nonce_out, uint64_t* value_out, uint64_t* nonces_done);

/* Batched first-win search over n roots (the DPoW burst: many work_generate
 * requests in flight at once, client/work_handler.py:83-125 per client).
 * Each root i gets its own threshold and its own cancel word cancel[i]
 * (cancel itself or any entry may be NULL) and is searched by every device in
 * device_mask; up to the pool's max_active roots share each kernel launch.
 * status_out[i] is NPOW_OK / NPOW_CANCELLED / NPOW_EXHAUSTED (or an error) per
 * root; *nonces_done = nonces hashed for all roots.  Returns NPOW_OK or the
 * first negative error. */
int npow_search_batch(const uint8_t* roots, const uint64_t* thresholds, uint32_t n,
                      uint64_t device_mask, uint64_t max_nonces_per_root,
                      const volatile uint32_t* const* cancel, uint64_t* nonces_out,
                      uint64_t* values_out, int32_t* status_out, uint64_t* nonces_done);

/* ---- Work pool: asynchronous first-win searches ----------------------------------
 * Every search is a job of the engine's pool.  Jobs queue FIFO; up to max_active
 * (default and maximum 64) are live at once, and each device searches all of its
 * live jobs in ONE kernel launch (a job won or cancelled mid-launch hands its waves
 * to the others).  Replaces the work server's request queue (nano-work-server.exe
 * @1679680 `status` generating / queue_size) with concurrent service.
 *
 * npow_submit: queue a search (arguments as npow_search) and return at once with a
 * ticket.  `cancel` (may be NULL) must stay valid until npow_wait returns a final
 * status for the ticket. */
int npow_submit(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t device_mask,
                uint64_t max_nonces_per_device, const volatile uint32_t* cancel, uint64_t* ticket);

/* Wait up to timeout_us (< 0: forever) for a ticket.  Returns NPOW_PENDING on timeout
 * (the ticket stays valid), otherwise the search's final status exactly as npow_search
 * returns it; the ticket is released then.  Outputs as npow_search. */
int npow_wait(uint64_t ticket, int64_t timeout_us, uint64_t* nonce_out, uint64_t* value_out,
              uint64_t* nonces_done);

/* npow_wait with the search's outcome and timeline in *info (info->size set by the caller; the
 * library writes at most that many bytes).  Returns as npow_wait. */
int npow_wait_info(uint64_t ticket, int64_t timeout_us, npow_search_info* info);

/* The search's outcome as soon as it is known (ABI 4): NPOW_OK with nonce / value once a winner has passed
 * CPU re-validation, NPOW_CANCELLED once the cancellation is seen, NPOW_EXHAUSTED or an error when the search
 * ends so, NPOW_PENDING on timeout.  Unlike npow_wait it does not wait for the other devices of a split
 * search to stop, nor release the ticket: collect it with npow_wait / npow_wait_info afterwards (nonces_done
 * is complete only there), and keep the cancel word valid until then.  The reference work server answers a
 * work_generate as soon as its result validates (nano-work-server.exe @1669040); the JSON server here replies
 * at this point and collects the ticket after the reply. */
int npow_wait_result(uint64_t ticket, int64_t timeout_us, uint64_t* nonce_out, uint64_t* value_out);

/* Cancel a ticket (same effect as raising its cancel word). */
int npow_cancel(uint64_t ticket);

/* Jobs searched at once (1..64).  Fewer gives the oldest requests every GPU sooner
 * (lower time-to-work under load); more keeps waves busy when jobs end mid-launch. */
int npow_pool_config(uint32_t max_active);

/* Jobs queued (not yet live) and live. */
int npow_pool_status(uint32_t* queued, uint32_t* active);

/* Exhaustive sweep: every nonce in [start, start+count) (mod 2^64) whose value
 * >= threshold, written to out[0..min(n,cap)) in ascending (nonce - start)
 * order; *n_out = exact hit count.  The range is split into contiguous parts
 * over the devices in device_mask.  Returns NPOW_ERR_CAPACITY when n > cap
 * (out then holds the first cap hits), NPOW_CANCELLED if *cancel fired. */
int npow_sweep(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t count,
               uint64_t device_mask, const volatile uint32_t* cancel, uint64_t* out, uint64_t cap,
               uint64_t* n_out);

/* Work values of `count` consecutive nonces start, start+1, ... for one root,
 * computed by the instruction stream the search and sweep kernels execute
 * (npow_values_kernel_ls2: the same uniform loads, priority runs and
 * workgroup shape), so the parity tests compare that stream's full 64-bit values
 * with the CPU.  device = logical device index. */
int npow_values(int device, const uint8_t root[32], uint64_t start, uint64_t count, uint64_t* values_out);

/* The same through a chosen hash path (NPOW_PATH_SEARCH = npow_values, NPOW_PATH_SEQ,
 * NPOW_PATH_GENERIC; the generic path takes count < 2^32). */
int npow_values_path(int device, const uint8_t root[32], uint64_t start, uint64_t count, int path,
                     uint64_t* values_out);

/* Work values of n independent (root_i, nonce_i) pairs on one device
 * (generic per-lane-root GPU path; server-side validation in bulk,
 * dpow_server.py:130,365). */
int npow_values_pairs(int device, const uint8_t* roots, const uint64_t* nonces, uint32_t n,
                      uint64_t* values_out);

/* Tuning knobs (0 keeps the current value).  iters_per_launch: the iteration cap of a
 * search launch (default 8192; a launch runs half as many wave iterations, each the time of two
 * hashes of another wave of its SIMD: 8 waves share it) and the span of bounded jobs' launches;
 * poll_interval: wave iterations between a wave's polls of the host kill / yield words
 * (rounded up to a power of two; 8 waves per iteration poll grid-wide at the default 1024);
 * blocks_per_cu: 256-lane workgroups per CU of the NPOW_PATH_SEQ values kernel. */
int npow_set_tuning(uint32_t iters_per_launch, uint32_t poll_interval, uint32_t blocks_per_cu);

/* Search (work pool) launches.  budget_us: wall-clock budget of a launch (default 20000;
 * 0 = iteration count only; 0xffffffff keeps the current value).  Workgroups searching unbounded
 * jobs stop together when it runs out -- VALU issue favours a SIMD's oldest wave, so a launch
 * of a fixed iteration count would end in a tail -- and iters_per_launch is then only the cap
 * (bounded jobs always complete their dense ranges).
 * The search kernel is npow_pool_kernel_ls2*: four 512-lane workgroups per CU, with
 * early finish (a won or cancelled job returns from the count its last workgroup publishes, not
 * at the end of the launch that held it) and dynamic entries (an unbounded job submitted while a
 * launch with other live jobs runs joins that launch).  A running launch is ended early (a yield)
 * only when a new job cannot join it: a bounded job, a one-job launch, a launch within 3 ms of its
 * budget, or a full ring of 32 dynamic entries.
 * blocks_per_cu: must be 0 or 4 (the workgroups per CU of the search kernel are fixed). */
int npow_set_pool_tuning(uint32_t budget_us, uint32_t blocks_per_cu);

/* Writes the ABI-2 prefix of npow_device_stats (through dyn_entries), as callers compiled
 * against that revision allocate. */
int npow_device_stats_get(int device, npow_device_stats* out);
/* Writes min(size, sizeof(npow_device_stats)) bytes. */
int npow_device_stats_get_sized(int device, npow_device_stats* out, uint64_t size);
int npow_device_stats_reset(int device);

/* Library / kernel identification string (gfx target, build flags). */
const char* npow_version(void);
/* NPOW_ABI_VERSION of the library. */
int npow_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* NANOPOW_H */
