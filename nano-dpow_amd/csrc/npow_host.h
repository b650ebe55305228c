// npow_host.h -- host-side state shared by the engine (npow_engine.cpp: devices, sweeps,
// values, C ABI) and the work pool (npow_pool.cpp: concurrent first-win searches).
#pragma once
#include <hip/hip_runtime.h>
#include <pthread.h>

#include <atomic>
#include <condition_variable>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nanopow.h"
#include "npow_blake2b.h"
#include "npow_internal.h"

namespace npow {

// Thread-local error message behind npow_last_error().
int fail(int code, const std::string& msg);
const std::string& last_error();

#define HIPTRY(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return ::npow::fail(NPOW_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int kEventRing = 4;
static_assert(kEventRing == sizeof(PoolMailbox::clk) / sizeof(PoolMailbox::clk[0]), "one clock record set per ring");

struct Device {
  int id = 0;       // logical index (device_mask bit)
  int cpu_threads = 0;  // > 0: not a GPU but the pool's CPU workers (npow_cpu.cpp, --cpu-threads); no HIP state
  int hip_id = 0;   // HIP device (== id unless NANOPOW_VIRTUAL_DEVICES is set)
  int cus = 0;       // CUs the device's kernels run on (its partition's, see cu_first)
  bool time_shared = false;  // one of several logical devices time-sharing a GPU (NANOPOW_VIRTUAL_PARTITION=share)
  int cu_first = -1; // -1: the whole GPU; else the first CU of this logical device's partition (a CU-masked
                     // stream over [cu_first, cu_first + cus) of HIP device hip_id; npow_engine.cpp init_device)
  hipStream_t stream = nullptr;
  DevState* st = nullptr;        // device memory (sweep / values tasks)
  HostMailbox* mb = nullptr;     // pinned host (coherent), host view
  HostMailbox* mb_dev = nullptr; // device view of the same bytes
  uint64_t* d_out = nullptr;     // sweep hits / values
  hipEvent_t ev_start[kEventRing] = {};
  hipEvent_t ev_stop[kEventRing] = {};
  std::mutex mu;                 // one task (sweep / values / pool work) per device at a time
  std::atomic<int> tasks_waiting{0};  // sweep / values calls waiting for `mu` (TaskLock)
  // work pool (npow_pool.cpp)
  PoolDevState* pst = nullptr;         // device memory
  PoolMailbox* pmb = nullptr;          // pinned host (coherent), host view
  PoolMailbox* pmb_dev = nullptr;      // device view
  PoolTable* d_tab[kEventRing] = {};   // per in-flight launch
  PoolTable* h_tab[kEventRing] = {};   // pinned staging
  unsigned long long* h_done = nullptr;  // pinned read-back of every slot's done shards
  hipEvent_t ev_done[kMaxSlots] = {};    // the read-back of a retiring slot has landed
  std::thread worker;
  // statistics
  std::mutex stats_mu;
  uint64_t launches = 0, nonces = 0, invalid = 0;
  uint64_t early = 0, early_mismatch = 0;  // jobs finished from a published final count (npow_pool.cpp)
  uint64_t yields = 0, dyn = 0;            // launches yielded / jobs that joined a running launch
  uint64_t linger_ends = 0;                // lingering launches ended early (Worker::end_linger)
  uint64_t kills_relayed = 0;              // losing jobs stopped by another device's decision (npow_pool.cpp)
  uint64_t late = 0;                       // device-side overshoot: nonces hashed after the job was known over
  uint64_t watcher_decisions = 0;          // jobs the win watcher decided from this device's win records
  uint64_t stale_drains = 0;               // won / killed slots of a lingering launch whose final count had not come
                                           // 1 ms after their stop (the worker then ended the launch) ...
  uint64_t stale_late = 0;                 // ... of which the count came later after all ...
  uint64_t stale_missing = 0;              // ... or never, though every launch holding the slot ended (a protocol hole)
  double stale_gpu_delay_us = 0.0;         // the latest late count's publish after the job's deciding win (GPU clock)
  uint64_t linger_relays = 0;              // final counts that followed a kill relayed by a lingering workgroup
  double linger_ms = 0.0;                  // host-timed waits of lingering launches with nothing to hash (in kernel_ms)
  double idle_ms = 0.0;                    // GPU idle between consecutive search launches (HIP events) ...
  uint64_t idle_gaps = 0;                  // ... over this many pairs (npow_pool.cpp Worker::retire)
  // Published by the pool worker for npow_device_stats_get: it has launches or slots in flight, and
  // how many of its slots are still searching.  A job finished early returns before the launch that
  // held it is retired; with no slot searching, the stats wait for the worker to retire the rest.
  std::atomic<bool> worker_busy{false};
  std::atomic<int> active_slots{0};
  // The pool worker naps between steps on its own condition variable (round 5; it napped on g_pool.cv_work with
  // g_pool.mu, and every admission or decision then woke all the workers into a convoy on that lock): new jobs,
  // decisions and shutdown bump wake_seq (under wake_mu) and notify.
  std::mutex wake_mu;
  std::condition_variable wake_cv;
  uint64_t wake_seq = 0;
  // The win watcher (npow_pool.cpp watcher_run): the slots whose win records it watches, armed by the pool worker
  // when it adopts a job (bit s of armed_mask, the generation in armed_gen[s], the job in armed_job[s] under
  // armed_mu) and disarmed when the slot is freed.
  std::atomic<uint64_t> armed_mask{0};
  std::atomic<uint64_t> armed_gen[kMaxSlots] = {};
  std::atomic<const volatile uint32_t*> armed_cancel[kMaxSlots] = {};  // the job's caller-owned cancel word, if any
  std::atomic<double> armed_spin_until[kMaxSlots] = {};  // steady-clock us until which the watcher spins for the slot
  std::mutex armed_mu;
  std::shared_ptr<void> armed_job[kMaxSlots];  // JobP (npow_pool.h), type-erased here
  double kernel_ms = 0.0;
  double clk_ticks = 0.0, clk_ref_ticks = 0.0;  // in-kernel s_memtime / s_memrealtime spans (stats)
  std::chrono::steady_clock::time_point stats_t0 = std::chrono::steady_clock::now();
  double worker_cpu0_ms = 0.0;                   // the pool worker's thread CPU time at the last reset
  // Dropped (dead) devices: select_devices() skips them; set once, by the device's worker (or
  // npow_init) -- 3 invalid results in a row or a failed HIP call (npow_pool.cpp, fault policy).
  std::atomic<bool> dead{false};
  int dead_code = NPOW_ERR_HIP;  // the error a job gets when no device is left to search it
  std::string dead_msg;
  // Test hook (NANOPOW_TEST_HOOKS=1): HIP call sites of this device at which the calling thread's current HIP
  // device was checked, and how many were wrong (check_device below)
  std::atomic<uint64_t> affinity_checks{0}, affinity_failures{0};
  // CPU device (cpu_threads > 0): its hashing threads, for their CPU time in the stats (npow_cpu.cpp)
  std::mutex cpu_tids_mu;
  std::vector<pthread_t> cpu_tids;
};

extern std::vector<std::unique_ptr<Device>> g_devs;
extern std::atomic<uint32_t> g_iters;          // wave iterations per launch
extern std::atomic<uint32_t> g_poll;           // host-word poll interval (iterations per wave)
extern std::atomic<uint32_t> g_blocks_per_cu;  // npow_values_kernel_seq: 256-lane workgroups per CU
extern std::atomic<uint32_t> g_budget_us;      // pool launches: wall-clock budget per wave (0 = off)

inline int grid_of(const Device& d) { return d.cus * (int)g_blocks_per_cu.load(); }  // npow_values_kernel_seq
// Search, sweep and values launches of the shipped stream: kLsGroups 512-lane workgroups per CU.
inline int ls_grid(const Device& d) { return d.cus * kLsGroups; }
inline PoolShape pool_shape(const Device& d) { return PoolShape{ls_grid(d)}; }
inline uint32_t poll_mask() {
  uint32_t p = g_poll.load();
  uint32_t m = 1;
  while (m < p) m <<= 1;
  return m - 1;
}

inline void store_release(volatile uint32_t* p, uint32_t v) { __atomic_store_n((uint32_t*)p, v, __ATOMIC_RELEASE); }
inline uint32_t load_acquire(const volatile uint32_t* p) { return __atomic_load_n((const uint32_t*)p, __ATOMIC_ACQUIRE); }
inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

// A sweep / values call takes the device from the work pool: it announces itself, the pool
// worker stops launching, lets its in-flight launches end (on their budget or a win) and
// releases `mu`; the worker resumes once the call has finished.  Without the announcement a
// device kept busy by a stream of searches would never be free for the call.
class TaskLock {
 public:
  explicit TaskLock(Device& d) : d_(d), lk_(d.mu, std::defer_lock) {
    d_.tasks_waiting.fetch_add(1);
    try {
      lk_.lock();
    } catch (...) {
      d_.tasks_waiting.fetch_sub(1);
      throw;
    }
    d_.tasks_waiting.fetch_sub(1);
  }

 private:
  Device& d_;
  std::unique_lock<std::mutex> lk_;
};

// Devices selected by a mask (0 = all), excluding dead ones; select_gpus also excludes the CPU device
// (sweeps and values run on GPUs only).
std::vector<Device*> select_devices(uint64_t mask);
std::vector<Device*> select_gpus(uint64_t mask);
// Per-launch event accounting (kernel time by HIP events on the launch's own stream).
void account_launch(Device& d, int ring);

// ---- work pool (npow_pool.cpp) ----------------------------------------------------------------
bool test_hooks_enabled();          // NANOPOW_TEST_HOOKS=1: the NANOPOW_FAULT_* hooks are honoured

// Device affinity.  Every logical device runs on HIP device hip_id, and its HIP calls must come
// from a thread whose current device is that one: streams, events and memory belong to a device, and on one
// physical GPU (every test box so far) a call from the wrong device would pass unnoticed.  With test hooks on, each
// HIP call site of a device checks hipGetDevice() == d.hip_id (counted in npow_device_stats.affinity_checks); a
// mismatch is reported on stderr and the call fails with NPOW_ERR_INTERNAL (affinity_failures).  Without the hooks
// the check costs nothing.  DESIGN.md section 5 lists the call sites and the threads that reach them.
int check_device_slow(Device& d, const char* site);
extern thread_local bool t_pool_worker;  // set by a device's pool worker thread (npow_pool.cpp Worker::run)
inline int check_device(Device& d, const char* site) {
  return test_hooks_enabled() ? check_device_slow(d, site) : NPOW_OK;
}
#define DEVCHECK(d, site)                                          \
  do {                                                             \
    if (int rc_ = ::npow::check_device((d), (site))) return rc_;   \
  } while (0)
// At npow_init (always): device memory of d must be owned by HIP device d.hip_id, and the pinned mailboxes must map
// to the device pointers the kernels are given (hipPointerGetAttributes).
int check_device_memory(const void* p, const Device& d, const char* what);
int check_pinned_mapping(const void* host, const void* dev, const char* what);
int pool_device_init(Device& d);     // allocate pool buffers of one device
void pool_device_free(Device& d);
void pool_start();                   // start one worker thread per device
void pool_stop();                    // stop and join the workers (pending jobs end with an error)
bool pool_exit();                    // process exit: drain and join the workers (bounded); false: the drain timed out
int pool_submit(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t device_mask,
                uint64_t max_nonces_per_device, const volatile uint32_t* cancel, uint64_t* ticket);
// info (may be null): the search's timeline and overshoot (npow_wait_info)
int pool_wait(uint64_t ticket, int64_t timeout_us, uint64_t* nonce, uint64_t* value, uint64_t* nonces_done,
              npow_search_info* info = nullptr);
int pool_wait_result(uint64_t ticket, int64_t timeout_us, uint64_t* nonce, uint64_t* value);
int pool_cancel(uint64_t ticket);
int pool_set_max_active(uint32_t n);
void pool_counts(uint32_t* queued, uint32_t* active);

}  // namespace npow
