// npow_pool.cpp -- the work pool of libnanopow.so: every first-win search (npow_search,
// npow_search_batch, npow_submit) is a job; up to max_active jobs are searched at once,
// all of them by ONE kernel launch per device (npow_pool_kernel_ls2*), each on a disjoint
// per-device stride of its nonce space.
//
// Replaces the request queue and GPU loop of the reference work server
// (client/bin/windows/nano-work-server.exe, Rust source not vendored; behaviour from its
// strings): requests queue FIFO (@1681064 `--shuffle` is the server's choice of order),
// every GPU scans nonce chunks for the queued root, each GPU result is re-validated on the
// CPU ("GPU returned invalid work", @1669040; a GPU is dropped after 3 invalid results in a
// row, @1669144), and work_cancel ends the request with "Cancelled" (@1673856).
// The reference serves ONE root at a time; a DPoW burst (many work_generate requests in
// flight, client/work_handler.py:83-125 per client) is served here by keeping up to
// kMaxSlots roots live in every launch, so a root that is won mid-launch costs nothing:
// its workgroups move on to the other live roots (npow_kernel.hip, pool_body_ls2).
//
// A job also leaves its launch early in both directions:
// a won or killed job finishes from the final nonce count the kernel publishes once no workgroup is
// left on its entry (early_finish; PoolMailbox::fin), and a new unbounded job joins the running
// launch as a dynamic entry (dyn_add; PoolMailbox::dyn) instead of ending it (yield_if_long, now
// the fallback).  DESIGN.md section 1.
//
// Threads: one persistent worker per device (started by npow_init) owns the device's
// stream, its slot table and up to two launches in flight (the second is queued only near
// the end of the first one's budget, or at once behind a launch with no live entry left);
// callers block in pool_wait.  The
// only cross-device datum is a job's outcome: the first device whose winner passes CPU
// re-validation decides the job, the others raise their slot's kill word (pinned host
// memory that the waves poll) and retire it.  No collective, no device-to-device traffic.
//
// Fault policy (per device, never per job): a device whose winners fail CPU re-validation 3
// times in a row (across jobs), or whose HIP calls fail, is marked dead: select_devices()
// skips it from then on, and every job it held hands the part of its nonce range the device
// had not finished to the job's surviving devices (re-striding; a bounded job's range stays
// covered exactly once more).  A job fails only when no device is left to search it.
// Test hooks (environment, read once, and only with NANOPOW_TEST_HOOKS=1 beside them -- a stray
// variable in a deployment must not drop GPUs; an active hook is reported on stderr):
// NANOPOW_FAULT_INVALID=d[,d...] makes the host read a corrupted value for every win of those
// logical devices; NANOPOW_FAULT_HIP=d:n makes device d's launches fail after its n-th.
// (npow_engine.cpp: NANOPOW_FAULT_INIT=d fails npow_init on d.)
#include <hip/hip_runtime.h>
#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <pthread.h>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "npow_pool.h"

namespace npow {
namespace {

constexpr double kYieldMinUs = 1500.0;  // yield a running launch only if more budget than this is left
// ... and only if it holds fewer live unbounded jobs than this.  A new job then waits at most one
// launch budget (20 ms), small beside its time-to-work when it shares the GPU with 8+ others
// (>= 8 x ~19 ms at fffffff8), and a burst (64 live jobs, a win every ~20 ms) no longer ends
// every launch early: each early end costs the GPU the gap before the next launch starts.
constexpr int kYieldMaxLive = 8;
constexpr int kIdleSpinUs = 2000;       // an idle worker polls for new jobs this long before sleeping
constexpr double kPrelaunchUs = 2000.0;  // queue the next launch when the running one has this much budget left
constexpr double kDynMinUs = 3000.0;     // join a running launch only with this much budget left
constexpr double kFreshSpinUs = 400.0;   // poll without sleeping this long after a launch starts (quick wins)
constexpr int kInvalidStreakMax = 3;     // consecutive invalid results that drop a device (@1669144)
constexpr double kStopSpinUs = 2000.0;   // nap(): poll without sleeping this long after a slot's job stopped
// Between steps a worker with a launch in flight sleeps this long (wakes early on new jobs):
// a win is seen within it, and the thread costs ~6 % of a core instead of spinning (nap()).
// NANOPOW_POLL_US overrides (0 = spin).
const double g_poll_us = [] {
  const char* e = getenv("NANOPOW_POLL_US");
  return e ? atof(e) : 50.0;
}();
const bool g_debug = getenv("NANOPOW_DEBUG") != nullptr;
// Lingering launches (round 5, PoolTable::linger): an unbounded launch's workgroups wait in it for the next dynamic
// entry once its entries are over, so a serial client's next search joins the running launch instead of needing one.
// The worker ends a launch that has lingered g_linger_us with nothing to do (end_linger): its sleeping waves hold the
// CUs, and a serial client's next search comes within ~0.1 ms.  Measured on the 2^26-nonce regime, interleaved with
// the same roots (profiles/r05aj_linger_by_partition_regime_ab.jsonl): over 8 CU partitions of 32
// CUs the node rate goes 0.956 -> 0.98-0.99 of the devices' full rate with the p50 within +-0.05 ms; over 4, 2 and 1
// (64 CUs and more) it costs -- node rate 0.97-0.995 against 0.996-1.0, p50 0.04-0.19 ms later -- since each
// workgroup's acquire of a new entry (an L2 invalidation each) spreads their start, the more the more workgroups share
// an XCD.  So by default on only for CU partitions of at most kLingerMaxCus CUs (lingers(); a whole GPU, and so every
// physical GPU of a node, launches per search); NANOPOW_LINGER=1 / 0 forces it on / off, NANOPOW_LINGER_US sets the
// wait.  Never for logical devices that time-share a GPU (Device::time_shared).
const int g_linger_env = [] {
  const char* e = getenv("NANOPOW_LINGER");
  return e ? (e[0] == '0' ? 0 : 1) : -1;
}();
constexpr int kLingerMaxCus = 32;
static bool lingers(const Device& d) {
  if (d.time_shared) return false;
  return g_linger_env >= 0 ? g_linger_env == 1 : (d.cu_first >= 0 && d.cus <= kLingerMaxCus);
}
const uint32_t g_linger_p = [] {  // NANOPOW_LINGER_P (A/B runs): the pinned-read period in looks (a power of two)
  const char* e = getenv("NANOPOW_LINGER_P");
  uint32_t p = e ? (uint32_t)atoi(e) : 0u, q = 1;
  while (p && q < p) q <<= 1;
  return p ? q : 0u;
}();
const double g_linger_us = [] {
  const char* e = getenv("NANOPOW_LINGER_US");
  return e ? atof(e) : 1000.0;
}();
// A slot whose job finished from its published final count is freed without reading its done counts back once the
// launches that held it have completed, except every kVerifyEvery-th, which still checks the count against the
// read-back (npow_device_stats.early_mismatches).  NANOPOW_READBACK=always reads every slot back (A/B runs).
constexpr uint64_t kVerifyEvery = 16;
const bool g_readback_always = [] {
  const char* e = getenv("NANOPOW_READBACK");
  return e && strcmp(e, "always") == 0;
}();
// The win watcher (watcher_run): on by default; NANOPOW_WATCHER=0 turns it off (A/B runs)
const bool g_watcher_on = [] {
  const char* e = getenv("NANOPOW_WATCHER");
  return !(e && strcmp(e, "0") == 0);
}();
const bool g_trace_lat = getenv("NANOPOW_TRACE_LATENCY") != nullptr;
// NANOPOW_TRACE_STEPS=1: each pool worker times the parts of its steps (adopt, check_slots, read-back, launch, retire,
// nap) and prints count / total / max / calls over 50 us per part when it exits (diagnostics of the host path)
const bool g_trace_steps = getenv("NANOPOW_TRACE_STEPS") != nullptr;
// Fault injection (tests): see the header comment.
struct Faults {
  uint64_t invalid_mask = 0;  // logical devices whose wins read back corrupted
  int hip_dev = -1;           // logical device whose launches fail ...
  uint64_t hip_after = 0;     // ... after this many
};
}  // namespace
bool test_hooks_enabled() {
  static const bool on = [] {
    const char* e = getenv("NANOPOW_TEST_HOOKS");
    return e && strcmp(e, "1") == 0;
  }();
  return on;
}
namespace {
const Faults& faults() {
  static const Faults f = [] {
    Faults x;
    if (!test_hooks_enabled()) {
      if (getenv("NANOPOW_FAULT_INVALID") || getenv("NANOPOW_FAULT_HIP"))
        fprintf(stderr, "nanopow: NANOPOW_FAULT_* ignored (test hooks need NANOPOW_TEST_HOOKS=1)\n");
      return x;
    }
    if (const char* e = getenv("NANOPOW_FAULT_INVALID")) {
      for (const char* p = e; *p;) {
        char* end = nullptr;
        const long d = strtol(p, &end, 10);
        if (end == p) break;
        if (d >= 0 && d < 64) x.invalid_mask |= 1ull << d;
        p = *end ? end + 1 : end;
      }
    }
    if (const char* e = getenv("NANOPOW_FAULT_HIP")) {
      char* end = nullptr;
      x.hip_dev = (int)strtol(e, &end, 10);
      if (end && *end == ':') x.hip_after = strtoull(end + 1, nullptr, 10);
    }
    if (x.invalid_mask || x.hip_dev >= 0)
      fprintf(stderr, "nanopow: TEST HOOKS ACTIVE: corrupt wins of device mask %#llx, fail launches of device %d after %llu\n",
              (unsigned long long)x.invalid_mask, x.hip_dev, (unsigned long long)x.hip_after);
    return x;
  }();
  return f;
}

#define NPOW_DBG(...)                     \
  do {                                    \
    if (g_debug) fprintf(stderr, __VA_ARGS__); \
  } while (0)
// the same with the steady clock's time first (ms; Python's time.monotonic() * 1e3 reads the same clock)
#define NPOW_DBGT(...)                                        \
  do {                                                        \
    if (g_debug) {                                            \
      fprintf(stderr, "[%.3f] ", now_us() * 1e-3);            \
      fprintf(stderr, __VA_ARGS__);                           \
    }                                                         \
  } while (0)

}  // namespace

// -- jobs shared with the CPU workers (npow_pool.h) ---------------------------------------------
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
Pool g_pool;
std::atomic<uint64_t> g_gen{0};
std::atomic<bool> g_exiting{false};
std::atomic<double> g_exit_deadline_us{0.0};

bool exit_now() {
  if (g_exiting.load(std::memory_order_relaxed)) return true;
  const double d = g_exit_deadline_us.load(std::memory_order_relaxed);
  if (d > 0 && now_us() > d) {
    g_exiting.store(true);
    return true;
  }
  return false;
}

// -- deferred notifications (PoolLock, npow_pool.h) ----------------------------------------------
namespace {
struct Deferred {
  int depth = 0;
  bool workers = false;
  std::vector<Job*> jobs;
};
thread_local Deferred t_defer;

void notify_waiters_now(Job& j) {
  { std::lock_guard<std::mutex> g(j.wmu); }  // a waiter between its check and its wait cannot miss the notify
  j.cv.notify_all();
}

void notify_workers_now() {
  g_pool.cv_work.notify_all();
  for (auto& dp : g_devs) {
    Device& d = *dp;
    {
      std::lock_guard<std::mutex> g(d.wake_mu);
      ++d.wake_seq;
    }
    d.wake_cv.notify_one();
  }
}
}  // namespace

PoolLock::PoolLock() : lk_(g_pool.mu) { t_defer.depth++; }

PoolLock::~PoolLock() {
  lk_.unlock();
  if (--t_defer.depth > 0) return;
  // the states these wake-ups announce were all written under the lock: a thread woken now finds them
  std::vector<Job*> jobs;
  jobs.swap(t_defer.jobs);
  const bool workers = t_defer.workers;
  t_defer.workers = false;
  for (Job* j : jobs) notify_waiters_now(*j);
  if (workers) notify_workers_now();
}

// -- job state transitions (caller holds g_pool.mu) ------------------------------------------
static void notify_waiters(Job& j) {
  if (t_defer.depth > 0) {
    if (std::find(t_defer.jobs.begin(), t_defer.jobs.end(), &j) == t_defer.jobs.end()) t_defer.jobs.push_back(&j);
    return;
  }
  notify_waiters_now(j);
}

void notify_workers_locked() {
  if (t_defer.depth > 0) {
    t_defer.workers = true;
    return;
  }
  notify_workers_now();
}

void decide_locked(Job& j, int status, uint64_t nonce, uint64_t value) {
  if (j.status != kPending) return;
  j.status = status;
  j.nonce = nonce;
  j.value = value;
  j.decided.store(true, std::memory_order_release);  // the outcome above is read by waiters that acquire this
  notify_waiters(j);  // npow_wait_result returns at the decision
}

void admit_locked() {
  bool added = false;
  while (g_pool.active.size() < g_pool.max_active && !g_pool.waiting.empty()) {
    JobP j = g_pool.waiting.front();
    g_pool.waiting.pop_front();
    j->admitted = true;
    g_pool.active.push_back(j);
    added = true;
  }
  if (added) {
    g_pool.version.fetch_add(1);
    notify_workers_locked();
  }
}

void finish_locked(const JobP& j) {
  if (j->finished) return;
  if (j->status == kPending) {
    if (j->cancel_seen()) j->status = NPOW_CANCELLED;
    else if (j->lost) j->status = j->lost_code;
    else j->status = NPOW_EXHAUSTED;
    j->decided = true;
  }
  j->t_finish = now_us();
  j->finished.store(true, std::memory_order_release);
  auto it = std::find(g_pool.active.begin(), g_pool.active.end(), j);
  if (it != g_pool.active.end()) g_pool.active.erase(it);
  auto wt = std::find(g_pool.waiting.begin(), g_pool.waiting.end(), j);
  if (wt != g_pool.waiting.end()) g_pool.waiting.erase(wt);
  admit_locked();
  notify_waiters(*j);
}

// Device k of job j is finished with it (retired, exhausted, or the device failed).
void device_done_locked(const JobP& j, size_t k, double t_seen) {
  if (j->dev_done[k]) return;
  j->dev_done[k] = 1;
  j->on_dev[k] = 0;
  if (j->seen_dev[k] && j->t_stop[k] == 0) j->t_stop[k] = t_seen > 0 ? t_seen : now_us();
  if (--j->pending_devs == 0) finish_locked(j);
}

// Device k of job j is dead: hand the ranges it had not finished (j->todo[k], including any a
// failed launch pushed back) to the job's surviving devices, split evenly (re-striding), then
// release it.  With no survivor the job has lost part of its nonce space and fails.
void abandon_locked(const JobP& j, size_t k, int code, const std::string& msg) {
  if (j->dev_done[k]) return;
  std::deque<Range> rest;
  rest.swap(j->todo[k]);
  if (!j->decided && !rest.empty()) {
    // the surviving GPUs take it; the CPU device (npow_cpu.cpp) only when no GPU of the job is left
    std::vector<size_t> surv, surv_cpu;
    for (size_t k2 = 0; k2 < j->devs.size(); ++k2) {
      const Device& d2 = *g_devs[(size_t)j->devs[k2]];
      if (k2 != k && !d2.dead) (d2.cpu_threads ? surv_cpu : surv).push_back(k2);
    }
    if (surv.empty()) surv.swap(surv_cpu);
    if (surv.empty()) {
      j->lost = true;
      j->lost_code = code;
      j->err = msg;
    } else {
      const uint64_t S = surv.size();
      for (const Range& r : rest) {
        uint64_t off = 0;
        for (uint64_t i = 0; i < S; ++i) {
          const uint64_t part = r.count / S + (i < r.count % S ? 1 : 0);
          if (part) j->todo[surv[i]].push_back({r.base + off, part});
          off += part;
        }
      }
      for (size_t k2 : surv)
        if (j->dev_done[k2] && !j->todo[k2].empty()) {  // it had finished its own part: reopen
          j->dev_done[k2] = 0;
          ++j->pending_devs;
        }
      g_pool.version.fetch_add(1);
      notify_workers_locked();
    }
  }
  device_done_locked(j, k);
}

// Job j has just been decided by device k_win's result: raise the kill word of every other device
// that holds it now, instead of waiting for that device's worker to notice the decision at its next
// step (it naps up to g_poll_us between steps), and wake the napping workers.  Each slot's kill
// word is the job's generation there; a slot reused later has a larger generation, so a late store
// could not stop another job -- and cannot happen anyway: a device releases a slot only under
// g_pool.mu, after device_done_locked or a re-arm cleared on_dev.
void stop_other_devices_locked(Job& j, size_t k_win) {
  if (j.devs.size() < 2) return;
  for (size_t k = 0; k < j.devs.size(); ++k) {
    if (k == k_win || !j.on_dev[k] || j.dev_slot[k] < 0) continue;  // (a CPU device has no slot: its threads
                                                                      // read the decision themselves)
    Device& d = *g_devs[(size_t)j.devs[k]];
    __atomic_store_n(&d.pmb->kill[j.dev_slot[k]], j.dev_gen[k], __ATOMIC_RELEASE);
    __atomic_fetch_add(&d.pmb->kills, 1ull, __ATOMIC_RELEASE);  // after the kill word: every poll then relays it
    std::lock_guard<std::mutex> sg(d.stats_mu);
    d.kills_relayed++;
  }
  g_pool.decisions.fetch_add(1, std::memory_order_release);
  notify_workers_locked();
}

int index_in(const Job& j, int dev) {
  for (size_t k = 0; k < j.devs.size(); ++k)
    if (j.devs[k] == dev) return (int)k;
  return -1;
}

// Needs (under g_pool.mu): some active job wants this device.
bool wants_device_locked(int dev) {
  for (const JobP& j : g_pool.active) {
    const int k = index_in(*j, dev);
    if (k >= 0 && !j->on_dev[k] && !j->dev_done[k]) return true;
  }
  return false;
}

// -- the win watcher ------------------------------------------------------------------------------
// A device's pool worker sees its winner records only between its naps (up to g_poll_us = 50 us once a launch is
// 0.4 ms old), and over 8 devices a worker woken by a notify queues for the pool lock behind the others.  One thread
// for the whole process instead spins over the win records of every armed slot of every GPU while any job is live
// (one core; it reads pinned host memory only, no HIP call), re-validates a winner on the CPU and decides the job
// at once: the result goes to the client and the other devices' kill words go up within microseconds of the
// record landing.  The winner's worker handles the same record at its next step as before (an invalid result, the
// device's invalid streak and the slot's retirement stay its business; a job already decided is left alone).
// It also watches each armed job's cancel word (a caller's work_cancel, or another rank's first win through a shared
// word, bench.py node_time_to_work) and wakes the device's worker at once, which then stops the job's waves.
// Spinning is bounded (round 6): the watcher spins while a job armed on a slot is within its spin window
// -- three times the job's expected time to a win at its devices' rate (a win comes in it with probability 0.95),
// at least kWatchSpinUs, at most kWatchSpinMaxUs; kWatchSpinUs only when a CPU device's hashing threads share the host
// (--cpu-threads) -- or within kWatchSpinUs of a record it handled, and otherwise naps g_watch_nap_us at a time (1-us
// timer slack).  So an endless or very hard search, or an idle lingering launch, costs a fraction of a core instead of
// all of it, while a search of the expected length (the serial client's, 2-15 ms at fffffff8 on 8 GPUs or on one)
// is watched spinning: a flat 2-ms window had put the nap's delay (~10-15 us) on every search longer than 2 ms -- the
// 8-GPU time regime's fixed cost per search 6 -> 16 us on one GPU (profiles/r06f_regime1.json).
// NANOPOW_WATCH_NAP_US=0 spins always.
namespace {
constexpr double kWatchSpinUs = 2000.0;
constexpr double kWatchSpinMaxUs = 50000.0;
constexpr double kNoncesPerCuUs = 139.0;  // a CU's search rate (35.6 Gnonce/s over 256 CUs)
const double g_watch_nap_us = [] {
  const char* e = getenv("NANOPOW_WATCH_NAP_US");
  return e ? atof(e) : 20.0;
}();
struct Watch {
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int> armed{0};        // armed slots over all devices
  std::atomic<uint64_t> arms{0};    // arms so far (a new one restarts the spin window)
  bool stop = false;
  std::thread th;
};
Watch g_watch;
}  // namespace

// The slot's spin window (above): 3 x the job's expected nonces to a win / its GPU devices' rate, in [2, 50] ms.
static double spin_window_us(const Job& j) {
  bool cpu_device = false;
  double rate = 0.0;  // nonces per us
  for (const auto& dp : g_devs) cpu_device = cpu_device || dp->cpu_threads > 0;
  if (cpu_device) return kWatchSpinUs;
  for (int id : j.devs) {
    const Device& d = *g_devs[(size_t)id];
    if (!d.cpu_threads) rate += d.cus * kNoncesPerCuUs;
  }
  const double expect = 18446744073709551616.0 / (18446744073709551616.0 - (double)j.threshold + 1.0);
  const double w = rate > 0 ? 3.0 * expect / rate : kWatchSpinMaxUs;
  return std::min(kWatchSpinMaxUs, std::max(kWatchSpinUs, w));
}

void watch_arm(Device& d, int s, uint64_t gen, const JobP& j) {
  if (!g_watcher_on) return;
  d.armed_spin_until[s].store(now_us() + j->spin_us, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> g(d.armed_mu);
    d.armed_job[s] = j;
  }
  d.armed_cancel[s].store(j->cancel, std::memory_order_release);
  d.armed_gen[s].store(gen, std::memory_order_release);
  const uint64_t bit = 1ull << s;
  g_watch.arms.fetch_add(1, std::memory_order_acq_rel);  // (a napping watcher sees it within its nap: no wake-up here,
                                                         // under the pool lock; a win comes ~0.2 ms after an arm at best)
  if (!(d.armed_mask.fetch_or(bit, std::memory_order_acq_rel) & bit) &&
      g_watch.armed.fetch_add(1, std::memory_order_acq_rel) == 0) {
    { std::lock_guard<std::mutex> g(g_watch.mu); }
    g_watch.cv.notify_one();
  }
}

void watch_disarm(Device& d, int s) {
  if (!g_watcher_on) return;
  const uint64_t bit = 1ull << s;
  if (d.armed_mask.fetch_and(~bit, std::memory_order_acq_rel) & bit) g_watch.armed.fetch_sub(1, std::memory_order_acq_rel);
  std::lock_guard<std::mutex> g(d.armed_mu);  // (see watch_stop_cancel)
  d.armed_gen[s].store(0, std::memory_order_release);
  d.armed_cancel[s].store(nullptr, std::memory_order_release);
  d.armed_job[s].reset();
}

// The slot leaves the searching state: the watcher stops reading its job's cancel word.  Under armed_mu, which the
// watcher holds while it reads the word: the device cannot finish with the job before this, so the job cannot end and
// its caller free the word while the watcher reads it.
void watch_stop_cancel(Device& d, int s) {
  if (!g_watcher_on) return;
  std::lock_guard<std::mutex> g(d.armed_mu);
  d.armed_cancel[s].store(nullptr, std::memory_order_release);
}

static void wake_worker(Device& d) {
  {
    std::lock_guard<std::mutex> g(d.wake_mu);
    ++d.wake_seq;
  }
  d.wake_cv.notify_one();
}

namespace {
void watch_handle(Device& d, int s, uint64_t gen) {
  const double t_seen = now_us();
  JobP j;
  {
    std::lock_guard<std::mutex> g(d.armed_mu);
    if (d.armed_gen[s].load(std::memory_order_acquire) == gen) j = std::static_pointer_cast<Job>(d.armed_job[s]);
  }
  if (!j) return;
  const PoolWin& pw = d.pmb->win[s];
  const uint64_t n = __atomic_load_n(&pw.nonce, __ATOMIC_RELAXED);
  uint64_t v = __atomic_load_n(&pw.value, __ATOMIC_RELAXED);
  if (__atomic_load_n(&pw.gen, __ATOMIC_ACQUIRE) != gen) return;  // the record moved on meanwhile
  if ((faults().invalid_mask >> d.id) & 1) v ^= 1;                 // NANOPOW_FAULT_INVALID (tests)
  if (host_work_value(j->pre.m, n) != v || v < j->threshold) return;  // invalid: the worker's business
  PoolLock g;  // (j, a local reference, outlives it)
  const int k = index_in(*j, d.id);
  if (j->status != kPending || k < 0 || j->dev_gen[(size_t)k] != gen) return;
  decide_locked(*j, NPOW_OK, n, v);
  j->t_decide = now_us();
  j->t_win_seen = t_seen;
  j->gpu_t_win = __atomic_load_n(&pw.t, __ATOMIC_RELAXED);
  if (j->t_win == 0) j->t_win = t_seen;
  j->winner_k = k;
  stop_other_devices_locked(*j, (size_t)k);
  if (j->devs.size() < 2) notify_workers_locked();  // (stop_other_devices_locked wakes them for split jobs)
  std::lock_guard<std::mutex> sg(d.stats_mu);
  d.watcher_decisions++;
}

void watcher_run() {
  prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
  std::vector<std::vector<uint64_t>> handled(g_devs.size(), std::vector<uint64_t>(kMaxSlots, 0));
  std::vector<std::vector<uint64_t>> cancelled(g_devs.size(), std::vector<uint64_t>(kMaxSlots, 0));
  uint64_t arms_seen = g_watch.arms.load(std::memory_order_acquire);
  double t_event = now_us();  // the last arm or record change: spin until kWatchSpinUs after it
  for (uint32_t round = 0;; ++round) {
    if (g_watch.armed.load(std::memory_order_acquire) == 0) {
      std::unique_lock<std::mutex> lk(g_watch.mu);
      g_watch.cv.wait(lk, [] { return g_watch.stop || g_watch.armed.load(std::memory_order_acquire) > 0; });
      if (g_watch.stop) return;
      t_event = now_us();
    }
    if (exit_now()) return;
    if ((round & 63u) == 0) {  // (the clock every 64 rounds: a round over a few armed slots is ~0.1 us)
      const uint64_t a = g_watch.arms.load(std::memory_order_acquire);
      const double t = now_us();
      double until = t_event + kWatchSpinUs;  // the armed slots' spin windows (watch_arm)
      for (const auto& dp : g_devs) {
        for (uint64_t m = dp->armed_mask.load(std::memory_order_acquire); m; m &= m - 1)
          until = std::max(until, dp->armed_spin_until[__builtin_ctzll(m)].load(std::memory_order_relaxed));
      }
      if (a != arms_seen) {
        arms_seen = a;
      } else if (g_watch_nap_us > 0 && t > until) {
        std::unique_lock<std::mutex> lk(g_watch.mu);
        g_watch.cv.wait_for(lk, std::chrono::duration<double, std::micro>(g_watch_nap_us), [&] {
          return g_watch.stop || g_watch.arms.load(std::memory_order_acquire) != arms_seen;
        });
        if (g_watch.stop) return;
      }
    }
    for (size_t di = 0; di < g_devs.size(); ++di) {
      Device& d = *g_devs[di];
      uint64_t m = d.armed_mask.load(std::memory_order_acquire);
      while (m) {
        const int s = __builtin_ctzll(m);
        m &= m - 1;
        const uint64_t gen = d.armed_gen[s].load(std::memory_order_acquire);
        if (gen && gen != handled[di][s] && __atomic_load_n(&d.pmb->win[s].gen, __ATOMIC_ACQUIRE) == gen) {
          handled[di][s] = gen;
          watch_handle(d, s, gen);
          t_event = now_us();
        }
        if (gen && gen != cancelled[di][s] && d.armed_cancel[s].load(std::memory_order_acquire)) {
          bool raised;
          {
            std::lock_guard<std::mutex> g(d.armed_mu);  // (watch_stop_cancel)
            const volatile uint32_t* c = d.armed_cancel[s].load(std::memory_order_acquire);
            raised = c && load_acquire(c);
          }
          if (raised) {
            cancelled[di][s] = gen;
            wake_worker(d);  // its check_slots sees the cancel word and raises the slot's kill word
          }
        }
      }
    }
    cpu_relax();
  }
}
}  // namespace

namespace {

// -- one device's worker ------------------------------------------------------------------------
enum class SlotState { kFree, kActive, kDraining };

struct Slot {
  SlotState state = SlotState::kFree;
  JobP job;
  size_t k = 0;            // the device's index within job->devs
  uint64_t gen = 0;
  uint64_t baseline = 0;   // done counter of this slot index at its last retirement
  uint64_t late_base = 0;  // ... and its late counter (kLateWord)
  bool win_seen = false;
  bool requeue = false;    // invalid GPU result: hand the job back to this device after retiring
  bool no_more = false;    // bounded range fully issued
  bool readback = false;   // done-shard read-back queued (ev_done[slot] marks it)
  bool no_readback = false;  // finished early and not sampled for verification: freed once inflight is empty
  bool fresh = false;      // adopted since the last launch was built
  bool new_job = false;    // adopted for the first time on this device (not a re-adoption)
  bool fin_seen = false;   // the kernel published this generation's final count (PoolMailbox::fin) ...
  bool early = false;      // ... and the job was finished from it before retiring
  double stop_us = 0;      // the job was won or killed at this time: the worker polls without napping
                           // until the slot's final count is in (a quick return, and an exact stop time)
  bool stale = false;      // its final count had not come g_linger_us after stop_us (npow_device_stats.stale_drains)
  struct Issued {
    uint64_t seq, base, count;
  };
  std::vector<Issued> inflight;  // ranges handed to launches that have not completed (in order)
  uint64_t unread = 0;           // bounded job: nonces of its completed ranges whose done shards have not
                                 // been read back (a failed device's fail_all counts them from this)
};

struct PoolInflight {
  uint64_t seq;
  int ring;
  uint64_t dyn_base;    // PoolTable::dyn_base of the launch
  uint64_t yield_base;  // PoolTable::yield_base of the launch
  bool counted;         // PoolTable::counted: early finish and dynamic entries are on in it
  bool linger;          // PoolTable::linger: its workgroups wait for dynamic entries until its budget or a yield
};

class Worker {
 public:
  explicit Worker(Device& d) : d_(d) {}
  void run();

 private:
  Device& d_;
  Slot slots_[kMaxSlots];
  std::deque<PoolInflight> q_;
  uint64_t seq_ = 0;  // launches issued by this worker
  uint64_t retired_seq_ = 0;  // the last launch retire() has dropped (launches retire in order)
  uint64_t seen_version_ = ~0ull;
  int ring_ = 0;
  std::chrono::steady_clock::time_point front_start_{};  // host estimate of the running launch's start
  uint64_t yields_ = 0;
  uint64_t ctl_ = 0;  // PoolMailbox::ctl (only this worker writes it): yields << 32 | dynamic entries
  uint64_t wake_seen_ = 0;  // Device::wake_seq as of this worker's last nap
  uint64_t early_count_ = 0;  // slots finished early so far (every kVerifyEvery-th is still read back)
  double idle_since_ = 0;     // launches in flight but no live slot since (end_linger after g_linger_us), 0 = busy
  double linger_t_ = 0;       // the last step that found a lingering launch idle (npow_device_stats.linger_ms), 0 = none
  int invalid_streak_ = 0;  // consecutive winners of this device that failed CPU re-validation
  int prev_stop_ring_ = -1;  // ring of the last retired launch (its stop event: the GPU idle before the next one),
                             // -1 when a sweep / values task used the device's events since
  uint64_t prev_g1_ = 0;     // NANOPOW_TRACE_LATENCY: the previous launch's end on the GPU clock
  struct StepProf {
    uint64_t n = 0, slow = 0;
    double total = 0, max = 0;
  };
  StepProf prof_[6];  // NANOPOW_TRACE_STEPS: adopt, check_slots, queue_readbacks, launch, retire, nap
  template <class F>
  auto timed(int part, F&& f) {
    if (!g_trace_steps) return f();
    const double t = now_us();
    auto r = f();
    const double dt = now_us() - t;
    StepProf& p = prof_[part];
    p.n++;
    p.total += dt;
    p.max = std::max(p.max, dt);
    if (dt > 50.0) p.slow++;
    return r;
  }
  void print_prof() const {
    static const char* names[6] = {"adopt", "check_slots", "read-back", "launch", "retire", "nap"};
    for (int i = 0; i < 6; ++i)
      fprintf(stderr, "nanopow-steps[%d] %-11s n %llu total_ms %.1f mean_us %.2f max_us %.1f over50us %llu\n", d_.id,
              names[i], (unsigned long long)prof_[i].n, prof_[i].total * 1e-3,
              prof_[i].n ? prof_[i].total / prof_[i].n : 0.0, prof_[i].max, (unsigned long long)prof_[i].slow);
  }
  std::unique_lock<std::mutex> dev_lock_{d_.mu, std::defer_lock};

  bool busy() const {
    if (!q_.empty()) return true;
    for (const Slot& s : slots_)
      if (s.state != SlotState::kFree) return true;
    return false;
  }
  void adopt();
  void yield_if_long();
  bool dyn_add(int s);
  bool live_slot() const {  // a slot some launch in flight (or a dynamic entry) is hashing
    for (const Slot& sl : slots_)
      if (sl.state == SlotState::kActive && !sl.fresh) return true;
    return false;
  }
  void end_linger();
  void handle_win(int s);
  bool win_published(int s) const;
  void early_finish(int s);
  // A stale slot's final count came after all (late): how late on the GPU's clock, after the job's deciding win at tw
  // (Job::gpu_t_win, read by the caller under g_pool.mu; npow_device_stats.stale_gpu_delay_us; one clock for CU
  // partitions of one GPU)
  void stale_fin_came(int s, uint64_t tw) {
    const uint64_t tf = __atomic_load_n(&d_.pmb->fin[s].t_fin, __ATOMIC_RELAXED);
    std::lock_guard<std::mutex> sg(d_.stats_mu);
    d_.stale_late++;
    if (tw && tf > tw) d_.stale_gpu_delay_us = std::max(d_.stale_gpu_delay_us, (double)(tf - tw) / 100.0);
  }
  void publish_busy() {
    int active = 0;
    for (const Slot& s : slots_) active += s.state == SlotState::kActive ? 1 : 0;
    d_.active_slots.store(active, std::memory_order_release);
    d_.worker_busy.store(busy(), std::memory_order_release);
  }
  void check_slots();
  int launch(bool empty_linger = false);
  int queue_readbacks();
  int retire();
  void fail_all(const std::string& msg);
  uint64_t push_back_locked(Slot& sl, size_t from, bool skip_done = false);
  bool launch_completed(uint64_t seq) const;
  bool launch_started(uint64_t seq) const;
  void account_clock(int ring, uint64_t seq, uint64_t* t0 = nullptr, uint64_t* t1 = nullptr);
  int step();
  void nap();
};

void Worker::adopt() {
  if (d_.dead) return;  // draining before it releases its jobs (run())
  const uint64_t v = g_pool.version.load();
  if (v == seen_version_) return;
  bool adopted = false;
  std::lock_guard<std::mutex> g(g_pool.mu);
  seen_version_ = g_pool.version.load();
  for (const JobP& j : std::vector<JobP>(g_pool.active)) {  // copy: device_done_locked may erase
    const int k = index_in(*j, d_.id);
    if (k < 0 || j->on_dev[k] || j->dev_done[k]) continue;
    if (j->decided || j->todo[k].empty()) {  // decided before this device got to it, or nothing left
      device_done_locked(j, k);
      continue;
    }
    int s = 0;
    while (s < kMaxSlots && slots_[s].state != SlotState::kFree) ++s;
    if (s == kMaxSlots) {  // cannot happen while max_active <= kMaxSlots; retry later
      seen_version_ = ~0ull;
      break;
    }
    Slot& sl = slots_[s];
    sl.state = SlotState::kActive;
    sl.job = j;
    sl.k = (size_t)k;
    sl.gen = ++g_gen;
    sl.win_seen = sl.requeue = sl.no_more = sl.readback = sl.fin_seen = sl.early = sl.no_readback = false;
    sl.stop_us = 0;
    sl.stale = false;
    sl.unread = 0;
    sl.fresh = true;
    sl.inflight.clear();
    j->on_dev[k] = 1;
    j->dev_slot[k] = s;
    j->dev_gen[k] = sl.gen;
    watch_arm(d_, s, sl.gen, j);
    if (j->t_adopt == 0) j->t_adopt = now_us();
    sl.new_job = !j->seen_dev[k];
    if (sl.new_job) adopted = true;  // a new job: worth ending a long launch for
    j->seen_dev[k] = 1;
  }
  // Unbounded jobs join the running launch as dynamic entries (no yield: the launch goes
  // on and workgroups move to them); a new job that cannot ends the long launch instead.
  bool waiting_new = false;
  const uint64_t ctl0 = ctl_;
  for (int s = 0; s < kMaxSlots; ++s) {
    Slot& sl = slots_[s];
    if (sl.state != SlotState::kActive || !sl.fresh) continue;
    if (!dyn_add(s) && sl.new_job) waiting_new = true;
  }
  // the entries published together (one release after all of them): workgroups of a lingering launch that see them
  // spread over all of them at once, where one at a time they would crowd onto the first and rebalance slowly
  if (ctl_ != ctl0) __atomic_store_n(&d_.pmb->ctl, ctl_, __ATOMIC_RELEASE);
  if (adopted && waiting_new) yield_if_long();
}

// Publish the job of fresh slot s as a dynamic entry of the running launch (npow_internal.h
// PoolDynEntry): exactly one launch in flight, enough of its budget left,
// not yielded, a free ring position, an unbounded job with a full region left, and either another live entry in it
// (workgroups to move) or a lingering launch (its workgroups wait for one).  Or (round 5) of the lingering launch
// queued behind an ending one whose ring is used up (step(): the replacement), at positions the ending one cannot
// read.  Its region is taken from the job's queue as launch() would, and counts as part of that launch.  Caller
// holds g_pool.mu (adopt()), and releases PoolMailbox::ctl after its calls.
bool Worker::dyn_add(int s) {
  Slot& sl = slots_[s];
  Job& j = *sl.job;
  if (q_.empty() || q_.size() > 2 || j.max_per_dev || g_budget_us.load() == 0) return false;
  const PoolShape sh = pool_shape(d_);
  const PoolInflight& f = q_.back();
  if (!f.counted) return false;  // a one-entry launch: the new job ends it (a yield) instead
  if ((uint32_t)((uint32_t)ctl_ - (uint32_t)f.dyn_base) >= (uint32_t)kDynEntries) return false;
  if ((ctl_ >> 32) != (f.yield_base >> 32)) return false;  // it is ending
  if (q_.size() == 2) {
    // the queued launch: a lingering one behind a launch that cannot see its ring positions (its own kDynEntries
    // were used up before this one was built: ring positions dyn_base .. dyn_base + kDynEntries - 1 of each, and
    // the ring holds both); it starts as soon as the other one's workgroups have left
    if (!f.linger || (uint32_t)(f.dyn_base - (uint32_t)q_.front().dyn_base) < (uint32_t)kDynEntries) return false;
  } else {
    bool other = false;  // another live entry keeps the launch running (workgroups to move)
    for (int k = 0; k < kMaxSlots && !other; ++k)
      other = k != s && slots_[k].state == SlotState::kActive && !slots_[k].fresh;
    if (!other && !f.linger) return false;  // they are leaving: the next launch, right after, takes the job
    const double left_us = g_budget_us.load() - std::chrono::duration<double, std::micro>(
                                                    std::chrono::steady_clock::now() - front_start_).count();
    if (left_us < kDynMinUs) return false;  // the next launch, queued soon, takes it
  }
  const uint32_t iters = sh.launch_iters(g_iters.load());
  const uint64_t full = sh.full(iters);
  std::deque<Range>& todo = j.todo[sl.k];
  if (todo.empty() || todo.front().count < full) return false;
  PoolEntry& pe = d_.pmb->dyn[(uint32_t)ctl_ % kDynRing].e;
  memcpy(pe.u, j.u, sizeof(pe.u));
  pe.threshold = j.threshold;
  pe.gen = sl.gen;
  pe.slot = (uint32_t)s;
  pe.bounded = 0;
  Range& r = todo.front();
  pe.base = r.base;
  pe.count = full;
  r.base += full;
  r.count -= full;
  if (r.count == 0) todo.pop_front();
  sl.inflight.push_back({f.seq, pe.base, pe.count});
  if (todo.empty()) sl.no_more = true;
  sl.fresh = false;
  {
    const double t = now_us();
    if (j.t_launch == 0) j.t_launch = t;
    if (j.t_launch_dev[sl.k] == 0) j.t_launch_dev[sl.k] = t;
  }
  ctl_ = (ctl_ & ~0xffffffffull) | (uint32_t)(ctl_ + 1);  // the low half wraps on its own (released by adopt())
  {
    std::lock_guard<std::mutex> sg(d_.stats_mu);
    d_.dyn++;
  }
  NPOW_DBGT("nanopow[%d]: dynamic entry %u: slot %d g%llu in launch %llu\n", d_.id, (uint32_t)ctl_ - 1u,
           s, (unsigned long long)sl.gen, (unsigned long long)f.seq);
  return true;
}

// New jobs wait for the next launch's table.  Launches run for a long time budget (their
// start costs ~0.1-0.2 ms of cold instruction/scalar caches, so long launches are faster), so
// when the running launch still has a while to go, end its unbounded entries now: bump the
// pinned yield word (polling waves mark those entries dead) and hand their jobs back for
// re-adoption with new generations next to the new ones.
void Worker::yield_if_long() {
  if (q_.empty() || g_budget_us.load() == 0) return;
  const double left_us = g_budget_us.load() - std::chrono::duration<double, std::micro>(
                                                  std::chrono::steady_clock::now() - front_start_).count();
  NPOW_DBG("nanopow[%d]: yield? inflight %zu left_us %.0f\n", d_.id, q_.size(), left_us);
  if (q_.size() < 2 && left_us < kYieldMinUs) return;
  int live = 0;
  for (const Slot& sl : slots_)
    if (sl.state == SlotState::kActive && !sl.fresh && !sl.job->max_per_dev) ++live;
  if (live >= kYieldMaxLive) return;
  bool any = false;
  for (Slot& sl : slots_) {
    if (sl.state != SlotState::kActive || sl.fresh || sl.job->max_per_dev) continue;
    sl.requeue = true;
    sl.state = SlotState::kDraining;
    watch_stop_cancel(d_, (int)(&sl - slots_));
    any = true;
  }
  NPOW_DBG("nanopow[%d]: yield %s\n", d_.id, any ? "raised" : "(no slot to hand back)");
  if (any) {
    ctl_ += 1ull << 32;
    __atomic_store_n(&d_.pmb->ctl, ctl_, __ATOMIC_RELEASE);
    ++yields_;
    std::lock_guard<std::mutex> sg(d_.stats_mu);
    d_.yields++;
  }
}

// A win published for slot s (this generation): CPU re-validation decides the job.
void Worker::handle_win(int s) {
  const double t_seen = now_us();
  Slot& sl = slots_[s];
  Job& j = *sl.job;
  PoolWin& pw = d_.pmb->win[s];
  sl.win_seen = true;
  const uint64_t n = __atomic_load_n(&pw.nonce, __ATOMIC_RELAXED);
  uint64_t v = __atomic_load_n(&pw.value, __ATOMIC_RELAXED);
  if ((faults().invalid_mask >> d_.id) & 1) v ^= 1;  // NANOPOW_FAULT_INVALID (tests)
  const uint64_t cpu_v = host_work_value(j.pre.m, n);
  PoolLock g;  // (the slot holds the job)
  if (j.t_win == 0) j.t_win = t_seen;
  if (cpu_v == v && v >= j.threshold) {
    invalid_streak_ = 0;
    if (j.status == kPending) {
      decide_locked(j, NPOW_OK, n, v);
      j.t_decide = now_us();
      j.t_win_seen = t_seen;
      j.gpu_t_win = __atomic_load_n(&pw.t, __ATOMIC_RELAXED);
      j.winner_k = (int)sl.k;
      stop_other_devices_locked(j, sl.k);
    }
  } else {
    // "GPU returned invalid work": the launches that held this generation stopped at the win,
    // so a bounded job gets back every range from the one holding the winner on; the job is
    // re-armed on this device after the slot retires.  The third in a row drops the device.
    {
      std::lock_guard<std::mutex> sg(d_.stats_mu);
      d_.invalid++;
    }
    fprintf(stderr, "nanopow: GPU %d returned invalid work %016llx (value %016llx, cpu %016llx)\n", d_.id,
            (unsigned long long)n, (unsigned long long)v, (unsigned long long)cpu_v);
    if (j.max_per_dev) {
      size_t from = 0;
      for (size_t i = 0; i < sl.inflight.size(); ++i)
        if (n - sl.inflight[i].base < sl.inflight[i].count) {
          from = i;
          break;
        }
      push_back_locked(sl, from);
    }
    sl.requeue = true;
    if (++invalid_streak_ >= kInvalidStreakMax && !d_.dead) {
      d_.dead_code = NPOW_ERR_INVALID_WORK;
      d_.dead_msg = "GPU " + std::to_string(d_.id) + " returned invalid work " + std::to_string(kInvalidStreakMax) +
                    " consecutive times";
      d_.dead = true;
      fprintf(stderr, "nanopow: %s, dropping it\n", d_.dead_msg.c_str());
    }
  }
  sl.state = SlotState::kDraining;  // the winning wave already marked the slot dead on the device
  watch_stop_cancel(d_, (int)(&sl - slots_));
  sl.stop_us = now_us();
}

// Ranges sl.inflight[from..] did not complete (their launches stopped on this generation or
// failed): hand them back to the front of the job's queue for this device, in order.  With
// skip_done, a range whose launch has already completed on the GPU (retire() has not seen it yet)
// stays: it was hashed in full, and handing it back would hash it again and over-count the job's
// nonces_done (a dropped device's check_slots / fail_all).  Returns the nonces of the ranges kept.
uint64_t Worker::push_back_locked(Slot& sl, size_t from, bool skip_done) {
  Job& j = *sl.job;
  std::vector<Slot::Issued> keep(sl.inflight.begin(), sl.inflight.begin() + (ptrdiff_t)from);
  uint64_t kept = 0;
  for (size_t i = sl.inflight.size(); i > from; --i) {
    const Slot::Issued& r = sl.inflight[i - 1];
    if (skip_done && launch_completed(r.seq)) {
      keep.insert(keep.begin() + (ptrdiff_t)from, r);
      kept += r.count;
      continue;
    }
    j.todo[sl.k].push_front({r.base, r.count});
  }
  sl.inflight.swap(keep);
  return kept;
}

// The launch with sequence number seq has begun on the GPU: retired, or the start event recorded
// right before it on the stream has fired (the launches ahead of it are done).
bool Worker::launch_started(uint64_t seq) const {
  if (seq <= retired_seq_) return true;
  (void)check_device(d_, "launch_started");
  for (const PoolInflight& f : q_)
    if (f.seq == seq) return hipEventQuery(d_.ev_start[f.ring]) == hipSuccess;
  return false;
}

// The launch with sequence number seq has completed on the GPU: retire() has dropped it, or its
// stop event has fired.  A launch whose issue failed (its ranges were assigned, then the HIP call
// failed: never in q_) has not.
bool Worker::launch_completed(uint64_t seq) const {
  if (seq <= retired_seq_) return true;
  (void)check_device(d_, "launch_completed");
  for (const PoolInflight& f : q_)
    if (f.seq == seq) return hipEventQuery(d_.ev_stop[f.ring]) == hipSuccess;
  return false;
}

// The launch's in-kernel clock records (PoolClk, one per XCD) into the device statistics.
void Worker::account_clock(int ring, uint64_t seq, uint64_t* t0, uint64_t* t1) {
  double cyc = 0, ref = 0;
  for (int x = 0; x < kClkWaves; ++x) {
    const PoolClk& c = d_.pmb->clk[ring][x];
    if (__atomic_load_n(&c.seq, __ATOMIC_ACQUIRE) != (uint32_t)seq) continue;
    if (t0) {  // the launch's span on the GPU's realtime clock: the earliest start, the latest end of the records
      const uint64_t a = __atomic_load_n(&c.t0, __ATOMIC_RELAXED), b = __atomic_load_n(&c.t1, __ATOMIC_RELAXED);
      if (*t0 == 0 || a < *t0) *t0 = a;
      if (b > *t1) *t1 = b;
    }
    const double cy = (double)__atomic_load_n(&c.cycles, __ATOMIC_RELAXED);
    const double rf = (double)__atomic_load_n(&c.ref, __ATOMIC_RELAXED);
    // a record from a wave that ran for a few ticks only (a launch that found its job already over) is
    // too coarse to price, and a clock outside 0.3-4 GHz is not a clock: skip both
    if (rf < 1000.0 || cy < 3.0 * rf || cy > 40.0 * rf) continue;
    cyc += cy;
    ref += rf;
  }
  std::lock_guard<std::mutex> sg(d_.stats_mu);
  d_.clk_ticks += cyc;
  d_.clk_ref_ticks += ref;
}

bool Worker::win_published(int s) const {
  const Slot& sl = slots_[s];
  return !sl.win_seen && __atomic_load_n(&d_.pmb->win[s].gen, __ATOMIC_ACQUIRE) == sl.gen;
}

// The kernel published slot s's final nonce count (npow_kernel.hip "Early
// finish"): no workgroup is on the entry and none can join it, so a decided job is finished now
// instead of after the launch -- which its other entries may keep running for the rest of its
// budget.  A yielded entry (the job is re-adopted) or an invalid win (re-armed) waits for retire().
void Worker::early_finish(int s) {
  const double t_obs = now_us();  // the device's stop as this worker saw it (not when it got the pool lock)
  Slot& sl = slots_[s];
  sl.fin_seen = true;
  if (win_published(s)) handle_win(s);  // the winner released its record before closing the entry
  const uint64_t total = __atomic_load_n(&d_.pmb->fin[s].total, __ATOMIC_RELAXED);
  const uint64_t late = __atomic_load_n(&d_.pmb->fin[s].late, __ATOMIC_RELAXED);
  PoolLock g;  // (the slot holds the job)
  Job& j = *sl.job;
  if (g_trace_lat && j.gpu_t_win) {  // GPU timeline (one GPU's clock: CU partitions), from the deciding win
    const double tw = (double)j.gpu_t_win, tr = (double)__atomic_load_n(&d_.pmb->fin[s].t_relay, __ATOMIC_RELAXED);
    fprintf(stderr, "[%.3f] nanopow-fin dev %d ticket %llu: relay %+.1f fin %+.1f seen %+.1f us (host) from the win%s\n",
            now_us() * 1e-3, d_.id, (unsigned long long)j.ticket, (tr - tw) / 100.0,
            ((double)__atomic_load_n(&d_.pmb->fin[s].t_fin, __ATOMIC_RELAXED) - tw) / 100.0,
            j.t_win_seen > 0 ? now_us() - j.t_win_seen : -1.0, (int)sl.k == j.winner_k ? " (winner)" : "");
#ifdef NPOW_DIAG_TIMES
    // absolute GPU times (100 MHz) of this entry's last start and its win, host times (us) of its launch / dynamic
    // entry and of its win seen: a serial client's gap between one search's win and the next one's hashing
    fprintf(stderr, "nanopow-join dev %d ticket %llu: gpu_join %llu gpu_win %llu host_launch %.1f host_win_seen %.1f\n",
            d_.id, (unsigned long long)j.ticket,
            (unsigned long long)__atomic_load_n(&d_.pmb->fin[s].t_join, __ATOMIC_RELAXED),
            (unsigned long long)j.gpu_t_win, j.t_launch_dev[sl.k], j.t_win_seen);
    {  // every workgroup's last entry start (a serial client: this search's) -- its spread
      std::vector<uint64_t> tj;
      const int G = ls_grid(d_) < 1024 ? ls_grid(d_) : 1024;
      for (int g = 0; g < G; ++g) tj.push_back(__atomic_load_n(&d_.pmb->diag_join[g], __ATOMIC_RELAXED));
      std::sort(tj.begin(), tj.end());
      fprintf(stderr, "nanopow-joins dev %d ticket %llu: min %llu p10 %llu p50 %llu p90 %llu max %llu\n", d_.id,
              (unsigned long long)j.ticket, (unsigned long long)tj[0], (unsigned long long)tj[G / 10],
              (unsigned long long)tj[G / 2], (unsigned long long)tj[G * 9 / 10], (unsigned long long)tj[G - 1]);
    }
#endif
  }
  if (__atomic_load_n(&d_.pmb->fin[s].linger_gen, __ATOMIC_RELAXED) == sl.gen) {  // relayed by a lingering workgroup
    std::lock_guard<std::mutex> sg(d_.stats_mu);
    d_.linger_relays++;
  }
  if (sl.stale) stale_fin_came(s, j.gpu_t_win);
  if (d_.dead || sl.requeue || !j.decided.load()) return;
  sl.early = true;
  const uint64_t delta = total - sl.baseline;
  sl.baseline = total;  // retire() then reads back the same total: a delta of 0
  j.done += delta;
  j.late[sl.k] += late - sl.late_base;
  {
    std::lock_guard<std::mutex> sg(d_.stats_mu);
    d_.late += late - sl.late_base;
  }
  sl.late_base = late;
  if (g_trace_lat && j.t_kend == 0) j.t_kend = now_us();
  {
    std::lock_guard<std::mutex> sg(d_.stats_mu);
    d_.nonces += delta;
    d_.early++;
  }
  device_done_locked(sl.job, sl.k, t_obs);
}

void Worker::check_slots() {
  for (int s = 0; s < kMaxSlots; ++s) {
    Slot& sl = slots_[s];
    if (sl.state == SlotState::kFree) continue;
    if (win_published(s)) {
      handle_win(s);
      continue;
    }
    if (sl.state != SlotState::kActive) continue;
    Job& j = *sl.job;
    if (d_.dead) {  // dropped device: stop every job's waves; retire() re-strides them
      if (j.max_per_dev) {  // the killed launches leave their ranges unfinished: hand them back
        std::lock_guard<std::mutex> g(g_pool.mu);
        push_back_locked(sl, 0, true);
      }
      __atomic_store_n(&d_.pmb->kill[s], sl.gen, __ATOMIC_RELEASE);
      __atomic_fetch_add(&d_.pmb->kills, 1ull, __ATOMIC_RELEASE);
      sl.state = SlotState::kDraining;
      watch_stop_cancel(d_, (int)(&sl - slots_));
    } else if (j.decided.load(std::memory_order_relaxed) || j.cancel_seen()) {
      {
        PoolLock g;  // (the slot holds the job)
        if (!j.decided.load()) {
          j.cancel_req = true;
          decide_locked(j, NPOW_CANCELLED);
        }
        // No launch holds the job on this device (adopted, waiting for the next launch's table): it hashes
        // nothing more of it, from now.  Otherwise the stop time (Job::t_stop) is taken when this worker sees
        // it stop hashing: its final count published, or the last launch that held it completed (retire()).
        // A launch queued behind another and started after the kill still hashes the job until one of its
        // waves polls the kill word (within an iteration), so "not started at the decision" is no proof of zero.
        if (sl.inflight.empty() && j.t_stop[sl.k] == 0) j.t_stop[sl.k] = now_us();
      }
      __atomic_store_n(&d_.pmb->kill[s], sl.gen, __ATOMIC_RELEASE);  // in-flight waves stop
      __atomic_fetch_add(&d_.pmb->kills, 1ull, __ATOMIC_RELEASE);
      sl.state = SlotState::kDraining;
      watch_stop_cancel(d_, (int)(&sl - slots_));
      sl.stop_us = now_us();
    } else if (sl.no_more) {
      sl.state = SlotState::kDraining;
      watch_stop_cancel(d_, (int)(&sl - slots_));
    }
  }
  publish_busy();  // before a job can finish early: its waiter may read the stats at once
  for (int s = 0; s < kMaxSlots; ++s) {
    const Slot& sl = slots_[s];
    if (sl.state == SlotState::kDraining && !sl.fin_seen &&
        __atomic_load_n(&d_.pmb->fin[s].gen, __ATOMIC_ACQUIRE) == sl.gen)
      early_finish(s);
  }
}

// No live entry in the launches in flight, and something waits for the device (a job that could not join them, a
// sweep / values task, shutdown, a dropped device): a lingering launch would hold the device until its budget ends
// (up to 20 ms), so end it now -- a yield (the high half of PoolMailbox::ctl), which its lingering workgroups read
// within a look (ls2_linger) and which ends nothing else, no entry being live.  Raised before the next table is built
// (launch() takes yield_base after it), so that launch is not ended too.
void Worker::end_linger() {
  bool lingering = false;
  for (const PoolInflight& f : q_) lingering = lingering || (f.linger && (f.yield_base >> 32) == (ctl_ >> 32));
  if (!lingering) return;
  ctl_ += 1ull << 32;
  __atomic_store_n(&d_.pmb->ctl, ctl_, __ATOMIC_RELEASE);
  NPOW_DBGT("nanopow[%d]: lingering launch ended (ctl %llx)\n", d_.id, (unsigned long long)ctl_);
  std::lock_guard<std::mutex> sg(d_.stats_mu);
  d_.linger_ends++;
}

int Worker::launch(bool empty_linger) {
  if (q_.size() >= 2 || d_.dead) return NPOW_OK;
  // The second launch in flight only has to be queued before the running one ends (its budget
  // is known): queued early, it would sit behind a launch that a win ends, and the job could
  // only be retired after it too had started and drained (~20 us of every search's latency).
  // ... unless no live entry is left in it (its jobs won or were killed: it ends within a hash, and a
  // job finished early returns before that) -- then the next launch queues behind it at once.
  if (q_.size() == 1 && g_budget_us.load() > 0 &&
      std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - front_start_).count() <
          (double)g_budget_us.load() - kPrelaunchUs) {
    bool live = false;
    for (int k = 0; k < kMaxSlots && !live; ++k) live = slots_[k].state == SlotState::kActive && !slots_[k].fresh;
    if (live) return NPOW_OK;
  }
  const PoolShape sh = pool_shape(d_);
  const uint32_t iters = sh.launch_iters(g_iters.load());
  PoolTable& t = *d_.h_tab[ring_];
  uint32_t n = 0;
  bool bounded = false;
  int idx[kMaxSlots];
  for (int s = 0; s < kMaxSlots; ++s)
    if (slots_[s].state == SlotState::kActive && !slots_[s].no_more) idx[n++] = s;
  if (n == 0 && !empty_linger) return NPOW_OK;
  if (!live_slot()) end_linger();  // (step() has raised it already when a job waits; a bounded range's next part)
  t.n = n;
  t.poll_mask = poll_mask();
  t.iters = iters;
  t.budget = g_budget_us.load() * 100u;  // s_memrealtime runs at 100 MHz
  t.yield_base = ctl_;
  t.dyn_base = (uint32_t)ctl_;
  // One entry: the launch ends with it, and counting workgroups on it only delays that end (the
  // final count would reach the host ~60 us after the launch's own end; measured with
  // NANOPOW_TRACE_LATENCY).  Two or more: a won entry's job need not wait for the others.  A lingering launch is
  // counted from its first entry (set below, once the entries are known to be unbounded).
  t.counted = n >= 2 ? 1u : 0u;
  t.linger = 0;
  t.kill_base = (uint32_t)__atomic_load_n(&d_.pmb->kills, __ATOMIC_ACQUIRE);
  ++seq_;
  t.ring = (uint32_t)ring_;
  t.seq = (uint32_t)seq_;
  {
    std::lock_guard<std::mutex> g(g_pool.mu);  // issued[] is shared with other workers' reads
    const double t_issue = now_us();
    for (uint32_t e = 0; e < n; ++e) {
      Slot& sl = slots_[idx[e]];
      Job& j = *sl.job;
      PoolEntry& pe = t.e[e];
      memcpy(pe.u, j.u, sizeof(pe.u));
      pe.threshold = j.threshold;
      pe.gen = sl.gen;
      pe.slot = (uint32_t)idx[e];
      // the next part of the device's queue of ranges: a bounded job's own waves cover it
      // densely; an unbounded job claims a full launch region (W * iters * 64, holes allowed)
      // unless less than that is left, which then becomes a dense bounded entry too
      std::deque<Range>& todo = j.todo[sl.k];
      const uint64_t own = sh.own(e, n, iters);
      const uint64_t full = sh.full(iters);
      if (todo.empty()) todo.push_back({j.start, 0});  // cannot happen (adopt / no_more); an empty entry
      Range& r = todo.front();
      const uint64_t want = j.max_per_dev ? own : full;
      pe.base = r.base;
      pe.count = std::min(want, r.count);
      pe.bounded = (j.max_per_dev || pe.count < full) ? 1 : 0;
      if (pe.bounded) {
        pe.count = std::min(pe.count, own);
        bounded = true;
      }
      r.base += pe.count;
      r.count -= pe.count;
      if (r.count == 0) todo.pop_front();
      sl.inflight.push_back({seq_, pe.base, pe.count});
      if (j.t_launch == 0) j.t_launch = t_issue;
      if (j.t_launch_dev[sl.k] == 0) j.t_launch_dev[sl.k] = t_issue;
      if (todo.empty()) sl.no_more = true;
      sl.fresh = false;
    }
  }
  if (lingers(d_) && !bounded && g_budget_us.load() > 0) {
    // each lingering workgroup reads the pinned ctl word once in P looks (phase g): ~2 reads per look grid-wide
    uint32_t P = 1;
    while (P * 2 < (uint32_t)sh.grid) P <<= 1;
    if (g_linger_p > 0) P = g_linger_p;
    t.linger = P;
    t.counted = 1u;
  }
  if (n == 0 && !t.linger) return NPOW_OK;
  const int r = ring_;
  ring_ = (ring_ + 1) % kEventRing;
  const size_t bytes = pool_table_bytes(n);
  DEVCHECK(d_, "pool launch");
  // Up to kArgEntries entries the table rides in the kernel arguments (no copy before the launch;
  // uploading it instead cost 2.5 %, profiles/r02_ab_table_upload.jsonl); a larger one goes up in
  // stream order right before its launch.  (Uploading it on a second stream beside the running
  // launch, joined by an event, cost 1.5-2 % of kernel throughput: the copy is a blit kernel that
  // competes with the running launch.)
  if (faults().hip_dev == d_.id && seq_ > faults().hip_after)  // NANOPOW_FAULT_HIP (tests)
    return fail(NPOW_ERR_HIP, "injected launch failure (NANOPOW_FAULT_HIP)");
  if (n <= (uint32_t)kArgEntries) {
    HIPTRY(hipEventRecord(d_.ev_start[r], d_.stream));
    HIPTRY(launch_pool_arg(d_.stream, sh.grid, t, bounded, d_.pst, d_.pmb_dev));
  } else {
    HIPTRY(hipMemcpyAsync(d_.d_tab[r], d_.h_tab[r], bytes, hipMemcpyHostToDevice, d_.stream));
    HIPTRY(hipEventRecord(d_.ev_start[r], d_.stream));
    HIPTRY(launch_pool(d_.stream, sh.grid, d_.d_tab[r], bounded, d_.pst, d_.pmb_dev));
  }
  HIPTRY(hipEventRecord(d_.ev_stop[r], d_.stream));
  if (q_.empty()) front_start_ = std::chrono::steady_clock::now();
  NPOW_DBGT("nanopow[%d]: launch %llu n=%u linger %u yield_base %llx slots:", d_.id, (unsigned long long)seq_, n,
            t.linger, (unsigned long long)t.yield_base);
  for (uint32_t e = 0; e < n; ++e) NPOW_DBG(" %d/g%llu", idx[e], (unsigned long long)t.e[e].gen);
  NPOW_DBG("\n");
  q_.push_back({seq_, r, (uint32_t)ctl_, t.yield_base, t.counted != 0, t.linger != 0});
  return NPOW_OK;
}

// Slots that just left the tables: read their done shards back in stream order, behind every
// launch that still holds them (later launches do not), and note when that copy lands.  Round 5: a won or killed
// slot's kernels publish its final count (every launch, one-entry ones included), so the read-back -- a copy on the
// stream between the dying launch and the next search's launch, ~GPU idle on every device each search -- waits for
// that record: a slot finished from it is freed without a read-back once its launches have completed (every
// kVerifyEvery-th still reads back and checks), and the read-back runs only when no record came (the launches ended
// first: a kill that no poll relayed before the budget ran out; a bounded range exhausted; an invalid win).
int Worker::queue_readbacks() {
  constexpr size_t row = kPoolDoneShards * 8;
  DEVCHECK(d_, "pool read-back");
  for (int s = 0; s < kMaxSlots; ++s) {
    Slot& sl = slots_[s];
    if (sl.state != SlotState::kDraining || sl.readback || sl.no_readback) continue;
    if (!g_readback_always && !d_.dead) {
      if (sl.early) {
        if (++early_count_ % kVerifyEvery != 0) {
          sl.no_readback = true;
          continue;
        }
      } else if (!sl.fin_seen && sl.stop_us > 0 && !sl.requeue && !sl.inflight.empty() &&
                 now_us() - sl.stop_us < g_linger_us) {
        continue;  // won or killed: its final count is on the way (or its launches end without one) -- for
                   // g_linger_us at most: then the read-back is queued now, before the next launch is issued
                   // (ADVICE r05), not behind it; a final count that still comes is checked against it (retire())
      }
    }
    HIPTRY(hipMemcpyAsync(d_.h_done + (size_t)s * row, &d_.pst->done[s][0], row * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, d_.stream));
    HIPTRY(hipEventRecord(d_.ev_done[s], d_.stream));
    sl.readback = true;
  }
  return NPOW_OK;
}

int Worker::retire() {
  DEVCHECK(d_, "pool retire");
  while (!q_.empty()) {
    const hipError_t e = hipEventQuery(d_.ev_stop[q_.front().ring]);
    if (e == hipErrorNotReady) break;
    if (e != hipSuccess) return fail(NPOW_ERR_HIP, std::string("pool launch: ") + hipGetErrorString(e));
    account_launch(d_, q_.front().ring);
    // the GPU idle before this launch: the previous launch's stop event to this one's start event (the ring slot of
    // the previous launch is not reused before this one retires: at most two launches are in flight)
    if (prev_stop_ring_ >= 0) {
      float gap = 0.f;
      if (hipEventElapsedTime(&gap, d_.ev_stop[prev_stop_ring_], d_.ev_start[q_.front().ring]) == hipSuccess &&
          gap >= 0.f) {
        std::lock_guard<std::mutex> sg(d_.stats_mu);
        d_.idle_ms += gap;
        d_.idle_gaps++;
      }
    }
    prev_stop_ring_ = q_.front().ring;
    uint64_t g0 = 0, g1 = 0;
    account_clock(q_.front().ring, q_.front().seq, &g0, &g1);
    if (g_trace_lat && g0) {  // the launch's event span against its clock waves' span (dispatch and drain)
      float ev = 0.f;
      if (hipEventElapsedTime(&ev, d_.ev_start[q_.front().ring], d_.ev_stop[q_.front().ring]) == hipSuccess)
        fprintf(stderr, "nanopow-launch dev %d launch %llu: events %.1f clock waves %.1f us, start %.1f us after the "
                "previous end\n", d_.id, (unsigned long long)q_.front().seq, ev * 1e3, (double)(g1 - g0) / 100.0,
                prev_g1_ ? ((double)g0 - (double)prev_g1_) / 100.0 : -1.0);
      prev_g1_ = g1;
    }
    if (g_trace_lat && g0)  // GPU timeline of a decided job's launch on this device, from the deciding win (the same
                            // clock only for devices on one GPU: CU partitions)
      for (const Slot& sl : slots_)
        if (sl.state != SlotState::kFree && sl.job && sl.job->gpu_t_win && !sl.inflight.empty() &&
            sl.inflight.front().seq <= q_.front().seq)
          fprintf(stderr, "nanopow-gpu dev %d ticket %llu launch %llu: start %+.1f end %+.1f us from the win\n", d_.id,
                  (unsigned long long)sl.job->ticket, (unsigned long long)q_.front().seq,
                  ((double)g0 - (double)sl.job->gpu_t_win) / 100.0, ((double)g1 - (double)sl.job->gpu_t_win) / 100.0);
    // The launch's ranges are complete, except those of a generation that won in it (or in an
    // earlier launch still unseen): handle such wins first, they hand back what did not finish.
    const uint64_t seq = q_.front().seq;
    for (int s = 0; s < kMaxSlots; ++s) {
      Slot& sl = slots_[s];
      if (sl.state == SlotState::kFree || sl.inflight.empty()) continue;
      if (win_published(s)) handle_win(s);
      size_t m = 0;
      while (m < sl.inflight.size() && sl.inflight[m].seq <= seq) ++m;
      // dense bounded ranges, hashed in full (fail_all's accounting) -- unless the slot's generation has
      // stopped (won or killed): its launches may have ended part-way, so nothing more is credited
      if (sl.job && sl.job->max_per_dev && !sl.win_seen && sl.stop_us == 0)
        for (size_t i = 0; i < m; ++i) sl.unread += sl.inflight[i].count;
      sl.inflight.erase(sl.inflight.begin(), sl.inflight.begin() + (ptrdiff_t)m);
      // a decided job's last launch on this device has completed: the device hashes nothing more of it, so
      // its stop time is now (npow_wait_info), not when the done counts' read-back lands
      // (a slot finished from its final count has its stop time already: no pool lock for it -- a lingering launch
      // retires with up to 33 of them, and 33 acquisitions of the contended lock held up this worker's next look at
      // a live search by up to ~0.1 ms)
      if (m > 0 && sl.inflight.empty() && sl.state == SlotState::kDraining && !sl.early && sl.job &&
          sl.job->decided.load()) {
        std::lock_guard<std::mutex> g(g_pool.mu);
        if (sl.job->t_stop[sl.k] == 0) {
          sl.job->t_stop[sl.k] = now_us();
          if (g_trace_lat)
            fprintf(stderr, "nanopow-nofin dev %d ticket %llu slot %d g%llu: stopped at its launch's end, no final "
                    "count (launch %llu, fin gen %llu)\n", d_.id, (unsigned long long)sl.job->ticket, s,
                    (unsigned long long)sl.gen, (unsigned long long)seq,
                    (unsigned long long)__atomic_load_n(&d_.pmb->fin[s].gen, __ATOMIC_ACQUIRE));
        }
      }
    }
    if (g_trace_lat)
      for (Slot& sl : slots_)
        if (sl.state == SlotState::kDraining && sl.job && sl.job->t_win != 0 && sl.job->t_kend == 0)
          sl.job->t_kend = now_us();
    NPOW_DBGT("nanopow[%d]: launch %llu done\n", d_.id, (unsigned long long)q_.front().seq);
    retired_seq_ = q_.front().seq;
    q_.pop_front();
    front_start_ = std::chrono::steady_clock::now();  // the next one (if any) has just started
  }
  constexpr size_t row = kPoolDoneShards * 8;
  for (int s = 0; s < kMaxSlots; ++s) {
    Slot& sl = slots_[s];
    if (sl.state == SlotState::kDraining && sl.no_readback && sl.inflight.empty()) {
      // finished from its published final count and every launch that held it has completed: nothing can still add
      // to its done counts, so the next job of this slot starts from the published total (sl.baseline)
      watch_disarm(d_, s);
      sl.job.reset();
      sl.state = SlotState::kFree;
      continue;
    }
    if (sl.state != SlotState::kDraining || !sl.readback) continue;
    const hipError_t e = hipEventQuery(d_.ev_done[s]);
    if (e == hipErrorNotReady) continue;
    if (e != hipSuccess) return fail(NPOW_ERR_HIP, std::string("pool read-back: ") + hipGetErrorString(e));
    // every launch that held the slot has completed: its done shards are final
    uint64_t sum = 0, late = 0;
    for (int i = 0; i < kPoolDoneShards; ++i) {
      sum += d_.h_done[(size_t)s * row + i * 8];
      late += d_.h_done[(size_t)s * row + i * 8 + kLateWord];
    }
    const uint64_t delta = sum - sl.baseline, late_delta = late - sl.late_base;
    sl.baseline = sum;
    sl.late_base = late;
    {
      std::lock_guard<std::mutex> sg(d_.stats_mu);
      d_.nonces += delta;
      d_.late += late_delta;
    }
    if (win_published(s)) handle_win(s);  // published by the last launch, not yet seen
    if (sl.stale && !sl.fin_seen) {  // every launch that held it has ended: its count came late, or never
      if (__atomic_load_n(&d_.pmb->fin[s].gen, __ATOMIC_ACQUIRE) == sl.gen) {
        uint64_t tw = 0;
        {
          std::lock_guard<std::mutex> g(g_pool.mu);
          tw = sl.job ? sl.job->gpu_t_win : 0;
        }
        stale_fin_came(s, tw);
      } else {
        std::lock_guard<std::mutex> sg(d_.stats_mu);
        d_.stale_missing++;
      }
    }
    NPOW_DBG("nanopow[%d]: retire slot %d g%llu done %llu requeue %d early %d\n", d_.id, s,
             (unsigned long long)sl.gen, (unsigned long long)delta, (int)sl.requeue, (int)sl.early);
    if (sl.early) {  // finished by early_finish(): the read-back must add nothing to its count
      if (delta != 0) {
        fprintf(stderr, "nanopow: GPU %d slot %d: read back %llu nonces past the published final count\n", d_.id,
                s, (unsigned long long)delta);
        std::lock_guard<std::mutex> sg(d_.stats_mu);
        d_.early_mismatch++;
      }
    } else {
      std::lock_guard<std::mutex> g(g_pool.mu);
      Job& j = *sl.job;
      j.done += delta;
      j.late[sl.k] += late_delta;
      if (d_.dead) {
        abandon_locked(sl.job, sl.k, d_.dead_code, d_.dead_msg);  // survivors take what is left
      } else if (!j.decided && (sl.requeue || !j.todo[sl.k].empty())) {
        j.on_dev[sl.k] = 0;  // adopt() picks it up again with a fresh generation
        g_pool.version.fetch_add(1);
      } else {
        device_done_locked(sl.job, sl.k);
      }
    }
    watch_disarm(d_, s);
    sl.job.reset();
    sl.state = SlotState::kFree;
  }
  return NPOW_OK;
}

// A HIP call failed: the device is dropped at once (no draining: its queue cannot be trusted).
// Ranges of launches that had not completed go back to their jobs, which re-stride them.
void Worker::fail_all(const std::string& msg) {
  fprintf(stderr, "nanopow: device %d failed: %s; dropping it\n", d_.id, msg.c_str());
  std::lock_guard<std::mutex> g(g_pool.mu);
  if (!d_.dead) {
    d_.dead_code = NPOW_ERR_HIP;
    d_.dead_msg = "device " + std::to_string(d_.id) + " failed: " + msg;
    d_.dead = true;
  }
  for (Slot& sl : slots_) {
    if (sl.state == SlotState::kFree) continue;
    if (sl.job->max_per_dev) {
      // no read-back from a failed device: the job counts its bounded ranges that completed here
      // (each hashed in full, dense) from their sizes; the rest go back to it and are re-strided.
      // Exact for a job that ends without a hit; once the slot's generation has stopped (a win, a kill)
      // its last launches may have ended part-way, so only the ranges retired before that are counted
      // (crediting them in full over-counted a won job): a lower bound then.
      const uint64_t kept = push_back_locked(sl, 0, true);
      const bool stopped = sl.win_seen || sl.stop_us > 0;
      if (!sl.early) sl.job->done += sl.unread + (stopped ? 0 : kept);
    }
    watch_disarm(d_, (int)(&sl - slots_));  // before the job can end (abandon_locked): the watcher reads its cancel word
    abandon_locked(sl.job, sl.k, d_.dead_code, d_.dead_msg);
    sl.job.reset();
    sl.inflight.clear();
    sl.state = SlotState::kFree;
  }
  q_.clear();
  prev_stop_ring_ = -1;
}

int Worker::step() {
  timed(0, [&] { adopt(); return 0; });
  timed(1, [&] { check_slots(); return 0; });
  if (!q_.empty() && !live_slot()) {
    // a lingering launch idle for g_linger_us, or something waiting for the device, or its time budget over.  Idle
    // means also no won or killed slot still draining in it (its final count not in): ended under such a slot, the
    // launch's yield would race the kill relay (npow_kernel.hip ls2_poll).  A slot whose final count has not come
    // g_linger_us after its stop no longer holds the launch (stale): its count then comes from the launch's completion
    // and the read-back -- rare (1 search in ~1,200 over 4 CU partitions, profiles/r05aj_linger_by_partition_overshoot
    // .jsonl), but without this bound the lingering launch ran on to its budget and the stop took 21 ms.
    const double t = now_us();
    bool draining = false, stale = false, lingering = false;
    for (const PoolInflight& f : q_) lingering = lingering || f.linger;
    for (Slot& sl : slots_) {
      if (sl.state != SlotState::kDraining || sl.fin_seen || sl.inflight.empty()) continue;
      // (the record read again after t: a worker descheduled for a millisecond between check_slots' look and here
      // would otherwise count a count that came meanwhile as stale -- round 6 saw 8 at once over 8 partitions)
      if (sl.stop_us > 0 && t - sl.stop_us > g_linger_us &&
          __atomic_load_n(&d_.pmb->fin[&sl - slots_].gen, __ATOMIC_ACQUIRE) != sl.gen) {
        stale = true;
        if (!sl.stale && lingering) {  // the fallback below fires for it: counted, and classified when the slot's count
                                       // comes late or not at all (early_finish / retire: stale_missing)
          sl.stale = true;
          std::lock_guard<std::mutex> sg(d_.stats_mu);
          d_.stale_drains++;
          NPOW_DBGT("nanopow[%d]: slot %d g%llu: no final count %.0f us after its stop\n", d_.id,
                    (int)(&sl - slots_), (unsigned long long)sl.gen, t - sl.stop_us);
        }
      } else {
        draining = true;
      }
    }
    if (idle_since_ == 0 && !draining) idle_since_ = t;
    // the GPU time a lingering launch spends waiting with nothing to hash (its HIP-event time includes it):
    // npow_device_stats.linger_ms, so that kernel_ms - linger_ms is the time the device hashed
    if (lingering && !draining && q_.front().linger) {
      if (linger_t_ > 0) {
        std::lock_guard<std::mutex> sg(d_.stats_mu);
        d_.linger_ms += (t - linger_t_) * 1e-3;
      }
      linger_t_ = t;
    } else {
      linger_t_ = 0;
    }
    bool waiting = d_.tasks_waiting.load() > 0 || d_.dead || g_pool.stopping.load(std::memory_order_relaxed) ||
                   (stale && !draining) ||
                   (idle_since_ > 0 && t - idle_since_ > g_linger_us) ||
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - front_start_).count() >
                       (double)g_budget_us.load();
    for (int s = 0; s < kMaxSlots && !waiting; ++s) waiting = slots_[s].state == SlotState::kActive;  // (fresh)
    if (waiting) {
      end_linger();
    } else if (!draining && q_.size() == 1 && q_.front().linger && d_.tasks_waiting.load() == 0 &&
               (uint32_t)((uint32_t)ctl_ - (uint32_t)q_.front().dyn_base) >= (uint32_t)kDynEntries) {
      // idle, and its dynamic entries used up: the next search could not join it, and would wait for it to end and
      // for a launch of its own (0.1-0.7 ms over 8 CU partitions, every 33rd search of a serial client).  End it now
      // and queue an empty lingering launch behind it, whose workgroups take the CUs as its own leave; the next
      // search joins that one (dyn_add), in ring positions the ending launch does not read.
      end_linger();
      if (int rc = timed(3, [&] { return launch(true); })) return rc;
    }
  } else {
    idle_since_ = 0;
    linger_t_ = 0;
  }
  if (int rc = timed(2, [&] { return queue_readbacks(); })) return rc;  // before the next launch: it no longer holds them
  if (d_.tasks_waiting.load() == 0)                                       // a sweep / values call is waiting: drain instead
    if (int rc = timed(3, [&] { return launch(); })) return rc;
  if (int rc = timed(4, [&] { return retire(); })) return rc;
  publish_busy();
  return NPOW_OK;
}

void Worker::run() {
  prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // nap(): 1-us timer slack instead of the default 50 us
  t_pool_worker = true;
  if (hipSetDevice(d_.hip_id) != hipSuccess) {
    d_.dead_code = NPOW_ERR_HIP;
    d_.dead_msg = "device " + std::to_string(d_.id) + ": hipSetDevice failed";
    d_.dead = true;
  }
  struct OnExit {
    const Worker& w;
    ~OnExit() {
      if (g_trace_steps) w.print_prof();
    }
  } on_exit{*this};
  for (;;) {
    if (exit_now()) return;
    if (d_.dead && !busy()) {
      // a dropped device (drained) hands every job that still names it to that job's survivors
      if (dev_lock_.owns_lock()) dev_lock_.unlock();
      std::unique_lock<std::mutex> lk(g_pool.mu);
      for (const JobP& j : std::vector<JobP>(g_pool.active)) {
        const int k = index_in(*j, d_.id);
        if (k >= 0 && !j->dev_done[k]) abandon_locked(j, (size_t)k, d_.dead_code, d_.dead_msg);
      }
      if (!g_pool.running) return;
      g_pool.cv_work.wait(lk);
      continue;
    }
    if (!busy()) adopt();  // jobs admitted since the last look
    if (!busy()) {
      publish_busy();
      if (dev_lock_.owns_lock()) dev_lock_.unlock();
      // Spin a little before sleeping: a serial client submits its next request a few tens of
      // microseconds after the last one ends, and a condition-variable wake-up costs about as
      // much as the search itself at receive difficulty.
      const auto spin_end = std::chrono::steady_clock::now() + std::chrono::microseconds(kIdleSpinUs);
      while (g_pool.version.load(std::memory_order_acquire) == seen_version_ &&
             !exit_now() && d_.tasks_waiting.load() == 0 &&
             std::chrono::steady_clock::now() < spin_end)
        cpu_relax();
      if (g_pool.version.load(std::memory_order_acquire) != seen_version_) continue;
      std::unique_lock<std::mutex> lk(g_pool.mu);
      g_pool.cv_work.wait(lk, [&] { return !g_pool.running || wants_device_locked(d_.id); });
      if (!g_pool.running) return;
      continue;
    }
    if (d_.tasks_waiting.load() > 0 && q_.empty()) {
      // hand the device to a waiting sweep / values call (TaskLock); lock() below then waits
      // for it to finish
      prev_stop_ring_ = -1;  // the task records the device's events too
      if (dev_lock_.owns_lock()) dev_lock_.unlock();
      while (d_.tasks_waiting.load() > 0 && !exit_now())
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      continue;
    }
    if (!dev_lock_.owns_lock()) dev_lock_.lock();  // waits behind a sweep / values task on this device
    int rc;
    try {
      rc = step();
    } catch (const std::exception& e) {  // nothing may leave the worker thread
      rc = fail(NPOW_ERR_INTERNAL, std::string("pool worker: ") + e.what());
    }
    if (rc != NPOW_OK) {
      fail_all(last_error());
      if (dev_lock_.owns_lock()) dev_lock_.unlock();
      continue;
    }
    timed(5, [&] { nap(); return 0; });
  }
}

// Between two steps.  While a launch runs there is nothing to do until a win is published, a
// job is decided or cancelled, new jobs arrive (they notify cv_work) or the next launch must be
// queued: poll without sleeping only during the first kFreshSpinUs of a launch (wins at receive
// difficulty come that early) and near the next launch's queueing point; otherwise sleep up to
// g_poll_us on cv_work.  A win is then seen within ~g_poll_us and the thread uses ~6 % of a core
// instead of all of it (50 us: 27.13 Gnonce/s on the serial bench vs 27.07 spinning, 26.98 at
// 200 us; profiles/r02_ab_worker_nap.txt).
void Worker::nap() {
  if (g_poll_us <= 0 || q_.empty() || d_.dead || d_.tasks_waiting.load() > 0) {
    cpu_relax();
    return;
  }
  // a won / killed slot drains within a hash or two (~20-40 us): poll until its count is in, for at
  // most kStopSpinUs after the stop
  const double t = now_us();
  for (const Slot& sl : slots_)
    if (sl.state == SlotState::kDraining && sl.stop_us > 0 && !sl.fin_seen && t - sl.stop_us < kStopSpinUs) {
      cpu_relax();
      return;
    }
  const double since = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - front_start_).count();
  if (since < kFreshSpinUs) {
    cpu_relax();
    return;
  }
  double us = g_poll_us;
  const double budget = (double)g_budget_us.load();
  if (q_.size() == 1 && budget > 0) {
    const double until_prelaunch = budget - kPrelaunchUs - since;
    if (until_prelaunch <= 0) {
      cpu_relax();
      return;
    }
    us = std::min(us, until_prelaunch);
  }
  // on the device's own condition variable (round 5): new jobs, decisions and shutdown bump wake_seq
  // (notify_workers_locked); one that came since the last nap returns at once
  std::unique_lock<std::mutex> wl(d_.wake_mu);
  d_.wake_cv.wait_for(wl, std::chrono::duration<double, std::micro>(us),
                      [&] { return d_.wake_seq != wake_seen_ || d_.tasks_waiting.load() > 0; });
  wake_seen_ = d_.wake_seq;
}

}  // namespace

// -- device resources -----------------------------------------------------------------------------
int pool_device_init(Device& d) {
  DEVCHECK(d, "pool_device_init");
  HIPTRY(hipMalloc(&d.pst, sizeof(PoolDevState)));
  if (int rc = check_device_memory(d.pst, d, "the pool state")) return rc;
  // on the device's own stream, not the null stream: a CU-partitioned device's stream is a blocking one
  HIPTRY(hipMemsetAsync(d.pst, 0, sizeof(PoolDevState), d.stream));
  HIPTRY(hipStreamSynchronize(d.stream));
  void* mb = nullptr;
  HIPTRY(hipHostMalloc(&mb, sizeof(PoolMailbox), hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
  memset(mb, 0, sizeof(PoolMailbox));
  d.pmb = (PoolMailbox*)mb;
  void* mbd = nullptr;  // taken with d.hip_id current (init_device), checked against the allocation's own mapping
  HIPTRY(hipHostGetDevicePointer(&mbd, mb, 0));
  d.pmb_dev = (PoolMailbox*)mbd;
  if (int rc = check_pinned_mapping(mb, mbd, "the pool mailbox")) return rc;
  for (int r = 0; r < kEventRing; ++r) {
    HIPTRY(hipMalloc(&d.d_tab[r], sizeof(PoolTable)));
    if (int rc = check_device_memory(d.d_tab[r], d, "a launch table")) return rc;
    void* h = nullptr;
    HIPTRY(hipHostMalloc(&h, sizeof(PoolTable), hipHostMallocDefault));
    memset(h, 0, sizeof(PoolTable));
    d.h_tab[r] = (PoolTable*)h;
  }
  void* hd = nullptr;
  HIPTRY(hipHostMalloc(&hd, (size_t)kMaxSlots * kPoolDoneShards * 8 * sizeof(unsigned long long), hipHostMallocDefault));
  d.h_done = (unsigned long long*)hd;
  for (int s = 0; s < kMaxSlots; ++s) HIPTRY(hipEventCreateWithFlags(&d.ev_done[s], hipEventDisableTiming));
  return NPOW_OK;
}

void pool_device_free(Device& d) {  // tolerates a partial pool_device_init
  if (d.pst) (void)hipFree(d.pst);
  if (d.pmb) (void)hipHostFree(d.pmb);
  for (int r = 0; r < kEventRing; ++r) {
    if (d.d_tab[r]) (void)hipFree(d.d_tab[r]);
    if (d.h_tab[r]) (void)hipHostFree(d.h_tab[r]);
  }
  if (d.h_done) (void)hipHostFree(d.h_done);
  for (int s = 0; s < kMaxSlots; ++s)
    if (d.ev_done[s]) (void)hipEventDestroy(d.ev_done[s]);
}

void pool_start() {
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    g_pool.running = true;
    g_pool.stopping = false;
  }
  if (g_watcher_on) {
    {
      std::lock_guard<std::mutex> g(g_watch.mu);
      g_watch.stop = false;
    }
    g_watch.th = std::thread(watcher_run);
  }
  for (auto& dp : g_devs) {
    Device* d = dp.get();
    if (d->cpu_threads) {
      d->worker = std::thread([d] { cpu_worker_run(*d); });
      continue;
    }
    d->worker = std::thread([d] {
      Worker w(*d);
      w.run();
    });
  }
}

// Process exit (npow_init's atexit hook).  Round 6: the workers used to leave at once, without a HIP
// call, and a lingering launch (up to its 20-ms budget of waiting, polling pinned memory) or a search launch could
// still be running while the HIP runtime and a profiler's tool library tore down -- the process then died with SIGSEGV
// in its exit handlers under rocprofv3 (profiles/r05aq_hip_api_trace_overshoot_g4.txt).  Now exit drains like
// npow_shutdown: every job is cancelled (its kill word raised), lingering launches get their yield, the workers retire
// their launches and leave once idle -- for up to kExitDrainMs; after that (a device that does not answer) they leave
// regardless.  The hook runs before the HIP runtime's own exit handlers (it was registered after the runtime was
// loaded and initialised: atexit runs in reverse order), so the workers' HIP calls (event queries) are still valid.
constexpr double kExitDrainMs = 250.0;
bool pool_exit() {
  g_exit_deadline_us.store(now_us() + kExitDrainMs * 1e3);
  pool_stop();
  const bool drained = !g_exiting.load();  // (set only by exit_now() once the deadline passed)
  g_exiting = true;
  return drained;
}

void pool_stop() {
  {
    std::lock_guard<std::mutex> g(g_pool.mu);
    g_pool.running = false;
    g_pool.stopping = true;  // workers end their lingering launches (end_linger)
    for (const JobP& j : g_pool.active) j->cancel_req = true;
    notify_workers_locked();
  }
  for (auto& d : g_devs)
    if (d->worker.joinable()) d->worker.join();
  if (g_watch.th.joinable()) {
    {
      std::lock_guard<std::mutex> g(g_watch.mu);
      g_watch.stop = true;
    }
    g_watch.cv.notify_all();
    g_watch.th.join();
  }
  for (auto& dp : g_devs)  // a worker that left with slots armed (shutdown): nothing is watched any more
    for (int s = 0; s < kMaxSlots; ++s) watch_disarm(*dp, s);
  std::lock_guard<std::mutex> g(g_pool.mu);
  for (auto& kv : g_pool.tickets) {
    const JobP& j = kv.second;
    if (!j->finished) {
      if (!j->decided) {  // a decided job keeps its outcome: waiters may read it without the lock
        j->err = "engine shut down";
        j->status = NPOW_ERR_NOT_INITIALISED;
        j->decided.store(true, std::memory_order_release);
      }
      j->finished.store(true, std::memory_order_release);
    }
  }
  for (auto& kv : g_pool.tickets) notify_waiters(*kv.second);
  g_pool.waiting.clear();
  g_pool.active.clear();
}

// -- jobs -------------------------------------------------------------------------------------------
int pool_submit(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t device_mask,
                uint64_t max_nonces_per_device, const volatile uint32_t* cancel, uint64_t* ticket) {
  // A bounded search over "all devices" (mask 0) leaves the CPU workers out: their stride would be as
  // long as a GPU's at ~1/1000 of its rate, nothing hands their leftover to an idle GPU, and they work on one job
  // at a time -- an exhausting search would wait for them.  An explicit mask may still name the CPU device.
  auto devs = max_nonces_per_device && device_mask == 0 ? select_gpus(0) : select_devices(device_mask);
  if (devs.empty() && max_nonces_per_device && device_mask == 0) devs = select_devices(0);  // only the CPU is left
  if (devs.empty()) return fail(NPOW_ERR_NO_DEVICE, "no usable device in device_mask");
  auto j = std::make_shared<Job>();
  j->pre = host_precompute(root);
  npow_asm_uniforms(j->pre.m, j->u);
  j->threshold = threshold;
  j->start = start;
  j->max_per_dev = max_nonces_per_device;
  j->cancel = cancel;
  const uint64_t G = devs.size();
  j->spacing = G > 1 ? (~0ull / G) + 1 : 0;  // 2^64 / G (exact for powers of two)
  for (Device* d : devs) j->devs.push_back(d->id);
  j->todo.resize(G);
  for (uint64_t k = 0; k < G; ++k) {
    // bounded: max_nonces_per_device; unbounded: the whole stride (2^64 / G; 2^64 - 1 with one device)
    const uint64_t cnt = max_nonces_per_device ? max_nonces_per_device : (G > 1 ? j->spacing : ~0ull);
    j->todo[k].push_back({start + k * j->spacing, cnt});
  }
  j->on_dev.assign(G, 0);
  j->seen_dev.assign(G, 0);
  j->dev_done.assign(G, 0);
  j->dev_slot.assign(G, -1);
  j->dev_gen.assign(G, 0);
  j->t_stop.assign(G, 0.0);
  j->t_launch_dev.assign(G, 0.0);
  j->late.assign(G, 0);
  j->pending_devs = (int)G;
  j->spin_us = spin_window_us(*j);
  j->t_submit = now_us();
  std::lock_guard<std::mutex> g(g_pool.mu);
  if (!g_pool.running) return fail(NPOW_ERR_NOT_INITIALISED, "engine is shut down");
  j->ticket = g_pool.next_ticket++;
  g_pool.tickets[j->ticket] = j;
  g_pool.waiting.push_back(j);
  admit_locked();
  *ticket = j->ticket;
  return NPOW_OK;
}

// Waiters of a search's outcome (npow_wait_result) poll instead of sleeping while at most kMaxSpinners of them do,
// for up to the job's spin window per call (Job::spin_us: ~3 x its expected time to a win, 2-50 ms; 2 ms beside CPU
// workers): a serial client's reply then leaves as soon as the job is decided instead of after a condition-variable
// wake-up (decided -> result in the client p50 11 -> 6 us), and a search far longer than
// expected -- or one nobody expects to end -- is waited for asleep (round 6, ADVICE r05: a flat 50 ms before).
// NANOPOW_WAIT_SPIN=0 turns it off (A/B runs).
constexpr int kMaxSpinners = 2;
std::atomic<int> g_spinners{0};
const bool g_wait_spin = [] {
  const char* e = getenv("NANOPOW_WAIT_SPIN");
  return !(e && e[0] == '0');
}();

// Wait, without g_pool.mu, until done() holds (NPOW_OK) or the timeout passes (NPOW_PENDING).  A queued job's
// cancel word is polled here every 2 ms (admitted ones are polled by the device workers), and such a job is cancelled
// under the pool lock.  spin: poll first (g_spinners above).
template <class Done>
static int wait_job(const JobP& j, int64_t timeout_us, Done done, bool spin = false) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us < 0 ? 0 : timeout_us);
  if (spin && g_wait_spin && timeout_us != 0) {
    if (g_spinners.fetch_add(1, std::memory_order_relaxed) < kMaxSpinners) {
      const int64_t spin_us = (int64_t)j->spin_us;
      const auto spin_end = std::chrono::steady_clock::now() +
                            std::chrono::microseconds(timeout_us < 0 ? spin_us : std::min(timeout_us, spin_us));
      for (uint32_t k = 0; !done(); ++k) {
        cpu_relax();
        if ((k & 255u) == 0 && (std::chrono::steady_clock::now() >= spin_end ||
                                (!j->admitted.load(std::memory_order_acquire) && j->cancel_seen())))
          break;
      }
    }
    g_spinners.fetch_sub(1, std::memory_order_relaxed);
  }
  for (;;) {
    if (done()) return NPOW_OK;
    if (!j->admitted.load(std::memory_order_acquire) && j->cancel_seen()) {
      std::lock_guard<std::mutex> g(g_pool.mu);
      if (!j->admitted && !j->finished) {
        j->cancel_req = true;
        decide_locked(*j, NPOW_CANCELLED);
        finish_locked(j);
      }
      continue;
    }
    const auto now = std::chrono::steady_clock::now();
    if (timeout_us >= 0 && now >= deadline) return NPOW_PENDING;
    std::unique_lock<std::mutex> wl(j->wmu);
    if (j->admitted.load(std::memory_order_acquire) && timeout_us < 0) {
      j->cv.wait(wl, done);
    } else {
      auto wake = j->admitted.load(std::memory_order_acquire) ? deadline : now + std::chrono::microseconds(2000);
      if (timeout_us >= 0) wake = std::min(wake, deadline);
      j->cv.wait_until(wl, wake, done);
    }
  }
}

static JobP find_ticket(uint64_t ticket) {
  std::lock_guard<std::mutex> g(g_pool.mu);
  auto it = g_pool.tickets.find(ticket);
  return it == g_pool.tickets.end() ? nullptr : it->second;
}

int pool_wait(uint64_t ticket, int64_t timeout_us, uint64_t* nonce, uint64_t* value, uint64_t* nonces_done,
              npow_search_info* info) {
  JobP j = find_ticket(ticket);
  if (!j) return fail(NPOW_ERR_BAD_ARGUMENT, "unknown ticket");
  if (wait_job(j, timeout_us, [&] { return j->finished.load(std::memory_order_acquire); }) == NPOW_PENDING)
    return NPOW_PENDING;
  std::unique_lock<std::mutex> lk(g_pool.mu);
  if (nonces_done) *nonces_done = j->done;
  if (info) {
    info->winner_device = j->winner_k >= 0 ? j->devs[(size_t)j->winner_k] : -1;
    info->n_devices = (int32_t)j->devs.size();
    info->decide_us = j->t_decide > 0 ? j->t_decide - j->t_submit : 0.0;
    info->finish_us = j->t_finish - j->t_submit;
    double worst = 0.0, over = 0.0;
    if (j->t_decide > 0)
      for (size_t k = 0; k < j->devs.size(); ++k) {
        if ((int)k == j->winner_k || j->t_stop[k] <= j->t_decide) continue;
        const double span = j->t_stop[k] - j->t_decide;
        worst = std::max(worst, span);
        Device& d = *g_devs[(size_t)j->devs[k]];
        std::lock_guard<std::mutex> sg(d.stats_mu);
        if (d.kernel_ms > 0) over += span * 1e-3 * (double)d.nonces / d.kernel_ms;  // us x nonces per ms
      }
    info->stop_after_decide_us = worst;
    info->overshoot_nonces = (uint64_t)over;
    uint64_t dev_late = 0;
    for (size_t k = 0; k < j->devs.size(); ++k)
      if ((int)k != j->winner_k) dev_late += j->late[k];
    info->late_nonces_losers = dev_late;
    info->late_nonces_winner = j->winner_k >= 0 ? j->late[(size_t)j->winner_k] : 0;
    auto since = [&](double t) { return t > 0 ? t - j->t_submit : 0.0; };
    info->adopt_us = since(j->t_adopt);
    info->launch_us = since(j->t_launch);
    double all = 0.0;
    for (size_t k = 0; k < j->devs.size(); ++k) {
      if (j->t_launch_dev[k] == 0) {  // a device that never launched it (decided before it got to it; the CPU device)
        all = 0.0;
        break;
      }
      all = std::max(all, j->t_launch_dev[k]);
    }
    info->launch_all_us = since(all);
    info->win_seen_us = since(j->t_win_seen);
  }
  if (g_trace_lat) {
    fprintf(stderr, "nanopow-lat adopt %.1f launch %.1f win %.1f kend %.1f finish %.1f return %.1f", j->t_adopt - j->t_submit,
            j->t_launch - j->t_submit, j->t_win - j->t_submit, j->t_kend - j->t_submit, j->t_finish - j->t_submit,
            now_us() - j->t_submit);
    if (j->devs.size() > 1 && j->t_decide > 0) {  // the devices' stop times after the decision
      fprintf(stderr, " decide %.1f stops", j->t_decide - j->t_submit);
      for (size_t k = 0; k < j->devs.size(); ++k)
        fprintf(stderr, " %s%.1f", (int)k == j->winner_k ? "*" : "", j->t_stop[k] > 0 ? j->t_stop[k] - j->t_decide : -1.0);
    }
    fprintf(stderr, "\n");
  }
  const int st = j->status;
  g_pool.tickets.erase(ticket);
  if (st == NPOW_OK) {
    if (nonce) *nonce = j->nonce;
    if (value) *value = j->value;
    return NPOW_OK;
  }
  if (st < 0) return fail(st, j->err.empty() ? std::string("work generation failed") : j->err);
  return st;
}

// The search's outcome as soon as it is known (npow_wait_result): the winner accepted or the job cancelled,
// while the other devices may still be stopping; the ticket stays valid for pool_wait.
int pool_wait_result(uint64_t ticket, int64_t timeout_us, uint64_t* nonce, uint64_t* value) {
  JobP j = find_ticket(ticket);
  if (!j) return fail(NPOW_ERR_BAD_ARGUMENT, "unknown ticket");
  if (wait_job(
          j, timeout_us,
          [&] { return j->decided.load(std::memory_order_acquire) || j->finished.load(std::memory_order_acquire); },
          true) == NPOW_PENDING)
    return NPOW_PENDING;
  // the outcome was written before `decided` was released, and is never written after it
  const int st = j->status;
  if (st == NPOW_OK) {
    if (nonce) *nonce = j->nonce;
    if (value) *value = j->value;
    return NPOW_OK;
  }
  if (st < 0) return fail(st, j->err.empty() ? std::string("work generation failed") : j->err);
  return st;
}

int pool_cancel(uint64_t ticket) {
  std::lock_guard<std::mutex> g(g_pool.mu);
  auto it = g_pool.tickets.find(ticket);
  if (it == g_pool.tickets.end()) return fail(NPOW_ERR_BAD_ARGUMENT, "unknown ticket");
  const JobP& j = it->second;
  if (j->finished) return NPOW_OK;
  j->cancel_req = true;
  if (!j->admitted) {
    decide_locked(*j, NPOW_CANCELLED);
    finish_locked(j);
  } else {
    notify_workers_locked();  // the devices' workers stop its waves at their next step, now rather than after a nap
  }
  return NPOW_OK;
}

int pool_set_max_active(uint32_t n) {
  if (n == 0 || n > (uint32_t)kMaxSlots)
    return fail(NPOW_ERR_BAD_ARGUMENT, "max_active must be in [1, " + std::to_string(kMaxSlots) + "]");
  std::lock_guard<std::mutex> g(g_pool.mu);
  g_pool.max_active = n;
  admit_locked();
  return NPOW_OK;
}

void pool_counts(uint32_t* queued, uint32_t* active) {
  std::lock_guard<std::mutex> g(g_pool.mu);
  if (queued) *queued = (uint32_t)g_pool.waiting.size();
  if (active) *active = (uint32_t)g_pool.active.size();
}

}  // namespace npow
