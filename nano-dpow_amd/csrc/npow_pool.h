// npow_pool.h -- the work pool's jobs and their state transitions, shared by the GPU workers
// (npow_pool.cpp) and the CPU workers (npow_cpu.cpp, `--cpu-threads`).  Internal to libnanopow.so.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "npow_host.h"

namespace npow {

constexpr int kPending = 100;  // job status before it is decided
double now_us();               // steady clock, microseconds

// [base, base + count) mod 2^64: nonces of a job still to be handed to launches
struct Range {
  uint64_t base, count;
};

struct Job {
  uint64_t ticket = 0;
  RootPrecomp pre{};
  uint64_t u[NPOW_ASM_N_UNIFORMS] = {};
  uint64_t threshold = 0, start = 0, max_per_dev = 0, spacing = 0;
  const volatile uint32_t* cancel = nullptr;
  std::vector<int> devs;  // device ids; the k-th starts on [start + k * spacing, + stride)
  // guarded by g_pool.mu
  std::vector<std::deque<Range>> todo;  // per device k: ranges not yet handed to a launch (a dead
                                        // device's remainder is re-strided onto the survivors')
  std::vector<uint8_t> on_dev;      // per device k: a slot holds the job
  std::vector<uint8_t> seen_dev;    // per device k: adopted at least once (re-adoptions do not yield)
  std::vector<uint8_t> dev_done;    // per device k: finished with the job
  std::vector<int> dev_slot;        // per device k: the slot holding it while on_dev[k] ...
  std::vector<uint64_t> dev_gen;    // ... and its generation there (the decider raises their kill words)
  std::vector<double> t_stop;       // per device k: when its worker saw it stop hashing the job (us; 0 = never adopted)
  std::vector<double> t_launch_dev; // per device k: when its first launch holding the job was issued (us; 0 = none)
  std::vector<uint64_t> late;       // per device k: nonces its waves hashed after they knew the job was over
                                    // (device-side count, PoolDevState kLateWord)
  int winner_k = -1;                // the device whose result decided the job
  int pending_devs = 0;
  std::atomic<bool> admitted{false};  // written under g_pool.mu; waiters read it without it
  bool lost = false;                // a dead device's remainder had no surviving device to go to
  int lost_code = NPOW_ERR_HIP;
  std::atomic<bool> finished{false};  // written under g_pool.mu; waiters may spin on it
  // Its waiters (pool_wait, pool_wait_result) sleep on cv with wmu, not g_pool.mu (round 5): a waiter woken at the
  // decision then returns without queueing for the pool lock behind the workers that the same decision woke (over 8
  // devices that convoy cost ~25 us per search, profiles/r05a_regime8_new.json).  decide_locked / finish_locked lock
  // wmu before they notify, and a job's outcome (status, nonce, value, err) is written before `decided` is
  // released and never after it, so a waiter reads it once it has acquired `decided`.
  std::mutex wmu;
  std::condition_variable cv;
  int status = kPending;
  uint64_t nonce = 0, value = 0, done = 0;
  std::string err;
  // lock-free flags the workers poll
  std::atomic<bool> decided{false};
  std::atomic<bool> cancel_req{false};

  bool cancel_seen() const { return cancel_req.load(std::memory_order_relaxed) || (cancel && load_acquire(cancel)); }
  // host timestamps of the job's life (steady clock, us): npow_wait_info reports them (t_kend only for
  // NANOPOW_TRACE_LATENCY, which prints the timeline in pool_wait).  t_win: the first win record read; t_win_seen:
  // the deciding one (CPU re-validation then decides at t_decide)
  double t_submit = 0, t_adopt = 0, t_launch = 0, t_win = 0, t_kend = 0, t_finish = 0, t_decide = 0, t_win_seen = 0;
  uint64_t gpu_t_win = 0;  // the deciding win's s_memrealtime (PoolWin::t; NANOPOW_TRACE_LATENCY GPU timelines)
  double spin_us = 2000.0;  // how long its result waiters and the win watcher poll before they sleep (npow_pool.cpp
                            // spin_window_us: ~3 x its expected time to a win, in [2, 50] ms)
};
using JobP = std::shared_ptr<Job>;

struct Pool {
  std::mutex mu;
  std::condition_variable cv_work;  // idle workers: new admissions / shutdown (busy ones nap on their device's wake_cv)
  std::deque<JobP> waiting;
  std::vector<JobP> active;
  std::unordered_map<uint64_t, JobP> tickets;
  uint64_t next_ticket = 1;
  uint32_t max_active = kMaxSlots;
  bool running = false;
  std::atomic<bool> stopping{false};  // pool_stop: workers end their lingering launches at once
  std::atomic<uint64_t> version{0};  // bumped whenever `active` gains a job
  std::atomic<uint64_t> decisions{0};  // bumped when a job split over devices is decided: wakes napping workers
};
extern Pool g_pool;  // npow_pool.cpp

extern std::atomic<uint64_t> g_gen;      // slot generations (unique, > 0)
extern std::atomic<bool> g_exiting;      // process exit, drain over (or its deadline passed): workers leave at once
// Process exit (pool_exit, round 6): the workers drain their launches like pool_stop until this deadline (steady clock
// us; 0 = not exiting), then leave.  exit_now(): the deadline has passed (it then sets g_exiting) or g_exiting is set.
extern std::atomic<double> g_exit_deadline_us;
bool exit_now();

// The pool lock with its notifications deferred (round 6): the waiters' condition variables and the
// workers' wakes that decide_locked / finish_locked / stop_other_devices_locked / admit_locked make under it are sent
// after the lock is released, not while it is held.  Each is a futex wake-up; made under the lock, the woken thread
// may preempt the holder on its CPU, and every other thread wanting the lock (the losing devices' workers publishing
// their stop) then waits for the holder to be scheduled again.  Use it only where every job decided or finished under
// it stays referenced past its scope (a slot's or a local JobP): the deferred list holds plain pointers.
class PoolLock {
 public:
  PoolLock();
  ~PoolLock();
  PoolLock(const PoolLock&) = delete;
  PoolLock& operator=(const PoolLock&) = delete;

 private:
  std::unique_lock<std::mutex> lk_;
};

// -- job state transitions (caller holds g_pool.mu; npow_pool.cpp) ------------------------------
void decide_locked(Job& j, int status, uint64_t nonce = 0, uint64_t value = 0);
void admit_locked();
void finish_locked(const JobP& j);
// t_seen: when the device's worker observed it stop hashing the job (its final count read), 0 = now
void device_done_locked(const JobP& j, size_t k, double t_seen = 0.0);
void abandon_locked(const JobP& j, size_t k, int code, const std::string& msg);
void stop_other_devices_locked(Job& j, size_t k_win);
int index_in(const Job& j, int dev);  // the job's index of logical device dev, or -1
void notify_workers_locked();         // wake the idle workers (cv_work) and the napping ones (each device's wake_cv)
bool wants_device_locked(int dev);    // some active job wants this device

// -- CPU workers (npow_cpu.cpp) ------------------------------------------------------------------
void cpu_worker_run(Device& d);  // the pool worker of a CPU device (Device::cpu_threads > 0)

}  // namespace npow
