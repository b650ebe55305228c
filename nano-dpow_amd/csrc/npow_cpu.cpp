// npow_cpu.cpp -- CPU workers of the work pool: nano-work-server's `--cpu-threads N`.
//
// The reference work server hashes on CPU threads beside its GPUs ("cpu_threads ... Specifies how many
// CPU threads to use", nano-work-server.exe @1681064): every thread scans nonces of the current request
// and the first valid result answers it.  Here N host threads form one more logical device of the
// pool (npow_config_cpu_threads before npow_init; its id follows the GPUs'): a job split over the GPUs
// and this device gives it a stride of its own like any GPU (start + k * 2^64 / G), and the first
// result from any device decides the job.  The hash is the product's own restatement of the work
// value, host_work_value (npow_blake2b.h -- what re-validates every GPU winner), never the oracle.
// CPU workers run only beside GPUs: npow_init still fails without one, so they are no fallback.
//
// One job at a time (the oldest one that lists this device), like the reference's CPU threads on its
// current request:
//   * a coordinator thread (cpu_worker_run, the device's pool worker) adopts the job, hands it to the
//     hashing threads, watches for the job's decision or cancellation every 100 us, and releases the
//     jobs other devices decided before it got to them (so a GPU-won job does not wait for the CPU);
//   * each hashing thread claims ranges of kCpuClaim nonces from the front of the job's queue for this
//     device (Job::todo, under g_pool.mu: a dropped GPU's remainder may be re-strided here) and hashes
//     them, testing the stop conditions every 256 nonces; a hit stops all of them.
// A bounded job's ranges are hashed exactly once, so exhaustion and nonces_done stay exact.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <thread>
#include <vector>

#include "npow_pool.h"

namespace npow {
namespace {

constexpr uint64_t kCpuClaim = 1ull << 16;  // nonces per claim (~20 ms of one thread)
constexpr uint64_t kCpuCheck = 256;         // nonces between two looks at the stop conditions (~80 us)
constexpr auto kCpuSupervise = std::chrono::microseconds(100);
// Test hook (with NANOPOW_TEST_HOOKS=1): NANOPOW_TEST_CPU_RELEASE_DELAY_US=n holds the coordinator for n us between
// its hashing threads' return and its look at the job (tests/fault_worker.py cpu_last: a GPU that dies in that window
// hands its ranges to this device, which must hash them before the job can end)
const long g_release_delay_us = [] {
  const char* e = test_hooks_enabled() ? getenv("NANOPOW_TEST_CPU_RELEASE_DELAY_US") : nullptr;
  if (e) fprintf(stderr, "nanopow: TEST HOOKS ACTIVE: CPU workers release their job %s us late\n", e);
  return e ? atol(e) : 0L;
}();

struct CpuShared {
  std::mutex m;
  std::condition_variable cv;       // hashers: a new job (epoch) or quit
  std::condition_variable done_cv;  // coordinator: every hasher finished the job
  uint64_t epoch = 0;
  bool quit = false;
  JobP job;
  size_t k = 0;
  int active = 0;                   // hashers still on the job
  std::atomic<bool> stop{false};    // the job is over for this device (a hit, a decision, a cancel, exit)
  std::atomic<uint64_t> hashed{0};  // nonces hashed for the job
  std::mutex hit_mu;
  bool hit = false;
  uint64_t hit_nonce = 0, hit_value = 0;
};

bool over(const Job& j, const CpuShared& sh) {
  return sh.stop.load(std::memory_order_relaxed) || j.decided.load(std::memory_order_relaxed) || j.cancel_seen() ||
         g_exiting.load(std::memory_order_relaxed);
}

// One hashing thread's share of the current job.  Each claim's nonces go into the device's statistics as soon as
// they are hashed (at the job's end only, a long unbounded search showed 0 nonces for the CPU device).
void hash_job(CpuShared& sh, Device& d, const JobP& jp, size_t k) {
  Job& j = *jp;
  for (;;) {
    Range r{0, 0};
    {
      std::lock_guard<std::mutex> g(g_pool.mu);
      if (over(j, sh) || j.todo[k].empty()) return;
      Range& f = j.todo[k].front();
      r = {f.base, std::min(f.count, kCpuClaim)};
      f.base += r.count;
      f.count -= r.count;
      if (f.count == 0) j.todo[k].pop_front();
    }
    uint64_t n = 0;
    bool stopped = false;
    while (n < r.count) {
      if (over(j, sh)) {
        stopped = true;
        break;
      }
      const uint64_t end = std::min(r.count, n + kCpuCheck);
      for (; n < end; ++n) {
        const uint64_t nonce = r.base + n;  // wraps mod 2^64 like the GPU strides
        const uint64_t v = host_work_value(j.pre.m, nonce);
        if (v >= j.threshold) {
          std::lock_guard<std::mutex> g(sh.hit_mu);
          if (!sh.hit) {
            sh.hit = true;
            sh.hit_nonce = nonce;
            sh.hit_value = v;
          }
          sh.stop = true;
          ++n;
          stopped = true;
          break;
        }
      }
      if (stopped) break;
    }
    sh.hashed.fetch_add(n, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> sg(d.stats_mu);
      d.nonces += n;
    }
    if (stopped) return;  // the rest of this claim is not hashed: the job is over for this device
  }
}

void hasher(CpuShared& sh, Device& d) {
  uint64_t seen = 0;
  for (;;) {
    JobP j;
    size_t k = 0;
    {
      std::unique_lock<std::mutex> lk(sh.m);
      sh.cv.wait(lk, [&] { return sh.quit || sh.epoch != seen; });
      if (sh.quit) return;
      seen = sh.epoch;
      j = sh.job;
      k = sh.k;
    }
    hash_job(sh, d, j, k);
    std::lock_guard<std::mutex> lk(sh.m);
    if (--sh.active == 0) sh.done_cv.notify_all();
  }
}

// Jobs that list this device but were decided (or have nothing left for it) before it adopted them:
// release them now (caller holds g_pool.mu).
void release_unadopted_locked(int dev) {
  for (const JobP& j : std::vector<JobP>(g_pool.active)) {  // copy: device_done_locked may erase
    const int k = index_in(*j, dev);
    if (k < 0 || j->on_dev[(size_t)k] || j->dev_done[(size_t)k]) continue;
    if (j->decided || j->todo[(size_t)k].empty()) device_done_locked(j, (size_t)k);
  }
}

}  // namespace

void cpu_worker_run(Device& d) {
  CpuShared sh;
  std::vector<std::thread> threads;
  threads.reserve((size_t)d.cpu_threads);
  for (int i = 0; i < d.cpu_threads; ++i) threads.emplace_back([&sh, &d] { hasher(sh, d); });
  {
    std::lock_guard<std::mutex> g(d.cpu_tids_mu);  // their CPU time goes into the device's host_cpu_ms
    for (auto& t : threads) d.cpu_tids.push_back(t.native_handle());
  }
  for (;;) {
    JobP j;
    size_t k = 0;
    {
      std::unique_lock<std::mutex> lk(g_pool.mu);
      release_unadopted_locked(d.id);
      if (!g_pool.running || g_exiting.load()) break;
      for (const JobP& c : g_pool.active) {  // the oldest live job that wants this device
        const int kk = index_in(*c, d.id);
        if (kk >= 0 && !c->on_dev[(size_t)kk] && !c->dev_done[(size_t)kk]) {
          j = c;
          k = (size_t)kk;
          break;
        }
      }
      if (!j) {
        d.worker_busy.store(false, std::memory_order_release);
        g_pool.cv_work.wait(lk, [&] { return !g_pool.running || g_exiting.load() || wants_device_locked(d.id); });
        continue;
      }
      j->on_dev[k] = 1;
      j->seen_dev[k] = 1;
      j->dev_slot[k] = -1;  // no kill word: the hashers read the job's decision themselves
      if (j->t_launch == 0) j->t_launch = now_us();
      if (j->t_launch_dev[k] == 0) j->t_launch_dev[k] = now_us();
    }
    d.worker_busy.store(true, std::memory_order_release);
    d.active_slots.store(1, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    sh.stop = false;
    sh.hashed = 0;
    {
      std::lock_guard<std::mutex> g(sh.hit_mu);
      sh.hit = false;
    }
    // Hash the job in epochs: the hashing threads return once this device's queue of ranges is empty (or the job
    // is over), and only then does this thread take g_pool.mu.  A GPU that died in between may have handed its
    // unfinished ranges to this device (abandon_locked: the CPU is the last survivor) -- releasing the job then
    // would end it EXHAUSTED with those ranges never hashed, so a new epoch hashes them first.
    for (bool again = true; again;) {
      {
        std::lock_guard<std::mutex> lk(sh.m);
        sh.job = j;
        sh.k = k;
        sh.active = d.cpu_threads;
        ++sh.epoch;
      }
      sh.cv.notify_all();
      for (;;) {
        {
          std::unique_lock<std::mutex> lk(sh.m);
          if (sh.done_cv.wait_for(lk, kCpuSupervise, [&] { return sh.active == 0; })) break;
        }
        if (over(*j, sh) || !g_pool.running) sh.stop = true;
        std::lock_guard<std::mutex> g(g_pool.mu);
        release_unadopted_locked(d.id);
      }
      if (g_release_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(g_release_delay_us));
      std::lock_guard<std::mutex> g(g_pool.mu);
      again = !over(*j, sh) && g_pool.running && !j->todo[k].empty();
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const uint64_t hashed = sh.hashed.load();
    bool hit;
    uint64_t hn, hv;
    {
      std::lock_guard<std::mutex> g(sh.hit_mu);
      hit = sh.hit;
      hn = sh.hit_nonce;
      hv = sh.hit_value;
    }
    {
      std::lock_guard<std::mutex> sg(d.stats_mu);
      d.launches++;  // jobs hashed (their nonces went into d.nonces claim by claim)
      d.kernel_ms += ms;
    }
    d.active_slots.store(0, std::memory_order_release);
    std::lock_guard<std::mutex> g(g_pool.mu);
    j->done += hashed;
    // re-validated like a GPU winner (the same function: a hit is valid by construction)
    if (hit && host_work_value(j->pre.m, hn) == hv && hv >= j->threshold && j->status == kPending) {
      decide_locked(*j, NPOW_OK, hn, hv);
      j->t_decide = now_us();
      j->winner_k = (int)k;
      stop_other_devices_locked(*j, k);
    } else if (!j->decided && j->cancel_seen()) {
      j->cancel_req = true;
      decide_locked(*j, NPOW_CANCELLED);
    }
    device_done_locked(j, k);
  }
  {
    std::lock_guard<std::mutex> g(d.cpu_tids_mu);  // no CPU clock of a joined thread is read after this
    d.cpu_tids.clear();
  }
  {
    std::lock_guard<std::mutex> lk(sh.m);
    sh.quit = true;
  }
  sh.cv.notify_all();
  for (auto& t : threads) t.join();
  d.worker_busy.store(false, std::memory_order_release);
}

}  // namespace npow
