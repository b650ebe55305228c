// npow_engine.cpp -- host engine of libnanopow.so: devices, streams, chunked
// launch loop, first-win across GPUs, cancellation, sweeps, C ABI.
//
// Replaces the GPU work loop of the reference work server
// (client/bin/windows/nano-work-server.exe; Rust source not vendored, behaviour
// from its strings): per request every GPU scans nonce chunks ("THREADS ...
// defaults to 1048576" @1681064), the host re-validates every GPU result on
// the CPU ("GPU returned invalid work", @1669040) and gives up on a device
// after 3 consecutive invalid results (@1669144), and work_cancel stops the
// search with "Cancelled" (@1673856).
//
// MI355X design: one host thread + one HIP stream per GPU, two
// launches in flight per stream so the next chunk is queued behind the
// running one, disjoint per-GPU nonce strides, first win published by the
// kernel into host-coherent pinned memory, and a pinned abort word every wave
// polls.  No collective: the only cross-GPU datum is the winner.
#include <hip/hip_runtime.h>

#include <pthread.h>
#include <time.h>

#include <algorithm>
#include <cstddef>
#include <exception>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "npow_host.h"

namespace npow {

namespace {
thread_local std::string t_err;
}  // namespace

int fail(int code, const std::string& msg) {
  t_err = msg;
  return code;
}
const std::string& last_error() { return t_err; }

std::vector<std::unique_ptr<Device>> g_devs;
std::atomic<uint32_t> g_iters{8192};    // search launches: iteration cap under the time budget (the oldest wave of a
                                        // SIMD runs ~4 us per iteration, ~5,000 in 20 ms) and the span of bounded jobs
constexpr uint64_t kSweepChunk = 1ull << 31;  // sweep launches: 2^31 nonces (~65 ms; a launch costs ~0.35 ms of
                                              // ramp-up and drain: 26.46 Gnonce/s at 20 ms, 26.93 at 80 ms in round 1)
// Sweep: most rows per claim (npow_sweep_kernel_ls2).  Plain guided self-scheduling (first claims
// remaining / 2W) assumes equally fast workers; here a SIMD's younger waves run slower than its
// oldest, and a young worker still holding a huge claim becomes the launch's tail (round 1, per-wave
// claims: 25.81 Gnonce/s vs 26.89 at a cap of 64).
// NANOPOW_SWEEP_CLAIM overrides (experiments).
uint32_t sweep_max_claim() {
  static const uint32_t v = [] {
    const char* e = getenv("NANOPOW_SWEEP_CLAIM");
    const int k = e ? atoi(e) : 0;
    return k > 0 ? (uint32_t)k : 64u;
  }();
  return v;
}
std::atomic<uint32_t> g_poll{1024};     // a wave reads the host word every g_poll iterations (8 waves per iteration grid-wide)
std::atomic<uint32_t> g_blocks_per_cu{8};  // npow_values_kernel_seq: 256-lane workgroups per CU
std::atomic<uint32_t> g_budget_us{20000};  // pool launches end on time, not on their slowest wave

std::vector<Device*> select_devices(uint64_t mask) {
  std::vector<Device*> out;
  for (auto& d : g_devs)
    if ((mask == 0 || (mask >> d->id) & 1ull) && !d->dead) out.push_back(d.get());
  return out;
}

std::vector<Device*> select_gpus(uint64_t mask) {
  std::vector<Device*> out;
  for (Device* d : select_devices(mask))
    if (!d->cpu_threads) out.push_back(d);
  return out;
}

thread_local bool t_pool_worker = false;  // this thread is a device's pool worker (Worker::run)

int check_device_slow(Device& d, const char* site) {
  // NANOPOW_TEST_AFFINITY_SKEW=d (with the test hooks): device d's pool worker expects the HIP device after its own,
  // so that the check's failure path runs on a one-GPU box, where every logical device is HIP device 0
  static const int skew = [] {
    const char* e = getenv("NANOPOW_TEST_AFFINITY_SKEW");
    if (e) fprintf(stderr, "nanopow: TEST HOOKS ACTIVE: device %s's pool worker expects the wrong HIP device\n", e);
    return e ? atoi(e) : -1;
  }();
  int cur = -1;
  const hipError_t e = hipGetDevice(&cur);
  d.affinity_checks.fetch_add(1, std::memory_order_relaxed);
  const int want = d.hip_id + (d.id == skew && t_pool_worker ? 1 : 0);
  if (e == hipSuccess && cur == want) return NPOW_OK;
  d.affinity_failures.fetch_add(1, std::memory_order_relaxed);
  fprintf(stderr, "nanopow: TEST HOOK: device affinity violated at %s: logical device %d runs on HIP device %d, "
                  "the calling thread's current device is %d\n", site, d.id, want, cur);
  return fail(NPOW_ERR_INTERNAL, std::string("HIP call for device ") + std::to_string(d.id) + " at " + site +
                                     " from a thread whose current HIP device is " + std::to_string(cur));
}

int check_device_memory(const void* p, const Device& d, const char* what) {
  hipPointerAttribute_t a{};
  HIPTRY(hipPointerGetAttributes(&a, p));
  if (a.type != hipMemoryTypeDevice || a.device != d.hip_id)
    return fail(NPOW_ERR_HIP, std::string("device ") + std::to_string(d.id) + ": " + what + " is not device memory of HIP device " +
                                  std::to_string(d.hip_id) + " (type " + std::to_string((int)a.type) + ", device " +
                                  std::to_string(a.device) + ")");
  return NPOW_OK;
}

int check_pinned_mapping(const void* host, const void* dev, const char* what) {
  hipPointerAttribute_t a{};
  HIPTRY(hipPointerGetAttributes(&a, host));
  if (a.type != hipMemoryTypeHost || a.devicePointer != dev)
    return fail(NPOW_ERR_HIP, std::string(what) + ": pinned host memory whose device mapping is not the pointer the "
                                                 "kernels are given");
  return NPOW_OK;
}

void account_launch(Device& d, int ring) {
  (void)check_device(d, "account_launch");
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, d.ev_start[ring], d.ev_stop[ring]) != hipSuccess) ms = 0.f;
  std::lock_guard<std::mutex> g(d.stats_mu);
  d.launches++;
  d.kernel_ms += ms;
}

namespace {

std::mutex g_mu;
bool g_init = false;
uint32_t g_cpu_threads = 0;  // npow_config_cpu_threads: CPU workers npow_init adds as one more device

constexpr uint64_t kHitCap = 1u << 20;        // per-device sweep hit buffer (8 MiB)
constexpr uint64_t kValuesChunk = 1u << 24;   // values mode: nonces per launch (128 MiB out)
constexpr uint64_t kPairsChunk = 1u << 22;    // npow_values_pairs: pairs per launch (168 MiB of host staging)

// One in-flight launch.
struct Inflight {
  int ring;
  uint64_t count;
};

// Launch one chunk on d's stream bracketed by timing events.
int launch_chunk(Device& d, Mode mode, const LaunchArgs& a, int ring, uint64_t* out) {
  DEVCHECK(d, "launch_chunk");
  HIPTRY(hipEventRecord(d.ev_start[ring], d.stream));
  // the shipped stream's kernels: four 512-lane workgroups per CU; the seq values kernel: 256-lane ones
  HIPTRY(launch_task(mode, mode == Mode::kValuesSeq ? grid_of(d) : ls_grid(d), d.stream, a, d.st, d.mb_dev, out));
  HIPTRY(hipEventRecord(d.ev_stop[ring], d.stream));
  return NPOW_OK;
}

// Wait for every in-flight launch, accounting its time.
int drain(Device& d, std::deque<Inflight>& q) {
  DEVCHECK(d, "drain");
  HIPTRY(hipStreamSynchronize(d.stream));
  while (!q.empty()) {
    account_launch(d, q.front().ring);
    q.pop_front();
  }
  return NPOW_OK;
}

int read_state(Device& d, DevState* hs) {
  DEVCHECK(d, "read_state");
  HIPTRY(hipMemcpyAsync(hs, d.st, sizeof(DevState), hipMemcpyDeviceToHost, d.stream));
  HIPTRY(hipStreamSynchronize(d.stream));
  std::lock_guard<std::mutex> g(d.stats_mu);
  d.nonces += hs->done();
  return NPOW_OK;
}

int reset_task(Device& d) {
  DEVCHECK(d, "reset_task");
  HIPTRY(hipMemsetAsync(d.st, 0, sizeof(DevState), d.stream));
  HIPTRY(hipStreamSynchronize(d.stream));
  store_release(&d.mb->found, 0);
  store_release(&d.mb->abort, 0);
  return NPOW_OK;
}

template <class F>
void run_on_devices(const std::vector<Device*>& devs, F&& fn) {
  if (devs.size() == 1) {
    fn(0, *devs[0]);
    return;
  }
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> errs(devs.size());
  th.reserve(devs.size());
  for (size_t k = 0; k < devs.size(); ++k)
    th.emplace_back([&, k] {
      try {
        fn(k, *devs[k]);
      } catch (...) {  // an exception may not leave a std::thread: hand it to the caller
        errs[k] = std::current_exception();
      }
    });
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

// Every extern "C" entry point is a function-try-block: no C++ exception (std::bad_alloc,
// std::system_error from thread creation, ...) may cross the C ABI.
int guard_exception() {
  try {
    throw;
  } catch (const std::bad_alloc&) {
    return fail(NPOW_ERR_INTERNAL, "out of host memory");
  } catch (const std::exception& e) {
    return fail(NPOW_ERR_INTERNAL, std::string("host-side failure: ") + e.what());
  } catch (...) {
    return fail(NPOW_ERR_INTERNAL, "host-side failure");
  }
}

int check_init() {
  if (!g_init) return fail(NPOW_ERR_NOT_INITIALISED, "npow_init() has not been called");
  return NPOW_OK;
}

// Release one device's resources (any of them may be missing: a partial npow_init).
void free_device(Device& d) {
  if (d.cpu_threads) return;  // no HIP state
  (void)hipSetDevice(d.hip_id);
  if (d.stream) (void)hipStreamSynchronize(d.stream);
  for (int r = 0; r < kEventRing; ++r) {
    if (d.ev_start[r]) (void)hipEventDestroy(d.ev_start[r]);
    if (d.ev_stop[r]) (void)hipEventDestroy(d.ev_stop[r]);
  }
  if (d.st) (void)hipFree(d.st);
  if (d.d_out) (void)hipFree(d.d_out);
  if (d.mb) (void)hipHostFree(d.mb);
  pool_device_free(d);
  if (d.stream) (void)hipStreamDestroy(d.stream);
}

// Create one device's stream, buffers and events (d is already in g_devs).  parts > 1: logical device
// d.id is partition d.id / n_physical of HIP device d.id % n_physical, a CU-masked stream
// (hipExtStreamCreateWithCUMask) over CUs [part * cus / parts, (part + 1) * cus / parts) -- measured on the
// MI355X (tools/experiments/cu_mask_probe.hip, profiles/r04_cu_mask_probe.txt): such a contiguous run of
// mask bits holds the same number of CUs on each of the 8 XCDs, the partitions are disjoint, and kernels
// on up to 8 of them run at the same time, each from its start; a mask of every parts-th CU is NOT a
// partition (its workgroups ran on every CU).
int init_device(Device& d, int n_physical, int parts) {
  d.hip_id = d.id % n_physical;
  HIPTRY(hipSetDevice(d.hip_id));
  const char* f = test_hooks_enabled() ? getenv("NANOPOW_FAULT_INIT") : nullptr;
  if (f)  // test hook (with NANOPOW_TEST_HOOKS=1): this logical device fails to open
    if (atoi(f) == d.id) {
      HIPTRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));  // something to clean up
      return fail(NPOW_ERR_HIP, "injected init failure (NANOPOW_FAULT_INIT)");
    }
  hipDeviceProp_t p;
  HIPTRY(hipGetDeviceProperties(&p, d.hip_id));
  d.cus = p.multiProcessorCount;
  if (parts > 1) {
    const int part = d.id / n_physical, all = p.multiProcessorCount;
    const int lo = part * all / parts, hi = (part + 1) * all / parts;
    std::vector<uint32_t> mask((size_t)(all + 31) / 32, 0u);
    for (int i = lo; i < hi; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    // the stream is a blocking one (no flags argument): every copy of this device goes on it, never on the
    // null stream, which would wait for the other partitions' launches
    HIPTRY(hipExtStreamCreateWithCUMask(&d.stream, (uint32_t)mask.size(), mask.data()));
    d.cus = hi - lo;
    d.cu_first = lo;
  } else {
    HIPTRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  }
  DEVCHECK(d, "init_device");
  HIPTRY(hipMalloc(&d.st, sizeof(DevState)));
  HIPTRY(hipMalloc(&d.d_out, kValuesChunk * sizeof(uint64_t)));
  if (int rc = check_device_memory(d.st, d, "the task state")) return rc;
  if (int rc = check_device_memory(d.d_out, d, "the hit / values buffer")) return rc;
  void* mb = nullptr;
  HIPTRY(hipHostMalloc(&mb, sizeof(HostMailbox), hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
  memset(mb, 0, sizeof(HostMailbox));
  d.mb = (HostMailbox*)mb;
  // the device pointer taken with d.hip_id current (hipSetDevice above; DEVCHECK under the test hooks), and
  // checked against the allocation's own mapping
  void* mbd = nullptr;
  HIPTRY(hipHostGetDevicePointer(&mbd, mb, 0));
  d.mb_dev = (HostMailbox*)mbd;
  if (int rc = check_pinned_mapping(mb, mbd, "the task mailbox")) return rc;
  for (int r = 0; r < kEventRing; ++r) {
    HIPTRY(hipEventCreate(&d.ev_start[r]));
    HIPTRY(hipEventCreate(&d.ev_stop[r]));
  }
  return pool_device_init(d);
}

// ---------------------------------------------------------------------------------------
// Sweep one contiguous sub-range on one device; hits (unsorted) appended to `hits`.
int device_sweep(Device& d, const RootPrecomp& pre, uint64_t threshold, uint64_t start, uint64_t count,
                 const volatile uint32_t* cancel, std::vector<uint64_t>& hits, uint64_t& n_total,
                 bool& cancelled) {
  TaskLock lk(d);
  HIPTRY(hipSetDevice(d.hip_id));
  DEVCHECK(d, "device_sweep");
  int rc = reset_task(d);
  if (rc) return rc;
  LaunchArgs a{};
  fill_uniforms(a, pre);
  a.threshold = threshold;
  a.poll_mask = poll_mask();
  a.cap = (uint32_t)kHitCap;
  a.max_claim = sweep_max_claim();
  const uint64_t chunk = kSweepChunk;
  uint64_t issued = 0;
  uint32_t launches = 0;  // parity picks the launch's claim counter (reset_task zeroed both)
  int ring = 0;
  std::deque<Inflight> q;
  cancelled = false;
  while (issued < count || !q.empty()) {
    while (q.size() < 2 && issued < count && !cancelled) {
      const uint64_t cnt = std::min(chunk, count - issued);
      a.base = start + issued;
      a.count = cnt;
      a.claim_slot = launches++ & 1;
      rc = launch_chunk(d, Mode::kSweep, a, ring, d.d_out);
      if (rc) return rc;
      q.push_back({ring, cnt});
      ring = (ring + 1) % kEventRing;
      issued += cnt;
    }
    while (!q.empty() && hipEventQuery(d.ev_stop[q.front().ring]) == hipSuccess) {
      account_launch(d, q.front().ring);
      q.pop_front();
    }
    if (!cancelled && cancel && load_acquire(cancel)) {
      cancelled = true;
      store_release(&d.mb->abort, 1);
    }
    if (cancelled && q.empty()) break;
    if (q.size() >= 2 || (issued >= count && !q.empty())) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  rc = drain(d, q);
  if (rc) return rc;
  DevState hs;
  rc = read_state(d, &hs);
  if (rc) return rc;
  n_total = hs.n_hits;
  const uint64_t k = std::min<uint64_t>(hs.n_hits, kHitCap);
  hits.resize(k);
  if (k) {
    HIPTRY(hipMemcpyAsync(hits.data(), d.d_out, k * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
    HIPTRY(hipStreamSynchronize(d.stream));
  }
  return NPOW_OK;
}

}  // namespace
}  // namespace npow

using namespace npow;

extern "C" {

const char* npow_last_error(void) { return t_err.c_str(); }

#define NPOW_STR2(x) #x
#define NPOW_STR(x) NPOW_STR2(x)
const char* npow_version(void) {
  // the ABI number from the header itself: the round-5 string still said "ABI 4" after the header moved to 5
  return "libnanopow 0.6 (ABI " NPOW_STR(NPOW_ABI_VERSION) "; gfx950 HIP kernels: blake2b-64 nonce search, four "
         "512-lane workgroups per CU, priority runs; v_lshl_add_u64 adds, v_alignbit rotations)";
}

int npow_abi_version(void) { return NPOW_ABI_VERSION; }

int npow_init(int* n_devices) try {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_init) {
    if (n_devices) *n_devices = (int)g_devs.size();
    return NPOW_OK;
  }
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0)
    return fail(NPOW_ERR_NO_DEVICE, std::string("no HIP device: ") + hipGetErrorString(e));
  // NANOPOW_VIRTUAL_DEVICES=N (testing): expose N logical devices over the physical ones
  // (logical i -> HIP device i mod n), each with its own stream, buffers and pool worker, so
  // the multi-device first-win path runs on a one-GPU machine.
  if (const char* b = getenv("NANOPOW_BUDGET_US")) g_budget_us = (uint32_t)atoi(b);  // A/B runs
  if (const char* p = getenv("NANOPOW_POLL")) g_poll = (uint32_t)atoi(p);             // A/B runs
  int n_logical = n;
  if (const char* v = getenv("NANOPOW_VIRTUAL_DEVICES")) {
    const int k = atoi(v);
    if (k > 0) n_logical = std::min(k, 64);
  }
  // Logical devices beyond the physical ones split each GPU's CUs into disjoint partitions (round 4: a
  // faithful stand-in for separate GPUs -- every device's launch runs from its start on CUs of its own),
  // when they divide evenly, at most 8 per GPU; NANOPOW_VIRTUAL_PARTITION=share makes them time-share
  // the whole GPU instead (rounds 1-3).
  int parts = 1;
  if (n_logical > n && n_logical % n == 0 && n_logical / n <= 8) {
    const char* vp = getenv("NANOPOW_VIRTUAL_PARTITION");
    if (!vp || strcmp(vp, "share") != 0) parts = n_logical / n;
  }
  // Test hook (with NANOPOW_TEST_HOOKS=1): NANOPOW_TEST_EXTRA_QUEUES=n creates n more CU-masked streams on HIP device 0
  // that nothing ever uses -- n more hardware queues of this process, idle -- to tell a queue count's effect on the
  // CU-partition rehearsal from a partition size's
  if (const char* q = test_hooks_enabled() ? getenv("NANOPOW_TEST_EXTRA_QUEUES") : nullptr) {
    static std::vector<hipStream_t> extra;
    static void* scratch = nullptr;
    fprintf(stderr, "nanopow: TEST HOOKS ACTIVE: %s idle extra CU-masked streams\n", q);
    HIPTRY(hipSetDevice(0));
    if (!scratch) HIPTRY(hipMalloc(&scratch, 64));
    for (int i = 0; i < atoi(q); ++i) {
      uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      m[i % 8] = 1u << (i / 8);  // one CU each
      hipStream_t st = nullptr;
      HIPTRY(hipExtStreamCreateWithCUMask(&st, 8, m));
      HIPTRY(hipMemsetAsync(scratch, 0, 64, st));  // one command, so that the stream holds its hardware queue
      HIPTRY(hipStreamSynchronize(st));
      extra.push_back(st);
    }
  }
  for (int i = 0; i < n_logical; ++i) {
    g_devs.push_back(std::make_unique<Device>());
    g_devs.back()->id = i;
    // several logical devices time-sharing one GPU's CUs: a lingering launch would hold them from the others
    g_devs.back()->time_shared = n_logical > n && parts == 1;
    if (int rc = init_device(*g_devs.back(), n, parts)) {
      // leave nothing behind: a retried npow_init starts from an empty device list
      const std::string msg = last_error();
      for (auto& d : g_devs) free_device(*d);
      g_devs.clear();
      return fail(rc, msg);
    }
  }
  if (g_cpu_threads > 0 && g_devs.size() < 64) {  // the CPU workers: one more logical device, after the GPUs
    g_devs.push_back(std::make_unique<Device>());
    Device& c = *g_devs.back();
    c.id = (int)g_devs.size() - 1;
    c.cpu_threads = (int)g_cpu_threads;
    c.cus = (int)g_cpu_threads;
    c.hip_id = -1;
  }
  g_init = true;
  pool_start();
  static bool exit_hook = false;
  if (!exit_hook) {
    // Process exit without npow_shutdown (round 6).  This hook is registered after the HIP runtime and
    // any profiler tool library were loaded and initialised, so it runs before their exit handlers and static
    // destructors (atexit order is the reverse of registration): the HIP runtime is still whole here.  It drains the
    // pool (pool_exit: jobs cancelled, launches ended and retired, workers joined -- a joinable std::thread would
    // terminate the process) and then frees every device's streams, events and memory, as npow_shutdown does.  Left
    // to the runtime's own teardown, the CU-masked streams of NANOPOW_VIRTUAL_DEVICES (and launches still running on
    // them, round 5) were destroyed after rocprofv3's tool had finalised: SIGSEGV in __cxa_finalize
    // (profiles/r06a_exit_sigsegv.txt).  The frees run on a thread of their own, as the drain's HIP calls run on the
    // pool workers: by the time exit() runs the atexit handlers, the calling thread's thread_local objects -- a
    // profiler's per-thread HIP stream stack among them -- are destroyed, and rocprofv3 aborted on a HIP call made
    // from it ("Check failed: 'get_stream_stack()' Must be non nullptr", profiles/r06d_exit_regime_tls_abort.txt).
    // A drain that timed out (a device that stopped answering) frees nothing: hipStreamSynchronize could block the
    // exit for good.  A device a caller's thread still holds (a sweep in flight at exit) is not freed either.
    exit_hook = true;
    atexit([] {
      std::lock_guard<std::mutex> g(g_mu);
      if (!g_init) return;
      if (!pool_exit()) return;
      try {
        std::thread([] {
          for (auto& d : g_devs) {
            std::unique_lock<std::mutex> lk(d->mu, std::try_to_lock);
            if (lk.owns_lock()) free_device(*d);
          }
        }).join();
      } catch (...) {  // no thread to be had at exit: leave the devices to the runtime's teardown
        return;
      }
      g_init = false;
    });
  }
  if (n_devices) *n_devices = (int)g_devs.size();
  return NPOW_OK;
} catch (...) { return guard_exception(); }

void npow_shutdown(void) try {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_init) pool_stop();
  for (auto& d : g_devs) {
    std::lock_guard<std::mutex> lk(d->mu);
    free_device(*d);
  }
  g_devs.clear();
  g_init = false;
} catch (...) { (void)guard_exception(); }

uint64_t npow_work_value(const uint8_t root[32], uint64_t nonce) {
  uint64_t m[4];
  for (int i = 0; i < 4; ++i) m[i] = host_load_le64(root + 8 * i);
  return host_work_value(m, nonce);
}

int npow_config_cpu_threads(uint32_t threads) try {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_init) return fail(NPOW_ERR_BAD_ARGUMENT, "npow_config_cpu_threads must precede npow_init");
  if (threads > 1024) return fail(NPOW_ERR_BAD_ARGUMENT, "threads must be <= 1024");
  g_cpu_threads = threads;
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_set_tuning(uint32_t iters_per_launch, uint32_t poll_interval, uint32_t blocks_per_cu) try {
  if (iters_per_launch) {
    if (iters_per_launch > 65536) return fail(NPOW_ERR_BAD_ARGUMENT, "iters_per_launch must be <= 65536");
    g_iters = iters_per_launch;
  }
  if (poll_interval) g_poll = poll_interval;
  if (blocks_per_cu) {
    if (blocks_per_cu > 32) return fail(NPOW_ERR_BAD_ARGUMENT, "blocks_per_cu must be <= 32");
    g_blocks_per_cu = blocks_per_cu;
  }
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_set_pool_tuning(uint32_t budget_us, uint32_t blocks_per_cu) try {
  if (budget_us != 0xffffffffu && budget_us > 1000000) return fail(NPOW_ERR_BAD_ARGUMENT, "budget_us must be <= 1000000");
  if (blocks_per_cu != 0 && blocks_per_cu != (uint32_t)kLsGroups)
    return fail(NPOW_ERR_BAD_ARGUMENT, "blocks_per_cu must be 0 or 4: the search kernel runs four workgroups per CU");
  if (budget_us != 0xffffffffu) g_budget_us = budget_us;
  return NPOW_OK;
} catch (...) { return guard_exception(); }

static double thread_cpu_ms(pthread_t t) {
  clockid_t cid;
  timespec ts;
  if (pthread_getcpuclockid(t, &cid) != 0 || clock_gettime(cid, &ts) != 0) return 0.0;
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// CPU time (ms) the device's pool worker thread has used so far (0 if unavailable); for the CPU device, its
// hashing threads' too.
static double worker_cpu_ms(Device& d) {
  if (!d.worker.joinable()) return 0.0;
  double ms = thread_cpu_ms(d.worker.native_handle());
  std::lock_guard<std::mutex> g(d.cpu_tids_mu);
  for (pthread_t t : d.cpu_tids) ms += thread_cpu_ms(t);
  return ms;
}

// A job that finished early (npow_pool.cpp early_finish) returns before the launch that held it
// is retired and counted; with no slot left searching, that launch ends within a hash, so the
// stats calls wait (bounded) until the worker has retired everything and the counters are whole.
static void settle_stats(const Device& d) {
  const auto end = std::chrono::steady_clock::now() + std::chrono::milliseconds(200);
  while (d.worker_busy.load(std::memory_order_acquire) && d.active_slots.load(std::memory_order_acquire) == 0 &&
         !d.dead && std::chrono::steady_clock::now() < end)
    std::this_thread::sleep_for(std::chrono::microseconds(20));
}

static int stats_fill(int device, npow_device_stats* out) {
  if (int rc = check_init()) return rc;
  if (device < 0 || device >= (int)g_devs.size() || !out) return fail(NPOW_ERR_BAD_ARGUMENT, "bad device");
  Device& d = *g_devs[device];
  settle_stats(d);
  const double cpu = worker_cpu_ms(d);
  std::lock_guard<std::mutex> g(d.stats_mu);
  *out = npow_device_stats{};
  out->launches = d.launches;
  out->nonces = d.nonces;
  out->kernel_ms = d.kernel_ms;
  out->invalid_work = d.invalid;
  out->cus = d.cus;
  out->grid = d.cpu_threads ? 0 : ls_grid(d);
  out->clock_mhz = d.clk_ref_ticks > 0 ? d.clk_ticks / d.clk_ref_ticks * 100.0 : 0.0;
  out->host_cpu_ms = cpu - d.worker_cpu0_ms;
  out->host_wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - d.stats_t0).count();
  out->dead = d.dead ? 1 : 0;
  out->pool_groups = kLsGroups;
  out->early_finishes = d.early;
  out->early_mismatches = d.early_mismatch;
  out->yields = d.yields;
  out->dyn_entries = d.dyn;
  out->kills_relayed = d.kills_relayed;
  out->late_nonces = d.late;
  out->hip_device = d.hip_id;
  out->cu_first = d.cu_first;
  out->idle_ms = d.idle_ms;
  out->idle_gaps = d.idle_gaps;
  out->affinity_checks = d.affinity_checks.load(std::memory_order_relaxed);
  out->affinity_failures = d.affinity_failures.load(std::memory_order_relaxed);
  out->watcher_decisions = d.watcher_decisions;
  out->stale_drains = d.stale_drains;
  out->linger_relays = d.linger_relays;
  out->stale_late = d.stale_late;
  out->stale_missing = d.stale_missing;
  out->stale_gpu_delay_us = d.stale_gpu_delay_us;
  out->linger_ms = d.linger_ms;
  return NPOW_OK;
}

// ABI 2 callers allocate the struct up to dyn_entries: never write past it here.
int npow_device_stats_get(int device, npow_device_stats* out) try {
  if (!out) return fail(NPOW_ERR_BAD_ARGUMENT, "out is required");
  npow_device_stats full;
  if (int rc = stats_fill(device, &full)) return rc;
  memcpy(out, &full, offsetof(npow_device_stats, kills_relayed));
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_device_stats_get_sized(int device, npow_device_stats* out, uint64_t size) try {
  if (!out || size == 0) return fail(NPOW_ERR_BAD_ARGUMENT, "out and size > 0 are required");
  npow_device_stats full;
  if (int rc = stats_fill(device, &full)) return rc;
  memcpy(out, &full, std::min<uint64_t>(size, sizeof(full)));
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_device_stats_reset(int device) try {
  if (int rc = check_init()) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return fail(NPOW_ERR_BAD_ARGUMENT, "bad device");
  Device& d = *g_devs[device];
  settle_stats(d);
  const double cpu = worker_cpu_ms(d);
  std::lock_guard<std::mutex> g(d.stats_mu);
  d.launches = d.nonces = d.invalid = d.early = d.early_mismatch = d.yields = d.dyn = d.kills_relayed = d.late = 0;
  d.idle_gaps = d.watcher_decisions = d.stale_drains = d.linger_relays = d.stale_late = d.stale_missing = 0;
  d.idle_ms = d.linger_ms = d.stale_gpu_delay_us = 0.0;
  d.kernel_ms = 0.0;
  d.clk_ticks = d.clk_ref_ticks = 0.0;
  d.stats_t0 = std::chrono::steady_clock::now();
  d.worker_cpu0_ms = cpu;
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_search(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t device_mask,
                uint64_t max_nonces_per_device, const volatile uint32_t* cancel, uint64_t* nonce_out,
                uint64_t* value_out, uint64_t* nonces_done) try {
  if (int rc = check_init()) return rc;
  if (!root || !nonce_out) return fail(NPOW_ERR_BAD_ARGUMENT, "root and nonce_out are required");
  uint64_t ticket = 0;
  if (int rc = pool_submit(root, threshold, start, device_mask, max_nonces_per_device, cancel, &ticket)) return rc;
  return pool_wait(ticket, -1, nonce_out, value_out, nonces_done);
} catch (...) { return guard_exception(); }

int npow_search_batch(const uint8_t* roots, const uint64_t* thresholds, uint32_t n, uint64_t device_mask,
                      uint64_t max_nonces_per_root, const volatile uint32_t* const* cancel, uint64_t* nonces_out,
                      uint64_t* values_out, int32_t* status_out, uint64_t* nonces_done) try {
  if (int rc = check_init()) return rc;
  if (nonces_done) *nonces_done = 0;
  if (n == 0) return NPOW_OK;
  if (!roots || !thresholds || !nonces_out || !status_out)
    return fail(NPOW_ERR_BAD_ARGUMENT, "roots, thresholds, nonces_out and status_out are required");
  std::vector<uint64_t> tickets(n, 0);
  int err = NPOW_OK;
  std::string err_msg;
  for (uint32_t i = 0; i < n; ++i) {
    // distinct start per root, derived from the root so repeated roots restart identically
    const uint8_t* r = roots + 32 * (size_t)i;
    const uint64_t start = host_load_le64(r) ^ host_load_le64(r + 24);
    int rc = pool_submit(r, thresholds[i], start, device_mask, max_nonces_per_root, cancel ? cancel[i] : nullptr,
                         &tickets[i]);
    if (rc) {
      status_out[i] = rc;
      if (err == NPOW_OK) {
        err = rc;
        err_msg = last_error();
      }
    }
  }
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (!tickets[i]) continue;
    uint64_t nonce = 0, value = 0, done = 0;
    const int rc = pool_wait(tickets[i], -1, &nonce, &value, &done);
    total += done;
    status_out[i] = rc;
    if (rc == NPOW_OK) {
      nonces_out[i] = nonce;
      if (values_out) values_out[i] = value;
    } else if (rc < 0 && err == NPOW_OK) {
      err = rc;
      err_msg = last_error();
    }
  }
  if (nonces_done) *nonces_done = total;
  if (err != NPOW_OK) return fail(err, err_msg);
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_submit(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t device_mask,
                uint64_t max_nonces_per_device, const volatile uint32_t* cancel, uint64_t* ticket) try {
  if (int rc = check_init()) return rc;
  if (!root || !ticket) return fail(NPOW_ERR_BAD_ARGUMENT, "root and ticket are required");
  return pool_submit(root, threshold, start, device_mask, max_nonces_per_device, cancel, ticket);
} catch (...) { return guard_exception(); }

int npow_wait(uint64_t ticket, int64_t timeout_us, uint64_t* nonce_out, uint64_t* value_out,
              uint64_t* nonces_done) try {
  if (int rc = check_init()) return rc;
  return pool_wait(ticket, timeout_us, nonce_out, value_out, nonces_done);
} catch (...) { return guard_exception(); }

int npow_wait_info(uint64_t ticket, int64_t timeout_us, npow_search_info* info) try {
  if (int rc = check_init()) return rc;
  if (!info || info->size < offsetof(npow_search_info, nonce))
    return fail(NPOW_ERR_BAD_ARGUMENT, "info with info->size set is required");
  npow_search_info full{};
  full.size = (uint32_t)sizeof(full);
  const int rc = pool_wait(ticket, timeout_us, &full.nonce, &full.value, &full.nonces_done, &full);
  full.status = rc;
  const uint32_t n = std::min<uint32_t>(info->size, (uint32_t)sizeof(full));
  full.size = n;
  memcpy(info, &full, n);
  return rc;
} catch (...) { return guard_exception(); }

int npow_wait_result(uint64_t ticket, int64_t timeout_us, uint64_t* nonce_out, uint64_t* value_out) try {
  if (int rc = check_init()) return rc;
  return pool_wait_result(ticket, timeout_us, nonce_out, value_out);
} catch (...) { return guard_exception(); }

int npow_cancel(uint64_t ticket) try {
  if (int rc = check_init()) return rc;
  return pool_cancel(ticket);
} catch (...) { return guard_exception(); }

int npow_pool_config(uint32_t max_active) try {
  if (int rc = check_init()) return rc;
  return pool_set_max_active(max_active);
} catch (...) { return guard_exception(); }

int npow_pool_status(uint32_t* queued, uint32_t* active) try {
  if (int rc = check_init()) return rc;
  pool_counts(queued, active);
  return NPOW_OK;
} catch (...) { return guard_exception(); }

int npow_sweep(const uint8_t root[32], uint64_t threshold, uint64_t start, uint64_t count, uint64_t device_mask,
               const volatile uint32_t* cancel, uint64_t* out, uint64_t cap, uint64_t* n_out) try {
  if (int rc = check_init()) return rc;
  if (!root || !n_out || (cap && !out)) return fail(NPOW_ERR_BAD_ARGUMENT, "root, n_out (and out when cap>0) required");
  auto devs = select_gpus(device_mask);
  if (devs.empty()) return fail(NPOW_ERR_NO_DEVICE, "no usable GPU in device_mask");
  const RootPrecomp pre = host_precompute(root);
  const size_t G = devs.size();
  std::vector<std::vector<uint64_t>> hits(G);
  std::vector<uint64_t> totals(G, 0);
  std::vector<int> rcs(G, 0);
  std::vector<std::string> msgs(G);
  std::vector<char> canc(G, 0);
  const uint64_t per = count / G, rem = count % G;
  std::vector<uint64_t> sub_start(G), sub_count(G);
  uint64_t off = 0;
  for (size_t k = 0; k < G; ++k) {
    sub_start[k] = start + off;
    sub_count[k] = per + (k < rem ? 1 : 0);
    off += sub_count[k];
  }
  run_on_devices(devs, [&](size_t k, Device& d) {
    bool c = false;
    rcs[k] = device_sweep(d, pre, threshold, sub_start[k], sub_count[k], cancel, hits[k], totals[k], c);
    canc[k] = c;
    if (rcs[k]) msgs[k] = t_err;
  });
  for (size_t k = 0; k < G; ++k)
    if (rcs[k]) return fail(rcs[k], msgs[k]);
  uint64_t total = 0;
  bool overflow = false;
  std::vector<uint64_t> all;
  for (size_t k = 0; k < G; ++k) {
    total += totals[k];
    if (totals[k] > hits[k].size()) overflow = true;
    all.insert(all.end(), hits[k].begin(), hits[k].end());
  }
  std::sort(all.begin(), all.end(), [start](uint64_t x, uint64_t y) { return x - start < y - start; });
  const uint64_t k = std::min<uint64_t>(all.size(), cap);
  if (k) memcpy(out, all.data(), k * sizeof(uint64_t));
  *n_out = total;
  for (size_t j = 0; j < G; ++j)
    if (canc[j]) return NPOW_CANCELLED;
  if (overflow) return fail(NPOW_ERR_CAPACITY, "device hit buffer overflow (more than 2^20 hits per device)");
  if (total > cap) return fail(NPOW_ERR_CAPACITY, "more hits than cap");
  return NPOW_OK;
} catch (...) { return guard_exception(); }

// Values of [start, start + count) through one hash path (npow_values / npow_values_path).
static int values_on(int device, const uint8_t root[32], uint64_t start, uint64_t count, Mode mode,
                     uint64_t* values_out) {
  if (int rc = check_init()) return rc;
  if (device < 0 || device >= (int)g_devs.size() || !root || (count && !values_out) || g_devs[device]->cpu_threads)
    return fail(NPOW_ERR_BAD_ARGUMENT, "bad device (or the CPU device) or null buffer");
  Device& d = *g_devs[device];
  TaskLock lk(d);
  HIPTRY(hipSetDevice(d.hip_id));
  DEVCHECK(d, "values");
  int rc = reset_task(d);
  if (rc) return rc;
  LaunchArgs a{};
  fill_uniforms(a, host_precompute(root));
  a.poll_mask = 0;
  for (uint64_t off = 0; off < count; off += kValuesChunk) {
    const uint64_t cnt = std::min(kValuesChunk, count - off);
    a.base = start + off;
    a.count = cnt;
    rc = launch_chunk(d, mode, a, 0, d.d_out);
    if (rc) return rc;
    HIPTRY(hipMemcpyAsync(values_out + off, d.d_out, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
    HIPTRY(hipStreamSynchronize(d.stream));
    account_launch(d, 0);
  }
  DevState hs;
  return read_state(d, &hs);
}

int npow_values(int device, const uint8_t root[32], uint64_t start, uint64_t count, uint64_t* values_out) try {
  return values_on(device, root, start, count, Mode::kValues, values_out);
} catch (...) { return guard_exception(); }

int npow_values_path(int device, const uint8_t root[32], uint64_t start, uint64_t count, int path,
                     uint64_t* values_out) try {
  if (path == NPOW_PATH_SEARCH) return values_on(device, root, start, count, Mode::kValues, values_out);
  if (path == NPOW_PATH_SEQ) return values_on(device, root, start, count, Mode::kValuesSeq, values_out);
  if (path == NPOW_PATH_GENERIC) {
    if (count > 0xffffffffull) return fail(NPOW_ERR_BAD_ARGUMENT, "generic path: count must be < 2^32");
    // in chunks of kPairsChunk pairs through one reused buffer (one call could otherwise
    // need ~160 GiB of host memory for its per-pair roots)
    const uint64_t chunk = std::min<uint64_t>(count, kPairsChunk);
    std::vector<uint8_t> roots((size_t)chunk * 32);
    std::vector<uint64_t> nonces((size_t)chunk);
    for (uint64_t i = 0; i < chunk; ++i) memcpy(&roots[(size_t)i * 32], root, 32);
    for (uint64_t off = 0; off < count; off += chunk) {
      const uint64_t cnt = std::min(chunk, count - off);
      for (uint64_t i = 0; i < cnt; ++i) nonces[(size_t)i] = start + off + i;
      if (int rc = npow_values_pairs(device, roots.data(), nonces.data(), (uint32_t)cnt, values_out + off)) return rc;
    }
    return NPOW_OK;
  }
  return fail(NPOW_ERR_BAD_ARGUMENT, "path must be NPOW_PATH_SEARCH, NPOW_PATH_SEQ or NPOW_PATH_GENERIC");
} catch (...) { return guard_exception(); }

int npow_values_pairs(int device, const uint8_t* roots, const uint64_t* nonces, uint32_t n, uint64_t* values_out) try {
  if (int rc = check_init()) return rc;
  if (device < 0 || device >= (int)g_devs.size() || (n && (!roots || !nonces || !values_out)) ||
      g_devs[device]->cpu_threads)
    return fail(NPOW_ERR_BAD_ARGUMENT, "bad device (or the CPU device) or null buffer");
  if (n == 0) return NPOW_OK;
  Device& d = *g_devs[device];
  TaskLock lk(d);
  HIPTRY(hipSetDevice(d.hip_id));
  DEVCHECK(d, "values_pairs");
  // chunks of kPairsChunk pairs through device buffers allocated once per call; every copy on the
  // device's own stream (a CU-partitioned logical device's stream is a blocking one, so the null
  // stream would wait for the other partitions' launches)
  const uint32_t chunk = (uint32_t)std::min<uint64_t>(n, kPairsChunk);
  std::vector<uint64_t> words((size_t)chunk * 4);
  uint64_t *dw = nullptr, *dn = nullptr, *dv = nullptr;
  int rc = NPOW_OK;
  hipError_t e = hipSuccess;
  if ((e = hipMalloc(&dw, words.size() * 8)) == hipSuccess && (e = hipMalloc(&dn, (size_t)chunk * 8)) == hipSuccess &&
      (e = hipMalloc(&dv, (size_t)chunk * 8)) == hipSuccess) {
    for (uint32_t off = 0; off < n && e == hipSuccess; off += std::min(chunk, n - off)) {
      const uint32_t cnt = std::min(chunk, n - off);
      for (uint32_t i = 0; i < cnt; ++i)
        for (int k = 0; k < 4; ++k)
          words[4 * (size_t)i + k] = host_load_le64(roots + 32 * ((size_t)off + i) + 8 * k);
      if ((e = hipMemcpyAsync(dw, words.data(), (size_t)cnt * 32, hipMemcpyHostToDevice, d.stream)) != hipSuccess ||
          (e = hipMemcpyAsync(dn, nonces + off, (size_t)cnt * 8, hipMemcpyHostToDevice, d.stream)) != hipSuccess ||
          (e = launch_pairs((int)((cnt + kBlock - 1) / kBlock), d.stream, dw, dn, cnt, dv)) != hipSuccess ||
          (e = hipMemcpyAsync(values_out + off, dv, (size_t)cnt * 8, hipMemcpyDeviceToHost, d.stream)) != hipSuccess ||
          (e = hipStreamSynchronize(d.stream)) != hipSuccess)
        break;
    }
  }
  if (e != hipSuccess) rc = fail(NPOW_ERR_HIP, std::string("values_pairs: ") + hipGetErrorString(e));
  if (dw) (void)hipFree(dw);
  if (dn) (void)hipFree(dn);
  if (dv) (void)hipFree(dv);
  return rc;
} catch (...) { return guard_exception(); }

}  // extern "C"
