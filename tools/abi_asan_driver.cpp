// Host AddressSanitizer / ThreadSanitizer driver for the C ABI (include/nanopow.h) -- TEST TOOL.
//
// Built by `make -C nano-dpow_amd/csrc asan` (and `tsan`, tools/tsan.supp): the engine, pool and kernel sources are
// compiled with -fsanitize=address on the host side only (device code untouched) and
// linked straight into this executable, so the ASan runtime is part of the program
// (a ctypes-loaded library cannot arrange that).  It drives every entry point the
// Python shim uses, from several threads at once, and checks each GPU result on the
// CPU with npow_work_value (the library's own CPU path; the hashlib oracle pins that
// one in tests/test_oracle.py).  Exit status 0 = every check passed and ASan saw no
// error.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "nanopow.h"

static std::atomic<int> g_fail{0};
// outcome counts, printed at the end so a run shows what it exercised
static std::atomic<int> g_won{0}, g_cancelled{0}, g_exhausted{0}, g_sweep_hits{0}, g_capacity{0};

#define CHECK(cond, ...)                                          \
  do {                                                            \
    if (!(cond)) {                                                \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);   \
      std::fprintf(stderr, __VA_ARGS__);                          \
      std::fprintf(stderr, " (%s)\n", npow_last_error());         \
      g_fail++;                                                   \
    }                                                             \
  } while (0)

static void make_root(uint64_t seed, uint8_t root[32]) {
  uint64_t x = seed * 0x9e3779b97f4a7c15ull + 1;
  for (int i = 0; i < 32; i++) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 29;
    root[i] = uint8_t(x >> 24);
  }
}

// Devices of the searches, tickets and bounded ranges: DRIVER_MASK (default 1 = device 0; 0 = every
// device, with NANOPOW_VIRTUAL_DEVICES / NANOPOW_FAULT_* to drive the device-drop path).
static const uint64_t g_mask = [] {
  const char* e = std::getenv("DRIVER_MASK");
  return e ? std::strtoull(e, nullptr, 0) : 1ull;
}();
// The bounded ranges name every device explicitly when DRIVER_MASK is 0: mask 0 leaves the CPU workers out of a
// bounded search (npow_pool.cpp pool_submit), and these runs are to cover them too.  Set in main() after npow_init.
static uint64_t g_bounded_mask = 1;

// first-win searches at an easy threshold, re-validated on the CPU
static void searches(int tid, int n) {
  for (int i = 0; i < n; i++) {
    uint8_t root[32];
    make_root(1000 * tid + i, root);
    const uint64_t thr = 0xfffff00000000000ull;
    uint64_t nonce = 0, value = 0, done = 0;
    int rc = npow_search(root, thr, uint64_t(i) << 40, g_mask, 0, nullptr, &nonce, &value, &done);
    CHECK(rc == NPOW_OK, "search rc %d", rc);
    CHECK(value == npow_work_value(root, nonce) && value >= thr, "search value");
    g_won++;
  }
}

// submit / cancel / abandon-by-timeout tickets
static void tickets(int tid, int n) {
  for (int i = 0; i < n; i++) {
    uint8_t root[32];
    make_root(50000 + 1000 * tid + i, root);
    volatile uint32_t cancel = 0;
    uint64_t ticket = 0;
    const uint64_t thr = (i % 3 == 0) ? 0xffffffffffff0000ull : 0xfffffe0000000000ull;
    int rc = npow_submit(root, thr, 0, g_mask, 0, &cancel, &ticket);
    CHECK(rc == NPOW_OK, "submit rc %d", rc);
    uint64_t nonce = 0, value = 0, done = 0;
    rc = npow_wait(ticket, 2000, &nonce, &value, &done);
    if (rc == NPOW_PENDING) {
      if (i & 1) __atomic_store_n(&cancel, 1u, __ATOMIC_RELEASE);  // the library load-acquires it
      else npow_cancel(ticket);
      rc = npow_wait(ticket, -1, &nonce, &value, &done);
    }
    CHECK(rc == NPOW_OK || rc == NPOW_CANCELLED, "ticket rc %d", rc);
    if (rc == NPOW_OK) CHECK(value == npow_work_value(root, nonce) && value >= thr, "ticket value");
    (rc == NPOW_OK ? g_won : g_cancelled)++;
  }
}

// bounded ranges that end exhausted, sweeps checked against a CPU scan
static void sweeps(int tid, int n) {
  const uint64_t count = 1 << 18, thr = 0xfff0000000000000ull;
  std::vector<uint64_t> out(256), ref;
  for (int i = 0; i < n; i++) {
    uint8_t root[32];
    make_root(90000 + 1000 * tid + i, root);
    const uint64_t start = ~uint64_t(0) - (count / 2) + uint64_t(i) * 977;  // wraps past 2^64
    ref.clear();
    for (uint64_t k = 0; k < count; k++)
      if (npow_work_value(root, start + k) >= thr) ref.push_back(start + k);
    uint64_t n_out = 0;
    const uint64_t cap = (i % 4 == 3) ? 2 : out.size();  // exercise NPOW_ERR_CAPACITY
    int rc = npow_sweep(root, thr, start, count, 1, nullptr, out.data(), cap, &n_out);
    CHECK(n_out == ref.size(), "sweep count %llu vs %zu", (unsigned long long)n_out, ref.size());
    CHECK(rc == (ref.size() > cap ? NPOW_ERR_CAPACITY : NPOW_OK), "sweep rc %d", rc);
    g_sweep_hits += int(n_out);
    if (rc == NPOW_ERR_CAPACITY) g_capacity++;
    for (uint64_t k = 0; k < n_out && k < cap && k < ref.size(); k++)
      CHECK(out[k] == ref[k], "sweep hit %llu", (unsigned long long)k);

    uint64_t nonce = 0, value = 0, done = 0;
    rc = npow_search(root, ~uint64_t(0), start, g_bounded_mask, 4096 + i, nullptr, &nonce, &value, &done);
    CHECK(rc == NPOW_EXHAUSTED || rc == NPOW_OK, "bounded rc %d", rc);
    if (rc == NPOW_EXHAUSTED) g_exhausted++;
  }
}

int main() {
  int n_dev = 0;
  // DRIVER_CPU_THREADS=N: the pool's CPU workers (--cpu-threads) as one more device; with DRIVER_MASK=0 every
  // search, ticket and bounded range also runs on them
  if (const char* c = std::getenv("DRIVER_CPU_THREADS")) {
    const int rc0 = npow_config_cpu_threads((uint32_t)std::atoi(c));
    if (rc0 != NPOW_OK) {
      std::fprintf(stderr, "npow_config_cpu_threads rc %d: %s\n", rc0, npow_last_error());
      return 2;
    }
  }
  int rc = npow_init(&n_dev);
  if (rc != NPOW_OK || n_dev < 1) {
    std::fprintf(stderr, "npow_init rc %d devices %d: %s\n", rc, n_dev, npow_last_error());
    return 2;
  }
  std::printf("%s, %d device(s)\n", npow_version(), n_dev);
  g_bounded_mask = g_mask ? g_mask : (n_dev >= 64 ? ~0ull : (1ull << n_dev) - 1);

  // value paths against the CPU
  {
    uint8_t root[32];
    make_root(7, root);
    std::vector<uint64_t> v(100003);
    rc = npow_values(0, root, 123456789, v.size(), v.data());
    CHECK(rc == NPOW_OK, "values rc %d", rc);
    for (size_t k = 0; k < v.size(); k += 101)
      CHECK(v[k] == npow_work_value(root, 123456789 + k), "values[%zu]", k);
    const uint32_t n = 4099;
    std::vector<uint8_t> roots(32 * n);
    std::vector<uint64_t> nonces(n), vals(n);
    for (uint32_t k = 0; k < n; k++) { make_root(k, &roots[32 * k]); nonces[k] = k * 0x1234567ull; }
    rc = npow_values_pairs(0, roots.data(), nonces.data(), n, vals.data());
    CHECK(rc == NPOW_OK, "pairs rc %d", rc);
    for (uint32_t k = 0; k < n; k++) CHECK(vals[k] == npow_work_value(&roots[32 * k], nonces[k]), "pair %u", k);
  }

  // a batch with cancel words, one raised up front
  {
    const uint32_t n = 9;
    std::vector<uint8_t> roots(32 * n);
    std::vector<uint64_t> thr(n, 0xfffff80000000000ull), nonces(n), values(n);
    std::vector<int32_t> status(n);
    std::vector<uint32_t> words(n, 0);
    std::vector<const volatile uint32_t*> cancel(n);
    for (uint32_t k = 0; k < n; k++) { make_root(777 + k, &roots[32 * k]); cancel[k] = &words[k]; }
    words[4] = 1;
    thr[6] = ~uint64_t(0);
    uint64_t done = 0;
    rc = npow_search_batch(roots.data(), thr.data(), n, 1, 1 << 22, cancel.data(), nonces.data(),
                           values.data(), status.data(), &done);
    CHECK(rc == NPOW_OK, "batch rc %d", rc);
    for (uint32_t k = 0; k < n; k++) {
      if (k == 4) CHECK(status[k] == NPOW_CANCELLED, "batch cancel status %d", status[k]);
      else if (status[k] == NPOW_OK)
        CHECK(values[k] == npow_work_value(&roots[32 * k], nonces[k]) && values[k] >= thr[k], "batch %u", k);
      else CHECK(status[k] == NPOW_EXHAUSTED, "batch status[%u] %d", k, status[k]);
    }
  }

  // everything at once, with the pool reconfigured underneath
  std::atomic<bool> stop{false};
  std::thread knob([&] {
    uint32_t m = 1;
    while (!stop) {
      npow_pool_config(m);
      m = m % 16 + 1;
      uint32_t q = 0, a = 0;
      npow_pool_status(&q, &a);
      std::this_thread::sleep_for(std::chrono::milliseconds(7));
    }
    npow_pool_config(4);
  });
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; t++) ts.emplace_back(searches, t, 40);
  for (int t = 0; t < 4; t++) ts.emplace_back(tickets, t, 40);
  for (int t = 0; t < 2; t++) ts.emplace_back(sweeps, t, 8);
  for (auto& t : ts) t.join();
  stop = true;
  knob.join();

  uint32_t q = 1, a = 1;
  npow_pool_status(&q, &a);
  CHECK(q == 0 && a == 0, "pool not empty: %u queued %u live", q, a);
  npow_shutdown();
  std::printf("won %d, cancelled %d, bounded exhausted %d, sweep hits %d (%d over capacity)\n",
              g_won.load(), g_cancelled.load(), g_exhausted.load(), g_sweep_hits.load(), g_capacity.load());
  std::printf("abi_asan_driver: %s (%d failures)\n", g_fail ? "FAILED" : "ok", g_fail.load());
  return g_fail ? 1 : 0;
}
