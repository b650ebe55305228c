import sys, time, os, random
sys.path.insert(0, 'nano-dpow_amd'); sys.path.insert(0, 'oracle')
import nanopow, oracle
e = nanopow.engine()
print("devices", e.n_devices, e.version())
rng = random.Random(1)
root = bytes(rng.getrandbits(8) for _ in range(32))
# values parity
t = time.time(); vals = e.values(root, 12345, 4096); print("values", time.time() - t)
ref = [oracle.work_value(root, 12345 + i) for i in range(4096)]
print("values match", vals == ref, sum(a != b for a, b in zip(vals, ref)))
roots = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(1000)]
nonces = [rng.getrandbits(64) for _ in range(1000)]
pv = e.values_pairs(roots, nonces)
print("pairs match", pv == [oracle.work_value(r, n) for r, n in zip(roots, nonces)])
# sweep parity
thr = 0xfffff00000000000
t = time.time(); hits = e.sweep(root, thr, 0, 1 << 26); dt = time.time() - t
ref = oracle.sweep(root, thr, 0, 1 << 26)
print("sweep 2^26", len(hits), len(ref), hits == ref, dt)
# search
for th in [0xfffffe0000000000, 0xfffffff800000000]:
    t = time.time(); r = e.search(root, th, 0); dt = time.time() - t
    print("search", hex(th), r, dt, "valid", oracle.work_value(root, r.nonce) == r.value and r.value >= th)
s = e.stats(0)
print("stats", s.launches, s.nonces, s.kernel_ms, s.grid, "Gnonce/s(kernel)", s.nonces / (s.kernel_ms * 1e-3) / 1e9 if s.kernel_ms else 0)
# throughput: big sweep
e.reset_stats(0)
t = time.time(); hits = e.sweep(root, 0xfffffff800000000, 0, 1 << 34); dt = time.time() - t
s = e.stats(0)
print("sweep 2^34", len(hits), dt, "Gnonce/s wall", (1 << 34) / dt / 1e9, "kernel", s.nonces / (s.kernel_ms * 1e-3) / 1e9, s.launches)
