import sys, time, os
sys.path.insert(0, 'nano-dpow_amd'); sys.path.insert(0, 'oracle')
from nanopow import _lib
import random
e = _lib.Engine()
e.set_pool_tuning(budget_us=200_000)
M64=(1<<64)-1
tok = _lib.CancelToken()
busy = e.submit(bytes(range(32)), M64, device_mask=1, cancel=tok)
time.sleep(0.05)
rng = random.Random(18)
for i in range(4):
    r = bytes(rng.getrandbits(8) for _ in range(32))
    t0 = time.perf_counter()
    print(f"--- submit {i}", file=sys.stderr, flush=True)
    res = e.submit(r, 0xfffffe0000000000, device_mask=1).wait(10)
    print(f"--- done {i} {time.perf_counter()-t0:.4f}", file=sys.stderr, flush=True)
tok.set(); busy.wait(10)
