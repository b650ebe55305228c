"""``python -m nanopow`` -- run the nano-work-server-compatible work server.

Accepts the reference work server's flags (nano-work-server.exe @1681064;
launched as ``--gpu 0:0 -l 127.0.0.1:7000`` by client/run_windows.bat:27 and
client/README.md:31):

  -l/--listen-address ADDR      default 127.0.0.1:7000 (the DPoW client's --worker_uri default)
  -g/--gpu PLATFORM:DEVICE[:THREADS]   repeatable; PLATFORM is ignored (HIP has one); THREADS
                                (nonces per launch in the reference, default 1048576) is a lower
                                bound on a search launch's nonces (see apply_threads)
  -c/--cpu-threads N            N CPU worker threads beside the GPUs (one more device of the work pool:
                                every request also gets a stride hashed on the host; default 0)
  --gpu-local-work-size N       accepted and ignored (search workgroups are 512 lanes on gfx950)
  --shuffle                     pick a random queued request instead of the oldest
  --max-active N                requests searched at once by the GPU work pool (default 4)

Without --gpu every visible GPU is used.
"""
from __future__ import annotations

import argparse
import logging
import sys

from . import work as W


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog="nanopow", description="Provides a work server for Nano without a full node "
                                 "(MI355X / gfx950 engine).")
    ap.add_argument("-l", "--listen-address", "--listen_address", dest="listen", default="127.0.0.1:7000",
                    metavar="ADDR", help="Specifies the address to listen on.")
    ap.add_argument("-g", "--gpu", action="append", default=[], metavar="PLATFORM:DEVICE:THREADS",
                    help="Specifies which GPU(s) to use. THREADS is optional and defaults to 1048576.")
    ap.add_argument("-c", "--cpu-threads", "--cpu_threads", dest="cpu_threads", type=int, default=0,
                    metavar="THREADS", help="Specifies how many CPU threads to use (beside the GPUs).")
    ap.add_argument("--gpu-local-work-size", "--gpu_local_work_size", dest="local_work_size", type=int,
                    default=None, metavar="N", help="Accepted for compatibility; gfx950 workgroups are fixed.")
    ap.add_argument("--shuffle", action="store_true",
                    help="Pick a random request from the queue instead of the oldest.")
    ap.add_argument("--max-active", type=int, default=4, metavar="N",
                    help="Requests searched at once by the GPU work pool (1 = strictly one at a time, "
                         "like the reference; at most 64).")
    ap.add_argument("--base-difficulty", default=W.fmt_u64(W.DEFAULT_BASE),
                    help="Threshold multipliers are quoted against (default fffffff800000000).")
    ap.add_argument("-v", "--verbose", action="store_true")
    return ap.parse_args(argv)


LS_CU_LANES = 2048  # lanes per CU of a search launch (npow_pool_kernel_ls2*: 8 waves of 64 per SIMD)


def apply_threads(eng, gpus) -> int:
    """Honour THREADS of ``--gpu P:D:THREADS``: the reference hashes THREADS nonces per kernel launch
    (nano-work-server.exe @1681064).  Here a search launch of the default cap hashes up to grid x
    (2,048 / pool_groups) lanes x cap / 2 nonces (8 waves per SIMD: a launch runs half the cap in wave
    iterations, npow_internal.h PoolShape::launch_iters) and ends on a time budget, so THREADS is
    applied as a lower bound: the cap is raised until one launch can hold THREADS nonces (at most
    65,536); below that it changes nothing.  Returns the cap in force (0 = left as it was)."""
    cap = 0
    for _platform, device, threads in gpus:
        st = eng.stats(device)
        lanes = st.grid * (LS_CU_LANES // max(st.pool_groups, 1))
        if lanes > 0:
            cap = max(cap, 2 * -(-threads // lanes))
    if cap > 8192:  # the engine's default cap: 2^31 nonces per launch on 256 CUs
        cap = min(cap, 65536)
        eng.set_tuning(cap, 0, 0)
        logging.info("THREADS: search launches capped at %d (%d wave iterations per launch)", cap, cap // 2)
        return cap
    return 0


def build(args: argparse.Namespace):
    """The configured HttpWorkServer (not yet serving), or an exit status (int) after printing why not."""
    if not 0 <= args.cpu_threads <= 1024:
        print("--cpu-threads must be in [0, 1024]", file=sys.stderr)
        return 2
    try:
        base = W.parse_threshold(args.base_difficulty)
        gpus = [W.parse_gpu_spec(s) for s in args.gpu]
        host, _, port = args.listen.rpartition(":")
        host = host.strip("[]") or "127.0.0.1"
        port_i = int(port)
    except (W.RequestError, ValueError) as e:
        print(f"Failed to parse options: {e}", file=sys.stderr)
        return 2

    from . import _lib  # loads libnanopow.so on first use; raises if it or the GPU is missing
    from .server import HttpWorkServer, WorkServer

    # CPU workers run beside the GPUs only: the engine still refuses to start without a GPU
    eng = _lib.engine(cpu_threads=args.cpu_threads)
    n_gpus = bin(eng.gpu_mask).count("1")
    mask = 0
    for _platform, device, _threads in gpus:
        if device >= n_gpus:
            print(f"GPU {device} not found ({n_gpus} visible)", file=sys.stderr)
            return 2
        mask |= 1 << device
    if mask and eng.cpu_device is not None:
        mask |= 1 << eng.cpu_device  # the selected GPUs and the CPU workers
    if not 1 <= args.max_active <= 64:
        print("--max-active must be in [1, 64]", file=sys.stderr)
        return 2
    apply_threads(eng, gpus)
    srv = HttpWorkServer(WorkServer(eng, base_threshold=base, shuffle=args.shuffle, device_mask=mask,
                                    max_active=args.max_active), host, port_i)
    logging.info("Configured for the live network with threshold %016x", base)
    logging.info("Ready to receive requests on %s (%d GPU(s)%s, %s)", srv.address,
                 bin(mask & eng.gpu_mask).count("1") if mask else n_gpus,
                 f" + {args.cpu_threads} CPU thread(s)" if eng.cpu_device is not None else "", eng.version())
    return srv


def _stop_on_sigterm() -> None:
    """SIGTERM (systemd's stop, `kill`) ends the server as Ctrl-C does: serve_forever is interrupted in the main thread,
    the listener closes, and the process exits normally -- so libnanopow's exit hook drains the running searches and
    frees the GPUs (round 6) instead of the process dying with launches in flight."""
    import signal

    def handler(signum, frame):
        raise KeyboardInterrupt(f"signal {signum}")

    signal.signal(signal.SIGTERM, handler)


def main(argv=None) -> int:
    args = parse_args(argv)
    _stop_on_sigterm()
    logging.basicConfig(level=logging.DEBUG if args.verbose else logging.INFO,
                        format="%(asctime)s %(levelname)s %(message)s")
    srv = build(args)
    if isinstance(srv, int):
        return srv
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    finally:
        srv.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
