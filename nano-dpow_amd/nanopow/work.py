"""Field rules of the nano-work-server JSON surface (hashes, work, thresholds, multipliers).

The DPoW client sends these fields verbatim from MQTT (client/dpow_client.py:63-75,
docs/specification.md:19-31): the hash as 64 hex characters in any case, the
difficulty as 16 hex characters.  Error strings follow the reference work
server's (client/bin/windows/nano-work-server.exe @1677928..1679336).
The multiplier formulas are the DPoW server's (server/dpow_server.py:250-255,
275-280, 296-305): multiplier = (2^64 - base) / (2^64 - d).
"""
from __future__ import annotations

import re
from typing import Any, Dict, Tuple

M64 = (1 << 64) - 1
TWO64 = 1 << 64

# Epoch-2 thresholds (the live network's send/change and receive thresholds).
SEND_THRESHOLD = 0xfffffff800000000
RECEIVE_THRESHOLD = 0xfffffe0000000000
# Base threshold the multiplier is quoted against (nano-work-server.exe @1681900:
# "Configured for the live network with threshold fffffff800000000").
DEFAULT_BASE = SEND_THRESHOLD

SUPPORTED = "Supported commands: work_generate, work_cancel, work_validate, benchmark, status"

# 1..16 hex digits and nothing else: int(x, 16) alone also takes "-1", "+f", "0x1f", " ff", "f_f"
_HEX64 = re.compile(r"[0-9a-fA-F]{1,16}")


class RequestError(Exception):
    """A request the server answers with {"error": ..., "hint": ...} (HTTP 200)."""

    def __init__(self, error: str, hint: str = "") -> None:
        super().__init__(error)
        self.error = error
        self.hint = hint

    def reply(self) -> Dict[str, str]:
        out = {"error": self.error}
        if self.hint:
            out["hint"] = self.hint
        return out


def parse_hash(req: Dict[str, Any]) -> bytes:
    if "hash" not in req:
        raise RequestError("Failed to deserialize JSON", "Hash field missing")
    h = req["hash"]
    if not isinstance(h, str):
        raise RequestError("Bad block hash", "Expecting a hex string")
    if h == "":
        raise RequestError("Bad block hash", "Hash is empty. Expecting a hex string")
    try:
        raw = bytes.fromhex(h)
    except ValueError:
        raise RequestError("Bad block hash", "Expecting a hex string") from None
    if len(raw) < 32:
        raise RequestError("Bad block hash", "Hash is too short (should be 32 bytes)")
    if len(raw) > 32:
        raise RequestError("Bad block hash", "Hash is too long (should be 32 bytes)")
    return raw


def parse_work(req: Dict[str, Any]) -> int:
    if "work" not in req:
        raise RequestError("Failed to deserialize JSON", "Work field missing")
    w = req["work"]
    if not isinstance(w, str):
        raise RequestError("Bad work", "Expecting a hex string for work")
    if w == "":
        raise RequestError("Bad work", "Work is empty. Expecting a hex string")
    if len(w) > 16:
        raise RequestError("Bad work", "Work is too long (should be 8 bytes)")
    if not _HEX64.fullmatch(w):
        raise RequestError("Bad work", "Expecting a hex string for work")
    return int(w, 16)


def parse_threshold(s: Any) -> int:
    if not isinstance(s, str):
        raise RequestError("Bad difficulty", "Expecting a hex string for difficulty")
    if not _HEX64.fullmatch(s):
        raise RequestError("Bad difficulty",
                           "Threshold not a valid unsigned long (u64). Example: 'ffffffc000000000'")
    return int(s, 16)


def parse_multiplier(x: Any) -> float:
    try:
        m = float(x)
    except (TypeError, ValueError):
        raise RequestError("Bad multiplier", "Expecting a positive number for multiplier") from None
    if not (m > 0.0) or m != m or m == float("inf"):
        raise RequestError("Bad multiplier", "Expecting a positive number for multiplier")
    return m


def from_multiplier(multiplier: float, base: int = DEFAULT_BASE) -> int:
    """d = 2^64 - (2^64 - base) / multiplier  (dpow_server.py:275-280)."""
    d = TWO64 - int((TWO64 - base) / multiplier)
    return max(0, min(M64, d))


def to_multiplier(difficulty: int, base: int = DEFAULT_BASE) -> float:
    """(2^64 - base) / (2^64 - d)  (dpow_server.py:250-255, 296-305)."""
    return float(TWO64 - base) / float(TWO64 - difficulty)


def requested_threshold(req: Dict[str, Any], base: int) -> int:
    """difficulty, else multiplier x base, else the base threshold."""
    if req.get("difficulty") is not None:
        return parse_threshold(req["difficulty"])
    if req.get("multiplier") is not None:
        return from_multiplier(parse_multiplier(req["multiplier"]), base)
    return base


def fmt_u64(x: int) -> str:
    return f"{x & M64:016x}"


def fmt_multiplier(m: float) -> str:
    return repr(float(m))


def parse_count(req: Dict[str, Any]) -> int:
    if "count" not in req:
        raise RequestError("Failed to deserialize JSON", "count field missing")
    try:
        c = int(req["count"])
    except (TypeError, ValueError):
        raise RequestError("Bad count", "Expecting a positive number for count") from None
    if c <= 0:
        raise RequestError("Bad count", "Expecting a positive number for count")
    return c


def parse_gpu_spec(spec: str) -> Tuple[int, int, int]:
    """``PLATFORM:DEVICE[:THREADS]`` (nano-work-server.exe @1681064).  HIP has a single
    platform, so PLATFORM is accepted and ignored; THREADS (nonces per launch,
    default 1048576) becomes a lower bound on the launch chunk (__main__.apply_threads)."""
    parts = spec.split(":")
    if len(parts) not in (2, 3):
        raise ValueError(f"bad --gpu spec {spec!r}: expected PLATFORM:DEVICE[:THREADS]")
    platform, device = int(parts[0]), int(parts[1])
    threads = int(parts[2]) if len(parts) == 3 else 1048576
    if platform < 0 or device < 0 or threads <= 0:
        raise ValueError(f"bad --gpu spec {spec!r}")
    return platform, device, threads
