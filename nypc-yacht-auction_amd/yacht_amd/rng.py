"""Host access to the engine's RNG contract (Philox4x32-10 per game, include/yacht_hip.h).

The draw function is the library's own (yk_common.h ``philox_draw``, compiled for the
host), so host-side sampling in the Python plugin classes uses bit-for-bit the stream the
kernels use."""
from __future__ import annotations

from ._lib import lib


def draw64(seed: int, env: int, ctr: int) -> int:
    return int(lib().yk_rng_draw64(seed & (2**64 - 1), env & (2**32 - 1), ctr & (2**64 - 1)))
