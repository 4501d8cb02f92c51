"""Per-stage device timing of the rasterizer (hipEvents recorded by libgsr on
the launch stream; see gsr_timing_* in include/gsr.h)."""
from __future__ import annotations

import ctypes

from ._lib import lib

STAGES = ("preprocess", "duplicate", "sort", "ranges", "render_fwd", "render_bwd", "gauss_bwd")
# the stages whose kernels stamp themselves in the device-clock mode (first workgroup's start to the last
# workgroup's end, no extra launches): every kernel of a captured tracking / mapping iteration except sh_eval /
# sh_bwd and the radix fallback
CLOCK_STAGES = ("preprocess", "ranges", "duplicate", "render_fwd", "render_bwd", "gauss_bwd")


GSR_TIMING_CLOCK = 0x100


def enable_timing(on: bool = True, clock_stages=None) -> None:
    """on: hipEvents around every stage.  clock_stages (names): device-clock
    stamps around those stages only -- works inside captured HIP graphs and
    accumulates over every replay."""
    if clock_stages:
        mask = 0
        for name in clock_stages:
            mask |= 1 << STAGES.index(name)
        lib.gsr_timing_enable(GSR_TIMING_CLOCK | mask)
    else:
        lib.gsr_timing_enable(1 if on else 0)


def read_timing() -> dict:
    n = len(STAGES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_longlong * n)()
    units = (ctypes.c_longlong * n)()
    lib.gsr_timing_read(ms, cnt, units, n)
    return {s: dict(ms=ms[i], launches=cnt[i], units=units[i],
                    avg_us=(1000.0 * ms[i] / cnt[i]) if cnt[i] else 0.0) for i, s in enumerate(STAGES)}
