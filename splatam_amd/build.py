"""Builds libgsr.so (all HIP kernels + the C ABI of include/gsr.h) for gfx950.

Invoked by __graft_entry__.build() and by `python -m splatam_amd.build`.
Plain hipcc, in-tree output (splatam_amd/libgsr.so), so the shared object
travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
OBJDIR = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libgsr.so")
SOURCES = ["gsr_forward.hip", "gsr_backward.hip", "gsr_backward_power.hip", "gsr_capi.hip", "gsr_glue.hip",
           "gsr_mapping.hip", "gsr_sh.hip"]
ARCH = os.environ.get("GSR_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the MI355X build needs ROCm's hipcc")


def flags():
    # -fno-slp-vectorize: keep f32 adds/muls single-issue; SLP packing into v_pk_*_f32
    # splits every DPP-fused add into v_mov_b32_dpp + v_pk_add (cdna_hip_programming.md App. B).
    return ["-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
            "-fno-slp-vectorize",
            "-I", os.path.join(ROOT, "include"), "-I", CSRC]


def _compile(src: str) -> str:
    obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
    srcp = os.path.join(CSRC, src)
    deps = [srcp, os.path.join(ROOT, "include", "gsr.h"), os.path.join(ROOT, "include", "gsr_glue.h")] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [hipcc(), *flags(), "-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    if force:
        for f in os.listdir(OBJDIR):
            os.remove(os.path.join(OBJDIR, f))
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
