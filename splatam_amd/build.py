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
DIAG = os.path.join(HERE, "_diag")  # experiment / diagnostics libraries that travel to the GPU box
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


def _compile(src: str, objdir: str = OBJDIR, extra=()) -> str:
    obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
    srcp = os.path.join(CSRC, src)
    deps = [srcp, os.path.join(ROOT, "include", "gsr.h"), os.path.join(ROOT, "include", "gsr_glue.h")] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [hipcc(), *flags(), *extra, "-c", srcp, "-o", obj]
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
    build_torch_binding(force=force)
    return LIB


TORCH_SRC = os.path.join(CSRC, "gsr_torch.cpp")


def torch_binding_path() -> str:
    import sysconfig
    return os.path.join(HERE, "_gsr_torch" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_torch_binding(force: bool = False) -> str:
    """The native torch binding of the drop-in path's per-iteration calls (csrc/gsr_torch.cpp): a host-only
    pybind11 module over libgsr.so (linked with an $ORIGIN rpath), in-tree so it travels with libgsr.so.
    Rebuilt when its sources are newer, when `force`, or when the torch it was built against (version, C++ ABI:
    the stamp file next to it) is not the one importing it now."""
    import sysconfig

    import torch
    from torch.utils import cpp_extension as ce
    out = torch_binding_path()
    stamp_file = out + ".stamp"
    stamp = f"{torch.__version__} abi={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"
    deps = [TORCH_SRC, os.path.join(ROOT, "include", "gsr.h")]  # (libgsr.so is resolved at load time)
    same_torch = os.path.exists(stamp_file) and open(stamp_file).read().strip() == stamp
    if (not force and same_torch and os.path.exists(out) and
            os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps)):
        return out
    inc = ce.include_paths() + [sysconfig.get_paths()["include"], os.path.join(ROOT, "include"), "/opt/rocm/include"]
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [hipcc(), "-x", "c++", "-std=c++17", "-O2", "-fPIC", "-shared", "-w", "-D__HIP_PLATFORM_AMD__=1",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_gsr_torch", "-DTORCH_API_INCLUDE_EXTENSION_H",
           *[f"-I{d}" for d in inc], TORCH_SRC, "-o", out, f"-L{tlib}", f"-L{HERE}", "-lgsr", "-lc10", "-lc10_hip",
           "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{tlib}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch binding build failed:\n{r.stdout[-4000:]}\n{r.stderr[-4000:]}")
    with open(stamp_file, "w") as f:
        f.write(stamp + "\n")
    return out


def build_diag() -> str:
    """Diagnostics library (tools/wgtime.py): libgsr with -DGSR_WGTIME=1 (per-workgroup render timelines),
    built to splatam_amd/_build_diag/libgsr_diag.so; loaded only through GSR_LIB by the diagnostics tool."""
    objdir = os.path.join(HERE, "_build_diag")
    os.makedirs(objdir, exist_ok=True)
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, ("-DGSR_WGTIME=1",)), SOURCES))
    lib = os.path.join(objdir, "libgsr_diag.so")
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in objs):
        r = subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return lib


def build_variant(tag: str, defines=()) -> str:
    """Timing-experiment library (tools/gpu_round.sh ab= / abbench= steps): libgsr built with extra -D flags into
    splatam_amd/_build_<tag>/libgsr_<tag>.so; loaded only through GSR_LIB."""
    objdir = os.path.join(HERE, f"_build_{tag}")
    os.makedirs(objdir, exist_ok=True)
    if isinstance(defines, dict):  # {"NAME": "value"} -> NAME=value (iterating a dict would drop the values)
        defines = [f"{k}={v}" for k, v in defines.items()]
    extra = tuple(f"-D{d}" for d in defines)
    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, extra), SOURCES))
    lib = os.path.join(objdir, f"libgsr_{tag}.so")
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in objs):
        r = subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    # the _build_<tag> trees stay on this machine (.gpurunignore); the experiment's library travels to the
    # GPU box from splatam_amd/_diag/ (delete that directory when the experiment is done)
    os.makedirs(DIAG, exist_ok=True)
    shutil.copy2(lib, os.path.join(DIAG, f"libgsr_{tag}.so"))
    return os.path.join(DIAG, f"libgsr_{tag}.so")


def build_from_rev(rev: str, tag: str) -> str:
    """A/B baseline without macros in the sources: libgsr built from the csrc/ and include/ trees of git
    revision `rev` (exported to a scratch directory) into splatam_amd/_diag/libgsr_<tag>.so, which
    tools/gpu_round.sh's ab= / abbench= steps load through GSR_LIB."""
    import io
    import tarfile
    import tempfile
    work = tempfile.mkdtemp(prefix=f"gsr_{tag}_")
    try:
        for sub in ("splatam_amd/csrc", "include"):
            r = subprocess.run(["git", "-C", ROOT, "archive", rev, sub], capture_output=True)
            if r.returncode != 0:
                raise RuntimeError(f"git archive {rev} {sub} failed: {r.stderr.decode(errors='replace')}")
            with tarfile.open(fileobj=io.BytesIO(r.stdout)) as tf:
                tf.extractall(work)
        csrc, inc = os.path.join(work, "splatam_amd", "csrc"), os.path.join(work, "include")
        objs = []
        for src in SOURCES:
            obj = os.path.join(work, os.path.splitext(src)[0] + ".o")
            base = flags()
            base = [f for i, f in enumerate(base) if f != "-I" and (i == 0 or base[i - 1] != "-I")]  # (drop -I pairs)
            cmd = [hipcc(), *base, "-I", inc, "-I", csrc, "-c", os.path.join(csrc, src), "-o", obj]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed for {src} at {rev}:\n{r.stderr}")
            objs.append(obj)
        os.makedirs(DIAG, exist_ok=True)
        lib = os.path.join(DIAG, f"libgsr_{tag}.so")
        r = subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        return lib
    finally:
        shutil.rmtree(work, ignore_errors=True)

if __name__ == "__main__":
    if "--from-rev" in sys.argv:  # python -m splatam_amd.build --from-rev REV TAG
        i = sys.argv.index("--from-rev")
        print(build_from_rev(sys.argv[i + 1], sys.argv[i + 2]))
    else:
        print(build(force="--force" in sys.argv))
