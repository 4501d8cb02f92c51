"""CPU checks of the drop-in boundary: libgsr.so loads and exports every symbol
include/*.h declare, the ctypes mirror matches the header, and the Python
wrapper hands `_C` exactly the argument lists the reference wrapper does
(golden: tests/golden/abi_signature.json, captured from the reference)."""
import ctypes
import inspect
import json
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsr.h")
GOLDEN = os.path.join(ROOT, "tests", "golden", "abi_signature.json")


def header_functions():
    import glob
    txt = "\n".join(open(h).read() for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\**(gsr_[a-z_0-9]+)\s*\(", txt, re.M)))


def header_struct_fields(name):
    txt = open(HEADER).read() + open(os.path.join(os.path.dirname(HEADER), "gsr_glue.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), txt, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    # "type name", "type name[N]" or "type a, b, c" per declaration
    names = []
    for d in body.split(";"):
        for part in d.strip().split(","):
            if part.strip():
                names.append(re.findall(r"(\w+)(?:\[\d+\])?$", part.strip())[0])
    return names


def test_library_exports_every_header_symbol():
    from splatam_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    fns = header_functions()
    assert len(fns) >= 10, fns
    missing = [f for f in fns if not hasattr(lib, f)]
    assert not missing, missing
    assert set(fns) == set(_lib.SIGNATURES), "ctypes signature table out of sync with include/*.h"
    assert lib.gsr_abi_version() == 8


@pytest.mark.parametrize("cname,pyname", [("gsr_settings", "GsrSettings"), ("gsr_gaussians", "GsrGaussians"),
                                          ("gsr_grads", "GsrGrads"), ("gsr_track_xform", "GsrTrackXform"),
                                          ("gsr_pose_track", "GsrPoseTrack"), ("gsr_map_adam", "GsrMapAdam")])
def test_ctypes_structs_match_header(cname, pyname):
    from splatam_amd import _lib
    fields = header_struct_fields(cname)
    assert [f[0] for f in getattr(_lib, pyname)._fields_] == fields


def test_buffer_size_queries_match_python_layout():
    from splatam_amd._lib import lib
    from splatam_amd.layout import image_layout
    for W, H in ((640, 480), (100, 75), (1200, 680)):
        assert lib.gsr_image_buffer_bytes(W, H) == image_layout(W, H)["total"]
    assert lib.gsr_geom_buffer_bytes(300000) > 48 * 300000
    assert lib.gsr_binning_buffer_bytes(677000, 640, 480) >= 4 * 677000


def _describe(x):
    if isinstance(x, torch.Tensor):
        return {"kind": "tensor", "dtype": str(x.dtype).replace("torch.", ""), "shape": list(x.shape),
                "numel": int(x.numel())}
    if isinstance(x, bool):
        return {"kind": "bool", "value": x}
    if isinstance(x, int):
        return {"kind": "int", "value": x}
    if isinstance(x, float):
        return {"kind": "float", "value": x}
    return {"kind": type(x).__name__}


class RecordingC:
    def __init__(self):
        self.calls = []

    def rasterize_gaussians(self, *args):
        self.calls.append(("rasterize_gaussians", [_describe(a) for a in args]))
        P, H, W = args[1].shape[0], args[12], args[13]
        u8 = torch.zeros(16, dtype=torch.uint8)
        return (7, torch.zeros(3, H, W), torch.zeros(P, dtype=torch.int32), u8, u8, u8, torch.zeros(1, H, W))

    def rasterize_gaussians_backward(self, *args, needs=None):  # `needs`: keyword-only extension
        self.calls.append(("rasterize_gaussians_backward", [_describe(a) for a in args]))
        P = args[1].shape[0]
        M = args[13].shape[1] if args[13].numel() else 0
        z = torch.zeros
        return (z(P, 3), z(P, 3), z(P, 1), z(P, 3), z(P, 6), z(P, M, 3), z(P, 3), z(P, 4))

    def mark_visible(self, *args):
        self.calls.append(("mark_visible", [_describe(a) for a in args]))
        return torch.zeros(args[0].shape[0], dtype=torch.bool)


def test_wrapper_passes_reference_argument_lists(monkeypatch):
    """Same positional args (types, dtypes, shapes, scalars) as the reference wrapper, power 1 and 2."""
    from splatam_amd import rasterizer
    gold = json.load(open(GOLDEN))
    rec = RecordingC()
    monkeypatch.setattr(rasterizer, "_C", rec)
    assert list(rasterizer.GaussianRasterizationSettings._fields) == gold["settings_fields"]
    torch.manual_seed(0)
    st = rasterizer.GaussianRasterizationSettings(48, 64, 1.0, 0.75, torch.zeros(3), 1.0, torch.eye(4).unsqueeze(0),
                                                  torch.eye(4).unsqueeze(0), 0, torch.zeros(3), False)
    P = 10
    leaf = lambda *s: torch.rand(*s, requires_grad=True)  # noqa: E731
    m3, m2, op, col, sc, ro = leaf(P, 3), torch.zeros(P, 3, requires_grad=True), leaf(P, 1), leaf(P, 3), leaf(P, 3), \
        leaf(P, 4)
    for power in (1, 2):
        rec.calls.clear()
        im, radii, depth = rasterizer.GaussianRasterizer(st, backward_power=power)(
            means3D=m3, means2D=m2, opacities=op, colors_precomp=col, scales=sc, rotations=ro)
        im.sum().backward()
        got = {name: args for name, args in rec.calls}
        want = gold[f"power{power}"]
        assert got["rasterize_gaussians"] == want["rasterize_gaussians"]
        assert got["rasterize_gaussians_backward"] == want["rasterize_gaussians_backward"]
        assert [_describe(t) for t in (im, radii, depth)] == want["outputs"]
    rec.calls.clear()
    rasterizer.GaussianRasterizer(st).markVisible(m3.detach())
    assert rec.calls[0][1] == gold["mark_visible"]


def test_wrapper_error_messages_match_reference():
    from splatam_amd import rasterizer
    gold = json.load(open(GOLDEN))
    st = rasterizer.GaussianRasterizationSettings(8, 8, 1.0, 1.0, torch.zeros(3), 1.0, torch.eye(4)[None],
                                                  torch.eye(4)[None], 0, torch.zeros(3), False)
    z = torch.zeros(2, 3)
    for case, kw in (("no_colors", dict(scales=z, rotations=torch.zeros(2, 4))), ("no_geometry", dict(colors_precomp=z))):
        with pytest.raises(Exception) as ei:
            rasterizer.GaussianRasterizer(st)(means3D=z, means2D=z, opacities=torch.zeros(2, 1), **kw)
        assert str(ei.value) == gold[f"error_{case}"]["message"]
        assert type(ei.value).__name__ == gold[f"error_{case}"]["type"]


def test_no_cpu_fallback():
    """The product path refuses CPU tensors instead of silently computing elsewhere."""
    from splatam_amd import _C
    z = torch.zeros(4, 3)
    with pytest.raises(RuntimeError, match="ROCm devices only"):
        _C.rasterize_gaussians(torch.zeros(3), z, z, torch.zeros(4, 1), z, torch.zeros(4, 4), 1.0, torch.Tensor([]),
                               torch.eye(4)[None], torch.eye(4)[None], 1.0, 1.0, 8, 8, torch.Tensor([]), 0,
                               torch.zeros(3), False)


def test_alias_packages():
    import diff_gaussian_rasterization as upstream
    import hessian_diff_gaussian_rasterization_w_depth as fork
    assert upstream.GaussianRasterizationSettings is fork.GaussianRasterizationSettings
    assert list(inspect.signature(upstream.GaussianRasterizer.__init__).parameters) == ["self", "raster_settings"]
    assert list(inspect.signature(fork.GaussianRasterizer.__init__).parameters) == ["self", "raster_settings",
                                                                                    "backward_power"]
    assert hasattr(upstream, "_C") and hasattr(fork._C, "rasterize_gaussians_backward")


def test_gsr_lib_override_stays_strict(tmp_path):
    """GSR_LIB alone loads another library under the full symbol / ABI checks; only GSR_LIB_AB=1 (an A/B
    baseline from an older revision) relaxes them (a stale ABI-4 build must not load silently)."""
    import subprocess
    import sys
    src = tmp_path / "stale.c"
    src.write_text("int gsr_abi_version(void) { return 4; }\n")
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    code = "import splatam_amd._lib"
    base = {k: v for k, v in os.environ.items() if k not in ("GSR_LIB", "GSR_LIB_AB")}
    strict = subprocess.run([sys.executable, "-c", code], env=dict(base, GSR_LIB=str(so)), capture_output=True,
                            text=True, cwd=ROOT)
    assert strict.returncode != 0 and "lacks" in strict.stderr, strict.stderr[-500:]
    relaxed = subprocess.run([sys.executable, "-c", code], env=dict(base, GSR_LIB=str(so), GSR_LIB_AB="1"),
                             capture_output=True, text=True, cwd=ROOT)
    assert relaxed.returncode == 0, relaxed.stderr[-500:]


def test_gsr_lib_override_keeps_calls_on_ctypes():
    """The native binding links the in-tree libgsr.so, so a library selected through GSR_LIB (A/B builds) must
    take every call, the drop-in path's two included: _C then keeps them on ctypes."""
    import subprocess
    import sys
    code = "from splatam_amd import _C; print(_C._NATIVE_ON)"
    base = {k: v for k, v in os.environ.items() if k not in ("GSR_LIB", "GSR_LIB_AB", "GSR_NATIVE_BINDING")}
    lib = os.path.join(ROOT, "splatam_amd", "libgsr.so")
    default = subprocess.run([sys.executable, "-c", code], env=base, capture_output=True, text=True, cwd=ROOT)
    override = subprocess.run([sys.executable, "-c", code], env=dict(base, GSR_LIB=lib), capture_output=True,
                              text=True, cwd=ROOT)
    assert default.returncode == 0 and default.stdout.strip() == "True", default.stderr[-500:]
    assert override.returncode == 0 and override.stdout.strip() == "False", override.stderr[-500:]
