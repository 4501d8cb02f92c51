"""ctypes front-end of the CPU restatement in ``oracle/gsr_oracle.c``.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s cpu_baseline leg, never by the product package ``splatam_amd``.

The restatement follows the reference CUDA sources line by line (see the
header of gsr_oracle.c).  Kernel-level parity is "parity unpinned" against the
reference binary (it cannot be built or run here); the oracle itself is pinned
in tests/ by torch.autograd through a dense formulation and by finite
differences in float64.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
UPSTREAM = 0  # backward.cu:586-748 decomposition (power == 1 only)
FUSED = 1     # backward.cu:850-1140 per-pair chain with powf(., power)


def build() -> None:
    """Compile both precisions of the oracle (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_libs: dict = {}
_threads = 0  # 0: OpenMP default (OMP_NUM_THREADS or every core); results do not depend on it


def threads() -> int:
    """Threads the oracle's parallel loops use."""
    lib = _lib(np.float32)[0]
    return int(lib.oracle_threads())


def set_threads(n: int) -> None:
    """Threads of the oracle's parallel loops (0 = OpenMP default).  The results are
    identical for any count (fixed-order per-instance sums, see gsr_oracle.c)."""
    global _threads
    _threads = int(n)
    for lib, *_ in _libs.values():
        lib.oracle_set_threads(_threads)


def _lib(dtype):
    key = np.dtype(dtype).name
    if key not in _libs:
        name = {"float32": "libgsr_oracle_f32.so", "float64": "libgsr_oracle_f64.so"}[key]
        path = os.path.join(_BUILD, name)
        if key == "float32" and os.environ.get("GSR_ORACLE_F32_LIB"):  # tools/alpha_forms.py experiment builds
            path = os.environ["GSR_ORACLE_F32_LIB"]
        if not os.path.exists(path):
            build()
        lib = ctypes.CDLL(path)
        real = ctypes.c_float if key == "float32" else ctypes.c_double
        P = ctypes.POINTER

        class In(ctypes.Structure):
            _fields_ = [("P", ctypes.c_int), ("D", ctypes.c_int), ("M", ctypes.c_int),
                        ("W", ctypes.c_int), ("H", ctypes.c_int),
                        ("bg", P(real)), ("means3D", P(real)), ("shs", P(real)),
                        ("colors", P(real)), ("opacities", P(real)), ("scales", P(real)),
                        ("rotations", P(real)), ("cov3D_precomp", P(real)),
                        ("scale_modifier", real), ("view", P(real)), ("proj", P(real)),
                        ("campos", P(real)), ("tan_fovx", real), ("tan_fovy", real)]

        class FwdOut(ctypes.Structure):
            _fields_ = [("out_color", P(real)), ("out_depth", P(real)), ("radii", P(ctypes.c_int)),
                        ("means2D", P(real)), ("depths", P(real)), ("conic_opacity", P(real)),
                        ("rgb", P(real)), ("clamped", P(ctypes.c_ubyte)),
                        ("tiles_touched", P(ctypes.c_int)), ("final_T", P(real)),
                        ("n_contrib", P(ctypes.c_int)), ("ranges", P(ctypes.c_int)),
                        ("point_list", P(ctypes.c_int)), ("unstable_pix", P(ctypes.c_ubyte)),
                        ("unstable", P(ctypes.c_ubyte))]

        class Grads(ctypes.Structure):
            _fields_ = [("dmeans2D", P(real)), ("dcolors", P(real)), ("dopacity", P(real)),
                        ("dmeans3D", P(real)), ("dcov3D", P(real)), ("dsh", P(real)),
                        ("dscales", P(real)), ("drot", P(real))]

        lib.oracle_forward.argtypes = [P(In), P(FwdOut), P(ctypes.c_longlong)]
        lib.oracle_forward.restype = ctypes.c_int
        lib.oracle_backward.argtypes = [P(In), P(FwdOut), P(real), ctypes.c_int, ctypes.c_int, P(Grads),
                                        P(ctypes.c_longlong), P(ctypes.c_longlong), P(Grads)]
        lib.oracle_backward.restype = ctypes.c_int
        lib.oracle_free_list.argtypes = [P(FwdOut)]
        lib.oracle_mark_visible.argtypes = [ctypes.c_int, P(real), P(real), P(ctypes.c_ubyte)]
        lib.oracle_set_threads.argtypes = [ctypes.c_int]
        lib.oracle_threads.restype = ctypes.c_int
        lib.oracle_set_threads(_threads)
        _libs[key] = (lib, real, In, FwdOut, Grads)
    return _libs[key]


def _ptr(a, ctype):
    if a is None:
        return ctypes.POINTER(ctype)()
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def _arr(a, dtype):
    if a is None:
        return None
    a = np.asarray(a, dtype=dtype)
    return np.ascontiguousarray(a)


@dataclass
class ForwardResult:
    """Forward outputs plus the intermediate state the backward needs."""
    num_rendered: int
    color: np.ndarray          # [3,H,W]
    depth: np.ndarray          # [1,H,W]
    radii: np.ndarray          # [P] int32
    means2D: np.ndarray        # [P,2] pixel coordinates
    depths: np.ndarray         # [P]
    conic_opacity: np.ndarray  # [P,4]
    rgb: np.ndarray            # [P,3]
    clamped: np.ndarray        # [P,3] uint8
    tiles_touched: np.ndarray  # [P] int32
    final_T: np.ndarray        # [H,W]
    n_contrib: np.ndarray      # [H,W] int32
    ranges: np.ndarray         # [tiles,2] int32
    point_list: np.ndarray     # [num_rendered] int32
    pair_evals: int
    unstable: np.ndarray       # [P] bool: evaluated at a pixel with an alpha / T decision near its threshold
    unstable_pix: np.ndarray   # [H,W] bool: an alpha / T(1e-4) decision near its threshold
    unstable_depth_pix: np.ndarray  # [H,W] bool: a T = 0.5 crossing (median depth) near its threshold
    _keep: dict = field(default_factory=dict, repr=False)


def forward(means3D, opacities, *, view, proj, campos, tanfovx, tanfovy, H, W, bg=(0.0, 0.0, 0.0),
            shs=None, colors=None, scales=None, rotations=None, cov3D=None, scale_modifier=1.0,
            sh_degree=0, dtype=np.float32) -> ForwardResult:
    """Reference forward (rasterizer_impl.cu:198-339) on the CPU."""
    lib, real, In, FwdOut, _ = _lib(dtype)
    keep = dict(
        means3D=_arr(means3D, dtype).reshape(-1, 3), opac=_arr(opacities, dtype).reshape(-1),
        shs=_arr(shs, dtype), colors=_arr(colors, dtype), scales=_arr(scales, dtype),
        rot=_arr(rotations, dtype), cov3D=_arr(cov3D, dtype),
        view=_arr(view, dtype).reshape(-1), proj=_arr(proj, dtype).reshape(-1),
        campos=_arr(campos, dtype).reshape(-1), bg=_arr(bg, dtype).reshape(-1))
    P = keep["means3D"].shape[0]
    M = 0 if keep["shs"] is None or keep["shs"].size == 0 else keep["shs"].shape[1]
    inp = In(P=P, D=int(sh_degree), M=M, W=int(W), H=int(H), bg=_ptr(keep["bg"], real),
             means3D=_ptr(keep["means3D"], real), shs=_ptr(keep["shs"] if M else None, real),
             colors=_ptr(keep["colors"], real), opacities=_ptr(keep["opac"], real),
             scales=_ptr(keep["scales"], real), rotations=_ptr(keep["rot"], real),
             cov3D_precomp=_ptr(keep["cov3D"], real), scale_modifier=float(scale_modifier),
             view=_ptr(keep["view"], real), proj=_ptr(keep["proj"], real),
             campos=_ptr(keep["campos"], real), tan_fovx=float(tanfovx), tan_fovy=float(tanfovy))
    gx, gy = (W + 15) // 16, (H + 15) // 16
    o = dict(color=np.zeros((3, H, W), dtype), depth=np.zeros((1, H, W), dtype),
             radii=np.zeros(P, np.int32), means2D=np.zeros((P, 2), dtype), depths=np.zeros(P, dtype),
             conic_opacity=np.zeros((P, 4), dtype), rgb=np.zeros((P, 3), dtype),
             clamped=np.zeros((P, 3), np.uint8), tiles_touched=np.zeros(P, np.int32),
             final_T=np.zeros((H, W), dtype), n_contrib=np.zeros((H, W), np.int32),
             ranges=np.zeros((gx * gy, 2), np.int32))
    unstable_pix = np.zeros((H, W), np.uint8)
    unstable = np.zeros(P, np.uint8)
    fo = FwdOut(unstable_pix=_ptr(unstable_pix, ctypes.c_ubyte), unstable=_ptr(unstable, ctypes.c_ubyte),
                out_color=_ptr(o["color"], real), out_depth=_ptr(o["depth"], real),
                radii=_ptr(o["radii"], ctypes.c_int), means2D=_ptr(o["means2D"], real),
                depths=_ptr(o["depths"], real), conic_opacity=_ptr(o["conic_opacity"], real),
                rgb=_ptr(o["rgb"], real), clamped=_ptr(o["clamped"], ctypes.c_ubyte),
                tiles_touched=_ptr(o["tiles_touched"], ctypes.c_int), final_T=_ptr(o["final_T"], real),
                n_contrib=_ptr(o["n_contrib"], ctypes.c_int), ranges=_ptr(o["ranges"], ctypes.c_int))
    evals = ctypes.c_longlong(0)
    n = lib.oracle_forward(ctypes.byref(inp), ctypes.byref(fo), ctypes.byref(evals))
    pl = np.ctypeslib.as_array(fo.point_list, shape=(max(n, 1),))[:n].copy()
    lib.oracle_free_list(ctypes.byref(fo))
    keep["inp"] = inp
    keep["dtype"] = np.dtype(dtype)
    keep["M"] = M
    return ForwardResult(num_rendered=n, point_list=pl, pair_evals=evals.value, _keep=keep,
                         unstable=unstable.astype(bool), unstable_pix=(unstable_pix & 1).astype(bool),
                         unstable_depth_pix=(unstable_pix & 2).astype(bool), **o)


def backward(fr: ForwardResult, dL_dcolor, *, power=1, mode=UPSTREAM, error_scale=False) -> dict:
    """Reference backward; returns a dict with the 8 gradient arrays of
    rasterize_points.cu:195 plus pair counters.  error_scale=True (upstream mode): also
    g["scale"], the per-element error scale of each gradient (|Jacobian of the chain| applied
    to each Gaussian's sums of |per-pair term|): a float32 implementation's error on an
    element is a small multiple of eps * scale, whatever cancellation the sum has."""
    dtype = fr._keep["dtype"]
    lib, real, In, FwdOut, Grads = _lib(dtype)
    P = fr.radii.shape[0]
    M = fr._keep["M"]
    H, W = fr.final_T.shape
    g = dict(dmeans2D=np.zeros((P, 3), dtype), dcolors=np.zeros((P, 3), dtype),
             dopacity=np.zeros((P, 1), dtype), dmeans3D=np.zeros((P, 3), dtype),
             dcov3D=np.zeros((P, 6), dtype), dsh=np.zeros((P, M, 3), dtype),
             dscales=np.zeros((P, 3), dtype), drot=np.zeros((P, 4), dtype))
    fo = FwdOut(out_color=_ptr(fr.color, real), out_depth=_ptr(fr.depth, real),
                radii=_ptr(fr.radii, ctypes.c_int), means2D=_ptr(fr.means2D, real),
                depths=_ptr(fr.depths, real), conic_opacity=_ptr(fr.conic_opacity, real),
                rgb=_ptr(fr.rgb, real), clamped=_ptr(fr.clamped, ctypes.c_ubyte),
                tiles_touched=_ptr(fr.tiles_touched, ctypes.c_int), final_T=_ptr(fr.final_T, real),
                n_contrib=_ptr(fr.n_contrib, ctypes.c_int), ranges=_ptr(fr.ranges, ctypes.c_int),
                point_list=_ptr(fr.point_list, ctypes.c_int))
    go = Grads(dmeans2D=_ptr(g["dmeans2D"], real), dcolors=_ptr(g["dcolors"], real),
               dopacity=_ptr(g["dopacity"], real), dmeans3D=_ptr(g["dmeans3D"], real),
               dcov3D=_ptr(g["dcov3D"], real), dsh=_ptr(g["dsh"] if M else None, real),
               dscales=_ptr(g["dscales"], real), drot=_ptr(g["drot"], real))
    dpix = np.ascontiguousarray(np.asarray(dL_dcolor, dtype).reshape(3, H, W))
    ev, ct = ctypes.c_longlong(0), ctypes.c_longlong(0)
    gsp = None
    if error_scale:
        sc = {k: np.zeros_like(v) for k, v in g.items()}
        gsp = Grads(dmeans2D=_ptr(sc["dmeans2D"], real), dcolors=_ptr(sc["dcolors"], real),
                    dopacity=_ptr(sc["dopacity"], real), dmeans3D=_ptr(sc["dmeans3D"], real),
                    dcov3D=_ptr(sc["dcov3D"], real), dsh=_ptr(sc["dsh"] if M else None, real),
                    dscales=_ptr(sc["dscales"], real), drot=_ptr(sc["drot"], real))
    rc = lib.oracle_backward(ctypes.byref(fr._keep["inp"]), ctypes.byref(fo), _ptr(dpix, real), int(mode),
                             int(power), ctypes.byref(go), ctypes.byref(ev), ctypes.byref(ct),
                             ctypes.byref(gsp) if gsp is not None else None)
    if rc != 0:
        raise ValueError("oracle_backward: upstream mode (and error_scale) support power == 1 only")
    if error_scale:
        g["scale"] = sc
    g["pair_evals"] = ev.value
    g["pair_contrib"] = ct.value
    return g


def mark_visible(means3D, view, dtype=np.float32) -> np.ndarray:
    lib, real, *_ = _lib(dtype)
    m = _arr(means3D, dtype).reshape(-1, 3)
    v = _arr(view, dtype).reshape(-1)
    out = np.zeros(m.shape[0], np.uint8)
    lib.oracle_mark_visible(m.shape[0], _ptr(m, real), _ptr(v, real), _ptr(out, ctypes.c_ubyte))
    return out.astype(bool)
