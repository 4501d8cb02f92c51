"""Generates the golden fixtures in tests/golden/ by importing the REFERENCE's own
Python code from /root/reference (read-only) on the CPU.

What is captured (all small):
  * abi_signature.json -- the exact positional argument lists that the reference
    autograd wrapper (hessian_diff_gaussian_rasterization_w_depth/__init__.py)
    passes to its `_C` extension in forward and backward, recorded through a
    stub `_C` module (type / dtype / shape / scalar value of every argument);
  * glue_*.npz -- outputs of SplaTAM's caller glue on seeded inputs:
    setup_camera (utils/recon_helpers.py:4-27), transform_to_frame,
    transformed_params2rendervar, transformed_params2depthplussilhouette,
    get_depth_and_silhouette (utils/slam_helpers.py), build_rotation
    (utils/slam_external.py:25-42), calc_ssim (slam_external.py:61-97, value and
    gradient) and the mapping transform's parameter gradients, with `.cuda()` /
    device="cuda" redirected to the CPU;
  * ref_params.npz -- a small parameter checkpoint written by the reference's own
    save_params (utils/common_utils.py:35-42), for checkpoint interop.

The reference's CUDA kernels cannot run here (no nvcc / NVIDIA GPU), so no
kernel-level golden exists; see DESIGN.md "Parity".  Run:
    python tests/golden/make_goldens.py
"""
from __future__ import annotations

import importlib
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _cpu_everywhere():
    """Redirect the reference's hard-coded CUDA placement to the CPU."""
    torch.Tensor.cuda = lambda self, *a, **k: self

    def strip(fn):
        def wrapped(*a, **k):
            if k.get("device") in ("cuda", torch.device("cuda")) or (isinstance(k.get("device"), str)
                                                                      and k["device"].startswith("cuda")):
                k["device"] = "cpu"
            return fn(*a, **k)
        return wrapped

    for name in ("tensor", "zeros", "ones", "eye", "zeros_like", "ones_like", "empty", "full"):
        setattr(torch, name, strip(getattr(torch, name)))


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


class StubC(types.ModuleType):
    """Stands in for the compiled `_C`: records the argument lists."""

    def __init__(self):
        super().__init__("_C")
        self.calls = []

    def rasterize_gaussians(self, *args):
        self.calls.append(("rasterize_gaussians", [_describe(a) for a in args]))
        bg, means3D = args[0], args[1]
        P, H, W = means3D.shape[0], args[12], args[13]
        u8 = torch.zeros(16, dtype=torch.uint8)
        return (7, torch.zeros(3, H, W), torch.zeros(P, dtype=torch.int32), u8, u8, u8, torch.zeros(1, H, W))

    def rasterize_gaussians_backward(self, *args):
        self.calls.append(("rasterize_gaussians_backward", [_describe(a) for a in args]))
        means3D = args[1]
        P = means3D.shape[0]
        sh = args[13]
        M = sh.shape[1] if sh.numel() else 0
        z = torch.zeros
        return (z(P, 3), z(P, 3), z(P, 1), z(P, 3), z(P, 6), z(P, M, 3), z(P, 3), z(P, 4))

    def mark_visible(self, *args):
        self.calls.append(("mark_visible", [_describe(a) for a in args]))
        return torch.zeros(args[0].shape[0], dtype=torch.bool)


def load_reference_wrapper(stub):
    pkg_parent = os.path.join(REF, "hessian-diff-gaussian-rasterization-w-depth")
    sys.path.insert(0, pkg_parent)
    sys.modules["hessian_diff_gaussian_rasterization_w_depth._C"] = stub
    mod = importlib.import_module("hessian_diff_gaussian_rasterization_w_depth")
    sys.path.remove(pkg_parent)
    return mod


def main():
    torch.manual_seed(0)
    _cpu_everywhere()
    stub = StubC()
    ref = load_reference_wrapper(stub)
    # SplaTAM's caller glue imports the upstream module name; serve it the reference wrapper
    sys.modules["diff_gaussian_rasterization"] = ref
    sys.path.insert(0, REF)
    recon = importlib.import_module("utils.recon_helpers")
    slam = importlib.import_module("utils.slam_helpers")
    ext = importlib.import_module("utils.slam_external")

    # ---- setup_camera (Replica room0 intrinsics scaled to 640x480, non-trivial pose)
    W, H = 640, 480
    K = np.array([[320.0, 0, 319.7333], [0, 423.5294, 239.6471], [0, 0, 1]])
    ang = 0.3
    w2c = np.eye(4)
    w2c[:3, :3] = np.array([[np.cos(ang), 0, np.sin(ang)], [0, 1, 0], [-np.sin(ang), 0, np.cos(ang)]])
    w2c[:3, 3] = [0.1, -0.2, 0.3]
    cam = recon.setup_camera(W, H, K, w2c)
    np.savez(os.path.join(OUT, "glue_setup_camera.npz"), W=W, H=H, K=K, w2c=w2c,
             viewmatrix=cam.viewmatrix.numpy(), projmatrix=cam.projmatrix.numpy(), campos=cam.campos.numpy(),
             tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=cam.bg.numpy(), scale_modifier=cam.scale_modifier,
             sh_degree=cam.sh_degree, prefiltered=cam.prefiltered)

    # ---- transform_to_frame + rendervar builders (iso and aniso)
    g = torch.Generator().manual_seed(1)
    P, T = 64, 3
    for iso in (True, False):
        params = {
            "means3D": torch.randn(P, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0]),
            "rgb_colors": torch.rand(P, 3, generator=g),
            "unnorm_rotations": torch.randn(P, 4, generator=g),
            "logit_opacities": torch.randn(P, 1, generator=g),
            "log_scales": torch.randn(P, 1 if iso else 3, generator=g) - 3.0,
            "cam_unnorm_rots": torch.randn(1, 4, T, generator=g),
            "cam_trans": 0.1 * torch.randn(1, 3, T, generator=g),
        }
        tg = slam.transform_to_frame(params, 1, gaussians_grad=True, camera_grad=True)
        rv = slam.transformed_params2rendervar(params, tg)
        dv = slam.transformed_params2depthplussilhouette(params, torch.tensor(w2c).float(), tg)
        name = "iso" if iso else "aniso"
        np.savez(os.path.join(OUT, f"glue_transform_{name}.npz"),
                 **{f"param_{k}": v.numpy() for k, v in params.items()},
                 time_idx=1, w2c=w2c.astype(np.float32),
                 tg_means3D=tg["means3D"].detach().numpy(), tg_unnorm_rotations=tg["unnorm_rotations"].detach().numpy(),
                 rv_rotations=rv["rotations"].detach().numpy(), rv_opacities=rv["opacities"].detach().numpy(),
                 rv_scales=rv["scales"].detach().numpy(), rv_colors=rv["colors_precomp"].detach().numpy(),
                 dv_colors=dv["colors_precomp"].detach().numpy())
    q = torch.randn(16, 4, generator=g)
    np.savez(os.path.join(OUT, "glue_build_rotation.npz"), q=q.numpy(), R=ext.build_rotation(q).numpy())

    # ---- calc_ssim (slam_external.py:61-97): value and gradient w.r.t. the first image (mapping loss)
    g2 = torch.Generator().manual_seed(2)
    img1 = torch.rand(3, 37, 53, generator=g2, requires_grad=True)
    img2 = (img1.detach() + 0.1 * torch.randn(3, 37, 53, generator=g2)).clamp(0.0, 1.0)
    ssim = ext.calc_ssim(img1, img2)
    ssim.backward()
    np.savez(os.path.join(OUT, "glue_ssim.npz"), img1=img1.detach().numpy(), img2=img2.numpy(),
             ssim=ssim.detach().numpy(), grad_img1=img1.grad.numpy())

    # ---- mapping transform backward: transform_to_frame(gaussians_grad=True, camera_grad=False) +
    # rendervar builders, seeded upstream gradients on every rendervar output
    for iso in (True, False):
        params = {
            "means3D": torch.randn(P, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0]),
            "rgb_colors": torch.rand(P, 3, generator=g),
            "unnorm_rotations": torch.randn(P, 4, generator=g),
            "logit_opacities": torch.randn(P, 1, generator=g),
            "log_scales": torch.randn(P, 1 if iso else 3, generator=g) - 3.0,
            "cam_unnorm_rots": torch.randn(1, 4, T, generator=g),
            "cam_trans": 0.1 * torch.randn(1, 3, T, generator=g),
        }
        for k in ("means3D", "rgb_colors", "unnorm_rotations", "logit_opacities", "log_scales"):
            params[k].requires_grad_(True)
        tg = slam.transform_to_frame(params, 2, gaussians_grad=True, camera_grad=False)
        rv = slam.transformed_params2rendervar(params, tg)
        dv = slam.transformed_params2depthplussilhouette(params, torch.tensor(w2c).float(), tg)
        ups = {"g_means": torch.randn(P, 3, generator=g), "g_rot": torch.randn(P, 4, generator=g),
               "g_opac": torch.randn(P, 1, generator=g), "g_scales": torch.randn(P, 3, generator=g),
               "g_dcol": torch.randn(P, 3, generator=g)}
        total = ((rv["means3D"] * ups["g_means"]).sum() + (rv["rotations"] * ups["g_rot"]).sum()
                 + (rv["opacities"] * ups["g_opac"]).sum() + (rv["scales"] * ups["g_scales"]).sum()
                 + (dv["colors_precomp"] * ups["g_dcol"]).sum())
        total.backward()
        name = "iso" if iso else "aniso"
        np.savez(os.path.join(OUT, f"glue_map_transform_{name}.npz"),
                 **{f"param_{k}": v.detach().numpy() for k, v in params.items()},
                 **{k: v.numpy() for k, v in ups.items()}, time_idx=2, w2c=w2c.astype(np.float32),
                 **{f"grad_{k}": params[k].grad.numpy()
                    for k in ("means3D", "unnorm_rotations", "logit_opacities", "log_scales")})

    # ---- params*.npz written by the reference's own save_params (utils/common_utils.py:35-42)
    cu = importlib.import_module("utils.common_utils")
    import tempfile
    g3 = torch.Generator().manual_seed(3)
    ck = {"means3D": torch.randn(16, 3, generator=g3), "rgb_colors": torch.rand(16, 3, generator=g3),
          "unnorm_rotations": torch.randn(16, 4, generator=g3), "logit_opacities": torch.randn(16, 1, generator=g3),
          "log_scales": torch.randn(16, 1, generator=g3), "cam_unnorm_rots": torch.randn(1, 4, 5, generator=g3),
          "cam_trans": torch.randn(1, 3, 5, generator=g3), "timestep": torch.zeros(16),
          "intrinsics": np.eye(3, dtype=np.float32), "w2c": np.eye(4, dtype=np.float32), "org_width": 640,
          "org_height": 480, "gt_w2c_all_frames": np.stack([np.eye(4, dtype=np.float32)] * 5),
          "keyframe_time_indices": np.array([0, 5])}
    with tempfile.TemporaryDirectory() as td:
        cu.save_params(ck, td)
        with open(os.path.join(td, "params.npz"), "rb") as f:
            blob = f.read()
    with open(os.path.join(OUT, "ref_params.npz"), "wb") as f:
        f.write(blob)

    # ---- ABI capture: forward + backward through the reference autograd wrapper
    st = ref.GaussianRasterizationSettings(
        image_height=48, image_width=64, tanfovx=1.0, tanfovy=0.75, bg=torch.zeros(3), scale_modifier=1.0,
        viewmatrix=torch.eye(4).unsqueeze(0), projmatrix=torch.eye(4).unsqueeze(0), sh_degree=0,
        campos=torch.zeros(3), prefiltered=False)
    P = 10
    m3 = torch.randn(P, 3, requires_grad=True)
    m2 = torch.zeros(P, 3, requires_grad=True)
    op = torch.rand(P, 1, requires_grad=True)
    col = torch.rand(P, 3, requires_grad=True)
    sc = torch.rand(P, 3, requires_grad=True)
    ro = torch.randn(P, 4, requires_grad=True)
    abi = {"settings_fields": list(ref.GaussianRasterizationSettings._fields)}
    for power in (1, 2):
        stub.calls.clear()
        im, radii, depth = ref.GaussianRasterizer(st, backward_power=power)(
            means3D=m3, means2D=m2, opacities=op, colors_precomp=col, scales=sc, rotations=ro)
        im.sum().backward()
        abi[f"power{power}"] = {name: args for name, args in stub.calls}
        abi[f"power{power}"]["outputs"] = [_describe(t) for t in (im, radii, depth)]
    stub.calls.clear()
    ref.GaussianRasterizer(st).markVisible(m3.detach())
    abi["mark_visible"] = stub.calls[0][1]
    for msg_case, kw in (("no_colors", dict(scales=sc, rotations=ro)),
                         ("no_geometry", dict(colors_precomp=col))):
        try:
            ref.GaussianRasterizer(st)(means3D=m3, means2D=m2, opacities=op, **kw)
        except Exception as exc:  # noqa: BLE001 - the reference raises bare Exception
            abi[f"error_{msg_case}"] = {"type": type(exc).__name__, "message": str(exc)}
    json.dump(abi, open(os.path.join(OUT, "abi_signature.json"), "w"), indent=1)
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith((".npz", ".json"))))


if __name__ == "__main__":
    main()
