"""Synthetic SplaTAM-style scenes and cameras for tests and benchmarks.

Follows SURVEY.md section 8(d): Gaussians are generated on the CPU with a seeded
``torch.Generator`` (so CPU and GPU see identical bits), already in the camera
frame (view = identity), with SplaTAM's projective scale initialisation
(scripts/splatam.py:103-106,131-132) and the camera of
utils/recon_helpers.py:4-27 (setup_camera).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

# Replica room0 intrinsics (configs/data/replica.yaml:3-8) at 1200x680 and the
# datautils.py:113-116 rescaling to smaller frames.
REPLICA_NATIVE = dict(W=1200, H=680, fx=600.0, fy=600.0, cx=599.5, cy=339.5)


def replica_intrinsics(W: int, H: int):
    """Scale Replica intrinsics to (W, H) like datasets/gradslam_datasets/datautils.py:73-117."""
    sx = W / REPLICA_NATIVE["W"]
    sy = H / REPLICA_NATIVE["H"]
    return (REPLICA_NATIVE["fx"] * sx, REPLICA_NATIVE["fy"] * sy,
            REPLICA_NATIVE["cx"] * sx, REPLICA_NATIVE["cy"] * sy)


@dataclass
class Camera:
    """Host-side copy of what setup_camera builds (recon_helpers.py:4-27)."""
    W: int
    H: int
    fx: float
    fy: float
    cx: float
    cy: float
    w2c: torch.Tensor        # [4,4] float32
    viewmatrix: torch.Tensor  # [1,4,4] = w2c^T
    projmatrix: torch.Tensor  # [1,4,4] = w2c^T @ opengl_proj^T
    campos: torch.Tensor      # [3]
    tanfovx: float
    tanfovy: float


def setup_camera(W, H, fx, fy, cx, cy, w2c=None, near=0.01, far=100.0) -> Camera:
    """Restates utils/recon_helpers.py:4-27 on the CPU (float32, like the reference)."""
    if w2c is None:
        w2c = torch.eye(4)
    w2c = torch.as_tensor(w2c, dtype=torch.float32).clone()
    cam_center = torch.inverse(w2c)[:3, 3]
    view = w2c.unsqueeze(0).transpose(1, 2)
    opengl_proj = torch.tensor([[2 * fx / W, 0.0, -(W - 2 * cx) / W, 0.0],
                                [0.0, 2 * fy / H, -(H - 2 * cy) / H, 0.0],
                                [0.0, 0.0, far / (far - near), -(far * near) / (far - near)],
                                [0.0, 0.0, 1.0, 0.0]]).float().unsqueeze(0).transpose(1, 2)
    full_proj = view.bmm(opengl_proj)
    return Camera(W=W, H=H, fx=fx, fy=fy, cx=cx, cy=cy, w2c=w2c, viewmatrix=view,
                  projmatrix=full_proj, campos=cam_center, tanfovx=W / (2 * fx), tanfovy=H / (2 * fy))


@dataclass
class Scene:
    """Rasterizer inputs (float32, CPU) of one synthetic scene."""
    means3D: torch.Tensor      # [P,3]
    scales: torch.Tensor       # [P,3]
    rotations: torch.Tensor    # [P,4] normalised (w,x,y,z)
    opacities: torch.Tensor    # [P,1]
    colors: torch.Tensor       # [P,3]
    shs: torch.Tensor | None   # [P,16,3] when sh_degree == 3
    sh_degree: int
    cam: Camera

    @property
    def P(self) -> int:
        return self.means3D.shape[0]

    def to(self, device):
        kw = {k: (getattr(self, k).to(device) if isinstance(getattr(self, k), torch.Tensor) else getattr(self, k))
              for k in ("means3D", "scales", "rotations", "opacities", "colors", "shs", "sh_degree")}
        return Scene(cam=self.cam, **kw)


def make_scene(P: int, W: int, H: int, *, seed: int = 0, anisotropic: bool = False, sh_degree: int = 0,
               intrinsics=None, z_range=(0.5, 5.0)) -> Scene:
    """SURVEY.md 8(d) synthetic distribution."""
    g = torch.Generator().manual_seed(seed)
    fx, fy, cx, cy = intrinsics if intrinsics is not None else replica_intrinsics(W, H)
    u = torch.rand(P, generator=g) * W
    v = torch.rand(P, generator=g) * H
    z = z_range[0] + torch.rand(P, generator=g) * (z_range[1] - z_range[0])
    means3D = torch.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], dim=1)
    log_scales = torch.log(z / ((fx + fy) / 2)).unsqueeze(1).repeat(1, 3)
    if anisotropic:
        log_scales = log_scales + 0.5 * torch.randn(P, 3, generator=g)
        rot = torch.randn(P, 4, generator=g)
        rot = rot / rot.norm(dim=1, keepdim=True)
    else:
        rot = torch.zeros(P, 4)
        rot[:, 0] = 1.0
    opac = torch.sigmoid(torch.randn(P, 1, generator=g))
    rgb = torch.rand(P, 3, generator=g)
    shs = None
    if sh_degree > 0:
        M = (sh_degree + 1) ** 2
        shs = 0.1 * torch.randn(P, M, 3, generator=g)
        shs[:, 0] = (rgb - 0.5) / 0.28209479177387814
    cam = setup_camera(W, H, fx, fy, cx, cy)
    return Scene(means3D=means3D.float(), scales=torch.exp(log_scales).float(), rotations=rot.float(),
                 opacities=opac.float(), colors=rgb.float(), shs=shs, sh_degree=sh_degree, cam=cam)


# BASELINE.json configs; config 3 is the headline bench workload.
CONFIGS = {
    1: dict(P=10_000, W=320, H=240, anisotropic=False, sh_degree=0),
    2: dict(P=100_000, W=640, H=480, anisotropic=False, sh_degree=0),
    3: dict(P=300_000, W=640, H=480, anisotropic=False, sh_degree=0),
    4: dict(P=1_000_000, W=1200, H=680, anisotropic=True, sh_degree=3,
            intrinsics=(600.0, 600.0, 599.5, 339.5)),
}


def config_scene(cfg: int, seed: int = 0) -> Scene:
    c = dict(CONFIGS[cfg])
    return make_scene(seed=seed, **c)
