"""SplaTAM parameter checkpoints (on-disk params*.npz interop).

Same files as utils/common_utils.py:25-52 (params2cpu, save_params ->
params.npz, save_params_ckpt -> params{t}.npz; the final file carries the extra
camera keys of scripts/splatam.py:993-1003), read back like
scripts/splatam.py:629-630 -- but with np.load(allow_pickle=False): every value
SplaTAM writes is a plain numeric array, so nothing needs unpickling.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def params2cpu(params: dict) -> dict:
    """common_utils.py:25-32."""
    return {k: (v.detach().cpu().contiguous().numpy() if isinstance(v, torch.Tensor) else v)
            for k, v in params.items()}


def save_params(params: dict, output_dir: str) -> str:
    """common_utils.py:35-42 -> output_dir/params.npz."""
    os.makedirs(output_dir, exist_ok=True)
    path = os.path.join(output_dir, "params.npz")
    np.savez(path, **params2cpu(params))
    return path


def save_params_ckpt(params: dict, output_dir: str, time_idx: int) -> str:
    """common_utils.py:45-52 -> output_dir/params{time_idx}.npz."""
    os.makedirs(output_dir, exist_ok=True)
    path = os.path.join(output_dir, f"params{time_idx}.npz")
    np.savez(path, **params2cpu(params))
    return path


def load_params(path: str, device="cuda", requires_grad: bool = True) -> dict:
    """splatam.py:629-630: every key -> float32 tensor on `device` (requiring grad, as the
    reference's checkpoint loader leaves them); allow_pickle=False."""
    with np.load(path, allow_pickle=False) as z:
        out = {}
        for k in z.files:
            t = torch.tensor(z[k]).to(device).float()
            out[k] = t.requires_grad_(True) if requires_grad else t
        return out
