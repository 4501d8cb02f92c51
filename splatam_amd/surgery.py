"""Gaussian-set surgery on the parameters and the optimizer state.

Restates utils/slam_external.py:100-243 (accumulate_mean2d_gradient, update_params_and_optimizer,
cat_params_to_optimizer, remove_points, prune_gaussians, densify) operating on any
optimizer that keeps torch.optim.Adam's state layout -- torch.optim.Adam itself
or splatam_amd.glue.FusedAdam, whose state uses the same keys ("step",
"exp_avg", "exp_avg_sq"), so these functions (and the reference's own) work on
it unchanged.  Plain torch (boolean-mask gathers); P changes here, so this runs
between HIP-graph replays, never inside one.
"""
from __future__ import annotations

import torch

CAM_KEYS = ("cam_unnorm_rots", "cam_trans")


def _group(optimizer, name):
    return [g for g in optimizer.param_groups if g.get("name") == name][0]


def update_params_and_optimizer(new_params, params, optimizer):
    """slam_external.py:107-119: replace tensors, reset their Adam moments."""
    for k, v in new_params.items():
        group = _group(optimizer, k)
        stored = optimizer.state.get(group["params"][0], None)
        stored["exp_avg"] = torch.zeros_like(v)
        stored["exp_avg_sq"] = torch.zeros_like(v)
        del optimizer.state[group["params"][0]]
        group["params"][0] = torch.nn.Parameter(v.requires_grad_(True))
        optimizer.state[group["params"][0]] = stored
        params[k] = group["params"][0]
    return params


def cat_params_to_optimizer(new_params, params, optimizer):
    """slam_external.py:122-138: append Gaussians, zero moments for the new rows."""
    for k, v in new_params.items():
        group = _group(optimizer, k)
        stored = optimizer.state.get(group["params"][0], None)
        joined = torch.nn.Parameter(torch.cat((group["params"][0], v), dim=0).requires_grad_(True))
        if stored is not None:
            stored["exp_avg"] = torch.cat((stored["exp_avg"], torch.zeros_like(v)), dim=0)
            stored["exp_avg_sq"] = torch.cat((stored["exp_avg_sq"], torch.zeros_like(v)), dim=0)
            del optimizer.state[group["params"][0]]
            optimizer.state[joined] = stored
        group["params"][0] = joined
        params[k] = joined
    return params


def remove_points(to_remove, params, variables, optimizer):
    """slam_external.py:141-163: drop Gaussians from every per-Gaussian tensor and its moments."""
    to_keep = ~to_remove
    for k in [k for k in params.keys() if k not in CAM_KEYS]:
        group = _group(optimizer, k)
        stored = optimizer.state.get(group["params"][0], None)
        kept = torch.nn.Parameter(group["params"][0][to_keep].requires_grad_(True))
        if stored is not None:
            stored["exp_avg"] = stored["exp_avg"][to_keep]
            stored["exp_avg_sq"] = stored["exp_avg_sq"][to_keep]
            del optimizer.state[group["params"][0]]
            optimizer.state[kept] = stored
        group["params"][0] = kept
        params[k] = kept
    for k in ("means2D_gradient_accum", "denom", "max_2D_radius", "timestep"):
        if k in variables:
            variables[k] = variables[k][to_keep]
    return params, variables


def inverse_sigmoid(x):
    return torch.log(x / (1 - x))


def prune_gaussians(params, variables, optimizer, iter, prune_dict):
    """slam_external.py:170-192 (opacity / size pruning and optional opacity reset)."""
    if iter <= prune_dict["stop_after"]:
        if iter >= prune_dict["start_after"] and iter % prune_dict["prune_every"] == 0:
            thr = (prune_dict["final_removal_opacity_threshold"] if iter == prune_dict["stop_after"]
                   else prune_dict["removal_opacity_threshold"])
            to_remove = (torch.sigmoid(params["logit_opacities"]) < thr).squeeze()
            if iter >= prune_dict["remove_big_after"]:
                big = torch.exp(params["log_scales"]).max(dim=1).values > 0.1 * variables["scene_radius"]
                to_remove = torch.logical_or(to_remove, big)
            params, variables = remove_points(to_remove, params, variables, optimizer)
        if iter > 0 and iter % prune_dict["reset_opacities_every"] == 0 and prune_dict["reset_opacities"]:
            new = {"logit_opacities": inverse_sigmoid(torch.ones_like(params["logit_opacities"]) * 0.01)}
            params = update_params_and_optimizer(new, params, optimizer)
    return params, variables


def accumulate_mean2d_gradient(variables):
    """slam_external.py:100-104: the densification statistic from the RGB render's own means2D.grad."""
    seen = variables["seen"]
    variables["means2D_gradient_accum"][seen] += torch.norm(variables["means2D"].grad[seen, :2], dim=-1)
    variables["denom"][seen] += 1
    return variables


def densify(params, variables, optimizer, iter, densify_dict):
    """slam_external.py:191-243 (Gaussian-Splatting-style clone / split / prune).  The split samples come
    from torch.normal on the current CUDA generator, like the reference's."""
    from .slam import build_rotation
    if iter <= densify_dict["stop_after"]:
        variables = accumulate_mean2d_gradient(variables)
        grad_thresh = densify_dict["grad_thresh"]
        if iter >= densify_dict["start_after"] and iter % densify_dict["densify_every"] == 0:
            grads = variables["means2D_gradient_accum"] / variables["denom"]
            grads[grads.isnan()] = 0.0
            to_clone = torch.logical_and(grads >= grad_thresh, torch.max(torch.exp(params["log_scales"]), dim=1).values
                                         <= 0.01 * variables["scene_radius"])
            new_params = {k: v[to_clone] for k, v in params.items() if k not in CAM_KEYS}
            params = cat_params_to_optimizer(new_params, params, optimizer)
            num_pts = params["means3D"].shape[0]
            padded_grad = torch.zeros(num_pts, device=grads.device)
            padded_grad[:grads.shape[0]] = grads
            to_split = torch.logical_and(padded_grad >= grad_thresh,
                                         torch.max(torch.exp(params["log_scales"]), dim=1).values
                                         > 0.01 * variables["scene_radius"])
            n = densify_dict["num_to_split_into"]
            new_params = {k: v[to_split].repeat(n, 1) for k, v in params.items() if k not in CAM_KEYS}
            stds = torch.exp(params["log_scales"])[to_split].repeat(n, 3)
            means = torch.zeros((stds.size(0), 3), device=stds.device)
            samples = torch.normal(mean=means, std=stds)
            rots = build_rotation(params["unnorm_rotations"][to_split]).repeat(n, 1, 1)
            new_params["means3D"] += torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1)
            new_params["log_scales"] = torch.log(torch.exp(new_params["log_scales"]) / (0.8 * n))
            params = cat_params_to_optimizer(new_params, params, optimizer)
            num_pts = params["means3D"].shape[0]
            variables["means2D_gradient_accum"] = torch.zeros(num_pts, device=grads.device)
            variables["denom"] = torch.zeros(num_pts, device=grads.device)
            variables["max_2D_radius"] = torch.zeros(num_pts, device=grads.device)
            to_remove = torch.cat((to_split, torch.zeros(n * int(to_split.sum()), dtype=torch.bool,
                                                         device=grads.device)))
            params, variables = remove_points(to_remove, params, variables, optimizer)
            thr = (densify_dict["final_removal_opacity_threshold"] if iter == densify_dict["stop_after"]
                   else densify_dict["removal_opacity_threshold"])
            to_remove = (torch.sigmoid(params["logit_opacities"]) < thr).squeeze()
            if iter >= densify_dict["remove_big_after"]:
                big = torch.exp(params["log_scales"]).max(dim=1).values > 0.1 * variables["scene_radius"]
                to_remove = torch.logical_or(to_remove, big)
            params, variables = remove_points(to_remove, params, variables, optimizer)
        if iter > 0 and iter % densify_dict["reset_opacities_every"] == 0 and densify_dict["reset_opacities"]:
            new = {"logit_opacities": inverse_sigmoid(torch.ones_like(params["logit_opacities"]) * 0.01)}
            params = update_params_and_optimizer(new, params, optimizer)
    return params, variables
