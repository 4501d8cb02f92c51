"""CPU experiment: how the render kernels' alpha arithmetic moves the per-element gradient statistics.

The float32 oracle is rebuilt with GSR_ORACLE_ALPHA_FORM=N (oracle/gsr_oracle.c alpha_power: the GPU's
render-record conic prescaled by -log2(e)/2, -log2(e), power in that variant's FMA order, exp2f) and run
on a BASELINE config next to the reference-order float32 oracle; both are scored against the float64
oracle with harness.grad_accuracy on the same stable set, as tests/test_gpu_configs.py does.

    python tools/alpha_forms.py --config 4 --forms 1,3,5
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import harness, oracle  # noqa: E402
from splatam_amd.scenes import config_scene  # noqa: E402


def build_form(form: int) -> str:
    out = os.path.join(ROOT, "oracle", "_build", f"libgsr_oracle_f32_alpha{form}.so")
    src = os.path.join(ROOT, "oracle", "gsr_oracle.c")
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-fopenmp", "-ffp-contract=off", "-fno-fast-math",
                    "-DREAL=float", f"-DGSR_ORACLE_ALPHA_FORM={form}", "-o", out, src, "-lm"], check=True)
    return out


def run_f32(scene, dpix, use_sh, lib=None):
    oracle._libs.pop("float32", None)
    if lib:
        os.environ["GSR_ORACLE_F32_LIB"] = lib
    else:
        os.environ.pop("GSR_ORACLE_F32_LIB", None)
    try:
        return harness.run_oracle(scene, dpix, use_sh=use_sh)
    finally:
        os.environ.pop("GSR_ORACLE_F32_LIB", None)
        oracle._libs.pop("float32", None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="4")
    ap.add_argument("--forms", default="1,3,5")
    a = ap.parse_args()
    cfg = int(a.config)
    scene = config_scene(cfg)
    c = scene.cam
    use_sh = scene.shs is not None
    dpix = np.random.RandomState(11).randn(3, c.H, c.W).astype(np.float32)
    fr64, ref64 = harness.run_oracle(scene, dpix, use_sh=use_sh, dtype=np.float64, error_scale=True)
    fr, ref = run_f32(scene, dpix, use_sh)
    stable = ~(fr.unstable | fr64.unstable)
    base = harness.grad_accuracy({k: v for k, v in ref.items() if k in harness.GRAD_KEYS and
                                  isinstance(v, np.ndarray)}, ref64, stable)
    keys = [k for k in base]
    print(f"config {cfg}: stable {int(stable.sum())} of {stable.size}")
    for k in keys:
        print(f"  reference order  {k:9s} rel_l2 {base[k]['rel_l2']:.3e} q9999 {base[k]['q9999']:.3e} "
              f"max {base[k]['max']:.4f} n>1e-3 {base[k]['n_over_1e3']}")
    def worst(grads, k):  # the element with the largest r (as harness.grad_accuracy forms it)
        x = np.asarray(grads[k], np.float64).reshape(stable.size, -1)
        b = np.asarray(ref64[k], np.float64).reshape(stable.size, -1)
        sc = np.asarray(ref64["scale"][k], np.float64).reshape(stable.size, -1)
        r = np.abs(x - b) / (1e-4 * np.abs(b) + sc + 1e-30)
        r[~stable] = 0
        i = np.unravel_index(np.argmax(r), r.shape)
        return i, r[i], b[i], sc[i]
    for k in keys:
        if k != "drot":
            print(f"  reference order worst {k}: element {worst(ref, k)}")
    for f in [int(x) for x in a.forms.split(",") if x]:
        lib = build_form(f)
        frv, refv = run_f32(scene, dpix, use_sh, lib)
        for k in keys:
            if k != "drot":
                print(f"  form {f} worst {k}: element {worst(refv, k)}")
        st = harness.grad_accuracy({k: refv[k] for k in keys}, ref64, stable)
        vs = harness.compare_grads({k: refv[k] for k in keys}, ref)
        same_nc = float((frv.n_contrib == fr.n_contrib).mean())
        print(f"form {f}: n_contrib equal to the reference order at {same_nc:.6f} of pixels")
        for k in keys:
            print(f"  form {f}  {k:9s} rel_l2 {st[k]['rel_l2']:.3e} q9999 {st[k]['q9999']:.3e} "
                  f"max {st[k]['max']:.4f} ({st[k]['max'] / max(base[k]['max'], 1e-30):.2f}x) "
                  f"n>1e-3 {st[k]['n_over_1e3']}  rel L2 vs ref-order f32 {vs[k]:.2e}")


if __name__ == "__main__":
    main()
