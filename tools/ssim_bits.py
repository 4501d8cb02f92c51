"""Mapping-loss (L1 + SSIM + masked depth L1) outputs of the loaded libgsr (GSR_LIB selects a variant) on a
seeded 680x1200 frame, saved for a bitwise comparison between two builds.
Usage: python tools/ssim_bits.py OUT.pt  |  python tools/ssim_bits.py --compare A.pt B.pt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    same = {k: bool(torch.equal(a[k], b[k])) for k in a}
    print("bitwise", same)
    sys.exit(0 if all(same.values()) else 1)

from splatam_amd.glue import mapping_loss  # noqa: E402

H, W = 680, 1200
g = torch.Generator().manual_seed(7)
im = torch.rand(3, H, W, generator=g)
gt = (im + 0.2 * torch.randn(3, H, W, generator=g)).clamp(0, 1)
ds = torch.stack([0.5 + 4 * torch.rand(H, W, generator=g), torch.rand(H, W, generator=g), torch.zeros(H, W)])
ds[2] = ds[0] * ds[0] + 0.01 * torch.rand(H, W, generator=g)
gd = (ds[0:1] + 0.3 * torch.randn(1, H, W, generator=g)).clamp_min(0)
im, ds, gt, gd = (t.cuda() for t in (im, ds, gt, gd))
a_im, a_ds = im.clone().requires_grad_(True), ds.clone().requires_grad_(True)
loss = mapping_loss(a_im, a_ds, gt, gd)
loss.backward()
torch.save({"loss": loss.detach().cpu(), "dim": a_im.grad.cpu(), "dds": a_ds.grad.cpu()}, sys.argv[1])
print("saved", float(loss))
