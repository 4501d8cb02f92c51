"""Byte layout of the opaque state buffers (mirror of GeomLayout / ImgLayout /
BinLayout in csrc/gsr_common.h), for diagnostics and tests only."""


def _al(x, a=256):
    return (x + a - 1) // a * a


def image_layout(W: int, H: int) -> dict:
    N = W * H
    T = ((W + 15) // 16) * ((H + 15) // 16)
    o = 0
    out = {}
    out["final_T"] = o; o = _al(o + 4 * max(N, 1))
    out["n_contrib"] = o; o = _al(o + 4 * max(N, 1))
    out["ranges"] = o; o = _al(o + 8 * max(T, 1))
    out["order"] = o; o = _al(o + 4 * max(T, 1))
    out["tile_count"] = o; o = _al(o + 8 * 64 * max(T, 1))
    out["rowmax"] = o; o = _al(o + 64 * max(T, 1))
    out["total"] = o
    return out


def views(img_buffer, bin_buffer, W, H, num_rendered):
    """Typed views (torch) of final_T, n_contrib, ranges and point_list."""
    import torch
    L = image_layout(W, H)
    N = W * H
    T = ((W + 15) // 16) * ((H + 15) // 16)
    final_T = img_buffer[L["final_T"]:L["final_T"] + 4 * N].view(torch.float32)
    n_contrib = img_buffer[L["n_contrib"]:L["n_contrib"] + 4 * N].view(torch.int32)
    ranges = img_buffer[L["ranges"]:L["ranges"] + 8 * T].view(torch.int32).reshape(T, 2)
    order = img_buffer[L["order"]:L["order"] + 4 * T].view(torch.int32)
    # (an older library's image buffer has no rowmax region: A/B baselines through GSR_LIB)
    rowmax = (img_buffer[L["rowmax"]:L["rowmax"] + 64 * T].view(torch.int32).reshape(T, 16)
              if img_buffer.numel() >= L["rowmax"] + 64 * T else None)
    # BinLayout.point_list is at offset 0: u64 entries (mask << 32 | Gaussian id), little-endian
    point_list = bin_buffer[:8 * num_rendered].view(torch.int32)[0::2]
    block_masks = bin_buffer[:8 * num_rendered].view(torch.int32)[1::2]
    return dict(final_T=final_T, n_contrib=n_contrib, ranges=ranges, point_list=point_list, block_masks=block_masks,
                order=order, rowmax=rowmax)
