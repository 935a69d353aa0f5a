"""Accuracy of the training entry's split-K convs (eosv_conv2d_f32 with a workspace) against a
torch f64 conv on the host, per R50 layer-2..4 shape at 96 frames; run once per library
(EOSV_LIBRARY) to compare split-K sizings.  Prints one line per shape: slices, relative error
(norm and max) of the split and unsplit results."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
from eosv._lib import check, lib, stream_ptr  # noqa: E402

SHAPES = [(96, 28, 28, 128, 128, 3), (96, 14, 14, 256, 256, 3), (96, 7, 7, 512, 512, 3), (96, 14, 14, 1024, 256, 1),
          (96, 7, 7, 2048, 512, 1)]


def main():
    L = lib()
    torch.set_num_threads(16)
    for (N, H, W, cin, cout, k) in SHAPES:
        pad = k // 2
        g = torch.Generator().manual_seed(cin + cout)
        x = torch.randn(N, H, W, cin, generator=g, dtype=torch.float64)
        w = torch.randn(cout, k, k, cin, generator=g, dtype=torch.float64) * (1.0 / (k * k * cin)) ** 0.5
        ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=pad).permute(0, 2, 3, 1)
        xd, wd = x.float().cuda().contiguous(), w.float().cuda().contiguous()
        out = {}
        for tag, use_ws in (("split", True), ("whole", False)):
            y = torch.empty(N * H * W * cout, device="cuda")
            kb = int(L.eosv_conv2d_f32_workspace(N, H, W, cin, cout, k, k, 1, pad)) if use_ws else 0
            kws = torch.empty(max(kb, 16) // 4 + 4, device="cuda")
            check(L.eosv_conv2d_f32(xd.data_ptr(), N, H, W, cin, wd.data_ptr(), cout, k, k, 1, pad, None, None, 0,
                                    y.data_ptr(), kws.data_ptr() if use_ws else None, kb, stream_ptr()), "conv")
            torch.cuda.synchronize()
            d = y.double().cpu().view_as(ref) - ref
            out[tag] = (float(d.norm() / ref.norm()), float(d.abs().max() / ref.abs().max()), kb)
        sl = out["split"][2] // (N * H * W * cout * 4) if out["split"][2] else 1
        print(f"{(N, H, W, cin, cout, k)} slices {sl}: split rel {out['split'][0]:.3e} max {out['split'][1]:.3e} | "
              f"whole rel {out['whole'][0]:.3e} max {out['whole'][1]:.3e}", flush=True)


if __name__ == "__main__":
    main()
