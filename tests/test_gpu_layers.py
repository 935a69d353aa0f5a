"""GPU: one-frame per-layer checksums (SURVEY 8(c) golden vector 5) against the reference's own
model wrapper (models.py:9-37, self.convnet = torchvision's children minus fc), captured by
tests/golden/capture_golden.py --layers: the map after the stem + maxpool (convnet.0-3) and
after each of layer1..layer4 (convnet.4-7), read from the library with eosv_backbone_probe.

Checksums are layout-free (sum, sum of squares, max |.|) plus a projection onto a fixed N(0,1)
tensor in the reference's NCHW order (the probe's NHWC map is transposed first).  Bounds: the
north star's 1e-4 relative for f32 and f32x3 (the projection through Cauchy-Schwarz,
|d proj| <= ||d a|| ||r||, with ||d a|| <= 1e-4 ||a||), 1e-2 for bf16.
"""
import numpy as np
import pytest
import torch

from _common import load_fixture
from eosv import arch, engine, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
@pytest.mark.parametrize("dtype", ["f32", "f32x3", "bf16"])
def test_per_layer_checksums_match_reference(name, dtype):
    meta, _ = load_fixture("layers_one_frame")
    vi, fid, H, W = meta["video_info"], meta["frame_id"], meta["H"], meta["W"]
    frame = torch.from_numpy(synth.synth_frame(vi.split("/")[0], vi, fid, H, W))[None].cuda()
    bb = engine.Backbone(name, dtype, H, W, max_frames=4, device=0)
    bb.load_state_dict(synth.synth_state_dict(arch.SPECS[name], 64, 0))
    tol = 1e-2 if dtype == "bf16" else 1e-4
    try:
        for stage, ref in enumerate(meta["archs"][name]):
            a = bb.probe(frame, stage)[0].permute(2, 0, 1).double().cpu().numpy()  # NHWC -> CHW
            assert list(a.shape) == ref["shape"], (stage, a.shape)
            r = np.random.default_rng(1000 + stage).standard_normal(a.shape)
            got = dict(sum=a.sum(), sumsq=(a * a).sum(), absmax=np.abs(a).max(), proj=(a * r).sum())
            norm = np.sqrt(ref["sumsq"])
            bounds = dict(sum=tol * np.abs(a).sum(), sumsq=2 * tol * ref["sumsq"], absmax=tol * ref["absmax"],
                          proj=tol * norm * np.sqrt(a.size))
            errs = {k: abs(got[k] - ref[k]) for k in got}
            print(f"[{name} {dtype} stage {stage}] " + " ".join(f"{k} {errs[k] / max(bounds[k], 1e-30):.2e}" for k in errs))
            for k in got:
                assert errs[k] <= bounds[k], (stage, k, got[k], ref[k])
    finally:
        bb.close()


def test_probe_rejects_bad_arguments():
    bb = engine.Backbone("resnet18", "f32", 112, 112, max_frames=2, device=0)
    bb.load_state_dict(synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0))
    x = torch.zeros(3, 3, 112, 112, device="cuda")
    try:
        with pytest.raises(Exception):
            bb.probe(x, 1)  # B > max_frames
        with pytest.raises(ValueError):
            bb.probe(x[:1], 5)
        assert tuple(bb.probe(x[:2], 4).shape) == (2, 4, 4, 512)
    finally:
        bb.close()
