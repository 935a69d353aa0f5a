"""GPU: bit-exact matching arithmetic and handle hygiene.

* eosv_match (protonet) on the SAME features as the reference's classifier.py gives the SAME f32
  distances bit for bit (scipy's sequential f64 sum, no fused multiply-add) and the same
  predictions, over thousands of random episodes (1- to 5-shot, 5- and 14-way, D 512 / 2048).
* eosv_segment_match_episodes at config 3's full size (40 support segments x 5120 gallery
  segments x 2048) gives the reference's smoothed distances (cdist f64 -> f32 -> TemporalLayer)
  bit for bit and its argsort(...)[:, 0] pool ids.
* the fc head for num_classes that are not multiples of 4 (5, 50: the reference's own
  models.py example) against torch fp32 Linear.
* reloading weights keeps device memory constant and the outputs identical.
"""
import numpy as np
import pytest
import torch
from scipy.spatial.distance import cdist

from eosv import arch, engine, synth
from oracle import harness_ref

pytestmark = pytest.mark.gpu


def _episodes(rng, E, n_way, k, D):
    sup, ys, q = [], [], []
    for _ in range(E):
        y = np.repeat(rng.permutation(n_way), k).astype(np.float32)  # labels in a shuffled first-appearance order
        sup.append(rng.standard_normal((n_way * k, D), dtype=np.float32) * 0.05 + rng.random(D, dtype=np.float32))
        ys.append(y)
        q.append(rng.random(D, dtype=np.float32))
    return sup, ys, q


@pytest.mark.parametrize("n_way,k,D,E", [(5, 1, 512, 1000), (5, 5, 2048, 300), (14, 1, 2048, 300), (5, 3, 512, 400)])
def test_protonet_distances_bit_exact(n_way, k, D, E):
    rng = np.random.default_rng(n_way * 100 + k * 10 + D)
    sup, ys, q = _episodes(rng, E, n_way, k, D)
    off, slots, nproto = [0], [], []
    for y in ys:
        seen = {}
        slots += [seen.setdefault(float(v), len(seen)) for v in y]
        off.append(off[-1] + len(y))
        nproto.append(len(seen))
    t = lambda a: torch.from_numpy(np.array(a, np.int32)).cuda()  # noqa: E731
    pred, score = engine.match(torch.from_numpy(np.stack(q)).cuda(), torch.from_numpy(np.concatenate(sup)).cuda(),
                               t(off), t(slots), t(nproto), "protonet")
    pred, score = pred.cpu().numpy(), score.cpu().numpy()
    bad = 0
    for e in range(E):
        rp, rd = harness_ref.protonet_predict(sup[e], ys[e], q[e][None], np.array([0.0]))
        assert np.array_equal(score[e, :n_way].view(np.uint32), rd[0].view(np.uint32)), e
        bad += int(pred[e] != rp[0])
    assert bad == 0


@pytest.mark.parametrize("E,S,G,D", [(2, 40, 5120, 2048), (3, 40, 700, 256), (1, 130, 300, 64)])
def test_segment_match_bit_exact(E, S, G, D):
    """(2, 40, 5120, 2048) is config 3's shape; S = 130 crosses the kernel's 64-row tiles."""
    rng = np.random.default_rng(S + G)
    seg = rng.random((E * S, D), dtype=np.float32)
    gal = rng.random((G, D), dtype=np.float32)
    ids, dist = engine.segment_match_episodes(torch.from_numpy(seg).cuda(), E, torch.from_numpy(gal).cuda(), 0.1, 1.0,
                                              with_dist=True)
    ids, dist = ids.cpu().numpy(), dist.cpu().numpy()
    for e in range(E):
        ref = harness_ref.temporal_smooth(cdist(seg[e * S:(e + 1) * S], gal, "euclidean"))
        assert np.array_equal(dist[e * S:(e + 1) * S].view(np.uint32), ref.view(np.uint32)), e
        assert np.array_equal(ids[e * S:(e + 1) * S], np.argsort(ref, axis=1)[:, 0])


@pytest.mark.parametrize("l1,l2", [(0.1, -1.0), (-0.6, 1.0)])
def test_segment_match_negative_lambdas(l1, l2):
    """utils.lamda1 / lamda2 are read at call time, so a user may set them negative: smoothed
    distances then go negative (all, or some of them) and the argmin must still be argsort's."""
    rng = np.random.default_rng(int(l1 * 10) + 50)
    S, G, D = 40, 700, 64
    seg = rng.random((S, D), dtype=np.float32)
    gal = rng.random((G, D), dtype=np.float32)
    ids, dist = engine.segment_match_episodes(torch.from_numpy(seg).cuda(), 1, torch.from_numpy(gal).cuda(), l1, l2,
                                              with_dist=True)
    ref = harness_ref.temporal_smooth(cdist(seg, gal, "euclidean"), l1, l2)
    assert (ref < 0).any()
    assert np.array_equal(dist.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(ids.cpu().numpy(), np.argsort(ref, axis=1)[:, 0])


def test_segment_match_ties_pick_first_column():
    """Identical gallery rows: equal smoothed values, the first column wins (argsort[:, 0])."""
    rng = np.random.default_rng(9)
    gal = np.repeat(rng.random((1, 128), dtype=np.float32), 300, axis=0)
    seg = rng.random((10, 128), dtype=np.float32)
    ids, _ = engine.segment_match_episodes(torch.from_numpy(seg).cuda(), 1, torch.from_numpy(gal).cuda(), 0.1, 1.0)
    assert (ids.cpu().numpy() == 0).all()


@pytest.mark.parametrize("num_classes", [5, 50, 64, 101])
def test_fc_head_any_num_classes(num_classes):
    sd = synth.synth_state_dict(arch.SPECS["resnet18"], num_classes, 0)
    bb = engine.Backbone("resnet18", "f32", 112, 112, max_frames=8, num_classes=num_classes)
    bb.load_state_dict(sd)
    feat = torch.rand(37, 512, generator=torch.Generator().manual_seed(num_classes))
    got = bb.fc(feat.cuda()).cpu()
    bb.close()
    ref = feat @ torch.from_numpy(sd["fc.weight"]).T + torch.from_numpy(sd["fc.bias"])
    assert got.shape == ref.shape
    assert (got - ref).abs().max() <= 1e-5 * ref.abs().max()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f32x3"])
def test_weight_reload_keeps_device_memory(dtype):
    sd = synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0)
    sd2 = synth.synth_state_dict(arch.SPECS["resnet18"], 64, 1)
    bb = engine.Backbone("resnet18", dtype, 112, 112, max_frames=8)
    x = torch.randn(4, 3, 112, 112, generator=torch.Generator().manual_seed(0)).cuda()
    bb.load_state_dict(sd)
    b0 = bb.device_bytes
    a = bb.forward(x).clone()
    for i in range(10):
        bb.load_state_dict(sd2 if i % 2 == 0 else sd)
    assert bb.device_bytes == b0
    assert torch.equal(bb.forward(x), a)  # the last reload was sd again
    bb.load_state_dict(sd2)
    assert not torch.equal(bb.forward(x), a)
    bb.close()
