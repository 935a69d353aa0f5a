"""GPU: the drop-in modules (models / network_test / classifier / TemporalLayer) against the
reference's own outputs (golden fixtures) and the CPU oracle."""
import os
import random

import numpy as np
import pytest
import torch

from _common import load_fixture
from eosv import arch, synth
from oracle import harness_ref, resnet_ref

pytestmark = pytest.mark.gpu


def _save_sd(name, path):
    sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, path)


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_models_dropin_forward(name):
    import models

    m = getattr(models, "model_" + name)(num_classes=64)
    m.eval()
    m.cuda()
    x = torch.randn(5, 3, 224, 224, generator=torch.Generator().manual_seed(0))
    feat, out = m(x.cuda())
    ref = resnet_ref.build_model(name, synth.synth_state_dict(arch.SPECS[name], 64, 0))
    with torch.no_grad():
        rf, ro = ref(x)
    assert feat.shape == rf.shape and out.shape == ro.shape
    for a, b in ((feat, rf), (out, ro)):
        err = (a.cpu() - b).abs().max() / b.abs().max()
        assert err < 2e-5, err
    # state_dict keys are the reference's
    assert list(m.state_dict().keys()) == list(ref.state_dict().keys())


@pytest.mark.parametrize("tag", ["c1_r18_protonet_seed1", "c1_r18_cosine_seed2", "c1_r50_protonet_seed3",
                                 "c1_r18_svm_seed5"])
def test_network_test_baseline_reproduces_reference_file(tag, tmp_path):
    import network_test
    import utils

    meta, arr = load_fixture(tag)
    pkl = str(tmp_path / "model.pkl")
    _save_sd(meta["arch"], pkl)
    acc_path = str(tmp_path / "acc.txt")
    old = utils.EPISODE_NUMS["test"]
    utils.EPISODE_NUMS["test"] = len(meta["episodes"])
    try:
        random.seed(meta["seed"])
        tn = network_test.TestNetwork(acc_path, meta["arch"], meta["classifier"], True)
        tn.episodes_per_batch = 7  # several batches, ragged last one
        tn.test_network_baseline(pre_model=pkl)
        tn.acc_file.close()
    finally:
        utils.EPISODE_NUMS["test"] = old
    assert open(acc_path).read() == meta["acc_file"]


def test_generate_epoch_features_matches_reference():
    import network_test
    import episode_novel_dataloader

    meta, arr = load_fixture("c1_r18_protonet_seed1")
    tn = network_test.TestNetwork("/tmp/eosv_unused.txt", "resnet18", "protonet", True)
    random.seed(meta["seed"])
    dl = episode_novel_dataloader.EpisodeDataloader("test")
    for e in range(2):
        d = dl.get_episode()
        sf = tn.generate_epoch_features(d["support_x"], True, d["support_x_frames"])
        qf = tn.generate_epoch_features(d["query_x"], True)
        np.testing.assert_allclose(sf, arr["support_feature"][e], rtol=0, atol=1e-4 * np.abs(arr["support_feature"][e]).max())
        np.testing.assert_allclose(qf, arr["query_feature"][e], rtol=0, atol=1e-4 * np.abs(arr["query_feature"][e]).max())
    # per-frame path (generate_epoch_features_2) == normalised features
    frames = d["support_x"][0]
    f2 = tn.generate_epoch_features_2(frames, True)
    ref = resnet_ref.build_model("resnet18", synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0))
    r2 = harness_ref.epoch_features_2(ref, frames, True)
    assert np.abs(f2 - r2).max() < 1e-4 * np.abs(r2).max()


@pytest.mark.parametrize("kind", ["protonet", "cosine"])
def test_classifier_dropin(kind):
    import classifier

    rng = np.random.default_rng(5)
    for k in (1, 3):
        sup = rng.random((5 * k, 512), dtype=np.float32)
        sy = np.repeat(np.arange(5), k).astype(np.float32)
        q = rng.random((1, 512), dtype=np.float32)
        d = {"support_feature": sup, "support_y": sy, "query_feature": q, "query_y": np.array([2.0])}
        got = classifier.Classifier(kind).predict(d)
        ref = harness_ref.predict(kind, sup, sy, q, np.array([2.0]))
        assert got.dtype == np.int64 and np.array_equal(got, ref)
    ids, feats = classifier.generate_prototypes_tensor_lowerdim(d)
    rids, rfeats = harness_ref.prototypes(sup, sy)
    assert ids == rids and np.array_equal(feats, rfeats)


def test_temporal_layer_dropin():
    import models
    import network_test

    rng = np.random.default_rng(7)
    dist = rng.random((40, 5120)) * 2
    tn = network_test.TestNetwork.__new__(network_test.TestNetwork)
    got = tn.temporal_convolution_flating_layer(dist)
    ref = harness_ref.temporal_smooth(dist)
    np.testing.assert_allclose(got, ref, rtol=1e-6)
    y = models.TemporalLayer()(torch.from_numpy(dist.T.astype(np.float32)).cuda().view(1, 1, 5120, 40))
    assert y.shape == (1, 1, 5120, 40)


def _run_c3(tmp_path, reforward, monkeypatch):
    import generate_augmented_datasets as gad
    import network_test
    import utils

    monkeypatch.setenv("EOSV_AUG_REFORWARD", reforward)
    meta, arr = load_fixture("c3_r50_aug_seed4")
    pkl = str(tmp_path / "model.pkl")
    _save_sd("resnet50", pkl)
    old = (utils.GALLERY_LIST, utils.EPISODE_NUMS["test"])
    utils.GALLERY_LIST = str(tmp_path / "gallery.list")
    utils.EPISODE_NUMS["test"] = len(meta["episodes"])
    try:
        random.seed(meta["seed"])
        np.random.seed(meta["seed"])
        gad.generate_gallery_list()
        assert gad.gallery_video_infos() == meta["gallery"]
        acc_path = str(tmp_path / f"acc{reforward}.txt")
        tn = network_test.TestNetwork(acc_path, "resnet50", "protonet", True)
        tn.debug = {}
        tn.test_network_aug_segment(pre_model=pkl)
        tn.acc_file.close()
    finally:
        utils.GALLERY_LIST, utils.EPISODE_NUMS["test"] = old
    return tn.debug, open(acc_path).read(), meta, arr


def test_aug_segment_reproduces_reference(tmp_path, monkeypatch):
    """Config-3 path (R50, aug_seg_T) against the reference's own run (2 episodes)."""
    dbg, acc_text, meta, arr = _run_c3(tmp_path, "0", monkeypatch)
    ref_pool = np.argsort(arr["smoothed"], axis=2)[:, :, 0]  # [E,40] (network_test.py:211-212)
    got_pool = dbg["pool"].cpu().numpy().reshape(len(meta["episodes"]), -1)
    assert np.array_equal(got_pool, ref_pool)
    sup = dbg["sup"].cpu().numpy().reshape(arr["aug_features"].shape)
    err = np.abs(sup - arr["aug_features"]).max() / np.abs(arr["aug_features"]).max()
    assert err < 1e-4, err
    q = dbg["q_emb"].cpu().numpy()
    assert np.abs(q - arr["query_feature"][:, 0]).max() / np.abs(arr["query_feature"]).max() < 1e-4
    assert np.array_equal(dbg["pred"].cpu().numpy(), arr["pred"][:, 0])
    assert acc_text == meta["acc_file"]


def test_aug_segment_feature_gather_equals_reforward(tmp_path, monkeypatch):
    """The augmented videos' features gathered from the gallery / support frame features are
    bit-identical to re-running the backbone on the assembled frames (the reference's way)."""
    a, acc_a, _, _ = _run_c3(tmp_path, "0", monkeypatch)
    b, acc_b, _, _ = _run_c3(tmp_path, "1", monkeypatch)
    assert torch.equal(a["sup"], b["sup"])
    assert torch.equal(a["q_emb"], b["q_emb"])
    assert torch.equal(a["pred"], b["pred"]) and acc_a == acc_b


def test_aug_segment_with_svm_classifier(tmp_path, monkeypatch):
    """aug_seg_T with classifier='SVM' (host sklearn on the GPU's augmented support set,
    network_test.py:251-255 -> classifier.py:109-111): the predictions equal SVC(C=10) fitted
    on the reference's own augmented features of the C3 fixture."""
    import generate_augmented_datasets as gad
    import network_test
    import utils

    meta, arr = load_fixture("c3_r50_aug_seed4")
    pkl = str(tmp_path / "model.pkl")
    _save_sd("resnet50", pkl)
    monkeypatch.setattr(utils, "GALLERY_LIST", str(tmp_path / "gallery.list"))
    monkeypatch.setitem(utils.EPISODE_NUMS, "test", len(meta["episodes"]))
    random.seed(meta["seed"])
    np.random.seed(meta["seed"])
    gad.generate_gallery_list()
    tn = network_test.TestNetwork(str(tmp_path / "acc.txt"), "resnet50", "SVM", True)
    tn.test_network_aug_segment(pre_model=pkl)
    tn.acc_file.close()
    for e, ep in enumerate(meta["episodes"]):
        ref = harness_ref.predict("SVM", arr["aug_features"][e], arr["aug_labels"][e], arr["query_feature"][e],
                                  np.array([ep["query_y"]], np.float32))
        assert tn.last_accs[e] == float(int(ref[0]) == ep["query_y"])
