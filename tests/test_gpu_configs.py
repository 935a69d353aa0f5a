"""GPU parity at the episode shapes of BASELINE configs 3-5, against fixtures captured from the
reference's own ``test_network_baseline`` / ``test_network_aug_segment`` (tests/golden/capture_golden.py
--shapes / --aug):

* config 4: 14-way 1-shot, 16 segments (T = 32), ResNet-50, over an UnrealAction-shaped novel split
  (14 classes x 10 videos, ``tests/golden/unreal14.list``; README.md:23-26);
* config 5: 5-way 5-shot, 32 segments (T = 64) at 256x256, ResNet-50 through the reference's
  wrapper, and ResNet-101 (the reference has no R101 wrapper: its model_resnet50 wrapped around the
  R101 structure, models.py:24-37) -- 5-shot prototype means (classifier.py:9-40);
* config 3: aug_seg_T (network_test.py:170-267) at its stated dtype bf16 and at f32x3.

Acceptance (north star): f32 predictions and the result file bit-exact, clip embeddings within 1e-4
relative.  bf16 / f32x3 rules are written at each test.
"""
import hashlib
import math
import os
import random

import numpy as np
import pytest
import torch

from _common import GOLDEN, load_fixture
from eosv import arch, synth

pytestmark = pytest.mark.gpu

SHAPED = ["c4_r50_14w1s_t32_seed7", "c5_r50_5w5s_t64_256_seed39", "c5_r101_5w5s_t64_256_seed39"]
# round-3 wide fixtures (capture_golden.py --wide): 30 config-4 episodes, 10 + 5 config-5 episodes
# (R50 / R101, sampled from tests/golden/test_long64.list: the reference cannot run a 256x256
# episode that holds a video shorter than T, utils.py:252), compact form
WIDE = ["c4_r50_14w1s_t32_seed8_wide", "c5_r50_5w5s_t64_256_seed40_wide", "c5_r101_5w5s_t64_256_seed41_wide"]
# round 4: 20 more R101 episodes (capture_golden.py --wide c5r101b)
WIDE += ["c5_r101_5w5s_t64_256_seed42_wide"]
WIDE = [t for t in WIDE if os.path.exists(os.path.join(GOLDEN, t + ".json"))]
# bf16 prediction agreement with the reference over many episodes (SURVEY section 7's rule, its
# bound set to the evidence in r04: C2 measured 0.9985 over 2000 episodes, every wide fixture 1.000)
BF16_MIN_AGREE = 0.97
# C3 bf16 pool-id agreement (argmin over 5120 smoothed distances; measured 0.887-0.931)
C3_BF16_MIN_POOL_AGREE = 0.85


def _save_sd(name, path):
    sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, path)


def _run_shaped(tag, tmp_path, monkeypatch, dtype="f32", batch=2):
    """The drop-in TestNetwork.test_network_baseline at the fixture's shape, set through the same
    utils globals a reference user edits (n_way / k_shot / VIDEO_FRAMES / TEST_LIST / crop size)."""
    import network_test
    import utils

    meta, arr = load_fixture(tag)
    monkeypatch.setattr(utils, "n_way", meta["n_way"])
    monkeypatch.setattr(utils, "k_shot", meta["k_shot"])
    monkeypatch.setattr(utils, "VIDEO_FRAMES", meta["video_frames"])
    monkeypatch.setattr(utils, "IMG_crop_size", (meta["H"], meta["W"]))
    if meta["test_list"] != "sources/data/test.list":
        monkeypatch.setattr(utils, "TEST_LIST", f"{GOLDEN}/{meta['test_list']}")
    monkeypatch.setitem(utils.EPISODE_NUMS, "test", len(meta["episodes"]))
    pkl = str(tmp_path / "model.pkl")
    _save_sd(meta["arch"], pkl)
    acc_path = str(tmp_path / f"acc_{dtype}.txt")
    random.seed(meta["seed"])
    tn = network_test.TestNetwork(acc_path, meta["arch"], meta["classifier"], True)
    tn.mymodel.compute_dtype = dtype
    tn.mymodel.max_frames = 1024
    tn.episodes_per_batch = batch
    tn.debug = {}
    tn.test_network_baseline(pre_model=pkl)
    tn.acc_file.close()
    sup = torch.cat([b["sup"] for b in tn.debug["batches"]]).cpu().numpy()
    q = torch.cat([b["q"] for b in tn.debug["batches"]]).cpu().numpy()
    return meta, arr, dict(sup=sup, q=q, preds=np.array(tn.last_preds), acc=open(acc_path).read())


def _rel(got, ref):
    """max over clips of max|got - ref| / max|ref| (the north star's 1e-4 relative bound)."""
    return float((np.abs(got - ref).max(-1) / np.abs(ref).max(-1)).max())


@pytest.mark.parametrize("tag", SHAPED)
def test_shaped_baseline_f32_reproduces_reference(tag, tmp_path, monkeypatch):
    meta, arr, got = _run_shaped(tag, tmp_path, monkeypatch)
    E = len(meta["episodes"])
    ref_sup = arr["support_feature"].reshape(E * meta["n_way"] * meta["k_shot"], -1)
    ref_q = arr["query_feature"].reshape(E, -1)
    assert got["sup"].shape == ref_sup.shape and got["q"].shape == ref_q.shape
    assert _rel(got["sup"], ref_sup) < 1e-4
    assert _rel(got["q"], ref_q) < 1e-4
    assert np.array_equal(got["preds"], arr["pred"][:, 0])
    assert got["acc"] == meta["acc_file"]


@pytest.mark.parametrize("tag,dtype", [("c4_r50_14w1s_t32_seed7", "f32x3"), ("c5_r50_5w5s_t64_256_seed39", "f32x3"),
                                       ("c4_r50_14w1s_t32_seed7", "bf16"), ("c5_r101_5w5s_t64_256_seed39", "bf16")])
def test_shaped_baseline_fast_legs(tag, dtype, tmp_path, monkeypatch):
    """f32x3: the f32 bound (1e-4) and identical predictions.  bf16 (config 5's stated dtype):
    embeddings within 1e-2 relative of the reference's f32 ones, predictions identical on these
    episodes (their top-2 distance margins are > 100x the bf16 embedding error)."""
    meta, arr, got = _run_shaped(tag, tmp_path, monkeypatch, dtype)
    E = len(meta["episodes"])
    tol = 1e-4 if dtype == "f32x3" else 1e-2
    assert _rel(got["sup"], arr["support_feature"].reshape(got["sup"].shape)) < tol
    assert _rel(got["q"], arr["query_feature"].reshape(E, -1)) < tol
    assert np.array_equal(got["preds"], arr["pred"][:, 0])


def _proj_within(got_sup, got_q, arr, E, tol):
    """|e . r - e_ref . r| <= tol * sqrt(D) * max|e| * |r| for every clip embedding (r: the fixture's
    fixed N(0,1) vector): the embedding bound `tol` (relative, max-norm) through a projection."""
    D = got_q.shape[-1]
    r = np.random.default_rng(int(arr["proj_vector_seed"])).standard_normal(D)
    got = np.concatenate([got_sup.reshape(E, -1, D), got_q.reshape(E, 1, D)], axis=1).astype(np.float64)
    bound = tol * math.sqrt(D) * np.abs(got).max(axis=2) * np.linalg.norm(r) * 1.01
    err = np.abs(got @ r - arr["proj"])
    return float((err / bound).max())


@pytest.mark.parametrize("dtype", ["f32", "f32x3", "bf16"])
@pytest.mark.parametrize("tag", WIDE)
def test_wide_fixture(tag, dtype, tmp_path, monkeypatch):
    """Configs 4 / 5 over the wide reference fixtures (network_test.py:143-164 at 14w1s T32 and
    5w5s T64 256x256).  f32 and f32x3: every prediction bit-exact, embeddings within 1e-4 (through
    the projection bound), the result file's sha256 the reference's.  bf16 (config 5's stated
    dtype; SURVEY section 7 rule, r04 bound): prediction agreement with the reference >= 0.97 and the accuracy
    within the 95 % binomial interval of the reference's, embeddings within 1e-2.  Prints the
    agreement, the near ties (top-2 margin < 1e-5) and the smallest margin."""
    meta, arr, got = _run_shaped(tag, tmp_path, monkeypatch, dtype)
    E = len(meta["episodes"])
    ref_pred = arr["pred"].reshape(E)
    agree = float((got["preds"] == ref_pred).mean())
    qy = np.array([ep["query_y"] for ep in meta["episodes"]])
    acc, ref_acc = float((got["preds"] == qy).mean()), float((ref_pred == qy).mean())
    tol = 1e-2 if dtype == "bf16" else 1e-4
    worst = _proj_within(got["sup"], got["q"], arr, E, tol)
    print(f"[{tag} {dtype}] {E} episodes, agreement {agree:.3f}, acc {acc:.3f} (reference {ref_acc:.3f}), "
          f"near ties {int((arr['margin'] < 1e-5).sum())}, min margin {arr['margin'].min():.2e}, "
          f"projection error / bound {worst:.3f}")
    assert worst <= 1.0
    if dtype == "bf16":
        half = 1.96 * math.sqrt(max(ref_acc * (1 - ref_acc), 1e-12) / E) + 1.0 / E
        assert agree >= BF16_MIN_AGREE and abs(acc - ref_acc) <= half
    else:
        assert np.array_equal(got["preds"], ref_pred)
        assert hashlib.sha256(got["acc"].encode()).hexdigest() == meta["acc_file_sha256"]


def test_five_shot_prototypes_through_native_match():
    """classifier.py:9-40 with k_shot = 5: per-label np.mean of 5 support embeddings, first-appearance
    label order, then f64 cdist / f32 softmax / argmax -- eosv_match on the config-5 fixture's own
    reference embeddings gives the reference's predictions, and on label-permuted supports too."""
    from eosv import engine
    from oracle import harness_ref

    meta, arr = load_fixture("c5_r50_5w5s_t64_256_seed39")
    rng = np.random.default_rng(3)
    sups, qs, offs, slots, nproto, refs = [], [], [0], [], [], []
    for e, ep in enumerate(meta["episodes"]):
        for perm in (np.arange(25), rng.permutation(25)):
            s = arr["support_feature"][e][perm]
            y = np.asarray(ep["support_y"], np.float32)[perm]
            seen = {}
            slots += [seen.setdefault(float(v), len(seen)) for v in y]
            nproto.append(len(seen))
            offs.append(offs[-1] + 25)
            sups.append(s)
            qs.append(arr["query_feature"][e][0])
            refs.append(harness_ref.protonet_predict(s, y, arr["query_feature"][e], np.array([ep["query_y"]], np.float32))[0][0])
    dev = torch.device("cuda", 0)
    t32 = lambda a: torch.tensor(np.asarray(a, np.int32), device=dev)  # noqa: E731
    pred, _ = engine.match(torch.tensor(np.stack(qs), device=dev), torch.tensor(np.concatenate(sups), device=dev),
                           t32(offs), t32(slots), t32(nproto), "protonet")
    assert pred.cpu().tolist() == refs
    # the unpermuted episodes are the reference's own predictions
    assert refs[0::2] == arr["pred"][:, 0].tolist()


# ---------------------------------------------------------------------------------- config 3
def _run_c3(tmp_path, monkeypatch, dtype, tag="c3_r50_aug_seed4"):
    import generate_augmented_datasets as gad
    import network_test
    import utils

    meta, arr = load_fixture(tag)
    pkl = str(tmp_path / "model.pkl")
    _save_sd("resnet50", pkl)
    monkeypatch.setattr(utils, "GALLERY_LIST", str(tmp_path / "gallery.list"))
    monkeypatch.setitem(utils.EPISODE_NUMS, "test", len(meta["episodes"]))
    random.seed(meta["seed"])
    np.random.seed(meta["seed"])
    gad.generate_gallery_list()
    assert gad.gallery_video_infos() == meta["gallery"]
    acc_path = str(tmp_path / f"acc_{dtype}.txt")
    tn = network_test.TestNetwork(acc_path, "resnet50", "protonet", True)
    tn.mymodel.compute_dtype = dtype
    tn.mymodel.max_frames = 1024
    tn.debug = {}
    tn.test_network_aug_segment(pre_model=pkl)
    tn.acc_file.close()
    return tn.debug, open(acc_path).read(), meta, arr


@pytest.mark.parametrize("dtype", ["bf16", "f32x3"])
def test_aug_segment_fast_legs(dtype, tmp_path, monkeypatch):
    """Config 3 (aug_seg_T, R50) at bf16 (its stated dtype) and f32x3 against the reference's f32 run.

    Pool ids are an argmin over 5120 temporally smoothed distances, so a lower-precision
    backbone may pick another gallery segment where two are nearly equidistant.  Rule: wherever
    the pick differs from the reference's, the reference's own smoothed distance at the pick is
    within ``delta`` (relative) of its minimum -- bf16 1e-2 (its embedding error ~3e-3), f32x3 1e-4 --
    and at least 85 % (bf16, r04: measured 0.887-0.931) / 95 % (f32x3) of the picks are identical.
    Predictions identical."""
    dbg, acc_text, meta, arr = _run_c3(tmp_path, monkeypatch, dtype)
    E = len(meta["episodes"])
    sm = arr["smoothed"]  # [E, 40, 5120] f32, the reference's temporal_convolution_flating_layer output
    ref_pool = np.argsort(sm, axis=2)[:, :, 0]
    got_pool = dbg["pool"].cpu().numpy().reshape(E, -1)
    agree = float((got_pool == ref_pool).mean())
    best = sm.min(axis=2)
    at_pick = np.take_along_axis(sm, got_pool[:, :, None], axis=2)[:, :, 0]
    slack = float(((at_pick - best) / np.abs(best)).max())
    delta, min_agree = (1e-2, C3_BF16_MIN_POOL_AGREE) if dtype == "bf16" else (1e-4, 0.95)
    print(f"[c3 {dtype}] pool-id agreement {agree:.3f}, max relative slack at differing picks {slack:.2e}")
    assert slack <= delta, slack
    assert agree >= min_agree, agree
    q = dbg["q_emb"].cpu().numpy()
    tol = 1e-2 if dtype == "bf16" else 1e-4
    assert _rel(q, arr["query_feature"][:, 0]) < tol
    assert np.array_equal(dbg["pred"].cpu().numpy(), arr["pred"][:, 0])
    assert acc_text == meta["acc_file"]


C3_COMPACT = [t for t in ("c3_r50_aug_seed6", "c3_r50_aug_seed9_wide") if os.path.exists(os.path.join(GOLDEN, t + ".json"))]


@pytest.mark.parametrize("dtype", ["f32", "f32x3", "bf16"])
@pytest.mark.parametrize("tag", C3_COMPACT)
def test_aug_segment_eight_reference_episodes(tag, dtype, tmp_path, monkeypatch):
    """Config 3 over 8 (seed 6) and 30 (seed 9, round 3) more reference episodes (320 / 1200 gallery
    matches; compact fixture: pool ids,
    each row's 16 smallest reference smoothed distances, augmented-feature projections).
    f32: pool ids identical.  f32x3 / bf16: where a pick differs it is among the reference's 16
    nearest and within delta (1e-4 / 1e-2, relative) of the row's minimum.  Augmented features
    within 1e-4 (f32, f32x3) / 1e-2 (bf16) through the projection bound; predictions and the
    result file identical."""
    dbg, acc_text, meta, arr = _run_c3(tmp_path, monkeypatch, dtype, tag=tag)
    E = len(meta["episodes"])
    ref_pool = arr["pool"].astype(np.int64)
    got_pool = dbg["pool"].cpu().numpy().reshape(E, -1)
    same = got_pool == ref_pool
    delta = 1e-4 if dtype != "bf16" else 1e-2
    best = arr["top16_val"][:, :, 0]
    worst_slack = 0.0
    for e, s_ in zip(*np.nonzero(~same)):
        hit = np.flatnonzero(arr["top16_idx"][e, s_] == got_pool[e, s_])
        assert hit.size, f"episode {e} segment {s_}: pick {got_pool[e, s_]} outside the reference's 16 nearest"
        slack = (arr["top16_val"][e, s_, hit[0]] - best[e, s_]) / abs(best[e, s_])
        worst_slack = max(worst_slack, float(slack))
    margins = arr["margin"] if "margin" in arr else None
    print(f"[c3 x{E} {dtype}] pool-id agreement {same.mean():.3f}, max relative slack {worst_slack:.2e}"
          + (f", prediction near ties {int((margins < 1e-5).sum())}, min top-2 margin {margins.min():.2e}"
             if margins is not None else ""))
    if dtype == "f32":
        assert same.all()
    elif dtype == "bf16":
        assert same.mean() >= C3_BF16_MIN_POOL_AGREE, same.mean()
    else:
        assert same.mean() >= 0.95, same.mean()
    assert worst_slack <= delta
    sup = dbg["sup"].cpu().numpy().astype(np.float64).reshape(E, 45, -1)
    D = sup.shape[-1]
    r = np.random.default_rng(20261017).standard_normal(D)
    tol = 1e-4 if dtype != "bf16" else 1e-2
    bound = tol * np.sqrt(D) * arr["aug_absmax"] * np.linalg.norm(r)
    assert (np.abs(sup @ r - arr["aug_proj"]) <= bound).all()
    pred, ref_pred = dbg["pred"].cpu().numpy(), arr["pred"][:, 0]
    if dtype == "bf16" and E > 8:
        # SURVEY section 7 rule for the lower-precision dtype over many episodes: prediction agreement
        # >= 0.9 and accuracy within the 95 % binomial interval of the reference's
        qy = np.array([ep["query_y"] for ep in meta["episodes"]])
        acc, ref_acc = float((pred == qy).mean()), float((ref_pred == qy).mean())
        half = 1.96 * np.sqrt(max(ref_acc * (1 - ref_acc), 1e-12) / E) + 1.0 / E
        print(f"[c3 x{E} bf16] prediction agreement {(pred == ref_pred).mean():.3f}, acc {acc:.3f} vs {ref_acc:.3f}")
        assert (pred == ref_pred).mean() >= BF16_MIN_AGREE and abs(acc - ref_acc) <= half
    else:
        assert np.array_equal(pred, ref_pred)
        assert acc_text == meta["acc_file"]
