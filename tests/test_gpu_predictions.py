"""GPU: prediction parity over 1000 reference episodes (BASELINE config 2's workload: R18, 5-way
1-shot, T = 16, 224x224, f32), captured from the reference's own test_network_baseline loop
(network_test.py:143-164; tests/golden/capture_golden.py --preds 1000).

The fixture holds, per episode, the reference's prediction, its f64 prototype distances
(classifier.py:63), the top-2 relative distance margin, and a fixed random projection of every
clip embedding (a size-independent check of the 6000 embeddings without storing them).  The test
runs the drop-in TestNetwork over all 1000 episodes and asserts identical predictions, the
result file's sha256, embeddings within the north star's 1e-4 relative bound, and reports the
near-tie episodes (margin < 1e-5) where a 1-ulp difference could flip a prediction.
"""
import hashlib
import random

import numpy as np
import pytest
import torch

from _common import load_fixture
from eosv import arch, synth

pytestmark = pytest.mark.gpu

TAG = "c2_r18_preds1000_seed0"


@pytest.mark.parametrize("dtype", ["f32", "f32x3"])
def test_thousand_reference_episodes_bit_exact(dtype, tmp_path, monkeypatch):
    """f32 (exact-f32 MFMA) and f32x3 (split-bf16, f32-accurate): identical predictions on all
    1000 reference episodes and embeddings within the 1e-4 bound."""
    import network_test
    import utils

    meta, arr = load_fixture(TAG)
    plans, _ = load_fixture(meta["plans"][:-len(".json")])
    n = meta["n_episodes"]
    monkeypatch.setitem(utils.EPISODE_NUMS, "test", n)
    pkl = str(tmp_path / "model.pkl")
    sd = synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0)
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, pkl)
    acc_path = str(tmp_path / "acc.txt")
    random.seed(meta["seed"])
    tn = network_test.TestNetwork(acc_path, "resnet18", "protonet", True)
    tn.mymodel.compute_dtype = dtype
    tn.mymodel.max_frames = 2048
    tn.episodes_per_batch = 250
    tn.debug = {}
    tn.test_network_baseline(pre_model=pkl)
    tn.acc_file.close()

    preds = np.array(tn.last_preds)
    ref_pred = arr["pred"]
    margin = arr["margin"]
    near = np.flatnonzero(margin < 1e-5)
    print(f"[c2 x{n} {dtype}] min top-2 margin {margin.min():.3e}, near ties (< 1e-5): {len(near)} {near.tolist()}")
    assert np.array_equal(preds, ref_pred), np.flatnonzero(preds != ref_pred).tolist()
    text = open(acc_path).read()
    assert hashlib.sha256(text.encode()).hexdigest() == meta["acc_file_sha256"]
    assert text.splitlines()[-1] == meta["acc_file_tail"]

    # embeddings: projections onto the fixture's fixed random vector.  |dproj| <= ||de||_2 ||r||_2 and the
    # 1e-4 relative bound (max|de| <= 1e-4 max|e|) gives ||de||_2 <= 1e-4 sqrt(D) max|e|.
    sup = torch.cat([b["sup"] for b in tn.debug["batches"]]).cpu().numpy().astype(np.float64)
    q = torch.cat([b["q"] for b in tn.debug["batches"]]).cpu().numpy().astype(np.float64)
    D = sup.shape[1]
    r = np.random.default_rng(int(arr["proj_vector_seed"])).standard_normal(D)
    n_sup = sup.shape[0] // n
    assert n_sup * n == sup.shape[0] == 5 * n  # every batch is full (250 | 1000): episode-major rows
    got = np.concatenate([(sup @ r).reshape(n, n_sup), (q @ r)[:, None]], axis=1)
    bound = 1e-4 * np.sqrt(D) * max(np.abs(sup).max(), np.abs(q).max()) * np.linalg.norm(r)
    err = np.abs(got - arr["proj"]).max()
    print(f"[c2 x{n} {dtype}] max projection error {err:.3e} (bound {bound:.3e})")
    assert err <= bound
    assert len(plans["episodes"]) >= n


def test_thousand_reference_episode_distances():
    """eosv_match's f64 prototype distances (rounded to f32, classifier.py:63-66) on the GPU
    embeddings of the first 250 episodes against the reference's."""
    from eosv import engine

    meta, arr = load_fixture(TAG)
    plans, _ = load_fixture(meta["plans"][:-len(".json")])
    eps = plans["episodes"][:250]
    bb = engine.Backbone("resnet18", "f32", 224, 224, max_frames=2048, device=0)
    bb.load_state_dict(synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0))
    dev = engine.DeviceEpisodes(engine.build_episode_batch(eps, T=16), 224, 224, device=0)
    pred, emb, score = engine.run_episodes(bb, dev, "protonet", True)
    bb.close()
    d = score.cpu().numpy()[:, :5].astype(np.float64)
    ref = arr["dists"][:250]
    rel = np.abs(d - ref).max() / np.abs(ref).max()
    print(f"[c2 x250] max relative distance error {rel:.3e}")
    assert rel < 1e-4
    assert np.array_equal(pred.cpu().numpy(), arr["pred"][:250])
