"""GPU: real-frame ingest -- JPEG clips on disk through the drop-in loaders
(host PIL decode, GPU crop / flip / ToTensor / Normalize) against the host restatement of the
reference's loaders (oracle/frames_ref.py, utils.py:57-91, 215-258), bit-exact, in test and
train mode (same RNG draws), for normal, narrow (resized) and short (zero-padded) videos.

The JPEGs are written here with PIL from seeded noise; the reference ships no frame data, so
the restatement, not the reference, is the checker (parity unpinned at the torchvision layer,
as for the backbone)."""
import random

import numpy as np
import pytest
import torch

from oracle import frames_ref

pytestmark = pytest.mark.gpu

# (video, width, height, frames on disk): normal 320x240, narrow 200x150 (resized to 224x256),
# exactly crop-sized (train window draws nothing), short clip (zero padding, count < T)
VIDEOS = [("walk/v_a", 320, 240, 24), ("walk/v_narrow", 200, 150, 21), ("run/v_exact", 224, 224, 20),
          ("run/v_short", 300, 260, 9)]


@pytest.fixture(scope="module")
def frame_dir(tmp_path_factory):
    from PIL import Image

    root = tmp_path_factory.mktemp("frames")
    rng = np.random.default_rng(11)
    for vi, w, h, n in VIDEOS:
        d = root / vi
        d.mkdir(parents=True)
        base = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        for f in range(1, n + 1):
            a = np.clip(base.astype(np.int16) + rng.integers(-20, 21, size=(h, w, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(a).save(d / ("image_%05d.jpg" % f), quality=90)
        (d / "extra.txt").write_text("x")  # the reference counts listdir() - 1
    return str(root)


def test_crop_normalize_kernel_window_and_flip():
    from eosv import engine

    rng = np.random.default_rng(3)
    rgb = rng.integers(0, 256, size=(2, 240, 300, 3), dtype=np.uint8)
    for top, left, flip in [(0, 0, False), (16, 76, True), (5, 3, True)]:
        out = engine.crop_normalize_frames(torch.from_numpy(rgb).cuda(), 224, top, left, flip).cpu().numpy()
        a = rgb[:, top:top + 224, left:left + 224]
        if flip:
            a = a[:, :, ::-1]
        x = a.astype(np.float32) / np.float32(255.0)
        ref = ((x - frames_ref.MEAN) / frames_ref.STD).transpose(0, 3, 1, 2)
        assert np.array_equal(out.view(np.uint32), np.ascontiguousarray(ref).view(np.uint32))
    with pytest.raises(RuntimeError):
        engine.crop_normalize_frames(torch.from_numpy(rgb).cuda(), 224, 20, 0, False)  # window past H


@pytest.mark.parametrize("mode", ["test", "train"])
@pytest.mark.parametrize("vi", [v[0] for v in VIDEOS])
def test_loader_matches_reference_restatement(frame_dir, vi, mode):
    import utils

    T = 16
    random.seed(7)
    torch.manual_seed(7)
    v, n = utils.get_video_from_video_info_3(vi, mode, video_frames=T, frame_dir=frame_dir)
    random.seed(7)
    torch.manual_seed(7)
    ref, ref_n = frames_ref.load_clip_padded(frame_dir, vi, mode, T=T)
    assert v.is_cuda and tuple(v.shape) == (T, 3, 224, 224)
    assert int(n) == ref_n
    assert np.array_equal(v.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    # the unpadded loader returns the real frames only (utils.py:96-136)
    random.seed(7)
    torch.manual_seed(7)
    u = utils.get_video_from_video_info(vi, mode, video_frames=T, frame_dir=frame_dir)
    assert u.shape[0] == min(T, ref_n) and torch.equal(u.cpu(), v[:u.shape[0]].cpu())


def test_transforms_dropin(frame_dir):
    import os

    from PIL import Image
    import utils

    img = Image.open(os.path.join(frame_dir, "walk/v_a", "image_00003.jpg"))
    a = np.asarray(img.convert("RGB"))
    out = utils.transforms("test")(img)
    i, j = int(round((240 - 224) / 2.0)), int(round((320 - 224) / 2.0))
    x = a[i:i + 224, j:j + 224].astype(np.float32) / np.float32(255.0)
    ref = ((x - frames_ref.MEAN) / frames_ref.STD).transpose(2, 0, 1)
    assert out.is_cuda and np.array_equal(out.cpu().numpy().view(np.uint32), np.ascontiguousarray(ref).view(np.uint32))


# end-to-end: 6 classes x 2 videos (5-way 1-shot needs k_shot + 1 = 2 videos of the query class)
E2E = [(f"c{c}/v{v}", 320 if (c + v) % 3 else 200, 240 if (c + v) % 3 else 150, 30 if v else 18)
       for c in range(6) for v in range(2)]
E2E[3] = ("c1/v1", 320, 240, 10)  # short clip: zero-padded support / truncated query


@pytest.fixture(scope="module")
def e2e_dir(tmp_path_factory):
    from PIL import Image

    root = tmp_path_factory.mktemp("e2e")
    rng = np.random.default_rng(12)
    for vi, w, h, n in E2E:
        d = root / vi
        d.mkdir(parents=True)
        cls = np.random.default_rng(int(vi[1])).integers(0, 256, size=(h, w, 3))
        for f in range(1, n + 1):
            a = np.clip(cls + rng.integers(-60, 61, size=(h, w, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(a).save(d / ("image_%05d.jpg" % f), quality=90)
        (d / "extra.txt").write_text("x")
    (root / "test.list").write_text("".join(vi + "\n" for vi, *_ in E2E))
    return str(root)


def test_network_baseline_on_jpeg_frames(e2e_dir, tmp_path, monkeypatch):
    """TestNetwork.test_network_baseline over real JPEG clips (batched GPU path: host decode,
    GPU ingest, backbone, clip embedding, protonet) == the reference's per-episode loop restated
    on the CPU (oracle: frames_ref loaders + torch-CPU ResNet-18 + classifier restatement):
    integer predictions bit-exact."""
    import os

    import network_test
    import utils
    from eosv import arch, synth
    from oracle import harness_ref, resnet_ref

    n_ep = 4
    monkeypatch.setattr(utils, "TEST_LIST", os.path.join(e2e_dir, "test.list"))
    monkeypatch.setattr(utils, "KINETICS_FRAME_DIR", e2e_dir)
    monkeypatch.setitem(utils.EPISODE_NUMS, "test", n_ep)
    sd = synth.synth_state_dict(arch.SPECS["resnet18"], 64, 0)
    pkl = str(tmp_path / "model.pkl")
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, pkl)

    random.seed(5)
    tn = network_test.TestNetwork(str(tmp_path / "acc.txt"), "resnet18", "protonet", True)
    tn.episodes_per_batch = 3  # two batches, ragged last one
    tn.test_network_baseline(pre_model=pkl)
    tn.acc_file.close()

    random.seed(5)
    lines = open(os.path.join(e2e_dir, "test.list")).readlines()
    index = harness_ref.class_index(lines)
    plans = [harness_ref.sample_episode_plan(index, 5, 1) for _ in range(n_ep)]

    def load(vi, support):
        v, n = frames_ref.load_clip_padded(e2e_dir, vi, "test", T=16)
        return (torch.from_numpy(v), n) if support else (torch.from_numpy(v[:n]), n)

    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    model = resnet_ref.build_model("resnet18", sd)
    ref = harness_ref.run_baseline(model, plans, load, L2=True, kind="protonet")
    assert [int(np.asarray(r["pred"]).reshape(-1)[0]) for r in ref] == [int(p) for p in tn.last_preds]
