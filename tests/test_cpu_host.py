"""CPU-only checks: C-ABI exports, host logic of the drop-in modules, episode sharding.

No compute call touches a GPU here."""
import ctypes
import json
import os
import random
import re
import subprocess
import sys

import numpy as np
import pytest
import torch

from _common import GOLDEN, load_fixture, load_video
from eosv import _lib, engine, episodes, synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "eosv.h")).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(eosv_\w+)\s*\(", txt, re.M)))


def test_cabi_library_exports_every_header_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    L = ctypes.CDLL(_lib.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.EXPORTS)


def test_cabi_library_links_no_vendor_blas():
    """Every GEMM of the path (inference convs, training GEMMs since r05) is an in-tree kernel: the
    library's dynamic section names no rocBLAS / hipBLAS(Lt) / MIOpen."""
    import subprocess

    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    dyn = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", dyn)
    assert needed, dyn
    bad = [n for n in needed if re.search(r"blas|miopen|hipblaslt", n, re.I)]
    assert not bad, needed


def test_cabi_null_arguments_fail_cleanly():
    L = _lib.lib()
    assert L.eosv_create(None, None) == -1
    assert b"null" in L.eosv_last_error()
    assert L.eosv_clip_embed(None, None, None, 0, 512, 1, None, None) == 0  # empty is fine
    assert L.eosv_clip_embed(None, None, None, 1, 4096, 1, None, None) == -1  # D > 2048
    assert L.eosv_match(None, None, None, None, None, 3, 512, 0, None, None, None) == -1
    assert L.eosv_feature_dim(None) == -1


def test_product_episode_sampler_matches_reference_plans():
    meta, _ = load_fixture("plans_test_seed0")
    got = episodes.sample_episodes(len(meta["episodes"]), 5, 1, "test", seed=meta["seed"])
    for a, b in zip(got, meta["episodes"]):
        assert a == {k: b[k] for k in ("support", "support_y", "query", "query_y")}


def test_native_plan_service_matches_reference_plans():
    """csrc/plan.hip (host-only C-ABI call) against the plans captured from the reference."""
    meta, _ = load_fixture("plans_test_seed0")
    got = episodes.plan_episodes(len(meta["episodes"]), 5, 1, "test", seed=meta["seed"])
    for a, b in zip(got, meta["episodes"]):
        assert a == {k: b[k] for k in ("support", "support_y", "query", "query_y")}


# both Random.sample strategies: 24 test classes / ~100 videos per class take the rejection
# set (k <= 5 -> setsize 21); n_way 20 (setsize 85) and the 14 x 10 synthetic list take the pool
@pytest.mark.parametrize("n,n_way,k_shot,seed,small", [(300, 5, 5, 7, False), (200, 3, 2, 2 ** 40 + 5, False),
                                                       (100, 20, 1, 123, False), (50, 5, 0, 9, False),
                                                       (200, 14, 1, 4, True), (100, 5, 8, 0, True)])
def test_native_plan_service_matches_python_sampler(n, n_way, k_shot, seed, small):
    lines = [f"c{c:02d}/v{v}\n" for c in range(14) for v in range(10)] if small else None
    want = episodes.sample_episodes(n, n_way, k_shot, "test", seed=seed, lines=lines)
    assert episodes.plan_episodes(n, n_way, k_shot, "test", seed=seed, lines=lines) == want


def test_native_plan_service_errors_like_random_sample():
    lines = [f"c{c}/v{v}\n" for c in range(6) for v in range(3)]
    with pytest.raises(_lib.EosvError, match="Sample larger"):
        episodes.plan_episodes(4, 7, 1, "test", seed=0, lines=lines)   # n_way > classes
    with pytest.raises(_lib.EosvError, match="Sample larger"):
        episodes.plan_episodes(4, 5, 3, "test", seed=0, lines=lines)   # query class needs k + 1 = 4 > 3
    with pytest.raises(ValueError):
        random.Random(0).sample(range(3), 4)
    assert episodes.plan_episodes(0, 5, 1, "test", seed=0) == []


def test_dropin_dataloader_matches_reference_episodes():
    import episode_novel_dataloader
    import utils

    meta, _ = load_fixture("c1_r18_protonet_seed1")
    random.seed(meta["seed"])
    dl = episode_novel_dataloader.EpisodeDataloader("test")
    for ep in meta["episodes"][:3]:
        d = dl.get_episode()
        assert d["support_y"].tolist() == ep["support_y"]
        assert d["query_y"].tolist() == [ep["query_y"]]
        assert [int(n) for n in d["support_x_frames"]] == ep["support_frames"]
        assert d["support_x"].shape == (5, 16, 3, 224, 224)
        assert d["query_x"].shape[1] == ep["query_frames"]
        v, _ = load_video(ep["query"], False)
        assert torch.equal(d["query_x"][0], v)
    assert utils.EPISODE_NUMS["test"] == 20000


def test_episode_batch_layout():
    eps = episodes.sample_episodes(7, 5, 2, "test", seed=3)
    b = engine.build_episode_batch(eps, T=16)
    assert b.n_clips == 7 * 11 and b.n_support == 70
    assert b.clip_off[0] == 0 and np.all(np.diff(b.clip_off) == b.clip_cnt[:-1])
    assert b.params.shape == (int(b.clip_cnt.sum()), 4)
    assert list(b.sup_off) == list(range(0, 71, 10))
    for e, ep in enumerate(eps):  # slot = first-appearance position of the label
        s0 = b.sup_off[e]
        first = {}
        for i, y in enumerate(ep["support_y"]):
            first.setdefault(y, len(first))
            assert b.sup_slot[s0 + i] == first[y]
    # each clip's rows carry the reference's frame ids
    vi = eps[0]["support"][0]
    ids, _ = synth.clip_frame_ids(vi, 16)
    assert list(b.params[:b.clip_cnt[0], 3]) == ids


def test_short_videos_only_in_novel_classes():
    train = {l.split("/")[0] for l in open(os.path.join(REPO, "embodied-one-shot-video-recognition_amd/sources/data/train.list"))}
    for line in open(os.path.join(GOLDEN, "test.list")).readlines()[:400]:
        vi = line.strip()
        assert synth.frame_count(vi) >= 4
    n_short = sum(synth.frame_count(l.strip()) < 16
                  for l in open(os.path.join(REPO, "embodied-one-shot-video-recognition_amd/sources/data/train.list")))
    assert n_short == 0 and len(train) == 64


_GLOO_SCRIPT = r"""
import os, sys, json
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from eosv import dist as edist, episodes
dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
d, rank, world = edist.world()
plans = episodes.sample_episodes(37, 5, 1, "test", seed=11)
mine = edist.shard_indices(len(plans), rank, world)
fake = [(e * 7 + 3) % 5 for e in mine]          # stand-in per-episode predictions
preds = edist.gather_predictions(mine, fake, len(plans))
accs = edist.episode_accs(preds, [p["query_y"] for p in plans])
t = edist.max_over_ranks(float(rank + 1))
n = edist.sum_over_ranks(len(mine))
# the config-3 gallery shard: 37 "videos" in contiguous blocks, one all-gather of their rows
lo, hi = edist.block_range(37, rank, world)
rows = torch.arange(lo * 3, hi * 3, dtype=torch.float32).view(-1, 3)
table = edist.all_gather_rows(rows)
if rank == 0:
    print(json.dumps({"preds": preds.tolist(), "accs": [float(a) for a in accs], "t": t, "n": n,
                      "table": table.tolist()}))
dist.destroy_process_group()
"""


@pytest.mark.parametrize("world", [2, 3])
def test_episode_sharding_gloo(world, tmp_path):
    script = tmp_path / "g.py"
    script.write_text(_GLOO_SCRIPT)
    pkg = os.path.join(REPO, "embodied-one-shot-video-recognition_amd")
    procs = []
    port = 29500 + world * 7 + (os.getpid() % 1000)
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(script), pkg], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    res = json.loads(outs[0][0].strip().splitlines()[-1])
    expect = [(e * 7 + 3) % 5 for e in range(37)]
    assert res["preds"] == expect
    plans = episodes.sample_episodes(37, 5, 1, "test", seed=11)
    assert res["accs"] == [float(p["query_y"] == e) for p, e in zip(plans, expect)]
    assert res["t"] == float(world) and res["n"] == 37
    assert res["table"] == np.arange(37 * 3, dtype=np.float32).reshape(37, 3).tolist()


def test_jpeg_clip_window_draws_follow_reference_order(tmp_path):
    """JpegFrames (GPU ingest path) host logic: decode + narrow-frame resize, and the train-mode
    window/flip drawn from `random` then `torch` exactly as the restated reference loader
    (oracle/frames_ref.py, utils.py:57-78) draws them -- checked without a GPU."""
    from PIL import Image

    from eosv import frames as fr

    d = tmp_path / "c" / "v"
    d.mkdir(parents=True)
    rng = np.random.default_rng(1)
    for f in (1, 2):
        Image.fromarray(rng.integers(0, 256, size=(150, 200, 3), dtype=np.uint8)).save(d / ("image_%05d.jpg" % f))
    src = fr.JpegFrames(str(tmp_path), crop=224, init_h=256)
    a = src.decode(str(d / "image_00001.jpg"))
    assert a.shape == (256, 224, 3) and a.dtype == np.uint8  # resized like utils.py:123-124
    for seed in range(5):
        random.seed(seed)
        torch.manual_seed(seed)
        got = src.window(a, "train")
        random.seed(seed)
        torch.manual_seed(seed)
        flip = random.random() < 0.5
        ij = (int(torch.randint(0, 256 - 224 + 1, size=(1,)).item()), int(torch.randint(0, 1, size=(1,)).item()))
        assert got == (ij, flip)
    assert src.window(a, "test") == (None, False)
    sq = np.zeros((224, 224, 3), np.uint8)
    torch.manual_seed(0)
    before = torch.get_rng_state()
    assert src.window(sq, "train")[0] == (0, 0)
    assert torch.equal(before, torch.get_rng_state())  # crop-sized frame: torchvision draws nothing


def test_crop_normalize_rejects_bad_window():
    """eosv_crop_normalize_frames validates its window before touching the device."""
    L = _lib.lib()
    m = (ctypes.c_float * 3)(0.5, 0.5, 0.5)
    assert L.eosv_crop_normalize_frames(None, 0, 240, 320, 224, 0, 0, 0, m, m, None, None) == 0  # empty
    assert L.eosv_crop_normalize_frames(None, 1, 240, 320, 224, 17, 0, 0, m, m, None, None) == -1  # past H
    assert L.eosv_crop_normalize_frames(None, 1, 240, 320, 224, 0, -1, 0, m, m, None, None) == -1
    assert b"window" in L.eosv_last_error()
    assert L.eosv_normalize_frames(None, 1, 200, 320, 224, m, m, None, None) == -1  # H < crop


# ----------------------------------------------------------------- host AddressSanitizer build
ASAN_BIN = os.path.join(REPO, "tests", "native", "asan_host")


def _asan_bin():
    src = os.path.join(REPO, "embodied-one-shot-video-recognition_amd", "csrc")
    subprocess.run(["make", "-s", "-C", src, "asan", "-j", str(min(8, os.cpu_count() or 4))], check=True,
                   capture_output=True)
    return ASAN_BIN


def test_asan_host_argument_validation():
    """the C++ glue under AddressSanitizer (+ LeakSanitizer): every entry point's argument
    checks return an error with a message and touch no memory they do not own."""
    r = subprocess.run([_asan_bin(), "args"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "asan_host args: ok" in r.stdout


@pytest.mark.parametrize("n_way,k_shot,seed,n,sizes", [
    (5, 1, 0, 200, None),                       # the test split, reference shape
    (14, 1, 7, 50, [10] * 14),                  # UnrealAction-shaped: every class every episode
    (5, 5, 39, 40, None),                       # config 5's 5-shot
    (20, 3, 2 ** 40 + 1, 30, None),             # pool strategy of random.sample
    (3, 2, 5, 10, [3, 2, 4, 3]),                # a class too small for the query draw -> error
])
def test_asan_host_plan_service_matches_library(n_way, k_shot, seed, n, sizes):
    """The plan service under ASan prints the same plans as the release library's (ctypes)."""
    if sizes is None:
        idx = episodes.class_index(episodes.read_list("test"))
        sizes = [len(v) for v in idx.values()]
    r = subprocess.run([_asan_bin(), "plan", str(n_way), str(k_shot), str(seed), str(n), *map(str, sizes)],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    assert r.returncode == 0, r.stderr[-4000:]
    import numpy as np

    cls = np.zeros((n, n_way), np.int32)
    q = np.zeros((n, 2), np.int32)
    sup = np.zeros((n, n_way, max(k_shot, 1)), np.int32)
    arr = np.array(sizes, np.int32)
    rc = _lib.lib().eosv_plan_episodes(arr.ctypes.data, len(sizes), n_way, k_shot, ctypes.c_uint64(seed), n,
                                       cls.ctypes.data, q.ctypes.data, sup.ctypes.data)
    if rc:
        assert r.stdout.startswith(f"ERR {rc} ")
        return
    want = " ".join(" ".join(map(str, [*cls[e], *q[e], *sup[e].reshape(-1)[:n_way * k_shot]])) for e in range(n))
    assert r.stdout.split() == want.split()


def test_dropin_classifier_host_kinds_follow_reference():
    """classifier.py:98-123 for the kinds the match kernel does not run: 'SVM' is sklearn's
    SVC(C=10) on the host, equal to the oracle's restatement on the SVM fixture's own reference
    embeddings; 'KNN' raises the reference's NameError (k_shot is never imported there);
    an unknown kind prints and raises UnboundLocalError."""
    import classifier
    from oracle import harness_ref

    meta, arr = load_fixture("c1_r18_svm_seed5")
    for e, ep in enumerate(meta["episodes"]):
        d = {"support_feature": arr["support_feature"][e], "support_y": np.array(ep["support_y"], np.float32),
             "query_feature": arr["query_feature"][e], "query_y": np.array([ep["query_y"]], np.float32)}
        got = classifier.Classifier("SVM").predict(d)
        ref = harness_ref.predict("SVM", d["support_feature"], d["support_y"], d["query_feature"], d["query_y"])
        assert np.array_equal(got, ref) and int(got[0]) == int(arr["pred"][e][0])
    with pytest.raises(NameError, match="k_shot"):
        classifier.Classifier("KNN").predict(d)
    with pytest.raises(UnboundLocalError):
        classifier.Classifier("LR").predict(d)


def test_train_network_steplr_matches_torch_schedule():
    """TrainNetwork.lr_at restates StepLR(step_size, 0.1) stepped at the start of each epoch
    (reference network_train.py:77-84) -- checked against torch's own scheduler, no GPU."""
    import types

    import network_train

    for step_size in (1, 3, 10):
        tn = types.SimpleNamespace(lr_1=1e-4, lr_2=1e-3, lr_step_size=step_size)
        p = torch.nn.Parameter(torch.zeros(1))
        o1 = torch.optim.SGD([p], lr=1e-4, momentum=0.9)
        o2 = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1e-3, momentum=0.9)
        s1 = torch.optim.lr_scheduler.StepLR(o1, step_size=step_size, gamma=0.1)
        s2 = torch.optim.lr_scheduler.StepLR(o2, step_size=step_size, gamma=0.1)
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for epoch in range(12):
                s1.step()
                s2.step()
                l1, l2 = network_train.TrainNetwork.lr_at(tn, epoch)
                assert abs(l1 - o1.param_groups[0]["lr"]) <= 1e-12 and abs(l2 - o2.param_groups[0]["lr"]) <= 1e-12


def test_conv_launch_bytes_and_per_layer_bound():
    """bench.py's per-layer roofline: arch.conv_launch_bytes follows the native plan's layer ids
    (a folded downsample's entry is empty, its weights on the block's last conv), and
    layer_bounds prices each launch at max(MFMA, HBM) with a fused conv1's bytes (less its
    input map) moved onto the launch it was fused into."""
    import types

    sys.path.insert(0, os.path.dirname(os.path.dirname(GOLDEN)))  # the repo root: bench.py
    import bench
    from eosv import arch

    spec = arch.SPECS["resnet50"]
    L = arch.conv_launch_bytes(spec, 224, 224, 2)
    assert len(L) == len(arch.conv_layer_bytes(spec, 224, 224, 2, True))
    # stem: f32 frame in, pooled bf16 map out
    assert L[0][0] == 3 * 224 * 224 * 4 + 56 * 56 * 64 * 2
    # layer1 block 0: conv3 reads its 64-ch input and the downsample's 64-ch input, writes 256 ch
    assert L[3][0] == (56 * 56 * 64 + 56 * 56 * 64 + 56 * 56 * 256) * 2
    assert L[3][1] == (256 * 64 + 256 * 64) * 2 and L[4] == (0, 0, 0)
    # block 1 conv3: + the 256-ch residual
    assert L[7][0] == (56 * 56 * 64 + 2 * 56 * 56 * 256) * 2
    # conv1 of block 1: input map 256 ch
    assert L[5][2] == 56 * 56 * 256 * 2
    frames = 1000
    n = len(L)
    ms, fl, nl = np.zeros(n), np.zeros(n), np.zeros(n)
    for i in range(n):  # every conv launched once, except the downsamples and block 2's conv1 (fused)
        if L[i][0] and i != 8:
            nl[i], ms[i] = 1, 1.0
    fl[7] = 2 * frames * 56 * 56 * (256 * 64 + 64 * 256)  # conv3 + the fused next conv1
    args = types.SimpleNamespace(arch="resnet50", res=224)
    out = bench.layer_bounds((ms, fl, nl), "bf16", args, arch, frames)
    hbm = bench.HBM_PEAK_GBPS * 1e9
    floors = []
    for i in range(n):
        if not nl[i]:
            continue
        b = frames * L[i][0] + L[i][1]
        if i == 7:  # the fused conv1's bytes, less its input map (never re-read)
            b += frames * (L[8][0] - L[8][2]) + L[8][1]
        floors.append(max(b / hbm * 1e3, fl[i] / (bench.MFMA_PEAK_TF["bf16"] * 1e12) * 1e3))
    assert out["layers"] == int(nl.sum()) and out["hbm_bound_layers"] == int(nl.sum())
    assert abs(out["frac"] - sum(floors) / ms.sum()) < 1e-4


def test_row_kernel_lds_layouts_conflict_free():
    """The LDS images of the row kernels (conv_rows_bf16 / conv_rowsr_bf16.hip: C 64 slots of 128 B
    with chunk c at c ^ (p & 7); C 128 slots of 256 B with c ^ ((2p + 8r) & 15)) serve every
    B-fragment ds_read_b128 in 4 LDS cycles (one per lane group: conflict-free), for every pixel
    tile, tap and 32-channel slice, at the four map widths the kernels take (tools/lds_sim.py,
    the b128 lane groups of MI355X_MICROARCH.md); the C 64 swizzle at 256-B slots does not."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("lds_sim", os.path.join(REPO, "tools", "lds_sim.py"))
    sim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sim)
    c64 = lambda p, c, r: c ^ (p & 7)  # noqa: E731
    c128 = lambda p, c, r: c ^ ((2 * p + 8 * r) & 15)  # noqa: E731
    assert sim.sim(56, 64, 128, c64, 7, 2) == (4, 4.0)
    assert sim.sim(64, 64, 128, c64, 8, 2) == (4, 4.0)
    assert sim.sim(28, 128, 256, c128, 7, 1) == (4, 4.0)
    assert sim.sim(32, 128, 256, c128, 8, 1) == (4, 4.0)
    assert sim.sim(28, 128, 256, c64, 7, 1)[0] > 4


def test_no_inline_asm_memory_instructions():
    """r06 (verdict r05, item 2): no kernel issues a load or store from inline asm.

    An asm load's destination is written asynchronously, which hipcc cannot see: under register
    pressure it may copy the destination, or reuse it as the next address, before the data lands
    (the r05 conv_rowsr_bf16 memory fault).  Every VMEM / LDS access is therefore a
    compiler-visible load / store or builtin; inline asm keeps only wait counts, DPP VALU, s_nop
    and empty compiler barriers.  This scans every asm statement's text in the kernel sources."""
    csrc = os.path.join(REPO, "embodied-one-shot-video-recognition_amd", "csrc")
    mem = re.compile(r"\b(ds|global|buffer|flat|scratch)_[a-z0-9_]+|\bs_(buffer_)?load")
    bad = []
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith((".hip", ".h")):
            continue
        src = open(os.path.join(csrc, fn)).read()
        src = re.sub(r"//[^\n]*", "", src)  # comments
        for m in re.finditer(r"\basm\s*(volatile\s*)?\(", src):
            # the asm statement up to its closing parenthesis (string literals hold no parentheses
            # here except inside operand constraints, which are balanced)
            i, depth = m.end(), 1
            while depth and i < len(src):
                depth += {"(": 1, ")": -1}.get(src[i], 0)
                i += 1
            text = " ".join(re.findall(r'"((?:[^"\\]|\\.)*)"', src[m.end():i]))
            text = re.sub(r"\\[nt]", " ", text)  # the asm's own line breaks and tabs
            if mem.search(text):
                bad.append(f"{fn}: {text[:80]}")
    assert not bad, bad


def test_no_store_data_hazard_in_library():
    """r06: no 128-/96-bit VMEM store in the built library is directly followed by a VALU write of
    its data VGPRs.  hipcc pads that pair only for an inline-constant soffset; with an SGPR soffset
    the write won on gfx950 (bneck_bf16_kernel<64,64,false>: one dword of lanes 12/13 held the
    next v_mov's LDS base, tests/native/bneck_check.cpp).  Disassembles every gfx950 code object of
    the release and profiling libraries (tools/isa_scan.py)."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import isa_scan
    if not os.path.exists(os.path.join(isa_scan.LLVM, "llvm-objdump")):
        pytest.skip("no llvm-objdump")
    pkg = os.path.dirname(_lib.LIB_PATH)
    libs = [p for p in (os.path.join(pkg, "libeosv.so"), os.path.join(pkg, "libeosv_prof.so")) if os.path.exists(p)]
    if not libs:
        pytest.skip("library not built")
    for lib in libs:
        n = len(isa_scan.code_objects(lib))
        assert n > 10, f"{lib}: {n} gfx950 code objects"
        found = isa_scan.scan(lib)
        assert not found, found[:4]


def test_fused_block_bytes_follow_the_profile():
    """r06: a stage-1 block run as ONE launch (bneck_bf16.hip: conv1 launched, conv2 / conv3 not) is
    priced as input map + output map (+ the next conv1's output when that one is fused too) and all
    its weights; its 64-channel maps never reach HBM.  Blocks launched conv by conv keep their bytes."""
    from eosv import arch

    spec = arch.SPECS["resnet50"]
    ids = arch.block_layer_ids(spec)
    assert ids[0] == (1, 2, 3, 4) and ids[1] == (5, 6, 7, None) and ids[3] == (11, 12, 13, 14)
    assert sum(len([x for x in b if x is not None]) for b in ids) + 1 == len(arch.conv_launch_bytes(spec))
    L = arch.conv_launch_bytes(spec, 224, 224, 2)
    n = len(L)
    nl = np.array([1 if L[i][0] else 0 for i in range(n)])
    nl[[2, 3, 6, 7, 8]] = 0  # blocks 0 and 1 fused (block 1 with block 2's conv1)
    F = arch.fuse_bneck_bytes(L, spec, nl)
    px = 56 * 56
    assert F[1][0] == (px * 64 + px * 256) * 2  # block 0: X0 in, Y0 out (the downsample reads X0 too)
    assert F[1][1] == (64 * 64 + 64 * 576 + 256 * 128) * 2
    assert F[5][0] == (px * 256 + px * 256) * 2  # block 1: Y0 in (also the residual), Y1 out
    assert F[2] == F[3] == F[6] == F[7] == (0, 0, 0)
    assert F[8] == L[8] and F[9:] == L[9:]  # block 2's conv1 keeps its entry (the generic next-conv1 rule)
    # blocks run conv by conv: unchanged
    assert arch.fuse_bneck_bytes(L, spec, np.array([1 if L[i][0] else 0 for i in range(n)])) == L


def test_fused_basic_block_bytes_follow_the_profile():
    """r06: an R18 stage-1 basic block run as ONE launch (bblock_bf16.hip: conv1 launched, conv2 not)
    is priced as block input + block output (conv1's input is conv2's residual, read once) with both
    weight tensors; the conv1 output never reaches HBM."""
    from eosv import arch

    spec = arch.SPECS["resnet18"]
    ids = arch.block_layer_ids(spec)
    assert ids[0] == (1, 2, None, None) and ids[1] == (3, 4, None, None)
    L = arch.conv_launch_bytes(spec, 224, 224, 2)
    n = len(L)
    nl = np.array([1 if L[i][0] else 0 for i in range(n)])
    nl[[2, 4]] = 0  # both stage-1 blocks fused
    F = arch.fuse_bneck_bytes(L, spec, nl)
    px = 56 * 56
    assert F[1] == (2 * px * 64 * 2, 2 * 64 * 576 * 2, px * 64 * 2) and F[3] == F[1]
    assert F[2] == F[4] == (0, 0, 0) and F[5:] == L[5:]
    assert arch.fuse_bneck_bytes(L, spec, np.array([1 if L[i][0] else 0 for i in range(n)])) == L
