"""GPU: the episode-sharded multi-rank paths with 2 ranks on the box's
one device.  RCCL refuses two ranks on one GPU, so these run the same code over gloo
(EOSV_DIST_BACKEND=gloo); on a node, the driver's N-GPU bench uses RCCL over xGMI.

* the drop-in TestNetwork.test_network_baseline over 2 ranks writes the reference's result file
  byte for byte (network_test.py:132-167);
* the config-3 driver (test_network_aug_segment) over 2 ranks: each rank forwards half of the
  640 gallery videos and one all-gather rebuilds the table; the result file, pool ids and
  augmented embeddings equal the 1-rank run's fixture (network_test.py:170-267);
* ``bench.py --gpus 2`` spawns its own ranks (no launcher), reports n_gpus = 2 and the same
  episode accuracy as the 1-rank run over the same timed episodes.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from _common import load_fixture

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "embodied-one-shot-video-recognition_amd")

_DROPIN = r"""
import os, random, sys
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
torch.cuda.set_device(0)
dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
import network_test, utils
from eosv import arch, synth
tag, out = sys.argv[3], sys.argv[4]
import json
meta = json.load(open(os.path.join(sys.argv[2], "tests", "golden", tag + ".json")))
utils.EPISODE_NUMS["test"] = len(meta["episodes"])
if "n_way" in meta:  # an episode shape set the way a reference user sets it: the utils globals
    utils.n_way, utils.k_shot, utils.VIDEO_FRAMES = meta["n_way"], meta["k_shot"], meta["video_frames"]
    utils.IMG_crop_size = (meta["H"], meta["W"])
    if meta.get("test_list", "sources/data/test.list") != "sources/data/test.list":
        utils.TEST_LIST = os.path.join(sys.argv[2], "tests", "golden", meta["test_list"])
pkl = out + ".model.pkl"
if dist.get_rank() == 0:
    sd = synth.synth_state_dict(arch.SPECS[meta["arch"]], 64, 0)
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, pkl)
dist.barrier()
random.seed(meta["seed"])
tn = network_test.TestNetwork(out, meta["arch"], meta["classifier"], True)
tn.episodes_per_batch = 4
tn.test_network_baseline(pre_model=pkl)
if dist.get_rank() == 0:
    tn.acc_file.close()
dist.destroy_process_group()
"""


def _spawn(argv, world, port, env_extra=None, timeout=240):
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), **(env_extra or {}))
        procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=timeout) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-3000:] for o in outs]
    return outs


C4_WIDE = "c4_r50_14w1s_t32_seed8_wide"


@pytest.mark.parametrize("tag", ["c1_r18_protonet_seed1", "c1_r18_cosine_seed2", "c4_r50_14w1s_t32_seed7"]
                         + ([C4_WIDE] if os.path.exists(os.path.join(REPO, "tests", "golden", C4_WIDE + ".json")) else []))
def test_dropin_baseline_two_ranks_writes_reference_file(tag, tmp_path):
    """Config 4's shape too (BASELINE configs[3]: 14-way 1-shot, 16 segments, R50 over the
    UnrealAction-shaped split, episodes sharded over ranks with one all-gather of the predictions):
    2 ranks write the reference's result file byte for byte (network_test.py:159-167)."""
    script = tmp_path / "dropin.py"
    script.write_text(_DROPIN)
    out = str(tmp_path / "acc.txt")
    _spawn([sys.executable, str(script), PKG, REPO, tag, out], 2, 29611 + os.getpid() % 500, timeout=300)
    meta, _ = load_fixture(tag)
    text = open(out).read()
    if "acc_file" in meta:
        assert text == meta["acc_file"]
    else:
        import hashlib
        assert hashlib.sha256(text.encode()).hexdigest() == meta["acc_file_sha256"]


_DROPIN_AUG = r"""
import os, random, sys
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
torch.cuda.set_device(0)
dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
rank = dist.get_rank()
import generate_augmented_datasets as gad, network_test, utils
from eosv import arch, synth
tag, out = sys.argv[3], sys.argv[4]
import json
meta = json.load(open(os.path.join(sys.argv[2], "tests", "golden", tag + ".json")))
utils.EPISODE_NUMS["test"] = len(meta["episodes"])
utils.GALLERY_LIST = out + f".gallery{rank}.list"
pkl = out + ".model.pkl"
if rank == 0:
    sd = synth.synth_state_dict(arch.SPECS["resnet50"], 64, 0)
    torch.save({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, pkl)
dist.barrier()
random.seed(meta["seed"]); np.random.seed(meta["seed"])
gad.generate_gallery_list()
assert gad.gallery_video_infos() == meta["gallery"]
tn = network_test.TestNetwork(out, "resnet50", "protonet", True)
tn.mymodel.compute_dtype = "f32"
tn.debug = {}
tn.test_network_aug_segment(pre_model=pkl)
if rank == 0:
    tn.acc_file.close()
np.savez(out + f".rank{rank}.npz", pool=tn.debug["pool"].cpu().numpy(), sup=tn.debug["sup"].cpu().numpy(),
         seg_sum=float(tn._gallery_raw.double().sum()), n_gal=tn._gallery_raw.shape[0])
dist.destroy_process_group()
"""


def test_aug_segment_two_ranks_shard_the_gallery(tmp_path):
    """Episodes e % 2 == r on rank r, the gallery forward split in two contiguous halves."""
    tag = "c3_r50_aug_seed6"
    script = tmp_path / "aug.py"
    script.write_text(_DROPIN_AUG)
    out = str(tmp_path / "acc.txt")
    _spawn([sys.executable, str(script), PKG, REPO, tag, out], 2, 29811 + os.getpid() % 500, timeout=300)
    meta, arr = load_fixture(tag)
    assert open(out).read() == meta["acc_file"]
    r0, r1 = (np.load(out + f".rank{r}.npz") for r in (0, 1))
    assert int(r0["n_gal"]) == int(r1["n_gal"]) == 640 * 16 and float(r0["seg_sum"]) == float(r1["seg_sum"])
    E = len(meta["episodes"])
    ref_pool = arr["pool"].astype(np.int64)
    for r, res in ((0, r0), (1, r1)):  # rank r ran episodes r, r + 2, ...
        got = res["pool"].reshape(-1, ref_pool.shape[1])
        assert np.array_equal(got, ref_pool[r::2]), r
        sup = res["sup"].astype(np.float64).reshape(-1, 45, 2048)
        rv = np.random.default_rng(20261017).standard_normal(2048)
        bound = 1e-4 * np.sqrt(2048) * arr["aug_absmax"][r::2] * np.linalg.norm(rv)
        assert (np.abs(sup @ rv - arr["aug_proj"][r::2]) <= bound).all()
    assert E == 8


def _bench(extra_env, gpus, eps):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--steps", "1", "--warmup", "1",
           "--episodes-per-step", str(eps), "--max-frames", "512", "--no-cpu-baseline", "--secondary-dtype", ""]
    env = dict(os.environ, **extra_env)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_bench_spawns_ranks_and_matches_one_rank():
    two = _bench({"EOSV_DIST_BACKEND": "gloo"}, 2, 12)
    one = _bench({}, 1, 24)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["episodes_timed"] == one["config"]["episodes_timed"] == 24
    assert two["config"]["parallelism"] == "episode-sharded dp2"
    # same 24 timed episodes (plans are drawn once in the reference's order and dealt e % world)
    assert two["episode_acc"] == one["episode_acc"]
    assert abs(two["value_per_gpu"] * 2 - two["value"]) < 0.02 * two["value"]
    # the self-verifying record: what the process group reports, and every rank's share
    d2, d1 = two["dist"], one["dist"]
    assert d2["backend"] == "gloo" and d2["world_size_reported_by_backend"] == 2 and d2["launched_world_size"] == 2
    assert d1["backend"] is None and d1["world_size_reported_by_backend"] == 1
    assert len(d2["per_rank_clips"]) == 2 and len(d2["per_rank_elapsed_s"]) == 2
    assert sum(d2["per_rank_clips"]) == sum(d1["per_rank_clips"]) == 24 * 6
    clips = sum(d2["per_rank_clips"])
    assert abs(two["value"] - clips / max(d2["per_rank_elapsed_s"])) <= 0.01 * two["value"]


# ------------------------------------------------------------------ RCCL (the "nccl" backend)
_RCCL_ONE = r"""
import os, sys
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from eosv import dist as edist
assert edist.describe() == {"backend": "nccl", "world_size_reported_by_backend": 1}, edist.describe()
# the collectives bench.py and the drop-in drivers run, through RCCL on the device
p = edist.gather_predictions([0, 2, 5], [4, 1, 3], 7)
assert p.tolist() == [4, -1, 1, -1, -1, 3, -1], p
x = torch.arange(48, dtype=torch.float32, device="cuda").reshape(6, 8)
y = edist.all_gather_rows(x)
assert y.device.type == "cuda" and torch.equal(y, x)
assert edist.gather_values(2.5) == [2.5]
assert edist.max_over_ranks(3.25) == 3.25 and edist.sum_over_ranks(11) == 11
dist.barrier()
dist.destroy_process_group()
print("rccl ok")
"""


def test_rccl_world_size_one_collectives(tmp_path):
    """The nccl (= RCCL) branch of eosv/dist.py executed on the device at world size 1: backend
    reported, the (episode, prediction) all-gather, the row all-gather, the value all-gather and the
    all-reduces (network_test.py:159-167 gathers its accuracies through these)."""
    script = tmp_path / "rccl1.py"
    script.write_text(_RCCL_ONE)
    (out, err), = _spawn([sys.executable, str(script), PKG], 1, 30011 + os.getpid() % 500, timeout=180)
    assert "rccl ok" in out, err[-3000:]


def test_bench_rccl_world_size_one():
    """bench.py's process-group path on RCCL (EOSV_DIST_BACKEND=nccl at N = 1, no launcher): the
    line reports backend nccl, and the same accuracy / clips as the single-process run."""
    rccl = _bench({"EOSV_DIST_BACKEND": "nccl"}, 1, 12)
    one = _bench({}, 1, 12)
    d = rccl["dist"]
    assert d["backend"] == "nccl" and d["world_size_reported_by_backend"] == 1 and d["launched_world_size"] == 1
    assert rccl["episode_acc"] == one["episode_acc"]
    assert d["per_rank_clips"] == one["dist"]["per_rank_clips"]
