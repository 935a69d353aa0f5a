#!/usr/bin/env python3
"""Throughput of the non-headline BASELINE configs on one GPU (the headline is bench.py).

  --config 3 : test_network_aug_segment (aug_seg_T), ResNet-50, 640-video gallery, the
               drop-in TestNetwork on synthetic frames.  Gallery features are computed once
               (timed separately); the timed region covers --episodes episodes end to end.
  --config 4 / 5 : delegate to bench.py with the config's shape (14-way 1-shot T=32 R50;
               5-way 5-shot T=64 256x256 R101).

Prints one JSON line.
"""
import argparse
import json
import os
import random
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "embodied-one-shot-video-recognition_amd")
sys.path.insert(0, PKG)


C3_KEY = "c3:resnet50@224x224/BASELINE configs[2]"


def config3(args):
    import numpy as np
    import torch

    import generate_augmented_datasets as gad
    import network_test
    import utils
    from eosv import arch

    td = tempfile.mkdtemp()
    utils.GALLERY_LIST = os.path.join(td, "gallery.list")
    random.seed(args.seed)
    gad.generate_gallery_list()
    utils.EPISODE_NUMS["test"] = args.episodes
    tn = network_test.TestNetwork(os.path.join(td, "acc.txt"), "resnet50", "protonet", True)
    tn.mymodel.compute_dtype = args.dtype
    tn.mymodel.max_frames = args.max_frames or 4096  # r02: 4096 +6 % over 1024 (tools/mf_configs.sh)
    import io
    import contextlib

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gal = tn.gallery_features()
    torch.cuda.synchronize()
    t_gal = time.perf_counter() - t0
    plans = [tn.myEpisodeDataloader.get_episode_plan() for _ in range(args.episodes)]
    B = args.batch
    tn._aug_batch(plans[:B], gal)  # warmup
    bb = tn.mymodel.native(224, 224)
    torch.cuda.synchronize()
    bb.profile(True)
    t0 = time.perf_counter()
    preds = []
    for b0 in range(0, len(plans), B):
        preds += tn._aug_batch(plans[b0:b0 + B], gal)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms, fl, nl = bb.profile_read()
    bb.profile(False)
    conv_ms = float(ms.sum())
    peak = {"f32": 157.3, "bf16": 2516.6, "f32x3": round(2516.6 / 3, 1)}[args.dtype]
    achieved = float(fl.sum()) / (conv_ms * 1e-3) / 1e12
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": None,
                "kernel": f"conv family: {int(nl.sum())} conv launches of the timed region, summed algorithmic "
                          "FLOPs / summed HIP-event durations",
                "conv_share_of_wall": round(conv_ms * 1e-3 / el, 3)}
    cpu = parity = None
    if args.cpu_episodes:
        cpu, parity = c3_cpu_baseline(tn, gal, plans[:args.cpu_episodes], preds[:args.cpu_episodes])
    acc = float(np.mean([p == q["query_y"] for p, q in zip(preds, plans)]))
    # like-for-like traffic (tools/gpu_traffic.sh, tools/traffic_json.py): the timed region's conv
    # launches, their algorithmic bytes per launch (bench.py's formula; frames from the stem's FLOPs)
    sys.path.insert(0, REPO)
    import bench as bench_mod
    stem_flops = 2.0 * 112 * 112 * 64 * 147
    frames_timed = int(round(float(fl[0]) / stem_flops))
    roofline["conv_launches"] = int(nl.sum())
    roofline["traffic_key"] = C3_KEY
    roofline["traffic_algorithmic"] = round(bench_mod.algorithmic_bytes_per_launch(
        argparse.Namespace(arch="resnet50", res=224), arch, args.dtype, frames_timed, (ms, fl, nl)))
    tr, roofline["traffic_source"] = bench_mod.measured_traffic(args.dtype, C3_KEY)
    roofline["traffic"] = tr["hbm_bytes_per_launch"] if tr else None
    if tr:
        roofline["traffic_profiled_run"] = {k: tr[k] for k in ("launches", "hbm_bytes_per_launch",
                                                                "algorithmic_bytes_per_launch", "ratio") if k in tr}
    roofline["traffic_unit"] = "HBM bytes per conv launch (PMC)"
    reforward = os.environ.get("EOSV_AUG_REFORWARD", "0") == "1"
    # backbone frames per episode: query (<=16) + 5 supports x 16 (+ 40 augmented clips x 16 when
    # they are re-forwarded as the reference does; by default their features are gathered)
    frames_ep = 16 + 5 * 16 + (40 * 16 if reforward else 0)
    gflop = 2 * arch.conv_macs_per_frame(arch.SPECS["resnet50"]) / 1e9
    fps = round(args.episodes * frames_ep / el, 1)
    return {"metric": "config-3 backbone frames/s (aug_seg_T 5-way 1-shot, R50, 224x224)",
            # the work rate: frames that go through the backbone (the 40 augmented clips per episode are
            # assembled from already-computed frame features unless EOSV_AUG_REFORWARD=1)
            "value": fps, "unit": "backbone frames/s",
            "config": "3: test_network_aug_segment aug_seg_T 5w1s R50 224 (drop-in TestNetwork)",
            "dtype": args.dtype, "aug_features": "reforward" if reforward else "gathered",
            "episodes": args.episodes, "batch": B, "episodes_per_s": round(args.episodes / el, 2),
            "clips_per_s": round(args.episodes * 46 / el, 1),
            "clips_per_s_note": "46 clips per episode (5 supports + 40 augmented + 1 query); only "
                                f"{frames_ep} frames per episode go through the backbone",
            "backbone_frames_per_episode": frames_ep, "backbone_frames_per_s": fps,
            "end_to_end_tflops": round(args.episodes * frames_ep * gflop / el / 1e3, 1),
            "gallery_s": round(t_gal, 3), "gallery_frames": 10240, "episode_acc": acc,
            "roofline": roofline, "cpu_baseline": cpu, "cpu_parity": parity}


def c3_cpu_baseline(tn, gal, plans, gpu_preds):
    """The oracle's aug_seg_T episode (oracle/harness_ref.aug_segment_episode, torch-CPU fp32
    restatement of network_test.py:195-259) on the box's host cores, per episode, with the gallery
    segment features handed over from the GPU run (the gallery is built once per run, outside the
    per-episode loop, on both sides) and gallery frames generated on demand.  Also reports whether
    the oracle's predictions equal the GPU leg's on those episodes."""
    sys.path.insert(0, REPO)
    import numpy as np
    import torch

    import generate_augmented_datasets as gad
    from eosv import arch, synth
    from oracle import harness_ref, resnet_ref

    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", 10 ** 6)))
    torch.set_num_threads(threads)
    model = resnet_ref.build_model("resnet50", {k: v.detach().cpu().numpy() for k, v in tn.mymodel.state_dict().items()})
    infos = gad.gallery_video_infos()

    t_synth = [0.0]  # frame synthesis time, excluded from the CPU time (as bench.py's C2 baseline)

    class GallerySegments:  # [G, seg_len, 3, H, W], generated when indexed
        def __getitem__(self, g):
            t0 = time.perf_counter()
            vi = infos[(2 * g) // 16 % len(infos)]
            ids, _ = synth.clip_frame_ids(vi, 16)
            f0 = (2 * g) % 16
            out = torch.from_numpy(synth.synth_video(vi.split("/")[0], vi, ids[f0:f0 + 2], 224, 224))
            t_synth[0] += time.perf_counter() - t0
            return out

    def load(vi, support):
        t0 = time.perf_counter()
        ids, n_all = synth.clip_frame_ids(vi, 16)
        v = torch.from_numpy(synth.synth_video(vi.split("/")[0], vi, ids, 224, 224))
        if support and v.shape[0] < 16:
            v = torch.cat([v, torch.zeros(16 - v.shape[0], 3, 224, 224)])
        t_synth[0] += time.perf_counter() - t0
        return v, v.shape[0]

    g = gal.cpu().numpy()
    t = 0.0
    equal = 0
    for p, gp in zip(plans, gpu_preds):
        t0 = time.perf_counter()
        r = harness_ref.aug_segment_episode(model, p, load, g, GallerySegments(), len(set(p["support_y"])),
                                            len(p["support"]) // len(set(p["support_y"])))
        t += time.perf_counter() - t0
        equal += int(int(r["pred"][0]) == int(gp))
        print(f"c3 cpu_baseline: {equal} of the episodes so far equal, {t:.0f}s", file=sys.stderr, flush=True)
    t -= t_synth[0]
    n = len(plans)
    # the same unit as the line's value (backbone frames/s); the oracle, as the reference, forwards
    # 736 frames per episode (the GPU path 96: it gathers the augmented clips' features), so the
    # like-for-like rate of the two is episodes_per_s, reported beside it
    base = {"value": round(n * (16 + 5 * 16 + 40 * 16) / t, 2), "unit": "backbone frames/s", "cores": threads,
            "kind": "port", "episodes_per_s": round(n / t, 4),
            "sample": f"{n} aug_seg_T episodes through oracle/harness_ref.aug_segment_episode (R50 fp32 torch-CPU, "
                      f"the reference's 736 backbone frames per episode, gallery features from the GPU run, "
                      f"frame synthesis excluded ({t_synth[0]:.1f}s of it), like the configs-1/2/4/5 baselines); {t:.1f}s"}
    parity = {"episodes": n, "pred_equal": equal, "against": "the GPU leg's predictions on the same episodes"}
    return base, parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--episodes", type=int, default=0, help="per step (default: 64 config 3, 40 config 4, 8 config 5)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5, help="configs 4 / 5: timed steps of --episodes episodes")
    ap.add_argument("--cpu-episodes", type=int, default=2, help="config 3: oracle episodes for cpu_baseline (0: none)")
    ap.add_argument("--max-frames", type=int, default=0, help="backbone chunk (default: 4096 config 3, 2048 configs 4 / 5)")
    ap.add_argument("--cpu-sec", type=float, default=10.0,
                    help="configs 4 / 5: seconds of oracle CPU time for cpu_baseline / cpu_parity (bench.py "
                         "--cpu-baseline-sec); C4 needs ~6 s per episode on 16 cores")
    ap.add_argument("--parity-dump", default=None, help="configs 4 / 5: bench.py --parity-dump")
    ap.add_argument("--secondary", default="", help="configs 4 / 5: bench.py --secondary-dtype")
    args = ap.parse_args()
    args.episodes = args.episodes or {3: 64, 4: 40, 5: 8}[args.config]
    if args.config == 3:
        print(json.dumps(config3(args)), flush=True)
        return
    # config 4 samples the UnrealAction-shaped split (14 classes x 10 videos, tests/golden/unreal14.list)
    shape = {4: ["--arch", "resnet50", "--n-way", "14", "--k-shot", "1", "--segments", "16",
                 "--list", os.path.join(REPO, "tests", "golden", "unreal14.list")],
             5: ["--arch", "resnet101", "--n-way", "5", "--k-shot", "5", "--segments", "32", "--res", "256"]}[args.config]
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), *shape, "--dtype", args.dtype,
           "--episodes-per-step", str(args.episodes), "--steps", str(args.steps), "--secondary-dtype", args.secondary,
           *(["--parity-dump", args.parity_dump] if args.parity_dump else []),
           "--cpu-baseline-sec", str(args.cpu_sec),
           "--max-frames", str(args.max_frames or 2048), "--config-label", f"BASELINE configs[{args.config - 1}]"]
    sys.exit(subprocess.call(cmd))


if __name__ == "__main__":
    main()
