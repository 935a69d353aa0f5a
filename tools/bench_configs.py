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
    tn.mymodel.max_frames = 1024
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
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    preds = []
    for b0 in range(0, len(plans), B):
        preds += tn._aug_batch(plans[b0:b0 + B], gal)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    acc = float(np.mean([p == q["query_y"] for p, q in zip(preds, plans)]))
    reforward = os.environ.get("EOSV_AUG_REFORWARD", "0") == "1"
    # backbone frames per episode: query (<=16) + 5 supports x 16 (+ 40 augmented clips x 16 when
    # they are re-forwarded as the reference does; by default their features are gathered)
    frames_ep = 16 + 5 * 16 + (40 * 16 if reforward else 0)
    gflop = 2 * arch.conv_macs_per_frame(arch.SPECS["resnet50"]) / 1e9
    return {"config": "3: test_network_aug_segment aug_seg_T 5w1s R50 224 (drop-in TestNetwork)",
            "dtype": args.dtype, "aug_features": "reforward" if reforward else "gathered",
            "episodes": args.episodes, "batch": B, "episodes_per_s": round(args.episodes / el, 2),
            "clips_per_s": round(args.episodes * 46 / el, 1),
            "backbone_frames_per_episode": frames_ep, "backbone_frames_per_s": round(args.episodes * frames_ep / el, 1),
            "end_to_end_tflops": round(args.episodes * frames_ep * gflop / el / 1e3, 1),
            "gallery_s": round(t_gal, 3), "gallery_frames": 10240, "episode_acc": acc}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--episodes", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-frames", type=int, default=2048, help="backbone chunk (configs 4 / 5)")
    args = ap.parse_args()
    if args.config == 3:
        print(json.dumps(config3(args)), flush=True)
        return
    shape = {4: ["--arch", "resnet50", "--n-way", "14", "--k-shot", "1", "--segments", "16"],
             5: ["--arch", "resnet101", "--n-way", "5", "--k-shot", "5", "--segments", "32", "--res", "256"]}[args.config]
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), *shape, "--dtype", args.dtype,
           "--episodes-per-step", str(args.episodes), "--steps", "2", "--no-cpu-baseline", "--secondary-dtype", "",
           "--max-frames", str(args.max_frames), "--config-label", f"BASELINE configs[{args.config - 1}]"]
    sys.exit(subprocess.call(cmd))


if __name__ == "__main__":
    main()
