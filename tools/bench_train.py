#!/usr/bin/env python3
"""Training-step throughput: the reference's finetune recipe
(network_train.py:140: ResNet-50, batch 6 clips x 16 frames at 224x224, SGD momentum) on
synthetic frames, through eosv.train.NativeTrainer.  Prints one JSON line: clips/s, frames/s,
ms/step and the conv FLOP rate (forward + input gradient + weight gradient = 3 x the forward
conv FLOPs, the stem's input gradient excluded) against the f32 MFMA peak; with --cpu-steps, the
same step on torch-CPU (the oracle model, f32) for a CPU baseline.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from eosv import arch, synth  # noqa: E402
from eosv.train import NativeTrainer  # noqa: E402

GFLOP_FWD = {"resnet18": 3.6271, "resnet50": 8.1743}  # per 224x224 frame


def measure(arch_name="resnet50", batch=6, frames_per_clip=16, res=224, steps=5, warmup=1, device=0):
    """One NativeTrainer on synthetic frames: warmup steps, then `steps` timed steps (synchronised
    on both sides).  Returns the JSON dict, plus the state dict, frames and labels for the CPU leg."""
    sd = synth.synth_state_dict(arch.SPECS[arch_name], 64, 0)
    tr = NativeTrainer(arch_name, 64, device=device)
    tr.load_state_dict(sd)
    g = torch.Generator().manual_seed(0)
    frames = torch.randn(batch * frames_per_clip, 3, res, res, generator=g).cuda(device)
    labels = np.arange(batch) % 64
    for _ in range(warmup):
        tr.step(frames, labels, frames_per_clip, 1e-4, 1e-3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss, _ = tr.step(frames, labels, frames_per_clip, 1e-4, 1e-3)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    nf = batch * frames_per_clip
    flops = 3 * GFLOP_FWD[arch_name] * 1e9 * (res / 224.0) ** 2 * nf
    out = {"metric": "training clips/s (network_train.py finetune step)", "arch": arch_name, "batch": batch,
           "frames_per_clip": frames_per_clip, "res": res, "dtype": "f32", "clips_per_s": round(batch / dt, 2),
           "frames_per_s": round(nf / dt, 1), "ms_per_step": round(dt * 1e3, 2), "steps": steps, "warmup": warmup,
           "loss": round(loss, 4), "conv_tflops": round(flops / dt / 1e12, 2),
           "conv_frac_f32_peak": round(flops / dt / 157.3e12, 4),
           "data": "synthetic frames, random-init weights of the reference architecture"}
    return out, sd, frames, labels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=6)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--res", type=int, default=224)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-steps", type=int, default=0)
    a = ap.parse_args()
    out, sd, frames, labels = measure(a.arch, a.batch, a.frames, a.res, a.steps, a.warmup)
    if a.cpu_steps:
        from oracle.resnet_ref import ModelResNetRef

        torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
        m = ModelResNetRef(a.arch, 64)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        m.train()
        o1 = torch.optim.SGD(m.convnet.parameters(), lr=1e-4, momentum=0.9)
        o2 = torch.optim.SGD(m.fc.parameters(), lr=1e-3, momentum=0.9)
        x = frames.cpu()
        lab = torch.as_tensor(labels, dtype=torch.long)
        t0 = time.perf_counter()
        for _ in range(a.cpu_steps):
            o1.zero_grad()
            o2.zero_grad()
            f, _ = m(x)
            torch.nn.CrossEntropyLoss()(m.fc(f.view(a.batch, a.frames, -1).mean(1)), lab).backward()
            o1.step()
            o2.step()
        cdt = (time.perf_counter() - t0) / a.cpu_steps
        out["cpu_baseline"] = {"clips_per_s": round(a.batch / cdt, 3), "cores": torch.get_num_threads(),
                               "kind": "port", "sample": f"{a.cpu_steps} steps of the same batch, torch-CPU f32"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
