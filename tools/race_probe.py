"""Repeat the backbone on identical inputs and report, per stage, how many runs differ bitwise
from the first (an LDS / DMA ordering race shows up as run-to-run differences; every kernel is
deterministic otherwise).  usage: python tools/race_probe.py [arch] [dtype] [reps] [frames]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
from eosv import arch, engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
nf = int(sys.argv[4]) if len(sys.argv) > 4 else 37
sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
x = torch.randn(nf, 3, 224, 224, generator=torch.Generator().manual_seed(5)).cuda()
bb = engine.Backbone(name, dtype, 224, 224, max_frames=nf)
bb.load_state_dict(sd)
for stage in range(5):
    ref = bb.probe(x, stage)
    bad = 0
    worst = 0.0
    frames = set()
    outs = []
    for _ in range(reps):
        o = bb.probe(x, stage)
        outs.append(o)
        if not torch.equal(o, ref):
            bad += 1
            d = (o - ref).abs()
            worst = max(worst, float(d.max()))
            frames |= set(torch.nonzero(d.flatten(1).amax(1)).flatten().tolist())
    distinct = len({hash(o.cpu().numpy().tobytes()) for o in [ref] + outs})
    print(f"{name} {dtype} stage {stage}: {bad}/{reps} runs differ, {distinct} distinct, max |d| {worst:.3g}, "
          f"frames {sorted(frames)[:12]}", flush=True)
    if bad:
        o = next(o for o in outs if not torch.equal(o, ref))
        d = (o - ref).abs()  # [B, h, w, C]
        f = int(torch.nonzero(d.flatten(1).amax(1)).flatten()[0])
        nz = torch.nonzero(d[f])
        print(f"   frame {f}: {nz.shape[0]} elements differ; rows {nz[:, 0].unique().tolist()} cols "
              f"{nz[:, 1].unique().tolist()[:16]} channels {nz[:, 2].min().item()}..{nz[:, 2].max().item()} "
              f"({nz[:, 2].unique().numel()} distinct)", flush=True)
        # a 5-frame batch of the tail frames
        t = bb.probe(x[nf - 5:nf].contiguous(), stage)
        print(f"   tail-only batch vs ref: {'equal' if torch.equal(t, ref[nf - 5:nf]) else 'differs'}; "
              f"vs first runs: {[torch.equal(t, o[nf - 5:nf]) for o in outs[:4]]}", flush=True)
ref = bb.forward(x)
bad = sum(0 if torch.equal(bb.forward(x), ref) else 1 for _ in range(reps))
print(f"{name} {dtype} forward: {bad}/{reps} runs differ", flush=True)
bb.close()
