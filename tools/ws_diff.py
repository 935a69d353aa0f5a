"""Per-stage backbone outputs under the current EOSV_* switches (profiling build), saved to a file,
or compared with an earlier save: locates the first stage where two kernel choices differ.
usage: python tools/ws_diff.py save out.pt [arch[:res]] [dtype] | python tools/ws_diff.py cmp a.pt b.pt"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))

if sys.argv[1] == "save":
    from eosv import arch, engine, synth  # noqa: E402
    name = sys.argv[3] if len(sys.argv) > 3 else "resnet50"  # arch, arch:res or arch:res:frames (e.g. resnet101:256)
    parts = name.split(":")
    name = parts[0]
    res = int(parts[1]) if len(parts) > 1 else 224
    nf = int(parts[2]) if len(parts) > 2 else 37
    dtype = sys.argv[4] if len(sys.argv) > 4 else "bf16"
    sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
    x = torch.randn(nf, 3, res, res, generator=torch.Generator().manual_seed(5)).cuda()
    bb = engine.Backbone(name, dtype, res, res, max_frames=nf)
    bb.load_state_dict(sd)
    outs = [bb.probe(x, s).float().cpu() for s in range(5)]
    torch.save(outs, sys.argv[2])
    bb.close()
else:
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for s, (u, v) in enumerate(zip(a, b)):
        d = (u - v).abs()
        nf = int((d.flatten(1).amax(1) > 0).sum())
        print(f"stage {s}: max |d| {float(d.max()):.4g} rel {float(d.max() / u.abs().max()):.3g}, frames differing {nf}/{u.shape[0]}")
        if nf:
            f = int(torch.nonzero(d.flatten(1).amax(1)).flatten()[0])
            nz = torch.nonzero(d[f])
            print(f"   frame {f}: {nz.shape[0]} of {d[f].numel()} differ; rows {nz[:, 0].unique().tolist()[:16]} "
                  f"cols {nz[:, 1].unique().tolist()[:16]} channels {nz[:, 2].unique().numel()} distinct")
