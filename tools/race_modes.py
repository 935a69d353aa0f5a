"""Features of repeated forwards under EOSV_POISON modes (profiling build), interleaved: which
runs agree bitwise with which.  A run-to-run difference inside one mode is a race; modes that
agree within themselves but not with each other point at what the mode changes.
  python tools/race_modes.py [arch] [dtype] [frames,...] [modes,...] [reps]"""
import hashlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
from eosv import arch, engine, synth  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16"
counts = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "64,130").split(",")]
modes = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "0,4").split(",")]
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 4
sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
bb = engine.Backbone(name, dtype, 224, 224, max_frames=max(counts))
bb.load_state_dict(sd)
for nf in counts:
    x = torch.randn(nf, 3, 224, 224, generator=torch.Generator().manual_seed(nf)).cuda()
    seen = {}
    rows = {m: [] for m in modes}
    for r in range(reps):
        for m in modes:
            os.environ["EOSV_POISON"] = str(m)
            f = bb.forward(x)
            torch.cuda.synchronize()
            os.environ["EOSV_POISON"] = "0"
            h = hashlib.sha1(f.cpu().numpy().tobytes()).hexdigest()[:8]
            if h not in seen:
                seen[h] = (len(seen), f.clone())
            rows[m].append(seen[h][0])
    base = next(v[1] for v in seen.values() if v[0] == 0)
    for h, (i, f) in seen.items():
        if i:
            bad = torch.nonzero((f != base).any(1)).flatten().tolist()
            print(f"  variant {i}: frames differing from variant 0: {bad[:16]}{'...' if len(bad) > 16 else ''}")
    print(f"{name} {dtype} frames {nf}: " + "; ".join(f"mode {m}: {rows[m]}" for m in modes), flush=True)
bb.close()
