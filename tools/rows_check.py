"""A/B correctness for a conv-kernel env switch: dump backbone features (R18, R50; DTYPE env,
default bf16) for a few batch sizes in one process, compare two dumps in another (bitwise;
with TOL set, max relative difference <= TOL passes).

  EOSV_BF16_ROWS=1 python tools/rows_check.py dump gpurun_out/rows_1.npz
  EOSV_BF16_ROWS=2 python tools/rows_check.py dump gpurun_out/rows_2.npz
  python tools/rows_check.py compare gpurun_out/rows_1.npz gpurun_out/rows_2.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "embodied-one-shot-video-recognition_amd"))


def dump(path):
    import torch
    from eosv import arch, engine, synth
    out = {}
    for name in ("resnet18", "resnet50"):
        sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
        bb = engine.Backbone(name, os.environ.get("DTYPE", "bf16"), 224, 224, max_frames=300)
        bb.load_state_dict(sd)
        for n in (1, 19, 37, 300):
            x = torch.randn(n, 3, 224, 224, generator=torch.Generator().manual_seed(n)).cuda()
            out[f"{name}_{n}"] = bb.forward(x).float().cpu().numpy()
        bb.close()
    np.savez(path, **out)
    print("dumped", path, sorted(out))


def compare(a, b):
    da, db = np.load(a), np.load(b)
    bad = 0
    for k in sorted(da.files):
        same = np.array_equal(da[k].view(np.uint32), db[k].view(np.uint32))
        rel = np.abs(da[k] - db[k]).max() / max(np.abs(da[k]).max(), 1e-30)
        print(f"{k}: {'bit-identical' if same else 'DIFFERENT'} max rel {rel:.3g}")
        bad += not same and not (os.environ.get("TOL") and rel <= float(os.environ["TOL"]))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
