"""Which op of the reference's training loop amplifies a rounding perturbation.

The R50 reference-fixture training test (tests/test_gpu_train.py::test_train_loop_matches_reference
_fixture) bounds the native loss at each step by max(4 x the reference f32 run's distance from
the f64 replay, 1e-4 relative).  Round 5's 4-slice split-K sizing (more accurate per conv) missed it
at epoch 1 step 5.  This tool replays the fixture's batches with oracle/train_ref.py in f64 and
evaluates ONE op class in f32 at a time -- the convolutions (forward and backward: the GEMMs), the
batch norms (statistics, normalisation and their backward), or the fc + loss -- and prints each
step's |loss - f64 loss| next to the all-f32 run's (the reference's own distance).  The op class
whose f32 rounding alone moves the loss as far as the whole f32 run is where a changed reduction
order gets amplified.  CPU only (test infrastructure: it runs the oracle, nothing is timed).

  python tools/train_sensitivity.py [train_r50_t8_96] [threads]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
sys.path.insert(0, REPO)
from eosv import arch, synth  # noqa: E402
from oracle import train_ref  # noqa: E402

_conv_fwd = torch.nn.Conv2d._conv_forward
_bn_fwd = torch.nn.BatchNorm2d.forward
_lin_fwd = torch.nn.Linear.forward


def conv_f32(self, x, w, b):
    return _conv_fwd(self, x.float(), w.float(), None if b is None else b.float()).to(x.dtype)


def bn_f32(self, x):
    # train mode: batch statistics in f32; the f64 running buffers are left alone (the losses of
    # the replay do not read them)
    return F.batch_norm(x.float(), None, None, self.weight.float(), self.bias.float(), True, 0.0, self.eps).to(x.dtype)


def lin_f32(self, x):
    return F.linear(x.float(), self.weight.float(), None if self.bias is None else self.bias.float()).to(x.dtype)


def run(meta, sd0, dtype, patch):
    torch.nn.Conv2d._conv_forward, torch.nn.BatchNorm2d.forward, torch.nn.Linear.forward = _conv_fwd, _bn_fwd, _lin_fwd
    if patch == "conv":
        torch.nn.Conv2d._conv_forward = conv_f32
    elif patch == "bn":
        torch.nn.BatchNorm2d.forward = bn_f32
    elif patch == "fc":
        torch.nn.Linear.forward = lin_f32
    try:
        losses, _ = train_ref.train_replay(meta, sd0, dtype)
    finally:
        torch.nn.Conv2d._conv_forward, torch.nn.BatchNorm2d.forward, torch.nn.Linear.forward = _conv_fwd, _bn_fwd, _lin_fwd
    return losses


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "train_r50_t8_96"
    torch.set_num_threads(int(sys.argv[2]) if len(sys.argv) > 2 else 8)
    meta = json.load(open(os.path.join(REPO, "tests", "golden", tag + ".json")))
    sd0 = synth.synth_state_dict(arch.SPECS[meta["arch"]], meta["num_classes"], meta["init_seed"])
    ref = [it["loss"] for ep in meta["epochs_data"] for it in ep["iterations"]]
    truth = run(meta, sd0, torch.float64, None)
    rows = {"reference f32 (fixture)": ref, "all f32 (oracle)": run(meta, sd0, torch.float32, None)}
    for p, name in (("conv", "convs in f32"), ("bn", "batch norms in f32"), ("fc", "fc + loss input in f32")):
        rows[name] = run(meta, sd0, torch.float64, p)
    out = {"tag": tag, "f64_losses": truth, "abs_err_vs_f64": {}}
    print(f"{tag}: |loss - f64 replay| per step (epoch-major)")
    for name, ls in rows.items():
        err = [abs(a - b) for a, b in zip(ls, truth)]
        out["abs_err_vs_f64"][name] = err
        print(f"  {name:28s} " + " ".join(f"{e:.2e}" for e in err))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
