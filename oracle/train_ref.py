"""CPU restatement of the reference's training loop (test infrastructure only).

``TrainNetwork.finetune_model`` (reference network_train.py:52-131) on recorded batches:

    optimizer_1 = SGD(convnet, lr_1, momentum=0.9); optimizer_2 = SGD(fc, lr_2, momentum=0.9)  # :75-76
    scheduler_i = StepLR(optimizer_i, step_size, gamma=0.1)                                     # :77-78
    for epoch: scheduler_1.step(); scheduler_2.step()                                          # :82-84
        for batch: feature, _ = model(video.view(-1, 3, H, W))                                 # :90, :99
                   feature = feature.view(b, T, -1).mean(dim=1); output = model.fc(feature)    # :100-112
                   loss = CrossEntropyLoss()(output, label); loss.backward(); step both        # :79, :113-116

The model is ``oracle.resnet_ref.ModelResNetRef`` (torchvision's structure, the reference's
state_dict keys).  Frames of a recorded clip are regenerated with ``eosv.synth.synth_frame``,
the generator the capture's ToTensor stub used (tests/golden/capture_golden.py).  Pinned by
``tests/golden/train_*.json``, captured by running the reference's own loop
(``capture_golden.py --train``); checked in ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from eosv import synth

from .resnet_ref import ModelResNetRef


def clip_frames(clip, H, W):
    """[n, 3, H, W] f32 frames start .. start + n - 1 of a recorded clip (utils.py:108-124)."""
    vi = clip["video"]
    cls = vi.split("/")[0]
    return torch.from_numpy(np.stack([synth.synth_frame(cls, vi, clip["start"] + i, H, W)
                                      for i in range(clip["n"])]))


def batch_frames(it, H, W):
    """The model's input for one recorded iteration: clips stacked, then view(-1, 3, H, W)."""
    return torch.cat([clip_frames(c, H, W) for c in it["clips"]], 0)


def train_replay(meta, state_dict, dtype=torch.float64):
    """Run the reference's loop over the fixture's batches.  Returns (losses, [state_dict after
    each epoch]) -- the checkpoints of network_train.py:130-131."""
    m = ModelResNetRef(meta["arch"], meta["num_classes"])
    m.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()})
    m = m.to(dtype).train()
    o1 = torch.optim.SGD(m.convnet.parameters(), lr=meta["lr_1"], momentum=0.9)
    o2 = torch.optim.SGD(m.fc.parameters(), lr=meta["lr_2"], momentum=0.9)
    s1 = torch.optim.lr_scheduler.StepLR(o1, step_size=meta["step_size"], gamma=0.1)
    s2 = torch.optim.lr_scheduler.StepLR(o2, step_size=meta["step_size"], gamma=0.1)
    crit = torch.nn.CrossEntropyLoss()
    losses, states = [], []
    T, H, W = meta["T"], meta["H"], meta["W"]
    for ep in meta["epochs_data"]:
        with warnings.catch_warnings():  # the reference steps the schedulers first (:83-84)
            warnings.simplefilter("ignore")
            s1.step()
            s2.step()
        for it in ep["iterations"]:
            video = batch_frames(it, H, W).to(dtype)
            o1.zero_grad()
            o2.zero_grad()
            feature, _ = m(video)
            feature = feature.view(len(it["clips"]), T, -1).mean(dim=1)
            out = m.fc(feature)
            loss = crit(out, torch.as_tensor(it["labels"], dtype=torch.long))
            loss.backward()
            o1.step()
            o2.step()
            losses.append(float(loss.detach()))
        states.append({k: v.detach().clone() for k, v in m.state_dict().items()})
    return losses, states


def tensor_stats(t, i):
    """The fixture's per-tensor summary (capture_golden._tensor_stats): sum, norm, projection onto
    numpy default_rng(2000 + i) N(0,1)."""
    a = torch.as_tensor(t).detach().double().numpy().reshape(-1)
    r = np.random.default_rng(2000 + i).standard_normal(a.shape)
    return dict(sum=float(a.sum()), norm=float(np.sqrt((a * a).sum())), proj=float((a * r).sum()))


def projections(t, i, n=8):
    """The fixture's n projections of tensor i (capture_golden._projections): onto numpy
    default_rng(3000 + 8 i + j) N(0,1), j < n."""
    a = torch.as_tensor(t).detach().double().numpy().reshape(-1)
    return [float((a * np.random.default_rng(3000 + 8 * i + j).standard_normal(a.shape)).sum()) for j in range(n)]
