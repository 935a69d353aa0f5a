"""Shared test helpers: load golden fixtures, synthesize the reference's inputs."""
import json
import os

import numpy as np
import torch

from eosv import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(tag):
    with open(os.path.join(GOLDEN, tag + ".json")) as f:
        meta = json.load(f)
    npz = os.path.join(GOLDEN, tag + ".npz")
    arrays = dict(np.load(npz)) if os.path.exists(npz) else {}
    return meta, arrays


def load_video(video_info, support, T=16, H=224, W=224):
    """Frames the reference loader hands over (utils.py:96-136 query / 215-258 support)."""
    ids, n_all = synth.clip_frame_ids(video_info, T)
    cls = video_info.split("/")[0]
    v = torch.from_numpy(synth.synth_video(cls, video_info, ids, H, W))
    if support:
        n = min(T, n_all)
        if v.shape[0] < T:
            v = torch.cat([v, torch.zeros(T - v.shape[0], 3, H, W)])
        return v, n
    return v, v.shape[0]
