"""Frame sources behind the reference's loaders (utils.py:80-136, 171-258).

The reference reads ``<frame_dir>/<class>/<video>/image_%05d.jpg`` with PIL, resizes
frames narrower than 224 px to 224x256, centre-crops 224 (test) or random-crops +
flips (train), applies ToTensor and ImageNet Normalize.  The frame *indexing* (start
frame, early stop, zero padding, returned count) is shared by every source here and
restated once in :func:`clip_frame_ids`.

Sources:
  * ``JpegFrames``  -- the on-disk layout above (host decode).
  * ``SyntheticFrames`` -- the deterministic generator of eosv/synth.py, used when no
    frame directory exists (this offline image).  Its frames can also be produced
    directly in HBM (eosv_synth_frames), which the batched episode path uses.
"""
from __future__ import annotations

import os
import random as _random
from typing import List, Tuple

import numpy as np
import torch

from . import synth

MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def clip_start(all_frames: int, T: int, mode: str, rnd=_random) -> int:
    """utils.py:105-112 (train draws from the global RNG like the reference)."""
    if all_frames - T - 1 > 1:
        if mode == "train":
            return rnd.randint(1, all_frames - T - 1)
        return all_frames // 2 - T // 2 + 1
    return 1


def clip_frame_ids(all_frames: int, T: int, mode: str, rnd=_random) -> List[int]:
    """Frame ids read by get_video_from_video_info (utils.py:114-131): stop after T or the last frame."""
    fid = clip_start(all_frames, T, mode, rnd)
    ids = []
    for _ in range(T):
        ids.append(fid)
        fid += 1
        if fid > all_frames:
            break
    return ids


class FrameSource:
    synthetic = False

    def frame_count(self, video_info: str) -> int:
        raise NotImplementedError

    def frames(self, video_info: str, ids: List[int], mode: str) -> np.ndarray:
        """[len(ids),3,H,W] f32 normalised frames."""
        raise NotImplementedError

    def video(self, video_info: str, T: int, mode: str, pad: bool) -> Tuple[torch.Tensor, int]:
        """Reference loader semantics: (tensor, real frame count).

        pad=False: get_video_from_video_info (<= T frames, utils.py:96-136).
        pad=True:  get_video_from_video_info_3 (zero-padded to T, count = min(T, all),
                   utils.py:215-258).
        """
        n_all = self.frame_count(video_info)
        ids = clip_frame_ids(n_all, T, mode)
        v = torch.from_numpy(self.frames(video_info, ids, mode))
        if pad:
            if v.shape[0] < T:
                v = torch.cat([v, torch.zeros((T - v.shape[0],) + tuple(v.shape[1:]), dtype=v.dtype)])
            return v, int(min(T, n_all))
        return v, v.shape[0]


class SyntheticFrames(FrameSource):
    synthetic = True

    def __init__(self, H: int = 224, W: int = 224):
        self.H, self.W = H, W

    def frame_count(self, video_info: str) -> int:
        return synth.frame_count(video_info)

    def frames(self, video_info, ids, mode):
        cls = video_info.split("/")[0]
        return synth.synth_video(cls, video_info, ids, self.H, self.W).reshape(len(ids), 3, self.H, self.W)


class JpegFrames(FrameSource):
    def __init__(self, frame_dir: str, crop: int = 224, init_h: int = 256):
        self.frame_dir, self.crop, self.init_h = frame_dir, crop, init_h

    def frame_count(self, video_info: str) -> int:
        return len(os.listdir(os.path.join(self.frame_dir, video_info))) - 1

    def _load(self, path: str, mode: str, crop_ij, flip: bool) -> np.ndarray:
        from PIL import Image

        img = Image.open(path).convert("RGB")
        if img.size[0] < self.crop:  # utils.py:123-124 (ANTIALIAS == LANCZOS)
            img = img.resize((self.crop, self.init_h), Image.LANCZOS)
        a = np.asarray(img)  # H,W,3 uint8
        h, w = a.shape[:2]
        c = self.crop
        if crop_ij is None:  # torchvision CenterCrop
            i, j = int(round((h - c) / 2.0)), int(round((w - c) / 2.0))
        else:
            i, j = crop_ij
        a = a[i:i + c, j:j + c]
        if flip:
            a = a[:, ::-1]
        x = a.astype(np.float32) / np.float32(255.0)  # ToTensor
        x = (x - MEAN) / STD  # Normalize
        return np.ascontiguousarray(x.transpose(2, 0, 1))

    def frames(self, video_info, ids, mode):
        crop_ij, flip = None, False
        if mode == "train":  # ClipRandomCrop / ClipRandomHorizontalFlip (utils.py:57-78)
            from PIL import Image

            flip = _random.random() < 0.5
            p0 = os.path.join(self.frame_dir, video_info, "image_%05d.jpg" % ids[0])
            w, h = Image.open(p0).size
            crop_ij = (int(torch.randint(0, max(1, h - self.crop + 1), (1,))),
                       int(torch.randint(0, max(1, w - self.crop + 1), (1,))))
        out = [self._load(os.path.join(self.frame_dir, video_info, "image_%05d.jpg" % f), mode, crop_ij, flip)
               for f in ids]
        return np.stack(out)


def default_source(frame_dir: str, H: int = 224, W: int = 224) -> FrameSource:
    """Real frames when the directory exists (or EOSV_FRAMES=jpeg), else synthetic."""
    mode = os.environ.get("EOSV_FRAMES", "auto")
    if mode == "jpeg" or (mode == "auto" and os.path.isdir(frame_dir)):
        return JpegFrames(frame_dir, crop=H)
    return SyntheticFrames(H, W)
