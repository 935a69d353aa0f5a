"""Frame sources behind the reference's loaders (utils.py:80-136, 171-258).

The reference reads ``<frame_dir>/<class>/<video>/image_%05d.jpg`` with PIL, resizes
frames narrower than 224 px to 224x256, centre-crops 224 (test) or random-crops +
flips (train), applies ToTensor and ImageNet Normalize.  The frame *indexing* (start
frame, early stop, zero padding, returned count) is shared by every source here and
restated once in :func:`clip_frame_ids`.

Sources:
  * ``JpegFrames``  -- the on-disk layout above (host JPEG decode, GPU crop + normalise;
    SURVEY 8(f1)).
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

    def frames_tensor(self, video_info: str, ids: List[int], mode: str) -> torch.Tensor:
        """frames() as a tensor (a device tensor where the source produces it on the GPU)."""
        return torch.from_numpy(self.frames(video_info, ids, mode))

    def video(self, video_info: str, T: int, mode: str, pad: bool) -> Tuple[torch.Tensor, int]:
        """Reference loader semantics: (tensor, real frame count).

        pad=False: get_video_from_video_info (<= T frames, utils.py:96-136).
        pad=True:  get_video_from_video_info_3 (zero-padded to T, count = min(T, all),
                   utils.py:215-258).
        """
        n_all = self.frame_count(video_info)
        ids = clip_frame_ids(n_all, T, mode)
        v = self.frames_tensor(video_info, ids, mode)
        if pad:
            if v.shape[0] < T:
                v = torch.cat([v, torch.zeros((T - v.shape[0],) + tuple(v.shape[1:]), dtype=v.dtype,
                                              device=v.device)])
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
    """``<frame_dir>/<class>/<video>/image_%05d.jpg``.  JPEG decode and the
    narrow-frame resize stay on the host (PIL, as the reference); crop, flip, ToTensor and
    Normalize run on the GPU (eosv_crop_normalize_frames) over the clip's uint8 frames, so
    ``video()`` returns a device tensor.  Needs libeosv and a HIP device like every product call."""

    def __init__(self, frame_dir: str, crop: int = 224, init_h: int = 256):
        self.frame_dir, self.crop, self.init_h = frame_dir, crop, init_h

    def frame_count(self, video_info: str) -> int:
        return len(os.listdir(os.path.join(self.frame_dir, video_info))) - 1

    def _path(self, video_info: str, f: int) -> str:
        return os.path.join(self.frame_dir, video_info, "image_%05d.jpg" % f)

    def decode(self, path: str) -> np.ndarray:
        """[h,w,3] uint8 RGB after the reference's resize of frames narrower than the crop."""
        from PIL import Image

        img = Image.open(path).convert("RGB")
        if img.size[0] < self.crop:  # utils.py:123-124 (ANTIALIAS == LANCZOS)
            img = img.resize((self.crop, self.init_h), Image.LANCZOS)
        return np.asarray(img)

    def window(self, first: np.ndarray, mode: str):
        """(crop_ij or None for centre, flip), drawing from the RNGs in the reference's order:
        ClipRandomHorizontalFlip draws random.random() when transforms() is built, then
        ClipRandomCrop.get_params draws torch.randint for i, j on the clip's first frame
        (torchvision draws nothing when the frame is exactly crop-sized)."""
        if mode != "train":
            return None, False
        flip = _random.random() < 0.5
        h, w = first.shape[:2]
        c = self.crop
        if h == c and w == c:
            return (0, 0), flip
        i = int(torch.randint(0, h - c + 1, size=(1,)).item())
        j = int(torch.randint(0, w - c + 1, size=(1,)).item())
        return (i, j), flip

    def frames_tensor(self, video_info, ids, mode):
        from . import engine

        raw = [self.decode(self._path(video_info, f)) for f in ids]
        crop_ij, flip = self.window(raw[0], mode)
        c = self.crop
        out = torch.empty(len(raw), 3, c, c, dtype=torch.float32, device="cuda")
        k = 0
        while k < len(raw):  # runs of equally sized frames share one upload and one launch
            e = k + 1
            while e < len(raw) and raw[e].shape == raw[k].shape:
                e += 1
            h, w = raw[k].shape[:2]
            if crop_ij is None:  # torchvision CenterCrop
                top, left = int(round((h - c) / 2.0)), int(round((w - c) / 2.0))
            else:
                top, left = crop_ij
            rgb = torch.from_numpy(np.ascontiguousarray(np.stack(raw[k:e]))).cuda()
            out[k:e] = engine.crop_normalize_frames(rgb, c, top, left, flip)
            k = e
        return out

    def frames(self, video_info, ids, mode):
        return self.frames_tensor(video_info, ids, mode).cpu().numpy()


def default_source(frame_dir: str, H: int = 224, W: int = 224) -> FrameSource:
    """Real frames when the directory exists (or EOSV_FRAMES=jpeg), else synthetic."""
    mode = os.environ.get("EOSV_FRAMES", "auto")
    if mode == "jpeg" or (mode == "auto" and os.path.isdir(frame_dir)):
        return JpegFrames(frame_dir, crop=H)
    return SyntheticFrames(H, W)
