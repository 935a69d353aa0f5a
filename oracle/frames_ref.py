"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product): host restatement of
the reference's JPEG clip loaders for checking the GPU ingest path.

Follows /root/reference/utils.py:
  * transforms(mode)                 :80-91   (train: ClipRandomCrop, ClipRandomHorizontalFlip,
                                               ToTensor, Normalize; test/val: CenterCrop, ...)
  * ClipRandomCrop / ..HorizontalFlip :57-78   (flip drawn from `random` when the transform is
                                               built; crop window from torch.randint on the
                                               clip's first frame, torchvision get_params)
  * get_video_from_video_info_3       :215-258 (start frame, zero padding to T, count)
with PIL decode and numpy arithmetic in the same order as ToTensor (x / 255, f32) and
Normalize ((x - mean) / std, f32).  torchvision is absent here, so its CenterCrop rounding
(int(round((h - c) / 2.0))) and get_params are restated from its published source.
Parity of this restatement against the reference itself is unpinned (no JPEG fixtures ship
with the reference; its frame directories are not in the image).
"""
import os
import random

import numpy as np
import torch

MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def _to_normalized(a):
    x = a.astype(np.float32) / np.float32(255.0)
    return ((x - MEAN) / STD).transpose(2, 0, 1)


def load_clip_padded(frame_dir, video_info, mode, T=16, crop=224, init_h=256):
    """utils.py:215-258 -> ([T,3,crop,crop] f32 numpy, min(T, frame count))."""
    from PIL import Image

    path = os.path.join(frame_dir, video_info)
    n_all = len(os.listdir(path)) - 1
    if n_all - T - 1 > 1:
        start = random.randint(1, n_all - T - 1) if mode == "train" else n_all // 2 - T // 2 + 1
    else:
        start = 1
    flip = random.random() < 0.5 if mode == "train" else False  # utils.py:71-72 at transforms()
    ij = None
    out = []
    fid = start
    for _ in range(T):
        img = Image.open(os.path.join(path, "image_%05d.jpg" % fid)).convert("RGB")
        if img.size[0] < crop:
            img = img.resize((crop, init_h), Image.LANCZOS)
        a = np.asarray(img)
        h, w = a.shape[:2]
        if mode == "train":
            if ij is None:  # get_params on the first frame only (utils.py:65-67)
                if h == crop and w == crop:
                    ij = (0, 0)
                else:
                    ij = (int(torch.randint(0, h - crop + 1, size=(1,)).item()),
                          int(torch.randint(0, w - crop + 1, size=(1,)).item()))
            i, j = ij
        else:
            i, j = int(round((h - crop) / 2.0)), int(round((w - crop) / 2.0))
        a = a[i:i + crop, j:j + crop]
        if flip:
            a = a[:, ::-1]
        out.append(_to_normalized(a))
        fid += 1
        if fid > n_all:
            out += [np.zeros((3, crop, crop), np.float32)] * (T - len(out))
            break
    return np.stack(out), int(min(T, n_all))
