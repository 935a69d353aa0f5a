"""Drop-in for the reference's ``utils.py``: globals + frame loaders.

Same global names and values as reference utils.py:14-44, and the same loader
functions (utils.py:80-258).  Differences, all deliberate:
  * frames come from ``eosv.frames`` (real JPEG dirs when present, else the
    deterministic synthetic generator -- this image has no dataset);
  * the other drop-in modules read these globals at call time (``utils.n_way = 14``
    reaches the episode loader), where the reference's star-import froze them.
"""
import copy
import os
import random  # noqa: F401  (the reference exposes the global RNG through utils)

import numpy as np
import torch

import sys as _sys
_here = os.path.dirname(os.path.abspath(__file__))
if _here not in _sys.path:
    _sys.path.insert(0, _here)

from eosv import frames as _frames  # noqa: E402

# global path (utils.py:14-30)
KINETICS_VIDEO_DIR = '/DATACENTER/2/lovelyqian/Kinetics/Kinetics/videos/'
KINETICS_FRAME_DIR = '/DATACENTER/2/lovelyqian/Kinetics/Kinetics/miniKinetics_frames/'
TRAIN_LIST = os.path.join(_here, 'sources/data/train.list')
VAL_LIST = os.path.join(_here, 'sources/data/val.list')
TEST_LIST = os.path.join(_here, 'sources/data/test.list')
GALLERY_LIST = os.path.join(_here, 'sources/data/gallery.list')
TrainAugSegDatasets_DIR_2_3 = '/DATACENTER/s/lovelyqian/miniKinetics_frames_2.3/'

# global variables (utils.py:32-44)
num_classes_train = 64
VIDEO_FRAMES = 16
IMG_INIT_H = 256
IMG_crop_size = (224, 224)
BATCH_SIZE = 6
n_way = 5
k_shot = 1
seg_len = 2
test_episodes = 20000
val_episodes = 100
lamda1, lamda2 = 0.1, 1.0
EPISODE_NUMS = {'test': test_episodes, 'val': val_episodes}

_SOURCES = {}


def frame_source(frame_dir=None):
    """The FrameSource serving ``frame_dir`` (cached)."""
    frame_dir = KINETICS_FRAME_DIR if frame_dir is None else frame_dir
    key = (frame_dir, IMG_crop_size)
    if key not in _SOURCES:
        _SOURCES[key] = _frames.default_source(frame_dir, IMG_crop_size[0], IMG_crop_size[1])
    return _SOURCES[key]


def transfer_weights(model_from, model_to):
    """utils.py:47-54."""
    wf = copy.deepcopy(model_from.state_dict())
    wt = model_to.state_dict()
    for k in wt.keys():
        if (k not in wf) or k == 'fc.weight' or k == 'fc.bias':
            wf[k] = wt[k]
    model_to.load_state_dict(wf)


def transforms(mode):
    """utils.py:80-91: PIL image -> normalised [3,224,224] tensor on the GPU
    (eosv_crop_normalize_frames).  test/val: centre crop.  train: one random window and flip
    per transform object, as ClipRandomCrop / ClipRandomHorizontalFlip (utils.py:57-78)."""
    import random as _rnd
    from eosv import engine as _engine

    c = IMG_crop_size[0]
    flip = _rnd.random() < 0.5 if mode == 'train' else False
    state = {}

    def apply(img):
        a = np.asarray(img.convert('RGB'))
        h, w = a.shape[:2]
        if mode == 'train':
            if 'ij' not in state:
                state['ij'] = (0, 0) if (h == c and w == c) else (
                    int(torch.randint(0, h - c + 1, size=(1,)).item()),
                    int(torch.randint(0, w - c + 1, size=(1,)).item()))
            i, j = state['ij']
        else:
            i, j = int(round((h - c) / 2.0)), int(round((w - c) / 2.0))
        rgb = torch.from_numpy(np.array(a)[None]).cuda()
        return _engine.crop_normalize_frames(rgb, c, i, j, flip)[0]

    return apply


def get_video_from_video_info(video_info, mode, video_frames=VIDEO_FRAMES, frame_dir=None, data_aug=None):
    """utils.py:96-136 -> [<=T,3,224,224] f32 (no padding)."""
    return frame_source(frame_dir).video(video_info, video_frames, mode, pad=False)[0]


def get_classname_from_video_info(video_info):
    """utils.py:140-147."""
    return video_info.split('/')[0]


def get_classInd(info_list):
    """utils.py:150-162."""
    classInd = {}
    for line in open(info_list).readlines():
        name = get_classname_from_video_info(line.strip('\n'))
        if name not in classInd:
            classInd[name] = len(classInd)
    return classInd


def get_label_from_video_info(video_info, info_list=TRAIN_LIST):
    """utils.py:164-168."""
    return get_classInd(info_list)[get_classname_from_video_info(video_info)]


def get_video_from_video_info_2(video_info, mode, video_frames=VIDEO_FRAMES, frame_dir=None):
    """utils.py:171-211 -> (video, np.array of frame paths)."""
    src = frame_source(frame_dir)
    n_all = src.frame_count(video_info)
    ids = _frames.clip_frame_ids(n_all, video_frames, mode)
    fd = KINETICS_FRAME_DIR if frame_dir is None else frame_dir
    paths = [os.path.join(fd, video_info, 'image_%05d.jpg' % f) for f in ids]
    return src.frames_tensor(video_info, ids, mode), np.array(paths)


def get_video_from_video_info_3(video_info, mode, video_frames=VIDEO_FRAMES, frame_dir=None):
    """utils.py:215-258 -> ([T,3,224,224] zero-padded, min(T, frame count))."""
    v, n = frame_source(frame_dir).video(video_info, video_frames, mode, pad=True)
    return v, np.int64(n)
