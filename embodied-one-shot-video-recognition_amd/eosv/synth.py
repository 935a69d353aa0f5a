"""Deterministic synthetic frames, frame counts and ResNet weights.

The reference reads JPEG frames from ``<FRAME_DIR>/<class>/<video>/image_%05d.jpg``
(``utils.py:96-136, 215-258``) and ImageNet weights from the network
(``models.py:13,28``).  Neither exists offline, so every input of this build is
synthetic and comes from one counter-based generator:

* ``splitmix64`` over a 64-bit counter, four 16-bit fields summed
  (Irwin-Hall, n=4) -> an integer in [-131070, 131070] -> ONE f32 multiply.

Every step is integer arithmetic or a single correctly rounded f32 operation,
so the host (numpy, here) and the device (``csrc/synth.hip``) produce
bit-identical frames.  No FMA contraction is allowed on either side.

Frames are produced directly in post-``Normalize`` space (``utils.py:88-91``),
i.e. what ``transforms('test')`` would hand to the backbone.  A frame is

    frame[c,y,x] = (A_CLS*Gc[c][gy][gx] + A_VID*Gv[c][gy][(gx + fid//4) % G])
                   + A_NOISE*Gn[c][y][x]

with ``gy = y*G//H``, ``gx = x*G//W`` (G = 14): a class pattern, a per-video
pattern that drifts one cell every four frames, and per-frame pixel noise.
"""
from __future__ import annotations

import zlib

import numpy as np

MASK64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
GAUSS_SCALE = np.float32(1.0 / 37837.2264)  # 1/std of the Irwin-Hall(4) sum of u16
GRID = 14
A_CLS = np.float32(1.0)
A_VID = np.float32(1.0)
A_NOISE = np.float32(0.5)

# stream tags (xor-ed into seeds so different tensors never share a stream)
TAG_CLS = 0x436C6173_73000000
TAG_VID = 0x56696465_6F000000
TAG_NOISE = 0x4E6F6973_65000000
TAG_WEIGHT = 0x57656967_68740000


def crc32(s: str) -> int:
    return zlib.crc32(s.encode("utf-8")) & 0xFFFFFFFF


def mix64(z):
    """splitmix64 finaliser on a numpy uint64 array (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def mix64_int(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def gauss_int(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Integer pseudo-gaussian stream: element i uses counter seed + (start+i+1)*GOLDEN."""
    idx = np.arange(start + 1, start + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = mix64(np.uint64(seed & MASK64) + idx * np.uint64(GOLDEN))
    s = ((z & np.uint64(0xFFFF)) + ((z >> np.uint64(16)) & np.uint64(0xFFFF))
         + ((z >> np.uint64(32)) & np.uint64(0xFFFF)) + (z >> np.uint64(48)))
    return s.astype(np.int64) - 131070


def gauss_f32(seed: int, n: int) -> np.ndarray:
    return gauss_int(seed, n).astype(np.float32) * GAUSS_SCALE


def uniform_f32(seed: int, n: int) -> np.ndarray:
    """U[0,1) with 24-bit resolution (exact in f32)."""
    idx = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = mix64(np.uint64(seed & MASK64) + idx * np.uint64(GOLDEN))
    return (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))


# --------------------------------------------------------------------------------------
# frames
# --------------------------------------------------------------------------------------

def class_seed(class_name: str) -> int:
    return mix64_int(crc32(class_name) ^ TAG_CLS)


def video_seed(video_info: str) -> int:
    return mix64_int(crc32(video_info) ^ TAG_VID)


def noise_seed(video_info: str, fid: int) -> int:
    return mix64_int(((crc32(video_info) << 20) + fid) ^ TAG_NOISE)


_TRAIN_CLASSES = None


def _train_classes():
    global _TRAIN_CLASSES
    if _TRAIN_CLASSES is None:
        import os

        p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sources/data/train.list")
        with open(p) as f:
            _TRAIN_CLASSES = frozenset(line.split("/")[0] for line in f if line.strip())
    return _TRAIN_CLASSES


def frame_count(video_info: str) -> int:
    """Number of JPEG frames the synthetic video has (``len(listdir) - 1``, utils.py:103).

    1 in 16 videos of the novel (non-train) classes is short (4..15 frames) so that the
    reference's zero-padding and truncation paths (utils.py:105-112, 249-257;
    network_test.py:54-55) are exercised.  Train-split videos are never short: the
    reference's gallery loader (generate_augmented_datasets.py:25-36) stacks them and
    needs full 16-frame clips, as the real miniKinetics videos provide.
    """
    h = crc32(video_info)
    if h % 16 == 0 and video_info.split("/")[0] not in _train_classes():
        return 4 + (h >> 8) % 12
    return 250 + h % 51


def clip_start(all_frame_count: int, video_frames: int) -> int:
    """Test-mode start frame, ``utils.py:105-112`` / ``224-231``."""
    if all_frame_count - video_frames - 1 > 1:
        return all_frame_count // 2 - video_frames // 2 + 1
    return 1


def clip_frame_ids(video_info: str, video_frames: int):
    """Frame ids (1-based) that the reference loads, and the real-frame count.

    Mirrors the loop of ``get_video_from_video_info`` (utils.py:114-131): frames
    ``start, start+1, ...`` until ``video_frames`` are read or the video ends.
    """
    n_all = frame_count(video_info)
    start = clip_start(n_all, video_frames)
    ids = []
    fid = start
    for _ in range(video_frames):
        ids.append(fid)
        fid += 1
        if fid > n_all:
            break
    return ids, n_all


def frame_params(class_name: str, video_info: str):
    return class_seed(class_name), video_seed(video_info), crc32(video_info)


def synth_frame(class_name: str, video_info: str, fid: int, H: int = 224, W: int = 224) -> np.ndarray:
    """One normalised frame [3,H,W] f32 (host reference of ``eosv_synth_frames``)."""
    gc = gauss_f32(class_seed(class_name), 3 * GRID * GRID).reshape(3, GRID, GRID)
    gv = gauss_f32(video_seed(video_info), 3 * GRID * GRID).reshape(3, GRID, GRID)
    gn = gauss_f32(noise_seed(video_info, fid), 3 * H * W).reshape(3, H, W)
    gy = (np.arange(H) * GRID) // H
    gx = (np.arange(W) * GRID) // W
    gxv = (gx + fid // 4) % GRID
    cls_part = gc[:, gy][:, :, gx] * A_CLS
    vid_part = gv[:, gy][:, :, gxv] * A_VID
    noise_part = gn * A_NOISE
    return ((cls_part + vid_part) + noise_part).astype(np.float32)


def synth_video(class_name: str, video_info: str, fids, H: int = 224, W: int = 224) -> np.ndarray:
    return np.stack([synth_frame(class_name, video_info, f, H, W) for f in fids])


# --------------------------------------------------------------------------------------
# weights (torchvision ResNet state_dict layout, models.py:9-37)
# --------------------------------------------------------------------------------------

def weight_seed(name: str, seed: int) -> int:
    return mix64_int(crc32(name) ^ TAG_WEIGHT ^ ((seed & 0xFFFFFFFF) << 32))


def synth_tensor(name: str, shape, seed: int = 0, last_bn: bool = False) -> np.ndarray:
    """Deterministic value for one state_dict entry of a torchvision ResNet + fc.

    ``last_bn`` marks the final BN of a residual branch (bn2 of a BasicBlock, bn3 of a
    Bottleneck): its gamma is damped so the residual stream of a random-weight net does
    not grow without bound through 8..33 blocks.
    """
    n = int(np.prod(shape)) if len(shape) else 1
    s = weight_seed(name, seed)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "weight" and len(shape) == 4:
        fan_out = shape[0] * shape[2] * shape[3]
        std = np.float32(np.sqrt(2.0 / fan_out))
        return (gauss_f32(s, n) * std).reshape(shape)
    if name.startswith("fc."):
        bound = np.float32(1.0 / np.sqrt(512.0 if leaf == "bias" else shape[-1]))
        u = uniform_f32(s, n) * np.float32(2.0) - np.float32(1.0)
        return (u * bound).reshape(shape)
    if leaf == "weight":
        base = np.float32(0.35) if last_bn else np.float32(1.0)
        return (base + gauss_f32(s, n) * np.float32(0.1)).reshape(shape)
    if leaf in ("bias", "running_mean"):
        return (gauss_f32(s, n) * np.float32(0.1)).reshape(shape)
    if leaf == "running_var":
        return (np.float32(0.5) + uniform_f32(s, n)).reshape(shape)
    raise KeyError(f"no synthetic rule for {name} {shape}")


def synth_state_dict(spec, num_classes: int = 64, seed: int = 0):
    """name -> np.ndarray for every entry of the reference model's state_dict."""
    from .arch import state_dict_shapes

    last = "bn2." if spec.block == "basic" else "bn3."
    out = {}
    for n, s in state_dict_shapes(spec, num_classes).items():
        out[n] = synth_tensor(n, s, seed, last_bn=(last in n))
    return out
