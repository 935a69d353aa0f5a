"""Device-side engine: thin torch-facing wrappers over the C ABI + the batched episode path.

PyTorch is only plumbing here (device memory, streams); every op below is a call
into libeosv.so.  There is no CPU path: without a HIP device the calls raise.

Batched episodes (the MI355X-first restructuring of network_test.py:132-167): the
reference runs one 16-frame forward per video and syncs twice per video.  Here a
whole batch of episodes is laid out as one frame table in HBM
    [supports of ep0 | supports of ep1 | ... | query of ep0 | query of ep1 | ...]
then ONE backbone call (chunked internally), ONE clip-embed launch and ONE match
launch produce every prediction; only int64 predictions return to the host.
Results are identical to the per-video order because frames are independent
through the backbone and every reduction keeps the reference's order.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import synth
from ._lib import (EOSV_BF16, EOSV_F32, EOSV_F32X3, MATCH_COSINE, MATCH_PROTONET, MAX_COLS, EosvDesc, EosvError, check,
                   lib, ptr, stream_ptr)
from .arch import SPECS

_DTYPES = {"f32": EOSV_F32, "fp32": EOSV_F32, "float32": EOSV_F32, "bf16": EOSV_BF16, "bfloat16": EOSV_BF16,
           "f32x3": EOSV_F32X3}


def _device(device) -> torch.device:
    if isinstance(device, torch.device):
        return device
    return torch.device("cuda", torch.cuda.current_device() if device is None else int(device))


def _require_cuda(t: torch.Tensor, name: str, dtype=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name} must be a HIP device tensor")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


class Backbone:
    """One native ResNet handle (arch, dtype, frame size) bound to one device."""

    def __init__(self, arch: str = "resnet18", dtype: str = "f32", height: int = 224, width: int = 224,
                 max_frames: int = 256, device: Optional[int] = None, num_classes: int = 64):
        if arch not in SPECS:
            raise ValueError(f"unknown arch {arch}")
        if not torch.cuda.is_available():
            raise RuntimeError("eosv.Backbone needs a HIP device (no CPU fallback)")
        self.arch, self.dtype, self.height, self.width = arch, dtype, height, width
        self.spec = SPECS[arch]
        self.device = torch.cuda.current_device() if device is None else device
        self.num_classes = num_classes
        self.max_frames = max_frames
        d = EosvDesc(self.spec.arch_id, _DTYPES[dtype], height, width, max_frames, self.device, num_classes)
        h = ctypes.c_void_p()
        check(lib().eosv_create(ctypes.byref(d), ctypes.byref(h)), "eosv_create")
        self._h = h
        self.D = lib().eosv_feature_dim(h)
        self.loaded = False

    def load_state_dict(self, state: Dict[str, object]):
        """Reference state_dict (names of models.py model_resnetXX) -> folded device weights."""
        keep = []
        names, ptrs, numels = [], [], []
        for k, v in state.items():
            if k.endswith("num_batches_tracked"):
                continue
            a = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
            a = np.ascontiguousarray(a, dtype=np.float32)
            keep.append(a)
            names.append(k.encode())
            ptrs.append(a.ctypes.data)
            numels.append(a.size)
        n = len(names)
        c_names = (ctypes.c_char_p * n)(*names)
        c_ptrs = (ctypes.c_void_p * n)(*ptrs)
        c_num = (ctypes.c_int64 * n)(*numels)
        check(lib().eosv_load_weights(self._h, c_names, c_ptrs, c_num, n), "eosv_load_weights")
        self.loaded = True

    def forward(self, frames: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """frames [B,3,H,W] f32 (device) -> features [B,D] f32 (device)."""
        _require_cuda(frames, "frames", torch.float32)
        if frames.dim() != 4 or tuple(frames.shape[1:]) != (3, self.height, self.width):
            raise ValueError(f"frames must be [B,3,{self.height},{self.width}], got {tuple(frames.shape)}")
        B = frames.shape[0]
        if out is None:
            out = torch.empty(B, self.D, device=frames.device, dtype=torch.float32)
        check(lib().eosv_backbone_forward(self._h, ptr(frames), B, ptr(out), stream_ptr(stream)),
              "eosv_backbone_forward")
        return out

    def stage_shape(self, stage: int):
        """(h, w, C) of the map after the stem + maxpool (stage 0) or after layer `stage`."""
        out = lambda n, k, st, p: (n + 2 * p - k) // st + 1  # noqa: E731
        h, w = out(out(self.height, 7, 2, 3), 3, 2, 1), out(out(self.width, 7, 2, 3), 3, 2, 1)
        if stage == 0:
            return h, w, 64
        for _ in range(2, stage + 1):
            h, w = out(h, 3, 2, 1), out(w, 3, 2, 1)
        return h, w, (64 << (stage - 1)) * (4 if self.D == 2048 else 1)

    def probe(self, frames: torch.Tensor, stage: int, stream=None) -> torch.Tensor:
        """The map after the stem + maxpool (stage 0) or after layer `stage` (1..4), f32 NHWC
        [B, h, w, C] (eosv_backbone_probe: diagnostics and the per-layer checksum test)."""
        frames = frames.contiguous()
        _require_cuda(frames, "frames", torch.float32)
        if not 0 <= stage <= 4:
            raise ValueError("stage must be 0..4")
        B = frames.shape[0]
        h, w, C = self.stage_shape(stage)
        out = torch.empty(B, h, w, C, device=frames.device, dtype=torch.float32)
        n = lib().eosv_backbone_probe(self._h, ptr(frames), B, int(stage), ptr(out), stream_ptr(stream))
        if n < 0:
            check(n, "eosv_backbone_probe")
        if n != h * w * C:
            raise EosvError(f"eosv_backbone_probe: {n} elements per frame, expected {h * w * C}")
        return out

    def fc(self, feat: torch.Tensor, stream=None) -> torch.Tensor:
        _require_cuda(feat, "feat", torch.float32)
        out = torch.empty(feat.shape[0], self.num_classes, device=feat.device, dtype=torch.float32)
        check(lib().eosv_fc_forward(self._h, ptr(feat), feat.shape[0], ptr(out), stream_ptr(stream)),
              "eosv_fc_forward")
        return out

    def profile(self, enable: bool = True):
        """Bracket every conv launch with HIP events (eosv_profile_enable); clears the log."""
        check(lib().eosv_profile_enable(self._h, int(enable)), "eosv_profile_enable")

    def profile_read(self, max_layers: int = 256):
        """Per-layer (ms, flops, launches) since profile(True); synchronises on the events."""
        ms = np.zeros(max_layers, np.float64)
        fl = np.zeros(max_layers, np.float64)
        n = np.zeros(max_layers, np.int64)
        rc = lib().eosv_profile_read(self._h, ms.ctypes.data, fl.ctypes.data, n.ctypes.data, max_layers)
        if rc < 0:
            check(rc, "eosv_profile_read")
        return ms[:rc], fl[:rc], n[:rc]

    @property
    def device_bytes(self) -> int:
        return int(lib().eosv_device_bytes(self._h))

    def close(self):
        if getattr(self, "_h", None):
            lib().eosv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ functional ops

def clip_embed(feat: torch.Tensor, offsets: torch.Tensor, counts: torch.Tensor, l2: bool = True,
               stream=None) -> torch.Tensor:
    """Per-clip mean of (L2-normalised) frame features (network_test.py:62-65)."""
    _require_cuda(feat, "feat", torch.float32)
    _require_cuda(offsets, "offsets", torch.int32)
    _require_cuda(counts, "counts", torch.int32)
    n, D = offsets.shape[0], feat.shape[1]
    emb = torch.empty(n, D, device=feat.device, dtype=torch.float32)
    check(lib().eosv_clip_embed(ptr(feat), ptr(offsets), ptr(counts), n, D, int(bool(l2)), ptr(emb),
                                stream_ptr(stream)), "eosv_clip_embed")
    return emb


def segment_mean(feat: torch.Tensor, seg_len: int, stream=None) -> torch.Tensor:
    _require_cuda(feat, "feat", torch.float32)
    n_seg, D = feat.shape[0] // seg_len, feat.shape[1]
    out = torch.empty(n_seg, D, device=feat.device, dtype=torch.float32)
    check(lib().eosv_segment_mean(ptr(feat), n_seg, seg_len, D, ptr(out), stream_ptr(stream)),
          "eosv_segment_mean")
    return out


def match(query: torch.Tensor, support: torch.Tensor, sup_off: torch.Tensor,
          sup_slot: Optional[torch.Tensor], n_proto: Optional[torch.Tensor], kind: str = "protonet",
          stream=None):
    """One-shot matching for a batch of episodes -> (pred int64 [E], score f32 [E,64])."""
    _require_cuda(query, "query", torch.float32)
    _require_cuda(support, "support", torch.float32)
    _require_cuda(sup_off, "sup_off", torch.int32)
    E, D = query.shape
    k = {"protonet": MATCH_PROTONET, "cosine": MATCH_COSINE}[kind]
    pred = torch.empty(E, device=query.device, dtype=torch.int64)
    score = torch.empty(E, MAX_COLS, device=query.device, dtype=torch.float32)
    check(lib().eosv_match(ptr(query), ptr(support), ptr(sup_off), ptr(sup_slot), ptr(n_proto), E, D, k,
                           ptr(pred), ptr(score), stream_ptr(stream)), "eosv_match")
    return pred, score


def segment_match(seg: torch.Tensor, gallery: torch.Tensor, lamda1: float, lamda2: float, stream=None):
    """Gallery segment ids (argmin of the temporally smoothed cdist), network_test.py:207-214."""
    _require_cuda(seg, "seg", torch.float32)
    _require_cuda(gallery, "gallery", torch.float32)
    S, D = seg.shape
    G = gallery.shape[0]
    ids = torch.empty(S, device=seg.device, dtype=torch.int64)
    dist = torch.empty(S, G, device=seg.device, dtype=torch.float32)
    check(lib().eosv_segment_match(ptr(seg), S, ptr(gallery), G, D, float(lamda1), float(lamda2),
                                   ptr(ids), ptr(dist), stream_ptr(stream)), "eosv_segment_match")
    return ids, dist


def segment_match_episodes(seg: torch.Tensor, n_episodes: int, gallery: torch.Tensor, lamda1: float,
                           lamda2: float, with_dist: bool = False, stream=None):
    """segment_match for n_episodes independent episodes in one call: seg [n_episodes*S, D]
    episode-major -> ids [n_episodes*S] (smoothing never crosses an episode boundary)."""
    _require_cuda(seg, "seg", torch.float32)
    _require_cuda(gallery, "gallery", torch.float32)
    R, D = seg.shape
    if n_episodes <= 0 or R % n_episodes:
        raise ValueError("seg rows must be a multiple of n_episodes")
    G = gallery.shape[0]
    ids = torch.empty(R, device=seg.device, dtype=torch.int64)
    dist = torch.empty(R, G, device=seg.device, dtype=torch.float32) if with_dist else None
    check(lib().eosv_segment_match_episodes(ptr(seg), n_episodes, R // n_episodes, ptr(gallery), G, D,
                                            float(lamda1), float(lamda2), ptr(ids),
                                            ptr(dist) if dist is not None else None, stream_ptr(stream)),
          "eosv_segment_match_episodes")
    return ids, dist


def temporal_smooth(x: torch.Tensor, lamda1: float, lamda2: float, stream=None) -> torch.Tensor:
    """3-tap [l1,l2,l1] smoothing along the last axis, zero padded (models.py:42-56)."""
    _require_cuda(x, "x", torch.float32)
    cols = x.shape[-1] if x.dim() else 1
    rows = x.numel() // max(cols, 1)
    y = torch.empty_like(x)
    check(lib().eosv_temporal_smooth(ptr(x), rows, cols, float(lamda1), float(lamda2), ptr(y), stream_ptr(stream)),
          "eosv_temporal_smooth")
    return y


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def normalize_frames(rgb: torch.Tensor, crop: int = 224, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                     stream=None) -> torch.Tensor:
    """Decoded uint8 frames [F,H,W,3] (device) -> centre-cropped, normalised [F,3,crop,crop] f32."""
    _require_cuda(rgb, "rgb", torch.uint8)
    F, H, W, C = rgb.shape
    if C != 3:
        raise ValueError("rgb must be [F,H,W,3]")
    out = torch.empty(F, 3, crop, crop, device=rgb.device, dtype=torch.float32)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    sd = (ctypes.c_float * 3)(*[float(v) for v in std])
    check(lib().eosv_normalize_frames(ptr(rgb), F, H, W, crop, m, sd, ptr(out), stream_ptr(stream)),
          "eosv_normalize_frames")
    return out


def crop_normalize_frames(rgb: torch.Tensor, crop: int, top: int, left: int, flip: bool = False,
                          mean=IMAGENET_MEAN, std=IMAGENET_STD, stream=None) -> torch.Tensor:
    """Decoded uint8 frames [F,H,W,3] (device) -> window (top, left, crop) [mirrored] -> normalised
    [F,3,crop,crop] f32 (utils.py:57-91: ClipRandomCrop / CenterCrop, hflip, ToTensor, Normalize)."""
    _require_cuda(rgb, "rgb", torch.uint8)
    F, H, W, C = rgb.shape
    if C != 3:
        raise ValueError("rgb must be [F,H,W,3]")
    out = torch.empty(F, 3, crop, crop, device=rgb.device, dtype=torch.float32)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    sd = (ctypes.c_float * 3)(*[float(v) for v in std])
    check(lib().eosv_crop_normalize_frames(ptr(rgb), F, H, W, crop, int(top), int(left), int(bool(flip)), m, sd,
                                           ptr(out), stream_ptr(stream)), "eosv_crop_normalize_frames")
    return out


def synth_frames(params: np.ndarray, H: int, W: int, device=None, out: Optional[torch.Tensor] = None,
                 stream=None) -> torch.Tensor:
    """Generate frames [F,3,H,W] on the device from a [F,4] u64 table (see frame_table)."""
    params = np.ascontiguousarray(params, dtype=np.uint64)
    F = params.shape[0]
    dev = _device(device)
    p = torch.from_numpy(params.view(np.int64)).to(dev)
    if out is None:
        out = torch.empty(F, 3, H, W, device=dev, dtype=torch.float32)
    check(lib().eosv_synth_frames(ptr(p), F, H, W, ptr(out), stream_ptr(stream)), "eosv_synth_frames")
    return out


# ------------------------------------------------------------------ episode batches

@dataclass
class EpisodeBatch:
    """Host-side layout of a batch of episodes as one frame/clip table."""
    params: np.ndarray           # [F,4] u64 synth params (class, video, noise seed, frame id)
    clip_off: np.ndarray         # [C] int32 first frame row of each clip
    clip_cnt: np.ndarray         # [C] int32 frames of each clip
    sup_off: np.ndarray          # [E+1] int32 support clip offsets
    sup_slot: np.ndarray         # [S] int32 prototype slot of each support clip
    n_proto: np.ndarray          # [E] int32
    query_y: np.ndarray          # [E] int64 label of each query
    n_support: int
    episodes: List[dict] = field(default_factory=list)

    @property
    def n_frames(self) -> int:
        return int(self.params.shape[0])

    @property
    def n_clips(self) -> int:
        return int(self.clip_off.shape[0])


def video_frames(video_info: str, T: int):
    """(frame ids, clip length) the reference feeds the backbone for one video.

    Support: get_video_from_video_info_3 zero-pads to T but returns min(T, all) and
    network_test.py:54-55 truncates to it; query: get_video_from_video_info stops at
    the last frame (utils.py:129-131).  Either way the clip = its real frames.
    """
    ids, _ = synth.clip_frame_ids(video_info, T)
    return ids


def build_episode_batch(episodes: Sequence[dict], T: int = 16) -> EpisodeBatch:
    """episodes: dicts with support, support_y, query, query_y (video_info strings)."""
    rows, clip_off, clip_cnt = [], [], []

    def add_clip(vi: str):
        cls = vi.split("/")[0]
        cs, vs, crc = synth.class_seed(cls), synth.video_seed(vi), synth.crc32(vi)
        ids = video_frames(vi, T)
        clip_off.append(len(rows))
        clip_cnt.append(len(ids))
        for f in ids:
            rows.append((cs, vs, synth.mix64_int(((crc << 20) + f) ^ synth.TAG_NOISE), f))

    sup_off, sup_slot, n_proto = [0], [], []
    for ep in episodes:
        seen: Dict[int, int] = {}
        for vi, y in zip(ep["support"], ep["support_y"]):
            add_clip(vi)
            sup_slot.append(seen.setdefault(int(y), len(seen)))
        sup_off.append(sup_off[-1] + len(ep["support"]))
        n_proto.append(len(seen))
    n_support = sup_off[-1]
    for ep in episodes:
        add_clip(ep["query"])
    return EpisodeBatch(
        params=np.array(rows, dtype=np.uint64).reshape(-1, 4),
        clip_off=np.array(clip_off, np.int32), clip_cnt=np.array(clip_cnt, np.int32),
        sup_off=np.array(sup_off, np.int32), sup_slot=np.array(sup_slot, np.int32),
        n_proto=np.array(n_proto, np.int32),
        query_y=np.array([ep["query_y"] for ep in episodes], np.int64),
        n_support=n_support, episodes=list(episodes))


class DeviceEpisodes:
    """An EpisodeBatch resident in HBM (frames generated on the device)."""

    def __init__(self, batch: EpisodeBatch, H: int, W: int, device=None, frames: Optional[torch.Tensor] = None):
        dev = _device(device)
        self.batch = batch
        self.frames = frames if frames is not None else synth_frames(batch.params, H, W, dev)
        t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        self.clip_off, self.clip_cnt = t(batch.clip_off), t(batch.clip_cnt)
        self.sup_off, self.sup_slot, self.n_proto = t(batch.sup_off), t(batch.sup_slot), t(batch.n_proto)


def run_episodes(backbone: Backbone, dev_eps: DeviceEpisodes, kind: str = "protonet", L2: bool = True,
                 feat: Optional[torch.Tensor] = None, stream=None):
    """Backbone over every frame, clip embeddings, matching.  Returns (pred, emb, score) on device."""
    b = dev_eps.batch
    feat = backbone.forward(dev_eps.frames, out=feat, stream=stream)
    emb = clip_embed(feat, dev_eps.clip_off, dev_eps.clip_cnt, L2, stream=stream)
    support, query = emb[:b.n_support], emb[b.n_support:]
    pred, score = match(query, support, dev_eps.sup_off, dev_eps.sup_slot, dev_eps.n_proto, kind,
                        stream=stream)
    return pred, emb, score
