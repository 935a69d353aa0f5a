"""ctypes binding of ``libeosv.so`` (the C ABI declared in include/eosv.h).

There is no CPU fallback: if the library is missing or no HIP device is visible the
calls raise.  The library is built in-tree (``csrc/Makefile`` or
``__graft_entry__.build()``) next to this package.
"""
from __future__ import annotations

import ctypes
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# EOSV_LIBRARY selects another build of the same ABI: tools/ set it to libeosv_prof.so (the
# profiling build with the A/B switches and ablations compiled in, `make -C csrc prof`)
LIB_PATH = os.environ.get("EOSV_LIBRARY") or os.path.join(PKG_ROOT, "libeosv.so")

def source_digest() -> str:
    """sha256 (16 hex) of the library's sources and build recipe (csrc/*.hip, common.h,
    include/eosv.h, csrc/Makefile): ties a profile (e.g. profiles/*_traffic.json) to the kernels it
    measured; computable on the GPU box, where there is no git history.  The library binary is NOT
    hashed here (r06: a non-reproducible rebuild, or a digest taken before the build, silently
    detached every profile): which build a profile ran is library_kind(), and its bytes are
    library_digest(), recorded beside it for information."""
    import glob
    import hashlib

    h = hashlib.sha256()
    repo = os.path.dirname(PKG_ROOT)
    files = sorted(glob.glob(os.path.join(PKG_ROOT, "csrc", "*.hip"))) + \
        [os.path.join(PKG_ROOT, "csrc", "common.h"), os.path.join(repo, "include", "eosv.h"),
         os.path.join(PKG_ROOT, "csrc", "Makefile")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def library_kind() -> str:
    """The build configuration this process loads: "release" (libeosv.so), else the library's file
    name (libeosv_prof.so: the profiling build with its A/B switches; libeosv_<variant>.so)."""
    name = os.path.basename(LIB_PATH)
    return "release" if name == "libeosv.so" else name


def library_digest() -> str:
    """sha256 (16 hex) of the bytes of the library this process loads ("" before it exists)."""
    import hashlib

    if not os.path.exists(LIB_PATH):
        return ""
    with open(LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


EOSV_F32, EOSV_BF16, EOSV_F32X3 = 0, 1, 2
MATCH_PROTONET, MATCH_COSINE = 0, 1
MAX_COLS = 64

_STATUS = {-1: "EOSV_ERR_ARG", -2: "EOSV_ERR_HIP", -3: "EOSV_ERR_OOM",
           -4: "EOSV_ERR_UNSUPPORTED", -5: "EOSV_ERR_STATE"}

# every symbol include/eosv.h declares
EXPORTS = ("eosv_create", "eosv_load_weights", "eosv_backbone_forward", "eosv_backbone_probe", "eosv_fc_forward",
           "eosv_clip_embed", "eosv_segment_mean", "eosv_match", "eosv_segment_match", "eosv_segment_match_episodes",
           "eosv_temporal_smooth", "eosv_normalize_frames", "eosv_crop_normalize_frames", "eosv_synth_frames", "eosv_plan_episodes", "eosv_profile_enable", "eosv_profile_read", "eosv_feature_dim", "eosv_device_bytes", "eosv_last_error",
           "eosv_destroy",
           # training path
           "eosv_sgemm", "eosv_im2col", "eosv_col2im", "eosv_bn_workspace_bytes", "eosv_bn_train_forward",
           "eosv_bn_train_backward", "eosv_maxpool_forward", "eosv_maxpool_backward", "eosv_avgpool_forward",
           "eosv_broadcast_rows", "eosv_softmax_xent", "eosv_sum_rows", "eosv_add_bias", "eosv_sgd_momentum",
           "eosv_axpy", "eosv_nchw_to_nhwc", "eosv_conv2d_f32", "eosv_flip_weights",
           "eosv_sgemm_tn_splitk_workspace", "eosv_sgemm_tn_splitk", "eosv_conv_wgrad_f32_workspace",
           "eosv_conv_wgrad_f32", "eosv_conv2d_f32_workspace")


class EosvDesc(ctypes.Structure):
    _fields_ = [("arch", ctypes.c_int), ("dtype", ctypes.c_int), ("height", ctypes.c_int),
                ("width", ctypes.c_int), ("max_frames", ctypes.c_int), ("device", ctypes.c_int),
                ("num_classes", ctypes.c_int)]


class EosvError(RuntimeError):
    pass


_lib = None


def lib():
    """Load libeosv.so once (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EosvError(f"{LIB_PATH} not built: run `make -C csrc` or __graft_entry__.build()")
    # RTLD_NOW: an unresolved symbol (e.g. a kernel stub the host pass dropped) fails here, at load
    L = ctypes.CDLL(LIB_PATH, mode=os.RTLD_NOW | os.RTLD_LOCAL)
    vp, i32, i64, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
    sig = {
        "eosv_create": (i32, [ctypes.POINTER(EosvDesc), ctypes.POINTER(vp)]),
        "eosv_load_weights": (i32, [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(vp),
                                    ctypes.POINTER(i64), i32]),
        "eosv_backbone_forward": (i32, [vp, vp, i32, vp, vp]),
        "eosv_backbone_probe": (i32, [vp, vp, i32, i32, vp, vp]),
        "eosv_fc_forward": (i32, [vp, vp, i32, vp, vp]),
        "eosv_clip_embed": (i32, [vp, vp, vp, i32, i32, i32, vp, vp]),
        "eosv_segment_mean": (i32, [vp, i32, i32, i32, vp, vp]),
        "eosv_match": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, vp]),
        "eosv_segment_match": (i32, [vp, i32, vp, i32, i32, f32, f32, vp, vp, vp]),
        "eosv_segment_match_episodes": (i32, [vp, i32, i32, vp, i32, i32, f32, f32, vp, vp, vp]),
        "eosv_temporal_smooth": (i32, [vp, i32, i32, f32, f32, vp, vp]),
        "eosv_normalize_frames": (i32, [vp, i32, i32, i32, i32, vp, vp, vp, vp]),
        "eosv_crop_normalize_frames": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
        "eosv_synth_frames": (i32, [vp, i32, i32, i32, vp, vp]),
        "eosv_plan_episodes": (i32, [vp, i32, i32, i32, ctypes.c_uint64, i32, vp, vp, vp]),
        "eosv_profile_enable": (i32, [vp, i32]),
        "eosv_profile_read": (i32, [vp, vp, vp, vp, i32]),
        "eosv_feature_dim": (i32, [vp]),
        "eosv_device_bytes": (i64, [vp]),
        "eosv_last_error": (ctypes.c_char_p, []),
        "eosv_destroy": (None, [vp]),
        "eosv_sgemm": (i32, [i32, i32, i32, i32, i32, f32, vp, i32, vp, i32, f32, vp, i32, vp]),
        "eosv_im2col": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
        "eosv_col2im": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
        "eosv_bn_workspace_bytes": (i64, [i32]),
        "eosv_bn_train_forward": (i32, [vp, i64, i32, vp, vp, f32, f32, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp]),
        "eosv_bn_train_backward": (i32, [vp, vp, vp, i32, vp, i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "eosv_maxpool_forward": (i32, [vp, i32, i32, i32, i32, vp, vp, vp]),
        "eosv_maxpool_backward": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
        "eosv_avgpool_forward": (i32, [vp, i32, i32, i32, vp, vp]),
        "eosv_broadcast_rows": (i32, [vp, i32, i32, i32, f32, vp, vp]),
        "eosv_softmax_xent": (i32, [vp, vp, i32, i32, vp, vp, vp]),
        "eosv_sum_rows": (i32, [vp, i32, i32, vp, i32, vp]),
        "eosv_add_bias": (i32, [vp, i32, i32, vp, vp]),
        "eosv_sgd_momentum": (i32, [vp, vp, vp, i64, f32, f32, i32, vp]),
        "eosv_axpy": (i32, [vp, vp, i64, f32, vp]),
        "eosv_nchw_to_nhwc": (i32, [vp, i32, i32, i32, i32, vp, vp]),
        "eosv_conv2d_f32": (i32, [vp, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, vp, vp, i32, vp, vp, i64,
                                  vp]),
        "eosv_conv2d_f32_workspace": (i64, [i32] * 9),
        "eosv_flip_weights": (i32, [vp, i32, i32, i32, i32, vp, vp]),
        "eosv_sgemm_tn_splitk_workspace": (i64, [i32, i32, i32]),
        "eosv_sgemm_tn_splitk": (i32, [i32, i32, i32, vp, i32, vp, i32, vp, i32, vp, i64, vp]),
        "eosv_conv_wgrad_f32_workspace": (i64, [i32] * 9),
        "eosv_conv_wgrad_f32": (i32, [vp, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, vp, vp, i64, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().eosv_last_error().decode(errors="replace")
        raise EosvError(f"{what} failed: {_STATUS.get(rc, rc)}: {msg}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (None -> NULL)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(stream=None) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
