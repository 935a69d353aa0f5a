#!/usr/bin/env python3
"""Time the in-tree training GEMMs (eosv_sgemm / eosv_sgemm_tn_splitk, gemm_f32.hip) on the
ResNet-50 finetune step's shapes (network_train.py:140: 6 clips x 16 frames at 224x224): the
stride-1 1x1 weight gradients (TN, split over the pixel count), the strided-conv input gradients
(NN) and the stem forward (NT, K = 147).  Prints one line per shape: ms and TF/s (HIP events,
median of 5).  A/B knobs (profiling build): EOSV_GEMM_AHEAD, EOSV_GEMM_WPC, EOSV_GEMM_MINROWS."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "embodied-one-shot-video-recognition_amd"))
import torch  # noqa: E402

from eosv._lib import check, lib, stream_ptr  # noqa: E402

F = 96
P = {1: F * 56 * 56, 2: F * 28 * 28, 3: F * 14 * 14, 4: F * 7 * 7}
TN = [(64, 256, P[1]), (256, 64, P[1]), (64, 64, P[1]), (128, 256, P[1]), (128, 512, P[2]), (512, 128, P[2]),
      (256, 512, P[2]), (256, 1024, P[3]), (1024, 256, P[3]), (512, 1024, P[3]), (512, 2048, P[4]),
      (2048, 512, P[4]), (64, 147, F * 112 * 112)]
NN = [(P[2], 9 * 128, 128), (P[3], 9 * 256, 256), (P[4], 9 * 512, 512), (P[2], 256, 512)]
NT = [(F * 112 * 112, 64, 147)]


def timed(fn):
    ts = []
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts[1:])[2]


L = lib()
s = stream_ptr()
tot = 0.0
for m, n, k in TN:
    A = torch.randn(k, m, device="cuda")
    B = torch.randn(k, n, device="cuda")
    C = torch.empty(m, n, device="cuda")
    wb = int(L.eosv_sgemm_tn_splitk_workspace(m, n, k))
    ws = torch.empty(max(wb // 4, 1) + 4, device="cuda")
    ms = timed(lambda: check(L.eosv_sgemm_tn_splitk(m, n, k, A.data_ptr(), m, B.data_ptr(), n, C.data_ptr(), n,
                                                    ws.data_ptr(), wb, s), "tn"))
    tot += ms
    print(f"TN m={m:5d} n={n:5d} k={k:7d}: {ms:7.3f} ms {2 * m * n * k / ms / 1e9:6.1f} TF/s")
for m, n, k in NN:
    A = torch.randn(m, k, device="cuda")
    B = torch.randn(k, n, device="cuda")
    C = torch.empty(m, n, device="cuda")
    ms = timed(lambda: check(L.eosv_sgemm(0, 0, m, n, k, 1.0, A.data_ptr(), k, B.data_ptr(), n, 0.0, C.data_ptr(), n, s),
                             "nn"))
    tot += ms
    print(f"NN m={m:7d} n={n:5d} k={k:5d}: {ms:7.3f} ms {2 * m * n * k / ms / 1e9:6.1f} TF/s")
for m, n, k in NT:
    A = torch.randn(m, k, device="cuda")
    B = torch.randn(n, k, device="cuda")
    C = torch.empty(m, n, device="cuda")
    ms = timed(lambda: check(L.eosv_sgemm(0, 1, m, n, k, 1.0, A.data_ptr(), k, B.data_ptr(), k, 0.0, C.data_ptr(), n, s),
                             "nt"))
    tot += ms
    print(f"NT m={m:7d} n={n:5d} k={k:5d}: {ms:7.3f} ms {2 * m * n * k / ms / 1e9:6.1f} TF/s")
print(f"total {tot:.3f} ms")
