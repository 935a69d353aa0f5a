"""Per-shape timing of the training step's convs (R50, 96 frames at 224): forward through
eosv_conv2d_f32, stride-1 dgrad through the same kernels with flipped weights, KxK weight
gradient through eosv_conv_wgrad_f32.  Prints TF/s per shape (f32 peak 157.3)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "embodied-one-shot-video-recognition_amd"))
import torch  # noqa: E402

from eosv._lib import check, lib, stream_ptr  # noqa: E402

L = lib()
N = 96
shapes = []  # (name, H, Cin, Cout, k, stride)
H = 56
inpl = 64
for li, (planes, nb) in enumerate(zip((64, 128, 256, 512), (3, 4, 6, 3))):
    for b in range(nb):
        s = 2 if li > 0 and b == 0 else 1
        shapes.append((f"l{li+1}.{b}.c1", H, inpl, planes, 1, 1))
        shapes.append((f"l{li+1}.{b}.c2", H, planes, planes, 3, s))
        Ho = H // s
        shapes.append((f"l{li+1}.{b}.c3", Ho, planes, planes * 4, 1, 1))
        if b == 0:
            shapes.append((f"l{li+1}.{b}.ds", H, inpl, planes * 4, 1, s))
        H, inpl = Ho, planes * 4
seen = set()
s = stream_ptr()
tot = {"fwd": [0, 0], "fwdk": [0, 0], "wgrad": [0, 0], "wgrad_blas": [0, 0]}
for name, H, cin, cout, k, st in shapes:
    key = (H, cin, cout, k, st)
    if key in seen:
        continue
    seen.add(key)
    pad = k // 2
    Ho = (H + 2 * pad - k) // st + 1
    x = torch.randn(N * H * H * cin, device="cuda")
    w = torch.randn(cout * k * k * cin, device="cuda") * 0.05
    y = torch.empty(N * Ho * Ho * cout, device="cuda")
    flops = 2.0 * N * Ho * Ho * cout * k * k * cin

    kb = int(L.eosv_conv2d_f32_workspace(N, H, H, cin, cout, k, k, st, pad))
    kws = torch.empty(kb // 4 + 4, device="cuda")

    def fwd():
        check(L.eosv_conv2d_f32(x.data_ptr(), N, H, H, cin, w.data_ptr(), cout, k, k, st, pad, None, None, 0,
                                y.data_ptr(), None, 0, s), "conv")

    def fwdk():
        check(L.eosv_conv2d_f32(x.data_ptr(), N, H, H, cin, w.data_ptr(), cout, k, k, st, pad, None, None, 0,
                                y.data_ptr(), kws.data_ptr(), kb, s), "conv")

    def wg():
        wb = int(L.eosv_conv_wgrad_f32_workspace(N, H, H, cin, cout, k, k, st, pad))
        ws = torch.empty(wb // 4 + 4, device="cuda")
        g = torch.empty(cout * k * k * cin, device="cuda")
        return lambda: check(L.eosv_conv_wgrad_f32(x.data_ptr(), N, H, H, cin, y.data_ptr(), cout, k, k, st, pad,
                                                   g.data_ptr(), ws.data_ptr(), wb, s), "wgrad")

    def wgb():
        if k != 1 or st != 1:
            return None
        P = N * Ho * Ho
        wb = int(L.eosv_sgemm_tn_splitk_workspace(cout, cin, P))
        ws = torch.empty(wb // 4 + 4, device="cuda")
        g = torch.empty(cout * cin, device="cuda")
        return lambda: check(L.eosv_sgemm_tn_splitk(cout, cin, P, y.data_ptr(), cout, x.data_ptr(), cin, g.data_ptr(),
                                                    cin, ws.data_ptr(), wb, s), "wgrad_blas")

    out = [name, f"{H}x{H} {cin}->{cout} k{k} s{st}"]
    for tag, fn in (("fwd", fwd), ("fwdk", fwdk), ("wgrad", wg()), ("wgrad_blas", wgb())):
        if fn is None:
            continue
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        tot[tag][0] += ms
        tot[tag][1] += flops
        out.append(f"{tag} {ms*1e3:7.1f} us {flops/ms/1e9:6.1f} TF/s")
    print("  ".join(out), flush=True)
for t, (ms, fl) in tot.items():
    print(f"{t}: {ms:.2f} ms over unique shapes, {fl/ms/1e9:.1f} TF/s")
