"""GPU: the native training step (eosv/train.py) against the reference's
recipe run by torch on the CPU (network_train.py:75-116: model.train(), clip mean over T frames,
fc, CrossEntropyLoss, backward, SGD(momentum=0.9) for convnet and fc).

The oracle is the torch.nn restatement of the reference model (oracle/resnet_ref.py, the same
module the inference parity uses) with torch's own autograd and optimiser, run twice: in f64
(the reference values) and in f32 (the yardstick: what torch's own f32 arithmetic gets).  Both
sides start from the same synthetic state_dict and see the same frames and labels for two
iterations (the second exercises the momentum buffers).

A small batch (8 frames of 96x96, 3x3 maps and 72 BN samples per channel at layer4) makes the
backward ill-conditioned: ResNet-50's gradients below layer4 move by ~4e-3 between torch f32
and f64, and a ReLU whose pre-activation sits within rounding of 0 can flip its mask between
two f32 forwards, which moves a cancelling BN gradient sum by ~1e-2 relative (measured: ResNet-50
layer4.2.bn2).  Bounds: the first loss within 1e-4 relative of f64; the second loss within
max(4 x torch-f32's distance, 1e-4 relative); every gradient of the first step within
max(4 x torch-f32's distance, 2e-2 relative) of f64 (a wrong kernel is off by O(1)); every
parameter / BN running statistic after two steps within max(4 x torch-f32's distance, 1e-5
relative), tensors compared by norm.
"""
import os

import numpy as np
import pytest
import torch

from eosv import arch, synth
from eosv.train import NativeTrainer

pytestmark = pytest.mark.gpu


def _oracle(name, sd, frames, labels, T, lr1, lr2, steps, dtype):
    from oracle.resnet_ref import ModelResNetRef

    m = ModelResNetRef(name, 64)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to(dtype).train()
    o1 = torch.optim.SGD(m.convnet.parameters(), lr=lr1, momentum=0.9)
    o2 = torch.optim.SGD(m.fc.parameters(), lr=lr2, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss()
    B = frames.shape[0] // T
    losses, grads0 = [], None
    for it in range(steps):
        o1.zero_grad()
        o2.zero_grad()
        feature, _ = m(frames.to(dtype))
        feature = feature.view(B, T, -1).mean(dim=1)
        out = m.fc(feature)
        loss = crit(out, torch.as_tensor(labels, dtype=torch.long))
        loss.backward()
        if it == 0:
            grads0 = {k: p.grad.detach().double().clone() for k, p in m.named_parameters()}
        o1.step()
        o2.step()
        losses.append(float(loss.detach()))
    return losses, grads0, m.state_dict()


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_train_step_matches_torch_reference(name):
    torch.manual_seed(0)
    T, B, H = 4, 2, 96
    frames = torch.randn(B * T, 3, H, H)
    labels = [3, 17]
    _check_two_steps(name, frames, labels, T, H)


@pytest.mark.timeout(600)
def test_train_step_reference_shape_resnet50():
    """The reference's own training shape (network_train.py:140,148: batch 6 clips x 16 frames at
    224x224, ResNet-50): two NativeTrainer steps against the f64 replay, with the same f32
    yardstick bounds as the small case (a batch of 96 frames conditions the backward far better,
    so the yardstick is tighter here)."""
    torch.manual_seed(1)
    T, B, H = 16, 6, 224
    frames = torch.randn(B * T, 3, H, H)
    labels = [5, 0, 63, 17, 5, 40]
    torch.set_num_threads(max(1, min(16, len(os.sched_getaffinity(0)))))
    _check_two_steps("resnet50", frames, labels, T, H)


def _check_two_steps(name, frames, labels, T, H):
    lr1, lr2 = 1e-3, 1e-2  # 10x the reference's (network_train.py:140)
    sd = synth.synth_state_dict(arch.SPECS[name], 64, 0)
    ref_losses, ref_g, ref_sd = _oracle(name, sd, frames, labels, T, lr1, lr2, 2, torch.float64)
    f32_losses, f32_g, f32_sd = _oracle(name, sd, frames, labels, T, lr1, lr2, 2, torch.float32)

    tr = NativeTrainer(name, 64, device=0)
    tr.load_state_dict(sd)
    l0, logits = tr.step(frames.cuda(), labels, T, lr1, lr2)
    g0 = tr.grads()
    l1, _ = tr.step(frames.cuda(), labels, T, lr1, lr2)
    print(f"[{name} {tuple(frames.shape)}] loss {l0:.6f} / {ref_losses[0]:.6f}, {l1:.6f} / {ref_losses[1]:.6f}")
    assert abs(l0 - ref_losses[0]) <= 1e-4 * abs(ref_losses[0])
    # the second loss inherits the first step's gradient conditioning: same yardstick
    assert abs(l1 - ref_losses[1]) <= max(4 * abs(f32_losses[1] - ref_losses[1]), 1e-4 * abs(ref_losses[1]))
    worst = (0.0, None, 0.0)
    ratio = (0.0, None)
    for k, gr in ref_g.items():
        norm = max(float(gr.norm()), 1e-12)
        err = float((g0[k].double() - gr).norm()) / norm
        yard = float((f32_g[k] - gr).norm()) / norm
        if err > worst[0]:
            worst = (err, k, yard)
        if yard > 0 and err / yard > ratio[0]:
            ratio = (err / yard, k)
        assert err <= max(4 * yard, 2e-2), (k, err, yard)
    # the tensor behind the worst error and torch-f32's own distance from f64 on it (the yardstick),
    # and the tensor where the native gradient is furthest from f32 relative to that yardstick
    print(f"[{name} {tuple(frames.shape)}] worst relative gradient error {worst[0]:.2e} at {worst[1]} "
          f"(torch-f32 yardstick there {worst[2]:.2e}); largest error / yardstick {ratio[0]:.2f} at {ratio[1]}")
    got = tr.state_dict()
    for k, v in ref_sd.items():
        if k.endswith("num_batches_tracked"):
            assert int(got[k]) == int(v), k
            continue
        v = v.double()
        err = float((got[k].double() - v).norm())
        yard = float((f32_sd[k].double() - v).norm())
        assert err <= max(4 * yard, 1e-6 * v.numel() ** 0.5 + 1e-5 * float(v.norm())), (k, err, yard)


def test_train_kernels_reject_bad_arguments():
    from eosv._lib import EosvError, check, lib

    L = lib()
    x = torch.zeros(16, device="cuda")
    with pytest.raises(EosvError):
        check(L.eosv_im2col(x.data_ptr(), 1, 2, 2, 1, 3, 3, 0, 1, x.data_ptr(), None), "eosv_im2col")
    with pytest.raises(EosvError):
        check(L.eosv_sgemm(0, 0, 2, 2, 2, 1.0, 0, 2, x.data_ptr(), 2, 0.0, x.data_ptr(), 2, None), "eosv_sgemm")
    with pytest.raises(EosvError):
        check(L.eosv_bn_train_forward(x.data_ptr(), 0, 4, x.data_ptr(), x.data_ptr(), 1e-5, 0.1, 0, 0, 0, 1,
                                      x.data_ptr(), None, x.data_ptr(), x.data_ptr(), x.data_ptr(), None),
              "eosv_bn_train_forward")


def test_train_rejects_out_of_range_labels():
    """nn.CrossEntropyLoss (network_train.py:85) raises 'Target out of bounds' for a label outside
    [0, num_classes): NativeTrainer.step raises before launching, and the kernel itself, given such a
    label through the C ABI, returns a NaN loss and a zero gradient row (no out-of-bounds read)."""
    from eosv._lib import check, lib, stream_ptr

    tr = NativeTrainer("resnet18", 5, device=0)
    tr.load_state_dict(synth.synth_state_dict(arch.SPECS["resnet18"], 5, 0))
    frames = torch.randn(2 * 2, 3, 64, 64, device="cuda")
    for bad in ([0, 5], [-1, 0]):
        with pytest.raises(ValueError, match="label out of range"):
            tr.step(frames, bad, 2, 1e-3, 1e-2)
    L = lib()
    B, C = 3, 5
    logits = torch.randn(B, C, device="cuda")
    lab = torch.tensor([1, 7, 4], dtype=torch.int32, device="cuda")
    row_loss = torch.empty(B, device="cuda")
    dlog = torch.full((B, C), 9.0, device="cuda")
    check(L.eosv_softmax_xent(logits.data_ptr(), lab.data_ptr(), B, C, row_loss.data_ptr(), dlog.data_ptr(),
                              stream_ptr()), "eosv_softmax_xent")
    torch.cuda.synchronize()
    assert torch.isnan(row_loss[1]) and torch.isfinite(row_loss[[0, 2]]).all()
    assert (dlog[1] == 0).all()
    ref = torch.softmax(logits[[0, 2]], 1)
    ref[0, 1] -= 1
    ref[1, 4] -= 1
    assert torch.allclose(dlog[[0, 2]], ref / B, atol=1e-6)


def _call(fn, *args):
    from eosv._lib import check, stream_ptr

    check(fn(*args, stream_ptr()), fn.__name__)
    torch.cuda.synchronize()


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k,pad,alpha,beta", [
    (6, 64, 2048, 0, 1.0, 0.0),      # fc logits / input gradient shapes
    (64, 2048, 6, 0, 1.0, 0.0),      # fc weight gradient (k = batch)
    (301, 147, 77, 0, 1.0, 0.0),     # stem-like: ragged m, n and k not multiples of 4 or 16
    (256, 192, 320, 3, 0.5, -2.0),   # padded leading dimensions (scalar path), alpha / beta
    (1000, 128, 256, 0, 1.0, 1.0)])  # several tiles, accumulate into C
def test_sgemm_in_tree_vs_torch(ta, tb, m, n, k, pad, alpha, beta):
    """eosv_sgemm (gemm_f32.hip, exact-f32 MFMA, in place of rocBLAS since r05) for every
    transpose pair against torch f64 matmul: C = alpha op(A) op(B) + beta C, row-major, with
    ragged edges and padded leading dimensions; 1e-5 relative.  Bitwise deterministic over runs."""
    from eosv._lib import lib

    L = lib()
    g = torch.Generator().manual_seed(m * 7 + n + k)
    ar, ac = (k, m) if ta else (m, k)
    br, bc = (n, k) if tb else (k, n)
    A = torch.randn(ar, ac + pad, generator=g, dtype=torch.float64)
    B = torch.randn(br, bc + pad, generator=g, dtype=torch.float64)
    C0 = torch.randn(m, n + pad, generator=g, dtype=torch.float64)
    opA = A[:, :ac].T if ta else A[:, :ac]
    opB = B[:, :bc].T if tb else B[:, :bc]
    ref = alpha * (opA @ opB) + beta * C0[:, :n]
    Ad, Bd = A.float().cuda(), B.float().cuda()
    outs = []
    for _ in range(2):
        Cd = C0.float().cuda()
        _call(L.eosv_sgemm, ta, tb, m, n, k, alpha, Ad.data_ptr(), ac + pad, Bd.data_ptr(), bc + pad, beta,
              Cd.data_ptr(), n + pad)
        outs.append(Cd)
    assert torch.equal(outs[0], outs[1])
    got = outs[0][:, :n].double().cpu()
    assert float((got - ref).norm() / ref.norm()) < 1e-5
    assert torch.equal(outs[0][:, n:].cpu(), C0[:, n:].float())  # padding columns untouched


@pytest.mark.parametrize("m,n,k", [(256, 64, 100352), (64, 147, 37632 + 5), (2048, 1024, 4704)])
def test_sgemm_tn_splitk_vs_torch(m, n, k):
    """The split-K weight-gradient GEMM C = A^T B (reduction over the pixel count, slices summed in
    order) against torch f64: 1e-5 relative, bitwise equal over runs, and equal to the one-slice
    result within 1e-5 (a different summation split)."""
    from eosv._lib import lib

    L = lib()
    g = torch.Generator().manual_seed(k)
    A = torch.randn(k, m, generator=g, dtype=torch.float64)
    B = torch.randn(k, n, generator=g, dtype=torch.float64)
    ref = A.T @ B
    Ad, Bd = A.float().cuda(), B.float().cuda()
    wb = int(L.eosv_sgemm_tn_splitk_workspace(m, n, k))
    assert wb > 0
    ws = torch.empty(wb // 4 + 4, device="cuda")
    outs = []
    for _ in range(2):
        C = torch.empty(m, n, device="cuda")
        _call(L.eosv_sgemm_tn_splitk, m, n, k, Ad.data_ptr(), m, Bd.data_ptr(), n, C.data_ptr(), n, ws.data_ptr(), wb)
        outs.append(C)
    assert torch.equal(outs[0], outs[1])
    assert float((outs[0].double().cpu() - ref).norm() / ref.norm()) < 1e-5
    one = torch.empty(m, n, device="cuda")
    _call(L.eosv_sgemm_tn_splitk, m, n, k, Ad.data_ptr(), m, Bd.data_ptr(), n, one.data_ptr(), n, ws.data_ptr(), 0)
    assert float((one - outs[0]).norm() / outs[0].norm()) < 1e-5


@pytest.mark.parametrize("k,stride,pad,cin,cout", [(3, 1, 1, 8, 16), (3, 2, 1, 8, 16), (1, 2, 0, 16, 8), (7, 2, 3, 3, 8)])
def test_conv_forward_and_gradients_vs_torch(k, stride, pad, cin, cout):
    """im2col + eosv_sgemm forward, weight gradient and col2im input gradient against torch
    autograd in f64 on well-conditioned random data (no BN, no ReLU): 1e-5 relative."""
    from eosv._lib import lib

    L = lib()
    torch.manual_seed(1)
    N, H, W = 2, 9, 11
    x = torch.randn(N, cin, H, W, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cout, cin, k, k, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, stride=stride, padding=pad)
    dy = torch.randn_like(y)
    y.backward(dy)
    Ho, Wo = y.shape[2], y.shape[3]
    P, K = N * Ho * Wo, k * k * cin
    xd = x.detach().permute(0, 2, 3, 1).contiguous().float().cuda()
    wd = w.detach().permute(0, 2, 3, 1).reshape(cout, K).contiguous().float().cuda()
    dyd = dy.permute(0, 2, 3, 1).reshape(P, cout).contiguous().float().cuda()
    col = torch.empty(P * K, device="cuda")
    _call(L.eosv_im2col, xd.data_ptr(), N, H, W, cin, k, k, stride, pad, col.data_ptr())
    yd = torch.empty(P * cout, device="cuda")
    _call(L.eosv_sgemm, 0, 1, P, cout, K, 1.0, col.data_ptr(), K, wd.data_ptr(), K, 0.0, yd.data_ptr(), cout)
    gw = torch.empty(cout * K, device="cuda")
    _call(L.eosv_sgemm, 1, 0, cout, K, P, 1.0, dyd.data_ptr(), cout, col.data_ptr(), K, 0.0, gw.data_ptr(), K)
    dcol = torch.empty(P * K, device="cuda")
    _call(L.eosv_sgemm, 0, 0, P, K, cout, 1.0, dyd.data_ptr(), cout, wd.data_ptr(), K, 0.0, dcol.data_ptr(), K)
    gx = torch.empty(N * H * W * cin, device="cuda")
    _call(L.eosv_col2im, dcol.data_ptr(), N, H, W, cin, k, k, stride, pad, gx.data_ptr())

    def rel(a, b):
        return float((a.double().cpu() - b).norm() / b.norm())

    assert rel(yd.view(N, Ho, Wo, cout).permute(0, 3, 1, 2), y.detach()) < 1e-5
    assert rel(gw.view(cout, k, k, cin).permute(0, 3, 1, 2), w.grad) < 1e-5
    assert rel(gx.view(N, H, W, cin).permute(0, 3, 1, 2), x.grad) < 1e-5


@pytest.mark.parametrize("k,stride,cin,cout,H", [(3, 1, 64, 64, 56), (3, 1, 128, 64, 14), (1, 1, 64, 256, 28),
                                                 (3, 2, 64, 128, 28), (1, 2, 256, 512, 14), (3, 1, 128, 256, 13),
                                                 (3, 2, 256, 512, 15), (1, 1, 256, 64, 28), (1, 1, 64, 128, 14),
                                                 (1, 1, 128, 64, 14)])
def test_native_conv_and_flipped_dgrad_vs_torch(k, stride, cin, cout, H):
    """The trainer's fast paths: eosv_conv2d_f32 forward (the inference conv kernels, exact f32),
    the stride-1 input gradient as a conv of dY with eosv_flip_weights' weights, the split-K
    weight gradient eosv_sgemm_tn_splitk (ragged last slice) and the implicit-GEMM one
    eosv_conv_wgrad_f32 (KxK; both tile shapes, stride 2, ragged last slice), against f64
    autograd."""
    from eosv._lib import lib

    L = lib()
    torch.manual_seed(2)
    N, pad = 3, k // 2
    x = torch.randn(N, cin, H, H, dtype=torch.float64, requires_grad=True)
    w = torch.randn(cout, cin, k, k, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.conv2d(x, w, stride=stride, padding=pad)
    dy = torch.randn_like(y)
    y.backward(dy)
    Ho, Wo = y.shape[2], y.shape[3]
    P, K = N * Ho * Wo, k * k * cin
    xd = x.detach().permute(0, 2, 3, 1).contiguous().float().cuda()
    wd = w.detach().permute(0, 2, 3, 1).reshape(cout, K).contiguous().float().cuda()
    dyd = dy.permute(0, 2, 3, 1).reshape(P, cout).contiguous().float().cuda()

    def rel(a, b):
        return float((a.double().cpu() - b).norm() / b.norm())

    yd = torch.empty(P * cout, device="cuda")
    _call(L.eosv_conv2d_f32, xd.data_ptr(), N, H, H, cin, wd.data_ptr(), cout, k, k, stride, pad, None, None, 0,
          yd.data_ptr(), None, 0)
    assert rel(yd.view(N, Ho, Wo, cout).permute(0, 3, 1, 2), y.detach()) < 1e-5
    # with a workspace: split-K over slices (small grids), same result within f32 rounding
    kb = int(L.eosv_conv2d_f32_workspace(N, H, H, cin, cout, k, k, stride, pad))
    kws = torch.empty(kb // 4 + 4, device="cuda")
    yk = torch.full_like(yd, float("nan"))
    _call(L.eosv_conv2d_f32, xd.data_ptr(), N, H, H, cin, wd.data_ptr(), cout, k, k, stride, pad, None, None, 0,
          yk.data_ptr(), kws.data_ptr(), kb)
    assert rel(yk.view(N, Ho, Wo, cout).permute(0, 3, 1, 2), y.detach()) < 1e-5
    col = torch.empty(P * K, device="cuda")
    _call(L.eosv_im2col, xd.data_ptr(), N, H, H, cin, k, k, stride, pad, col.data_ptr())
    wb = int(L.eosv_sgemm_tn_splitk_workspace(cout, K, P))
    ws = torch.empty(wb // 4 + 1, device="cuda")
    gw = torch.empty(cout * K, device="cuda")
    _call(L.eosv_sgemm_tn_splitk, cout, K, P, dyd.data_ptr(), cout, col.data_ptr(), K, gw.data_ptr(), K,
          ws.data_ptr(), wb)
    assert rel(gw.view(cout, k, k, cin).permute(0, 3, 1, 2), w.grad) < 1e-5
    # the implicit-GEMM weight gradient (no im2col buffer; every tile shape across the cases)
    wb = int(L.eosv_conv_wgrad_f32_workspace(N, H, H, cin, cout, k, k, stride, pad))
    ws = torch.empty(wb // 4 + 4, device="cuda")
    gw2 = torch.full((cout * K,), float("nan"), device="cuda")
    _call(L.eosv_conv_wgrad_f32, xd.data_ptr(), N, H, H, cin, dyd.data_ptr(), cout, k, k, stride, pad,
          gw2.data_ptr(), ws.data_ptr(), wb)
    assert rel(gw2.view(cout, k, k, cin).permute(0, 3, 1, 2), w.grad) < 1e-5
    if stride == 1:
        wf = torch.empty(cout * K, device="cuda")
        _call(L.eosv_flip_weights, wd.data_ptr(), cout, k, k, cin, wf.data_ptr())
        gx = torch.empty(N * H * H * cin, device="cuda")
        _call(L.eosv_conv2d_f32, dyd.data_ptr(), N, Ho, Wo, cout, wf.data_ptr(), cin, k, k, 1, pad, None, None, 0,
              gx.data_ptr(), None, 0)
        assert rel(gx.view(N, H, H, cin).permute(0, 3, 1, 2), x.grad) < 1e-5
        # the shortcut's gradient fused as the epilogue residual (the trainer's first-conv dgrad)
        sk = torch.randn(N, H, H, cin, dtype=torch.float64)
        skd = sk.float().cuda().contiguous()
        kb = int(L.eosv_conv2d_f32_workspace(N, Ho, Wo, cout, cin, k, k, 1, pad))
        kws = torch.empty(kb // 4 + 4, device="cuda")
        for ws, wsb in ((None, 0), (kws.data_ptr(), kb)):
            _call(L.eosv_conv2d_f32, dyd.data_ptr(), N, Ho, Wo, cout, wf.data_ptr(), cin, k, k, 1, pad, None,
                  skd.data_ptr(), 0, gx.data_ptr(), ws, wsb)
            assert rel(gx.view(N, H, H, cin).permute(0, 3, 1, 2), x.grad + sk.permute(0, 3, 1, 2)) < 1e-5


@pytest.mark.parametrize("shape", [(3, 40, 5, 7), (4, 256, 41, 43), (2, 6, 5, 7)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, True)])
@pytest.mark.parametrize("mask,want_dres", [(False, True), (True, True), (True, False)])
def test_batchnorm_train_forward_backward_vs_torch(relu, res, shape, mask, want_dres):
    """eosv_bn_train_forward / _backward against nn.BatchNorm2d in train mode (f64 autograd):
    output, saved statistics, running estimates, dx, dgamma, dbeta, residual gradient.  The
    second shape (7052 rows) gives every lane several 4-row groups and a ragged tail; the third
    (C = 6) takes the scalar kernels.  mask: the forward writes the ReLU mask bytes (checked equal
    to y > 0) and the backward reads them with no y at all; want_dres: with the residual gradient
    written, dx reads it in place of dy and the mask."""
    from eosv._lib import lib

    L = lib()
    torch.manual_seed(2)
    N, C, H, W = shape
    P = N * H * W
    x = torch.randn(N, C, H, W, dtype=torch.float64, requires_grad=True) * 2 + 0.5
    x.retain_grad()
    r = torch.randn(N, C, H, W, dtype=torch.float64, requires_grad=True)
    bn = torch.nn.BatchNorm2d(C).double().train()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C) + 0.5)
        bn.bias.copy_(torch.randn(C))
        bn.running_mean.copy_(torch.randn(C))
        bn.running_var.copy_(torch.rand(C) + 0.5)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    y = bn(x) + (r if res else 0)
    if relu:
        y = torch.relu(y)
    dy = torch.randn_like(y)
    y.backward(dy)
    nhwc = lambda t: t.detach().permute(0, 2, 3, 1).reshape(P, C).contiguous().float().cuda()  # noqa: E731
    xd, rd, dyd = nhwc(x), nhwc(r), nhwc(dy)
    g, b = bn.weight.detach().float().cuda(), bn.bias.detach().float().cuda()
    rm, rv = rm0.float().cuda(), rv0.float().cuda()
    yd, mean, inv = torch.empty_like(xd), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    work = torch.empty(int(L.eosv_bn_workspace_bytes(C)) // 4 + 4, device="cuda")
    mk = torch.full((P * C,), 7, dtype=torch.uint8, device="cuda") if mask else None
    _call(L.eosv_bn_train_forward, xd.data_ptr(), P, C, g.data_ptr(), b.data_ptr(), 1e-5, 0.1, rm.data_ptr(),
          rv.data_ptr(), rd.data_ptr() if res else 0, int(relu), yd.data_ptr(), mk.data_ptr() if mask else None,
          mean.data_ptr(), inv.data_ptr(), work.data_ptr())
    if mask and relu:
        assert torch.equal(mk.view(P, C).bool(), yd > 0) and int(mk.max()) == 1
    dx, dg, db = torch.empty_like(xd), torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    dres = torch.empty_like(xd) if want_dres else None
    _call(L.eosv_bn_train_backward, dyd.data_ptr(), None if (mask and relu) else yd.data_ptr(),
          mk.data_ptr() if mask else None, int(relu), xd.data_ptr(), P, C, g.data_ptr(), mean.data_ptr(),
          inv.data_ptr(), dx.data_ptr(), dg.data_ptr(), db.data_ptr(), dres.data_ptr() if want_dres else None,
          work.data_ptr())

    def rel(a, bref):
        return float((a.double().cpu() - bref).norm() / bref.norm())

    back = lambda t: t.view(N, H, W, C).permute(0, 3, 1, 2)  # noqa: E731
    assert rel(back(yd), y.detach()) < 1e-6
    assert rel(rm, bn.running_mean) < 1e-6 and rel(rv, bn.running_var) < 1e-6
    assert rel(back(dx), x.grad) < 1e-5
    assert rel(dg, bn.weight.grad) < 1e-5 and rel(db, bn.bias.grad) < 1e-5
    if res and want_dres:
        assert rel(back(dres), r.grad) < 1e-6


def test_train_r05_passes_bitwise_equal_r04():
    """The r05 training passes against the r04 ones (EOSV_TRAIN_R04=1) on R50-shaped and ragged
    inputs, every output bitwise equal (tools/train_r05_check.py, profiling build, which reads the
    switch per call): the batch-norm statistics with 4 rows per lane loaded ahead, im2col with
    16-byte stores, col2im over four channels per lane."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "embodied-one-shot-video-recognition_amd", "libeosv_prof.so")
    if not os.path.exists(prof):
        pytest.fail("libeosv_prof.so missing: run __graft_entry__.build()")
    r = subprocess.run([sys.executable, os.path.join(repo, "tools", "train_r05_check.py")],
                       env=dict(os.environ, EOSV_LIBRARY=prof), capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "0 differing" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("C", [5, 12])  # scalar and float4 kernels
def test_maxpool_forward_backward_vs_torch(C):
    from eosv._lib import lib

    L = lib()
    torch.manual_seed(3)
    N, H, W = 2, 9, 8
    x = torch.randn(N, C, H, W, dtype=torch.float64, requires_grad=True)
    y = torch.nn.functional.max_pool2d(x, 3, 2, 1)
    dy = torch.randn_like(y)
    y.backward(dy)
    Ho, Wo = y.shape[2], y.shape[3]
    xd = x.detach().permute(0, 2, 3, 1).contiguous().float().cuda()
    yd = torch.empty(N * Ho * Wo * C, device="cuda")
    idx = torch.empty(N * Ho * Wo * C, dtype=torch.int32, device="cuda")
    _call(L.eosv_maxpool_forward, xd.data_ptr(), N, H, W, C, yd.data_ptr(), idx.data_ptr())
    dyd = dy.permute(0, 2, 3, 1).contiguous().float().cuda()
    dx = torch.empty(N * H * W * C, device="cuda")
    _call(L.eosv_maxpool_backward, dyd.data_ptr(), idx.data_ptr(), N, H, W, C, dx.data_ptr())
    assert torch.equal(yd.view(N, Ho, Wo, C).permute(0, 3, 1, 2).cpu(), y.detach().float())
    # the argmax is torch CPU's (first maximum in window order)
    ref_idx = torch.nn.functional.max_pool2d(x.detach(), 3, 2, 1, return_indices=True)[1]
    assert torch.equal(idx.view(N, Ho, Wo, C).permute(0, 3, 1, 2).cpu().long(), ref_idx)
    assert torch.allclose(dx.view(N, H, W, C).permute(0, 3, 1, 2).double().cpu(), x.grad, rtol=0, atol=1e-6)


def test_dropin_train_network_checkpoints_follow_reference(tmp_path, monkeypatch):
    """The drop-in TrainNetwork.finetune_model (network_train.py:52-131) over a 4-video train list,
    2 epochs of 2 batches, StepLR(step_size=1): every batch the native step sees is recorded and
    replayed through the torch reference (f64 and f32, SGD momentum, the same lr schedule); the
    epoch-2 checkpoint must match it under the bounds of test_train_step_matches_torch_reference."""
    import network_train
    import utils
    from eosv import train as etrain

    lines = [l for l in open(utils.TRAIN_LIST).read().splitlines() if l][:2] + \
            [l for l in open(utils.TRAIN_LIST).read().splitlines() if l][-2:]
    lst = tmp_path / "train.list"
    lst.write_text("\n".join(lines) + "\n")
    monkeypatch.setattr(utils, "IMG_crop_size", (64, 64))
    monkeypatch.setattr(network_train, "TRAIN_LIST", str(lst))
    rec = []
    step0 = etrain.NativeTrainer.step

    def step(self, frames, labels, T, lr_conv, lr_fc, momentum=0.9):
        rec.append((frames.detach().cpu().clone(), list(np.asarray(labels).reshape(-1)), T, lr_conv, lr_fc))
        return step0(self, frames, labels, T, lr_conv, lr_fc, momentum)

    monkeypatch.setattr(etrain.NativeTrainer, "step", step)
    torch.manual_seed(5)
    tn = network_train.TrainNetwork(str(tmp_path / "loss.txt"), str(tmp_path) + "/ckp/", 2, 2, 1e-3, 1e-2,
                                    lr_step_size=1, resnet_model="resnet18")
    init = {k: v.detach().cpu().clone() for k, v in tn.mymodel.state_dict().items()}
    tn.finetune_model()
    assert len(rec) == 4 and np.allclose([r[3] for r in rec], [1e-4, 1e-4, 1e-5, 1e-5], rtol=1e-12, atol=0)
    got = torch.load(str(tmp_path / "ckp" / "model2.pkl"), weights_only=True)
    assert (tmp_path / "ckp" / "model1.pkl").exists()

    from oracle.resnet_ref import ModelResNetRef

    def replay(dtype):
        m = ModelResNetRef("resnet18", 64)
        m.load_state_dict(init)
        m = m.to(dtype).train()
        o1 = torch.optim.SGD(m.convnet.parameters(), lr=1e-3, momentum=0.9)
        o2 = torch.optim.SGD(m.fc.parameters(), lr=1e-2, momentum=0.9)
        for frames, labels, T, l1, l2 in rec:
            for g in o1.param_groups:
                g["lr"] = l1
            for g in o2.param_groups:
                g["lr"] = l2
            o1.zero_grad()
            o2.zero_grad()
            f, _ = m(frames.to(dtype))
            out = m.fc(f.view(len(labels), T, -1).mean(dim=1))
            torch.nn.CrossEntropyLoss()(out, torch.as_tensor(labels, dtype=torch.long)).backward()
            o1.step()
            o2.step()
        return m.state_dict()

    ref, f32 = replay(torch.float64), replay(torch.float32)
    for k, v in ref.items():
        if k.endswith("num_batches_tracked"):
            assert int(got[k]) == int(v), k
            continue
        v = v.double()
        err = float((got[k].double() - v).norm())
        yard = float((f32[k].double() - v).norm())
        assert err <= max(4 * yard, 1e-6 * v.numel() ** 0.5 + 1e-5 * float(v.norm())), (k, err, yard)


@pytest.mark.parametrize("tag", ["train_r18_t8_96", "train_r50_t8_96"])
def test_train_loop_matches_reference_fixture(tag, golden_dir):
    """The native step replayed over the batches the reference's own finetune_model consumed
    (tests/golden/train_*.json, capture_golden.py --train: 2 epochs x 3 batches of 2 clips x 8
    frames at 96x96, StepLR(1) so the second epoch runs at the decayed rate), with the drop-in
    TrainNetwork's schedule.  Truth: the restated loop (oracle/train_ref.py, bit-identical to the
    reference in f32 -- tests/test_oracle_golden.py) run in f64; yardstick: the reference's own f32
    run.  Every loss within max(4 x the reference's distance, 1e-4 relative); every checkpoint
    tensor's update (final - initial) within max(4 x the reference's distance, 2e-2 of the
    update's norm), distances as norms (the reference's estimated from the fixture's 8 random
    projections of its update: E (r.d)^2 = |d|^2); num_batches_tracked equal."""
    import json
    import os
    import types

    from network_train import TrainNetwork
    from oracle import train_ref

    meta = json.load(open(os.path.join(golden_dir, tag + ".json")))
    sd0 = synth.synth_state_dict(arch.SPECS[meta["arch"]], meta["num_classes"], meta["init_seed"])
    truth_losses, truth_states = train_ref.train_replay(meta, sd0, torch.float64)
    tr = NativeTrainer(meta["arch"], meta["num_classes"], device=0)
    tr.load_state_dict(sd0)
    sched = types.SimpleNamespace(lr_1=meta["lr_1"], lr_2=meta["lr_2"], lr_step_size=meta["step_size"])
    k, worst = 0, 0.0
    # margins: the largest fraction of its bound any loss / any update error used
    loss_use, state_use = (0.0, None), (0.0, None)
    for e, ep in enumerate(meta["epochs_data"]):
        lr1, lr2 = TrainNetwork.lr_at(sched, e)
        for it in ep["iterations"]:
            frames = train_ref.batch_frames(it, meta["H"], meta["W"])
            loss, _ = tr.step(frames.cuda(), it["labels"], meta["T"], lr1, lr2)
            t = truth_losses[k]
            bound = max(4 * abs(it["loss"] - t), 1e-4 * abs(t))
            if abs(loss - t) / bound > loss_use[0]:
                loss_use = (abs(loss - t) / bound, (e, k, abs(loss - t), abs(it["loss"] - t)))
            assert abs(loss - t) <= bound, (e, k, loss, t, it["loss"])
            k += 1
        got = tr.state_dict()
        for i, key in enumerate(ep["state"]):
            st = ep["state"][key]
            if key.endswith("num_batches_tracked"):
                assert int(got[key]) == st, key
                continue
            init = torch.as_tensor(np.asarray(sd0[key])).double()
            d_truth = truth_states[e][key].double() - init
            p_truth = np.asarray(train_ref.projections(d_truth, i))
            yard = float(np.sqrt(np.mean((np.asarray(st["dproj8"]) - p_truth) ** 2)))
            tn = float(d_truth.norm())
            err = float((got[key].double() - init - d_truth).norm())
            worst = max(worst, err / max(tn, 1e-30))
            bound = max(4 * yard, 2e-2 * tn) + 1e-12
            if err / bound > state_use[0]:
                state_use = (err / bound, (e, key))
            assert err <= bound, (e, key, err, yard, tn)
    print(f"[{tag}] worst update error {worst:.2e} of the update's norm; bound use: loss "
          f"{loss_use[0]:.3f} (epoch, step, |native - f64|, |reference f32 - f64| = {loss_use[1]}), "
          f"update {state_use[0]:.3f} ({state_use[1]})")
