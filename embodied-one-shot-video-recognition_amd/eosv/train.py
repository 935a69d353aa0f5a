"""Native training step for TrainNetwork.finetune_model.

Restates one iteration of the reference's loop (network_train.py:86-116) on the device:

    feature, output = model(video)                  # ResNet in train mode: batch-statistics BN
    feature = feature.view(b, T, -1).mean(dim=1)    # :100, :110
    output = model.fc(feature); loss = CrossEntropyLoss()(output, label)
    loss.backward(); optimizer_1.step(); optimizer_2.step()   # SGD(momentum=0.9): convnet / fc

with the f32 kernels of csrc/train.hip behind the C ABI (eosv_sgemm, eosv_im2col,
eosv_bn_train_forward, ...).  PyTorch only provides the device buffers; every arithmetic step
is a library call, and there is no CPU path.  Layouts: activations NHWC ([P][C] rows), conv
weights [Cout][KH][KW][Cin] (the state_dict's [Cout][Cin][KH][KW] permuted at load / export).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from . import arch as _arch
from ._lib import check, lib, ptr, stream_ptr

BN_EPS = 1e-5
_UNSUPPORTED = -4  # EOSV_ERR_UNSUPPORTED
BN_MOMENTUM = 0.1


def _f(t):
    return ptr(t)


@dataclass
class _Conv:
    name: str
    cin: int
    cout: int
    k: int
    stride: int
    pad: int
    w: torch.Tensor = None      # [Cout][K] with K = (kh, kw, cin)
    g: torch.Tensor = None
    buf: torch.Tensor = None

    @property
    def K(self):
        return self.k * self.k * self.cin


@dataclass
class _BN:
    name: str
    c: int
    gamma: torch.Tensor = None
    beta: torch.Tensor = None
    rm: torch.Tensor = None
    rv: torch.Tensor = None
    nbt: int = 0
    dgamma: torch.Tensor = None
    dbeta: torch.Tensor = None
    buf_g: torch.Tensor = None
    buf_b: torch.Tensor = None


@dataclass
class _Block:
    convs: List[_Conv]
    bns: List[_BN]
    ds: Optional[_Conv] = None
    ds_bn: Optional[_BN] = None
    saved: Dict[str, object] = field(default_factory=dict)


class NativeTrainer:
    """ResNet-18/50 + fc trained with the reference's recipe (network_train.py:75-79)."""

    def __init__(self, arch: str = "resnet50", num_classes: int = 64, device: int = 0):
        self.spec = _arch.SPECS[arch]
        self.num_classes = num_classes
        self.dev = torch.device("cuda", device)
        self.L = lib()
        self.stem = _Conv("convnet.0", 3, 64, 7, 2, 3)
        self.stem_bn = _BN("convnet.1", 64)
        self.blocks: List[_Block] = []
        inplanes = 64
        for li, (planes, n) in enumerate(zip((64, 128, 256, 512), self.spec.layers)):
            for bi in range(n):
                stride = 2 if (li > 0 and bi == 0) else 1
                p = f"convnet.{4 + li}.{bi}"
                if self.spec.block == "basic":
                    convs = [_Conv(p + ".conv1", inplanes, planes, 3, stride, 1),
                             _Conv(p + ".conv2", planes, planes, 3, 1, 1)]
                    bns = [_BN(p + ".bn1", planes), _BN(p + ".bn2", planes)]
                else:
                    convs = [_Conv(p + ".conv1", inplanes, planes, 1, 1, 0),
                             _Conv(p + ".conv2", planes, planes, 3, stride, 1),
                             _Conv(p + ".conv3", planes, planes * 4, 1, 1, 0)]
                    bns = [_BN(p + ".bn1", planes), _BN(p + ".bn2", planes), _BN(p + ".bn3", planes * 4)]
                cout = planes * self.spec.expansion
                blk = _Block(convs, bns)
                if bi == 0 and (stride != 1 or inplanes != cout):
                    blk.ds = _Conv(p + ".downsample.0", inplanes, cout, 1, stride, 0)
                    blk.ds_bn = _BN(p + ".downsample.1", cout)
                self.blocks.append(blk)
                inplanes = cout
        self.D = inplanes
        self.fc_w = self.fc_b = None
        self.step_count = 0
        self._scratch: Dict[str, torch.Tensor] = {}
        self._col_key = None  # what the "col" scratch holds (_im2col); reset by every step
        # the BN backward's ReLU mask from 1-byte forward masks (r05) or from y (EOSV_TRAIN_RELU_MASK=0, A/B)
        self._relu_mask = os.environ.get("EOSV_TRAIN_RELU_MASK", "1") != "0"
        self.work = torch.empty(int(self.L.eosv_bn_workspace_bytes(2048)) // 4 + 4, dtype=torch.float32,
                                device=self.dev)

    # ------------------------------------------------------------------ parameters
    def _convs(self):
        yield self.stem
        for b in self.blocks:
            yield from b.convs
            if b.ds is not None:
                yield b.ds

    def _bns(self):
        yield self.stem_bn
        for b in self.blocks:
            yield from b.bns
            if b.ds_bn is not None:
                yield b.ds_bn

    def load_state_dict(self, sd: Dict[str, object]):
        """The reference model's state_dict (numpy arrays or tensors, any device)."""
        def t(name):
            v = sd[name]
            v = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.asarray(v))
            return v.detach().to(self.dev, torch.float32).contiguous()

        # optimizer_1's parameters (convnet: conv weights, BN gamma / beta) live in one flat buffer
        # (each tensor 16-byte aligned), with flat gradient and momentum buffers: one SGD launch
        sizes = [c.cout * c.K for c in self._convs()] + [b.c for b in self._bns() for _ in range(2)]
        total = sum((n + 3) // 4 * 4 for n in sizes)
        self.p_flat = torch.zeros(total, dtype=torch.float32, device=self.dev)
        self.g_flat = torch.zeros_like(self.p_flat)
        self.m_flat = torch.zeros_like(self.p_flat)
        off = [0]

        def views(n):
            o = off[0]
            off[0] += (n + 3) // 4 * 4
            return self.p_flat[o:o + n], self.g_flat[o:o + n], self.m_flat[o:o + n]

        for c in self._convs():
            w = t(c.name + ".weight")                       # [Cout][Cin][KH][KW]
            p, g, m = views(c.cout * c.K)
            p.copy_(w.permute(0, 2, 3, 1).reshape(-1))
            c.w, c.g, c.buf = p.view(c.cout, c.K), g.view(c.cout, c.K), m.view(c.cout, c.K)
        for b in self._bns():
            b.gamma, b.dgamma, b.buf_g = views(b.c)
            b.beta, b.dbeta, b.buf_b = views(b.c)
            b.gamma.copy_(t(b.name + ".weight"))
            b.beta.copy_(t(b.name + ".bias"))
            b.rm, b.rv = t(b.name + ".running_mean"), t(b.name + ".running_var")
            nbt = sd.get(b.name + ".num_batches_tracked", 0)
            b.nbt = int(nbt.item() if isinstance(nbt, torch.Tensor) else np.asarray(nbt))
        self.fc_w, self.fc_b = t("fc.weight"), t("fc.bias")
        self.fc_gw, self.fc_gb = torch.zeros_like(self.fc_w), torch.zeros_like(self.fc_b)
        self.fc_bw, self.fc_bb = torch.zeros_like(self.fc_w), torch.zeros_like(self.fc_b)
        self.step_count = 0

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """The reference's state_dict layout, on the CPU (torch.save, network_train.py:131)."""
        out = {}
        for c in self._convs():
            out[c.name + ".weight"] = c.w.view(c.cout, c.k, c.k, c.cin).permute(0, 3, 1, 2).contiguous().cpu()
        for b in self._bns():
            out[b.name + ".weight"] = b.gamma.cpu()
            out[b.name + ".bias"] = b.beta.cpu()
            out[b.name + ".running_mean"] = b.rm.cpu()
            out[b.name + ".running_var"] = b.rv.cpu()
            out[b.name + ".num_batches_tracked"] = torch.tensor(b.nbt, dtype=torch.int64)
        out["fc.weight"] = self.fc_w.cpu()
        out["fc.bias"] = self.fc_b.cpu()
        return out

    # ------------------------------------------------------------------ building blocks
    def _buf(self, key, n):
        t = self._scratch.get(key)
        if t is None or t.numel() < n:
            t = torch.empty(n, dtype=torch.float32, device=self.dev)
            self._scratch[key] = t
        return t[:n]

    def _im2col(self, x, shape, c: _Conv, P, s):
        """The explicit im2col buffer of conv c over x (the stem: Cin = 3).  The forward's buffer is
        kept and the weight gradient of the same step reuses it instead of gathering it again
        (r05: 0.71 GB and one 0.2 ms pass per step at R50 / 96 frames): every write of the
        buffer goes through here and records what it holds."""
        col = self._buf("col", P * c.K)
        key = (id(c), x.data_ptr(), tuple(shape), col.data_ptr())
        if self._col_key != key:
            N, H, W, _ = shape
            check(self.L.eosv_im2col(_f(x), N, H, W, c.cin, c.k, c.k, c.stride, c.pad, _f(col), s), "eosv_im2col")
            self._col_key = key
        return col

    def _conv_fwd(self, x, shape, c: _Conv, s):
        N, H, W, _ = shape
        Ho, Wo = (H + 2 * c.pad - c.k) // c.stride + 1, (W + 2 * c.pad - c.k) // c.stride + 1
        P = N * Ho * Wo
        y = torch.empty(P * c.cout, dtype=torch.float32, device=self.dev)
        # the inference conv kernels (exact-f32 MFMA) where they apply, else im2col + the in-tree GEMM
        kb = int(self.L.eosv_conv2d_f32_workspace(N, H, W, c.cin, c.cout, c.k, c.k, c.stride, c.pad))
        kw = self._buf("ksplit", kb // 4 + 4)
        rc = self.L.eosv_conv2d_f32(_f(x), N, H, W, c.cin, _f(c.w), c.cout, c.k, c.k, c.stride, c.pad, None, None, 0,
                                    _f(y), _f(kw), kb, s)
        if rc == _UNSUPPORTED:
            if c.k == 1 and c.stride == 1:
                col = x
            else:
                col = self._im2col(x, shape, c, P, s)
            check(self.L.eosv_sgemm(0, 1, P, c.cout, c.K, 1.0, _f(col), c.K, _f(c.w), c.K, 0.0, _f(y), c.cout, s),
                  "eosv_sgemm")
        else:
            check(rc, "eosv_conv2d_f32")
        return y, (N, Ho, Wo, c.cout)

    def _conv_bwd(self, dz, x, shape, c: _Conv, s, need_dx=True, acc=None):
        """dW = dz^T . col(x); returns dx = col2im(dz . W) (NHWC, shape of x) when need_dx, plus
        acc (same shape) when given -- fused into the conv epilogue on the fast path."""
        N, H, W, _ = shape
        Ho, Wo = (H + 2 * c.pad - c.k) // c.stride + 1, (W + 2 * c.pad - c.k) // c.stride + 1
        P = N * Ho * Wo
        direct = c.k == 1 and c.stride == 1
        rc = _UNSUPPORTED
        if c.cin % 4 == 0 and not direct:
            # KxK and strided 1x1: implicit-GEMM weight gradient (no im2col buffer).  Stride-1 1x1
            # convs take the plain split-K GEMM (X is already its operand: gemm_f32.hip TN)
            wb = int(self.L.eosv_conv_wgrad_f32_workspace(N, H, W, c.cin, c.cout, c.k, c.k, c.stride, c.pad))
            ws = self._buf("splitk", wb // 4 + 4)
            rc = self.L.eosv_conv_wgrad_f32(_f(x), N, H, W, c.cin, _f(dz), c.cout, c.k, c.k, c.stride, c.pad, _f(c.g),
                                            _f(ws), wb, s)
        if rc == _UNSUPPORTED:
            if direct:
                col = x
            else:
                col = self._im2col(x, shape, c, P, s)
            wb = int(self.L.eosv_sgemm_tn_splitk_workspace(c.cout, c.K, P))
            ws = self._buf("splitk", wb // 4 + 1)
            check(self.L.eosv_sgemm_tn_splitk(c.cout, c.K, P, _f(dz), c.cout, _f(col), c.K, _f(c.g), c.K, _f(ws), wb,
                                              s), "eosv_sgemm_tn_splitk")
        else:
            check(rc, "eosv_conv_wgrad_f32")
        if not need_dx:
            return None
        dx = torch.empty(N * H * W * c.cin, dtype=torch.float32, device=self.dev)
        if c.stride == 1 and c.k % 2 == 1 and c.pad == c.k // 2:
            # stride 1: dx = conv(dz, W flipped and transposed) on the inference conv kernels
            wf = self._buf("wflip", c.cout * c.K)
            check(self.L.eosv_flip_weights(_f(c.w), c.cout, c.k, c.k, c.cin, _f(wf), s), "eosv_flip_weights")
            kb = int(self.L.eosv_conv2d_f32_workspace(N, Ho, Wo, c.cout, c.cin, c.k, c.k, 1, c.pad))
            kw = self._buf("ksplit", kb // 4 + 4)
            rc = self.L.eosv_conv2d_f32(_f(dz), N, Ho, Wo, c.cout, _f(wf), c.cin, c.k, c.k, 1, c.pad, None, _f(acc),
                                        0, _f(dx), _f(kw), kb, s)
            if rc != _UNSUPPORTED:
                check(rc, "eosv_conv2d_f32")
                return dx
        dcol = dx if direct else self._buf("dcol", P * c.K)
        check(self.L.eosv_sgemm(0, 0, P, c.K, c.cout, 1.0, _f(dz), c.cout, _f(c.w), c.K, 0.0, _f(dcol), c.K, s),
              "eosv_sgemm")
        if not direct:
            check(self.L.eosv_col2im(_f(dcol), N, H, W, c.cin, c.k, c.k, c.stride, c.pad, _f(dx), s), "eosv_col2im")
        if acc is not None:
            check(self.L.eosv_axpy(_f(dx), _f(acc), dx.numel(), 1.0, s), "eosv_axpy")
        return dx

    def _bn_fwd(self, z, P, b: _BN, relu, res, s):
        """Returns y and the backward's saved state: mean, 1/std and, with the ReLU, its mask (one
        byte per element: the backward reads it instead of y, r05)."""
        y = torch.empty_like(z)
        mean = torch.empty(b.c, dtype=torch.float32, device=self.dev)
        invstd = torch.empty_like(mean)
        mask = torch.empty(z.numel(), dtype=torch.uint8, device=self.dev) if relu and self._relu_mask else None
        check(self.L.eosv_bn_train_forward(_f(z), P, b.c, _f(b.gamma), _f(b.beta), BN_EPS, BN_MOMENTUM, _f(b.rm),
                                           _f(b.rv), _f(res), int(relu), _f(y), _f(mask), _f(mean), _f(invstd),
                                           _f(self.work), s), "eosv_bn_train_forward")
        b.nbt += 1
        return y, (mean, invstd, mask)

    def _bn_bwd(self, dy, y, relu, z, P, b: _BN, stats, s, want_dres=False):
        dz = torch.empty_like(z)
        dres = torch.empty_like(z) if want_dres else None
        mask = stats[2] if relu else None  # None without the forward's mask: y is read
        check(self.L.eosv_bn_train_backward(_f(dy), None if mask is not None else _f(y), _f(mask), int(relu), _f(z),
                                            P, b.c, _f(b.gamma), _f(stats[0]), _f(stats[1]), _f(dz), _f(b.dgamma),
                                            _f(b.dbeta), _f(dres), _f(self.work), s), "eosv_bn_train_backward")
        return dz, dres

    # ------------------------------------------------------------------ one iteration
    def step(self, frames: torch.Tensor, labels, T: int, lr_conv: float, lr_fc: float, momentum: float = 0.9):
        """frames [B*T, 3, H, W] f32 (clip-major, as video.view(-1, 3, H, W)), labels [B] ints.
        Runs forward, loss, backward and both SGD updates; returns (loss, logits [B, C])."""
        if self.fc_w is None:
            raise RuntimeError("NativeTrainer.step: load_state_dict first")
        frames = frames.to(self.dev, torch.float32).contiguous()
        self._col_key = None  # new frames (possibly at the same address): the forward gathers afresh
        NT, _, H, W = frames.shape
        if NT % T:
            raise ValueError("frames must be B*T clip-major rows")
        B = NT // T
        lab_h = np.asarray(labels).reshape(-1).astype(np.int64)
        if lab_h.size != B:
            raise ValueError("one label per clip")
        C = int(self.fc_w.shape[0])
        if lab_h.size and (lab_h.min() < 0 or lab_h.max() >= C):
            # nn.CrossEntropyLoss (network_train.py:85) raises on such a target
            raise ValueError(f"NativeTrainer.step: label out of range [0, {C}): "
                             f"min {int(lab_h.min())}, max {int(lab_h.max())} (num_classes too small for the list?)")
        lab = torch.as_tensor(lab_h.astype(np.int32), device=self.dev)
        s = stream_ptr()
        L = self.L
        # ---- forward
        x0 = torch.empty(NT * H * W * 3, dtype=torch.float32, device=self.dev)
        check(L.eosv_nchw_to_nhwc(_f(frames), NT, 3, H, W, _f(x0), s), "eosv_nchw_to_nhwc")
        shp0 = (NT, H, W, 3)
        z0, shp1 = self._conv_fwd(x0, shp0, self.stem, s)
        P1 = shp1[0] * shp1[1] * shp1[2]
        a0, st0 = self._bn_fwd(z0, P1, self.stem_bn, True, None, s)
        Hq, Wq = (shp1[1] - 1) // 2 + 1, (shp1[2] - 1) // 2 + 1
        h = torch.empty(NT * Hq * Wq * 64, dtype=torch.float32, device=self.dev)
        idx = torch.empty(NT * Hq * Wq * 64, dtype=torch.int32, device=self.dev)
        check(L.eosv_maxpool_forward(_f(a0), shp1[0], shp1[1], shp1[2], 64, _f(h), _f(idx), s), "eosv_maxpool_forward")
        shp = (NT, Hq, Wq, 64)
        for blk in self.blocks:
            sv = blk.saved = {"x": h, "shape": shp, "z": [], "y": [], "st": [], "in": [], "inshape": []}
            cur, cshp = h, shp
            nl = len(blk.convs)
            if blk.ds is not None:
                zd, dshp = self._conv_fwd(h, shp, blk.ds, s)
                Pd = dshp[0] * dshp[1] * dshp[2]
                sc, std = self._bn_fwd(zd, Pd, blk.ds_bn, False, None, s)
                sv["ds"] = (zd, sc, std, Pd)
            else:
                sc = h
            for i, (c, b) in enumerate(zip(blk.convs, blk.bns)):
                z, oshp = self._conv_fwd(cur, cshp, c, s)
                P = oshp[0] * oshp[1] * oshp[2]
                last = i == nl - 1
                y, st = self._bn_fwd(z, P, b, True, sc if last else None, s)
                sv["in"].append(cur)
                sv["inshape"].append(cshp)
                sv["z"].append(z)
                sv["y"].append(y)
                sv["st"].append((st, P))
                cur, cshp = y, oshp
            h, shp = cur, cshp
        N4, H4, W4, D = shp
        feat = torch.empty(N4 * D, dtype=torch.float32, device=self.dev)
        check(L.eosv_avgpool_forward(_f(h), N4, H4 * W4, D, _f(feat), s), "eosv_avgpool_forward")
        fm = torch.empty(B * D, dtype=torch.float32, device=self.dev)
        check(L.eosv_avgpool_forward(_f(feat), B, T, D, _f(fm), s), "eosv_avgpool_forward")  # mean over the T frames
        C = self.num_classes
        logits = torch.empty(B * C, dtype=torch.float32, device=self.dev)
        check(L.eosv_sgemm(0, 1, B, C, D, 1.0, _f(fm), D, _f(self.fc_w), D, 0.0, _f(logits), C, s), "eosv_sgemm")
        check(L.eosv_add_bias(_f(logits), B, C, _f(self.fc_b), s), "eosv_add_bias")
        row_loss = torch.empty(B, dtype=torch.float32, device=self.dev)
        dlog = torch.empty(B * C, dtype=torch.float32, device=self.dev)
        check(L.eosv_softmax_xent(_f(logits), _f(lab), B, C, _f(row_loss), _f(dlog), s), "eosv_softmax_xent")
        # ---- backward
        check(L.eosv_sgemm(1, 0, C, D, B, 1.0, _f(dlog), C, _f(fm), D, 0.0, _f(self.fc_gw), D, s), "eosv_sgemm")
        check(L.eosv_sum_rows(_f(dlog), B, C, _f(self.fc_gb), 0, s), "eosv_sum_rows")
        dfm = torch.empty(B * D, dtype=torch.float32, device=self.dev)
        check(L.eosv_sgemm(0, 0, B, D, C, 1.0, _f(dlog), C, _f(self.fc_w), D, 0.0, _f(dfm), D, s), "eosv_sgemm")
        dfeat = torch.empty(N4 * D, dtype=torch.float32, device=self.dev)
        check(L.eosv_broadcast_rows(_f(dfm), B, T, D, 1.0 / T, _f(dfeat), s), "eosv_broadcast_rows")
        dh = torch.empty(N4 * H4 * W4 * D, dtype=torch.float32, device=self.dev)
        check(L.eosv_broadcast_rows(_f(dfeat), N4, H4 * W4, D, 1.0 / (H4 * W4), _f(dh), s), "eosv_broadcast_rows")
        for blk in reversed(self.blocks):
            sv = blk.saved
            nl = len(blk.convs)
            dres = None
            g = dh
            for i in reversed(range(nl)):
                c, b = blk.convs[i], blk.bns[i]
                st, P = sv["st"][i]
                dz, dr = self._bn_bwd(g, sv["y"][i], True, sv["z"][i], P, b, st, s, want_dres=(i == nl - 1))
                if i == nl - 1:
                    dres = dr
                skip = None
                if i == 0:
                    # the block input's gradient through the shortcut, added to the first conv's dx
                    if blk.ds is not None:
                        zd, sc, std, Pd = sv["ds"]
                        dzd, _ = self._bn_bwd(dres, None, False, zd, Pd, blk.ds_bn, std, s)
                        skip = self._conv_bwd(dzd, sv["x"], sv["shape"], blk.ds, s, need_dx=True)
                    else:
                        skip = dres
                g = self._conv_bwd(dz, sv["in"][i], sv["inshape"][i], c, s, need_dx=True, acc=skip)
            dh = g
            blk.saved = {}
        da0 = torch.empty(P1 * 64, dtype=torch.float32, device=self.dev)
        check(L.eosv_maxpool_backward(_f(dh), _f(idx), shp1[0], shp1[1], shp1[2], 64, _f(da0), s),
              "eosv_maxpool_backward")
        dz0, _ = self._bn_bwd(da0, a0, True, z0, P1, self.stem_bn, st0, s)
        self._conv_bwd(dz0, x0, shp0, self.stem, s, need_dx=False)
        # ---- SGD (optimizer_1: convnet, optimizer_2: fc; first step initialises the momentum)
        first = int(self.step_count == 0)
        check(L.eosv_sgd_momentum(_f(self.p_flat), _f(self.g_flat), _f(self.m_flat), self.p_flat.numel(), lr_conv,
                                  momentum, first, s), "sgd")
        check(L.eosv_sgd_momentum(_f(self.fc_w), _f(self.fc_gw), _f(self.fc_bw), self.fc_w.numel(), lr_fc, momentum,
                                  first, s), "sgd")
        check(L.eosv_sgd_momentum(_f(self.fc_b), _f(self.fc_gb), _f(self.fc_bb), self.fc_b.numel(), lr_fc, momentum,
                                  first, s), "sgd")
        self.step_count += 1
        return float(row_loss.sum().item()), logits.view(B, C)

    def grads(self) -> Dict[str, torch.Tensor]:
        """The last step's gradients in the state_dict layout (CPU), for parity checks."""
        out = {}
        for c in self._convs():
            out[c.name + ".weight"] = c.g.view(c.cout, c.k, c.k, c.cin).permute(0, 3, 1, 2).contiguous().cpu()
        for b in self._bns():
            out[b.name + ".weight"] = b.dgamma.cpu()
            out[b.name + ".bias"] = b.dbeta.cpu()
        out["fc.weight"] = self.fc_gw.cpu()
        out["fc.bias"] = self.fc_gb.cpu()
        return out
