"""Drop-in for the reference's ``models.py`` (lines 9-56), backed by the native library.

``model_resnet18/50(num_classes)`` keep the reference's module tree and state_dict
keys (``convnet.{0,1,4..7}.*`` + ``fc.*``) so ``load_state_dict(torch.load(pkl))``
and ``.eval()/.cuda()`` work unchanged; ``forward(x)`` returns ``(feature, output)``
like models.py:18-22 but runs the eosv HIP backbone (libeosv.so) -- the torch
submodules are parameter containers only.  ``model_resnet101`` is an extension for
BASELINE config 5 (the reference has no R101 wrapper).

ImageNet weights (``pretrained=True``, models.py:13/28) cannot be downloaded offline:
fresh models are initialised from the deterministic generator in eosv/synth.py.
There is no CPU fallback; forward raises without a HIP device.
"""
import torch
import torch.nn as nn

import utils
from eosv import arch as _arch, engine as _engine, synth as _synth


def _bn(c):
    return nn.BatchNorm2d(c)


class _Basic(nn.Module):
    def __init__(self, inplanes, planes, stride, ds):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = _bn(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = _bn(planes)
        self.downsample = ds


class _Bottleneck(nn.Module):
    def __init__(self, inplanes, planes, stride, ds):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = _bn(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = _bn(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = _bn(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = ds


def _convnet(spec):
    """torchvision resnet children()[:-1] as a parameter-container tree (same keys)."""
    block = _Basic if spec.block == "basic" else _Bottleneck
    mods = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), _bn(64), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, 1)]
    inplanes = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), spec.layers)):
        blocks = []
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            cout = planes * spec.expansion
            ds = None
            if bi == 0 and (stride != 1 or inplanes != cout):
                ds = nn.Sequential(nn.Conv2d(inplanes, cout, 1, stride, bias=False), _bn(cout))
            blocks.append(block(inplanes, planes, stride, ds))
            inplanes = cout
        mods.append(nn.Sequential(*blocks))
    mods.append(nn.AdaptiveAvgPool2d((1, 1)))
    return nn.Sequential(*mods)


class _NativeResNet(nn.Module):
    ARCH = None
    #: arithmetic of the native conv stack: 'f32' (exact-f32 MFMA, reference parity), 'f32x3'
    #: (f32-accurate split-bf16 MFMA, within 1e-4 of f32, ~2.4x faster) or 'bf16'
    compute_dtype = "f32"
    #: frames per internal chunk of the native handle (workspace size: 4 activation buffers of
    #: max_frames x the largest map, e.g. R50 bf16 6.4 GB, R50 f32 26 GB at 2048).  Grids of a
    #: few hundred frames leave CUs idle (R50 layer 3 at 256 frames: 196 tiles on 256 CUs); the
    #: episode drivers batch thousands of frames per call (config 3: +6 % from 1024 to 4096)
    max_frames = 2048

    def __init__(self, num_classes):
        super().__init__()
        spec = _arch.SPECS[self.ARCH]
        self.spec = spec
        self.convnet = _convnet(spec)
        self.fc = nn.Linear(spec.feature_dim, num_classes)
        self.num_classes = num_classes
        sd = _synth.synth_state_dict(spec, num_classes, 0)
        with torch.no_grad():
            nn.Module.load_state_dict(self, {k: torch.from_numpy(v) for k, v in sd.items()})
        self._native = None
        self._native_key = None
        self._dirty = True

    # -- weight sync -------------------------------------------------------------
    def load_state_dict(self, state_dict, strict=True, **kw):
        r = super().load_state_dict(state_dict, strict=strict, **kw)
        self._dirty = True
        return r

    def _apply(self, fn, *a, **kw):
        r = super()._apply(fn, *a, **kw)
        self._dirty = True
        return r

    def mark_weights_dirty(self):
        """Call after modifying parameters in place; the next forward re-uploads them."""
        self._dirty = True

    def native(self, H, W, device=None):
        """The eosv.engine.Backbone serving frames of size HxW (created / synced lazily)."""
        if device is None:
            device = torch.cuda.current_device()
        key = (H, W, int(device), self.compute_dtype, self.max_frames)
        if self._native is None or self._native_key != key:
            if self._native is not None:
                self._native.close()
            self._native = _engine.Backbone(self.ARCH, self.compute_dtype, H, W, max_frames=self.max_frames,
                                            device=int(device), num_classes=self.num_classes)
            self._native_key = key
            self._dirty = True
        if self._dirty:
            self._native.load_state_dict(self.state_dict())
            self._dirty = False
        return self._native

    # -- forward (models.py:18-22) ------------------------------------------------
    def forward(self, x):
        if x.dim() != 4 or x.shape[1] != 3:
            raise ValueError(f"expected [B,3,H,W], got {tuple(x.shape)}")
        if not x.is_cuda:
            x = x.cuda()
        x = x.float().contiguous()
        bb = self.native(x.shape[2], x.shape[3], x.device.index)
        feature = bb.forward(x)
        output = bb.fc(feature)
        return feature, output


class model_resnet18(_NativeResNet):
    ARCH = "resnet18"


class model_resnet50(_NativeResNet):
    ARCH = "resnet50"


class model_resnet101(_NativeResNet):
    """Extension (BASELINE config 5); the reference ships only R18/R50 wrappers."""
    ARCH = "resnet101"


# for temporal convolution flating layer (models.py:41-56)
class TemporalLayer(nn.Module):
    def __init__(self):
        super().__init__()
        kernal = torch.FloatTensor([utils.lamda1, utils.lamda2, utils.lamda1])
        kernal = kernal.unsqueeze(0).unsqueeze(0).unsqueeze(0)
        self.weight = nn.Parameter(data=kernal, requires_grad=False)

    def forward(self, x):
        """x [..., S] -> 3-tap smoothing along the last axis, zero padded (PyTorch-1.x
        meaning of the reference's F.conv1d(x, w, padding=(0,1)) on a 4-D input)."""
        w = self.weight.detach().reshape(-1).cpu()
        if not x.is_cuda:
            x = x.cuda()
        return _engine.temporal_smooth(x.float().contiguous(), float(w[0]), float(w[1]))
