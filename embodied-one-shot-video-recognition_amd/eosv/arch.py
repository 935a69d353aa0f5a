"""ResNet backbone specs in the reference's state_dict layout.

``models.model_resnet18/50`` (reference ``models.py:9-37``) wrap
``torchvision.models.resnetXX`` minus its ``fc``: the children ``[:-1]`` become
``self.convnet`` (``convnet.0`` conv1, ``.1`` bn1, ``.2`` relu, ``.3`` maxpool,
``.4``-``.7`` layer1-4, ``.8`` avgpool) and a fresh ``fc`` maps the pooled
feature to ``num_classes`` logits.  The native library builds its own layer plan
from the same arch id (``csrc/eosv_api.cpp``); this module only supplies the
tensor names/shapes the Python side needs.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Tuple

ARCH_IDS = {"resnet18": 18, "resnet50": 50, "resnet101": 101}


@dataclass(frozen=True)
class ResNetSpec:
    name: str
    block: str            # "basic" | "bottleneck"
    layers: Tuple[int, int, int, int]

    @property
    def expansion(self) -> int:
        return 1 if self.block == "basic" else 4

    @property
    def feature_dim(self) -> int:
        return 512 * self.expansion

    @property
    def arch_id(self) -> int:
        return ARCH_IDS[self.name]


SPECS = {
    "resnet18": ResNetSpec("resnet18", "basic", (2, 2, 2, 2)),
    "resnet50": ResNetSpec("resnet50", "bottleneck", (3, 4, 6, 3)),
    "resnet101": ResNetSpec("resnet101", "bottleneck", (3, 4, 23, 3)),
}


def _bn(prefix: str, c: int, out: Dict[str, tuple]):
    out[prefix + ".weight"] = (c,)
    out[prefix + ".bias"] = (c,)
    out[prefix + ".running_mean"] = (c,)
    out[prefix + ".running_var"] = (c,)
    out[prefix + ".num_batches_tracked"] = ()


def state_dict_shapes(spec: ResNetSpec, num_classes: int = 64) -> Dict[str, tuple]:
    """Ordered name -> shape of ``model_resnetXX(num_classes).state_dict()``."""
    out: Dict[str, tuple] = {}
    out["convnet.0.weight"] = (64, 3, 7, 7)
    _bn("convnet.1", 64, out)
    inplanes = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), spec.layers)):
        for bi in range(n):
            stride = 2 if (li > 0 and bi == 0) else 1
            p = f"convnet.{4 + li}.{bi}"
            if spec.block == "basic":
                out[p + ".conv1.weight"] = (planes, inplanes, 3, 3)
                _bn(p + ".bn1", planes, out)
                out[p + ".conv2.weight"] = (planes, planes, 3, 3)
                _bn(p + ".bn2", planes, out)
            else:
                out[p + ".conv1.weight"] = (planes, inplanes, 1, 1)
                _bn(p + ".bn1", planes, out)
                out[p + ".conv2.weight"] = (planes, planes, 3, 3)
                _bn(p + ".bn2", planes, out)
                out[p + ".conv3.weight"] = (planes * 4, planes, 1, 1)
                _bn(p + ".bn3", planes * 4, out)
            cout = planes * spec.expansion
            if bi == 0 and (stride != 1 or inplanes != cout):
                out[p + ".downsample.0.weight"] = (cout, inplanes, 1, 1)
                _bn(p + ".downsample.1", cout, out)
            inplanes = cout
    out["fc.weight"] = (num_classes, spec.feature_dim)
    out["fc.bias"] = (num_classes,)
    return out


def conv_macs_per_frame(spec: ResNetSpec, H: int = 224, W: int = 224) -> int:
    """Multiply-accumulates of every conv of the backbone for one frame."""
    def out_hw(h, k, s, p):
        return (h + 2 * p - k) // s + 1

    macs = 0
    h, w = out_hw(H, 7, 2, 3), out_hw(W, 7, 2, 3)
    macs += h * w * 64 * 3 * 49
    h, w = out_hw(h, 3, 2, 1), out_hw(w, 3, 2, 1)
    inplanes = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), spec.layers)):
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            cout = planes * spec.expansion
            ho, wo = out_hw(h, 3, s, 1), out_hw(w, 3, s, 1)
            if spec.block == "basic":
                macs += ho * wo * planes * inplanes * 9 + ho * wo * planes * planes * 9
            else:
                macs += h * w * planes * inplanes          # 1x1 at input res
                macs += ho * wo * planes * planes * 9       # 3x3 (stride here)
                macs += ho * wo * cout * planes              # 1x1 expand
            if bi == 0 and (s != 1 or inplanes != cout):
                macs += ho * wo * cout * inplanes
            h, w = ho, wo
            inplanes = cout
    return macs


def conv_layer_bytes(spec: ResNetSpec, H: int = 224, W: int = 224, elem: int = 4, stem_pool_fused: bool = False):
    """Algorithmic HBM bytes of every conv launch, in the native plan's layer-id order
    (stem, then per block c1, c2[, c3][, downsample]: csrc/eosv_api.hip): a list of
    (per-frame bytes, per-launch weight bytes).  Per frame: the input map read once, the
    output map written once, plus the residual map read once by the block's last conv.
    The stem reads the 3-channel frame; with ``stem_pool_fused`` (bf16 path) it writes the
    pooled map.  This is the floor the rocprofv3 FETCH/WRITE traffic is compared with."""
    def out_hw(h, k, s, p):
        return (h + 2 * p - k) // s + 1

    layers = []
    h, w = out_hw(H, 7, 2, 3), out_hw(W, 7, 2, 3)
    ph, pw = out_hw(h, 3, 2, 1), out_hw(w, 3, 2, 1)
    out = (ph * pw if stem_pool_fused else h * w) * 64
    layers.append(((3 * H * W + out) * elem, 64 * 147 * elem))
    h, w = ph, pw
    inplanes = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), spec.layers)):
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            cout = planes * spec.expansion
            ho, wo = out_hw(h, 3, s, 1), out_hw(w, 3, s, 1)
            if spec.block == "basic":
                layers.append(((h * w * inplanes + ho * wo * planes) * elem, planes * inplanes * 9 * elem))
                layers.append(((2 * ho * wo * planes + ho * wo * cout) * elem, cout * planes * 9 * elem))
            else:
                layers.append(((h * w * inplanes + h * w * planes) * elem, planes * inplanes * elem))
                layers.append(((h * w * planes + ho * wo * planes) * elem, planes * planes * 9 * elem))
                layers.append(((ho * wo * planes + 2 * ho * wo * cout) * elem, cout * planes * elem))
            if bi == 0 and (s != 1 or inplanes != cout):
                layers.append(((ho * wo * inplanes + ho * wo * cout) * elem, cout * inplanes * elem))
            h, w = ho, wo
            inplanes = cout
    return layers


def block_layer_ids(spec: ResNetSpec):
    """(conv1, conv2, conv3 or None, downsample or None) layer ids of every residual block, in the
    native plan's order (stem = 0; csrc/eosv_api.hip build_plan)."""
    out, i = [], 1
    inplanes = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), spec.layers)):
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            cout = planes * spec.expansion
            ds = bi == 0 and (s != 1 or inplanes != cout)
            if spec.block == "basic":
                ids = (i, i + 1, None)
                i += 2
            else:
                ids = (i, i + 1, i + 2)
                i += 3
            out.append(ids + ((i,) if ds else (None,)))
            i += 1 if ds else 0
            inplanes = cout
    return out


def fuse_bneck_bytes(layers, spec: ResNetSpec, nl):
    """conv_launch_bytes adjusted for the blocks the native forward ran as ONE launch
    (bneck_bf16.hip, r06): recognised from the profile itself -- conv1 launched, conv2 and conv3
    not.  Such a launch reads the block input once (conv1's input is also conv3's residual, or the
    folded stride-1 downsample's input: the same pixels, read once) and writes the block output; its
    64-channel maps (conv1's and conv2's outputs) never reach HBM.  Its entry moves onto conv1's id,
    with all three weight matrices; conv2 / conv3 become empty.  (A next conv1 fused into it keeps the
    generic rule: an unlaunched conv's bytes less its input map join the previous launch.)
    Basic blocks run as one launch (bblock_bf16.hip, r06: conv1 launched, conv2 not) read the
    block input once (conv1's input is conv2's residual) and write the block output: conv2's bytes
    less its input map, with both weight tensors."""
    L = [tuple(x) for x in layers]
    for c1, c2, c3, _ in block_layer_ids(spec):
        if c3 is None:
            if c2 < len(L) and c2 < len(nl) and nl[c1] and not nl[c2]:
                pf2, wb2, pin2 = L[c2]
                L[c1] = (pf2 - pin2, L[c1][1] + wb2, L[c1][2])
                L[c2] = (0, 0, 0)
            continue
        if c3 >= len(L) or c3 >= len(nl):
            continue
        if nl[c1] and not nl[c2] and not nl[c3]:
            pf1, wb1, pin1 = L[c1]
            pf2, wb2, pin2 = L[c2]
            pf3, wb3, pin3 = L[c3]
            L[c1] = (pf1 - pin2 + pf3 - pin3 - pin1, wb1 + wb2 + wb3, pin1)
            L[c2] = L[c3] = (0, 0, 0)
    return L


def conv_launch_bytes(spec: ResNetSpec, H: int = 224, W: int = 224, elem: int = 4):
    """Algorithmic HBM bytes per conv launch as the native forward runs it, in the plan's layer-id
    order (conv_layer_bytes' list, same indices): the fused stem + maxpool reads the caller's f32
    NCHW frame and writes the pooled map; the downsample 1x1 is folded into its block's last conv
    (csrc/eosv_api.hip), which then reads the downsample's input pixels instead of a residual map,
    so the downsample's own entry is (0, 0, 0) and its weights move to that conv.  ``elem`` = bytes
    per stored activation element (f32 4, bf16 2, f32x3 4: the (hi, lo) bf16 pair).  This is the
    floor of each launch's traffic that the per-layer roofline (bench.py) prices at HBM peak.
    Entries: (per-frame bytes, per-launch weight bytes, per-frame bytes of the input map) -- the
    last is what a bf16 bottleneck conv1 fused with the previous conv3 (pair1x1_bf16.hip) saves."""
    def out_hw(h, k, s, p):
        return (h + 2 * p - k) // s + 1

    h, w = out_hw(H, 7, 2, 3), out_hw(W, 7, 2, 3)
    ph, pw = out_hw(h, 3, 2, 1), out_hw(w, 3, 2, 1)
    layers = [(3 * H * W * 4 + ph * pw * 64 * elem, 64 * 147 * elem, 3 * H * W * 4)]
    h, w = ph, pw
    inplanes = 64
    for li, (planes, n) in enumerate(zip((64, 128, 256, 512), spec.layers)):
        for bi in range(n):
            s = 2 if (li > 0 and bi == 0) else 1
            cout = planes * spec.expansion
            ho, wo = out_hw(h, 3, s, 1), out_hw(w, 3, s, 1)
            ds = bi == 0 and (s != 1 or inplanes != cout)
            # the last conv reads the residual, or (folded downsample) the block input at stride s
            last_extra = ho * wo * inplanes if ds else ho * wo * cout
            if spec.block == "basic":
                layers.append(((h * w * inplanes + ho * wo * planes) * elem, planes * inplanes * 9 * elem, h * w * inplanes * elem))
                layers.append(((ho * wo * planes + last_extra + ho * wo * cout) * elem, cout * planes * 9 * elem,
                               ho * wo * planes * elem))
            else:
                layers.append(((h * w * inplanes + h * w * planes) * elem, planes * inplanes * elem, h * w * inplanes * elem))
                layers.append(((h * w * planes + ho * wo * planes) * elem, planes * planes * 9 * elem, h * w * planes * elem))
                layers.append(((ho * wo * planes + last_extra + ho * wo * cout) * elem, cout * planes * elem,
                               ho * wo * planes * elem))
            if ds:
                pf, wb, pin = layers[-1]
                layers[-1] = (pf, wb + cout * inplanes * elem, pin)
                layers.append((0, 0, 0))
            h, w = ho, wo
            inplanes = cout
    return layers
