"""Poisoned against plain forwards on the GPU (tools/poison_check.py, profiling build): every
activation buffer filled with NaN bytes at each chunk's start and every CU's LDS filled with NaN
before each launch must leave every stage map and the features bitwise unchanged.  A kernel
whose valid outputs read rows or LDS words nobody wrote fails this on its first run; the r04
race of the 256-pixel stage-2 pair showed here at 64 and 130 frames per
chunk and not in the repeat probes at 37 / 1024."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "embodied-one-shot-video-recognition_amd", "libeosv_prof.so")


def test_poisoned_forwards_match_plain():
    if not os.path.exists(LIB):
        pytest.fail("libeosv_prof.so missing: run __graft_entry__.build()")
    env = dict(os.environ, EOSV_LIBRARY=LIB)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "poison_check.py"), "resnet50,resnet18",
                        "bf16,f32", "17,64,130"], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and "poison_check: 0 failing" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("switch,name", [("EOSV_STEM_V5", "resnet18"), ("EOSV_STEM_V5", "resnet50"),
                                         ("EOSV_BF16_S2ROWS", "resnet18"), ("EOSV_BF16_ROWSR", "resnet18"),
                                         ("EOSV_BF16_ROWSR", "resnet50"), ("EOSV_BF16_ROWSR", "resnet101:256")])
def test_r05_kernels_bitwise_equal_r04(switch, name, tmp_path):
    """The r05 kernels against the r04 ones they replace (profiling build, the switch at 0 selects
    the r04 kernel): every stage map bitwise equal (37 frames of 224x224, child processes since the
    switches are read once per process).  EOSV_STEM_V5: stem_pool_bf16_cb5_kernel (one barrier per
    step, unrolled ring addressing, zero-line staging, DPP column max, packed ReLU);
    EOSV_BF16_S2ROWS: conv_s2rows_bf16 (R18 layer2.0.conv1 row strips) against the 512x128 tile;
    EOSV_BF16_ROWSR: conv_rowsr_bf16 (3x3 row strips, weights in registers) against conv_rows_bf16
    (stage 1 at 224), the tap-shift tile (stage 2) and the 128x64 implicit GEMM (stage 1 at 256:
    resnet101:256 = config 5's shapes)."""
    _switch_stage_maps_equal(switch, name, tmp_path, "r05", "r04")


def _switch_stage_maps_equal(switch, name, tmp_path, new="new", old="old", dtype="bf16"):
    if not os.path.exists(LIB):
        pytest.fail("libeosv_prof.so missing: run __graft_entry__.build()")
    outs = []
    for v in ("1", "0"):
        out = str(tmp_path / f"{switch}_{v}.pt")
        env = dict(os.environ, EOSV_LIBRARY=LIB, **{switch: v})
        r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "ws_diff.py"), "save", out, name, dtype],
                           env=env, capture_output=True, text=True, timeout=200)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(out)
    import torch
    a, b = torch.load(outs[0]), torch.load(outs[1])
    if not all(torch.equal(u, v) for u, v in zip(a, b)):
        cmp = subprocess.run([sys.executable, os.path.join(REPO, "tools", "ws_diff.py"), "cmp", outs[0], outs[1]],
                             capture_output=True, text=True, timeout=120).stdout
        pytest.fail(f"stage maps differ between the {new} and {old} kernels ({switch}):\n{cmp}")


@pytest.mark.parametrize("name", ["resnet50", "resnet50:224:601", "resnet101:256", "resnet101:256:300"])
def test_bneck_bitwise_equal_unfused(name, tmp_path):
    """r06: the whole-block stage-1 kernel (bneck_bf16.hip: conv1 -> conv2 -> conv3 in one launch,
    plus the next block's conv1) against the r05 path it replaces (EOSV_BNECK=0: the 1x1 conv,
    conv_rows_bf16 / conv_rowsr_bf16 and the pair kernels): every stage map bitwise equal, at 224
    (R50: 56x56 maps, 8 idle lanes in each row's last pixel tile) and 256 (R101: 64x64), with one image per
    workgroup (37 frames) and with 2-3 images per workgroup (601 / 300 frames on 256 CUs: the
    stream crosses images through the zero step, ragged image counts per workgroup)."""
    _switch_stage_maps_equal("EOSV_BNECK", name, tmp_path, "bneck", "r05 stage-1")


@pytest.mark.parametrize("name", ["resnet18", "resnet18:224:601", "resnet18:256", "resnet18:256:300"])
def test_bblock_bitwise_equal_unfused(name, tmp_path):
    """r06: the whole basic-block stage-1 kernel (bblock_bf16.hip: conv1 -> conv2 + x in one launch)
    against the two 3x3 launches it replaces (EOSV_BBLOCK=0: conv_rows_bf16 at 56x56, the 64x64
    kernels at 256): every stage map bitwise equal, one image per workgroup (37 frames) and several
    (601 / 300 frames: the stream crosses images through the zero step)."""
    _switch_stage_maps_equal("EOSV_BBLOCK", name, tmp_path, "bblock", "two-launch stage-1")


@pytest.mark.parametrize("name", ["resnet18:224:601", "resnet18:256:300"])
def test_bblock2_bitwise_equal_bblock(name, tmp_path):
    """r06: the split-conv basic block (bblock2_bf16_kernel: one conv per wave for 32 couts, the two
    convs of different steps in one phase, the rolling fragment lead) against the one-wave-both-convs
    kernel it replaces (EOSV_BBLOCK2=0): every stage map bitwise equal at 56x56 and 64x64, with the
    stream crossing images (601 / 300 frames on 256 CUs)."""
    _switch_stage_maps_equal("EOSV_BBLOCK2", name, tmp_path, "bblock2", "bblock")
