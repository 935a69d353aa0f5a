"""Layer-level native checks on the GPU: tests/native/conv_check (built by
__graft_entry__.build()) runs every bf16 / f32 conv kernel family of libeosv.so on
seeded random operands against a double-precision CPU conv, including the zero-padding
taps, M tails, stride-2 entries, 1x1 convs, both K orders, and the fused stem + pool."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "conv_check")


def test_conv_check():
    if not os.path.exists(BIN):
        pytest.fail("tests/native/conv_check missing: run __graft_entry__.build()")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "\n0 failures" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
