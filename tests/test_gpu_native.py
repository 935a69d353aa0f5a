"""Layer-level native checks on the GPU: tests/native/conv_check (built by
__graft_entry__.build()) runs every bf16 / f32 conv kernel family of libeosv.so on
seeded random operands against a double-precision CPU conv, including the zero-padding
taps, M tails, stride-2 entries, 1x1 convs, both K orders, and the fused stem + pool."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "conv_check")


# phased kernel: default shapes / every eligible shape / off; stem_cb 0: full-width bf16 stem workgroups
@pytest.mark.parametrize("p8,stem_cb", [("1", "1"), ("2", "1"), ("0", "0")])
def test_conv_check(p8, stem_cb):
    if not os.path.exists(BIN):
        pytest.fail("tests/native/conv_check missing: run __graft_entry__.build()")
    env = dict(os.environ, EOSV_BF16_P8=p8, EOSV_STEM_CB=stem_cb)
    r = subprocess.run([BIN], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "\n0 failures" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
