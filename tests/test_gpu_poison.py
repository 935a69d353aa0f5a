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
