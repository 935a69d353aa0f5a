#!/bin/bash
# r06 session AC: bblock2 wave priorities (release variants -DEOSV_BB2_PRIO=1 conv2 waves, =2 conv1 waves at priority 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06ac; mkdir -p $O
ROUNDS=2 LIBS="libeosv.so libeosv_prio1.so libeosv_prio2.so" ARGS="--dtype bf16 --secondary-dtype none" timeout -k 10 600 bash tools/ab_release.sh > $O/ab_r18.log 2>&1 || { cat $O/ab_r18.log; exit 1; }
cat $O/ab_r18.log
