#!/bin/bash
# conv_check + per-layer R50 bf16 (new build), then an interleaved A/B of tools/ablib/libeosv_base.so
# vs the tree's build on R18 bf16 (ab_lib.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ARCHS=${ARCHS:-resnet50} bash tools/gpu_layers.sh || exit $?
[ -n "$NOAB" ] && exit 0
DTYPE=${DTYPE:-bf16} bash tools/ab_lib.sh
