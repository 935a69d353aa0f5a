#!/bin/bash
# Register / spill / LDS table of every kernel in the given .hip files (compile only, no GPU):
#   tools/regs.sh csrc/pairw_bf16.hip [more.hip] [-DFLAG ...]
cd "$(dirname "$0")/../embodied-one-shot-video-recognition_amd/csrc"
srcs=(); flags=()
for a in "$@"; do case $a in -*) flags+=("$a");; *) srcs+=("$(basename "$a")");; esac; done
for f in "${srcs[@]}"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include "${flags[@]}" -c "$f" -o /tmp/regs_$$.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//; s/^[^:]*:[0-9]*:[0-9]*: remark: *//' |
  awk '/Function Name/ {n=$3} /^VGPRs:/ {v=$2} /^AGPRs:/ {ag=$2} /^SGPRs Spill/ {ss=$3} /^VGPRs Spill/ {vs=$3} /^LDS Size/ {l=$4; printf "%-90s v%-4s a%-4s sspill %-3s vspill %-3s lds %s\n", substr(n,1,90), v, ag, ss, vs, l}'
done
rm -f /tmp/regs_$$.o
