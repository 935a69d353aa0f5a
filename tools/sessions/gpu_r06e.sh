#!/bin/bash
# r06 session E: which bneck variant races at W 64 (block 0 only / the 256-input blocks only),
# repeated saves compared pairwise.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-3} "$O/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; }
save() { step "save_$1" 200 env $2 python tools/ws_diff.py save $O/$1.pt $3 bf16; }
cmp() { TAILN=3 step "cmp_$1_$2" 100 python tools/ws_diff.py cmp $O/$1.pt $O/$2.pt; }
for m in 3 2; do
  save m${m}a "EOSV_BNECK=$m EOSV_BNECK_TAIL=0" resnet101:256
  save m${m}b "EOSV_BNECK=$m EOSV_BNECK_TAIL=0" resnet101:256
  save m${m}c "EOSV_BNECK=$m EOSV_BNECK_TAIL=0" resnet101:256
  cmp m${m}a m${m}b
  cmp m${m}a m${m}c
done
rm -f $O/*.pt
echo done_r06e
