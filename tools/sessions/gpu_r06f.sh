#!/bin/bash
# r06 session F: is conv_rowsr_bf16<64, 64> (the r05 W-64 stage-1 3x3) the nondeterministic kernel
# at R101@256?  Repeats with it off (EOSV_BF16_ROWSR=0), then poisoned runs of the r05 path at 256.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-3} "$O/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; fi; return 0; }
save() { step "save_$1" 200 env $2 python tools/ws_diff.py save $O/$1.pt $3 bf16; }
cmp() { TAILN=3 step "cmp_$1_$2" 100 python tools/ws_diff.py cmp $O/$1.pt $O/$2.pt; }
save m3r0a "EOSV_BNECK=3 EOSV_BNECK_TAIL=0 EOSV_BF16_ROWSR=0" resnet101:256
save m3r0b "EOSV_BNECK=3 EOSV_BNECK_TAIL=0 EOSV_BF16_ROWSR=0" resnet101:256
save m3r0c "EOSV_BNECK=3 EOSV_BNECK_TAIL=0 EOSV_BF16_ROWSR=0" resnet101:256
cmp m3r0a m3r0b
cmp m3r0a m3r0c
save m1r0 "EOSV_BNECK=1 EOSV_BNECK_TAIL=0 EOSV_BF16_ROWSR=0" resnet101:256
save m1t1r0 "EOSV_BNECK=1 EOSV_BNECK_TAIL=1 EOSV_BF16_ROWSR=0" resnet101:256
save m0r0 "EOSV_BNECK=0 EOSV_BF16_ROWSR=0" resnet101:256
save m0r1 "EOSV_BNECK=0" resnet101:256
cmp m0r0 m0r1
cmp m1r0 m0r0
cmp m1t1r0 m0r0
cmp m3r0a m0r0
rm -f $O/*.pt
TAILN=12 step poison_r101_256 280 env EOSV_BNECK=0 python tools/poison_check.py resnet101:256 bf16 17,64
TAILN=12 step poison_r101_256_rowsr0 280 env EOSV_BNECK=0 EOSV_BF16_ROWSR=0 python tools/poison_check.py resnet101:256 bf16 17,64
echo done_r06f
