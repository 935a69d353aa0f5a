#!/bin/bash
# r06 session D: which side of the R101@256 (W 64) bneck mismatch is nondeterministic: repeated
# stage-map saves per mode, compared pairwise.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -n ${TAILN:-3} "$O/$name.log"; if [ $rc -ne 0 ]; then echo "STOP $name rc=$rc"; exit $rc; fi; }
save() { step "save_$1" 200 env $2 python tools/ws_diff.py save $O/$1.pt $3 bf16; }
cmp() { TAILN=8 step "cmp_$1_$2" 100 python tools/ws_diff.py cmp $O/$1.pt $O/$2.pt; }
save f1a "EOSV_BNECK=1 EOSV_BNECK_TAIL=0" resnet101:256
save f1b "EOSV_BNECK=1 EOSV_BNECK_TAIL=0" resnet101:256
save u0a "EOSV_BNECK=0" resnet101:256
save u0b "EOSV_BNECK=0" resnet101:256
cmp f1a f1b
cmp u0a u0b
cmp f1a u0a
save ft1 "EOSV_BNECK=1 EOSV_BNECK_TAIL=1" resnet101:256
cmp ft1 u0a
save r50u "EOSV_BNECK=0" resnet50
save r50t "EOSV_BNECK=1 EOSV_BNECK_TAIL=1" resnet50
cmp r50t r50u
rm -f $O/*.pt
echo done_r06d
