set -e
export EOSV_LIBRARY=$PWD/embodied-one-shot-video-recognition_amd/libeosv_prof.so
for t in ${TARGETS:-64 128 256}; do for mr in ${MINROWS:-1024 2048 4096}; do
  r=$(EOSV_SPLITK_TARGET=$t EOSV_SPLITK_MINROWS=$mr timeout -k 10 120 python tools/bench_train.py --cpu-steps 0 2>/dev/null | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
  echo "target $t minrows $mr ms $r"
done; done
