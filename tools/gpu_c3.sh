cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -v -k aug --timeout 300 --timeout-method thread > gpurun_out/c3_tests.log 2>&1; echo tests_rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/c3_tests.log | head
SPECS="3 bf16 512" bash tools/gpu_configs.sh
EOSV_AUG_REFORWARD=1 timeout -k 10 600 python tools/bench_configs.py --config 3 --dtype bf16 --episodes 64 2>&1 | grep "^{"
