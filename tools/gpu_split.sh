#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/split_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|Error|assert" gpurun_out/split_tests.log | head -20; tail -2 gpurun_out/split_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 env SG_PATHS=followed_by python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 > gpurun_out/split_fb.log 2>&1; rc=$?
tail -2 gpurun_out/split_fb.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --config 1 --steps 5 --warmup 2 --no-cpu > gpurun_out/split_bench1.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/split_bench1.log
