#!/bin/bash
# round 3: stack matcher tests + config-4 bench (no CPU baseline) on one GPU
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_keyed_stack.py \
  > gpurun_out/r03_ks_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SG_KT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 5 --warmup 2 > gpurun_out/r03_bench_c4.log 2>&1
echo "bench rc=$?"
tail -3 gpurun_out/r03_ks_tests.log
tail -5 gpurun_out/r03_bench_c4.log
