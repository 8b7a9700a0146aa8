#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_keyed.py tests/test_gpu_keyed_stack.py \
  tests/test_gpu_compaction.py tests/test_gpu_shard_rehearsal.py > gpurun_out/r03_kt_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03_kt_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SG_KT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 5 --warmup 2 > gpurun_out/r03_bench_c4_order.log 2>&1
echo "bench rc=$?"; grep -o '"kernel_ms": {[^}]*}' gpurun_out/r03_bench_c4_order.log; grep -o '"value": [0-9.e+]*' gpurun_out/r03_bench_c4_order.log
