#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard_nfa.py \
  tests/test_gpu_shard_rehearsal.py tests/test_gpu_keyed.py > gpurun_out/r03_shard_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r03_shard_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/record_sched_logs.py gpurun_out/sched_collision_w2.npz
echo "record rc=$?"
SG_KT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 5 --warmup 2 > gpurun_out/r03_bench_c4_order.log 2>&1
echo "bench rc=$?"; grep -o '"kernel_ms": {[^}]*}' gpurun_out/r03_bench_c4_order.log; grep -o '"value": [0-9.e+]*' gpurun_out/r03_bench_c4_order.log
