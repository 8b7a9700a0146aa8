#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_keyed_stack.py \
  > gpurun_out/r03_ks_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03_ks_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for exp in 0 3; do
  SG_KS_EXP=$exp SG_KT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/r03_bench_c4_exp$exp.log 2>&1
  rc=$?; echo "bench exp=$exp rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep -o '"kernel_ms": {[^}]*}' gpurun_out/r03_bench_c4_exp$exp.log
done
