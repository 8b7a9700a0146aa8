#!/bin/bash
# Batched Scheduler-collision resolution: absent/NFA GPU tests, then the natural-collision probe by size.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_partitioned_absent.py \
  tests/test_gpu_shard_nfa.py tests/test_gpu_absent.py tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_gpu_purge.py \
  > gpurun_out/r03_col_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r03_col_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/r03_col_tests.log | head -10; exit 1; }
for n in ${SIZES:-5000 20000 100000}; do
  timeout -k 10 240 python -u tools/probe_collisions.py $n 1000 10 >> gpurun_out/r03_col_probe.log 2>&1
  rc=$?; echo "n=$n rc=$rc"; tail -1 gpurun_out/r03_col_probe.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
