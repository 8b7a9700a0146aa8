#!/bin/bash
# round 3: collision debug, snapshot + shard tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dbg_shard_col.py > gpurun_out/r03_dbg_col.log 2>&1
echo "dbg rc=$?"; tail -12 gpurun_out/r03_dbg_col.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_snapshot.py \
  tests/test_gpu_shard_rehearsal.py tests/test_gpu_keyed.py > gpurun_out/r03_snap_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r03_snap_tests.log | grep -v PASSED | head -20; tail -2 gpurun_out/r03_snap_tests.log
