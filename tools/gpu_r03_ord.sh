#!/bin/bash
# Order-pass rows with absolute slots + LDS-staged output: keyed GPU tests, then the config-4 bench, its
# rocprofv3 kernel stats and the PMC passes (with the calibration binary).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_keyed.py tests/test_gpu_keyed_headline.py \
  tests/test_gpu_shard_rehearsal.py tests/test_gpu_compaction.py tests/test_gpu_snapshot.py tests/test_gpu_parity.py > gpurun_out/r03_ord_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03_ord_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r03_ord_tests.log | head; exit 1; fi
STEPS="b4 prof4 pmc4 calib" T=${T:-r03p} bash tools/gpu_r03_final.sh
