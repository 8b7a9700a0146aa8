#!/bin/bash
# XCD-contiguous matcher tiles / order groups: keyed GPU tests, then config-4 bench lines per variant (one box).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_keyed.py tests/test_gpu_keyed_headline.py \
  tests/test_gpu_shard_rehearsal.py tests/test_gpu_compaction.py > gpurun_out/r03_xcd_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r03_xcd_tests.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error" gpurun_out/r03_xcd_tests.log | head; exit 1; fi
for v in "1 1" "0 1" "1 0" "0 0" "1 1"; do
  set -- $v
  SG_KT_XCD=$1 SG_KO_XCD=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 5 --warmup 2 > gpurun_out/r03_xcd_$1$2.log 2>&1
  rc=$?; echo "kt_xcd=$1 ko_xcd=$2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
  grep -o '"kernel_ms": {[^}]*}' gpurun_out/r03_xcd_$1$2.log | cut -c1-200
done
