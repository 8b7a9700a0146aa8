#!/bin/bash
# window fix check + keyed phase probes + scatter-only measurement
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 env SG_PATHS=window_agg python -m pytest tests/test_gpu_window.py -x -q -p no:cacheprovider --timeout 240 > gpurun_out/ex2_wa.log 2>&1; rc=$?
tail -2 gpurun_out/ex2_wa.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 2 --steps 5 --warmup 2 > gpurun_out/ex2_bench2.log 2>&1 || exit $?
grep -o '"kernel_ms": {[^}]*}' gpurun_out/ex2_bench2.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ex2_bench2.log
timeout -k 10 300 env SG_KT_DEBUG=1 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu > gpurun_out/ex2_dbg.log 2>&1 || exit $?
grep "kt match phases\|kt host" gpurun_out/ex2_dbg.log | tail -3
bash tools/sweep_keyed.sh ex2 "SG_KT_EXP=3"
