#!/bin/bash
# One GPU-box session: build, smoke, GPU tests, bench, rocprof kernel stats.
# usage: tools/gpu_check.sh [events] [tag]
set -o pipefail
EV=${1:-100000000}
TAG=${2:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --events $EV > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --events $EV --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo PROF FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -name "*kernel_stats*" | head -3
