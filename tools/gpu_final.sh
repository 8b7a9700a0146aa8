#!/bin/bash
# Round-end style session: smoke, full GPU suite, bench (N=1, with CPU baseline), kernel-trace profile,
# PMC traffic passes.  TAG names the outputs.
set -o pipefail
TAG=${1:-fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_all.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_all.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o prof -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $R/gpurun_out/${TAG}_prof.log 2>&1 || { cd $R; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
cd $R
PASSES="FETCH_SIZE WRITE_SIZE" bash tools/pmc.sh $TAG "--config 4 --steps 2 --warmup 1 --no-cpu --no-e2e"
for c in 1 2 3 5; do
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_c$c.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_c$c.log; exit 1; }
  tail -1 gpurun_out/${TAG}_bench_c$c.log | cut -c1-200
done
