#!/bin/bash
# One bench line per config plus a rocprofv3 kernel-stats summary of each (round-end evidence).
# usage: tools/bench_all.sh TAG   -> gpurun_out/bench_TAG_c{N}.log, gpurun_out/prof_TAG_c{N}/
set -o pipefail
TAG=${1:-rNN}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for c in 1 2 3 5; do
  echo "== config $c ($(date +%T))"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_c$c -o run -- \
    python3 $R/bench.py --config $c --steps 3 --warmup 1 > $R/gpurun_out/bench_${TAG}_c$c.log 2>&1 || exit $?
  grep '^{' $R/gpurun_out/bench_${TAG}_c$c.log | cut -c1-300
done
