#!/bin/bash
# Exploration session: kernel stats of configs 2 and 1, and keyed tuning variants.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for c in 2 1; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c$c -o prof -- python3 $R/bench.py --config $c --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof_c$c.log 2>&1
  rc=$?; cd $R; echo "== prof c$c rc=$rc"; tail -1 gpurun_out/prof_c$c.log | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
done
bash tools/sweep_keyed.sh ex "SG_KT_CHUNK=2048" "SG_KT_CHUNK=4096" "SG_KT_CHUNK=8192" "SG_KT_TILE=4096" "SG_KT_EXP=1"
