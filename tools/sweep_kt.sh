#!/bin/bash
# Keyed tiled pipeline tuning sweep: one bench run per setting (env assignments as arguments).
# usage: tools/sweep_kt.sh "SG_KT_CHUNK=2048" "SG_KT_CHUNK=4096" ...   -> gpurun_out/sweep_kt.log
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/sweep_kt.log
: > $OUT
for setting in "$@"; do
  echo "== $setting" | tee -a $OUT
  env $setting timeout -k 10 240 python3 $R/bench.py --config 4 --steps 5 --warmup 2 --no-cpu >> $OUT 2>&1 || exit $?
done
