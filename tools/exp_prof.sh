#!/bin/bash
# rocprofv3 kernel traces of the keyed bench under SG_KT_EXP variants; summaries only (dbs deleted).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for v in ${EXPS:-0 9 1}; do
  cd /tmp
  SG_KT_EXP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/exp_$v -o run -- python3 $R/bench.py --config 4 --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/exp_$v.log 2>&1 || exit 1
  cd $R
  python3 tools/prof_summary.py $(ls /tmp/exp_$v/*/run_results.db /tmp/exp_$v/run_results.db 2>/dev/null | head -1) > gpurun_out/exp_$v.csv
done
