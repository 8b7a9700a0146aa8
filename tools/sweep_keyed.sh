#!/bin/bash
# Keyed bench under tuning env vars (one bench per variant); lines to gpurun_out/sweep_TAG.log
set -o pipefail
TAG=${1:-sw}; shift
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v ($(date +%T))"
  timeout -k 10 300 env $v python bench.py --config 4 --steps 3 --warmup 1 --no-cpu > gpurun_out/sweep_${TAG}_cur.log 2>&1
  rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/sweep_${TAG}_cur.log; exit $rc; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${TAG}_cur.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,2), 'Gev/s', round(d['ms_per_step'],2), 'ms', {k: round(x,2) for k,x in d.get('kernel_ms',{}).items()})" | tee -a gpurun_out/sweep_${TAG}.log
done
