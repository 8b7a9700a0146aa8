#!/bin/bash
# NFA build variants: config 3 and config 5 bench with each alternative library (SG_LIB).  TAG names outputs.
set -o pipefail
TAG=${1:-nv}; shift
mkdir -p gpurun_out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$GRAFT_REPO_ROOT/siddhi_amd/_build/var/libsg_$v.so
  for c in 3 5; do
    SG_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_${v}_c$c.log 2>&1 || { echo "$v c$c FAILED"; tail -5 gpurun_out/${TAG}_${v}_c$c.log; exit 1; }
    echo "$v c$c $(tail -1 gpurun_out/${TAG}_${v}_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,2), 'Mev/s', round(d['ms_per_step'],1), 'ms', {k: round(v,1) for k,v in d.get('kernel_ms',{}).items()})")"
  done
done
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_c4.log 2>&1 || { tail -5 gpurun_out/${TAG}_c4.log; exit 1; }
tail -1 gpurun_out/${TAG}_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value']/1e9, d['ms_per_step'], d.get('end_to_end'))"
