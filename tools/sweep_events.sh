#!/bin/bash
# Keyed bench at several flush sizes: per-event kernel cost vs working-set size (Infinity Cache residency)
set -o pipefail
mkdir -p gpurun_out
for ev in "$@"; do
  timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu --events $ev > gpurun_out/sweep_ev_cur.log 2>&1 || { tail -5 gpurun_out/sweep_ev_cur.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sweep_ev_cur.log').read().strip().splitlines()[-1]); n=$ev; print(n, round(d['value']/1e9,2), 'Gev/s', {k: round(x/n*1e9,3) for k,x in d.get('kernel_ms',{}).items() if x>0}, 'ns/kev')" | tee -a gpurun_out/sweep_ev.log
done
