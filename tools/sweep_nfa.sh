#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 300 env $v python bench.py --config 3 --steps 2 --warmup 1 --no-cpu > gpurun_out/nfa_sweep_cur.log 2>&1 || { tail -5 gpurun_out/nfa_sweep_cur.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/nfa_sweep_cur.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'Mev/s', d['kernel_ms'])"
done
