#!/bin/bash
# config 3 NFA lanes: lanes per workgroup sweep (SG_NFA_TPB)
for t in "$@"; do
  SG_NFA_TPB=$t timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu > gpurun_out/nfa_tpb_cur.log 2>&1 || { tail -3 gpurun_out/nfa_tpb_cur.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/nfa_tpb_cur.log').read().strip().splitlines()[-1]); print('tpb $t', round(d['value']/1e6,2), 'Mev/s', round(d['ms_per_step'],1), 'ms step', d['kernel_ms'])"
done
