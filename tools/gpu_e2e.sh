#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/e2e_c4.log 2>&1 || { tail -5 gpurun_out/e2e_c4.log; exit 1; }
tail -1 gpurun_out/e2e_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value']/1e9, d['ms_per_step'], d.get('end_to_end'))"
