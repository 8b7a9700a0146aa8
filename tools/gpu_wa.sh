#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config 2 --steps 5 --warmup 2 --no-cpu > gpurun_out/wa_c2.log 2>&1 || { tail -5 gpurun_out/wa_c2.log; exit 1; }
tail -1 gpurun_out/wa_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,2), round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernel_ms'].items() if v>0}, d['roofline'].get('frac'))"
