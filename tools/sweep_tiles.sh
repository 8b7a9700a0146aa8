#!/bin/bash
# tile-shape sweep of the followed-by kernel (bench, no CPU leg)
for cfg in "2048 512" "2048 1024" "4096 512" "1024 512" "4096 1024"; do
  set -- $cfg
  SG_FB_TILE_T=$1 SG_FB_TILE_H=$2 timeout -k 10 200 python bench.py --steps 5 --warmup 1 --events ${EV:-100000000} --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('T=$1 H=$2', round(d['value']/1e9,3), 'Gev/s', round(d['roofline']['kernel_ms'],3), 'ms', round(d['roofline']['frac'],4))" || exit 1
done
