#!/bin/bash
# Host-side phase times (SG_HOST_TIMING) of the NFA-path benches (configs 3 and 5).
set -o pipefail
mkdir -p gpurun_out
for c in 3 5; do
  SG_HOST_TIMING=1 timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu > gpurun_out/ht_c$c.log 2>&1 || { tail -5 gpurun_out/ht_c$c.log; exit 1; }
  grep "sg phase\|HostTimer\|\[sg" gpurun_out/ht_c$c.log | tail -30
done
