#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dbg_ks.py > gpurun_out/r03_dbg_ks.log 2>&1; echo "dbg rc=$?"; cat gpurun_out/r03_dbg_ks.log | tail -40
for lb in 10 9; do
  SG_KS_LB=$lb SG_KT_DEBUG=1 timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/r03_bench_c4_lb$lb.log 2>&1
  rc=$?; echo "bench lb=$lb rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  grep -o '"kernel_ms": {[^}]*}' gpurun_out/r03_bench_c4_lb$lb.log
done
SG_KEYED_NO_STACK=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r03_bench_c4_tiles.log 2>&1
echo "bench tiles rc=$?"; grep -o '"kernel_ms": {[^}]*}' gpurun_out/r03_bench_c4_tiles.log; grep -o '"end_to_end": {[^}]*}' gpurun_out/r03_bench_c4_tiles.log
