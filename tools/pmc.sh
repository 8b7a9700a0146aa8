#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only) over a short bench run.
# usage: tools/pmc.sh TAG "BENCH_ARGS"   -> gpurun_out/pmc_TAG/<pass>/..._counter_collection.csv
set -o pipefail
TAG=${1:-pmc}; ARGS=${2:-"--config 4 --steps 2 --warmup 1 --no-cpu --no-e2e"}
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
i=0
for pass in ${PASSES:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES"}; do
  i=$((i+1)); pass=${pass//_SQ_/ SQ_}
  echo "== pass $i: $pass ($(date +%T))"
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $R/gpurun_out/pmc_$TAG/p$i -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_${TAG}_p$i.log 2>&1
  rc=$?
  echo "== pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/pmc_${TAG}_p$i.log; exit $rc; }
done
echo "== done"
