#!/bin/bash
# round 3 session 2: smoke, full GPU suite, bench lines (config 4 with rocprof stats, configs 3/5 with the
# specialised and the generic NFA interpreter).  Any non-test failure (rc not 0/1) ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-r03a}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_$name.log" 2>&1
  local rc=$?
  tail -2 "gpurun_out/${T}_$name.log" | cut -c1-400
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for s in ${STEPS:-smoke all c4 prof4 c3 c3g c5}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    all) step all 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    c4) step c4 400 python bench.py --steps 10 --warmup 2 ;;
    prof4) cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${T}_c4 -o run -- \
             python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $R/gpurun_out/${T}_prof4.log 2>&1; rc=$?; cd $R
           echo "== prof4 rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    c3) step c3 300 python bench.py --config 3 --steps 3 --warmup 1 ;;
    c3g) step c3g 300 env SG_NFA_GENERIC=1 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu ;;
    c5) step c5 300 python bench.py --config 5 --steps 3 --warmup 1 ;;
    c5g) step c5g 300 env SG_NFA_GENERIC=1 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    c3s0) step c3s0 300 env SG_NFA_SPEC=0 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu ;;
    c3ht) step c3ht 300 env SG_HOST_TIMING=1 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    spec) step spec 600 python -u -m pytest tests/test_gpu_nfa_spec.py -v -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    fails) step fails 600 python -u -m pytest tests/test_gpu_shard_nfa.py tests/test_gpu_keyed_headline.py \
             tests/test_gpu_parity.py::test_gpu_kat_coverage_floor -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    nfakat) step nfakat 600 env SG_PATHS=nfa python -u -m pytest tests/test_gpu_parity.py -k kat -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    c3sweep) for cfg in ${SWEEP:-"SG_NFA_SEG=256 SG_NFA_WARM=32"}; do
               cfg=${cfg//,/ }
               echo "-- $cfg"
               timeout -k 10 200 env $cfg python bench.py --config 3 --steps 2 --warmup 1 --no-cpu > gpurun_out/${T}_sweep.log 2>&1 || { echo "sweep rc=$?"; exit 3; }
               grep '^{' gpurun_out/${T}_sweep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), 'M ev/s', round(d['ms_per_step'],1), 'ms', {k: round(v,1) for k,v in d['kernel_ms'].items()})"
             done ;;
    keyed) step keyed 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_keyed_headline.py tests/test_gpu_keyed_stack.py \
             tests/test_gpu_shard_rehearsal.py tests/test_gpu_compaction.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    prof3) cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${T}_c3 -o run -- \
             python3 $R/bench.py --config 3 --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/${T}_prof3.log 2>&1; rc=$?; cd $R
           echo "== prof3 rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    absent) step absent 900 python -u -m pytest tests/test_gpu_partitioned_absent.py tests/test_gpu_absent.py tests/test_gpu_shard_nfa.py \
             tests/test_gpu_nfa_configs.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    c5stats) step c5stats 300 env SG_NFA_SPEC_STATS=1 python bench.py --config 5 --steps 1 --warmup 1 --no-cpu
             grep '^{' gpurun_out/${T}_c5stats.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), 'M ev/s', {k: round(v,1) for k,v in d['kernel_ms'].items()})" ;;
    c5s0) step c5s0 300 env SG_NFA_SPEC=0 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "== done"
