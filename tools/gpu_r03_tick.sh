#!/bin/bash
# NFA tick indexes: absent/NFA GPU tests, then config-5 (and config-3) bench lines with the indexes and with
# the per-event binary searches (SG_NFA_TICK_SEARCH=1), on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${T:-tick}
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread ${TESTS:-tests/test_gpu_absent.py \
  tests/test_gpu_partitioned_absent.py tests/test_gpu_nfa_configs.py tests/test_gpu_nfa_spec.py tests/test_gpu_shard_nfa.py \
  tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_gpu_purge.py} > gpurun_out/r03_${T}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/r03_${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in ${CONFIGS:-5}; do
for v in ${VARIANTS:-idx search}; do
  if [ $v = search ]; then export SG_NFA_TICK_SEARCH=1; else unset SG_NFA_TICK_SEARCH; fi
  timeout -k 10 400 python -u bench.py --config $c --no-cpu --steps 2 --warmup 1 > gpurun_out/r03_${T}_bench_c${c}_$v.log 2>&1
  rc=$?; echo "bench c$c $v rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/r03_${T}_bench_c${c}_$v.log; exit $rc; fi
  grep -o '"kernel_ms": {"k_nfa_lanes": [0-9.]*\|"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' gpurun_out/r03_${T}_bench_c${c}_$v.log
done
done
