#!/bin/bash
# One GPU-box session: build, smoke, GPU tests per path, bench, rocprof kernel stats.
# A step that fails with an ordinary test failure (rc 1) does not stop the session; anything else
# (timeout 124/137, abort 134, segfault 139, GPU fault) ends it there.
# usage: tools/gpu_round.sh TAG "PROF_BENCH_ARGS" [steps...]   steps: smoke fb wa keyed nfa bench bench1 bench2 small4 prof
set -o pipefail
TAG=${1:-run}; PROF_ARGS=${2:-"--config 4"}; shift 2
STEPS=${*:-"smoke fb wa bench prof nfa"}
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/${TAG}_$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/${TAG}_build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/${TAG}_build.log; exit 1; }
for s in $STEPS; do
  case $s in
    smoke) run dbg 120 python -u tools/dbg_smoke.py 2000 && run smoke 240 python -c "import __graft_entry__ as g; g.smoke()" ;;
    fb) run fb 600 env SG_PATHS=followed_by python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 ;;
    wa) run wa 600 env SG_PATHS=window_agg python -m pytest tests/test_gpu_window.py -q -p no:cacheprovider --timeout 240 &&
        run wakat 600 env SG_PATHS=window_agg python -m pytest tests/test_gpu_parity.py -k kat -q -p no:cacheprovider --timeout 240 ;;
    keyed) run keyed 600 env SG_PATHS=keyed python -m pytest tests/test_gpu_keyed.py -x -q -p no:cacheprovider --timeout 240 &&
        run keyedkat 600 env SG_PATHS=keyed python -m pytest tests/test_gpu_parity.py -k kat -q -p no:cacheprovider --timeout 240 ;;
    nfa) run nfa 600 env SG_PATHS=nfa python -m pytest tests/test_gpu_parity.py -k kat -q -p no:cacheprovider --timeout 240 ;;
    all) run all 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ;;
    bench) run bench 500 python bench.py --steps 5 --warmup 2 ;;
    bench1) run bench1 400 python bench.py --config 1 --steps 5 --warmup 2 ;;
    bench2) run bench2 400 python bench.py --config 2 --steps 5 --warmup 2 ;;
    small4) run small4 300 python bench.py --config 4 --events 100000000 --steps 3 --warmup 1 --no-cpu ;;
    prof) cd /tmp && run_dir=$R/gpurun_out/prof_$TAG && \
          timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $run_dir -o prof -- python3 $R/bench.py --steps 5 --warmup 1 $PROF_ARGS --no-cpu > $R/gpurun_out/${TAG}_prof.log 2>&1; rc=$?; cd $R; echo "== prof rc=$rc"; \
          [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_prof.log; exit $rc; } ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "== done"
