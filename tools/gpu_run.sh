#!/bin/bash
# GPU evidence runs: T names the outputs (gpurun_out/${T}_<step>.log), STEPS picks the steps.  Default: smoke,
# the full GPU suite, the default bench line (config 4 with the end-to-end sample and the CPU baseline), its
# rocprofv3 kernel stats, and the PMC passes (config 4 and the access-width calibration binary).
# Other steps: b1 b2 b3 b5 (bench the other configs), prof3 prof5, pmc3, rec (record the cross-rank collision
# fixture tests/golden/sched_collision_w2.npz into gpurun_out/), abs colt shd (absent / collision / shard tests),
# col20 col100 col100t col1m (tools/probe_collisions.py at 20K-1M colliding events).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${T:-r04a}
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_$name.log" 2>&1
  local rc=$?
  tail -2 "gpurun_out/${T}_$name.log" | cut -c1-300
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
prof() {  # name timeout args...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  (cd /tmp && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${T}_$name -o run -- \
     python3 $R/bench.py "$@" > $R/gpurun_out/${T}_$name.log 2>&1)
  local rc=$?
  echo "== $name rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
pmc() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  echo "== pmc $name $ctr ($(date +%T))"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmc_${T}_$name/$ctr -o run -- "$@" \
     > $R/gpurun_out/pmc_${T}_${name}_$ctr.log 2>&1)
  local rc=$?
  echo "== pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
  return 0
}
for s in ${STEPS:-smoke all b4 prof4 pmc4 calib}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    all) step all 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
    b4) step b4 500 python bench.py ;;
    prof4) prof prof4 300 --steps 5 --warmup 1 --no-cpu --no-e2e ;;
    pmc4) pmc c4 FETCH_SIZE python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e &&
          pmc c4 WRITE_SIZE python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e ;;
    pmc4w) pmc c4 WRITE_SIZE python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e ;;
    calibw) pmc calib WRITE_SIZE $R/tools/micro/pmc_calib ;;
    calib) pmc calib FETCH_SIZE $R/tools/micro/pmc_calib && pmc calib WRITE_SIZE $R/tools/micro/pmc_calib ;;
    kc) step kc 900 python -u -m pytest tests/test_gpu_keyed_chunks.py tests/test_gpu_keyed_headline.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    keyed) step keyed 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_snapshot.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    nfa3) step nfa3 600 python -u -m pytest tests/test_gpu_nfa_bench_defaults.py tests/test_gpu_snapshot.py -x -q -s -p no:cacheprovider --timeout 400 --timeout-method thread ;;
    kcexp) for v in 0 1 2 3; do step kcexp$v 300 env SG_KC_EXP=$v SG_KT_DEBUG=1 python bench.py --no-cpu --no-e2e --steps 3 --warmup 1; done ;;
    nfa) step nfa 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nfa_configs.py tests/test_gpu_nfa_state.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    wdev) step wdev 900 python -u -m pytest tests/test_gpu_window_dev.py tests/test_gpu_window_gen.py tests/test_gpu_parity.py tests/test_gpu_snapshot.py tests/test_gpu_window.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    h5) step h5 400 env SG_HOST_TIMING=1 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    cmp) step cmp 900 python -u -m pytest tests/test_gpu_nfa_compaction.py tests/test_gpu_nfa_bench_defaults.py tests/test_gpu_snapshot.py tests/test_gpu_nfa_state.py -q -x -p no:cacheprovider --timeout 400 --timeout-method thread ;;
    d3) step d3 150 env SG_HOST_TIMING=1 python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    t3) for sw in "128 32" "64 32" "96 32" "192 32" "256 48" "128 16" "128 64"; do set -- $sw
          step t3_$1_$2 120 env SG_NFA_SEG=$1 SG_NFA_WARM=$2 python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    p5) step p5 200 env SG_LIB=siddhi_amd/_probe/libsiddhi_gfx.so python -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu ;;
    p3) step p3 200 env SG_LIB=siddhi_amd/_probe/libsiddhi_gfx.so python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    p3n) step p3n 200 env SG_LIB=siddhi_amd/_probe/libsiddhi_gfx.so SG_NFA_SPEC=0 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    nst) step nst 400 python -u -m pytest tests/test_gpu_nfa_state.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    ext) step ext 300 python -u -m pytest tests/test_gpu_ext.py tests/test_gpu_snapshot.py -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
    r2) for c in 3 5 4; do
          ev=2000000; [ $c = 4 ] && ev=100000000
          step r2c$c 400 env SG_BENCH_DIST=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port $((29500 + c)) bench.py --gpus 2 --config $c --events $ev --steps 2 \
            --warmup 1 --no-cpu --no-e2e
        done ;;
    kpar) step kpar 600 env SG_HOST_PAR_MIN=64 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_absent.py tests/test_gpu_partitioned_absent.py tests/test_gpu_nfa_configs.py tests/test_gpu_window_gen.py tests/test_gpu_window.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sst) step sst 600 python -u -m pytest tests/test_gpu_shard_stream.py -q -x -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    r25) step r25 400 env SG_BENCH_DIST=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port 29505 bench.py --gpus 2 --config 5 --events 2000000 --steps 2 \
            --warmup 1 --no-cpu --no-e2e ;;
    kt) step kt 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_keyed_chunks.py tests/test_gpu_compaction.py tests/test_gpu_shard_rehearsal.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    b4e) step b4e 600 python bench.py --no-cpu ;;
    b4q) step b4q 300 python bench.py --no-cpu --no-e2e ;;
    rec) step rec 300 python tools/record_sched_logs.py gpurun_out/sched_collision_w2.npz ;;
    b1) step b1 400 python bench.py --config 1 ;;
    b2) step b2 400 python bench.py --config 2 ;;
    b3) step b3 400 python bench.py --config 3 ;;
    b5) step b5 500 python bench.py --config 5 ;;
    prof3) prof prof3 300 --config 3 --steps 3 --warmup 1 --no-cpu ;;
    prof5) prof prof5 400 --config 5 --steps 2 --warmup 1 --no-cpu ;;
    pmc3) pmc c3 FETCH_SIZE python3 $R/bench.py --config 3 --steps 2 --warmup 1 --no-cpu &&
          pmc c3 WRITE_SIZE python3 $R/bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    pmc5) pmc c5 FETCH_SIZE python3 $R/bench.py --config 5 --steps 2 --warmup 1 --no-cpu &&
          pmc c5 WRITE_SIZE python3 $R/bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    abs) step abs 900 python -u -m pytest tests/test_gpu_partitioned_absent.py tests/test_gpu_nfa_spec.py tests/test_gpu_shard_nfa.py tests/test_gpu_collisions.py tests/test_gpu_snapshot.py -q -x -s -p no:cacheprovider --timeout 400 --timeout-method thread ;;
    colt) step colt 600 python -u -m pytest tests/test_gpu_collisions.py -v -s -p no:cacheprovider --timeout 150 --timeout-method thread ;;
    colnc) step colnc 300 env SG_NFA_NO_COMPACT=1 python -u -m pytest tests/test_gpu_collisions.py -v -s -p no:cacheprovider --timeout 150 --timeout-method thread -k "across or snapshot" ;;
    shd) step shd 600 python -u -m pytest tests/test_gpu_shard_nfa.py tests/test_gpu_shard_rehearsal.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    col20) step col20 300 python -u tools/probe_collisions.py 20000 ;;
    colx) for v in "SG_NFA_NO_LDS=1" "SG_NFA_TPB=64" "SG_NFA_TPB=16" "SG_NFA_SWEEP_TICKS=128" "SG_NFA_SWEEP_TICKS=8" "SG_NFA_NO_LDS=1 SG_NFA_TPB=64"; do
            step "colx_${v// /_}" 300 env $v python -u tools/probe_collisions.py 20000; done ;;
    col100) step col100 400 python -u tools/probe_collisions.py 100000 ;;
    col100t) step col100t 400 env SG_HOST_TIMING=1 python -u tools/probe_collisions.py 100000 ;;
    col1m) step col1m 900 python -u tools/probe_collisions.py 1000000 ;;
    b3r0) step b3r0 300 env SG_NFA_RTC=0 python bench.py --config 3 --no-cpu --steps 3 --warmup 1 ;;
    b3r1) step b3r1 300 env SG_NFA_RTC=1 python bench.py --config 3 --no-cpu --steps 3 --warmup 1 ;;
    b5r0) step b5r0 400 env SG_NFA_RTC=0 python bench.py --config 5 --no-cpu --steps 2 --warmup 1 ;;
    b5r1) step b5r1 400 env SG_NFA_RTC=1 python bench.py --config 5 --no-cpu --steps 2 --warmup 1 ;;
    rtc) step rtc 900 python -u -m pytest tests/test_gpu_nfa_rtc.py -v -s -x --tb=short -p no:cacheprovider --timeout 600 --timeout-method thread ;;
    rtc3) step rtc3 600 python -u -m pytest tests/test_gpu_nfa_rtc.py -v -s --tb=short -p no:cacheprovider --timeout 300 --timeout-method thread -k "config3 or config5 or sweep" ;;
    rtcall) step rtcall 1150 env SG_RTC_ALL_KATS=1 SG_RTC_CACHE=$R/siddhi_amd/_build/rtc_kats python -u -m pytest tests/test_gpu_nfa_rtc.py -q -s -p no:cacheprovider --timeout 1100 --timeout-method thread -k reference_kat ;;
    kcb) step kcb 300 python bench.py --no-cpu --no-e2e --steps 5 --warmup 1 ;;
    kcb2) step kcb2 300 python bench.py --no-cpu --no-e2e --steps 5 --warmup 1 ;;
    kcar) step kcar 300 env SG_KC_PEER_RANK=1 python bench.py --no-cpu --no-e2e --steps 5 --warmup 1 &&
          step kcart 600 env SG_KC_PEER_RANK=1 python -u -m pytest tests/test_gpu_keyed_chunks.py tests/test_gpu_keyed_headline.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    fbw) step fbw 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_window.py tests/test_gpu_split.py tests/test_gpu_nulls.py tests/test_gpu_ext.py tests/test_gpu_compaction.py -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    kcph) step kcph 300 env SG_KT_DEBUG=1 python bench.py --no-cpu --no-e2e --steps 3 --warmup 1 ;;
    kcw) for v in 6 8 4; do step kcw$v 300 env SG_KC_WPE=$v python bench.py --no-cpu --no-e2e --steps 5 --warmup 1; done ;;
    b3np) step b3np 300 env SG_NFA_NO_PACK=1 python bench.py --config 3 --no-cpu --steps 3 --warmup 1 ;;
    b5np) step b5np 400 env SG_NFA_NO_PACK=1 python bench.py --config 5 --no-cpu --steps 2 --warmup 1 ;;
    nfat) step nfat 900 python -u -m pytest tests/test_gpu_nfa_spec.py tests/test_gpu_partitioned_absent.py tests/test_gpu_nfa_configs.py tests/test_gpu_config5_bench_size.py tests/test_gpu_nfa_bench_defaults.py -q -x -s -p no:cacheprovider --timeout 400 --timeout-method thread ;;
    kcsq) echo "== kcsq ($(date +%T))"
          PASSES="SQ_WAVE_CYCLES_SQ_WAIT_ANY_SQ_WAIT_INST_ANY_SQ_ACTIVE_INST_ANY_SQ_WAIT_INST_LDS_SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT_SQ_INSTS_VALU_SQ_INSTS_VMEM_RD_SQ_INSTS_VMEM_WR_SQ_BUSY_CYCLES_SQ_WAVES" \
            bash tools/pmc.sh ${T}_kcsq "--config 4 --steps 2 --warmup 1 --no-cpu --no-e2e" > gpurun_out/${T}_kcsq.log 2>&1 || exit $? ;;
    nat) step nat 600 python -u -m pytest tests/test_gpu_shard_nfa.py -v -s -p no:cacheprovider --timeout 500 --timeout-method thread -k natural ;;
    nsq) for c in 3 5; do echo "== nsq$c ($(date +%T))"
           PASSES="SQ_WAVE_CYCLES_SQ_WAIT_ANY_SQ_WAIT_INST_ANY_SQ_ACTIVE_INST_ANY_SQ_WAIT_INST_LDS_SQ_INSTS_LDS SQ_INSTS_VALU_SQ_INSTS_VMEM_RD_SQ_INSTS_VMEM_WR_SQ_BUSY_CYCLES_SQ_WAVES" \
             bash tools/pmc.sh ${T}_nsq$c "--config $c --steps 2 --warmup 1 --no-cpu" > gpurun_out/${T}_nsq$c.log 2>&1 || exit $?; done ;;
    shr) step shr 900 python -u tools/probe_shard_rounds.py 200000 2 1 2 3 ;;
    shr2) step shr2a 300 python -u tools/probe_shard_rounds.py 20000 2 1 10 && step shr2b 300 python -u tools/probe_shard_rounds.py 50000 2 1 10 &&
          step shr2c 300 python -u tools/probe_shard_rounds.py 20000 4 1 10 ;;
    src) echo "== src ($(date +%T))"   # from-source build() on the box, then smoke (heartbeat: a silent compile is taken as hung)
         (timeout -k 10 1000 python -u -c "import time; t=time.time(); import __graft_entry__ as g; g.build(); print('build() %.0f s' % (time.time()-t), flush=True); g.smoke(); print('smoke ok', flush=True)" > gpurun_out/${T}_src.log 2>&1) &
         pid=$!; while kill -0 $pid 2>/dev/null; do sleep 30; echo "  building/smoke ($(date +%T))"; done; wait $pid; rc=$?
         tail -3 gpurun_out/${T}_src.log; echo "== src rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    r2e) for c in 4 3; do
          ev=2000000; [ $c = 4 ] && ev=50000000
          step r2e$c 400 env SG_BENCH_DIST=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
            --master-addr 127.0.0.1 --master-port $((29600 + c)) bench.py --gpus 2 --config $c --events $ev --steps 2 \
            --warmup 1 --no-cpu
        done ;;
    s1) for v in 32 16 8 4 2; do step s1_$v 200 env SG_FB_S1=$v python bench.py --config 1 --no-cpu --steps 10 --warmup 2; done ;;
    pmc1) pmc c1 FETCH_SIZE python3 $R/bench.py --config 1 --steps 3 --warmup 1 --no-cpu &&
          pmc c1 WRITE_SIZE python3 $R/bench.py --config 1 --steps 3 --warmup 1 --no-cpu ;;
    pmc2) pmc c2 FETCH_SIZE python3 $R/bench.py --config 2 --steps 3 --warmup 1 --no-cpu &&
          pmc c2 WRITE_SIZE python3 $R/bench.py --config 2 --steps 3 --warmup 1 --no-cpu ;;
    prof1) prof prof1 300 --config 1 --steps 5 --warmup 1 --no-cpu ;;
    prof2) prof prof2 300 --config 2 --steps 5 --warmup 1 --no-cpu ;;
    exp) step exp 900 python -u -m pytest tests/test_gpu_nfa_expiry.py -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bg) step bg 600 python -u -m pytest tests/test_gpu_nfa_rtc.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "background or config3 or config5" ;;
    b3q) step b3q 300 python bench.py --config 3 --no-cpu --steps 5 --warmup 1 ;;
    b5q) step b5q 400 python bench.py --config 5 --no-cpu --steps 3 --warmup 1 ;;
    b5spec) for w in ${WARMS:-32 128 512}; do
              step b5spec_w$w 400 env SG_NFA_SPEC=1 SG_NFA_SPEC_STATS=${STATS:-1} SG_NFA_WARM=$w SG_NFA_SEG=${SEG:-512} \
                python bench.py --config 5 --no-cpu --no-e2e --steps 2 --warmup 1
            done ;;
    spect) step spect 600 python -u -m pytest tests/test_gpu_nfa_spec.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    wpe) for w in ${WPES:-2 3 4}; do
           step b5wpe$w 300 env SG_RTC_WPE=$w python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 &&
           step b3wpe$w 300 env SG_RTC_WPE=$w python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    tpb) for v in ${TPBS:-4 8 16 32}; do
           step b5tpb$v 300 env SG_NFA_TPB=$v python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 &&
           step b3tpb$v 300 env SG_NFA_TPB=$v python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    sh5) for sw in ${SHS:-"192 128" "256 96" "384 128" "256 160"}; do set -- $sw
           step b5sh_$1_$2 300 env SG_NFA_SEG=$1 SG_NFA_WARM=$2 python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1; done ;;
    lds) for v in "SG_NFA_NO_LDS=1" "SG_NFA_SPEC_CAPS=8,32,8" "SG_NFA_SPEC_CAPS=12,32,12" "SG_NFA_SPEC_CAPS=8,16,8"; do
           step "b5_${v//[=,]/_}" 300 env $v python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 &&
           step "b3_${v//[=,]/_}" 300 env $v python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    nolds) for v in "SG_NFA_TPB=32" "SG_NFA_TPB=16" "SG_RTC_WPE=2" "SG_RTC_WPE=3" "SG_RTC_WPE=2 SG_NFA_TPB=32"; do
           step "b5nl_${v//[= ]/_}" 300 env SG_NFA_NO_LDS=1 $v python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 &&
           step "b3nl_${v//[= ]/_}" 300 env SG_NFA_NO_LDS=1 $v python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    offt) for v in 0 1 0 1; do step b4offt$v 300 env SG_KC_OFFT=$v python bench.py --no-cpu --no-e2e --steps 10 --warmup 2; done ;;
    caps) for v in ${CAPSS:-"8,32,8" "8,16,8" "12,48,12"}; do
           step "b5caps_${v//,/_}" 300 env SG_NFA_SPEC_CAPS=$v python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 &&
           step "b3caps_${v//,/_}" 300 env SG_NFA_SPEC_CAPS=$v python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    blk) for v in 1 0; do if [ $v = 1 ]; then e="SG_NFA_NO_BLOCK=1"; else e="SG_NFA_X=0"; fi
           step b5blk$v 300 env $e python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 &&
           step b3blk$v 300 env $e python bench.py --config 3 --no-cpu --steps 3 --warmup 1; done ;;
    c5t) step c5t 400 python -u -m pytest tests/test_gpu_config5_bench_size.py -q -x -s -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    chn) step chn 900 python -u -m pytest tests/test_gpu_config5_bench_size.py tests/test_gpu_nfa_configs.py tests/test_gpu_parity.py tests/test_gpu_partitioned_absent.py tests/test_gpu_purge.py tests/test_gpu_nfa_state.py -q -x -s -p no:cacheprovider --timeout 400 --timeout-method thread ;;
    b5n) step b5n 300 python bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 ;;
    b3n) step b3n 300 python bench.py --config 3 --no-cpu --steps 3 --warmup 1 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "== done"
