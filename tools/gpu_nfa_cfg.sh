#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nfa_configs.py -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/nfacfg_tests.log 2>&1; rc=$?
tail -12 gpurun_out/nfacfg_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py --config 3 --steps 3 --warmup 1 > gpurun_out/nfacfg_bench3.log 2>&1 || { tail -5 gpurun_out/nfacfg_bench3.log; exit 1; }
tail -1 gpurun_out/nfacfg_bench3.log
