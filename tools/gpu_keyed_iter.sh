#!/bin/bash
# Keyed-pipeline iteration: bench with matcher phase probes, then the keyed parity tests.  TAG names outputs.
set -o pipefail
TAG=${1:-kt}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['kernel_ms'])"
SG_KT_DEBUG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/${TAG}_dbg.log 2>&1 || { tail -20 gpurun_out/${TAG}_dbg.log; exit 1; }
grep "match phases" gpurun_out/${TAG}_dbg.log | tail -1
timeout -k 10 900 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_keyed_headline.py tests/test_gpu_shard_rehearsal.py tests/test_gpu_compaction.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.log
exit $rc
