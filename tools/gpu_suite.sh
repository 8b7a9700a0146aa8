#!/bin/bash
# Full GPU suite (or the tests named in $2).  TAG names the outputs.
set -o pipefail
TAG=${1:-suite}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${*:-tests -m gpu} -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}.log 2>&1; rc=$?
tail -15 gpurun_out/${TAG}.log
exit $rc
