#!/bin/bash
# Rebuild every HIP source from scratch on the GPU box (hipcc gfx950), then smoke the rebuilt library.
set -o pipefail
mkdir -p gpurun_out
( time timeout -k 10 900 python -c "from siddhi_amd import build as b; print(b.build(force=True, verbose=True))" ) > gpurun_out/box_build.log 2>&1 || { tail -20 gpurun_out/box_build.log; exit 1; }
tail -6 gpurun_out/box_build.log
ls -la siddhi_amd/_build/libsiddhi_gfx.so >> gpurun_out/box_build.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/box_build.log 2>&1 || { tail -5 gpurun_out/box_build.log; exit 1; }
tail -2 gpurun_out/box_build.log
