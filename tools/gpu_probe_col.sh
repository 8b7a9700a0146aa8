#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for n in ${SIZES:-5000 20000 50000}; do
  timeout -k 10 ${TL:-240} python -u tools/probe_collisions.py $n 1000 10 >> gpurun_out/r03_probe_col.log 2>&1
  rc=$?; echo "n=$n rc=$rc"; tail -1 gpurun_out/r03_probe_col.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
