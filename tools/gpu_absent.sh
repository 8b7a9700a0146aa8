mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_absent.py -q -p no:cacheprovider --timeout 240 > gpurun_out/abs_tests.log 2>&1; echo "absent rc=$?"; tail -3 gpurun_out/abs_tests.log
timeout -k 10 200 python tools/kat_lowering.py absent > gpurun_out/abs_lowering.log 2>&1; echo "lowering rc=$?"; head -20 gpurun_out/abs_lowering.log
timeout -k 10 200 python tools/kat_lowering.py Window > gpurun_out/win_lowering.log 2>&1; head -12 gpurun_out/win_lowering.log
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/abs_all.log 2>&1; echo "all rc=$?"; tail -3 gpurun_out/abs_all.log
