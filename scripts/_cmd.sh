mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
KANO_TUNE=mcrows=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu0.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_gpu0.log; [ $rc -eq 0 ] || exit $rc
REPS=3 bash scripts/tab.sh "" "mcrows=0"
