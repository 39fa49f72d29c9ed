mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_path.py tests/test_matrix_io.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/path_tests.log 2>&1; rc=$?; tail -3 gpurun_out/path_tests.log; [ $rc -eq 0 ] || exit $rc
SPECS="C4:2:auto,bitwise,mfma C4:0:auto C3:2:auto" bash scripts/path_prof.sh
