mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/kab.sh "k_cls_insert|k_cls_assign|k_sel_place|k_pol_counts|k_rows" "" || exit 1
CFG=C4 EXTRA=--no-shadow bash scripts/kab.sh "k_cls_insert|k_cls_assign|k_sel_place|k_pol_counts|k_rows" "" || exit 1
REPS=2 bash scripts/tab.sh ""
