# k_rows_w: the forced-variant parity tests and C5 at full size, then C5
# rank 0 of 8 and C5 under the given settings
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_configs.py -x -q -m gpu --timeout 300 --timeout-method thread -k "rows_variants_forced or c5_full" > gpurun_out/rw_tests.log 2>&1; rc=$?; tail -3 gpurun_out/rw_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 scripts/ab_tune.py --config C5 --steps 12 --warmup 3 --reps 1 --timeout 280 --extra "--rank-of 8 --alone 3" -- "$@" || exit $?
timeout -k 10 900 python3 scripts/ab_tune.py --config C5 --steps 5 --warmup 2 --reps 1 --timeout 300 --extra "--alone 3" -- "$@"
