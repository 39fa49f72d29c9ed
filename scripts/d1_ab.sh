# D1 and C4 under KANO_TUNE settings (ab_tune), then a D1 step timeline
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 scripts/ab_tune.py --config D1 --steps 100 --warmup 10 --reps 1 --timeout 200 -- "$@" || exit $?
timeout -k 10 600 python3 scripts/ab_tune.py --config C4 --steps 200 --warmup 10 --reps 1 --timeout 200 -- "$@" || exit $?
rm -rf gpurun_out/d1tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/d1tl -o run --output-format csv -- \
  python3 bench.py --config D1 --steps 10 --warmup 5 --cpu-baseline 0 --cold 0 --alone 0 > gpurun_out/d1tl.log 2>&1 || exit $?
python3 scripts/steps_tl.py $(find gpurun_out/d1tl -name "*kernel_trace.csv" | head -1) 8 > gpurun_out/d1_timeline.txt
