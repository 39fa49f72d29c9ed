set -u
O=gpurun_out/d1tl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf $O/tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tl -o run --output-format csv -- \
  python3 bench.py --config D1 --steps 6 --warmup 2 --cpu-baseline 0 --cold 0 --alone 0 > $O/tl.log 2>&1 || exit 1
python3 scripts/steps_tl.py $(find $O/tl -name "*kernel_trace.csv" | head -1) > $O/d1_step_timeline.txt
cp $(find $O/tl -name "*kernel_stats.csv" | head -1) $O/d1_kernel_stats.csv
rm -rf $O/tl
