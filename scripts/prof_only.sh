set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 2 --cpu-baseline 0 > gpurun_out/prof.log 2>&1 || exit $?
bash scripts/pmc.sh > gpurun_out/pmc_run.log 2>&1 || exit $?
echo done
