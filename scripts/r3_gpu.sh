#!/bin/bash
# Round-3 GPU iteration: the GPU test suite, the driver's bench command, and
# k_rows kernel stats under the matrix-write forms.  Every step bounded;
# the script stops at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYK:+-k "$PYK"} > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
  tail -3 gpurun_out/gpu_tests.txt
fi
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.json 2> gpurun_out/b20.err || { tail gpurun_out/b20.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/b20.json").read().strip().splitlines()[-1])
print("b20", d["ms_per_step"], d["step_ms"], d["roofline"]["kernel"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d.get("host_us"), d["verified"])
PY
for t in ${AB:-"" "store=0"}; do
  KANO_TUNE="$t" timeout -k 10 200 python3 bench.py --steps 300 --warmup 20 --cpu-baseline 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python3 - "$t" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
print("AB", repr(sys.argv[1]), "ms", round(d["ms_per_step"], 4), "median", d["step_ms"]["median"], d["roofline"]["kernel"], round(d["roofline"]["avg_launch_ms"], 4), round(d["roofline"]["frac"], 3), d["verified"])
PY
done
rm -rf gpurun_out/ks
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/ks.log 2>&1 || exit $?
f=$(find gpurun_out/ks -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/ks_stats.csv
head -12 gpurun_out/ks_stats.csv | cut -c1-150
