#!/bin/bash
# The driver's exact bench command repeated (stall hunt), then one run under
# rocprofv3 --hip-trace --kernel-trace (host API + kernels of the same command).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in ${REPS:-1 2 3}; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/b20_$k.json 2> gpurun_out/b20_$k.err || { tail gpurun_out/b20_$k.err; exit 1; }
  python3 - "$k" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/b20_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("b20", sys.argv[1], round(d["ms_per_step"], 4), d["step_ms"]["median"], d["step_ms"]["max"], d["step_ms"]["worst5_at"], round(d["roofline"]["avg_launch_ms"], 4), round(d["roofline"]["frac"], 3), d["host_us"], d["verified"])
PY
done
if [ "${TRACE:-1}" = 1 ]; then
  rm -rf gpurun_out/ht
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/ht -o run --output-format csv -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/ht.json 2> gpurun_out/ht.err || { tail gpurun_out/ht.err; exit 1; }
  python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/ht.json").read().strip().splitlines()[-1])
print("traced", round(d["ms_per_step"], 4), d["step_ms"], d["host_us"])
PY
fi
