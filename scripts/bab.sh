#!/bin/bash
# Bench A/B: the default bench line under each KANO_TUNE setting (CFG, EXTRA
# from the env), printing mean / median step and k_rows' launch time.
#   bab.sh "t1" "t2" ...
set -u
mkdir -p gpurun_out
for t in "$@"; do
  KANO_TUNE="$t" timeout -k 10 150 python3 bench.py --steps ${STEPS:-50} --warmup ${WARMUP:-5} --cpu-baseline 0 \
    --config ${CFG:-C3} ${EXTRA:-} > gpurun_out/bab.log 2>&1
  rc=$?
  # rc 1: the line printed, results differ from the golden (experiments)
  case $rc in 0|1) ;; *) echo "$t rc=$rc"; tail -5 gpurun_out/bab.log; exit $rc ;; esac
  T="$t" python3 - <<'PY'
import json, os
for line in open("gpurun_out/bab.log"):
    if line.startswith('{"metric"'):
        d = json.loads(line)
        print(os.environ["T"] or "(default)", "| step", round(d["ms_per_step"], 4), "median",
              d["step_ms"]["median"], "| k_rows", round(d["roofline"]["avg_launch_ms"], 4), "fill", d["roofline"].get("box_fill_gbs"),
              "| front", round(d["step_ms"]["median"] - d["roofline"]["avg_launch_ms"], 4),
              "| max", d["step_ms"]["max"], "engine", d["step_ms"].get("engine_call_max"), "at", d["step_ms"]["worst5_at"][-1], "| verified", d.get("verified"))
PY
done
