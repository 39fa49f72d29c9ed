#!/bin/bash
# Bench lines: C3 (driver's command, with cpu_baseline and the cold drop-in
# call), C4 auto / --path mfma, C5; each JSON under gpurun_out/lines/.
set -u
mkdir -p gpurun_out/lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {   # name, timeout, args...
  local nm=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > gpurun_out/lines/$nm.json 2> gpurun_out/lines/$nm.err || { echo "$nm failed"; tail -5 gpurun_out/lines/$nm.err; exit 1; }
  python3 - "$nm" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/lines/{sys.argv[1]}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], "ms", round(d["ms_per_step"], 4), "med", d["step_ms"]["median"], "max", d["step_ms"]["max"],
      "k_rows", round(r["avg_launch_ms"], 4), "frac", round(r["frac"], 3), "verified", d["verified"],
      "mfma", None if not d.get("mfma_roofline") else {k: d["mfma_roofline"][k] for k in ("achieved", "frac", "avg_ms", "ops_per_build")},
      "cpu", None if "cpu_baseline" not in d else (d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"], d["cpu_baseline"]["seconds"], d["cpu_baseline"]["verified"]),
      "cold", d.get("cold_drop_in", {}).get("total_s"), d.get("cold_drop_in", {}).get("verified"))
PY
}
for L in ${LINES:-c3 c4 c4m c5}; do
  case $L in
    c3) run c3 300 --gpus 1 --steps 20 --warmup 5 ;;
    c3long) run c3long 300 --steps 1000 --warmup 50 --cpu-baseline 0 --cold 0 ;;
    c4) run c4 300 --config C4 --steps 200 --warmup 10 --cpu-baseline 0 ;;
    c4m) run c4m 300 --config C4 --path mfma --steps 200 --warmup 10 --cpu-baseline 0 ;;
    c5) run c5 400 --config C5 --steps 10 --warmup 2 --cpu-baseline 0 ;;
  esac
done
