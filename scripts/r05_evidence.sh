#!/bin/bash
# Round-5 evidence for the headline line: the driver's bench command, the same
# command under rocprofv3 --kernel-trace --stats, and the FETCH / WRITE PMC
# passes.  Each GPU step has its own time limit; a failure ends the script.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.log 2>&1 || exit $?
grep "^{" gpurun_out/b20.log | tail -1 > gpurun_out/b20.json
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --cold 0 > gpurun_out/prof.log 2>&1 || exit $?
grep "^{" gpurun_out/prof.log | tail -1 > gpurun_out/prof_line.json
bash scripts/pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/b20.json"))
r = d["roofline"]
print("bench: mean %.4f median %.4f k_rows %.4f frac %.3f alone %s verified %s" % (
    d["ms_per_step"], d["step_ms"]["median"], r["avg_launch_ms"], r["frac"],
    (r.get("alone") or {}).get("frac"), d.get("verified")))
PY
