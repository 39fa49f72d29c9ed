#!/bin/bash
# Round-5 bench lines of the other configurations: C4, D1, C5, and the
# emulated rank 0 of 8 of C3 and C5.  Each GPU step has its own time limit;
# a failure ends the script.
set -u
mkdir -p gpurun_out/r05
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name seconds args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python3 bench.py "$@" > gpurun_out/r05/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  grep "^{" gpurun_out/r05/$name.log | tail -1 > gpurun_out/r05/$name.json
}
run c4 300 --config C4 --steps 300 --warmup 20 --cpu-baseline 0
run d1 300 --config D1 --steps 100 --warmup 10 --cpu-baseline 0
run c3r8 300 --config C3 --rank-of 8 --steps 300 --warmup 20 --cpu-baseline 0
run c5r8 400 --config C5 --rank-of 8 --steps 20 --warmup 3 --cpu-baseline 0
run c5 600 --config C5 --steps 5 --warmup 2 --cpu-baseline 0
python3 - <<'PY'
import json
for n in ("c4", "d1", "c3r8", "c5r8", "c5"):
    d = json.load(open("gpurun_out/r05/%s.json" % n))
    r = d["roofline"]
    print("%-5s mean %.4f median %.4f k_rows %.4f frac %.3f alone %s verified %s" % (
        n, d["ms_per_step"], d["step_ms"]["median"], r["avg_launch_ms"], r["frac"],
        (r.get("alone") or {}).get("frac"), d.get("verified")))
PY
