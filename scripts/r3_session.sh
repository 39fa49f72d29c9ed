#!/bin/bash
# Round-3 GPU iteration: (optionally) the GPU test suite, the driver's bench
# command, then A/B knob settings of the C3 step at N=1 and of the emulated
# rank 0 of N.  Every GPU step is bounded; the script stops at the first
# failure.
#   TESTS=0|1  PYK=<-k expr>  AB="knobs ..."  RANKS="2 4 8"  RAB="knobs ..."
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYK:+-k "$PYK"} > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
  tail -2 gpurun_out/gpu_tests.txt
fi
summ() {  # $1 file, $2 label
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "ms", round(d["ms_per_step"], 4), "med", d["step_ms"]["median"], "max", d["step_ms"]["max"],
      "k_rows", round(r["avg_launch_ms"], 4), "frac", round(r["frac"], 3), "cus", r.get("cus"), "alone", (round(r["alone"]["avg_launch_ms"], 4), round(r["alone"]["frac"], 3)) if r.get("alone") else None,
      "host", {k: d["host_us"][k] for k in ("front_mean", "back_mean", "waits_mean", "tailwait_mean", "issue_mean", "between_mean")} if d.get("host_us") else None, "ok", d["verified"])
PY
}
if [ "${B20:-1}" = 1 ]; then
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.json 2> gpurun_out/b20.err || { tail gpurun_out/b20.err; exit 1; }
  summ gpurun_out/b20.json b20
fi
for t in ${AB:-}; do
  [ "$t" = none ] && tt="" || tt="$t"
  KANO_TUNE="$tt" timeout -k 10 200 python3 bench.py --steps ${ABSTEPS:-300} --warmup 20 --cpu-baseline 0 ${ABARGS:-} > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  summ gpurun_out/ab.json "AB $t"
done
for N in ${RANKS:-}; do
  for t in ${RAB:-none}; do
    [ "$t" = none ] && tt="" || tt="$t"
    KANO_TUNE="$tt" timeout -k 10 200 python3 bench.py --steps 300 --warmup 20 --rank-of $N --cpu-baseline 0 \
        > gpurun_out/r8.json 2> gpurun_out/r8.err || { tail gpurun_out/r8.err; exit 1; }
    summ gpurun_out/r8.json "rank_of $N $t"
  done
done

if [ -n "${MICRO:-}" ]; then
  for m in $MICRO; do
    timeout -k 10 120 ./scripts/micro/$m > gpurun_out/micro_$m.txt 2>&1 || { tail gpurun_out/micro_$m.txt; exit 1; }
    echo "micro $m done"
  done
fi
echo done
