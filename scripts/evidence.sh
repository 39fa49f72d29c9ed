#!/bin/bash
# The GPU evidence behind DESIGN.md's numbers, in one script (run on the GPU
# box through gpurun; every GPU step bounded by its own timeout, the script
# stops at the first failure).  Steps, chosen with STEPS (default "tests b20"):
#
#   tests    pytest -m gpu (PYK=<-k expr> narrows it)         gpurun_out/gpu_tests.txt
#   b20      the driver's bench command (C3, 20 steps)         gpurun_out/b20.json
#   lines    bench lines LINES="c3 c3long c4 c4m c5 g2 dense"  gpurun_out/lines/*.json
#            (g2: --gpus 2 in one process, KANO_DEVICES=0,0; dense: the MFMA sweep's
#            cluster, --config D1)
#   ab       A/B of KANO_TUNE settings AB="none knob=v ..." on C3 (ABSTEPS, ABARGS)
#   rank     the emulated rank 0 of N, RANKS="2 4 8" (bench.py --rank-of N)
#   kstats   rocprofv3 --kernel-trace --stats of the driver's command, plus its
#            step timeline (scripts/steps_tl.py)              gpurun_out/kstats_*.{csv,txt}
#   pmc      FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh)  gpurun_out/pmc_summary.json
#   trace    kernel (+ HIPTR=1: HIP API) traces, SPECS="label|KANO_TUNE|bench args;..."
#   sweep    the dense-path crossover sweep (scripts/mfma_sweep.py) gpurun_out/sweep.jsonl
#   ilaunch  the indirect-launch micro (scripts/micro/indirect_launch.sh)
set -u
mkdir -p gpurun_out gpurun_out/lines
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

summ() {  # $1 file, $2 label: one summary line of a bench JSON
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
out = {"ms": round(d["ms_per_step"], 4), "med": d["step_ms"]["median"], "max": d["step_ms"]["max"],
       "k_rows": round(r["avg_launch_ms"], 4), "frac": round(r["frac"], 3), "cus": r.get("cus"),
       "ok": d["verified"]}
if r.get("alone"):
    out["alone"] = (round(r["alone"]["avg_launch_ms"], 4), round(r["alone"]["frac"], 3))
if d.get("host_us"):
    out["host"] = {k: d["host_us"][k] for k in ("front_mean", "waits_mean", "tailwait_mean",
                                                "issue_mean", "between_mean") if k in d["host_us"]}
if d.get("mfma_roofline"):
    m = d["mfma_roofline"]
    out["mfma"] = {k: round(m[k], 3) for k in ("achieved", "frac", "avg_ms")}
    if m.get("alone"):
        out["mfma"]["alone"] = (round(m["alone"]["avg_ms"], 3), round(m["alone"]["frac"], 3))
if "cpu_baseline" in d:
    c = d["cpu_baseline"]
    out["cpu"] = (c["value"], c["cores"], c["verified"])
if "cold_drop_in" in d:
    out["cold"] = (d["cold_drop_in"]["total_s"], d["cold_drop_in"]["verified"])
print(sys.argv[2], out)
PY
}

bench() {  # name, timeout, args...
  local nm=$1 to=$2; shift 2
  timeout -k 10 "$to" python3 bench.py "$@" > gpurun_out/lines/$nm.json 2> gpurun_out/lines/$nm.err \
    || { echo "$nm failed"; tail -5 gpurun_out/lines/$nm.err; exit 1; }
  summ gpurun_out/lines/$nm.json "$nm"
}

for step in ${STEPS:-tests b20}; do
  case $step in
    tests)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        ${PYK:+-k "$PYK"} > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
      tail -2 gpurun_out/gpu_tests.txt ;;
    b20) bench b20 300 --gpus 1 --steps 20 --warmup 5 ;;
    lines)
      for L in ${LINES:-c3 c4}; do
        case $L in
          c3) bench c3 300 --gpus 1 --steps 20 --warmup 5 ;;
          c3long) bench c3long 300 --steps 1000 --warmup 50 --cpu-baseline 0 --cold 0 ;;
          c4) bench c4 300 --config C4 --steps 200 --warmup 10 --cpu-baseline 0 --cold 0 ;;
          c4m) bench c4m 300 --config C4 --path mfma --steps 200 --warmup 10 --cpu-baseline 0 --cold 0 ;;
          c5) bench c5 400 --config C5 --steps 10 --warmup 2 --cpu-baseline 0 ;;
          g2) KANO_DEVICES=0,0 bench g2 300 --gpus 2 --steps 300 --warmup 20 ;;
          dense) bench dense 300 --config D1 --steps 50 --warmup 5 --cpu-baseline 0 --cold 0 ;;
        esac
      done ;;
    ab)
      for t in ${AB:-none}; do
        [ "$t" = none ] && tt="" || tt="$t"
        KANO_TUNE="$tt" bench "ab_${t//[=,]/_}" 300 --steps ${ABSTEPS:-300} --warmup 20 --cpu-baseline 0 --cold 0 ${ABARGS:-}
      done ;;
    rank)
      for N in ${RANKS:-2 4 8}; do
        bench rank_of_$N 200 --steps 300 --warmup 20 --rank-of $N --cpu-baseline 0 --cold 0
      done ;;
    kstats)
      rm -rf gpurun_out/kstats
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats -o run --output-format csv -- \
        python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 --cold 0 --alone 0 ${KARGS:-} \
        > gpurun_out/kstats.json 2> gpurun_out/kstats.err || { tail gpurun_out/kstats.err; exit 1; }
      cp "$(find gpurun_out/kstats -name "*kernel_stats.csv" | head -1)" gpurun_out/kstats_stats.csv
      python3 scripts/steps_tl.py "$(find gpurun_out/kstats -name "*kernel_trace.csv" | head -1)" \
        > gpurun_out/kstats_tl.txt
      rm -rf gpurun_out/kstats
      summ gpurun_out/kstats.json kstats_line
      head -8 gpurun_out/kstats_stats.csv | cut -c1-150 ;;
    pmc)
      BENCH_ARGS="--alone 0 --cold 0 ${KARGS:-}" bash scripts/pmc.sh > gpurun_out/pmc.out 2>&1 \
        || { tail -5 gpurun_out/pmc.out; exit 1; }
      tail -c 600 gpurun_out/pmc.out; echo ;;
    trace)
      IFS=';' read -ra specs <<< "${SPECS:-base||}"
      for s in "${specs[@]}"; do
        IFS='|' read -r label tune args <<< "$s"
        rm -rf gpurun_out/tr_$label
        KANO_TUNE="$tune" timeout -k 10 200 rocprofv3 --kernel-trace ${HIPTR:+--hip-trace} --stats \
          -d gpurun_out/tr_$label -o run --output-format csv -- \
          python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --cold 0 --alone 0 $args > gpurun_out/tr_$label.log 2>&1 \
          || { echo "$label failed"; tail -5 gpurun_out/tr_$label.log; exit 1; }
        python3 scripts/steps_tl.py "$(find gpurun_out/tr_$label -name "*kernel_trace.csv" | head -1)" \
          > gpurun_out/tl_$label.txt && tail -50 gpurun_out/tl_$label.txt
        cp "$(find gpurun_out/tr_$label -name "*kernel_stats.csv" | head -1)" gpurun_out/ks_$label.csv
        rm -rf gpurun_out/tr_$label
      done ;;
    sweep)
      timeout -k 10 900 python3 -u scripts/mfma_sweep.py ${SWEEPARGS:-} > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err \
        || { tail -20 gpurun_out/sweep.err; exit 1; }
      cat gpurun_out/sweep.jsonl ;;
    ilaunch)
      bash scripts/micro/indirect_launch.sh > gpurun_out/ilaunch.txt 2>&1 || { cat gpurun_out/ilaunch.txt; exit 1; }
      cat gpurun_out/ilaunch.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
