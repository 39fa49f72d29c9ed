#!/bin/bash
# Kernel A/B: rocprofv3 kernel-trace of the bench under each KANO_TUNE
# setting, printing the average duration of the kernels matching PATTERN.
#   kab.sh PATTERN "t1" "t2" ...        (CFG, EXTRA from the env)
set -u
pat=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in "$@"; do
  rm -rf gpurun_out/kab
  KANO_TUNE="$t" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kab -o run \
    --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 \
    --config ${CFG:-C3} ${EXTRA:-} > gpurun_out/kab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$t rc=$rc"; tail -5 gpurun_out/kab.log; exit $rc; }
  PAT="$pat" T="$t" python3 - <<'EOF'
import csv, glob, os, re, json
f = glob.glob("gpurun_out/kab/**/*kernel_stats.csv", recursive=True)[0]
pat = re.compile(os.environ["PAT"])
tot = 0.0
out = []
for r in csv.DictReader(open(f)):
    if pat.search(r["Name"]):
        out.append(f"{r['Name'].split('(')[0][-40:]} {float(r['AverageNs'])/1000:.1f}us")
    tot += float(r["TotalDurationNs"])
ms = None
for line in open("gpurun_out/kab.log").read().splitlines():
    if line.startswith('{"metric"'):
        ms = json.loads(line)["step_ms"]["median"]
print(os.environ["T"], "|", "; ".join(out), "| busy/step", round(tot / 12 / 1000, 1), "us | step", ms)
EOF
done
