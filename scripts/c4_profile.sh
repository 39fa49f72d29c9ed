#!/bin/bash
# C4 (broad selectors, the int8 MFMA contraction path) evidence: the bench
# line, a kernel-trace --stats profile, and one PMC pass of MFMA counters.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --config C4 --no-shadow --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/c4_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- \
  python3 bench.py --config C4 --no-shadow --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/prof_c4.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/pmc_c4
rm -rf gpurun_out/prof_c4m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4m -o run --output-format csv -- \
  python3 bench.py --config C4 --no-shadow --path mfma --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/prof_c4m.log 2>&1
rc=$?; echo "prof mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace -d gpurun_out/pmc_c4 -o run --output-format csv -- \
  python3 bench.py --config C4 --no-shadow --path mfma --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/pmc_c4.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_c4/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "mfma" in k or "heavy" in k or "k_rows" in k:
        print(k, {c: sum(v) / len(v) for c, v in d.items()})
PY
