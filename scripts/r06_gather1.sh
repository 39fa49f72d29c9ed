#!/bin/bash
# C3 at one GPU: the fused kano_verify against the same step through
# kano_verify_gather (one rank, the exchange a device copy), alternating;
# then the gathered step's kernel timeline
set -u
mkdir -p gpurun_out
: > gpurun_out/g1.jsonl
for rep in 1 2 3; do
  for mode in plain gather1; do
    a=""; [ $mode = gather1 ] && a="--gather1"
    timeout -k 10 200 python bench.py --steps 600 --warmup 30 --cpu-baseline 0 --cold 0 --alone 0 $a > gpurun_out/g1.log 2>&1 || exit 1
    tail -1 gpurun_out/g1.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
h=d.get('host_us') or {}
print(json.dumps({'mode':'$mode','mean':round(d['ms_per_step'],4),'median':d['step_ms']['median'],'rows_ms':round(d['roofline']['avg_launch_ms'],4),'idle':d.get('boundary_idle_us'),'issue':h.get('issue_mean'),'waits':h.get('waits_mean'),'tailwait':h.get('tailwait_mean'),'verified':d['verified']}))" >> gpurun_out/g1.jsonl
  done
done
cat gpurun_out/g1.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/g1tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/g1tl -o run --output-format csv -- \
  python3 bench.py --steps 12 --warmup 4 --cpu-baseline 0 --cold 0 --alone 0 --gather1 > gpurun_out/g1tl.log 2>&1 || exit 3
python3 scripts/steps_tl.py gpurun_out/g1tl/run_kernel_trace.csv 10 > gpurun_out/tl_gather1.txt
rm -rf gpurun_out/g1tl
