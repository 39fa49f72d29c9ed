#!/bin/bash
# KANO_TUNE A/B on one engine build, alternating: TUNES (';'-separated, "-" =
# none), CFG (bench.py arguments)
set -u
mkdir -p gpurun_out
: > gpurun_out/tune_ab.jsonl
IFS=';' read -ra TU <<< "${TUNES:--}"
for rep in $(seq 1 ${REPS:-2}); do
  for t in "${TU[@]}"; do
    tt=$t; [ "$tt" = "-" ] && tt=""
    KANO_TUNE="$tt" timeout -k 10 200 python bench.py --cpu-baseline 0 --cold 0 --alone 0 ${CFG:---steps 300 --warmup 20} > gpurun_out/ab.json 2>gpurun_out/ab.err
    rc=$?; case $rc in 0) ;; *) echo "$t rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc ;; esac
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print(json.dumps({'tune':'$t','mean':round(d['ms_per_step'],4),'median':d['step_ms']['median'],'verified':d['verified'],'rows_ms':round(d['roofline']['avg_launch_ms'],4),'cus':d['roofline']['cus'],'gemm_ms':round((d.get('mfma_roofline') or {}).get('avg_ms',0),4)}))" >> gpurun_out/tune_ab.jsonl
  done
done
cat gpurun_out/tune_ab.jsonl
