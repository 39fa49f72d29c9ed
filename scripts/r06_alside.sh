#!/bin/bash
# the flat allowed-pod lists on stream2 (wide rows): parity, then C5 rank 0
# of 8 and C5 with and without (alternating)
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_configs.py -k "rows_variants or c5_full" > gpurun_out/r06_as_t.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/r06_as_t.log
case $rc in 0) ;; *) exit $rc ;; esac
: > gpurun_out/r06_alside_ab.jsonl
for rep in 1 2; do
  for a in 1 0; do
    for cfg in "--config C5 --rank-of 8" ; do
      KANO_TUNE=alside=$a timeout -k 10 200 python bench.py --steps 30 --warmup 3 --cpu-baseline 0 --cold 0 --alone 0 $cfg > gpurun_out/ab.json 2>gpurun_out/ab.err
      rc=$?; echo "a=$a cfg=$cfg rc=$rc"; case $rc in 0) ;; *) tail -5 gpurun_out/ab.err; exit $rc ;; esac
      python3 -c "
import json
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print(json.dumps({'alside':$a,'cfg':'$cfg','mean':d['ms_per_step'],'median':d['step_ms']['median'],'verified':d['verified'],'write':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac']}))" >> gpurun_out/r06_alside_ab.jsonl
    done
  done
done
cat gpurun_out/r06_alside_ab.jsonl
