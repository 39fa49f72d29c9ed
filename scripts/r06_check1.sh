#!/bin/bash
# round 6, first GPU call: the new C3 shard parity, the forced variants after
# the kernel/knob removal, the group tests, and the --rank-of lines verified
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_configs.py -k "row_shards or rows_variants or config_vs" > gpurun_out/r06_t1.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/r06_t1.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for N in 8; do
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --cpu-baseline 0 --cold 0 --rank-of $N > gpurun_out/r06_c3r$N.json 2>gpurun_out/r06_c3r$N.err
rc=$?; echo "c3r${N}_rc=$rc"; case $rc in 0|1) ;; *) exit $rc ;; esac
done
timeout -k 10 300 python bench.py --config C5 --steps 20 --warmup 3 --cpu-baseline 0 --cold 0 --rank-of 8 > gpurun_out/r06_c5r8.json 2>gpurun_out/r06_c5r8.err
rc=$?; echo "c5r8_rc=$rc"
python3 - <<'PY'
import json
for f in ["r06_c3", "r06_c3r8", "r06_c5r8"]:
    try:
        d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
        print(f, d["ms_per_step"], d["step_ms"]["median"], d["verified"], str(d["verified_against"])[:200], d["roofline"]["frac"], d["host_us"])
    except Exception as e:
        print(f, "ERR", e)
PY
