#!/bin/bash
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) of C3 and of C5's rank 0
# of 8, summarised per kernel (median launch: scripts/pmc_summary.py)
set -u
O=gpurun_out/r06m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for tag in C3 C5r8; do
  args="--config C3"; [ $tag = C5r8 ] && args="--config C5 --rank-of 8"
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$O/pmc_${tag}_$(echo $c | cut -d_ -f1 | tr A-Z a-z); rm -rf $d
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $d -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --cold 0 --alone 0 $args > $d.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc $tag $c rc=$rc"; tail -3 $d.log; exit $rc; }
  done
  python3 scripts/pmc_summary.py $O/pmc_${tag}_fetch $O/pmc_${tag}_write > $O/pmc_$tag.json
  rm -rf $O/pmc_${tag}_fetch $O/pmc_${tag}_write
done
python3 -c "
import json
for t in ['C3','C5r8']:
    d=json.load(open('$O/pmc_'+t+'.json'))['kernels']
    for k,v in d.items():
        if 'k_rows' in k: print(t, k, v['dispatches'], v['hbm_bytes_per_launch'], [round(x/1e9,3) for x in v['write_bytes_each']])
"
