#!/bin/bash
# Round 6 evidence on the final tree, one GPU call:
#  1. the driver's bench command under rocprofv3 --kernel-trace --stats with
#     --alone 0 (the k_rows average = the timed steps' launches only) and the
#     step timeline from the same trace;
#  2. FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) of C3 and of C5's
#     rank 0 of 8, summarised per kernel (scripts/pmc_summary.py);
#  3. the config lines (verified), C5 rank 0 of 8 and D1 timelines.
set -u
O=gpurun_out/r06
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 at $2"; exit "$1" ;; esac; }
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --alone 0 --cold 0 > $O/c3_profiled.json 2> $O/c3_profiled.err
fatal $? prof
python3 scripts/steps_tl.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/c3_step_timeline.txt
for tag in C3 C5r8; do
  args="--config C3"; [ $tag = C5r8 ] && args="--config C5 --rank-of 8"
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$O/pmc_${tag}_$(echo $c | cut -d_ -f1 | tr A-Z a-z); rm -rf $d
    timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $d -o run --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 --cold 0 --alone 0 $args > $d.log 2>&1
    fatal $? "pmc $tag $c"
  done
  python3 scripts/pmc_summary.py $O/pmc_${tag}_fetch $O/pmc_${tag}_write > $O/pmc_$tag.json
done
for cfg in "C4" "D1" "C5" "C3 --rank-of 2" "C3 --rank-of 4" "C3 --rank-of 8" "C5 --rank-of 8"; do
  tag=$(echo "$cfg" | tr -d ' -' | sed 's/rankof/r/')
  steps=300; case "$cfg" in C5*|D1*) steps=30 ;; esac
  timeout -k 10 300 python3 bench.py --config $cfg --steps $steps --warmup 5 --cpu-baseline 0 --cold 0 > $O/$tag.json 2> $O/$tag.err
  fatal $? "line $cfg"
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
m=d.get('mfma_roofline') or {}
print('$tag', round(d['ms_per_step'],4), d['step_ms']['median'], d['verified'], round(d['roofline']['frac'],3), round((d['roofline'].get('alone') or {}).get('frac',0),3), round(m.get('frac',0),3))"
done
for cfg in "D1" "C5 --rank-of 8"; do
  tag=$(echo "$cfg" | tr -d ' -' | sed 's/rankof/r/')
  rm -rf $O/tl_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_$tag -o run --output-format csv -- \
    python3 bench.py --config $cfg --steps 6 --warmup 2 --cpu-baseline 0 --cold 0 --alone 0 > $O/tl_$tag.log 2>&1
  fatal $? "tl $cfg"
  python3 scripts/steps_tl.py $(find $O/tl_$tag -name "*kernel_trace.csv" | head -1) > $O/${tag}_step_timeline.txt
  rm -rf $O/tl_$tag
done
rm -rf $O/pmc_*_fetch $O/pmc_*_write
ls $O
