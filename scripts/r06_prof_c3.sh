#!/bin/bash
# the driver's bench command under rocprofv3 --kernel-trace --stats, with
# --alone 0 --cold 0 (the trace's k_rows launches are then exactly the line's
# 25 in-step launches: 5 warm-up + 20 timed), and its step timeline
set -u
O=gpurun_out/r06p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --alone 0 --cold 0 ${EXTRA:-} > $O/c3_profiled.json 2> $O/c3_profiled.err
rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $O/c3_profiled.err; exit $rc; }
python3 scripts/steps_tl.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/c3_step_timeline.txt
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/c3_kernel_stats.csv
rm -rf $O/prof
head -4 $O/c3_kernel_stats.csv
python3 -c "
import json
d=json.loads(open('$O/c3_profiled.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches_timed'], d['verified'])"
