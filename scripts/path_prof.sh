#!/bin/bash
# rocprofv3 kernel-trace --stats of scripts/path_bench.py (C3 two-hop and closure).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "${@:-C3:2:bitwise,mfma C3:0:auto}"; do :; done
i=0
for spec in ${SPECS:-C3:2:bitwise,mfma C3:0:auto}; do
  IFS=: read cfg hops modes <<< "$spec"
  rm -rf gpurun_out/pprof$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pprof$i -o run --output-format csv \
    -- python3 scripts/path_bench.py --config $cfg --hops $hops --modes $modes --reps 1 \
    > gpurun_out/pprof$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$spec rc=$rc"; tail -5 gpurun_out/pprof$i.log; exit $rc; }
  echo "== $spec"; grep '^{"config' gpurun_out/pprof$i.log | cut -c1-300
  f=$(find gpurun_out/pprof$i -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "path" in r["Name"] or "transpose" in r["Name"] or "popcount" in r["Name"]:
        print(f"  {r['Name'].split('(')[0][:60]:<60} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:9.1f} us  total {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
  i=$((i+1))
done
