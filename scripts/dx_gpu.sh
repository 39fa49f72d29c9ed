# the whole GPU suite, then D1 / C4 / C3 lines
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for c in D1:100 C4:300 C3:300; do
  n=${c%%:*}; k=${c##*:}
  timeout -k 10 300 python3 bench.py --config $n --steps $k --warmup 10 --cpu-baseline 0 > gpurun_out/$n.log 2>&1 || exit $?
  grep "^{" gpurun_out/$n.log | tail -1 > gpurun_out/$n.json
done
python3 - <<'PY'
import json
for n in ("D1", "C4", "C3"):
    d = json.load(open("gpurun_out/%s.json" % n)); r = d["roofline"]; m = d.get("mfma_roofline") or {}
    print("%s mean %.4f median %.4f k_rows %.4f (%.3f) mfma %s verified %s" % (n, d["ms_per_step"], d["step_ms"]["median"], r["avg_launch_ms"], r["frac"], m.get("frac"), d.get("verified")))
PY
