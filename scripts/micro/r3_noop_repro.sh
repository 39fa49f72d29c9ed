#!/bin/bash
# Round 3's host-sanitizer failure ("matrix not built": a scan launched through
# the function-pointer triple-chevron never ran) reproduced from the source as
# it was before the fix (commit eb53095; binaries tests/asan/kano_asan_r3_*,
# built in the build container from `git archive eb53095`), one sanitizer at a
# time: which one makes the launch a no-op?
set -u
cd "$(dirname "$0")/../.."
export ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=1:quarantine_size_mb=0"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
for v in plain ubsan asan nofunc san; do
  b=tests/asan/kano_asan_r3_$v
  [ -x "$b" ] || { echo "$v: missing"; continue; }
  timeout -k 5 120 "$b" > gpurun_out/r3noop_$v.txt 2>&1
  rc=$?
  echo "== $v rc=$rc: $(grep -c 'CHECK failed\|FAIL' gpurun_out/r3noop_$v.txt) failure lines; $(grep -m1 -o 'host signal not raised[^)]*)' gpurun_out/r3noop_$v.txt) | $(tail -n 1 gpurun_out/r3noop_$v.txt | cut -c1-160)"
done
