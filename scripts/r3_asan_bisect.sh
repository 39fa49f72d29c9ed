export ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=1:quarantine_size_mb=0"
mkdir -p gpurun_out
run() { # label tune binary
  KANO_TUNE="$2" timeout -k 10 200 tests/asan/$3 > gpurun_out/bis_$1.txt 2>&1; r=$?
  echo "$1 ($2, $3) rc=$r $(grep -m1 FAIL gpurun_out/bis_$1.txt) | $(tail -n 1 gpurun_out/bis_$1.txt)"
  [ $r -le 1 ] || exit $r
}
run head "" kano_asan; run head_sp0 "sidepre=0,sidetail=0" kano_asan
