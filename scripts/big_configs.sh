set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C4 --no-shadow --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4.log 2>&1; rc=$?; echo "c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C4 --path bitwise --no-shadow --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/c4b.log 2>&1; rc=$?; echo "c4b rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config C5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; exit $rc
