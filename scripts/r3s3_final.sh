#!/bin/bash
# Round-3 final evidence: the driver's default bench and its 20-step command
# (C3), a C4 line, then the kernel stats + PMC passes of the driver's command.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/final_c3_default.json 2> gpurun_out/final_c3_default.err || { tail gpurun_out/final_c3_default.err; exit 1; }
tail -c 300 gpurun_out/final_c3_default.json; echo
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/final_c3_s20.json 2> gpurun_out/final_c3_s20.err || { tail gpurun_out/final_c3_s20.err; exit 1; }
timeout -k 10 300 python3 bench.py --config C4 --cpu-baseline 0 --cold 0 > gpurun_out/final_c4.json 2> gpurun_out/final_c4.err || { tail gpurun_out/final_c4.err; exit 1; }
bash scripts/r3s2_kstats.sh
