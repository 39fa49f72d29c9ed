for t in ${TUNES:-"shardearly=1" "shardearly=0"}; do
KANO_TUNE=$t timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --shard-path --steps 100 --warmup 5 --cpu-baseline 0 > gpurun_out/rccl1.log 2>&1 || exit 1
tail -1 gpurun_out/rccl1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', round(d['ms_per_step'],4), d['step_ms']['median'], round(d['roofline']['avg_launch_ms'],4), d['result_sizes'])"
done
