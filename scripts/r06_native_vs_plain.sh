#!/bin/bash
# C3 at one GPU: the fused kano_verify (the driver's N=1 command) against the
# shard path under torch.distributed.run with the native RCCL exchange
# (kano_verify_gather, world size 1), alternating on one box
set -u
mkdir -p gpurun_out
: > gpurun_out/nvp.jsonl
for rep in 1 2 3; do
  for mode in plain native; do
    if [ $mode = plain ]; then
      timeout -k 10 200 python bench.py --steps 600 --warmup 30 --cpu-baseline 0 --cold 0 --alone 0 > gpurun_out/nvp.log 2>&1 || exit 1
    else
      timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29511 bench.py --shard-path --steps 600 --warmup 30 --cpu-baseline 0 --cold 0 --alone 0 > gpurun_out/nvp.log 2>&1 || exit 2
    fi
    tail -1 gpurun_out/nvp.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
h=d.get('host_us') or {}
print(json.dumps({'mode':'$mode','mean':round(d['ms_per_step'],4),'median':d['step_ms']['median'],'rows_ms':round(d['roofline']['avg_launch_ms'],4),'cus':d['roofline'].get('cus'),'idle':d.get('boundary_idle_us'),'issue':h.get('issue_mean'),'waits':h.get('waits_mean'),'tailwait':h.get('tailwait_mean'),'verified':d['verified'],'pipelined':d['config'].get('pipelined')}))" >> gpurun_out/nvp.jsonl
  done
done
cat gpurun_out/nvp.jsonl
