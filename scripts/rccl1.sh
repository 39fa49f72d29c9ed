#!/bin/bash
# One-rank RCCL run of bench.py's shard path (torch.distributed.run, nccl):
# the exchange as torch's collective vs the engine's own (kano_verify_gather).
set -u
for x in ${XCHG:-1 0 1 0}; do
  KANO_NATIVE_EXCHANGE=$x timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --shard-path --steps ${STEPS:-300} --warmup 20 \
    --cpu-baseline 0 > gpurun_out/rccl1.log 2>&1 || exit 1
  tail -1 gpurun_out/rccl1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('native=$x', d['config']['exchange'], round(d['ms_per_step'],4), 'median', d['step_ms']['median'], 'k_rows', round(d['roofline']['avg_launch_ms'],4), 'verified', d['verified'])"
done
