#!/bin/bash
# The N > 1 bench path rehearsed on ONE GPU: N ranks share cuda:0 and
# exchange over gloo (RCCL refuses two ranks on one device).  Checks that
# every rank's step runs and rank 0 prints its line; timings are meaningless.
set -u
mkdir -p gpurun_out
for N in ${NS:-2 4}; do
  KANO_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) \
    bench.py --gpus $N --steps ${STEPS:-5} --warmup 2 --config ${CFG:-C3} > gpurun_out/dist_$N.log 2>&1
  rc=$?; echo "N=$N rc=$rc"
  tail -1 gpurun_out/dist_$N.log | cut -c1-300
  case "$rc" in 0) ;; *) tail -20 gpurun_out/dist_$N.log; exit $rc ;; esac
done
