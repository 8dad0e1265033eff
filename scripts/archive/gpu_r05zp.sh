#!/bin/bash
# N > 1 rehearsal on the one-GPU box with the final library: bench.py --gpus 2 starts its two ranks itself (gloo, since
# RCCL refuses two ranks on one GPU), 2,000 scenarios per rank, overlapped tagged all-gather; then under torch.distributed.run
set -o pipefail
O=gpurun_out/r05zp; mkdir -p $O
DVH_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --scenarios 2000 --steps 3 --warmup 1 --no-cpu --no-cold-ref > $O/self_launch.log 2>&1 || { echo "self-launch failed"; tail -30 $O/self_launch.log; exit 1; }
tail -1 $O/self_launch.log | cut -c1-400
DVH_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --scenarios 2000 --steps 3 --warmup 1 --no-cpu --no-cold-ref > $O/torchrun.log 2>&1 || { echo "torchrun failed"; tail -30 $O/torchrun.log; exit 1; }
grep '^{' $O/torchrun.log | tail -1 | cut -c1-400
