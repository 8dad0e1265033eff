#!/bin/bash
# N > 1 bench path rehearsed with 2 ranks on the box's one GPU over gloo (RCCL needs one GPU per rank): bench.py
# launching its own ranks (the driver's `bench.py --gpus N` form) with the gather overlapped, then under an outside
# torch.distributed.run launcher with the gather after each step.
set -o pipefail
TAG=${1:-rehearse}; S=${2:-2000}
O=gpurun_out/$TAG; mkdir -p $O
DVH_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 --scenarios $S \
  --no-cpu --no-cold-ref --overlap-gather 1 > $O/self1.log 2>&1 || { echo "self-launched failed"; tail -20 $O/self1.log; exit 1; }
python -c "import json; l=[x for x in open('$O/self1.log') if x.startswith('{')][-1]; j=json.loads(l); print('self-launched overlap 1', j['n_gpus'], j['value'], j['ms_per_step'], j['gather'])"
DVH_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 2 --steps 3 --warmup 1 --scenarios $S \
  --no-cpu --no-cold-ref --overlap-gather 0 > $O/torchrun0.log 2>&1 || { echo "torchrun failed"; tail -20 $O/torchrun0.log; exit 1; }
python -c "import json; l=[x for x in open('$O/torchrun0.log') if x.startswith('{')][-1]; j=json.loads(l); print('torchrun overlap 0', j['n_gpus'], j['value'], j['ms_per_step'], j['gather'])"
