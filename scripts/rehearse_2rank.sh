#!/bin/bash
# N > 1 bench path rehearsed with 2 ranks on the box's one GPU over gloo (RCCL needs one GPU per rank): the gather
# after each step vs overlapped with the next step's solve.
set -o pipefail
TAG=${1:-rehearse}; S=${2:-2000}
O=gpurun_out/$TAG; mkdir -p $O
for ov in 0 1; do
  DVH_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29500 + ov)) bench.py --gpus 2 --steps 3 --warmup 1 --scenarios $S \
    --no-cpu --no-cold-ref --overlap-gather $ov > $O/overlap$ov.log 2>&1 || { echo "overlap $ov failed"; tail -20 $O/overlap$ov.log; exit 1; }
  python -c "import json; l=[x for x in open('$O/overlap$ov.log') if x.startswith('{')][-1]; j=json.loads(l); print('overlap', $ov, j['value'], j['ms_per_step'], j['gather'])"
done
