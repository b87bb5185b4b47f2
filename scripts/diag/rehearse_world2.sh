#!/bin/bash
# Round 6: rehearse bench.py's multi-rank path (torchrun, weak-scaling batch per rank, each
# rank's phase-locked sub-batch split with its issue threads, max-over-ranks timing, rank-0
# JSON line) with 2 ranks on this one-GPU box over gloo (RCCL refuses two ranks on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
O=gpurun_out/${TAG:-r06aa}
mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --batch 224 --no-b1 --no-cpu-baseline --scan-reps 2 --dist-backend gloo > $O/world2.json 2> $O/world2.err || { tail -30 $O/world2.err; exit 1; }
tail -c 1500 $O/world2.json
