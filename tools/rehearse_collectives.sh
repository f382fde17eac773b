# Rehearse bench.py's multi-GPU collectives probe and chosen-grid projection
# on the one GPU of a box: 4 ranks over gloo (C2), 2 and 4 ranks over gloo (C4 train). Host-memory
# collectives: the numbers say nothing about xGMI; this checks the fields end to end.
# usage: gpurun -- 'bash tools/rehearse_collectives.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rehearse_coll}; mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29523 bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo > $O/c2_n4.log 2>&1 && \
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29524 bench.py --workload train --gpus 2 --steps 20 --warmup 2 --dist-backend gloo > $O/c4_n2.log 2>&1 && \
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29525 bench.py --workload train --gpus 4 --steps 20 --warmup 2 --dist-backend gloo > $O/c4_n4.log 2>&1 && \
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29526 bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo --shard 2x2 --exchange-mode reduce > $O/c2_n4_2x2_reduce.log 2>&1
