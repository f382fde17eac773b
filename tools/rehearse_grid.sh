# Rehearse the multi-GPU C2 bench on the one GPU of a box: N ranks over gloo (the exchanges go
# through host memory, so times say nothing about xGMI; this checks the path end to end,
# including the timed grid choice among lgcn_amd.sharded.grid_candidates and the p2p exchange).
# usage: gpurun -- 'bash tools/rehearse_grid.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rehearse_grid}; mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $O/c2_n2_default.log 2>&1 && \
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29513 bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo > $O/c2_n4_default.log 2>&1 && \
timeout -k 10 300 $R --nproc-per-node 4 --master-port 29514 bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo --shard 4x1 --exchange-mode p2p > $O/c2_n4_4x1_p2p.log 2>&1 && \
timeout -k 10 400 $R --nproc-per-node 8 --master-port 29515 bench.py --gpus 8 --steps 5 --warmup 2 --dist-backend gloo > $O/c2_n8_default.log 2>&1
