# C4 DP path at W = 8 on the one GPU of a box (8 gloo ranks; exchange through host memory: a path
# check, not a timing). usage: gpurun -- 'bash tools/rehearse_train8.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rehearse_train8}; mkdir -p $O
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29531 \
  --nproc-per-node 8 bench.py --workload train --gpus 8 --steps 16 --warmup 4 --dist-backend gloo > $O/c4_n8_gloo.log 2>&1
