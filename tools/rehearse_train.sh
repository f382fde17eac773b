# C3/C4 training bench on the one GPU of a box: the one-GPU step with and without the row exchange
# (W = 1 measures the exchange's kernels), then 2 and 4 DP ranks over gloo (exchange through host
# memory: checks the path end to end, times say nothing about xGMI).
# usage: gpurun -- 'bash tools/rehearse_train.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rehearse_train}; mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 python -u bench.py --workload train > $O/c3_w1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --exchange > $O/c3_w1_exchange.log 2>&1 && \
timeout -k 10 300 $R --nproc-per-node 2 --master-port 29521 bench.py --workload train --gpus 2 --steps 20 --warmup 4 --dist-backend gloo > $O/c4_n2_gloo.log 2>&1 && \
timeout -k 10 400 $R --nproc-per-node 4 --master-port 29522 bench.py --workload train --gpus 4 --steps 20 --warmup 4 --dist-backend gloo > $O/c4_n4_gloo.log 2>&1
