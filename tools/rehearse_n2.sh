set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r01n_rehearse; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo > $O/c2_n2_gloo.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload train --steps 50 --warmup 5 > $O/train_c3.log 2>&1
