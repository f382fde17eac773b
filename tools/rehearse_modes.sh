# Rehearse bench.py --gpus 4's post-trial path for EVERY exchange family the grid trials can pick
# (a node run with RCCL may pick any of them; a gloo rehearsal on one GPU picks a 1 x F grid, so
# the others are forced with --shard): 2 x 2 allgather / reduce / reduce-fused / reduce-a2a /
# reduce-a2a-fused and 4 x 1 p2p, each to its JSON line (collectives, projection, roofline).
# usage: gpurun -- 'bash tools/rehearse_modes.sh OUTTAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rehearse_modes}; mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4"
P=29540
for spec in 2x2:allgather 2x2:reduce 2x2:reduce-fused 2x2:reduce-a2a 2x2:reduce-a2a-fused 4x1:p2p; do
  g=${spec%%:*}; m=${spec##*:}; P=$((P + 1))
  timeout -k 10 240 $R --master-port $P bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo \
    --shard $g --exchange-mode $m --no-cpu-baseline > $O/c2_n4_${g}_${m}.log 2>&1 || exit 1
done
