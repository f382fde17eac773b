#!/bin/bash
# C2 reduce-mode rank compute: hub chunk sweep (LGCN_RANK_CHUNK) and a kernel trace of one
# 8 x 1 / 4 x 2 rank; then the training bench's DP modes rehearsed with 2 gloo ranks on one GPU.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
for c in 64 128 256; do
  LGCN_RANK_CHUNK=$c timeout -k 10 300 python -u tools/reduce_rank_probe.py --grids 8x1,4x2,2x4 > $O/reduce_chunk$c.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/trace -o run --output-format csv -- python3 tools/reduce_rank_probe.py --grids 8x1,4x2 --steps 20 > $O/trace.log 2>&1 || exit $?
for m in replicated owner columns; do
  timeout -k 10 300 python -u bench.py --workload train --gpus 2 --dist-backend gloo --dp-mode $m --steps 40 --warmup 4 > $O/train_gpus2_$m.log 2>&1 || exit $?
done
