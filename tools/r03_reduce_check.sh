#!/bin/bash
# Reduce mode with the last layer reduce-scattered: its GPU tests, the rank probe, and the bench's
# grid trials over 4 gloo ranks on one GPU (every candidate incl. reduce runs through bench.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
bash tools/r03_tests.sh $T tests/test_gpu_sharded.py
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/reduce_rank_probe.py --grids 8x1,4x2,2x4 > $O/reduce_rank_probe.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 4 --dist-backend gloo --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_gpus4_gloo.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --shard 2x1 --exchange-mode reduce --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_gpus2_reduce.log 2>&1
