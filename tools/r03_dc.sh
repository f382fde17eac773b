#!/bin/bash
# The RCCL branches of the multi-GPU paths driven over gloo (LGCN_DEVICE_COLLECTIVES=1) on the one
# GPU: their tests, then the self-launched C2 bench at N = 4 with every grid candidate.
# usage: gpurun -- 'bash tools/r03_dc.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03_dc}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_exchange.py -k "device_collectives" -x -v --timeout 400 --timeout-method thread > $O/pytest_dc.log 2>&1 && \
LGCN_DEVICE_COLLECTIVES=1 timeout -k 10 400 python -u bench.py --gpus 4 --dist-backend gloo --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_gpus4_dc.log 2>&1
