#!/bin/bash
# Fused split-row combine: its bitwise tests, the parity suites that run through lgcn_spmm, then
# the C2 bench and the reduce-mode rank probe with and without it (LGCN_FUSED_COMBINE A/B).
# usage: gpurun -- 'bash tools/r03_fused.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03_fused}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_combine.py -x -v --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_sliced.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_fused.log 2>&1 && \
LGCN_FUSED_COMBINE=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_twolaunch.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_fused2.log 2>&1 && \
timeout -k 10 300 python -u tools/reduce_rank_probe.py > $O/rank_fused.log 2>&1 && \
LGCN_FUSED_COMBINE=0 timeout -k 10 300 python -u tools/reduce_rank_probe.py > $O/rank_twolaunch.log 2>&1
