#!/bin/bash
# Round-3 fresh-box check: -m gpu suite, smoke, default bench, the self-launched 2-rank bench
# (gloo on one GPU: launcher + grid trials path check), then the C2 profile with the PMC passes.
# usage: gpurun -- 'bash tools/r03_check.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r03_check}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 > $O/bench_gpus2_gloo.log 2>&1 && \
PROF_TAG=$TAG/prof bash tools/profile_round.sh
