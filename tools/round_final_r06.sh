#!/bin/bash
# Round-final evidence, part 1 (one fresh box): the -m gpu suite, smoke(), the driver's bench
# command and the default bench. Part 2 is tools/profile_round.sh (kernel trace + PMC passes).
# usage: gpurun -- 'bash tools/round_final_r06.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-round_final}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.log 2>&1
