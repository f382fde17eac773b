#!/bin/bash
# Round-final evidence on one fresh box: the -m gpu suite, smoke(), the default bench line, and the
# C2 profile (kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes + calibration) for
# profiles/pmc_traffic.json (tools/pmc_to_traffic.py). usage: gpurun -- 'bash tools/round_final.sh TAG'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-round_final}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
PROF_TAG=$TAG/prof bash tools/profile_round.sh
