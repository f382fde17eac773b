#!/bin/bash
# End-of-round check without the profile passes: -m gpu suite, smoke, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r03_final_tests}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
