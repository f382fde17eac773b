#!/bin/bash
# The whole -m gpu suite, smoke(), then the bench lines; stops after a crash.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
bash tools/r03_tests.sh $T tests
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.add_path(); g.smoke()" > $O/smoke.log 2>&1 && \
bash tools/r03_benches.sh $T
