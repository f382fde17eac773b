#!/bin/bash
# Scatter tests (the grouping), then the planted training bench under the kernel tracer.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
bash tools/r03_tests.sh $T tests/test_gpu_scatter.py
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/planted -o run --output-format csv -- python3 bench.py --workload train --graph planted --steps 100 --warmup 10 > $O/planted.log 2>&1
