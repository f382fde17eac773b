#!/bin/bash
# k_bpr_fused with speculative F-row loads on small batches (B < 49152) vs the committed kernel:
# the training / program / harness GPU tests on the new build, then interleaved C3 bench pairs.
#   bash tools/bpr_spec_ab.sh TAG VARIANT.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1; VAR=$2
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_program.py tests/test_gpu_harness.py \
  tests/test_gpu_configs.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 || exit $?
L=movie-recommender-system-with-gnns_amd/lgcn_amd/liblgcn.so
cp $L "$O/base.so"
B="python -u bench.py --workload train --steps 300 --warmup 30 --no-cpu-baseline --no-harness"
for i in 1 2 3; do
  cp "$O/base.so" $L && timeout -k 10 300 $B > "$O/spec_$i.log" 2>&1 || exit 1
  cp "$VAR" $L && timeout -k 10 300 $B > "$O/head_$i.log" 2>&1 || exit 1
done
cp "$O/base.so" $L; rm -f "$O/base.so"
