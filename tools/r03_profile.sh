#!/bin/bash
# Round-3 evidence run: the GPU tests not yet run on the current code (multi-GPU recall, reduce
# mode), then the C2 round profile (kernel trace + FETCH/WRITE_SIZE passes + calibration,
# tools/profile_round.sh) and the training kernel traces (tools/profile_train.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; O=gpurun_out/$T; mkdir -p $O
bash tools/r03_tests.sh $T tests/test_gpu_dp_recall.py tests/test_gpu_sharded.py
rc=$?
[ $rc -le 1 ] || exit $rc
PROF_TAG=$T/prof bash tools/profile_round.sh && bash tools/profile_train.sh $T/train
