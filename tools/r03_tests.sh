#!/bin/bash
# Run a subset of the -m gpu tests (args: pytest selectors) on the box, log under gpurun_out/TAG.
# Exit status: pytest's, so a caller can go on after plain test failures (1) but must stop after
# a crash, abort or time limit (>= 2: 124/134/137/139 ...).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
