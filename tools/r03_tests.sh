#!/bin/bash
# Run a subset of the -m gpu tests (args: pytest selectors) on the box, log under gpurun_out/TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
