#!/bin/bash
# Interleaved A/B of the default library against a variant built by tools/build_variant.py:
# the C2 bench alternately with each (the box's tree is a scratch copy, so the variant is copied
# over lgcn_amd/liblgcn.so and back).  usage: gpurun -- 'bash tools/ab_lib.sh TAG ab/VARIANT.so [bench args]'
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
L=movie-recommender-system-with-gnns_amd/lgcn_amd/liblgcn.so
cp $L $O/base.so
for i in 1 2; do
  cp $O/base.so $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/base_$i.log 2>&1 || exit 1
  cp $VAR $L && timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $O/var_$i.log 2>&1 || exit 1
done
cp $O/base.so $L; rm -f $O/base.so
