#!/bin/bash
# Builds k_score_filter A/B variants of liblgcn.so into tools/_variants/ (see tools/recall_variants.py).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/movie-recommender-system-with-gnns_amd/csrc
mkdir -p "$R/tools/_variants"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -ffp-contract=off -I$R/include"
SRC="$C/lgcn_plan.hip $C/lgcn_spmm.hip $C/lgcn_optim.hip $C/lgcn_bpr.hip $C/lgcn_recall.hip $C/lgcn_partition.cpp $C/lgcn_sample.cpp"
for v in "$@"; do
  /opt/rocm/bin/hipcc $F -DLGCN_VARIANT_$v $SRC -o "$R/tools/_variants/$v.so" &
done
wait
