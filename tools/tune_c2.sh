#!/bin/bash
# C2 headline tuning sweep: slice size x chunk x gather unroll (one bench line each).
set -e
mkdir -p gpurun_out/tune
for mb in 8 10 12; do
  for ch in 128 256 512; do
    for v in 0 1; do
      LGCN_SLICE_MB=$mb LGCN_SPMM_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu-baseline --chunk $ch --steps 30 \
        > gpurun_out/tune/mb${mb}_ch${ch}_v${v}.log 2>&1
      echo "mb=$mb chunk=$ch variant=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tune/mb${mb}_ch${ch}_v${v}.log)"
    done
  done
done
