#!/bin/bash
# Issue/wait/instruction counters for ONE kernel (rocprofv3 --kernel-include-regex), each group its
# own --pmc pass, of any bench.py command. Summarise with tools/pmc_limiter.py <out dir> --kernel K.
# usage (GPU box): bash tools/pmc_kernel.sh OUTTAG KERNEL_REGEX [bench args...]
set -uo pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_kernel}
KRE=${2:-k_row_adam}
shift 2 || true
ARGS=${*:---steps 3 --warmup 1 --no-cpu-baseline}
mkdir -p "$OUT"
cd "$R"
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES"
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum"
)
i=0
for g in "${GROUPS_[@]}"; do
  i=$((i + 1))
  echo "pass $i: $g" | tee -a "$OUT/passes.txt"
  timeout -s KILL 180 rocprofv3 --kernel-include-regex "$KRE" --pmc $g -T -d "$OUT/p$i" -o run --output-format csv \
    -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  find "$OUT/p$i" -type f ! -name '*counter_collection.csv' -delete
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc" | tee -a "$OUT/passes.txt"; exit $rc; fi
done
echo done > "$OUT/DONE"
