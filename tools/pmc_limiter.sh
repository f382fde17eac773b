#!/bin/bash
# Counters that name what bounds the C2 item pass (k_spmm_vec): issue/wait split, vmem and VALU
# instruction counts, TA busy, L1/L2 request counts and hit rates. Each group is its own --pmc pass
# (slot limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 GRBM); counters the box does not list are dropped
# from a group before it runs. Summarise with tools/pmc_limiter.py <out dir>.
# usage (GPU box): bash tools/pmc_limiter.sh OUTTAG [bench args...]
set -uo pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-pmc_limiter}
shift || true
ARGS=${*:---steps 3 --warmup 1 --no-cpu-baseline}
mkdir -p "$OUT"
cd "$R"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || { echo "counter listing failed"; exit 1; }
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES"
  "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TA_FLAT_READ_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
  "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TA_TCP_STATE_READ_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_READ_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_TAG_STALL_sum TCC_BUSY_sum"
)
i=0
for g in "${GROUPS_[@]}"; do
  keep=""
  for c in $g; do
    base=${c%_sum}
    if grep -qw -- "$c" "$OUT/avail.txt" || grep -qw -- "$base" "$OUT/avail.txt"; then keep="$keep $c"; fi
  done
  i=$((i + 1))
  [ -z "$keep" ] && continue
  echo "pass $i:$keep" | tee -a "$OUT/passes.txt"
  timeout -s KILL 120 rocprofv3 --pmc $keep -T -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py $ARGS \
    > "$OUT/p$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc" | tee -a "$OUT/passes.txt"; exit $rc; fi
done
echo done > "$OUT/DONE"
