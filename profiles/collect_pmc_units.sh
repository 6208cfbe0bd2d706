#!/bin/bash
# Which hardware unit bounds each large kernel: per-kernel PMC passes over the
# serial leg of the bench workload (pipeline 0: every kernel alone; per-dispatch counter collection
# serialises dispatches anyway), one rocprofv3 pass per counter group within gfx950's per-block
# slot limits (SQ 8, TCC 4, TCP 4, TA 2, TD 2, GRBM 2; SQC alone), each under its own KILL timeout.
# Usage (GPU box, repo root):  bash profiles/collect_pmc_units.sh gpurun_out/units
set -o pipefail
OUT=${1:-gpurun_out/units}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-profile --pipeline 0"
# the first torch import of a fresh box pages the image in (minutes): not under a pass's limit
timeout -k 10 400 python3 -c "import torch; torch.zeros(1).cuda(); print('warm')" > "$OUT/warm.log" 2>&1 || exit 1
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_IFETCH" \
           "SQ_IFETCH_LEVEL SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS_ATOMIC SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ATOMIC_RETURN" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_ATOMIC_WITH_RET_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCC_REQ_sum TCC_ATOMIC_sum TCC_BUSY_sum TCC_TAG_STALL_sum" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "tsdf::" --output-format csv \
      -d "$OUT/p$i" -o pmc -- $CMD > "$OUT/p$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i ($grp) failed rc=$rc"; tail -5 "$OUT/p$i.log"
    # a killed or crashed pass ends the call (no further GPU step after a failure)
    [ $rc -ge 124 ] && break
  fi
done
python3 profiles/summarize_pmc.py "$OUT" > "$OUT/summary.txt" || true
python3 profiles/units_report.py "$OUT" > "$OUT/units.txt" || true
rm -rf "$OUT"/p[0-9]*/
cat "$OUT/units.txt"
