#!/bin/bash
# Collect per-kernel PMC counters for the bench workload, one rocprofv3 pass per counter group
# (gfx950: FETCH_SIZE and WRITE_SIZE do not fit one pass; --pmc never combined with tracing).
# Usage (on the GPU box, from the repo root):  bash profiles/collect_pmc.sh gpurun_out/pmc
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-profile"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum" \
           "SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
           "SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "tsdf::" --output-format csv -d "$OUT/p$i" -o pmc -- $CMD \
    > "$OUT/p$i.log" 2>&1 || { rc=$?; echo "pass $i ($grp) failed rc=$rc"; tail -5 "$OUT/p$i.log"; [ $rc -ge 124 ] && exit 1; }
done
python3 profiles/summarize_pmc.py "$OUT" > "$OUT/summary.txt" || true
rm -rf "$OUT"/p[0-9]*/
cat "$OUT/summary.txt"
