"""Per-unit utilisation of the tsdf kernels from profiles/collect_pmc_units.sh's passes.

Reads <dir>/summary.json (per-dispatch means, profiles/summarize_pmc.py) and prints, per kernel,
each unit's busy share of the kernel's cycles, so the unit that saturates (if any) stands out:
  cycles      GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; MI355X_MICROARCH.md, DVFS note)
  VALU        SQ_INSTS_VALU x 2 cycles (wave64 on a SIMD-32) / (1024 SIMDs x cycles)
  SALU        SQ_INST_CYCLES_SALU / (256 CUs x cycles)   (one scalar unit per CU)
  TA / TD     TA_TA_BUSY_sum, TD_TD_BUSY_sum / (256 x cycles)
  TCC         TCC_BUSY_sum / (128 L2 channels x cycles), requests and atomics per cycle
  waits       SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_WAIT_INST_LDS, SQ_ACTIVE_INST_ANY as shares of
              SQ_WAVE_CYCLES (all four in the same quad-cycle unit)
  I-cache     SQC_ICACHE_MISSES / (hits + misses)
Usage: python3 profiles/units_report.py gpurun_out/units
"""
import json
import os
import sys

CUS, SIMDS, TCC_CH = 256, 1024, 128


def main(root):
    with open(os.path.join(root, "summary.json")) as f:
        s = json.load(f)
    out = {}
    for k in ("k_count", "k_place", "k_integrate", "k_compact_sum", "k_compact_write"):
        d = s.get(k)
        if not d:
            continue
        g = lambda n: d.get(n, float("nan"))  # noqa: E731
        cyc = g("GRBM_GUI_ACTIVE") / 8.0
        wc = g("SQ_WAVE_CYCLES")
        r = {
            "cycles": cyc,
            "valu_pipe": g("SQ_INSTS_VALU") * 2.0 / (SIMDS * cyc),
            "valu_active_share": g("SQ_ACTIVE_INST_VALU") / wc,
            "salu_unit": g("SQ_INST_CYCLES_SALU") / (CUS * cyc),
            "salu_per_valu": g("SQ_INSTS_SALU") / g("SQ_INSTS_VALU"),
            "ta_busy": g("TA_TA_BUSY_sum") / (CUS * cyc),
            "ta_stalled_by_tc": g("TA_ADDR_STALLED_BY_TC_CYCLES_sum") / (CUS * cyc),
            "td_busy": g("TD_TD_BUSY_sum") / (CUS * cyc),
            "td_tc_stall": g("TD_TC_STALL_sum") / (CUS * cyc),
            "tcc_busy": g("TCC_BUSY_sum") / (TCC_CH * cyc),
            "tcc_req_per_cycle": g("TCC_REQ_sum") / cyc,
            "tcc_atomic_per_cycle": g("TCC_ATOMIC_sum") / cyc,
            "tcc_tag_stall": g("TCC_TAG_STALL_sum") / (TCC_CH * cyc),
            "tcp_tcc_read_per_cu_cycle": g("TCP_TCC_READ_REQ_sum") / (CUS * cyc),
            "tcp_tcc_write_per_cu_cycle": g("TCP_TCC_WRITE_REQ_sum") / (CUS * cyc),
            "tcp_tcc_atomic_ret_per_cu_cycle": g("TCP_TCC_ATOMIC_WITH_RET_REQ_sum") / (CUS * cyc),
            "tcp_pending_stall": g("TCP_PENDING_STALL_CYCLES_sum") / (CUS * cyc),
            "tcp_ta_data_stall": g("TCP_TCP_TA_DATA_STALL_CYCLES_sum") / (CUS * cyc),
            "tcp_tcr_stall": g("TCP_TCR_TCP_STALL_CYCLES_sum") / (CUS * cyc),
            "wait_any": g("SQ_WAIT_ANY") / wc,
            "wait_inst_any": g("SQ_WAIT_INST_ANY") / wc,
            "wait_inst_lds": g("SQ_WAIT_INST_LDS") / wc,
            "active_inst_any": g("SQ_ACTIVE_INST_ANY") / wc,
            "lds_active_share": g("SQ_ACTIVE_INST_LDS") / wc,
            "waves_per_simd": wc * 4.0 / (SIMDS * cyc),
            "ifetch_per_wave_cycle": g("SQ_IFETCH") / wc,
            "icache_miss_rate": g("SQC_ICACHE_MISSES") / (g("SQC_ICACHE_HITS") + g("SQC_ICACHE_MISSES")),
            "lds_atomics": g("SQ_INSTS_LDS_ATOMIC"),
            "lds_addr_conflict": g("SQ_LDS_ADDR_CONFLICT"),
            "lds_data_fifo_full": g("SQ_LDS_DATA_FIFO_FULL"),
            "lds_cmd_fifo_full": g("SQ_LDS_CMD_FIFO_FULL"),
            "inst_level_vmem_per_wave": g("SQ_INST_LEVEL_VMEM") / wc,
            "inst_level_lds_per_wave": g("SQ_INST_LEVEL_LDS") / wc,
        }
        out[k] = r
        print(k)
        for n, v in r.items():
            print("  %-32s %12.4g" % (n, v))
    with open(os.path.join(root, "units.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/units")
