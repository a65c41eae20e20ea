"""Utilisation of the vector-memory gather pipeline (TA -> TCP (L1) -> TD) of the march kernel
from tools/pmc_passes.sh output with tools/pmc_sets_ta.txt.  Per-CU-cycle figures divide the
counter's sum over the 256 CUs by 256 x the XCD cycles of the dispatch (GRBM_GUI_ACTIVE / 8).
Usage: python tools/gather_report.py <pmc dir> [kernel substring]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_report  # noqa: E402

N_CU = 256
PER_CU = ("TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum",
          "TA_ADDR_STALLED_BY_TD_CYCLES_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum",
          "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_PENDING_STALL_CYCLES_sum",
          "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum",
          "TCP_TD_TCP_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum")


def main():
    d = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else "march_kernel"
    c, dur = pmc_report.load(d, kname)
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    out = {"dispatch_ms": round(dur * 1e3, 4), "clock_ghz": round(cyc / dur / 1e9, 3),
           "per_cu_cycle": {k: round(c[k] / N_CU / cyc, 3) for k in PER_CU if k in c}}
    acc = c.get("TCP_TOTAL_CACHE_ACCESSES_sum")
    if acc:
        out["l1_hit_rate"] = round(1 - c["TCP_TCC_READ_REQ_sum"] / acc, 3)
        out["tcp_accesses_per_vmem_instr"] = round(acc / c["SQ_INSTS_VMEM_RD"], 2)
        out["tcp_latency_cycles_per_access"] = round(c.get("TCP_TCP_LATENCY_sum", 0) / acc, 1)
    wc = c["SQ_WAVE_CYCLES"]
    out["wave_cycles_waiting_frac"] = round(c["SQ_WAIT_ANY"] / wc, 3)
    out["wave_cycles_valu_frac"] = round(c["SQ_ACTIVE_INST_VALU"] / wc, 3)
    out["valu_instr_per_vmem_instr"] = round(c["SQ_INSTS_VALU"] / c["SQ_INSTS_VMEM_RD"], 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
