#!/usr/bin/env python3
"""Summarise the SQ counter passes written by scripts/gemm_counters.sh.

Per kernel (name substring): mean duration from the kernel trace, effective
shader clock (GRBM_GUI_ACTIVE / XCDs / duration), the issue/wait breakdown as
fractions of SQ_WAVE_CYCLES, MFMA-busy as a fraction of SIMD-cycles, and the
instruction mix per MFMA.
"""
import csv
import sys
from collections import defaultdict

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
KERNELS = sys.argv[2].split(",") if len(sys.argv) > 2 else ["gemm_nt_x3g", "k_aggregate_vec", "k_sage_normalize"]
CUS, XCDS, SIMDS = 256, 8, 4


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def durations(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return acc


def pick(d, sub):
    for k, v in d.items():
        if sub in k:
            return v
    return None


def mean(x):
    return sum(x) / len(x) if x else float("nan")


def main():
    c1 = counters(f"{OUT}/pmc_sq/run_counter_collection.csv")
    c2 = counters(f"{OUT}/pmc_sq2/run_counter_collection.csv")
    kt = durations(f"{OUT}/kt_sq/run_kernel_trace.csv")
    try:
        c3 = counters(f"{OUT}/pmc_sq3/run_counter_collection.csv")
    except FileNotFoundError:
        c3 = {}
    for sub in KERNELS:
        a, b, t = pick(c1, sub), pick(c2, sub), pick(kt, sub)
        if not (a and b and t):
            print(f"{sub}: not found")
            continue
        dur = mean(t)
        clk = mean(b["GRBM_GUI_ACTIVE"]) / XCDS / dur
        wave = mean(a["SQ_WAVE_CYCLES"])
        simd_cycles = dur * clk * CUS * SIMDS
        mfma = mean(b["SQ_INSTS_MFMA"])
        print(f"{sub}: {dur * 1e3:.2f} ms  clock {clk / 1e9:.3f} GHz  "
              f"wait_any {mean(a['SQ_WAIT_ANY']) / wave:.2f}  wait_inst {mean(a['SQ_WAIT_INST_ANY']) / wave:.2f}  "
              f"active {mean(a['SQ_ACTIVE_INST_ANY']) / wave:.2f}  "
              f"mfma_busy {mean(a['SQ_VALU_MFMA_BUSY_CYCLES']) / simd_cycles:.3f}  "
              f"lds_conflict {mean(a['SQ_LDS_BANK_CONFLICT']):.3g}  wait_lds {mean(a['SQ_WAIT_INST_LDS']):.3g}")
        c = pick(c3, sub) if c3 else None
        if c:
            lds_cycles = dur * clk * CUS
            print(f"    vmem_rd issue {mean(c['SQ_INST_CYCLES_VMEM_RD']) / wave:.3f}  active_vmem {mean(c['SQ_ACTIVE_INST_VMEM']) / wave:.3f}  "
                  f"active_lds {mean(c['SQ_ACTIVE_INST_LDS']) / wave:.3f}  ta_addr_full {mean(c['SQ_VMEM_TA_ADDR_FIFO_FULL']):.3g}  "
                  f"ta_cmd_full {mean(c['SQ_VMEM_TA_CMD_FIFO_FULL']):.3g}  lds_active {mean(c['SQ_LDS_IDX_ACTIVE']) / lds_cycles:.3f} "
                  f"lds_data_full {mean(c['SQ_LDS_DATA_FIFO_FULL']):.3g}  coexec {mean(c['SQ_VALU_MFMA_COEXEC_CYCLES']) / simd_cycles:.3f}")
        if mfma:
            print(f"    per MFMA: VALU {mean(b['SQ_INSTS_VALU']) / mfma:.2f}  LDS {mean(b['SQ_INSTS_LDS']) / mfma:.2f}  "
                  f"(MFMA {mfma:.3g})")


if __name__ == "__main__":
    main()
