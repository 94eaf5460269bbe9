"""Sum rocprofv3 --pmc counters over the conv dispatches of one counter-collection CSV
(tuning aid for scripts/tune_conv_x6.py runs under the profiler):

    python scripts/pmc_layer.py <..._counter_collection.csv> [kernel-substring]

Prints each counter's total over the matching dispatches and the usual ratios: MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES per SIMD-cycle), and the wave-cycle split (SQ_WAIT_ANY parked at
s_waitcnt / barrier, SQ_WAIT_INST_ANY issue-stalled, SQ_ACTIVE_INST_ANY issuing)."""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "conv_x6_kernel"
    tot = defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(path)):
        if sub not in r["Kernel_Name"]:
            continue
        disp.add(r["Dispatch_Id"])
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"{len(disp)} dispatches of *{sub}*")
    for k, v in sorted(tot.items()):
        print(f"  {k:28s} {v:.4g}")
    if "GRBM_GUI_ACTIVE" in tot and "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
        print(f"  MFMA busy {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (tot['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    w = tot.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in tot:
                print(f"  {k} / SQ_WAVE_CYCLES = {tot[k] / w:.3f}")
    if "SQ_LDS_IDX_ACTIVE" in tot and "SQ_LDS_BANK_CONFLICT" in tot:
        print(f"  LDS bank-conflict cycles / LDS active = "
              f"{tot['SQ_LDS_BANK_CONFLICT'] / tot['SQ_LDS_IDX_ACTIVE']:.3f}")


if __name__ == "__main__":
    main()
