"""Summarise scripts/gpu_pmc_deep.sh's PMC passes per conv launch shape (the ab_f16.py
layers, in run order): averages over the launches of each kernel + grid, and the derived
ratios (MFMA busy per SIMD-cycle, wait fractions, LDS bank-conflict share)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_deep"
vals = defaultdict(lambda: defaultdict(list))
names = {}
for f in sorted(glob.glob(os.path.join(d, "pass*_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "conv_x6_kernel" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("ConvTileG<")[-1][:40], r["Grid_Size"])
        names[key] = r["Kernel_Name"]
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, c in vals.items():
    a = {k: sum(v) / len(v) for k, v in c.items()}
    g = a.get("GRBM_GUI_ACTIVE", 0)
    simd_cyc = g / 8 * 1024 if g else 0   # GRBM sums the 8 XCDs; 1024 SIMDs
    print(f"{key[0]} grid {key[1]}")
    for k in sorted(a):
        print(f"    {k:28s} {a[k]:16.0f}")
    if simd_cyc:
        print(f"    MFMA busy / SIMD-cycle        {a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / simd_cyc:.3f}")
    w = a.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in a:
                print(f"    {k} / WAVE_CYCLES {a[k] / w:.3f}")
    if a.get("SQ_LDS_IDX_ACTIVE"):
        print(f"    LDS bank conflict share       {a.get('SQ_LDS_BANK_CONFLICT', 0) / a['SQ_LDS_IDX_ACTIVE']:.3f}")
