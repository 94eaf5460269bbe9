"""Reduce the rocprofv3 --pmc passes of the headline bench command (scripts/gpu.sh pmc:
FETCH_SIZE, WRITE_SIZE and SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE, each
its own run) to per-launch figures of the dominant kernel family (conv_x6_kernel +
conv3x3_thin_kernel + stem_f16x3_kernel + bottleneck_f16x3_kernel):

* HBM bytes per launch with the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
  counts half the bytes of 16-B/lane streaming reads: doubled; WRITE_SIZE exact; KiB);
* MFMA-pipe busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
  (GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; 256 CUs x 4 SIMDs) and the effective clock.

Writes tcam_wsol_video_amd/perfdata/pmc_traffic.json (bench.py reports it as
roofline.traffic) and prints a markdown summary for profiles/.

    python scripts/pmc_traffic.py [gpurun_out/pmc]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONV = ("conv_x6_kernel", "conv3x3_thin_kernel", "stem_f16x3_kernel", "bottleneck_f16x3_kernel")


def dispatches(path):
    """{dispatch id: {counter: value}} of the conv launches, in dispatch order."""
    out = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        if not any(k in r["Kernel_Name"] for k in CONV):
            continue
        d = int(r["Dispatch_Id"])
        out[d][r["Counter_Name"]] = out[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    return [out[d] for d in sorted(out)], [names[d] for d in sorted(out)]


def _one(d, prefix):
    f = glob.glob(os.path.join(d, f"{prefix}*counter_collection.csv"))
    if not f:
        sys.exit(f"no {prefix}*counter_collection.csv under {d}")
    return dispatches(f[0])


def main(d=os.path.join(ROOT, "gpurun_out", "pmc")):
    fv, _ = _one(d, "fetch_size")
    wv, _ = _one(d, "write_size")
    mv, _ = _one(d, "sq_valu_mfma_busy_cycles")
    n = min(len(fv), len(wv))
    if n == 0:
        sys.exit("no conv dispatches found")
    fetch = sum(x["FETCH_SIZE"] for x in fv[:n]) * 1024.0 * 2.0 / n
    write = sum(x["WRITE_SIZE"] for x in wv[:n]) * 1024.0 / n
    busy = sum(x["SQ_VALU_MFMA_BUSY_CYCLES"] for x in mv)
    gui = sum(x["GRBM_GUI_ACTIVE"] for x in mv)
    sys.path.insert(0, ROOT)
    import bench
    prec = os.environ.get("TCAM_CONV_PRECISION", "f16x3")
    res = {"kernel": "conv_x6_kernel + conv3x3_thin_kernel + stem_f16x3_kernel + bottleneck_f16x3_kernel", "launches": n,
           "precision": prec, "conv_sources_sha": bench.conv_sources_sha(),
           "commit": os.environ.get("TCAM_COMMIT", "?"),
           "hbm_bytes_per_launch": fetch + write, "fetch_bytes_per_launch": fetch,
           "write_bytes_per_launch": write,
           "mfma_busy_frac": busy / (gui / 8.0 * 1024.0) if gui else None,
           "method": "rocprofv3 --pmc, one pass per counter set, over the headline bench command "
                     "(2 forward streams); FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md §HBM); "
                     "KiB; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024)"}
    os.makedirs(os.path.join(ROOT, "tcam_wsol_video_amd", "perfdata"), exist_ok=True)
    with open(os.path.join(ROOT, "tcam_wsol_video_amd", "perfdata", "pmc_traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(f"| conv launches | fetch GB/launch | write GB/launch | HBM GB/launch | MFMA busy |")
    print("|---|---|---|---|---|")
    print(f"| {n} | {fetch / 1e9:.4f} | {write / 1e9:.4f} | {(fetch + write) / 1e9:.4f} | "
          f"{res['mfma_busy_frac']:.3f} |")


if __name__ == "__main__":
    main(*sys.argv[1:])
