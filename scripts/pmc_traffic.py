"""Reduce the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py
(scripts/gpu_pmc_traffic.sh) to HBM bytes per launch of the dominant kernel family
(conv_x6_kernel), with the gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads: doubled; WRITE_SIZE exact).  The
counters are in KiB.  Writes tcam_wsol_video_amd/perfdata/pmc_traffic.json, which bench.py
reports as roofline.traffic."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if "conv_x6_kernel" not in r["Kernel_Name"] and "conv3x3_thin_kernel" not in r["Kernel_Name"]:
            continue
        out[int(r["Dispatch_Id"])] = float(r["Counter_Value"]) * 1024.0
    return out


def main(d=os.path.join(ROOT, "gpurun_out", "pmc_traffic")):
    f = per_dispatch(os.path.join(d, "fetch_counter_collection.csv"))
    w = per_dispatch(os.path.join(d, "write_counter_collection.csv"))
    # the two passes replay the same program: the conv launches pair up in order
    fv, wv = list(f.values()), list(w.values())
    n = min(len(fv), len(wv))
    if n == 0:
        sys.exit("no conv_x6 dispatches found")
    fetch = sum(fv[:n]) * 2.0 / n
    write = sum(wv[:n]) / n
    res = {"kernel": "conv_x6_kernel + conv3x3_thin_kernel", "launches": n,
           "hbm_bytes_per_launch": fetch + write, "fetch_bytes_per_launch": fetch,
           "write_bytes_per_launch": write,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over bench.py "
                     "--steps 3 --warmup 1; FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md §HBM); KiB"}
    os.makedirs(os.path.join(ROOT, "tcam_wsol_video_amd", "perfdata"), exist_ok=True)
    with open(os.path.join(ROOT, "tcam_wsol_video_amd", "perfdata", "pmc_traffic.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:])
