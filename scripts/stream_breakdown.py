"""Per-stream CU-time breakdown of a rocprofv3 kernel trace (the training steps' overlap
evidence): for every HIP stream, the summed kernel time, its union (busy wall time), and a
CU-time estimate per kernel = duration x min(1, workgroups / (256 CUs x resident blocks per
CU)), the resident blocks from the dispatch's LDS / VGPR / thread counts (gfx950: 160 KiB
LDS, 512 VGPRs x 4 SIMDs of 64 lanes per CU).  Kernels are grouped by family.

    python scripts/stream_breakdown.py <kernel_trace.csv> [--skip-steps N --steps K]
"""
import argparse
import collections
import csv
import json
import re

CUS = 256
FAMILIES = [
    ("conv_fwd_dgrad", r"conv_x6_kernel|bottleneck_f16x3_kernel|stem_f16x3"),
    ("wgrad", r"wgrad"),
    ("bn", r"bn_|dy_amax|dy_scale|dy_to_s2"),
    ("crf_lattice", r"bilateral|lattice|splat|slice|blur|crf_|radix|hash"),
    ("loss_softmax", r"loss|softmax|chansum"),
    ("sgd_amp", r"sgd|amp_unscale|amp_update"),
    ("pack", r"pack_"),
    ("resample", r"up2|resize|mosaic|pool|seghead|wgap|cls_|ce_loss|zero_up2|grad_add"),
    ("copy", r"rocclr|copyBuffer|fillBuffer"),
]


def family(name: str) -> str:
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def resident(lds: int, vgpr: int, agpr: int, threads: int) -> int:
    waves = max(1, (threads + 63) // 64)
    regs = max(1, vgpr + agpr)
    per_simd = max(1, 512 // regs)              # waves per SIMD by registers
    by_regs = max(1, (4 * per_simd) // waves)   # blocks per CU by registers
    by_lds = 160 * 1024 // lds if lds > 0 else 64
    by_waves = max(1, 32 // waves)
    return max(1, min(by_regs, by_lds, by_waves))


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=0.0,
                    help="keep only the last WINDOW ms of the trace (0: all)")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows = [r for r in rows if r["Kind"] == "KERNEL_DISPATCH"]
    t_end = max(int(r["End_Timestamp"]) for r in rows)
    if args.window:
        t0 = t_end - int(args.window * 1e6)
        rows = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
    t_start = min(int(r["Start_Timestamp"]) for r in rows)
    per_stream = collections.defaultdict(lambda: {"kernel_ms": 0.0, "cu_ms": 0.0, "iv": [],
                                                  "fam": collections.Counter()})
    fam_tot = collections.Counter()
    cu_tot = 0.0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e6
        wg = max(1, int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) //
                 max(1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) *
                     int(r["Workgroup_Size_Z"])))
        thr = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        res = resident(int(r["LDS_Block_Size"]), int(r["VGPR_Count"]),
                       int(r["Accum_VGPR_Count"]), thr)
        frac = min(1.0, wg / (CUS * res))
        key = (r["Queue_Id"], r["Stream_Id"])
        st = per_stream[key]
        st["kernel_ms"] += d
        st["cu_ms"] += d * frac
        st["iv"].append((s, e))
        f = family(r["Kernel_Name"])
        st["fam"][f] += d * frac
        fam_tot[f] += d * frac
        cu_tot += d * frac
    wall = (t_end - t_start) / 1e6
    out = {"wall_ms": round(wall, 3),
           "union_all_ms": round(union([iv for st in per_stream.values() for iv in st["iv"]]) / 1e6, 3),
           "cu_time_ms": round(cu_tot, 3),
           "cu_time_over_wall": round(cu_tot / wall, 3) if wall else None,
           "families_cu_ms": {k: round(v, 3) for k, v in fam_tot.most_common()},
           "streams": {}}
    for (q, sid), st in sorted(per_stream.items(), key=lambda kv: -kv[1]["cu_ms"]):
        out["streams"][f"queue{q}/stream{sid}"] = {
            "kernel_ms": round(st["kernel_ms"], 3), "busy_ms": round(union(st["iv"]) / 1e6, 3),
            "cu_ms": round(st["cu_ms"], 3),
            "families_cu_ms": {k: round(v, 3) for k, v in st["fam"].most_common(6)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
