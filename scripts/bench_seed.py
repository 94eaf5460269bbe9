"""Time the device TCAM seeder (one training step's batch: 8 clips x 32 frames of
224x224 cams_inter, README seeding config) and prepare_std_cams, against the
per-sample CPU restatement (oracle/seed_ref.py, numpy, 1 thread) on a sample."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tcam_wsol_video_amd.seeding import TCAMSeeder, prepare_std_cams  # noqa: E402


def main():
    B, h, w = int(os.environ.get("B", 256)), 224, 224
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    low = np.zeros((B, 1, 28, 28), np.float32)
    for i in range(B):
        c = np.zeros((28, 28), np.float32)
        for _ in range(3):
            cy, cx, s = rng.uniform(0, 28), rng.uniform(0, 28), rng.uniform(2, 7)
            c += np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
        c += 0.05 * rng.random((28, 28))
        low[i, 0] = (c - c.min()) / (c.max() - c.min())
    res = {"frames": B, "HxW": [h, w]}
    for name, kw in (("readme", dict(seed_tech="seed_weighted", min_=1, max_=1, max_p=0.6,
                                     min_p=0.1, ksz=3, roi_method="roi_all", use_roi=True)),
                     ("config_default", dict(seed_tech="seed_uniform", min_=10, max_=10,
                                             max_p=0.2, min_p=0.2, ksz=1, roi_method="roi_all",
                                             use_roi=False)),
                     ("largest_roi", dict(seed_tech="seed_weighted", min_=10, max_=10,
                                          max_p=0.6, min_p=0.1, ksz=3, roi_method="largest",
                                          use_roi=True))):
        s = TCAMSeeder(fg_erode_k=11, fg_erode_iter=0, support_background=False,
                       multi_label_flag=False, seg_ignore_idx=-255, cuda_id=0,
                       p_min_area_roi=0.05, **kw)
        x = torch.from_numpy(low).to(dev)
        for _ in range(3):
            cams = prepare_std_cams(x, (h, w))
            seeds = s.seeds_i32(cams)
        torch.cuda.synchronize()
        reps = 10
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        for _ in range(reps):
            cams = prepare_std_cams(x, (h, w))
        e[1].record()
        for _ in range(reps):
            seeds = s.seeds_i32(cams)
        e[2].record()
        torch.cuda.synchronize()
        prep_ms = e[0].elapsed_time(e[1]) / reps
        seed_ms = e[1].elapsed_time(e[2]) / reps
        r = {"prepare_std_cams_ms": round(prep_ms, 4), "seeder_ms": round(seed_ms, 4),
             "frames_per_s": round(B / (prep_ms + seed_ms) * 1e3, 1),
             "fg_per_frame": float((seeds == 1).sum().item() / B),
             "bg_per_frame": float((seeds == 0).sum().item() / B)}
        try:
            from oracle import seed_ref as SR
            cfg = SR.default_cfg(seed_tech=kw["seed_tech"], min_=kw["min_"], max_=kw["max_"],
                                 max_p=kw["max_p"], min_p=kw["min_p"], ksz=kw["ksz"],
                                 roi_method=kw["roi_method"], use_roi=kw["use_roi"])
            n_cpu = 8
            camsn = cams[:n_cpu].cpu().numpy()
            t = time.perf_counter()
            ref = SR.seeder(camsn, cfg, seed=0, offset=s._offset - 1)
            dt = time.perf_counter() - t
            r["cpu_oracle_frames_per_s"] = round(n_cpu / dt, 2)
            r["cpu_sample"] = f"{n_cpu} frames, numpy restatement, 1 thread"
            r["bitexact_vs_oracle"] = bool(np.array_equal(seeds[:n_cpu].cpu().numpy(), ref))
        except Exception as ex:  # noqa: BLE001
            r["cpu_error"] = str(ex)
        res[name] = r
    print(json.dumps(res))


if __name__ == "__main__":
    main()
