"""Diagnostic: repeat the bbox stage on the bench's CAMs under each (fill, level) variant
pair and count the runs whose boxes differ from the per-level CCL reference."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcam_wsol_video_amd import ops, _lib  # noqa: E402


def main():
    dev = torch.device("cuda")
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench_cam_u8.npy"
    u8 = torch.from_numpy(np.load(path)).to(dev)
    lib = _lib.load()
    reps = int(os.environ.get("REPS", "20"))

    def run(fill, level):
        lib.tcam_bbox_fill_variant(fill)
        lib.tcam_bbox_level_variant(level)
        b, v = ops.bbox_levels(u8)
        torch.cuda.synchronize()
        valid = (torch.arange(256, device=dev)[None, :] < v[:, None])[..., None]
        return b * valid, v

    ref = run(2, 1)
    for fill, level in [(2, 1), (2, 2), (2, 0), (0, 1), (0, 2), (0, 0), (1, 0)]:
        bad, where = 0, set()
        for _ in range(reps):
            b, v = run(fill, level)
            if not (torch.equal(v, ref[1]) and torch.equal(b, ref[0])):
                bad += 1
                diff = (b != ref[0]).any(-1).nonzero()
                where.update((int(f), int(L)) for f, L in diff[:4].tolist())
        print(f"fill {fill} level {level}: {bad}/{reps} runs differ  {sorted(where)[:8]}",
              flush=True)
    lib.tcam_bbox_fill_variant(0)
    lib.tcam_bbox_level_variant(0)


if __name__ == "__main__":
    main()
