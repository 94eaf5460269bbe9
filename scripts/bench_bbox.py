"""Time the bbox kernels alone on the bench's CAMs (fill variants 2 = register lines,
1 = LDS sweeps, 0 = clamp scans, the default); dump the CAMs for analysis.  Per-kernel
times: run it under rocprofv3 --kernel-trace --stats (scripts/gpu.sh bboxprof)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tcam_wsol_video_amd import ops  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402

dev = torch.device("cuda")
model = build_r50_tcam(seed=0).to(dev)
x, targets, gt = bench.make_clip(32, seed=1000)
with torch.no_grad():
    model(x.to(dev), want_fcams=False)
u8 = model.cam_u8
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/bench_cam_u8.npy", u8.cpu().numpy())
from tcam_wsol_video_amd import _lib  # noqa: E402
ref = None
for variant in (2, 1, 0):
    _lib.load().tcam_bbox_fill_variant(variant)
    for _ in range(3):
        out = ops.bbox_levels(u8)
    torch.cuda.synchronize()
    boxes, vm = out
    valid = torch.arange(256, device=dev)[None, :] < vm[:, None]  # levels >= vmax unused
    cur = (boxes * valid[..., None], vm)
    if ref is None:
        ref = [t.clone() for t in cur]
    else:
        assert all(torch.equal(a, b) for a, b in zip(ref, cur)), "fill variants disagree"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.bbox_levels(u8)
    e1.record()
    torch.cuda.synchronize()
    print(f"fill variant {variant}: bbox_levels {e0.elapsed_time(e1) / 10:.3f} ms per clip",
          flush=True)
_lib.load().tcam_bbox_fill_variant(0)

# fill phases of the default (clamp-scan) fill (s_memrealtime, 100 MHz ticks)
B = u8.shape[0]
dbg = torch.zeros(2 * B * 16 * 16, dtype=torch.int64, device=dev)
_lib.load().tcam_bbox_set_debug(dbg.data_ptr())
ops.bbox_levels(u8)
torch.cuda.synchronize()
_lib.load().tcam_bbox_set_debug(None)
d = dbg.view(-1, 16).cpu().numpy()[:B]
print("fill us/frame: load %.1f sweeps %.1f hist+tables %.1f emit %.1f | iters %.1f" % (
    d[:, 0].mean() / 100, d[:, 1].mean() / 100, d[:, 2].mean() / 100, d[:, 4].mean() / 100,
    d[:, 3].mean()), flush=True)
