"""Per-phase time of the level sweep on the bench's CAMs (s_memrealtime, 100 MHz ticks):
TCAM_LEVEL_VARIANT=0 the sorted-list sweep (default), 2 the incremental sweep."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from tcam_wsol_video_amd import ops, _lib  # noqa: E402
from tcam_wsol_video_amd.models import build_r50_tcam  # noqa: E402

dev = torch.device("cuda")
_lib.load().tcam_bbox_level_variant(int(os.environ.get("TCAM_LEVEL_VARIANT", "0")))
model = build_r50_tcam(seed=0).to(dev)
x, targets, gt = bench.make_clip(32, seed=1000)
with torch.no_grad():
    model(x.to(dev), want_fcams=False)
u8 = model.cam_u8
for _ in range(3):
    ops.bbox_levels(u8)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    ops.bbox_levels(u8)
e1.record()
torch.cuda.synchronize()
print(f"bbox_levels {e0.elapsed_time(e1) / 10:.3f} ms per clip")
B = u8.shape[0]
dbg = torch.zeros(8 * B * 16, dtype=torch.int64, device=dev)
_lib.load().tcam_bbox_set_inc_debug(dbg.data_ptr())
ops.bbox_levels(u8)
torch.cuda.synchronize()
_lib.load().tcam_bbox_set_inc_debug(None)
d = dbg.cpu().numpy().reshape(-1, 16)
nwg = int((d[:, 8] > 0).sum())
d = d[:nwg]
names = (["clear", "slice+activate", "unite", "handover", "key+area+box", "compress+max",
          "reduce", "box"] if os.environ.get("TCAM_LEVEL_VARIANT", "0") == "0" else
         ["threshold+list", "activate", "unite", "handover", "key+area", "compress+max", "reduce",
          "bbox"])
tot = d[:, :8].sum()
print(f"{nwg} workgroups, levels per WG mean {d[:, 8].mean():.1f}, max WG time {d[:, :8].sum(1).max() / 100:.0f} us")
print(f"levels with a full bbox scan / compression pass {d[:, 9].sum() / d[:, 8].sum():.3f}, "
      f"with a full winner pass "
      f"{d[:, 10].sum() / d[:, 8].sum():.3f}")
for k, n in enumerate(names):
    print(f"  {n:16s} {100 * d[:, k].sum() / tot:5.1f} %  mean/level {d[:, k].sum() / d[:, 8].sum() / 100:.2f} us")
