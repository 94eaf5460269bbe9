"""Diagnostic: the fill stage's outputs (psi, level tables) of each fill variant on the same
CAMs, read from the bbox workspace (tcam_bbox_levels with the per-level CCL sweep)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcam_wsol_video_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda")
    u8 = torch.from_numpy(np.load(sys.argv[1])).to(dev)
    B, H, W = u8.shape
    lib = _lib.load()
    nws = lib.tcam_bbox_ws_bytes(B, H, W)
    lib.tcam_bbox_level_variant(1)
    outs = {}
    for v in (2, 0):
        lib.tcam_bbox_fill_variant(v)
        if v == 0:
            lib.tcam_bbox_fill_variant(100 + int(os.environ.get("FILL_WAVES", "16")))
            lib.tcam_bbox_fill_variant(1000 + int(os.environ.get("FILL_MAXIT", "0")))
        ws = torch.zeros(nws, dtype=torch.uint8, device=dev)
        boxes = torch.zeros(B, 256, 4, dtype=torch.int32, device=dev)
        vmax = torch.zeros(B, dtype=torch.int32, device=dev)
        rc = lib.tcam_bbox_levels(u8.data_ptr(), boxes.data_ptr(), vmax.data_ptr(),
                                  ws.data_ptr(), B, H, W, None)
        torch.cuda.synchronize()
        assert rc == 0, rc
        w = ws.cpu().numpy()
        off = (B * H * W + 15) // 16 * 16
        psi = w[:B * H * W].reshape(B, H, W)
        canon = w[off:off + B * 256 * 4].view(np.int32).reshape(B, 256)
        lev = w[off + B * 256 * 4:off + B * 512 * 4].view(np.int32).reshape(B, 256)
        nlev = w[off + B * 512 * 4:off + B * 512 * 4 + B * 4].view(np.int32)
        outs[v] = (psi, canon, lev, nlev, vmax.cpu().numpy())
    lib.tcam_bbox_fill_variant(0)
    lib.tcam_bbox_level_variant(0)
    lib.tcam_bbox_fill_variant(1000)
    lib.tcam_bbox_fill_variant(116)
    if len(sys.argv) > 2:
        np.savez_compressed(sys.argv[2], psi2=outs[2][0], psi0=outs[0][0])
    a, b = outs[2], outs[0]
    for f in range(B):
        vm = a[4][f]
        dpsi = np.argwhere(a[0][f] != b[0][f])
        dcan = np.nonzero(a[1][f][:vm] != b[1][f][:vm])[0]
        n = a[3][f]
        dlev = np.nonzero(a[2][f][:n] != b[2][f][:n])[0]
        if len(dpsi) or len(dcan) or len(dlev) or a[3][f] != b[3][f] or a[4][f] != b[4][f]:
            print(f"frame {f}: vmax {a[4][f]}/{b[4][f]} nlev {a[3][f]}/{b[3][f]} psi diffs "
                  f"{len(dpsi)} first {dpsi[:3].tolist()} vals "
                  f"{[(int(a[0][f][y, x]), int(b[0][f][y, x])) for y, x in dpsi[:3]]} "
                  f"canon diffs {dcan[:5].tolist()} lev diffs {dlev[:5].tolist()}", flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
