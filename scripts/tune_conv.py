"""Per-shape tile/stage sweep of tcam_conv2d on the GPU (tuning aid).

For every distinct convolution of ResNet50-TCAM at 224x224, batch 32, time
every tile configuration (tcam_conv_force_tile) with HIP events, interleaved
in one process, and print the best per shape.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcam_wsol_video_amd import _lib, ops  # noqa: E402
from tcam_wsol_video_amd.ops import ConvSrc  # noqa: E402

B = int(os.environ.get("B", "32"))
# (name, [(C, H, W, stride, up2)], Cout, k, pad, Hout, Wout)
SHAPES = [
    ("stem", [(3, 224, 224, 2, 0)], 64, 7, 3, 112, 112),
    ("l1.c1", [(256, 56, 56, 1, 0)], 64, 1, 0, 56, 56),
    ("l1.c2", [(64, 56, 56, 1, 0)], 64, 3, 1, 56, 56),
    ("l1.c3", [(64, 56, 56, 1, 0)], 256, 1, 0, 56, 56),
    ("l1.c3ds", [(64, 56, 56, 1, 0), (64, 56, 56, 1, 0)], 256, 1, 0, 56, 56),
    ("l2.c1", [(512, 28, 28, 1, 0)], 128, 1, 0, 28, 28),
    ("l2.c2", [(128, 28, 28, 1, 0)], 128, 3, 1, 28, 28),
    ("l2.c3", [(128, 28, 28, 1, 0)], 512, 1, 0, 28, 28),
    ("l3.c1", [(1024, 28, 28, 1, 0)], 256, 1, 0, 28, 28),
    ("l3.c2", [(256, 28, 28, 1, 0)], 256, 3, 1, 28, 28),
    ("l3.c3", [(256, 28, 28, 1, 0)], 1024, 1, 0, 28, 28),
    ("l4.c1", [(2048, 28, 28, 1, 0)], 512, 1, 0, 28, 28),
    ("l4.c2", [(512, 28, 28, 1, 0)], 512, 3, 1, 28, 28),
    ("l4.c3", [(512, 28, 28, 1, 0)], 2048, 1, 0, 28, 28),
    ("l4.c3ds", [(512, 28, 28, 1, 0), (1024, 28, 28, 1, 0)], 2048, 1, 0, 28, 28),
    ("d0.c1", [(2048, 28, 28, 1, 0), (1024, 28, 28, 1, 0)], 256, 3, 1, 28, 28),
    ("d1.c1", [(256, 28, 28, 1, 0), (512, 28, 28, 1, 0)], 128, 3, 1, 28, 28),
    ("d2.c1", [(128, 28, 28, 1, 1), (256, 56, 56, 1, 0)], 64, 3, 1, 56, 56),
    ("d3.c1", [(64, 56, 56, 1, 1), (64, 112, 112, 1, 0)], 32, 3, 1, 112, 112),
    ("d3.c2", [(32, 112, 112, 1, 0)], 32, 3, 1, 112, 112),
    ("d4.c1", [(32, 112, 112, 1, 1)], 16, 3, 1, 224, 224),
    ("d4.c2", [(16, 224, 224, 1, 0)], 16, 3, 1, 224, 224),
]

# SPG-InceptionV3-TCAM at 299^2 (the 39 x 39 stage; B = 8 frames per shard): the launches that
# take the time in scripts/layer_times.py inceptionv3 (k: int or (kh, kw), pad likewise)
INC_SHAPES = [
    ("i.h1", [(1024, 39, 39, 1, 0)], 1024, 3, 1, 39, 39),
    ("i.h0", [(768, 39, 39, 1, 0)], 1024, 3, 1, 39, 39),
    ("i.d0", [(1024, 39, 39, 1, 0), (768, 39, 39, 1, 0)], 256, 3, 1, 39, 39),
    ("i.d1", [(256, 39, 39, 1, 0), (288, 39, 39, 1, 0)], 128, 3, 1, 39, 39),
    ("i.b3", [(288, 39, 39, 1, 0)], 384, 3, 1, 39, 39),
    ("i.7a", [(192, 39, 39, 1, 0)], 192, (1, 7), (0, 3), 39, 39),
    ("i.7b", [(160, 39, 39, 1, 0)], 160, (7, 1), (3, 0), 39, 39),
    ("i.7c", [(160, 39, 39, 1, 0)], 192, (1, 7), (0, 3), 39, 39),
    ("i.1x", [(768, 39, 39, 1, 0)], 192, 1, 0, 39, 39),
]
if os.environ.get("SHAPESET") == "inception":
    SHAPES = INC_SHAPES


def main():
    lib = _lib.load()
    ntile = lib.tcam_conv_force_tile(-1)
    dev = torch.device("cuda")
    reps = int(os.environ.get("REPS", "5"))
    only = os.environ.get("ONLY")
    for name, srcs, cout, k, pad, ho, wo in SHAPES:
        if only and name not in only.split(","):
            continue
        xs = [ConvSrc(torch.randn(B, c, h, w, device=dev), s, u) for c, h, w, s, u in srcs]
        ws = [torch.randn(cout, c, k, k, device=dev) * 0.01 for c, *_ in srcs]
        wt = ops.pack_conv_weight(ws)
        bias = torch.zeros(cout, device=dev)
        flops = 2.0 * cout * wt.shape[0] * B * ho * wo
        kdim = sum(c for c, *_ in srcs) * k * k
        flops = 2.0 * cout * kdim * B * ho * wo
        res = {}
        for rnd in range(2):
            tiles = [int(t) for t in os.environ["TILES"].split(",")] if os.environ.get("TILES") \
                else [-1] + list(range(ntile))
            for t in tiles:
                lib.tcam_conv_force_tile(t)
                ops.conv2d(xs, wt, bias, cout, ho, wo, k, pad, True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    ops.conv2d(xs, wt, bias, cout, ho, wo, k, pad, True)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                res[t] = min(res.get(t, 1e9), ms)
        lib.tcam_conv_force_tile(-1)
        best = min((v, t) for t, v in res.items() if t >= 0)
        line = " ".join(f"{t}:{flops / res[t] / 1e9:5.1f}" for t in sorted(res) if t >= 0)
        auto = f"{flops / res[-1] / 1e9:6.1f}" if -1 in res else "  -   "
        print(f"{name:8s} auto {auto} TF  best t{best[1]} "
              f"{flops / best[0] / 1e9:6.1f} TF | {line}", flush=True)


if __name__ == "__main__":
    main()
