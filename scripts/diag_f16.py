"""f16x3 conv error vs fp64 on inputs with / without fp16-subnormal lo parts (diagnostic)."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcam_wsol_video_amd import ops  # noqa: E402
from tcam_wsol_video_amd.ops import ConvSrc  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
for name, scale, off in (("randn", 1.0, 0.0), ("big", 1.0, 4.0), ("small", 1e-3, 0.0)):
    x = torch.randn(2, 64, 14, 14, generator=g) * scale + off * torch.sign(torch.randn(2, 64, 14, 14, generator=g))
    w = torch.randn(64, 64, 1, 1, generator=g) / 8
    ref = F.conv2d(x.double(), w.double())
    absd = F.conv2d(x.double().abs(), w.double().abs())
    wt, sc = ops.pack_conv_weight_f16([w.to(dev)])
    xs = ops.s3_from_nchw(x.to(dev), fmt="f16x3")
    xr = ops.s3_to_nchw(xs).cpu().double()
    rep = ((xr - x.double()).abs() / x.double().abs().clamp_min(1e-30)).max().item()
    out = ops.conv2d_x6([ConvSrc(xs)], wt, torch.zeros(64, device=dev), 64, 14, 14, 1, 0, False,
                        wscale=sc)
    got = ops.s3_to_nchw(out).cpu().double()
    err = ((got - ref).abs() / absd).max().item()
    # emulation with exact products of the stored parts
    h = xs[..., 0, :].float().reshape(2, 14, 14, 64).permute(0, 3, 1, 2).double().cpu()
    l = xs[..., 1, :].float().reshape(2, 14, 14, 64).permute(0, 3, 1, 2).double().cpu()
    wtd = wt.float().cpu().double()
    print(f"{name}: input repr rel {rep:.2e}  conv err/sum|wx| {err:.2e}  "
          f"lo==0 frac {(l == 0).double().mean().item():.3f}", flush=True)
    # the same conv with the lo parts dropped: what a denormal flush would give
    out2 = F.conv2d(h, w.double())
    print(f"   hi-only err/sum|wx| {((out2 - ref).abs() / absd).max().item():.2e}")
