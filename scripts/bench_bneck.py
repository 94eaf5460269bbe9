"""Time of ResNet50 layer 1 at the bench geometry (32 x 56^2): the three fused bottleneck
launches against the nine unfused f16x3 convs (same folded weights), interleaved rounds."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tcam_wsol_video_amd import ops  # noqa: E402
from tcam_wsol_video_amd.models import _ResNetPlanX6, build_r50_tcam  # noqa: E402


def main():
    dev = torch.device("cuda")
    B = int(os.environ.get("FRAMES", "32"))
    plan = _ResNetPlanX6(build_r50_tcam(seed=0).encoder, dev, "f16x3")
    g = torch.Generator().manual_seed(0)
    x0 = ops.s3_from_nchw(torch.randn(B, 64, 56, 56, generator=g).relu().to(dev), fmt="f16x3")

    def run(fused):
        f = x0
        for c1, c2, c3, has_ds, _ in plan.layers[0]:
            if fused:
                f = ops.bottleneck_f16x3(f, c1, c2, c3, has_ds)
                continue
            H, W = f.shape[1], f.shape[2]
            h1 = ops.conv2d_x6([ops.ConvSrc(f)], c1.wt, c1.bias, 64, H, W, 1, 0, True,
                               wscale=c1.wscale)
            h2 = ops.conv2d_x6([ops.ConvSrc(h1)], c2.wt, c2.bias, 64, H, W, 3, 1, True,
                               wscale=c2.wscale)
            if has_ds:
                f = ops.conv2d_x6([ops.ConvSrc(h2), ops.ConvSrc(f)], c3.wt, c3.bias, 256, H, W,
                                  1, 0, True, wscale=c3.wscale)
            else:
                f = ops.conv2d_x6([ops.ConvSrc(h2)], c3.wt, c3.bias, 256, H, W, 1, 0, True,
                                  residual=f, wscale=c3.wscale)
        return f
    times = {False: [], True: []}
    for v in (False, True):
        run(v)
    torch.cuda.synchronize()
    for _ in range(7):
        for v in (False, True):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    ops.check_f16_overflow(dev)
    for v in (False, True):
        print(f"layer1 {'fused  ' if v else 'unfused'} median {statistics.median(times[v]):.4f} ms"
              f"  min {min(times[v]):.4f} ms", flush=True)


if __name__ == "__main__" and not os.environ.get("PHASES"):
    main()


def phases():
    """Per-block phase times of the fused kernel (s_memrealtime stamps), block 1 of layer 1."""
    import numpy as np
    from tcam_wsol_video_amd import _lib
    dev = torch.device("cuda")
    B = int(os.environ.get("FRAMES", "32"))
    plan = _ResNetPlanX6(build_r50_tcam(seed=0).encoder, dev, "f16x3")
    g = torch.Generator().manual_seed(0)
    x = ops.s3_from_nchw(torch.randn(B, 256, 56, 56, generator=g).relu().to(dev), fmt="f16x3")
    c1, c2, c3, has_ds, _ = plan.layers[0][1]
    for _ in range(3):
        ops.bottleneck_f16x3(x, c1, c2, c3, has_ds)
    dbg = torch.zeros(4 * B * 64, dtype=torch.int64, device=dev)
    lib = _lib.load()
    lib.tcam_bottleneck_set_debug(dbg.data_ptr())
    ops.bottleneck_f16x3(x, c1, c2, c3, has_ds)
    torch.cuda.synchronize()
    lib.tcam_bottleneck_set_debug(None)
    d = dbg.cpu().numpy().reshape(-1, 4)
    d = d[d[:, 0] > 0].astype(np.float64) / 100.0   # us
    t0 = d[:, 0].min()
    print(f"blocks {len(d)}, launch span {d[:, 3].max() - t0:.1f} us")
    print(f"per block: conv1 {np.median(d[:, 1] - d[:, 0]):.1f} us, conv2 "
          f"{np.median(d[:, 2] - d[:, 1]):.1f}, conv3+epilogue {np.median(d[:, 3] - d[:, 2]):.1f}"
          f", total {np.median(d[:, 3] - d[:, 0]):.1f}")
    st = np.sort(d[:, 0] - t0)
    print("start times (us) quantiles:", [round(float(v), 1) for v in np.quantile(st, [0, .25, .5, .75, 1])])


if __name__ == "__main__" and os.environ.get("PHASES"):
    phases()
