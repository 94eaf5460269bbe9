"""A/B timing of tcam_conv2d_x6 debug variants in one process (tuning aid).

For every ResNet50-TCAM layer in ONLY (default: the residual 1x1 layers), times the
auto-chosen tile (or TILES=a,b,..) with tcam_conv_x6_debug(0) and with each flag set in
AB (comma list, e.g. AB=16), interleaved over ROUNDS rounds so both see the same clock
and thermal state (cdna_hip_programming.md §5.4 rule 24).  Reports the median and min
TF per variant.  Outputs of the A variant are checked against the fp64 reference.
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tune_conv_x6 import B, from_s3, pack, reference, run, to_s3  # noqa: E402
from tune_conv import SHAPES  # noqa: E402
from tcam_wsol_video_amd import _lib  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    only = os.environ.get("ONLY", "l1.c3,l2.c3,l3.c3,l4.c3,l1.c3ds,l4.c3ds").split(",")
    flags = [0] + [int(x) for x in os.environ.get("AB", "16").split(",")]
    tiles = [int(x) for x in os.environ["TILES"].split(",")] if os.environ.get("TILES") else [-1]
    rounds = int(os.environ.get("ROUNDS", "5"))
    reps = int(os.environ.get("REPS", "5"))
    for name, specs, cout, k, pad, ho, wo in SHAPES:
        if name not in only:
            continue
        torch.manual_seed(0)
        xs32 = [torch.randn(B, h, w, c, device=dev) for c, h, w, s, u in specs]
        xs = [to_s3(x) for x in xs32]
        ws = [torch.randn(cout, c, k, k, device=dev) / (c * k * k) ** 0.5 for c, *_ in specs]
        bias = torch.randn(cout, device=dev) * 0.1
        wt = pack(lib, ws)
        res32 = torch.randn(B, ho, wo, cout, device=dev) if name.endswith("c3") else None
        res = to_s3(res32) if res32 is not None else None
        out = torch.empty(B, ho, wo, cout // 8, 3, 8, device=dev, dtype=torch.bfloat16)
        ref, scale = reference(xs32, specs, ws, bias, k, pad, ho, wo, res32)
        kdim = sum(c for c, *_ in specs) * k * k
        flops = 2.0 * cout * kdim * B * ho * wo
        times = {}
        for t in tiles:
            lib.tcam_conv_x6_force_tile(t)
            for f in flags:
                lib.tcam_conv_x6_debug(f)
                out.zero_()
                run(lib, xs, specs, wt, bias, cout, ho, wo, k, pad, out, res)
                torch.cuda.synchronize()
                if not f & 8:
                    e = (from_s3(out).double() - ref).abs().max().item() / scale
                    if e > 2e-6:
                        print(f"  {name} tile {t} dbg {f}: rel err {e:.1e} ** WRONG **", flush=True)
        for _ in range(rounds):
            for t in tiles:
                lib.tcam_conv_x6_force_tile(t)
                for f in flags:
                    lib.tcam_conv_x6_debug(f)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(reps):
                        run(lib, xs, specs, wt, bias, cout, ho, wo, k, pad, out, res)
                    e1.record()
                    torch.cuda.synchronize()
                    times.setdefault((t, f), []).append(e0.elapsed_time(e1) / reps)
        lib.tcam_conv_x6_debug(0)
        lib.tcam_conv_x6_force_tile(-1)
        parts = []
        for (t, f), v in sorted(times.items()):
            parts.append(f"t{t}/d{f}: med {flops / statistics.median(v) / 1e9:6.1f} "
                         f"max {flops / min(v) / 1e9:6.1f} TF")
        print(f"{name:8s} " + " | ".join(parts), flush=True)


if __name__ == "__main__":
    main()
