"""A/B timing of the f16x3 convolution (tcam_conv2d_f16x3) on ResNet50-TCAM layers, one
process, variants interleaved over ROUNDS rounds (same clock / thermal state).

Variants (VARIANTS, comma list of name=spec): spec is "t<id>" (forced tile), "d<flags>"
(tcam_conv_x6_debug flags: 8 = no epilogue traffic, 16 = no residual prefetch), "nores"
(the same layer without its residual), "s<grid>" (stream-K over a forced grid of <grid>
blocks, tcam_conv_x6_force_streamk), joined with '+'; "auto" = the chooser.
    ONLY=l4.c3,l3.c3 VARIANTS=auto,noepi=d8,nores python scripts/ab_f16.py
Prints per layer and variant the median / min time and TF (algorithmic 2*M*K*N).
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tune_conv import SHAPES  # noqa: E402
from tcam_wsol_video_amd import _lib, ops  # noqa: E402
from tcam_wsol_video_amd.ops import ConvSrc  # noqa: E402

B = int(os.environ.get("FRAMES", "32"))
FMT = os.environ.get("FMT", "f16x3")   # f16x3 | amp (one fp16 part, S1 activations)


def parse(spec):
    tile, dbg, nores, sk = -1, 0, False, -1
    for part in spec.split("+"):
        if part == "auto":
            continue
        if part == "nores":
            nores = True
        elif part.startswith("t"):
            tile = int(part[1:])
        elif part.startswith("d"):
            dbg = int(part[1:])
        elif part.startswith("s"):
            sk = int(part[1:])
    return tile, dbg, nores, sk


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    only = os.environ.get("ONLY", "l4.c3,l3.c3").split(",")
    variants = []
    for v in os.environ.get("VARIANTS", "auto,noepi=d8,nores").split(","):
        name, _, spec = v.partition("=")
        variants.append((name, parse(spec or name)))
    rounds = int(os.environ.get("ROUNDS", "7"))
    reps = int(os.environ.get("REPS", "10"))
    for name, specs, cout, k, pad, ho, wo in SHAPES:
        if name not in only:
            continue
        g = torch.Generator().manual_seed(0)
        xs = [ops.s3_from_nchw(torch.randn(B, c, h, w, generator=g).to(dev), fmt=FMT)
              for c, h, w, s, u in specs]
        ws = [(torch.randn(cout, c, k, k, generator=g) / (c * k * k) ** 0.5).to(dev)
              for c, *_ in specs]
        if FMT == "amp":
            wt, wsc = ops.pack_conv_weight_h1(ws), None
        else:
            wt, wsc = ops.pack_conv_weight_f16(ws)
        bias = (torch.randn(cout, generator=g) * 0.1).to(dev)
        res = None
        if name.endswith("c3"):
            res = ops.s3_from_nchw(torch.randn(B, cout, ho, wo, generator=g).to(dev),
                                   fmt=FMT)
        srcs = [ConvSrc(x, s, bool(u)) for x, (c, h, w, s, u) in zip(xs, specs)]
        kdim = sum(c for c, *_ in specs) * k * k
        flops = 2.0 * cout * kdim * B * ho * wo
        times = {vn: [] for vn, _ in variants}

        def run(v):
            tile, dbg, nores, sk = v
            lib.tcam_conv_x6_force_tile(tile)
            lib.tcam_conv_x6_debug(dbg)
            lib.tcam_conv_x6_force_streamk(sk)
            try:
                return ops.conv2d_x6(srcs, wt, bias, cout, ho, wo, k, pad, True,
                                     residual=None if nores else res, wscale=wsc)
            finally:
                lib.tcam_conv_x6_force_tile(-1)
                lib.tcam_conv_x6_debug(0)
                lib.tcam_conv_x6_force_streamk(-1)
        for vn, v in variants:   # warm
            run(v)
        torch.cuda.synchronize()
        for _ in range(rounds):
            for vn, v in variants:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                times[vn].append(e0.elapsed_time(e1) / reps)
        ops.check_f16_overflow(dev)
        for vn, _ in variants:
            med, mn = statistics.median(times[vn]), min(times[vn])
            print(f"{name:8s} {vn:12s} median {med:.4f} ms ({flops / med / 1e9:6.1f} TF)  "
                  f"min {mn:.4f} ms ({flops / mn / 1e9:6.1f} TF)", flush=True)


if __name__ == "__main__":
    main()
