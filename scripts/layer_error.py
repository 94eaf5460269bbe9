"""Per-layer error of the GPU convolutions against fp64 on the bench's own operands.

Every convolution of the ResNet50-TCAM forward on one frame of the bench clip (inputs
and weights captured from the oracle's fp32 forward, oracle/model_ref.py) is run through
tcam_conv2d_x6 (S3) and tcam_conv2d_f16x3 (S2) on the device; the table gives, per layer,
max |out - fp64| / max sum_k |w x| (the scale an fp32 FMA chain's error is proportional
to; the MI355X fp32 MFMA measures 0.75-3.5e-7 on it).

    python scripts/layer_error.py > profiles/round3_f16x3_layer_error.txt
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model_ref as R  # noqa: E402
from tcam_wsol_video_amd import ops  # noqa: E402
from tcam_wsol_video_amd.ops import ConvSrc  # noqa: E402


def main():
    import bench
    from tcam_wsol_video_amd.models import build_r50_tcam
    dev = torch.device("cuda:0")
    x, _, _ = bench.make_clip(1, seed=1000, size=224)
    sd = {k: v.detach() for k, v in build_r50_tcam(seed=0).state_dict().items()}
    rec, conv = [], F.conv2d

    def hook(inp, w, b=None, stride=1, padding=0, *a, **k):
        rec.append((inp.detach().clone(), w.detach().clone(), stride, padding))
        return conv(inp, w, b, stride, padding, *a, **k)

    F.conv2d = hook
    try:
        R.tcam_forward(sd, x)
    finally:
        F.conv2d = conv
    print("| # | input | Cout | k | max|x| | x6 err / sum|wx| | f16x3 err / sum|wx| |")
    print("|---|---|---|---|---|---|---|")
    worst = {"x6": 0.0, "f16x3": 0.0}
    for i, (inp, w, st, pad) in enumerate(rec):
        if w.shape[0] % 8:
            continue    # the 2-channel segmentation head runs its own fp32 kernel
        cin = inp.shape[1]
        cpad = (cin + 7) // 8 * 8
        if cpad != cin:
            inp = torch.cat([inp, inp.new_zeros((1, cpad - cin) + tuple(inp.shape[2:]))], 1)
            w = torch.cat([w, w.new_zeros((w.shape[0], cpad - cin) + tuple(w.shape[2:]))], 1)
        ref = conv(inp.double(), w.double(), None, st, pad)
        den = conv(inp.double().abs(), w.double().abs(), None, st, pad).max().item()
        Ho, Wo = ref.shape[2:]
        k = w.shape[2]
        errs = {}
        for prec in ("x6", "f16x3"):
            xs = ops.s3_from_nchw(inp.to(dev), fmt=prec)
            if prec == "x6":
                wt, sc = ops.pack_conv_weight_x6([w.to(dev)]), None
            else:
                wt, sc = ops.pack_conv_weight_f16([w.to(dev)])
            out = ops.conv2d_x6([ConvSrc(xs, st)], wt, torch.zeros(w.shape[0], device=dev),
                                w.shape[0], Ho, Wo, k, pad, False, wscale=sc)
            got = ops.s3_to_nchw(out).cpu().double()
            errs[prec] = (got - ref).abs().max().item() / den
            worst[prec] = max(worst[prec], errs[prec])
        print(f"| {i} | {cin}x{inp.shape[2]}x{inp.shape[3]} | {w.shape[0]} | {k} | "
              f"{inp.abs().max().item():.3g} | {errs['x6']:.2e} | {errs['f16x3']:.2e} |",
              flush=True)
    ops.check_f16_overflow(dev)
    print(f"\nworst: x6 {worst['x6']:.2e}, f16x3 {worst['f16x3']:.2e} (fp32 FMA chain on "
          f"MI355X: 0.75-3.5e-7)")


if __name__ == "__main__":
    main()
