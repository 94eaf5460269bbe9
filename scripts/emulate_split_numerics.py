"""CPU emulation of two operand-splitting schemes for the MFMA convolutions (a design aid):

* x6: a = ah + am + al (three bf16 parts, exact), six cross terms of order <= 2;
* f16x3: a = s (h + l) (two fp16 parts, s a power of two), three cross terms
  (hh + hl + lh) — the same products the fp16 MFMA (bf16 rate) would form.

For every convolution of the ResNet50-TCAM forward on one bench frame (the oracle's
fp32 restatement, BN folded into the weights as the device plan does) it reports
max |emulated - fp64| / max sum_k |w x| (products exact in fp64, so this is the
representation + dropped-term error; the fp32 accumulation in the MFMA adds the same
amount to both), and the activation range (max |x|, the fraction of nonzeros below the
fp16 normal range).  Usage: python scripts/emulate_split_numerics.py [scale_log2]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle import model_ref as R  # noqa: E402


def split_bf16x3(x):
    h = x.to(torch.bfloat16).double()
    r = x - h
    m = r.to(torch.bfloat16).double()
    lo = (r - m).to(torch.bfloat16).double()
    return h, m, lo


def split_f16x2(x, s):
    y = x / s
    h = y.to(torch.float16).double()
    lo = (y - h).to(torch.float16).double()
    return h * s, lo * s


def pow2_scale(t, dims, target=2.0 ** 10):
    m = t.abs().amax(dim=dims, keepdim=True).clamp_min(1e-30)
    return torch.exp2(torch.floor(torch.log2(target / m))).reciprocal()


def main():
    act_log2 = float(sys.argv[1]) if len(sys.argv) > 1 else 0.0
    torch.set_num_threads(os.cpu_count())
    import bench
    from tcam_wsol_video_amd.models import build_r50_tcam
    x, _, _ = bench.make_clip(1, seed=1000, size=224)
    sd = {k: v.detach() for k, v in build_r50_tcam(seed=0).state_dict().items()}
    rec = []
    conv = F.conv2d

    def hook(inp, w, b=None, stride=1, padding=0, *a, **k):
        rec.append((inp.detach().clone(), w.detach().clone(), stride, padding))
        return conv(inp, w, b, stride, padding, *a, **k)

    F.conv2d = hook
    try:
        R.tcam_forward(sd, x)
    finally:
        F.conv2d = conv
    sa = 2.0 ** act_log2
    print(f"{'layer':>5} {'shape':>24} {'max|x|':>10} {'sub16':>7} {'x6':>9} {'f16x3':>9}")
    worst = [0.0, 0.0]
    for i, (inp, w, st, pad) in enumerate(rec):
        xd, wd = inp.double(), w.double()
        ref = conv(xd, wd, None, st, pad)
        absd = conv(xd.abs(), wd.abs(), None, st, pad)
        den = absd.max().item()
        xa, wa = split_bf16x3(xd), split_bf16x3(wd)
        terms = [(2, 0), (0, 2), (1, 1), (1, 0), (0, 1), (0, 0)]
        y6 = sum(conv(xa[p], wa[q], None, st, pad) for p, q in terms)
        sw = pow2_scale(wd, (1, 2, 3))
        xh, xl = split_f16x2(xd, sa)
        wh, wl = split_f16x2(wd, sw)
        y3 = conv(xh, wl, None, st, pad) + conv(xl, wh, None, st, pad) + \
            conv(xh, wh, None, st, pad)
        e6 = (y6 - ref).abs().max().item() / den
        e3 = (y3 - ref).abs().max().item() / den
        nz = inp[inp != 0].abs() / sa
        sub = (nz < 2.0 ** -14).double().mean().item() if nz.numel() else 0.0
        worst = [max(worst[0], e6), max(worst[1], e3)]
        print(f"{i:5d} {str(tuple(inp.shape[1:]))+'x'+str(w.shape[0]):>24} "
              f"{inp.abs().max().item():10.3g} {sub:7.4f} {e6:9.2e} {e3:9.2e}", flush=True)
    print(f"worst x6 {worst[0]:.2e}  f16x3 {worst[1]:.2e}  (activation scale 2^{act_log2:g})")


if __name__ == "__main__":
    main()
