"""Per-shape tile sweep + accuracy check of tcam_conv2d_x6 (tuning aid).

Shapes: ResNet50-TCAM at 224x224, batch B (tune_conv.SHAPES; the stem reads
the image padded to 8 channels).  Accuracy: max |out - fp64 conv| / max
sum_k |w x| (the scale an fp32 FMA chain's error is proportional to).
"""
import ctypes as C
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tcam_wsol_video_amd import _lib, ops  # noqa: E402
from tcam_wsol_video_amd._lib import check, tcam_conv_src  # noqa: E402
from tune_conv import SHAPES  # noqa: E402

B = int(os.environ.get("B", "32"))
PREC = os.environ.get("PREC", "x6")   # x6 (S3, bf16 x3) or f16x3 (S2, fp16 x2)
_WSC = {}


def split3(x):
    hi = x.to(torch.bfloat16)
    r = x - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return hi, mid, lo


def to_s3(x):  # (B, H, W, C) fp32 -> (B, H, W, C/8, 3, 8) bf16 (S2 under PREC=f16x3)
    if PREC == "f16x3":
        return ops.s3_from_nchw(x.permute(0, 3, 1, 2).contiguous(), fmt="f16x3")
    b, h, w, c = x.shape
    parts = [t.reshape(b, h, w, c // 8, 8) for t in split3(x)]
    return torch.stack(parts, dim=4).contiguous()


def from_s3(s):
    if ops.is_s2(s):
        return ops.s3_to_nchw(s).permute(0, 2, 3, 1)
    v = (s[..., 0, :].float() + s[..., 1, :].float()) + s[..., 2, :].float()
    return v.reshape(*s.shape[:3], -1)


def pack(lib, ws):
    if PREC == "f16x3":
        wt, sc = ops.pack_conv_weight_f16(ws)
        _WSC[wt.data_ptr()] = sc
        return wt
    w = torch.cat(ws, dim=1)
    cout, ctot, kh, kw = w.shape
    k = ctot * kh * kw
    kp, mp = C.c_int(), C.c_int()
    check(lib.tcam_conv_x6_weight_dims(k, cout, C.byref(kp), C.byref(mp)), "dims")
    kp, mp = kp.value, mp.value
    wt = torch.zeros((kp, mp), dtype=torch.float32, device=w.device)
    wt[:k, :cout] = w.permute(2, 3, 1, 0).reshape(k, cout)
    parts = [t.view(kp // 32, 4, 8, mp).permute(0, 1, 3, 2) for t in split3(wt)]
    return torch.stack(parts, dim=2).contiguous()


def run(lib, xs, specs, wt, bias, cout, ho, wo, k, pad, out, res=None):
    srcs = [ops.ConvSrc(x, s, bool(u)) for x, (c, h, w, s, u) in zip(xs, specs)]
    ops.conv2d_x6(srcs, wt, bias, cout, ho, wo, k, pad, True, residual=res, out=out,
                  wscale=_WSC.get(wt.data_ptr()))


def reference(xs32, specs, ws, bias, k, pad, ho, wo, res=None):
    outs, absd = 0, 0
    for x, (c, h, w, s, u), wgt in zip(xs32, specs, ws):
        t = x.permute(0, 3, 1, 2).double()
        if u:
            t = F.interpolate(t, scale_factor=2, mode="nearest")
        outs = outs + F.conv2d(t, wgt.double(), stride=s, padding=pad)[:, :, :ho, :wo]
        absd = absd + F.conv2d(t.abs(), wgt.double().abs(), stride=s, padding=pad)[:, :, :ho, :wo]
    outs = outs + bias.double()[None, :, None, None]
    if res is not None:
        outs = outs + res.permute(0, 3, 1, 2).double()
    return torch.relu(outs).permute(0, 2, 3, 1), absd.max().item()


def main():
    lib = _lib.load()
    ntile = lib.tcam_conv_x6_force_tile(-1)
    lib.tcam_conv_x6_force_streamk(int(os.environ.get("SK", "-1")))
    dbg = int(os.environ.get("DBG", "0"))
    dev = torch.device("cuda")
    reps = int(os.environ.get("REPS", "5"))
    only = os.environ.get("ONLY")
    tot = {}
    for name, specs, cout, k, pad, ho, wo in SHAPES:
        if only and name not in only.split(","):
            continue
        if name == "stem":
            specs = [(8, 224, 224, 2, 0)]
        torch.manual_seed(0)
        xs32 = [torch.randn(B, h, w, c, device=dev) for c, h, w, s, u in specs]
        if name == "stem":
            xs32[0][..., 3:] = 0
        xs = [to_s3(x) for x in xs32]
        kh, kw = (k, k) if isinstance(k, int) else k
        ws = [torch.randn(cout, c, kh, kw, device=dev) / (c * kh * kw) ** 0.5 for c, *_ in specs]
        bias = torch.randn(cout, device=dev) * 0.1
        wt = pack(lib, ws)
        res32 = torch.randn(B, ho, wo, cout, device=dev) if name.endswith("c3") else None
        res = to_s3(res32) if res32 is not None else None
        out = (ops.s2_empty if PREC == "f16x3" else ops.s3_empty)(B, ho, wo, cout, dev)
        run(lib, xs, specs, wt, bias, cout, ho, wo, k, pad, out, res)
        lib.tcam_conv_x6_debug(dbg)
        ref, scale = reference(xs32, specs, ws, bias, k, pad, ho, wo, res32)
        err = (from_s3(out).double() - ref).abs().max().item()
        kdim = sum(c for c, *_ in specs) * kh * kw
        flops = 2.0 * cout * kdim * B * ho * wo
        res_t, errs = {}, {}
        for rnd in range(2):
            tl = os.environ.get("TILES", "")
            tiles = [-1] if tl == "auto" else ([int(x) for x in tl.split(",")] if tl else
                                               [-1] + list(range(ntile)))
            for t in tiles:
                lib.tcam_conv_x6_force_tile(t)
                out.zero_()
                run(lib, xs, specs, wt, bias, cout, ho, wo, k, pad, out, res)
                if rnd == 0 and not dbg:   # every tile's output vs the fp64 reference
                    et = (from_s3(out).double() - ref).abs().max().item() / scale
                    errs[t] = et
                    if et > 2e-6:
                        print(f"  {name} tile {t}: rel err {et:.1e}  ** WRONG **", flush=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    run(lib, xs, specs, wt, bias, cout, ho, wo, k, pad, out, res)
                e1.record()
                torch.cuda.synchronize()
                res_t[t] = min(res_t.get(t, 1e9), e0.elapsed_time(e1) / reps)
        lib.tcam_conv_x6_force_tile(-1)
        cand = [(v, t) for t, v in res_t.items() if t >= 0]
        best = min(cand) if cand else (res_t[-1], -1)
        tot[name] = (res_t.get(-1, best[0]), best[0])
        line = " ".join(f"{t}:{flops / res_t[t] / 1e9:5.1f}" for t in sorted(res_t) if t >= 0)
        print(f"{name:8s} err {err:.1e} rel {err / scale:.1e} auto {flops / res_t.get(-1, best[0]) / 1e9:6.1f}"
              f" TF best t{best[1]} {flops / best[0] / 1e9:6.1f} TF | {line}", flush=True)
    print("sum ms auto %.3f best %.3f" % (sum(a for a, _ in tot.values()),
                                          sum(b for _, b in tot.values())))


if __name__ == "__main__":
    main()
