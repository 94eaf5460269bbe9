"""Torch-tensor wrappers over the C ABI (include/tcam_hip.h).

PyTorch is plumbing here: it owns device memory and the current HIP stream;
every op below launches a hand-written gfx950 kernel from libtcam_hip.so and
refuses CPU tensors (no fallback path exists).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import check, tcam_conv_dst, tcam_conv_prob, tcam_conv_src


# Optional launch timer (bench.py's live roofline measurement): a list that
# receives (kind, algorithmic_flops, start_event, end_event) per conv launch,
# recorded on the stream the kernel is launched on (torch's current stream).
_TIMER = None


_EVENT_POOL: list = []
_EVENT_NEXT = 0


def set_launch_timer(timer: Optional[list], reserve: int = 0) -> None:
    """Start (a list) or stop (None) per-launch timing.  Events come from a pool
    that is reused from the start at every ``set_launch_timer(list)``; ``reserve``
    creates that many launches' events up front (outside a timed region).  The
    HIP convolutions bind the events to their own kernel dispatches
    (``tcam_timer_arm``: no marker packets between kernels); the fp32 conv
    records them around its launch."""
    global _TIMER, _EVENT_NEXT
    _TIMER = timer
    if timer is not None:
        _EVENT_NEXT = 0
        _grow_event_pool(2 * int(reserve))


def _grow_event_pool(n: int) -> None:
    while len(_EVENT_POOL) < n:
        e = torch.cuda.Event(enable_timing=True)
        e.record()   # creates the HIP event (torch creates it lazily)
        _EVENT_POOL.append(e)


def _timer_events():
    global _EVENT_NEXT
    _grow_event_pool(_EVENT_NEXT + 2)
    e = _EVENT_POOL[_EVENT_NEXT], _EVENT_POOL[_EVENT_NEXT + 1]
    _EVENT_NEXT += 2
    return e


def _timer_arm(lib, e0, e1) -> None:
    """The next HIP conv call's kernels carry e0 (first dispatch) / e1 (every dispatch)."""
    check(lib.tcam_timer_arm(e0.cuda_event, e1.cuda_event), "tcam_timer_arm")


def _timer_disarm(lib) -> None:
    check(lib.tcam_timer_arm(None, None), "tcam_timer_arm")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _dev(*ts: Optional[torch.Tensor]) -> None:
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("tcam ops run on the GPU only (no CPU fallback); got a CPU tensor")
        if not t.is_contiguous():
            raise RuntimeError("tcam ops require contiguous tensors")


class ConvSrc:
    """One input source of :func:`conv2d` (see ``tcam_conv_src``)."""

    __slots__ = ("t", "stride", "up2")

    def __init__(self, t: torch.Tensor, stride: int = 1, up2: bool = False):
        self.t, self.stride, self.up2 = t, int(stride), bool(up2)


def conv_weight_dims(k: int, cout: int) -> Tuple[int, int]:
    """(Kpad, Mpad) of the packed weight matrix expected by :func:`conv2d`."""
    kp, mp = C.c_int(), C.c_int()
    check(_lib.load().tcam_conv_weight_dims(k, cout, C.byref(kp), C.byref(mp)),
          "tcam_conv_weight_dims")
    return kp.value, mp.value


def pack_conv_weight(ws: Sequence[torch.Tensor]) -> torch.Tensor:
    """PyTorch conv weights (Cout, C_s, KH, KW) of the sources, in source
    order, -> the tap-major, zero-padded (Kpad, Mpad) matrix of tcam_conv2d."""
    w = torch.cat(list(ws), dim=1)
    cout, ctot, kh, kw = w.shape
    k = ctot * kh * kw
    kp, mp = conv_weight_dims(k, cout)
    wt = w.permute(2, 3, 1, 0).reshape(k, cout)
    out = torch.zeros((kp, mp), dtype=torch.float32, device=w.device)
    out[:k, :cout] = wt
    return out.contiguous()


def conv2d(srcs: Sequence[ConvSrc], wt: torch.Tensor, bias: torch.Tensor, cout: int,
           hout: int, wout: int, ksize: int, pad: int, relu: bool,
           residual: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = _lib.load()
    B = srcs[0].t.shape[0]
    _dev(wt, bias, residual, *[s.t for s in srcs])
    if out is None:
        out = torch.empty((B, cout, hout, wout), device=wt.device, dtype=torch.float32)
    arr = (tcam_conv_src * len(srcs))()
    for i, s in enumerate(srcs):
        t = s.t
        assert t.dtype == torch.float32 and t.dim() == 4 and t.shape[0] == B
        arr[i] = tcam_conv_src(t.data_ptr(), t.shape[1], t.shape[2], t.shape[3], s.stride,
                               1 if s.up2 else 0)
    timer = _TIMER
    if timer is not None:
        e0, e1 = _timer_events()
        e0.record()
    check(lib.tcam_conv2d(arr, len(srcs), B, _ptr(wt), _ptr(bias), _ptr(residual), _ptr(out),
                          cout, hout, wout, ksize, ksize, pad, 1 if relu else 0, _stream()),
          "tcam_conv2d")
    if timer is not None:
        e1.record()
        kdim = wt.shape[0]
        timer.append(("conv", 2.0 * cout * kdim * B * hout * wout, e0, e1,
                      f"M{cout} K{kdim} N{B * hout * wout} k{ksize} src{len(srcs)}"))
    return out


def maxpool3x3s2(x: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    _dev(x)
    B, Cc, H, W = x.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = torch.empty((B, Cc, Ho, Wo), device=x.device, dtype=x.dtype)
    check(lib.tcam_maxpool3x3s2(_ptr(x), _ptr(out), B, Cc, H, W, Ho, Wo, _stream()),
          "tcam_maxpool3x3s2")
    return out


def up2_resize(x: torch.Tensor, size: Tuple[int, int]) -> torch.Tensor:
    lib = _lib.load()
    _dev(x)
    B, Cc, H, W = x.shape
    out = torch.empty((B, Cc, size[0], size[1]), device=x.device, dtype=x.dtype)
    check(lib.tcam_up2_resize(_ptr(x), _ptr(out), B, Cc, H, W, size[0], size[1], _stream()),
          "tcam_up2_resize")
    return out


def wgap(x: torch.Tensor, fc_w: torch.Tensor, fc_b: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    _dev(x, fc_w, fc_b)
    B, Cc, H, W = x.shape
    classes = fc_w.shape[0]
    ws = torch.empty((B, Cc), device=x.device, dtype=torch.float32)
    out = torch.empty((B, classes), device=x.device, dtype=torch.float32)
    check(lib.tcam_wgap(_ptr(x), _ptr(fc_w), _ptr(fc_b), _ptr(out), _ptr(ws), B, Cc, H * W,
                        classes, _stream()), "tcam_wgap")
    return out


def seghead_cam(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, want_fcams: bool = True,
                want_u8: bool = True, argmax: bool = False):
    """Fused SegmentationHead conv3x3 -> softmax[:,1] -> uint8 quantisation."""
    lib = _lib.load()
    _dev(x, w, b)
    B, Cin, H, W = x.shape
    fcams = torch.empty((B, 2, H, W), device=x.device) if want_fcams else None
    cam = torch.empty((B, H, W), device=x.device)
    u8 = torch.empty((B, H, W), device=x.device, dtype=torch.uint8) if want_u8 else None
    check(lib.tcam_seghead_cam(_ptr(x), _ptr(w), _ptr(b), _ptr(fcams), _ptr(cam), _ptr(u8), B,
                               Cin, H, W, 1 if argmax else 0, _stream()), "tcam_seghead_cam")
    return fcams, cam, u8


def std_cam(A: torch.Tensor, fc_w: torch.Tensor, cls: torch.Tensor, size: Tuple[int, int],
            want_u8: bool = True):
    """STD_CL CAM of the hooked layer: (low-res normalised, resized, uint8)."""
    lib = _lib.load()
    cls = cls.to(device=A.device, dtype=torch.int32).contiguous()
    _dev(A, fc_w, cls)
    if is_act(A):
        B, h, w, Cc = s3_dims(A)
        name = f"tcam_std_cam_{_lay(A)}"
        fn = getattr(lib, name)
    else:
        B, Cc, h, w = A.shape
        fn, name = lib.tcam_std_cam, "tcam_std_cam"
    low = torch.empty((B, h, w), device=A.device)
    cam = torch.empty((B, size[0], size[1]), device=A.device)
    u8 = torch.empty((B, size[0], size[1]), device=A.device, dtype=torch.uint8) if want_u8 else None
    check(fn(_ptr(A), _ptr(fc_w), _ptr(cls), _ptr(low), _ptr(cam), _ptr(u8), B, Cc, h, w,
             size[0], size[1], _stream()), name)
    return low, cam, u8


def temporal_max(cams: torch.Tensor, idx: torch.Tensor, t: float = 0.0) -> torch.Tensor:
    """out[i] = max_j renorm(cams[idx[i, j]]) (idx < 0 = absent)."""
    lib = _lib.load()
    idx = idx.to(device=cams.device, dtype=torch.int32).contiguous()
    _dev(cams, idx)
    N = cams.shape[0]
    hw_shape = cams.shape[1:]
    M, k1 = idx.shape
    out = torch.empty((M,) + tuple(hw_shape), device=cams.device, dtype=torch.float32)
    hw = int(torch.tensor(hw_shape).prod().item()) if len(hw_shape) else 1
    check(lib.tcam_temporal_max(_ptr(cams), _ptr(idx), _ptr(out), M, k1, hw, float(t),
                                _stream()), "tcam_temporal_max")
    return out


def temporal_cam(cams: torch.Tensor, idx: torch.Tensor, t: float = 0.0,
                 want_cam: bool = True, want_u8: bool = True):
    """Full-resolution temporal CAM: out[i] = max_j renorm(cams[idx[i, j]]) and its
    uint8 quantisation.  cams (N, H, W) fp32; idx (M, k1) int (-1 = absent)."""
    lib = _lib.load()
    idx = idx.to(device=cams.device, dtype=torch.int32).contiguous()
    _dev(cams, idx)
    if cams.dtype != torch.float32 or cams.dim() != 3:
        raise ValueError("cams must be a (N, H, W) float32 tensor")
    N, H, W = cams.shape
    M, k1 = idx.shape
    if M > 65535:
        raise ValueError("at most 65535 output frames per launch")
    out = torch.empty((M, H, W), device=cams.device) if want_cam else None
    u8 = torch.empty((M, H, W), device=cams.device, dtype=torch.uint8) if want_u8 else None
    scale = torch.empty(N, device=cams.device) if t > 0 else None
    check(lib.tcam_temporal_cam(_ptr(cams), N, _ptr(idx), _ptr(out), _ptr(u8), M, k1, H * W,
                                float(t), _ptr(scale), _stream()), "tcam_temporal_cam")
    return out, u8


def topk_flags(logits: torch.Tensor, target: torch.Tensor):
    lib = _lib.load()
    target = target.to(device=logits.device, dtype=torch.int32).contiguous()
    _dev(logits, target)
    B, Cc = logits.shape
    top1 = torch.empty(B, device=logits.device, dtype=torch.int32)
    top5 = torch.empty(B, device=logits.device, dtype=torch.int32)
    check(lib.tcam_topk_flags(_ptr(logits), _ptr(target), _ptr(top1), _ptr(top5), B, Cc,
                              _stream()), "tcam_topk_flags")
    return top1, top5


def bbox_levels(cam_u8: torch.Tensor, chunks: int = 0):
    """Per-frame, per-level best box: (boxes (B,256,4) int32, vmax (B,) int32).
    ``chunks`` (1..4, 0 = the default): level ranges per frame of the sweep — more = shorter
    latency for more CU-time; the boxes are the same."""
    lib = _lib.load()
    _dev(cam_u8)
    assert cam_u8.dtype == torch.uint8 and cam_u8.dim() == 3
    B, H, W = cam_u8.shape
    boxes = torch.empty((B, 256, 4), device=cam_u8.device, dtype=torch.int32)
    vmax = torch.empty((B,), device=cam_u8.device, dtype=torch.int32)
    ws = torch.empty(int(lib.tcam_bbox_ws_bytes(B, H, W)), device=cam_u8.device,
                     dtype=torch.uint8)
    lib.tcam_bbox_set_chunks(int(chunks))
    try:
        check(lib.tcam_bbox_levels(_ptr(cam_u8), _ptr(boxes), _ptr(vmax), _ptr(ws), B, H, W,
                                   _stream()), "tcam_bbox_levels")
    finally:
        lib.tcam_bbox_set_chunks(0)
    return boxes, vmax


def box_accumulate(boxes: torch.Tensor, vmax: torch.Tensor, taus: torch.Tensor,
                   gt: torch.Tensor, ngt: torch.Tensor, top1: torch.Tensor, top5: torch.Tensor,
                   iou_thr: torch.Tensor, counters: torch.Tensor,
                   best_iou: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = _lib.load()
    _dev(boxes, vmax, taus, gt, ngt, top1, top5, iou_thr, counters, best_iou)
    B = boxes.shape[0]
    T = taus.shape[0]
    G = gt.shape[1]
    assert taus.dtype == torch.float64 and iou_thr.dtype == torch.float64
    assert gt.dtype == torch.int32 and counters.dtype == torch.int32
    assert counters.shape == (3, iou_thr.shape[0], T)
    check(lib.tcam_box_accumulate(_ptr(boxes), _ptr(vmax), _ptr(taus), T, _ptr(gt), _ptr(ngt),
                                  G, _ptr(top1), _ptr(top5), _ptr(iou_thr), iou_thr.shape[0],
                                  _ptr(counters), _ptr(best_iou), B, _stream()),
          "tcam_box_accumulate")
    return counters


_STREAM_WS = {}


def _stream_workspace(name: str, device: torch.device, nbytes: int) -> torch.Tensor:
    """A scratch buffer kept per (name, device, stream), grown on demand: kernels that run
    one at a time on a stream reuse it instead of a fresh ~200 MB allocation per call (the
    BoxAcc v2 sweep's per-workgroup contour images)."""
    key = (name, device, _stream())
    ws = _STREAM_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(nbytes, 256), device=device, dtype=torch.uint8)
        _STREAM_WS[key] = ws
    return ws


def bbox_multi_iou(cam_u8: torch.Tensor, gt: torch.Tensor, ngt: torch.Tensor):
    """BoxAcc v2 (multi_contour_eval): per frame and level, the best IoU over every contour
    box and GT box.  Returns (iou (B,256) fp64, canon (B,256) int32, vmax (B,) int32)."""
    lib = _lib.load()
    _dev(cam_u8, gt, ngt)
    assert cam_u8.dtype == torch.uint8 and cam_u8.dim() == 3
    assert gt.dtype == torch.int32 and gt.dim() == 3 and gt.shape[0] == cam_u8.shape[0]
    B, H, W = cam_u8.shape
    dev = cam_u8.device
    iou = torch.empty((B, 256), device=dev, dtype=torch.float64)
    canon = torch.empty((B, 256), device=dev, dtype=torch.int32)
    vmax = torch.empty((B,), device=dev, dtype=torch.int32)
    ws = _stream_workspace("bbox_multi", dev, int(lib.tcam_bbox_multi_ws_bytes(B, H, W)))
    check(lib.tcam_bbox_multi_iou(_ptr(cam_u8), _ptr(gt), _ptr(ngt.to(torch.int32)),
                                  gt.shape[1], _ptr(iou), _ptr(vmax), _ptr(canon), _ptr(ws),
                                  B, H, W, _stream()), "tcam_bbox_multi_iou")
    return iou, canon, vmax


def box_accumulate_multi(iou: torch.Tensor, canon: torch.Tensor, vmax: torch.Tensor,
                         taus: torch.Tensor, gt: torch.Tensor, ngt: torch.Tensor,
                         top1: torch.Tensor, top5: torch.Tensor, iou_thr: torch.Tensor,
                         counters: torch.Tensor,
                         best_iou: Optional[torch.Tensor] = None) -> torch.Tensor:
    lib = _lib.load()
    _dev(iou, canon, vmax, taus, gt, ngt, top1, top5, iou_thr, counters, best_iou)
    B, T = iou.shape[0], taus.shape[0]
    assert counters.shape == (3, iou_thr.shape[0], T) and counters.dtype == torch.int32
    check(lib.tcam_box_accumulate_multi(_ptr(iou), _ptr(canon), _ptr(vmax), _ptr(taus), T,
                                        _ptr(gt), _ptr(ngt), gt.shape[1], _ptr(top1),
                                        _ptr(top5), _ptr(iou_thr), iou_thr.shape[0],
                                        _ptr(counters), _ptr(best_iou), B, _stream()),
          "tcam_box_accumulate_multi")
    return counters


def bbox_contours(cam_u8: torch.Tensor, level: int, cap: Optional[int] = None):
    """Every contour of findContours(u8 > level, RETR_TREE) of ONE frame (H, W) uint8 as an
    (n, 8) int32 host array (is_hole, key, parent key, x0, y0, x1, y1, 0), unordered."""
    lib = _lib.load()
    _dev(cam_u8)
    assert cam_u8.dtype == torch.uint8 and cam_u8.dim() == 2
    H, W = cam_u8.shape
    cap = int(cap or H * W + 4)
    dev = cam_u8.device
    rec = torch.empty((cap, 8), device=dev, dtype=torch.int32)
    cnt = torch.zeros(1, device=dev, dtype=torch.int32)
    ws = torch.empty(int(lib.tcam_bbox_contours_ws_bytes(H, W)), device=dev, dtype=torch.uint8)
    check(lib.tcam_bbox_contours(_ptr(cam_u8.contiguous()), int(level), _ptr(rec), cap,
                                 _ptr(cnt), _ptr(ws), H, W, _stream()), "tcam_bbox_contours")
    n = int(cnt.item())
    if n > cap:
        raise RuntimeError(f"bbox_contours: {n} contours > capacity {cap}")
    return rec[:n].cpu().numpy()


def flag_count(flags: torch.Tensor, acc: torch.Tensor) -> torch.Tensor:
    """acc[0] += count of nonzero int32 flags (device, no sync)."""
    lib = _lib.load()
    _dev(flags, acc)
    assert flags.dtype == torch.int32 and acc.dtype == torch.int32
    check(lib.tcam_flag_count(_ptr(flags.contiguous()), flags.numel(), _ptr(acc), _stream()),
          "tcam_flag_count")
    return acc


# ------------------------------------------------------------------ S3 path
# S3 activations: (B, H, W, C/8, 3, 8) bfloat16, value = (hi + mid) + lo
# (include/tcam_hip.h, csrc/conv_x6.hip).  Used by the x6 convolution path.

def is_s3(t: torch.Tensor) -> bool:
    return t.dim() == 6 and t.dtype == torch.bfloat16 and t.shape[-2:] == (3, 8)


# S2 activations (the f16x3 inference path): (B, H, W, C/8, 2, 8) float16, value = h + l
# (h = fp16(x), l = fp16(x - h); |x| <= 65504).
def is_s2(t: torch.Tensor) -> bool:
    return t.dim() == 6 and t.dtype == torch.float16 and t.shape[-2:] == (2, 8)


# S1 activations (the AMP path, autocast's fp16 tensors): (B, H, W, C/8, 1, 8) float16.
def is_s1(t: torch.Tensor) -> bool:
    return t.dim() == 6 and t.dtype == torch.float16 and t.shape[-2:] == (1, 8)


def is_act(t: torch.Tensor) -> bool:
    """An S3, S2 or S1 activation tensor."""
    return is_s3(t) or is_s2(t) or is_s1(t)


def _lay(t: torch.Tensor) -> str:
    """ABI suffix of an activation tensor's layout ("s3" / "s2" / "s1")."""
    if is_s3(t):
        return "s3"
    if is_s2(t):
        return "s2"
    if is_s1(t):
        return "s1"
    raise ValueError(f"not an S3 / S2 / S1 activation tensor: {tuple(t.shape)} {t.dtype}")


# activation layout of each conv precision
FMT_LAYOUT = {"x6": "s3", "f16x3": "s2", "amp": "s1"}


def s3_dims(t: torch.Tensor) -> Tuple[int, int, int, int]:
    """(B, H, W, C) of an S3 (or S2) tensor."""
    return t.shape[0], t.shape[1], t.shape[2], t.shape[3] * 8


def s3_empty(B: int, H: int, W: int, C: int, device) -> torch.Tensor:
    assert C % 8 == 0
    return torch.empty((B, H, W, C // 8, 3, 8), device=device, dtype=torch.bfloat16)


def s2_empty(B: int, H: int, W: int, C: int, device) -> torch.Tensor:
    assert C % 8 == 0
    return torch.empty((B, H, W, C // 8, 2, 8), device=device, dtype=torch.float16)


def s1_empty(B: int, H: int, W: int, C: int, device) -> torch.Tensor:
    assert C % 8 == 0
    return torch.empty((B, H, W, C // 8, 1, 8), device=device, dtype=torch.float16)


_EMPTY = {"s3": s3_empty, "s2": s2_empty, "s1": s1_empty}


def lay_empty(lay: str, B: int, H: int, W: int, C: int, device) -> torch.Tensor:
    return _EMPTY[lay](B, H, W, C, device)


def act_empty(like: torch.Tensor, B: int, H: int, W: int, C: int) -> torch.Tensor:
    """A new activation tensor in the layout of ``like``."""
    return lay_empty(_lay(like), B, H, W, C, like.device)


def s3_from_nchw(x: torch.Tensor, cpad: Optional[int] = None, fmt: str = "x6") -> torch.Tensor:
    """fp32 NCHW -> S3 (fmt "x6"), S2 (fmt "f16x3") or S1 (fmt "amp": rounded to fp16),
    channels zero-padded to ``cpad``."""
    lib = _lib.load()
    _dev(x)
    assert x.dtype == torch.float32 and x.dim() == 4
    B, Cc, H, W = x.shape
    cpad = cpad or (Cc + 7) // 8 * 8
    lay = FMT_LAYOUT[fmt]
    out = lay_empty(lay, B, H, W, cpad, x.device)
    check(getattr(lib, f"tcam_{lay}_from_nchw")(_ptr(x), _ptr(out), B, Cc, H, W, cpad,
                                                _stream()), f"tcam_{lay}_from_nchw")
    # the zero channels added by cpad are layout, not work: the launch timer counts
    # algorithmic FLOPs over the logical channels only (the 3-channel image)
    out.tcam_logical_channels = Cc
    return out


def s3_to_nchw(t: torch.Tensor) -> torch.Tensor:
    """S3 / S2 / S1 -> fp32 NCHW (exact)."""
    lib = _lib.load()
    _dev(t)
    lay = _lay(t)
    B, H, W, Cc = s3_dims(t)
    out = torch.empty((B, Cc, H, W), device=t.device, dtype=torch.float32)
    check(getattr(lib, f"tcam_{lay}_to_nchw")(_ptr(t), _ptr(out), B, Cc, H, W, _stream()),
          f"tcam_{lay}_to_nchw")
    return out


def relayout(t: torch.Tensor, fmt: str) -> torch.Tensor:
    """An S2 / S3 activation in the other layout ("x6" -> S3, "f16x3" -> S2); the same tensor
    when it is already there.  S2 -> S3 is exact."""
    lib = _lib.load()
    _dev(t)
    if fmt == "amp":
        if is_s1(t):
            return t
        raise ValueError("S1 (amp) activations come from the amp plans, not from a relayout")
    want_s2 = fmt == "f16x3"
    if is_s2(t) == want_s2:
        return t
    B, H, W, Cc = s3_dims(t)
    out = (s2_empty if want_s2 else s3_empty)(B, H, W, Cc, t.device)
    name = "tcam_s3_to_s2" if want_s2 else "tcam_s2_to_s3"
    check(getattr(lib, name)(_ptr(t), _ptr(out), B * H * W * (Cc // 8), _stream()), name)
    return out


def scale_channels(t: torch.Tensor, e: Optional[torch.Tensor],
                   negate: bool = False) -> torch.Tensor:
    """An S3 / S1 activation with channel c multiplied by 2^e[c] (2^-e[c] when ``negate``):
    the f16x3 plans' channel exponents (models.act_exponents) taken out of an S3 copy,
    exact (bf16 parts keep fp32's exponent range).  ``e`` None: ``t`` itself."""
    if e is None:
        return t
    if is_s2(t):
        raise ValueError("scale an S3 / S1 tensor (fp16 S2 parts could leave their range)")
    B, H, W, Cc = s3_dims(t)
    f = torch.pow(2.0, (-e if negate else e).double())
    f = torch.cat([f, torch.ones(Cc - f.numel(), dtype=torch.float64)]) if f.numel() < Cc else f
    f = f.reshape(Cc // 8, 1, 8).to(device=t.device, dtype=t.dtype)
    return t * f


def split3(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Exact fp32 -> (hi, mid, lo) bf16 split (round-to-nearest-even each step)."""
    hi = x.to(torch.bfloat16)
    r = x - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return hi, mid, lo


def conv_x6_weight_dims(k: int, cout: int) -> Tuple[int, int]:
    kp, mp = C.c_int(), C.c_int()
    check(_lib.load().tcam_conv_x6_weight_dims(k, cout, C.byref(kp), C.byref(mp)),
          "tcam_conv_x6_weight_dims")
    return kp.value, mp.value


def pack_conv_weight_x6(ws: Sequence[torch.Tensor]) -> torch.Tensor:
    """PyTorch conv weights (Cout, C_s, KH, KW) of the sources -> the split,
    packed (Kpad/32, 4, 3, Mpad, 8) bf16 operand of tcam_conv2d_x6."""
    w = torch.cat(list(ws), dim=1).float()
    cout, ctot, kh, kw = w.shape
    k = ctot * kh * kw
    kp, mp = conv_x6_weight_dims(k, cout)
    wt = torch.zeros((kp, mp), dtype=torch.float32, device=w.device)
    wt[:k, :cout] = w.permute(2, 3, 1, 0).reshape(k, cout)
    parts = [t.view(kp // 32, 4, 8, mp).permute(0, 1, 3, 2) for t in split3(wt)]
    return torch.stack(parts, dim=2).contiguous()


def pack_conv_weight_f16(ws: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
    """PyTorch conv weights (Cout, C_s, KH, KW) of the sources -> (the packed
    (Kpad/32, 4, 2, Mpad, 8) float16 operand of tcam_conv2d_f16x3, the (Mpad,) fp32
    per-output-channel scales).  Column m holds W[:, m] / s_m split as h + l, s_m the power
    of two that puts max_k |W[k, m]| / s_m in [2^14, 2^15): the hi parts use fp16's top
    binades, the lo parts stay normal for weights within 2^-14 of the column's largest."""
    w = torch.cat(list(ws), dim=1).float()
    cout, ctot, kh, kw = w.shape
    k = ctot * kh * kw
    kp, mp = conv_x6_weight_dims(k, cout)
    wt = torch.zeros((kp, mp), dtype=torch.float32, device=w.device)
    wt[:k, :cout] = w.permute(2, 3, 1, 0).reshape(k, cout)
    amax = wt.abs().amax(dim=0)
    e = torch.floor(torch.log2(torch.where(amax > 0, amax, torch.ones_like(amax))))
    scale = torch.where(amax > 0, torch.exp2(e - 14), torch.ones_like(amax)).contiguous()
    u = wt / scale
    h = u.to(torch.float16)
    lo = (u - h.float()).to(torch.float16)
    parts = [t.view(kp // 32, 4, 8, mp).permute(0, 1, 3, 2) for t in (h, lo)]
    return torch.stack(parts, dim=2).contiguous(), scale


def pack_conv_weight_h1(ws: Sequence[torch.Tensor]) -> torch.Tensor:
    """PyTorch conv weights (Cout, C_s, KH, KW) of the sources -> the packed
    (Kpad/32, 4, 1, Mpad, 8) float16 operand of tcam_conv2d_f16: the weight rounded to fp16,
    as autocast casts it (the AMP path)."""
    w = torch.cat(list(ws), dim=1).float()
    cout, ctot, kh, kw = w.shape
    k = ctot * kh * kw
    kp, mp = conv_x6_weight_dims(k, cout)
    wt = torch.zeros((kp, mp), dtype=torch.float32, device=w.device)
    wt[:k, :cout] = w.permute(2, 3, 1, 0).reshape(k, cout)
    h = wt.to(torch.float16).view(kp // 32, 4, 8, mp).permute(0, 1, 3, 2)
    return h.unsqueeze(2).contiguous()


class StemF16:
    """The f16x3 stem operands of a folded first conv (tcam_stem_f16x3): the weight rows in
    (tap, channel) order over the C * KH * KW real pairs padded to a 32 multiple, packed and
    split as :func:`pack_conv_weight_f16`, and their planar-image offsets (per input size)."""

    __slots__ = ("wt", "wscale", "bias", "nk", "cout", "cin", "k", "stride", "pad", "_tabs")

    def __init__(self, w: torch.Tensor, bias: torch.Tensor, stride: int, pad: int):
        cout, cin, kh, kw = w.shape
        assert kh == kw and cout <= 64 and cout % 8 == 0
        k = cin * kh * kw
        kp = (k + 31) // 32 * 32
        rows = w.float().permute(0, 2, 3, 1).reshape(cout, k)   # k = (kh * KW + kw) * C + c
        wk = torch.zeros((cout, kp, 1, 1), dtype=torch.float32, device=w.device)
        wk[:, :k, 0, 0] = rows
        self.wt, self.wscale = pack_conv_weight_f16([wk])
        self.nk = kp // 32
        self.bias = bias.float().contiguous().to(w.device)
        self.cout, self.cin, self.k, self.stride, self.pad = cout, cin, kh, stride, pad
        self._tabs = {}

    def ktab(self, device) -> torch.Tensor:
        """Packed row k -> its offset c * IR * IC + kh * IC + kw in the kernel's LDS window
        of IR x IC input pixels per channel (tcam_stem_window); -1 = zero padding."""
        t = self._tabs.get(device)
        if t is None:
            ir, ic = C.c_int(), C.c_int()
            check(_lib.load().tcam_stem_window(self.k, self.k, self.stride, C.byref(ir),
                                               C.byref(ic)), "tcam_stem_window")
            k = self.cin * self.k * self.k
            tab = torch.full((self.nk * 32,), -1, dtype=torch.int32)
            i = torch.arange(k)
            c, tap = i % self.cin, i // self.cin
            tab[:k] = (c * ir.value * ic.value + (tap // self.k) * ic.value +
                       tap % self.k).to(torch.int32)
            t = tab.to(device)
            self._tabs[device] = t
        return t


def stem_f16x3(x: torch.Tensor, st: StemF16) -> torch.Tensor:
    """tcam_stem_f16x3: fp32 NCHW image -> the stem's S2 output (conv + bias + ReLU)."""
    lib = _lib.load()
    _dev(x, st.wt)
    assert x.dtype == torch.float32 and x.dim() == 4 and x.shape[1] == st.cin
    x = x.contiguous()
    B, _, H, W = x.shape
    Ho = (H + 2 * st.pad - st.k) // st.stride + 1
    Wo = (W + 2 * st.pad - st.k) // st.stride + 1
    out = s2_empty(B, Ho, Wo, st.cout, x.device)
    tab = st.ktab(x.device)
    timer = _TIMER
    if timer is not None:
        e0, e1 = _timer_events()
        _timer_arm(lib, e0, e1)
    check(lib.tcam_stem_f16x3(_ptr(x), _ptr(st.wt), _ptr(st.wscale), _ptr(st.bias), _ptr(tab),
                              st.nk, _ptr(out), B, st.cin, H, W, st.cout, st.k, st.k, st.stride,
                              st.pad, _ptr(f16_overflow_flag(x.device)), _stream()),
          "tcam_stem_f16x3")
    if timer is not None:
        _timer_disarm(lib)
        timer.append(("conv", 2.0 * st.cout * st.cin * st.k * st.k * B * Ho * Wo, e0, e1,
                      f"M{st.cout} K{st.cin * st.k * st.k} N{B * Ho * Wo} k{st.k}x{st.k} stem"))
    return out


def weight_fmt(wt: torch.Tensor) -> str:
    """The conv precision a packed weight operand selects."""
    if wt.dtype == torch.bfloat16:
        return "x6"
    return "amp" if wt.shape[2] == 1 else "f16x3"


_F16_OFLOW = {}
_F16_REDIRECT = {}


def f16_overflow_flag(device: torch.device) -> torch.Tensor:
    """The device's int32 flag the f16x3 convolutions set when an output leaves the S2
    range (|x| > 65504): their results are then invalid.  Inside
    :func:`f16_overflow_into` the launches set the given flag instead."""
    r = _F16_REDIRECT.get(device)
    if r is not None:
        return r
    f = _F16_OFLOW.get(device)
    if f is None:
        f = torch.zeros(1, dtype=torch.int32, device=device)
        _F16_OFLOW[device] = f
    return f


class f16_overflow_into:
    """Context: the f16x3 launches issued inside it set ``flag`` (an int32 device tensor)
    instead of the device's flag — work running ahead on a side stream (the training step's
    next-batch encoder) keeps its overflow apart until the step that consumes its result
    merges it (:func:`merge_f16_overflow`)."""

    def __init__(self, flag: torch.Tensor):
        self.flag = flag

    def __enter__(self):
        dev = self.flag.device
        self._prev = _F16_REDIRECT.get(dev)
        _F16_REDIRECT[dev] = self.flag
        return self.flag

    def __exit__(self, *exc):
        dev = self.flag.device
        if self._prev is None:
            _F16_REDIRECT.pop(dev, None)
        else:
            _F16_REDIRECT[dev] = self._prev
        return False


def merge_f16_overflow(flag: torch.Tensor) -> None:
    """OR a side flag into the device's flag, on the current stream."""
    f16_overflow_flag(flag.device).bitwise_or_(flag)


def _all_ranks_max(t: torch.Tensor) -> torch.Tensor:
    """MAX over the ranks of the default group (RCCL on the device, gloo via the host)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return t
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t
    h = t.cpu()
    dist.all_reduce(h, op=dist.ReduceOp.MAX)
    return h


def check_f16_overflow(device: torch.device, reset: bool = True,
                       all_ranks: bool = False) -> None:
    """Raise if any f16x3 convolution on ``device`` overflowed the S2 range since the last
    check (a host synchronisation).  ``all_ranks`` (the evaluator, the trainers, bench.py's
    end of region — call sites every rank reaches together): under torch.distributed the
    flag is first reduced (MAX) over every rank — a collective — and then EVERY rank raises,
    or none does (a rank-local raise would leave the others blocked in their next
    collective).  The default is this rank's flag alone (no collective)."""
    f = _F16_OFLOW.get(device)
    if f is None:
        f = f16_overflow_flag(device) if all_ranks else None
        if f is None:
            return
    v = f.clone()
    if reset:
        f.zero_()
    if all_ranks:
        v = _all_ranks_max(v)
    if int(v.item()):
        raise FloatingPointError(
            "an activation exceeded the f16x3 (S2) range |x| <= 65504: results of this "
            "pass are invalid; run it with conv_precision='x6'")


_X6_WS = {}


def _x6_workspace(device: torch.device, stream: int) -> torch.Tensor:
    """Stream-K workspace (zeroed once; one per device and stream)."""
    key = (device, stream)
    ws = _X6_WS.get(key)
    if ws is None:
        n = int(_lib.load().tcam_conv_x6_ws_bytes())
        ws = torch.zeros(n, dtype=torch.uint8, device=device)
        _X6_WS[key] = ws
    return ws


def _pair(v) -> Tuple[int, int]:
    return (int(v[0]), int(v[1])) if isinstance(v, (tuple, list)) else (int(v), int(v))


def _x6_srcs(srcs: Sequence[ConvSrc], B: int, kh: int, kw: int, fmt: str = "x6"):
    """ctypes source array + the logical K (stem padding not counted) of an x6 conv."""
    arr = (tcam_conv_src * len(srcs))()
    kdim = 0
    lay = FMT_LAYOUT[fmt]
    for i, s in enumerate(srcs):
        t = s.t
        assert is_act(t) and _lay(t) == lay and t.shape[0] == B, \
            "sources must be in the weights' layout (S3 for x6, S2 for f16x3, S1 for amp)"
        _, H, W, Cc = s3_dims(t)
        arr[i] = tcam_conv_src(t.data_ptr(), Cc, H, W, s.stride, 1 if s.up2 else 0)
        kdim += getattr(t, "tcam_logical_channels", Cc) * kh * kw
    return arr, kdim


def conv2d_x6(srcs: Sequence[ConvSrc], wt: torch.Tensor, bias: torch.Tensor, cout: int,
              hout: int, wout: int, ksize, pad, relu: bool,
              residual: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None, out_coff: int = 0,
              stream_k: bool = True, wscale: Optional[torch.Tensor] = None) -> torch.Tensor:
    """tcam_conv2d_x6 over S3 sources; returns the S3 output (B, hout, wout, cout).
    ``ksize`` / ``pad``: int or (h, w).  ``out`` may be a wider S3 tensor: the conv
    writes channels [out_coff, out_coff + cout) of it (a fused channel concat).
    ``stream_k`` lets the kernel balance partial tile waves with the per-stream
    workspace (deterministic; False = one block per tile).
    float16 weights (:func:`pack_conv_weight_f16`, with their ``wscale``) select
    tcam_conv2d_f16x3: S2 sources, S2 output; single-part float16 weights
    (:func:`pack_conv_weight_h1`) select tcam_conv2d_f16 (AMP): S1 sources, S1 output."""
    lib = _lib.load()
    B = srcs[0].t.shape[0]
    kh, kw = _pair(ksize)
    ph, pw = _pair(pad)
    fmt = weight_fmt(wt)
    lay = FMT_LAYOUT[fmt]
    f16 = fmt == "f16x3"
    _dev(wt, bias, residual, wscale, *[s.t for s in srcs])
    if out is None:
        out = lay_empty(lay, B, hout, wout, cout, wt.device)
        cstride = cout
    else:
        assert _lay(out) == lay and tuple(out.shape[:3]) == (B, hout, wout)
        cstride = s3_dims(out)[3]
    if residual is not None:
        assert _lay(residual) == lay
    arr, kdim = _x6_srcs(srcs, B, kh, kw, fmt)
    timer = _TIMER
    if timer is not None:
        e0, e1 = _timer_events()
        _timer_arm(lib, e0, e1)
    stream = _stream()
    ws = _x6_workspace(wt.device, stream) if stream_k else None
    if f16:
        if wscale is None:
            raise ValueError("f16x3 weights need their per-channel scales (wscale)")
        check(lib.tcam_conv2d_f16x3(arr, len(srcs), B, _ptr(wt), _ptr(wscale), _ptr(bias),
                                    _ptr(residual), _ptr(out), cout, hout, wout, kh, kw, ph, pw,
                                    1 if relu else 0, cstride, out_coff,
                                    _ptr(f16_overflow_flag(wt.device)), _ptr(ws),
                                    0 if ws is None else ws.numel(), stream),
              "tcam_conv2d_f16x3")
    elif fmt == "amp":
        check(lib.tcam_conv2d_f16(arr, len(srcs), B, _ptr(wt), _ptr(bias), _ptr(residual),
                                  _ptr(out), cout, hout, wout, kh, kw, ph, pw, 1 if relu else 0,
                                  cstride, out_coff, _ptr(ws), 0 if ws is None else ws.numel(),
                                  stream), "tcam_conv2d_f16")
    else:
        check(lib.tcam_conv2d_x6(arr, len(srcs), B, _ptr(wt), _ptr(bias), _ptr(residual),
                                 _ptr(out), cout, hout, wout, kh, kw, ph, pw, 1 if relu else 0,
                                 cstride, out_coff, _ptr(ws), 0 if ws is None else ws.numel(),
                                 stream), "tcam_conv2d_x6")
    if timer is not None:
        _timer_disarm(lib)
        timer.append(("conv", 2.0 * cout * kdim * B * hout * wout, e0, e1,
                      f"M{cout} K{kdim} N{B * hout * wout} k{kh}x{kw} src{len(srcs)}"))
    return out


def conv2d_f16x3_s3out(srcs: Sequence[ConvSrc], wt: torch.Tensor, wscale: torch.Tensor,
                       bias: torch.Tensor, cout: int, hout: int, wout: int, ksize,
                       pad) -> torch.Tensor:
    """tcam_conv2d_f16x3_s3out: the f16x3 convolution of S2 sources (f16x3 weights +
    wscale) with an S3 output — the training step's data gradient of a scaled dy copy."""
    lib = _lib.load()
    B = srcs[0].t.shape[0]
    kh, kw = _pair(ksize)
    ph, pw = _pair(pad)
    if weight_fmt(wt) != "f16x3":
        raise ValueError("tcam_conv2d_f16x3_s3out takes f16x3 weights")
    _dev(wt, bias, wscale, *[s.t for s in srcs])
    out = lay_empty("s3", B, hout, wout, cout, wt.device)
    arr, kdim = _x6_srcs(srcs, B, kh, kw, "f16x3")
    stream = _stream()
    ws = _x6_workspace(wt.device, stream)
    check(lib.tcam_conv2d_f16x3_s3out(arr, len(srcs), B, _ptr(wt), _ptr(wscale), _ptr(bias),
                                      _ptr(out), cout, hout, wout, kh, kw, ph, pw, 0, cout, 0,
                                      _ptr(ws), ws.numel(), stream), "tcam_conv2d_f16x3_s3out")
    return out


def bottleneck_f16x3(x: torch.Tensor, c1, c2, c3, ds: bool) -> torch.Tensor:
    """One fused ResNet50 layer-1 Bottleneck (encoders/resnet.py:175-232 at stride 1):
    tcam_bottleneck_f16x3 on S2 activations (f16x3 weights with their ``wscale``) or
    tcam_bottleneck_f16 on S1 activations (the AMP path's single-part fp16 weights).
    ``c1`` / ``c2`` / ``c3``: the block's folded convs (``wt``, ``wscale``, ``bias``); ``ds``:
    ``c3`` carries the projection shortcut of ``x`` (the first block, x with 64 channels),
    else ``x`` (256 channels) is the residual.  Returns the block output (B, H, W, 256) in
    the input's layout, bit-identical to the three unfused convs."""
    lib = _lib.load()
    B, H, W, cin = s3_dims(x)
    fmt = weight_fmt(c1.wt)
    if fmt not in ("f16x3", "amp") or any(weight_fmt(c.wt) != fmt for c in (c2, c3)):
        raise ValueError("bottleneck_f16x3 takes f16x3 or amp weights")
    _dev(x, c1.wt, c2.wt, c3.wt)
    out = lay_empty(FMT_LAYOUT[fmt], B, H, W, 256, x.device)
    timer = _TIMER
    if timer is not None:
        e0, e1 = _timer_events()
        _timer_arm(lib, e0, e1)
    if fmt == "f16x3":
        if any(c.wscale is None for c in (c1, c2, c3)):
            raise ValueError("f16x3 weights need their per-channel scales (wscale)")
        check(lib.tcam_bottleneck_f16x3(_ptr(x), B, H, W, cin, _ptr(c1.wt), _ptr(c1.wscale),
                                        _ptr(c1.bias), _ptr(c2.wt), _ptr(c2.wscale),
                                        _ptr(c2.bias), _ptr(c3.wt), _ptr(c3.wscale),
                                        _ptr(c3.bias), 1 if ds else 0, _ptr(out),
                                        _ptr(f16_overflow_flag(x.device)), _stream()),
              "tcam_bottleneck_f16x3")
    else:
        check(lib.tcam_bottleneck_f16(_ptr(x), B, H, W, cin, _ptr(c1.wt), _ptr(c1.bias),
                                      _ptr(c2.wt), _ptr(c2.bias), _ptr(c3.wt), _ptr(c3.bias),
                                      1 if ds else 0, _ptr(out), _stream()),
              "tcam_bottleneck_f16")
    if timer is not None:
        _timer_disarm(lib)
        n = B * H * W
        flop = 2.0 * n * (64 * cin + 64 * 576 + 256 * (64 + (cin if ds else 0)))
        timer.append(("conv", flop, e0, e1, f"bottleneck cin{cin} N{n}{' ds' if ds else ''}"))
    return out


def conv2d_x6_multi(srcs: Sequence[ConvSrc], wt: torch.Tensor, bias: torch.Tensor,
                    couts: Sequence[int], hout: int, wout: int, ksize, pad, relu: bool,
                    outs: Sequence[Optional[Tuple[torch.Tensor, int]]],
                    stream_k: bool = True,
                    wscale: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
    """Grouped launch (tcam_conv2d_x6_multi): one x6 conv over weights stacked along the
    output channels, ``couts`` channels per member; member i writes channels
    [coff, coff + couts[i]) of ``outs[i] = (tensor, coff)`` or, for None, a new S3 tensor.
    Returns the member outputs (the given tensors or the new ones)."""
    lib = _lib.load()
    B = srcs[0].t.shape[0]
    kh, kw = _pair(ksize)
    ph, pw = _pair(pad)
    cout = int(sum(couts))
    assert len(outs) == len(couts) and 1 <= len(couts) <= 3
    fmt = weight_fmt(wt)
    if fmt == "amp":
        raise NotImplementedError("grouped launches run the x6 / f16x3 formats")
    f16 = fmt == "f16x3"
    _dev(wt, bias, wscale, *[s.t for s in srcs])
    arr, kdim = _x6_srcs(srcs, B, kh, kw, fmt)
    dst = (tcam_conv_dst * len(couts))()
    res, c0 = [], 0
    for i, (c, o) in enumerate(zip(couts, outs)):
        if o is None:
            t, coff = (s2_empty if f16 else s3_empty)(B, hout, wout, c, wt.device), 0
        else:
            t, coff = o
            assert (is_s2(t) if f16 else is_s3(t)) and tuple(t.shape[:3]) == (B, hout, wout)
        dst[i] = tcam_conv_dst(t.data_ptr(), c0, s3_dims(t)[3], coff)
        res.append(t)
        c0 += c
    timer = _TIMER
    if timer is not None:
        e0, e1 = _timer_events()
        _timer_arm(lib, e0, e1)
    stream = _stream()
    ws = _x6_workspace(wt.device, stream) if stream_k else None
    if f16:
        check(lib.tcam_conv2d_f16x3_multi(arr, len(srcs), B, _ptr(wt), _ptr(wscale), _ptr(bias),
                                          cout, hout, wout, kh, kw, ph, pw, 1 if relu else 0,
                                          dst, len(couts), _ptr(f16_overflow_flag(wt.device)),
                                          _ptr(ws), 0 if ws is None else ws.numel(), stream),
              "tcam_conv2d_f16x3_multi")
    else:
        check(lib.tcam_conv2d_x6_multi(arr, len(srcs), B, _ptr(wt), _ptr(bias), cout, hout,
                                       wout, kh, kw, ph, pw, 1 if relu else 0, dst, len(couts),
                                       _ptr(ws), 0 if ws is None else ws.numel(), stream),
              "tcam_conv2d_x6_multi")
    if timer is not None:
        _timer_disarm(lib)
        timer.append(("conv", 2.0 * cout * kdim * B * hout * wout, e0, e1,
                      f"M{cout} K{kdim} N{B * hout * wout} k{kh}x{kw} src{len(srcs)} x{len(couts)}"))
    return res


class ConvMember:
    """One convolution of a grouped launch (:func:`conv2d_group`): source, packed weights
    (+ wscale on f16x3), bias, output geometry and the (tensor, channel offset) it writes
    (None: a new tensor)."""

    __slots__ = ("src", "wt", "wscale", "bias", "cout", "hout", "wout", "ksize", "pad", "relu",
                 "out", "out_coff")

    def __init__(self, src: ConvSrc, wt: torch.Tensor, bias: torch.Tensor, cout: int,
                 hout: int, wout: int, ksize, pad, relu: bool = True,
                 wscale: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                 out_coff: int = 0):
        self.src, self.wt, self.wscale, self.bias = src, wt, wscale, bias
        self.cout, self.hout, self.wout = int(cout), int(hout), int(wout)
        self.ksize, self.pad, self.relu = _pair(ksize), _pair(pad), bool(relu)
        self.out, self.out_coff = out, int(out_coff)


GROUP_MAX = 4


def conv2d_group(members: Sequence[ConvMember], tile: int = -1) -> List[torch.Tensor]:
    """tcam_conv2d_group: up to GROUP_MAX independent convolutions of one precision (x6 or
    f16x3) in ONE launch — each member's output is what :func:`conv2d_x6` gives for it
    alone.  ``tile``: -1 automatic (128x128 LDS-DMA when every source has C % 32 == 0,
    else the register-staged 128x64), or 15 / 26 / 17 / 18 / 20.  Returns the outputs."""
    lib = _lib.load()
    assert 1 <= len(members) <= GROUP_MAX
    B = members[0].src.t.shape[0]
    fmt = weight_fmt(members[0].wt)
    if fmt == "amp":
        raise NotImplementedError("grouped launches run the x6 / f16x3 formats")
    f16 = fmt == "f16x3"
    lay = FMT_LAYOUT[fmt]
    arr = (tcam_conv_prob * len(members))()
    outs, flops, desc = [], 0.0, []
    for i, m in enumerate(members):
        assert weight_fmt(m.wt) == fmt and m.src.t.shape[0] == B and not m.src.up2
        if f16 and m.wscale is None:
            raise ValueError("f16x3 weights need their per-channel scales (wscale)")
        _dev(m.wt, m.bias, m.wscale, m.src.t)
        src, kdim = _x6_srcs([m.src], B, m.ksize[0], m.ksize[1], fmt)
        if m.out is None:
            out = lay_empty(lay, B, m.hout, m.wout, m.cout, m.wt.device)
        else:
            out = m.out
            assert _lay(out) == lay and tuple(out.shape[:3]) == (B, m.hout, m.wout)
        arr[i] = tcam_conv_prob(src[0], _ptr(m.wt), _ptr(m.wscale) if f16 else None,
                                _ptr(m.bias), _ptr(out), m.cout, m.hout, m.wout, m.ksize[0],
                                m.ksize[1], m.pad[0], m.pad[1], 1 if m.relu else 0,
                                s3_dims(out)[3], m.out_coff)
        outs.append(out)
        flops += 2.0 * m.cout * kdim * B * m.hout * m.wout
        desc.append(f"M{m.cout} K{kdim} N{B * m.hout * m.wout} k{m.ksize[0]}x{m.ksize[1]}")
    timer = _TIMER
    if timer is not None:
        e0, e1 = _timer_events()
        _timer_arm(lib, e0, e1)
    dev = members[0].wt.device
    check(lib.tcam_conv2d_group(arr, len(members), B, 1 if f16 else 0, int(tile),
                                _ptr(f16_overflow_flag(dev)) if f16 else None, _stream()),
          "tcam_conv2d_group")
    if timer is not None:
        _timer_disarm(lib)
        timer.append(("conv", flops, e0, e1, "group[" + " | ".join(desc) + "]"))
    return outs


def maxpool3x3s2_s3(x: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    _dev(x)
    B, H, W, Cc = s3_dims(x)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    out = act_empty(x, B, Ho, Wo, Cc)
    lay = _lay(x)
    check(getattr(lib, f"tcam_maxpool3x3s2_{lay}")(_ptr(x), _ptr(out), B, Cc, H, W, Ho, Wo,
                                                   _stream()), f"tcam_maxpool3x3s2_{lay}")
    return out


def pool_out_size(n: int, k: int, stride: int, pad: int, ceil_mode: bool = False) -> int:
    """torch's pooling output size (incl. the ceil_mode last-window rule)."""
    num = n + 2 * pad - k
    o = (-(-num // stride) if ceil_mode else num // stride) + 1
    if ceil_mode and (o - 1) * stride >= n + pad:
        o -= 1
    return o


def pool2d_s3(x: torch.Tensor, k, stride: int, pad: int, mode: str = "max",
              ceil_mode: bool = False, out: Optional[torch.Tensor] = None,
              out_coff: int = 0) -> torch.Tensor:
    """max_pool2d / avg_pool2d(count_include_pad=True) on S3; optional fused concat
    into channels [out_coff, out_coff + C) of ``out``."""
    lib = _lib.load()
    _dev(x)
    kh, kw = _pair(k)
    B, H, W, Cc = s3_dims(x)
    Ho = pool_out_size(H, kh, stride, pad, ceil_mode)
    Wo = pool_out_size(W, kw, stride, pad, ceil_mode)
    if out is None:
        out = act_empty(x, B, Ho, Wo, Cc)
    lay = _lay(x)
    assert _lay(out) == lay and tuple(out.shape[:3]) == (B, Ho, Wo)
    check(getattr(lib, f"tcam_pool2d_{lay}")(_ptr(x), _ptr(out), B, Cc, H, W, Ho, Wo, kh, kw,
                                             stride, pad, 0 if mode == "max" else 1,
                                             s3_dims(out)[3], out_coff, _stream()),
          f"tcam_pool2d_{lay}")
    return out


def up2_resize_s3(x: torch.Tensor, size: Tuple[int, int]) -> torch.Tensor:
    lib = _lib.load()
    _dev(x)
    B, H, W, Cc = s3_dims(x)
    out = act_empty(x, B, size[0], size[1], Cc)
    lay = _lay(x)
    check(getattr(lib, f"tcam_up2_resize_{lay}")(_ptr(x), _ptr(out), B, Cc, H, W, size[0],
                                                 size[1], _stream()), f"tcam_up2_resize_{lay}")
    return out


def wgap_s3(x: torch.Tensor, fc_w: torch.Tensor, fc_b: torch.Tensor) -> torch.Tensor:
    lib = _lib.load()
    _dev(x, fc_w, fc_b)
    B, H, W, Cc = s3_dims(x)
    classes = fc_w.shape[0]
    ws = torch.empty(int(lib.tcam_wgap_s3_ws_bytes(B, Cc, H * W)), device=x.device,
                     dtype=torch.uint8)
    out = torch.empty((B, classes), device=x.device, dtype=torch.float32)
    lay = _lay(x)
    check(getattr(lib, f"tcam_wgap_{lay}")(_ptr(x), _ptr(fc_w), _ptr(fc_b), _ptr(out), None,
                                           _ptr(ws), B, Cc, H * W, classes, _stream()),
          f"tcam_wgap_{lay}")
    return out


def seghead_cam_s3(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, want_fcams: bool = True,
                   want_u8: bool = True, argmax: bool = False):
    lib = _lib.load()
    _dev(x, w, b)
    B, H, W, Cin = s3_dims(x)
    fcams = torch.empty((B, 2, H, W), device=x.device) if want_fcams else None
    cam = torch.empty((B, H, W), device=x.device)
    u8 = torch.empty((B, H, W), device=x.device, dtype=torch.uint8) if want_u8 else None
    lay = _lay(x)
    check(getattr(lib, f"tcam_seghead_cam_{lay}")(_ptr(x), _ptr(w), _ptr(b), _ptr(fcams),
                                                  _ptr(cam), _ptr(u8), B, Cin, H, W,
                                                  1 if argmax else 0, _stream()),
          f"tcam_seghead_cam_{lay}")
    return fcams, cam, u8


def resize_cam(fcams: torch.Tensor, size: Tuple[int, int], want_fcams: bool = True,
               want_u8: bool = True, argmax: bool = False):
    """fcams resized (bilinear, align_corners=True) to the input size, then the CAM."""
    lib = _lib.load()
    _dev(fcams)
    B, _, Hi, Wi = fcams.shape
    Ho, Wo = size
    fo = torch.empty((B, 2, Ho, Wo), device=fcams.device) if want_fcams else None
    cam = torch.empty((B, Ho, Wo), device=fcams.device)
    u8 = torch.empty((B, Ho, Wo), device=fcams.device, dtype=torch.uint8) if want_u8 else None
    check(lib.tcam_resize_cam(_ptr(fcams), _ptr(fo), _ptr(cam), _ptr(u8), B, Hi, Wi, Ho, Wo,
                              1 if argmax else 0, _stream()), "tcam_resize_cam")
    return fo, cam, u8
