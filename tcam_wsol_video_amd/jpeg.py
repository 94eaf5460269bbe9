"""Frame decode on the device: the reference loader's ``Image.open(path).convert('RGB')``
(datasets/wsol_loader.py:581-582) for a batch of baseline JPEG files, bit-identical to
Pillow 12.2 / libjpeg-turbo (JDCT_ISLOW, fancy upsampling, YCbCr -> RGB).

The host side (C++ ``tcam_jpeg_pack``) walks the markers and packs the unstuffed
entropy bytes, deduplicated Huffman tables and quantisers into one staging blob; the
device (``tcam_jpeg_decode``) does Huffman decode, islow IDCT, upsampling and colour
conversion (csrc/jpeg.hip).  Files the decoder does not support (progressive,
arithmetic-coded, 12-bit, CMYK, multi-scan) raise :class:`UnsupportedJPEG` naming the
file -- there is no host-decode fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib
from ._lib import check

E_NOTJPEG, E_UNSUPPORTED, E_CORRUPT = -20, -21, -22
E_NOMEM = -2   # TCAM_E_NOMEM: staging blob too small (sizes[0] holds the exact size)
_ERRS = {E_NOTJPEG: "not a JPEG file", E_UNSUPPORTED: "unsupported JPEG variant "
         "(progressive / arithmetic / 12-bit / CMYK / multi-scan)",
         E_CORRUPT: "corrupt JPEG data"}


class UnsupportedJPEG(ValueError):
    pass


def read_bytes(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


class JpegDecoder:
    """Reusable decoder: pinned host staging + device blob / workspace grown on demand.

    ``decode(datas)`` -> list of (H, W, 3) uint8 device tensors (views of one output
    buffer, images in input order); ``decode_batch`` -> (B, H, W, 3) for same-size
    files.  Work is enqueued on the current stream of ``device``.  Two pinned staging blobs
    alternate, so the host packs batch i+1 while batch i's upload is still queued (it waits
    only for the upload of batch i-1 before refilling that blob); the device blob /
    workspace are reused only after the previous decode's kernels are done (the new stream
    waits on them), so consecutive decodes may use different streams.
    """

    def __init__(self, device: Union[str, torch.device, None] = None):
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("JpegDecoder decodes on the GPU; no CPU fallback")
        self._host: List[Optional[torch.Tensor]] = [None, None]
        self._dev: Optional[torch.Tensor] = None
        self._ws: Optional[torch.Tensor] = None
        self._upload_done: List[Optional[torch.cuda.Event]] = [None, None]
        self._k = 0                              # staging blob of the next call
        self._decode_done: Optional[torch.cuda.Event] = None
        self.last_sizes = None

    @staticmethod
    def plan(datas: Sequence[bytes], names: Optional[Sequence[str]] = None):
        """(sizes[4], dims (n, 3)) without packing; raises on unsupported files."""
        datas = [d if isinstance(d, bytes) else bytes(d) for d in datas]   # c_char_p needs bytes
        n = len(datas)
        ptrs = (C.c_char_p * n)(*datas)
        lens = (C.c_size_t * n)(*[len(d) for d in datas])
        sizes = np.zeros(4, np.int64)
        dims = np.zeros((max(n, 1), 3), np.int32)
        lib = _lib.load()
        rc = lib.tcam_jpeg_pack(C.cast(ptrs, C.c_void_p), C.cast(lens, C.c_void_p), n, None, 0,
                                sizes.ctypes.data_as(C.c_void_p),
                                dims.ctypes.data_as(C.c_void_p))
        _raise_bad(rc, dims[:n], names)
        return sizes, dims[:n], (ptrs, lens)

    def decode(self, datas: Sequence[bytes],
               names: Optional[Sequence[str]] = None) -> List[torch.Tensor]:
        n = len(datas)
        if n == 0:
            return []
        datas = [d if isinstance(d, bytes) else bytes(d) for d in datas]
        ptrs = (C.c_char_p * n)(*datas)
        lens = (C.c_size_t * n)(*[len(d) for d in datas])
        sizes = np.zeros(4, np.int64)
        dims = np.zeros((n, 3), np.int32)
        stream = torch.cuda.current_stream(self.device)
        k = self._k
        self._k ^= 1
        if self._upload_done[k] is not None:
            self._upload_done[k].synchronize()   # that blob's last H2D copy has read it
        lib = _lib.load()
        # one parse + pack into a generously sized staging blob; the packer reports the
        # exact size when it does not fit (restart-heavy files), then packs again
        want = int(sum(len(d) for d in datas) * 1.25) + 64 * n + (1 << 16)
        for _ in range(2):
            if self._host[k] is None or self._host[k].numel() < want:
                self._host[k] = torch.empty(_grow(want), dtype=torch.uint8, pin_memory=True)
            host = self._host[k]
            rc = lib.tcam_jpeg_pack(C.cast(ptrs, C.c_void_p), C.cast(lens, C.c_void_p), n,
                                    host.data_ptr(), host.numel(),
                                    sizes.ctypes.data_as(C.c_void_p),
                                    dims.ctypes.data_as(C.c_void_p))
            if rc != E_NOMEM:
                break
            want = int(sizes[0])
        _raise_bad(rc, dims, names)
        blob_b, ws_b, out_b = int(sizes[0]), int(sizes[1]), int(sizes[2])
        grow = (self._dev is None or self._dev.numel() < blob_b or self._ws is None
                or self._ws.numel() < ws_b)
        if grow and self._decode_done is not None:
            # the old buffers go back to the caching allocator's pool of the stream they
            # were allocated on; a decode still reading them on another stream must finish
            # before that stream can reuse the memory
            self._decode_done.synchronize()
        if self._dev is None or self._dev.numel() < blob_b:
            self._dev = torch.empty(_grow(blob_b), dtype=torch.uint8, device=self.device)
        if self._ws is None or self._ws.numel() < ws_b:
            self._ws = torch.empty(_grow(ws_b), dtype=torch.uint8, device=self.device)
        hp = host.data_ptr()
        with torch.cuda.stream(stream):
            if self._decode_done is not None:
                stream.wait_event(self._decode_done)   # blob / workspace of the last decode
            # the cached buffers are used on whichever stream the caller decodes on
            self._dev.record_stream(stream)
            self._ws.record_stream(stream)
            self._dev[:blob_b].copy_(host[:blob_b], non_blocking=True)
            self._upload_done[k] = torch.cuda.Event()
            self._upload_done[k].record(stream)
            out = torch.empty(out_b, dtype=torch.uint8, device=self.device)
            check(lib.tcam_jpeg_decode(hp, self._dev.data_ptr(), self._ws.data_ptr(),
                                       self._ws.numel(), out.data_ptr(), stream.cuda_stream),
                  "tcam_jpeg_decode")
            self._decode_done = torch.cuda.Event()
            self._decode_done.record(stream)
        self.last_sizes = sizes
        res, off = [], 0
        for h, w, _ in dims.tolist():
            res.append(out[off:off + h * w * 3].view(h, w, 3))
            off += h * w * 3
        return res

    def decode_batch(self, datas: Sequence[bytes],
                     names: Optional[Sequence[str]] = None) -> torch.Tensor:
        imgs = self.decode(datas, names)
        if not imgs:
            raise ValueError("empty batch")
        shp = imgs[0].shape
        if any(i.shape != shp for i in imgs):
            raise ValueError("decode_batch needs same-size frames; use decode()")
        base = imgs[0]
        return base.as_strided((len(imgs),) + tuple(shp), (shp[0] * shp[1] * 3, shp[1] * 3, 3, 1))

    def open_rgb(self, paths: Sequence[str]) -> List[torch.Tensor]:
        """[Image.open(p).convert('RGB') for p in paths] as device tensors."""
        return self.decode([read_bytes(p) for p in paths], names=list(paths))


def _grow(n: int) -> int:
    return max(1 << 16, int(n * 1.25) + 4096)


def _raise_bad(rc: int, dims: np.ndarray, names: Optional[Sequence[str]]):
    if rc == 0:
        return
    bad = [(i, int(dims[i, 2])) for i in range(len(dims)) if dims[i, 2] != 0]
    if bad:
        i, e = bad[0]
        who = names[i] if names is not None else f"frame {i}"
        raise UnsupportedJPEG(f"{who}: {_ERRS.get(e, e)} ({len(bad)} of {len(dims)} files)")
    check(rc, "tcam_jpeg_pack")


_DECODERS = {}


def decode(datas: Sequence[bytes], device=None,
           names: Optional[Sequence[str]] = None) -> List[torch.Tensor]:
    """One-shot batch decode with a per-device cached :class:`JpegDecoder`."""
    dev = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if dev not in _DECODERS:
        _DECODERS[dev] = JpegDecoder(dev)
    return _DECODERS[dev].decode(datas, names)


def image_dims(data: bytes) -> Tuple[int, int]:
    """(height, width) from the headers (host only, no device work)."""
    _, dims, _ = JpegDecoder.plan([data])
    return int(dims[0, 0]), int(dims[0, 1])
