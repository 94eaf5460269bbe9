/*
 * tcam_hip.h — C ABI of libtcam_hip.so, the MI355X (gfx950) hot path of TCAM.
 *
 * Plain C types only: device pointers, sizes, a hipStream_t passed as void*.
 * Every entry point returns 0 on success or a hipError_t / negative
 * TCAM_E_* code; nothing here throws or prints.  Callers own all buffers.
 * Layout of every image/feature tensor is NCHW fp32, contiguous.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to the reference repo sbelharbi/tcam-wsol-video).
 */
#ifndef TCAM_HIP_H
#define TCAM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCAM_OK 0
#define TCAM_E_ARG (-1)       /* bad shape / argument */
#define TCAM_E_NOMEM (-2)     /* workspace too small */

/* ---------------------------------------------------------------- info */
/* ABI version (bumped on any signature change). */
int tcam_abi_version(void);
/* Name of the device the library was built for ("gfx950"). */
const char* tcam_arch(void);

/* ------------------------------------------------- convolution (MFMA) */
/*
 * One input source of an implicit-GEMM convolution.  Sources are
 * concatenated along channels (decoder skip concat, decoder.py:44-53, and the
 * fused conv3+downsample of a bottleneck, resnet.py:214-232).
 *   up2 = 1: the source is read through a nearest x2 upsample
 *            (F.interpolate(scale_factor=2, mode="nearest"), decoder.py:43).
 */
typedef struct tcam_conv_src {
    const float* ptr;   /* (B, C, H, W) */
    int C, H, W;
    int stride;         /* spatial stride of this source's taps */
    int up2;            /* 0/1 */
} tcam_conv_src;

/*
 * out = act( conv(srcs) + bias [+ residual] ), BN already folded into w/bias.
 * Replaces: nn.Conv2d + nn.BatchNorm2d(eval) + nn.ReLU sequences of
 *   encoders/resnet.py:140-153,214-232 (torchvision Bottleneck / stem),
 *   base/modules.py:10-49 (Conv2dReLU), base/heads.py:19-36 (SegmentationHead).
 * wt: (Kpad, Mpad) row-major, zero padded (tcam_conv_weight_dims), with
 *     K = KH * KW * Ctot ordered tap-major, k = (kh * KW + kw) * Ctot + c,
 *     c over the concatenated source channels: PyTorch's (Cout, Cin, KH, KW)
 *     permuted to (KH, KW, Cin, Cout).
 * relu: 0/1.  residual: NULL or (B, Cout, Hout, Wout).
 */
/* Padded weight dims for tcam_conv2d: Kpad = roundup(K, 32),
 * Mpad = roundup(Cout, 128). */
int tcam_conv_weight_dims(int K, int Cout, int* Kpad, int* Mpad);

int tcam_conv2d(const tcam_conv_src* srcs, int nsrc, int B,
                const float* wt, const float* bias, const float* residual,
                float* out, int Cout, int Hout, int Wout,
                int KH, int KW, int pad, int relu, void* stream);

/* Tuning hook: force tile configuration `id` for every following
 * tcam_conv2d call (-1 = automatic choice).  Returns the number of configs. */
int tcam_conv_force_tile(int id);

/* fp32-accurate convolution on the bf16 MFMA pipe ("x6": each fp32 operand
 * split exactly into hi + mid + lo bf16 parts, the six cross products of
 * order <= 2 accumulated in fp32; see csrc/conv_x6.hip).
 * Activations (srcs, residual, out) are in the S3 layout: NHWC, channels in
 * groups of 8, each group [hi x8][mid x8][lo x8] bf16 — a (B, H, W, C/8, 3, 8)
 * bf16 array; every source C % 8 == 0, Cout % 8 == 0.
 * wt: (Kpad/32, 4, 3, Mpad, 8) bf16, element [kt][g][p][m][e] = part p of
 * W[32 kt + 8 g + e][m] (K tap-major as tcam_conv2d), zero padded;
 * Kpad = roundup(K, 32), Mpad = roundup(Cout, 32) (tcam_conv_x6_weight_dims).
 * All pointers 16-byte aligned.
 * ws: optional stream-K workspace of tcam_conv_x6_ws_bytes() bytes, zeroed once
 * at allocation (its arrival counters return to 0 after every call), 256-B
 * aligned, used by one stream at a time; NULL = plain one-block-per-tile grid.
 * Results are deterministic either way. */
int tcam_conv_x6_weight_dims(int K, int Cout, int* Kpad, int* Mpad);
size_t tcam_conv_x6_ws_bytes(void);
/* KH x KW taps (each <= 7; rectangular 1x7 / 7x1 / 1x3 / 3x1 included) with
 * zero padding pad_h / pad_w (InceptionV3 BasicConv2d, wsol_backbones/inceptionv3.py:52-64).
 * out_cstride: channels per pixel of `out` (0 = Cout); the conv writes channels
 * [out_coff, out_coff + Cout) — a fused torch.cat along channels (Inception
 * branches, inceptionv3.py:88-89).  With a residual, out_cstride must be Cout. */
int tcam_conv2d_x6(const tcam_conv_src* srcs, int nsrc, int B,
                   const void* wt, const float* bias, const void* residual,
                   void* out, int Cout, int Hout, int Wout,
                   int KH, int KW, int pad_h, int pad_w, int relu,
                   int out_cstride, int out_coff, void* ws, size_t ws_bytes,
                   void* stream);
/* Grouped launch: ONE x6 conv over the output-stacked weights of several convs that read
 * the same sources (the branch-parallel 1x1 convs on an Inception block's input,
 * inceptionv3.py:86-96 (branch1x1, branch5x5_1, branch3x3dbl_1) and :150-170
 * (branch1x1, branch7x7_1, branch7x7dbl_1), which torchvision runs as separate convs).
 * Output channels [dst[i].c_begin, dst[i+1].c_begin) (the last up to Cout) go to
 * channels [dst[i].coff, ...) of dst[i].ptr, an S3 tensor of dst[i].cstride channels per
 * pixel.  1 <= ndst <= 3, dst[0].c_begin = 0, c_begin multiples of 8; no residual. */
typedef struct tcam_conv_dst {
    void* ptr;
    int c_begin, cstride, coff;
} tcam_conv_dst;
int tcam_conv2d_x6_multi(const tcam_conv_src* srcs, int nsrc, int B,
                         const void* wt, const float* bias, int Cout, int Hout, int Wout,
                         int KH, int KW, int pad_h, int pad_w, int relu,
                         const tcam_conv_dst* dst, int ndst, void* ws, size_t ws_bytes,
                         void* stream);
int tcam_conv_x6_force_tile(int id);
/* -1 automatic stream-K choice, 0 never (and a tile choice that ignores how full the
 * launch is: each frame's output is then independent of how the frames are batched, e.g.
 * a clip sharded over ranks vs one process), > 0 always, over `grid` blocks (tests). */
int tcam_conv_x6_force_streamk(int grid);
/* Timing experiments only (results are wrong when set): 1 = every B load reads
 * pixel 0, 2 = no global loads after the first K-step; 0 = normal. */
int tcam_conv_x6_debug(int flags);

/* ---- S3-layout kernels (csrc/s3.hip) for the x6 path ---- */
/* NCHW fp32 (B, C, H, W) -> S3 (B, H, W, Cpad/8, 3, 8), channels >= C zero. */
int tcam_s3_from_nchw(const float* in, void* out, int B, int C, int H, int W, int Cpad,
                      void* stream);
/* S3 -> NCHW fp32 (exact: value = (hi + mid) + lo). */
int tcam_s3_to_nchw(const void* in, float* out, int B, int C, int H, int W, void* stream);
/* MaxPool2d(3, 2, 1) on S3 (resnet.py:99). */
int tcam_maxpool3x3s2_s3(const void* in, void* out, int B, int C, int H, int W, int Ho,
                         int Wo, void* stream);
/* Pooling on S3 with torch semantics (caller's Ho/Wo encode ceil_mode):
 * mode 0 = max_pool2d, 1 = avg_pool2d(count_include_pad=True).  Used for VGG's
 * MaxPool2d(2, 2) (encoders/vgg.py:146-161), InceptionV3's MaxPool2d(3, 2, 1,
 * ceil_mode=True) / max_pool2d(3, 1, 1) / avg_pool2d(3, 1, 1)
 * (wsol_backbones/inceptionv3.py:96, 127, 181, 283-290).  Output channels
 * [out_coff, out_coff + C) of a tensor with out_cstride channels (0 = C). */
int tcam_pool2d_s3(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                   int KH, int KW, int stride, int pad, int mode, int out_cstride,
                   int out_coff, void* stream);
/* nearest x2 + bilinear(align_corners=True) to (Ho, Wo) on S3 (decoder.py:43-51). */
int tcam_up2_resize_s3(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                       void* stream);
/* WGAP on S3 (poolings/core.py:96-115); mean (B, C) optional; ws of
 * tcam_wgap_s3_ws_bytes(B, C, HW) bytes. */
size_t tcam_wgap_s3_ws_bytes(int B, int C, int HW);
int tcam_wgap_s3(const void* x, const float* fc_w, const float* fc_b, float* logits,
                 float* mean, float* ws, int B, int C, int HW, int classes, void* stream);
/* tcam_seghead_cam with an S3 input (Cin % 8 == 0, Cin <= 64). */
int tcam_seghead_cam_s3(const void* x, const float* w, const float* b, float* fcams,
                        float* cam, uint8_t* cam_u8, int B, int Cin, int H, int W,
                        int argmax, void* stream);
/* fcams (B, 2, Hi, Wi) -> bilinear(align_corners=True) to (Ho, Wo) (base/model.py:148-154),
 * then SegmentationCam + u8 as tcam_seghead_cam (fcams_out / cam / cam_u8 optional). */
int tcam_resize_cam(const float* fcams_in, float* fcams_out, float* cam, uint8_t* cam_u8,
                    int B, int Hi, int Wi, int Ho, int Wo, int argmax, void* stream);

/* Adjoint of tcam_resize_cam's fcams resize (bilinear, align_corners=True) for the
 * training backward of FCAMModel.forward's resize (base/model.py:148-154):
 * dout (BC, Ho, Wo) -> din (BC, Hi, Wi), deterministic gather. */
int tcam_resize_ac_bwd(const float* dout, float* din, int BC, int Hi, int Wi, int Ho, int Wo,
                       void* stream);
/* tcam_std_cam with S3 activations A (B, h, w, C/8, 3, 8). */
int tcam_std_cam_s3(const void* A, const float* fc_w, const int32_t* cls, float* low,
                    float* cam, uint8_t* cam_u8, int B, int C, int h, int w, int Ho, int Wo,
                    void* stream);

/* ---- the f16x3 inference path: S2 activations, fp16 MFMA ---- */
/*
 * S2 layout: NHWC with channels in groups of 8, each group stored as [h x8][l x8] fp16
 * (32 B), value = h + l with h = rne_f16(x), l = rne_f16(x - h): 22 significand bits,
 * representable for |x| <= 65504 (the convolutions set *oflow when an output exceeds it;
 * the results of that pass are then invalid).  A (B, H, W, C/8, 2, 8) fp16 array.
 *
 * tcam_conv2d_f16x3: tcam_conv2d_x6 (same sources / geometry / output semantics, same tile
 * machinery) on S2 operands.  Weights: (Kpad/32, 4, 2, Mpad, 8) fp16, element [kt][g][p][m][e]
 * = part p of W[32 kt + 8 g + e][m] / wscale[m], wscale (Mpad,) fp32 powers of two, 16-B
 * aligned.  Each product keeps the three cross terms al*bh + ah*bl + ah*bh (the dropped
 * al*bl < 2^-22 |ab|) on v_mfma_f32_{16x16x32,32x32x16}_f16, accumulated in fp32; the
 * epilogue computes acc * wscale[m] + bias[m] (+ residual, ReLU) and splits to S2.
 * oflow: an int the kernels set to 1 on an out-of-range output (NULL: no check).
 */
int tcam_conv2d_f16x3(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                      const float* wscale, const float* bias, const void* residual, void* out,
                      int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                      int relu, int out_cstride, int out_coff, int* oflow, void* ws,
                      size_t ws_bytes, void* stream);
int tcam_conv2d_f16x3_multi(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                            const float* wscale, const float* bias, int Cout, int Hout,
                            int Wout, int KH, int KW, int pad_h, int pad_w, int relu,
                            const tcam_conv_dst* dst, int ndst, int* oflow, void* ws,
                            size_t ws_bytes, void* stream);
/*
 * Heterogeneous grouped launch: up to 4 independent convolutions — each with its own
 * source, packed weights (+ wscale), bias, KHxKW / pads and output slice — of one precision
 * in ONE kernel launch.  Replaces: the independent branch convolutions of an Inception block
 * (wsol_backbones/inceptionv3.py:80-94 InceptionA, :109-120 InceptionB, :141-158
 * InceptionC), which the reference runs one after another.  Each member's result is the one
 * tcam_conv2d_x6 / tcam_conv2d_f16x3 gives on its own (same arithmetic, same order).
 * fmt: 0 = x6 (S3, wscale NULL), 1 = f16x3 (S2, wscale required, oflow as in
 * tcam_conv2d_f16x3).  tile: -1 = automatic, else 15 / 26 (128x128 LDS-DMA, every source
 * C % 32 == 0), 17 (64x64), 18 (128x64), 20 (64x128).  No residual; out_cstride 0 = Cout.
 */
typedef struct tcam_conv_prob {
    tcam_conv_src src;
    const void* wt;
    const float* wscale;
    const float* bias;
    void* out;
    int Cout, Hout, Wout, KH, KW, pad_h, pad_w, relu, out_cstride, out_coff;
} tcam_conv_prob;
int tcam_conv2d_group(const tcam_conv_prob* probs, int nprob, int B, int fmt, int tile,
                      int* oflow, void* stream);
/* The encoder stem on the f16x3 path straight from the fp32 NCHW image (B, C, H, W): conv
 * KHxKW / stride / pad + bias, ReLU, S2 output (B, Ho, Wo, Cout) with Cout <= 64 — ResNet50's
 * conv1 + bn1 + relu (encoders/resnet.py:60-62).  K is the C*KH*KW real (tap, channel) pairs
 * padded to nk * 32 (no per-tap channel padding, no NCHW -> S2 pass): each block stages an
 * IR x IC window per channel (tcam_stem_window; zero outside the image, split into fp16
 * h + l once) and the weight in LDS.  ktab (nk * 32 int32, 16-B aligned) gives packed row k's
 * window offset c * IR * IC + kh * IC + kw, -1 for padding; wt / wscale: tcam_conv2d_f16x3's
 * weight operand over those rows (Mpad = 32 or 64; C * IR * IC <= 4608, nk <= 8,
 * nk * 8 * Mpad <= 2560).  Same products as tcam_conv2d_f16x3 (fp16 h + l splits, three
 * cross terms, fp32 sums). */
int tcam_stem_window(int KH, int KW, int stride, int* IR, int* IC);
int tcam_stem_f16x3(const float* img, const void* wt, const float* wscale, const float* bias,
                    const int32_t* ktab, int nk, void* out, int B, int C, int H, int W,
                    int Cout, int KH, int KW, int stride, int pad, int* oflow, void* stream);
/* The S3 kernels above on S2 activations (same arguments; tcam_wgap_s3_ws_bytes sizes the
 * WGAP workspace of both). */
int tcam_s2_from_nchw(const float* in, void* out, int B, int C, int H, int W, int Cpad,
                      void* stream);
int tcam_s2_to_nchw(const void* in, float* out, int B, int C, int H, int W, void* stream);
int tcam_maxpool3x3s2_s2(const void* in, void* out, int B, int C, int H, int W, int Ho,
                         int Wo, void* stream);
int tcam_pool2d_s2(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                   int KH, int KW, int stride, int pad, int mode, int out_cstride,
                   int out_coff, void* stream);
int tcam_up2_resize_s2(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                       void* stream);
int tcam_wgap_s2(const void* x, const float* fc_w, const float* fc_b, float* logits,
                 float* mean, float* ws, int B, int C, int HW, int classes, void* stream);
int tcam_seghead_cam_s2(const void* x, const float* w, const float* b, float* fcams,
                        float* cam, uint8_t* cam_u8, int B, int Cin, int H, int W,
                        int argmax, void* stream);
int tcam_std_cam_s2(const void* A, const float* fc_w, const int32_t* cls, float* low,
                    float* cam, uint8_t* cam_u8, int B, int C, int h, int w, int Ho, int Wo,
                    void* stream);

/* ---- the AMP training path (--amp True: train_wsol.py:1077, 1155-1184): S1 activations ----
 * S1 layout: NHWC with channels in groups of 8, each group one fp16 part [h x8] (16 B), the
 * autocast fp16 activation: h = rne_f16(x), beyond 65504 -> inf (caught by the loss
 * scaler's non-finite check).  A (B, H, W, C/8, 1, 8) fp16 array.
 *
 * tcam_conv2d_f16: tcam_conv2d_x6 (same sources / geometry / output semantics) on S1
 * operands = the fp16 conv of torch.cuda.amp.autocast: weights (Kpad/32, 4, 1, Mpad, 8) fp16
 * (tcam_pack_weight_f16, no scale), ONE product per MAC on v_mfma_f32_*_f16 accumulated in
 * fp32, + bias (+ residual, ReLU) in fp32, output rounded to fp16. */
int tcam_conv2d_f16(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                    const float* bias, const void* residual, void* out, int Cout, int Hout,
                    int Wout, int KH, int KW, int pad_h, int pad_w, int relu, int out_cstride,
                    int out_coff, void* ws, size_t ws_bytes, void* stream);
/* The S3 layout kernels on S1 activations (same arguments). */
int tcam_s1_from_nchw(const float* in, void* out, int B, int C, int H, int W, int Cpad,
                      void* stream);
int tcam_s1_to_nchw(const void* in, float* out, int B, int C, int H, int W, void* stream);
int tcam_maxpool3x3s2_s1(const void* in, void* out, int B, int C, int H, int W, int Ho,
                         int Wo, void* stream);
int tcam_pool2d_s1(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                   int KH, int KW, int stride, int pad, int mode, int out_cstride,
                   int out_coff, void* stream);
int tcam_up2_resize_s1(const void* in, void* out, int B, int C, int H, int W, int Ho, int Wo,
                       void* stream);
int tcam_wgap_s1(const void* x, const float* fc_w, const float* fc_b, float* logits,
                 float* mean, float* ws, int B, int C, int HW, int classes, void* stream);
int tcam_seghead_cam_s1(const void* x, const float* w, const float* b, float* fcams,
                        float* cam, uint8_t* cam_u8, int B, int Cin, int H, int W,
                        int argmax, void* stream);
int tcam_std_cam_s1(const void* A, const float* fc_w, const int32_t* cls, float* low,
                    float* cam, uint8_t* cam_u8, int B, int C, int h, int w, int Ho, int Wo,
                    void* stream);

/* MaxPool2d(3, stride 2, pad 1) (resnet.py:99). */
int tcam_maxpool3x3s2(const float* in, float* out, int B, int C, int H, int W,
                      int Ho, int Wo, void* stream);

/* nearest x2 then bilinear(align_corners=True) to (Ho, Wo)
 * (decoder.py:43-51, when the upsampled map and the skip differ in size). */
int tcam_up2_resize(const float* in, float* out, int B, int C, int H, int W,
                    int Ho, int Wo, void* stream);

/* WGAP head: logits = Linear(AdaptiveAvgPool(x)) (poolings/core.py:96-115).
 * ws: >= B*C floats of workspace. */
int tcam_wgap(const float* x, const float* fc_w, const float* fc_b,
              float* logits, float* ws, int B, int C, int HW, int classes,
              void* stream);

/* -------------------------------------------------------------- CAMs */
/*
 * TCAM segmentation head fused with SegmentationCam (builtincam.py:201-225)
 * and the per-frame eval quantisation (inference_wsol.py:323-346,
 * wsol_metrics.py:153):
 *   fcams = conv3x3(x; w, b)                       (B, 2, H, W)   [optional]
 *   cam   = softmax(fcams, dim=1)[:, 1]            (B, H, W) fp32
 *   cam_u8 = uint8((double)cam * 255)              (B, H, W)      [optional]
 * argmax = 1 returns argmax(fcams, 1) as float instead of the softmax.
 * w: (2, Cin, 3, 3) PyTorch layout, b: (2,).
 */
int tcam_seghead_cam(const float* x, const float* w, const float* b,
                     float* fcams, float* cam, uint8_t* cam_u8,
                     int B, int Cin, int H, int W, int argmax, void* stream);

/* STD_CL CAM (cams/cam.py:31-99 + cams/core.py:162-193):
 * low[b] = minmax_normalise( sum_c w[cls[b], c] * A[b, c] )      (h, w)
 * cam[b] = bilinear(align_corners=False)(low[b]) to (Ho, Wo);
 * cam_u8 optional.  A: (B, C, h, w).  fc_w: (classes, C). */
int tcam_std_cam(const float* A, const float* fc_w, const int32_t* cls,
                 float* low, float* cam, uint8_t* cam_u8, int B, int C,
                 int h, int w, int Ho, int Wo, void* stream);

/* Temporal CAM aggregation (datasets/wsol_loader.py:591-601, 630-635):
 * out[i] = max_j renorm(cams[idx[i, j]]) over the (k+1) frames j with
 * idx >= 0, renorm(c) = nan_to_num(exp(t (c + 1e-6)) / max) when t > 0,
 * identity otherwise.  cams: (N, h, w); idx: (M, k1) int32. */
int tcam_temporal_max(const float* cams, const int32_t* idx, float* out,
                      int M, int k1, int hw, float t, void* stream);

/* Full-resolution temporal CAM of a (sharded) clip: the same aggregation as
 * tcam_temporal_max over N gathered frame CAMs (N, hw), plus the eval-time
 * quantisation out_u8 = uint8(double(out) * 255) (wsol_metrics.py:153).  Feeds the
 * bbox sweep with CAM-TMP maps (BASELINE configs[4]: per-frame CAMs all-gathered
 * over the ranks of a clip, dlib/parallel/__init__.py:14-23).  idx entries < 0 or
 * >= N are absent neighbours.  out or out_u8 may be NULL (not both).  scale_ws:
 * N floats, required when t > 0 (per-frame re_normalize_cam denominators). */
int tcam_temporal_cam(const float* cams, int N, const int32_t* idx, float* out,
                      uint8_t* out_u8, int M, int k1, int hw, float t, float* scale_ws,
                      void* stream);

/* top1[b] = (target[b] == preds_ordered[0]), top5[b] = target in preds[:5]
 * with preds_ordered = torch.sort(logits[b], descending, stable)
 * (inference_wsol.py:368-369, wsol_metrics.py:362-368). */
int tcam_topk_flags(const float* logits, const int32_t* target, int32_t* top1,
                    int32_t* top5, int B, int C, void* stream);

/* ------------------------------------------------------------ bbox */
/* Level ranges per frame of the next tcam_bbox_levels calls (1..4; 0 = the default, one range
 * or TCAM_BBOX_INC_CHUNKS): more ranges = shorter latency, more CU-time.  The evaluator sets 4
 * for the last clip of a pass, whose sweep nothing else overlaps (round 5). */
void tcam_bbox_set_chunks(int n);
/*
 * Batched compute_bboxes_from_scoremaps (wsol_metrics.py:127-197) with
 * multi_contour_eval=False: for every frame b and every level L in
 * [0, 255), the box of the contour of max cv2.contourArea among
 * findContours(u8 > L, RETR_TREE, CHAIN_APPROX_SIMPLE), as
 * (x0, y0, min(x0+w, W-1), min(y0+h, H-1)); [0,0,0,0] if none.
 *   cam_u8: (B, H, W);  boxes: (B, 256, 4) int32 (row L; rows >= max unused);
 *   vmax: (B,) int32 = max(cam_u8).  ws: tcam_bbox_ws_bytes(B, H, W) bytes.
 */
size_t tcam_bbox_ws_bytes(int B, int H, int W);
int tcam_bbox_levels(const uint8_t* cam_u8, int32_t* boxes, int32_t* vmax,
                     void* ws, int B, int H, int W, void* stream);

/* Profiling hook (scripts/bench_bbox.py): device buffer of
 * 2 * B * 16 * 16 uint64 receiving per-phase s_memrealtime ticks of the bbox
 * kernels, or NULL to disable. */
int tcam_bbox_set_debug(uint64_t* buf);
/* Fill-stage implementation: 0 = wave-parallel clamp scans per line (default), 1 = LDS
 * sweeps (round 1), 2 = register-line sweeps (round 2), kept for A/B timing.  All give
 * identical psi. */
int tcam_bbox_fill_variant(int v);
/* Re-layout of `groups` 8-channel groups between the S2 (f16x3) and S3 (x6) activation
 * layouts: S2 -> S3 exact; S3 -> S2 rounds to the 22-bit pair (|x| <= 65504). */
int tcam_s2_to_s3(const void* in, void* out, long groups, void* stream);
int tcam_s3_to_s2(const void* in, void* out, long groups, void* stream);
/* Test hook: one line sweep of the clamp-scan fill on device bytes p (psi), u (u8) -> out,
 * n <= 256; mode 0 = forward then backward, 1 = forward only. */
int tcam_bbox_scan_line(const uint8_t* p, const uint8_t* u, uint8_t* out, int n, int mode,
                        void* stream);
/* Level-stage implementation where a level sweep applies (frames up to 224 x 224):
 * 0 = sorted-list sweep (default: new pixels from the fill's psi-sorted pixel list, per-root
 * boxes), 1 = per-level CCL (level_kernel) always, 2 = incremental sweep (round 2).
 * Identical boxes. */
int tcam_bbox_level_variant(int v);
/* Profiling hook: device buffer of B * 16 uint64 receiving per-workgroup phase ticks of the
 * incremental level sweep (slots 0-7; slot 8 = levels processed), or NULL. */
int tcam_bbox_set_inc_debug(uint64_t* buf);

/*
 * BoxEvaluator.accumulate for a batch (wsol_metrics.py:295-370 with
 * calculate_multiple_iou 77-124): for every frame b and threshold index i,
 *   thr = int(taus[i] * vmax[b]); box = boxes[b, thr];
 *   iou = max_g IoU(box, gt[b, g]) (inclusive-pixel convention, fp64);
 *   for each IoU threshold j: if iou >= iou_thr[j]: counters[0][j][i] += 1,
 *     counters[1][j][i] += top1[b], counters[2][j][i] += top5[b].
 * gt: (B, G, 4) int32 with G = max boxes per frame, padded with ngt[b].
 * counters: (3, n_iou, T) int32, accumulated (not cleared).
 * best_iou (optional): (B, T) fp64 per-threshold IoU.
 */
int tcam_box_accumulate(const int32_t* boxes, const int32_t* vmax,
                        const double* taus, int T, const int32_t* gt,
                        const int32_t* ngt, int G, const int32_t* top1,
                        const int32_t* top5, const double* iou_thr, int n_iou,
                        int32_t* counters, double* best_iou, int B,
                        void* stream);

/* BoxAcc v2 (--box_v2_metric True, parseit.py:684-689): compute_bboxes_from_scoremaps with
 * multi_contour_eval=True (metrics/wsol_metrics.py:155-181) keeps the boundingRect of every
 * contour of findContours(u8 > thr, RETR_TREE, CHAIN_APPROX_SIMPLE), and
 * BoxEvaluator.accumulate scores a threshold by the best IoU over those boxes
 * (wsol_metrics.py:342-368).  Replaces that per-frame, per-threshold cv2 loop.
 *   tcam_bbox_multi_iou: iou (B, 256) fp64 — row L (L < vmax[b], the levels where the
 *     binary image changes): max over contour boxes and GT boxes of the IoU (+1 inclusive
 *     convention); canon (B, 256) int32: the computed level whose image level L shares;
 *     vmax (B,) = max(cam_u8); gt (B, G, 4) int32, ngt (B,), G <= 64; frames <= 320^2;
 *     ws: tcam_bbox_multi_ws_bytes(B, H, W) bytes (no initialisation needed).
 *   tcam_box_accumulate_multi: the counters as tcam_box_accumulate, from those IoUs.
 *   tcam_bbox_contours: ONE frame, one level: every contour as 8 int32
 *     (is_hole, key, parent_key, x0, y0, x1, y1, 0) — key = raster index of the contour's
 *     component's first pixel, parent_key = the enclosing contour's key or -1 — in no
 *     particular order (the host orders them as OpenCV lists them); *count = the number of
 *     contours (records beyond cap are dropped).  ws: tcam_bbox_contours_ws_bytes(H, W). */
size_t tcam_bbox_multi_ws_bytes(int B, int H, int W);
int tcam_bbox_multi_iou(const uint8_t* cam_u8, const int32_t* gt, const int32_t* ngt, int G,
                        double* iou, int32_t* vmax, int32_t* canon, void* ws, int B, int H,
                        int W, void* stream);
int tcam_box_accumulate_multi(const double* iou, const int32_t* canon, const int32_t* vmax,
                              const double* taus, int T, const int32_t* gt,
                              const int32_t* ngt, int G, const int32_t* top1,
                              const int32_t* top5, const double* iou_thr, int n_iou,
                              int32_t* counters, double* best_iou, int B, void* stream);
size_t tcam_bbox_contours_ws_bytes(int H, int W);
int tcam_bbox_contours(const uint8_t* cam_u8, int level, int32_t* records, int cap,
                       int32_t* count, void* ws, int H, int W, void* stream);

/* Trainer._compute_accuracy (learning/train_wsol.py:1400-1435): acc[0] += the number of
 * nonzero flags (B,) int32 — the per-frame argmax == target flags (tcam_topk_flags' top1:
 * rank 0 with ties to the lower class index = torch.argmax). */
int tcam_flag_count(const int32_t* flags, int B, int32_t* acc, void* stream);

/* --------------------------------------------------- bilateral / CRF */
/*
 * Permutohedral-lattice bilateral filter (csrc/bilateral.hip), the device
 * version of bilateralfilter_batch
 * (crf/crfwrapper/bilateralfilter/bilateralfilter.cpp:4-55 over
 * permutohedral.cpp:105-571, called by crf/dense_crf_loss.py:59-60):
 *   images (N, 3, H, W) fp32 (values in [0, 255]), ins (N, K, H, W) -> outs (N, K, H, W);
 *   features per pixel (x/s_xy, y/s_xy, r/s_rgb, g/s_rgb, b/s_rgb), d = 5.
 * Output is bit-identical to the reference's x86-64 (SSE) build; deterministic.
 * K <= 8.  Keys must fit the packed lattice word: |lattice coordinate| <= 12287
 * for d = 5 (features up to ~2000; TCAM uses s_rgb 15, s_xy 100 -> < 100);
 * a key outside that range sets the status word (tcam_bilateral_status).
 * ws: tcam_bilateral_ws_bytes(N, K, H, W, d) bytes, ZERO-FILLED before its first use
 * (every call leaves its lattice hash table empty again); one stream at a time.
 * The size query is host arithmetic; 0 = invalid.
 */
size_t tcam_bilateral_ws_bytes(int N, int K, int H, int W, int dim);
int tcam_bilateral_batch(const float* images, const float* ins, float* outs,
                         void* ws, size_t ws_bytes, int N, int K, int H, int W,
                         float s_rgb, float s_xy, void* stream);

/* tcam_bilateral_batch in two phases on one workspace: _prepare builds the lattice of
 * `images` (everything that does not depend on `ins`: elevation, keys, hash table, the
 * vertex-ordered entry layout, the blur neighbours; it empties the hash table again), _apply
 * filters `ins` through it (splat, blur, slice).  Exactly one _apply per _prepare, same N, K, H, W and sigmas; the two may run on
 * different streams when the caller orders them (e.g. _prepare on a side stream while the
 * network producing `ins` runs, an event before _apply).  Output bit-identical to
 * tcam_bilateral_batch. */
int tcam_bilateral_prepare(const float* images, void* ws, size_t ws_bytes, int N, int K,
                           int H, int W, float s_rgb, float s_xy, void* stream);
int tcam_bilateral_apply(const float* ins, float* outs, void* ws, size_t ws_bytes, int N,
                         int K, int H, int W, float s_rgb, float s_xy, void* stream);

/* Colour-only filter, the device version of colorbilateralfilter_batch
 * (crf/crfwrapper/colorbilateralfilter/colorbilateralfilter.cpp:4-54, called by
 * crf/color_dense_crf_loss.py:61-62): features = the first `dim` image planes
 * / s_rgb (dim <= 3; images keep the reference's stride of 3 planes per image).
 * ws: tcam_bilateral_ws_bytes(N, K, H, W, dim). */
int tcam_colorbilateral_batch(const float* images, const float* ins, float* outs,
                              void* ws, size_t ws_bytes, int N, int K, int H, int W,
                              float s_rgb, int dim, void* stream);

/* Reads the status word of the last call that used `ws` (synchronous):
 * 0 = ok; bit 1 = a lattice key exceeded the packable range, bit 2 = an image part held
 * more than 2^15 x 6144 distinct vertices (outputs invalid either way). */
int tcam_bilateral_status(const void* ws, int N, int* status);
/* (profiling) per-block phase stamps of the lattice build (s_memrealtime, 100 MHz), or NULL =
 * off: the merge's N * 8 blocks x 4 uint64 (start, table built, vertices placed, end), then the
 * scatter's N * ceil(Pv * (d + 1) / 4096) blocks x 4 (start, before the sort, after it, end). */
void tcam_bilateral_set_debug(void* dbg);

/* Host-compat symbols with the reference SWIG signatures
 * (bilateralfilter.hpp:9-11, colorbilateralfilter.hpp): host buffers in, host
 * buffer out (H2D -> device filter -> D2H on the null stream).  len_* are
 * ignored, as in the reference. */
void bilateralfilter_batch(float* images, int len_images, float* ins,
                           int len_ins, float* outs, int len_outs, int N,
                           int K, int H, int W, float sigmargb,
                           float sigmaxy);
void colorbilateralfilter_batch(float* images, int len_images, float* ins,
                                int len_ins, float* outs, int len_outs, int N,
                                int K, int H, int W, float sigmargb, int DIM);

/* DenseCRFLossFunction (crf/dense_crf_loss.py:33-77) around the filter:
 *   loss[0] = -sum_i seg[i] * AS[i] / N        (deterministic 2-stage sum)
 *   grad[i] = -2 * grad_out[0] * AS[i] / N
 * ws: tcam_crf_energy_ws_bytes() bytes.  n = N * K * H * W. */
size_t tcam_crf_energy_ws_bytes(void);
int tcam_crf_energy(const float* seg, const float* as, long n, int N, float* loss,
                    float* ws, void* stream);
int tcam_crf_grad(const float* as, const float* grad_out, long n, int N, float* grad,
                  void* stream);

/* ------------------------------------------- training step (csrc/train.hip) */
/* The TCAM decoder + segmentation head train with freeze_cl=True
 * (learning/train_wsol.py:685-884, base/model.py:141-142): these kernels are its
 * forward-with-batch-statistics, backward, losses and optimizer step.  S3 tensors as
 * tcam_conv2d_x6; P = B * H * W pixels. */

/* nn.BatchNorm2d.train(): mean / biased-var over (B, H, W) (fp64 partial sums),
 * invstd = 1 / sqrt(var + eps); running stats updated in place (momentum, unbiased
 * var) when run_mean != NULL.  ws: tcam_bn_ws_bytes(P, C). */
size_t tcam_bn_ws_bytes(long P, int C);
int tcam_bn_stats_s3(const void* y, long P, int C, float eps, float momentum, float* mean,
                     float* invstd, float* run_mean, float* run_var, void* ws, void* stream);
/* out = relu(gamma * (y - mean) * invstd + beta)   (Conv2dReLU, base/modules.py:10-49) */
int tcam_bn_relu_s3(const void* y, const float* mean, const float* invstd, const float* gamma,
                    const float* beta, void* out, long P, int C, void* stream);
/* backward of bn_relu: dy, dgamma, dbeta from dout and the forward's y / out. */
int tcam_bn_relu_bwd_s3(const void* dout, const void* out, const void* y, const float* mean,
                        const float* invstd, const float* gamma, void* dy, float* dgamma,
                        float* dbeta, long P, int C, void* ws, void* stream);
/* gradient of F.interpolate(scale_factor=2, mode="nearest") (decoder.py:43):
 * gx (B, H, W) = sum of the 2x2 blocks of gup (B, 2H, 2W). */
int tcam_up2_bwd_s3(const void* gup, void* gx, int B, int C, int H, int W, void* stream);
/* Weight gradient of tcam_conv2d_x6 (same sources / geometry): dW (Cout, Ctot, KH, KW)
 * fp32 = sum over pixels of dy x (deterministic split reduction).  3x3 / stride 1 / pad 1
 * (every trainable decoder conv): bf16-split MFMA at fp32 accuracy (x6, the forward's
 * arithmetic); other shapes: fp32 MFMA.  ws: tcam_conv_wgrad_ws_bytes(...) bytes. */
size_t tcam_conv_wgrad_ws_bytes(const tcam_conv_src* srcs, int nsrc, int B, int Cout,
                                int Hout, int Wout, int KH, int KW);
int tcam_conv_wgrad_s3(const tcam_conv_src* srcs, int nsrc, int B, const void* dy, int Cout,
                       int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                       int cout_store, float* dw, void* ws, size_t ws_bytes, void* stream);
/* The same weight gradient on the same S3 tensors at half x6's MFMA work (the default of the
 * fp32-accurate training step): 3x3 / stride 1 / pad 1 re-splits dy (times a per-channel
 * power-of-two scale, max |dy| s in [2^14, 2^15), divided out exactly) and x into two fp16
 * parts and keeps three products on v_mfma_f32_32x32x16_f16 (f16x3, as tcam_conv2d_f16x3);
 * *oflow = 1 when an x value exceeds the fp16 range (|x| >= 65520: the result is invalid).
 * Other shapes: fp32 MFMA, as tcam_conv_wgrad_s3. */
int tcam_conv_wgrad_s3_f16x3(const tcam_conv_src* srcs, int nsrc, int B, const void* dy,
                             int Cout, int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                             int cout_store, float* dw, void* ws, size_t ws_bytes, int* oflow,
                             void* stream);
/* ---- the f16x3 training step (activations S2, gradients S3; DESIGN.md "Training"):
 * BatchNorm statistics / affine on S2 activations (as the _s3 entries). */
int tcam_bn_stats_s2(const void* y, long P, int C, float eps, float momentum, float* mean,
                     float* invstd, float* run_mean, float* run_var, void* ws, void* stream);
int tcam_bn_relu_s2(const void* y, const float* mean, const float* invstd, const float* gamma,
                    const float* beta, void* out, long P, int C, void* stream);
/* backward of bn_relu: dout and dy S3 (gradients), out and y S2 (the forward's
 * activations); amax (C uint32, or NULL): the per-channel max |dy| as float bit patterns. */
int tcam_bn_relu_bwd_s3s2(const void* dout, const void* out, const void* y, const float* mean,
                          const float* invstd, const float* gamma, void* dy, float* dgamma,
                          float* dbeta, long P, int C, void* ws, uint32_t* amax, void* stream);
/* dy (S3) -> scale[c] (power of two, max |dy_c| scale in [2^14, 2^15)) and dy2 = its scaled
 * S2 copy (P x C x 4 B).  amax: from tcam_bn_relu_bwd_s3s2, or computed here (compute = 1). */
int tcam_dy_scaled_s2(const void* dy, long P, int C, uint32_t* amax, int compute, float* scale,
                      void* dy2, void* stream);
/* The same backward fused with the scaled copy (round 6): dy2 (S2) = dy * scale[c] with
 * scale[c] a power of two from the bound |dy_c| <= |gamma invstd| (max|g| + |mean g| +
 * max|xhat| |mean g xhat|) (max |dy_c| scale < 2^15, no max pass); dy3 (S3 dy, or NULL).
 * out NULL: the ReLU mask is recomputed from y (gamma xhat + beta > 0 as tcam_bn_relu_s2
 * computes it, an fma) — a BN-ReLU; else out's sign (the Bottleneck tail).  C / 8 must
 * divide 256.  ws: tcam_bn_bwd_scaled_ws_bytes(P, C). */
size_t tcam_bn_bwd_scaled_ws_bytes(long P, int C);
int tcam_bn_relu_bwd_scaled_s3s2(const void* dout, const void* out, const void* y,
                                 const float* mean, const float* invstd, const float* gamma,
                                 const float* beta, void* dy3, void* dy2, float* scale,
                                 float* dgamma, float* dbeta, long P, int C, void* ws,
                                 void* stream);
/* The AMP step's BN-ReLU backward in the same two passes (S1 dout / y / out / dy; out NULL:
 * the mask from y).  ws: tcam_bn_ws_bytes(P, C). */
int tcam_bn_relu_bwd_fused_s1(const void* dout, const void* out, const void* y,
                              const float* mean, const float* invstd, const float* gamma,
                              const float* beta, void* dy, float* dgamma, float* dbeta, long P,
                              int C, void* ws, void* stream);
/* 3x3 / stride 1 / pad 1 weight gradient on S2 sources and dy2 / dscale from
 * tcam_dy_scaled_s2: three fp16 products per MAC, the reduction divides by dscale exactly.
 * ws: tcam_conv_wgrad_ws_bytes(...). */
int tcam_conv_wgrad_s2_f16x3(const tcam_conv_src* srcs, int nsrc, int B, const void* dy2,
                             const float* dscale, int Cout, int Hout, int Wout, int KH, int KW,
                             int pad_h, int pad_w, int cout_store, float* dw, void* ws,
                             size_t ws_bytes, void* stream);
/* PyTorch conv weight -> the split f16x3 operand (Kpad/32, 4, 2, Mpad, 8) fp16 and its
 * per-column power-of-two scales wscale (Mpad floats), on the device (mode / c0 /
 * cout_sel / cin_pad as tcam_pack_weight_x6); kdiv (or NULL): a power of two per input
 * channel of the selected conv that the weights are divided by (mode 1: dy's scales). */
int tcam_pack_weight_f16x3(const float* w, void* out, float* wscale, int mode, int CoutW,
                           int CtotW, int KH, int KW, int c0, int cout_sel, int cin_pad,
                           const float* kdiv, void* stream);
/* Batched weight packs (a trainer's repack after each optimizer step): n items, each the
 * arguments of tcam_pack_weight_f16 (f16x3 == 0; wscale / kdiv unused) or of
 * tcam_pack_weight_f16x3 (f16x3 == 1), packed in one launch (two for f16x3: the column
 * scales, then the parts); results equal the per-item calls bit for bit.  `table`: device
 * memory of tcam_pack_table_bytes(n) bytes for the descriptor table (copied on the stream
 * only when it differs from the table last copied to that address). */
typedef struct tcam_pack_item {
    const float* w;
    void* out;
    float* wscale;
    const float* kdiv;
    int mode, CoutW, CtotW, KH, KW, c0, cout_sel, cin_pad;
} tcam_pack_item;
size_t tcam_pack_table_bytes(int n);
int tcam_pack_weights(const tcam_pack_item* items, int n, int f16x3, void* table, void* stream);
/* Fused ResNet50 layer-1 bottleneck on the f16x3 path (replaces the three
 * tcam_conv2d_f16x3 calls of one encoders/resnet.py:175-232 Bottleneck at stride 1, Cmid 64,
 * Cout 256): x (B, H, W, cin) S2 -> out (B, H, W, 256) S2.  w1 / w2 / w3: the packed f16x3
 * weights of conv1 (1x1, cin -> 64), conv2 (3x3 pad 1, 64 -> 64) and conv3 (1x1, 64 -> 256;
 * with ds = 1 the K-concat [conv3 | downsample] of (conv2 out, x), cin = 64), each with its
 * scales s* and (BN-folded) bias b*; without ds, x (cin = 256) is the residual.  ReLU after
 * each conv.  Bit-identical to the three unfused calls; out-of-range values set *oflow. */
int tcam_bottleneck_f16x3(const void* x, int B, int H, int W, int cin, const void* w1,
                          const float* s1, const float* b1, const void* w2, const float* s2,
                          const float* b2, const void* w3, const float* s3, const float* b3,
                          int ds, void* out, int* oflow, void* stream);
/* The same fused block on the AMP path: S1 activations, the single-part fp16 weights of
 * tcam_conv2d_f16 (no scales), S1 output; bit-identical to the three tcam_conv2d_f16 calls. */
int tcam_bottleneck_f16(const void* x, int B, int H, int W, int cin, const void* w1,
                        const float* b1, const void* w2, const float* b2, const void* w3,
                        const float* b3, int ds, void* out, void* stream);
/* (profiling) per-block phase stamps of tcam_bottleneck_f16x3: 4 uint64 per block
 * (s_memrealtime, 100 MHz: start, after conv1, after conv2, end), or NULL = off. */
void tcam_bottleneck_set_debug(void* dbg);
/* tcam_conv2d_f16x3 (S2 sources, f16x3 weights + wscale) writing an S3 output: the data
 * gradient dx = conv(dy2, W / dscale) of the f16x3 step, dx ~ 1e-7 kept in S3.  No
 * residual. */
int tcam_conv2d_f16x3_s3out(const tcam_conv_src* srcs, int nsrc, int B, const void* wt,
                            const float* wscale, const float* bias, void* out, int Cout,
                            int Hout, int Wout, int KH, int KW, int pad_h, int pad_w, int relu,
                            int out_cstride, int out_coff, void* ws, size_t ws_bytes,
                            void* stream);
/* Launch timing (bench.py's roofline): bind hipEvent_t `start` to the next conv kernel
 * dispatch and `stop` to every conv dispatch (hipExtLaunchKernelGGL) until disarmed with
 * (NULL, NULL).  Covers tcam_conv2d_x6 / _f16x3 / _f16 (+ _multi) and tcam_stem_f16x3. */
int tcam_timer_arm(void* start, void* stop);
/* Test / A-B hook: 1 = run the 3x3 wgrad on the fp32 MFMA instead of x6 (process-wide). */
int tcam_wgrad_force_fp32(int on);
/* PyTorch conv weight (CoutW, CtotW, KH, KW) fp32 -> the packed split operand of
 * tcam_conv2d_x6.  mode 0: as is.  mode 1 (data gradient): the conv whose outputs are
 * W's input channels [c0, c0 + cout_sel) and whose inputs are W's outputs (zero-padded to
 * cin_pad channels), taps rotated 180 degrees, so dx = tcam_conv2d_x6(dy) (stride 1,
 * pad KH-1-pad).  cout_store in the wgrad: rows of dW written (<= Cout, padded dy). */
int tcam_pack_weight_x6(const float* w, void* out, int mode, int CoutW, int CtotW, int KH,
                        int KW, int c0, int cout_sel, int cin_pad, void* stream);
/* Adjoint of tcam_up2_resize_s3 (B, C, H, W) -> (Ho, Wo): gx from g. */
int tcam_up2_resize_bwd_s3(const void* g, void* gx, int B, int C, int H, int W, int Ho, int Wo,
                           void* stream);
/* out[c] = sum_{b, hw} x[b, c, hw] (deterministic; bias gradients). */
size_t tcam_chansum_ws_bytes(int B, int C, long HW);
int tcam_chansum_nchw(const float* x, int B, int C, long HW, float* out, void* ws,
                      void* stream);
/* S = softmax(fcams, dim=1) for 2-channel fcams (B, 2, HW). */
int tcam_softmax2(const float* fcams, float* S, int B, long HW, void* stream);
/* TCAM losses on fcams (B, 2, HW) (losses/tcam.py:48-278):
 *   sl   = lam_sl * CrossEntropy(fcams, seeds, ignore_index=-255)      (seeds NULL: off)
 *   crf  = lam_crf * -sum(S * AS) / B,  AS = bilateral(S)              (AS NULL: off)
 *   size = lam_size * 0.5 * sum_c mean_b ELB_t(-sum_hw S[b, c])        (lam_size 0: off)
 * losses[4] = {total, sl, crf, size}; dfcams = d total / d fcams (through the softmax;
 * the CRF term's gradient is -2 lam AS / B as DenseCRFLossFunction.backward).
 * ws: tcam_tcam_loss_ws_bytes(B, HW). */
size_t tcam_tcam_loss_ws_bytes(int B, long HW);
int tcam_tcam_losses(const float* fcams, const float* S, const int32_t* seeds, const float* AS,
                     int B, long HW, float lam_sl, float lam_crf, float lam_size, float elb_t,
                     float* losses, float* dfcams, void* ws, void* stream);
/* The same with one more term computed by the caller (RgbJointConRanFieldTcams,
 * losses/tcam.py:158-232): extra[0] its value (added to the total, stored as losses[4] —
 * losses then holds 5 floats) and gx (B, 2, HW) its d loss / d S, added before the softmax
 * backward.  Both NULL = tcam_tcam_losses. */
int tcam_tcam_losses_ex(const float* fcams, const float* S, const int32_t* seeds,
                        const float* AS, const float* gx, const float* extra, int B, long HW,
                        float lam_sl, float lam_crf, float lam_size, float elb_t, float* losses,
                        float* dfcams, void* ws, void* stream);
/* RgbJointConRanFieldTcams.pair_samples (losses/tcam.py:207-232) and its adjoint.
 * gather: out (G, C, H, L*W) [g, c, y, p*W + x] = src (B, C, H, W) [idx[g*L + p], c, y, x].
 * scatter: dst[b, c, y, x] = (accumulate ? dst : 0) + coef * sum_k mosaic[g_k, c, y,
 * p_k*W + x] over the occurrences k of frame b, occ[occ_start[b] .. occ_start[b+1]) each
 * g*L + p, summed in that order (deterministic; a frame with no occurrence is left as is
 * when accumulating, else zeroed). */
int tcam_mosaic_gather(const float* src, const int32_t* idx, int G, int L, int C, int H, int W,
                       float* out, void* stream);
int tcam_mosaic_scatter(const float* mosaic, const int32_t* occ_start, const int32_t* occ,
                        int B, int L, int C, int H, int W, float coef, int accumulate,
                        float* dst, void* stream);
/* torch.optim.SGD step (momentum, dampening, weight_decay, nesterov; first = 1 on the
 * first step: buf = d); the gradient is read as g * grad_scale (1 / world for the
 * DDP average of an all-reduced sum). */
int tcam_sgd_step(float* p, const float* g, float* buf, long n, float lr, float momentum,
                  float dampening, float weight_decay, int nesterov, int first,
                  float grad_scale, void* stream);
/* The same step gated on the device by the all-reduced loss (learning/train_wsol.py:1181,
 * ``if loss.requires_grad and torch.isfinite(loss).item()``): when *gate is not finite the
 * parameters and momentum stay untouched and *skipped (if non-null) is incremented; else
 * the step is applied and *steps incremented.  The first applied step (*steps == 0)
 * initialises the momentum buffer. */
int tcam_sgd_step_gated(float* p, const float* g, float* buf, long n, float lr, float momentum,
                        float dampening, float weight_decay, int nesterov, float grad_scale,
                        const float* gate, int* steps, int* skipped, void* stream);

/* AMP (train_wsol.py:1077 GradScaler(enabled=amp), 1180-1183): the training kernels above on
 * S1 tensors (fp16 in / out, fp32 arithmetic inside; tcam_conv_wgrad_s1: one fp16 product on
 * v_mfma_f32_32x32x16_f16 for 3x3 / stride 1, fp32 MFMA otherwise, dW rounded to fp16 as an
 * autocast conv's weight gradient), and torch.cuda.amp.GradScaler on the device:
 *   tcam_amp_unscale: g *= 1 / *scale; *found_inf = 1 when any g is not finite (unscale_);
 *   tcam_sgd_step_amp: gate = {all-reduced loss, all-reduced found_inf}: the SGD step of
 *     tcam_sgd_step_gated runs when gate[0] is finite and gate[1] == 0; then scaler.update():
 *     gate[1] != 0 -> *scale *= backoff_factor, *tracker = 0; a clean step -> ++*tracker and
 *     at growth_interval *scale *= growth_factor; a non-finite loss changes nothing (the
 *     reference skips backward, step and update). */
int tcam_bn_stats_s1(const void* y, long P, int C, float eps, float momentum, float* mean,
                     float* invstd, float* run_mean, float* run_var, void* ws, void* stream);
int tcam_bn_relu_s1(const void* y, const float* mean, const float* invstd, const float* gamma,
                    const float* beta, void* out, long P, int C, void* stream);
int tcam_bn_relu_bwd_s1(const void* dout, const void* out, const void* y, const float* mean,
                        const float* invstd, const float* gamma, void* dy, float* dgamma,
                        float* dbeta, long P, int C, void* ws, void* stream);
int tcam_up2_bwd_s1(const void* gup, void* gx, int B, int C, int H, int W, void* stream);
int tcam_up2_resize_bwd_s1(const void* g, void* gx, int B, int C, int H, int W, int Ho, int Wo,
                           void* stream);
int tcam_conv_wgrad_s1(const tcam_conv_src* srcs, int nsrc, int B, const void* dy, int Cout,
                       int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                       int cout_store, float* dw, void* ws, size_t ws_bytes, void* stream);
/* tcam_pack_weight_x6's packing as the fp16 operand of tcam_conv2d_f16. */
int tcam_pack_weight_f16(const float* w, void* out, int mode, int CoutW, int CtotW, int KH,
                         int KW, int c0, int cout_sel, int cin_pad, void* stream);
int tcam_amp_unscale(float* g, long n, const float* scale, float* found_inf, void* stream);
int tcam_sgd_step_amp(float* p, const float* g, float* buf, long n, float lr, float momentum,
                      float dampening, float weight_decay, int nesterov, float grad_scale,
                      const float* gate, int* steps, int* skipped, float* scale, int* tracker,
                      float growth_factor, float backoff_factor, int growth_interval,
                      void* stream);

/* ------------------------------------ encoder training step (csrc/enc_train.hip) */
/* Stage 1 (task STD_CL, learning/train_wsol.py:710-714 with --freeze_encoder False,
 * README.md:239-266): the ResNet50 encoder + WGAP head trained end to end.  The convolutions
 * are the kernels above (forward: tcam_conv2d_f16x3 / tcam_conv2d_f16; data gradient: the same
 * conv of dy with tcam_pack_weight_* mode 1); BatchNorm statistics / BN-ReLU / its backward are
 * the tcam_bn_* entries.  Suffixes: _s2 / _s3s2 the fp32-accurate step (activations S2,
 * gradients S3), _s1 the AMP step (--amp True: autocast's fp16 tensors). */
/* The Bottleneck tail (encoders/resnet.py:221-232): out = relu(bn3(y) + r), r = bn_ds(yd)
 * (projection shortcut: yd, meand .. betad given, res NULL) or res (identity: yd NULL).
 * _s1: each BN output and the sum rounded to fp16 (autocast). */
int tcam_bn_add_relu_s2(const void* y, const float* mean, const float* invstd, const float* gamma,
                        const float* beta, const void* yd, const float* meand,
                        const float* invstdd, const float* gammad, const float* betad,
                        const void* res, void* out, long P, int C, void* stream);
int tcam_bn_add_relu_s1(const void* y, const float* mean, const float* invstd, const float* gamma,
                        const float* beta, const void* yd, const float* meand,
                        const float* invstdd, const float* gammad, const float* betad,
                        const void* res, void* out, long P, int C, void* stream);
/* r = a + [o > 0] d: the identity shortcut's gradient (dout masked by relu3) added to the
 * conv1 data gradient; a, d, r gradients (S3 / S1), o the block output (S2 / S1). */
int tcam_grad_add_mask_s3s2(const void* a, const void* d, const void* o, void* r, long P, int C,
                            void* stream);
int tcam_grad_add_mask_s1(const void* a, const void* d, const void* o, void* r, long P, int C,
                          void* stream);
/* MaxPool2d(3, 2, 1) backward (encoders/resnet.py:97): gin (B, H, W, C) = the sum of gout
 * (B, Ho, Wo, C) over the outputs whose window argmax (first maximum in (kh, kw) order, NaN
 * wins: torch's max_pool2d rule) is that pixel, recomputed from the forward input x.
 * ws: tcam_maxpool_bwd_ws_bytes(B, C, Ho, Wo). */
size_t tcam_maxpool_bwd_ws_bytes(int B, int C, int Ho, int Wo);
int tcam_maxpool3x3s2_bwd_s3s2(const void* gout, const void* x, void* gin, void* ws, int B, int C,
                               int H, int W, int Ho, int Wo, void* stream);
int tcam_maxpool3x3s2_bwd_s1(const void* gout, const void* x, void* gin, void* ws, int B, int C,
                             int H, int W, int Ho, int Wo, void* stream);
/* Zero insertion (the data gradient of a stride-2 conv = the stride-1 conv of dy spread onto
 * the input grid): out (B, H, W, C) [2y][2x] = in (B, Hi, Wi, C) [y][x], 0 elsewhere; gbytes
 * = bytes per 8-channel group (16 S1, 32 S2, 48 S3). */
int tcam_zero_up2(const void* in, void* out, int gbytes, int B, int C, int H, int W, int Hi,
                  int Wi, void* stream);
/* im2col in 8-channel groups (the stem's weight gradient as a 1x1 GEMM over pixels):
 * out (B, Ho, Wo, KH*KW*C) [p][(kh*KW + kw)*C + c] = x (B, H, W, C) [stride*oy - pad + kh]
 * [stride*ox - pad + kw][c], 0 outside the frame; gbytes 16 (S1) or 32 (S2). */
int tcam_im2col(const void* x, void* out, int gbytes, int B, int C, int H, int W, int KH, int KW,
                int stride, int pad, int Ho, int Wo, void* stream);
/* 1x1 weight gradient (every Bottleneck conv1 / conv3 / projection, resnet.py:198-216):
 * dW (Cout, Cin) fp32 = sum over the B*Ho*Wo output pixels p of dy[p] x[stride * p].
 * _s2_f16x3: x S2, dy2 / dscale = tcam_dy_scaled_s2's scaled S2 copy (three fp16 products per
 * MAC on v_mfma_f32_32x32x16_f16, the sum divided by dscale exactly); _s1: x, dy S1 (one
 * product; dW rounded to fp16, an autocast conv's weight gradient).  Deterministic (fixed
 * pixel splits reduced in order).  ws: tcam_wgrad11_ws_bytes(...). */
size_t tcam_wgrad11_ws_bytes(int B, int Cin, int Hin, int Win, int stride, int Cout, int Ho,
                             int Wo);
int tcam_wgrad11_s2_f16x3(const void* x, int B, int Cin, int Hin, int Win, int stride,
                          const void* dy2, const float* dscale, int Cout, int Ho, int Wo,
                          float* dw, void* ws, size_t ws_bytes, void* stream);
int tcam_wgrad11_s1(const void* x, int B, int Cin, int Hin, int Win, int stride, const void* dy,
                    int Cout, int Ho, int Wo, float* dw, void* ws, size_t ws_bytes, void* stream);
/* Weight gradient of any KH x KW / stride / pad conv with dy S3 and S2 sources (the 7x7/2 stem,
 * the 3x3/2 conv2 of layer2.0): fp32 MFMA, deterministic.  ws: the _generic_ws_bytes. */
size_t tcam_conv_wgrad_generic_ws_bytes(const tcam_conv_src* srcs, int nsrc, int B, int Cout,
                                        int Hout, int Wout, int KH, int KW);
int tcam_conv_wgrad_s3s2(const tcam_conv_src* srcs, int nsrc, int B, const void* dy, int Cout,
                         int Hout, int Wout, int KH, int KW, int pad_h, int pad_w,
                         int cout_store, float* dw, void* ws, size_t ws_bytes, void* stream);
/* WGAP head for training (poolings/core.py:109-115): pooled (B, C) = mean over the HW pixels of
 * x (B, HW, C) (fixed-order sums), logits (B, K) = pooled fc_w^T + fc_b; _s1 rounds pooled and
 * logits to fp16 (autocast).  ws: tcam_cls_pool_ws_bytes(B, C). */
size_t tcam_cls_pool_ws_bytes(int B, int C);
int tcam_cls_fwd_s2(const void* x, int B, long HW, int C, const float* w, const float* bias,
                    int K, float* pooled, float* logits, void* ws, void* stream);
int tcam_cls_fwd_s1(const void* x, int B, long HW, int C, const float* w, const float* bias,
                    int K, float* pooled, float* logits, void* ws, void* stream);
/* ClLoss (losses/std.py:19-53): loss[0] = lam * CrossEntropy(logits, labels) (mean over B);
 * dlogits (or NULL) = d loss / d logits times *gscale (the AMP loss scale; NULL = 1). */
int tcam_ce_loss(const float* logits, const int32_t* labels, int B, int K, float lam,
                 const float* gscale, float* loss, float* dlogits, void* stream);
/* fc backward: dw (K, C), db (K), dpooled (B, C) from dlogits (B, K); r16: fp16 gradients. */
int tcam_cls_bwd(const float* dlogits, const float* pooled, const float* w, int B, int K, int C,
                 int r16, float* dw, float* db, float* dpooled, void* stream);
/* AdaptiveAvgPool2d(1) backward: dout (B, HW, C) = dpooled / HW (S3 / S1). */
int tcam_pool_bwd_s3(const float* dpooled, int B, long HW, int C, void* dout, void* stream);
int tcam_pool_bwd_s1(const float* dpooled, int B, long HW, int C, void* dout, void* stream);

/* ------------------------------------------------------------- seeding */
/*
 * TCAM pseudo-label seeds, batched: TCAMSeeder.forward (dlib/cams/tcam_seeding.py:187-258)
 * with _OneSample/_SFG/_SBG (:409-563) and GetRoiSingleCam (:303-406), one workgroup per
 * frame.  cams: (B, H, W) fp32 (the (B,1,H,W) cams_inter); roi: NULL or (B, H, W) 0/1
 * (the caller's roi, used only when use_roi); seeds: (B, H, W) int32 = 1 fg, 0 bg,
 * ignore_idx elsewhere.  seed_tech 0 = seed_uniform, 1 = seed_weighted; roi_method
 * 0 = roi_all, 1 = roi_high_density, 2 = largest.  The multinomial draws are
 * topk(p / q) with q ~ Exp(1) from Philox4x32-10(pixel, frame, offset; seed).
 * roi_out (optional): the (eroded) ROI actually used; th_out (optional): Otsu threshold.
 * H * W <= 320 * 320.  ws: tcam_seeder_ws_bytes(B, H, W).
 */
size_t tcam_seeder_ws_bytes(int B, int H, int W);
/* prepare_std_cams_disq (learning/train_wsol.py:417-432): stage-1 CAMs (B, h, w) ->
 * nan_to_num -> bilinear (align_corners=False) to (B, Ho, Wo) -> nan_to_num. */
int tcam_prepare_std_cams(const float* cams, float* out, int B, int h, int w, int Ho, int Wo,
                          void* stream);
int tcam_tcam_seeder(const float* cams, const uint8_t* roi, int32_t* seeds, int B, int H,
                     int W, int seed_tech, int min_, int max_, float max_p, float min_p,
                     int fg_erode_k, int fg_erode_iter, int ksz, int ignore_idx,
                     int roi_method, double p_min_area_roi, int use_roi,
                     unsigned long long seed, unsigned long long offset, uint8_t* roi_out,
                     float* th_out, void* ws, size_t ws_bytes, void* stream);
/* GetRoiSingleCam.__call__ (tcam_seeding.py:312-396), batched: roi_out (B, H, W) 0/1,
 * bbox_out (B, 4) int32 x0 y0 x1 y1 (the mask is bbox[y0:y1, x0:x1]), th_out (B,) the
 * Otsu threshold in [0, 255] (thresh < 0) or thresh * 255. */
int tcam_get_roi(const float* cams, int B, int H, int W, int roi_method,
                 double p_min_area_roi, double thresh, const double* thresh_b,
                 uint8_t* roi_out, int32_t* bbox_out, float* th_out, void* ws,
                 size_t ws_bytes, void* stream);
/* thresh_b: NULL or (B,) per-frame thresholds in [0, 1] (< 0 or NaN: Otsu) — the
 * std_cams_thresh_file values the loader passes per frame (wsol_loader.py:573-611). */
/* STOtsu ROI threshold of stored CAMs (inference_wsol.py:1107-1124, 1144-1159):
 * th_out[b] = STOtsu(floor(bilinear_align_corners(cams[b], S x S) * 255)) in [0, 255]
 * (cams/core_seeding.py:23-56); the reference writes th / 255 to <tag>.txt. */
int tcam_stotsu_roi_thresh(const float* cams, int B, int h, int w, int S, float* th_out,
                           void* stream);

/* ---- frame preprocessing (datasets/wsol_loader.py:903-908 eval,
 * :960-970 train transforms).  Replaces the per-frame PIL Resize(BILINEAR) + ToTensor +
 * Normalize of the reference's DataLoader workers for a batch of decoded frames. */
/* Pillow's BILINEAR resample coefficients (Resample.c precompute_coeffs +
 * normalize_coeffs_8bpc), host function: bounds (out_size, 2) = (first tap, taps), kk
 * (out_size, ksize) int32 with 22 fraction bits.  Returns ksize (< 0: error); with
 * bounds / kk NULL it only returns ksize. */
int tcam_resample_coeffs(int in_size, int out_size, int* bounds, int* kk);
/* frames (B, Hin, Win, 3) uint8 (device) -> resize to (Rh, Rw) with the coefficients above
 * (device copies), crop (th, tw) at crop[b] = (top, left) (device, or NULL = (0, 0)), then
 * flip[b] (device uint8, or NULL) -> norm = (x / 255 - mean) / std (B, 3, th, tw) fp32,
 * raw = x as float (B, 3, th, tw), u8 = x (B, th, tw, 3); each output optional (NULL).
 * mean3 / std3: host arrays of 3 floats.  Bit-identical to Pillow + torchvision. */
int tcam_frames_preprocess(const uint8_t* frames, int B, int Hin, int Win, const int* bh,
                           const int* kh, int ksh, int Rw, const int* bv, const int* kv,
                           int ksv, int Rh, const int* crop, const uint8_t* flip, int th,
                           int tw, const float* mean3, const float* std3, float* norm,
                           float* raw, uint8_t* u8, void* stream);


/* ------------------------------------------------------------ JPEG decode */
/*
 * Batched baseline-JPEG decode, bit-identical to the reference loader's
 * Image.open(path).convert('RGB') (datasets/wsol_loader.py:581-582: Pillow 12.2 over
 * libjpeg-turbo, JDCT_ISLOW, fancy upsampling, jdcolor.c YCbCr->RGB).  Supported:
 * SOF0/SOF1 8-bit Huffman, one interleaved scan (or grayscale), any integral chroma
 * subsampling, restart intervals, JFIF / Adobe / component-id colour spaces.
 */
#define TCAM_JPEG_E_NOTJPEG (-20)      /* no SOI marker */
#define TCAM_JPEG_E_UNSUPPORTED (-21)  /* progressive / arithmetic / 12-bit / CMYK / multi-scan */
#define TCAM_JPEG_E_CORRUPT (-22)      /* malformed markers, tables or restart segments */
/* Host: parse n files (data[i], len[i]) and pack headers, deduplicated Huffman tables and
 * the unstuffed entropy bytes into one staging blob.  Always fills
 * sizes[4] = {blob bytes, device workspace bytes, output bytes, total 8x8 blocks} and
 * dims[3*i] = {height, width, status} (dims may be NULL); with blob == NULL only sizes.
 * Returns 0, TCAM_E_NOMEM (cap too small) or the first image's TCAM_JPEG_E_* code. */
int tcam_jpeg_pack(const uint8_t* const* data, const size_t* len, int n, void* blob,
                   size_t cap, int64_t* sizes, int* dims);
/* Device: decode a packed batch.  host_blob = the packed blob (launch geometry is read
 * from it), dev_blob = its copy in device memory, ws = sizes[1] bytes of device scratch,
 * out = sizes[2] bytes: image i as (h, w, 3) uint8 RGB at the running offset
 * sum_{j<i} h_j * w_j * 3 (so a same-size batch is one (n, h, w, 3) tensor). */
int tcam_jpeg_decode(const void* host_blob, const void* dev_blob, void* ws, size_t ws_bytes,
                     uint8_t* out, void* stream);
/* Diagnostics: later decodes record the self-synchronisation round count of every Huffman
 * workgroup in dev_rounds (device int array; NULL = off).  Returns the workgroup count of
 * host_blob (0 if NULL). */
int tcam_jpeg_debug_rounds(const void* host_blob, int* dev_rounds);

#ifdef __cplusplus
}
#endif
#endif /* TCAM_HIP_H */
