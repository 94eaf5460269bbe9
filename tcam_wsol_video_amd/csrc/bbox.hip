// CAM -> bbox on the GPU: a batched, exact replacement of
// compute_bboxes_from_scoremaps (metrics/wsol_metrics.py:127-197) with
// multi_contour_eval=False, i.e. for every threshold level L the box of
//   max(cv2.findContours(u8 > L, RETR_TREE, CHAIN_APPROX_SIMPLE), key=contourArea)
// followed by BoxEvaluator.accumulate (wsol_metrics.py:295-370).
//
// OpenCV semantics reproduced (contours.cpp, Suzuki-Abe border following on
// a zero-padded copy; contourArea = shoelace over the chain vertices):
//  * foreground is 8-connected, background 4-connected;
//  * the outer contour of a component C encloses C plus its holes, and its
//    shoelace area through pixel centres equals, summed over every 2x2
//    window of pixel centres, 1 if all four pixels lie in fill(C), 1/2 if
//    exactly three do, 0 otherwise;
//  * fill(C) of the top-level components are the 8-connected components of
//    {psi > L}, psi = grayscale hole-fill of u8 (min over 4-paths from the
//    image border of the max along the path);
//  * hole contours and contours nested in holes never win the max (strictly
//    smaller than their enclosing outer contour, and listed after it);
//  * ties between top-level contours resolve to the first in OpenCV's list
//    order = the LAST discovered in raster order = the largest raster index
//    of the component's first pixel;
//  * boundingRect of the outer contour = bbox of C.
// The oracle (oracle/contours.c, a restatement of the border follower) pins
// this characterisation on random images in tests/test_bbox_oracle.py.
//
// Kernels:
//  fill_kernel   one workgroup per frame: vmax = max(u8); psi by alternating
//                row/column min-max sweeps to the fixpoint.
//  level_kernel  one workgroup per (frame, level): block-based union-find
//                (2x2 pixel blocks, 8-connectivity) in LDS, window-area
//                accumulation, argmax with OpenCV's tie order, bbox.
//  accumulate    one thread per (frame, tau): IoU vs GT (+1 inclusive
//                convention, fp64) and the BoxEvaluator counters.
#include "common.h"

namespace {

constexpr int MAXH = 224, MAXW = 224;
constexpr int MAXP = 228;                 // padded row pitch in bytes
constexpr int MAXBH = MAXH / 2, MAXBW = MAXW / 2;
constexpr uint32_t INACT = 0xFFFFFFFFu;
constexpr int NTB = 1024;

__host__ __device__ inline int pitch_of(int W) {
    int d = (W + 3) / 4;
    if ((d & 1) == 0) d += 1;  // odd dword pitch: conflict-free column walks
    return 4 * d;
}

// Block-wide reductions over NTB threads (16 waves).
__device__ inline int block_max_i(int v, int* red) {
    v = wave_max_i(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = red[0];
        for (int i = 1; i < NTB / 64; ++i) m = max(m, red[i]);
        red[NTB / 64] = m;
    }
    __syncthreads();
    return red[NTB / 64];
}
__device__ inline int block_min_i(int v, int* red) {
    return -block_max_i(-v, red);
}

// ---------------------------------------------------------------- fill
__global__ __launch_bounds__(NTB) void fill_kernel(const uint8_t* __restrict__ cam_u8,
                                                   uint8_t* __restrict__ psi_out,
                                                   int32_t* __restrict__ vmax_out, int H,
                                                   int W) {
    __shared__ uint8_t img[MAXH * MAXP];
    __shared__ uint8_t psi[MAXH * MAXP];
    __shared__ int red[NTB / 64 + 1];
    __shared__ int changed;
    const int b = blockIdx.x;
    const int P = pitch_of(W);
    const uint8_t* src = cam_u8 + (long)b * H * W;
    int vm = 0;
    for (int i = threadIdx.x; i < H * W; i += NTB) {
        int y = i / W, x = i - y * W;
        uint8_t v = src[i];
        img[y * P + x] = v;
        psi[y * P + x] = 255;
        vm = max(vm, (int)v);
    }
    vm = block_max_i(vm, red);
    if (threadIdx.x == 0) vmax_out[b] = vm;
    // psi(p) = max(u8(p), min over 4-neighbours psi(q)), outside = -1.
    // Row sweeps (thread per row) alternate with column sweeps (thread per
    // column); each thread only reads/writes its own line, values only
    // decrease, and the loop stops after a full cycle without change.
    for (;;) {
        if (threadIdx.x == 0) changed = 0;
        __syncthreads();
        int ch = 0;
        if (threadIdx.x < H) {
            uint8_t* row = psi + threadIdx.x * P;
            const uint8_t* irow = img + threadIdx.x * P;
            int prev = -1;
            for (int x = 0; x < W; ++x) {
                int cur = row[x];
                int nv = max((int)irow[x], min(cur, prev));
                if (nv != cur) { row[x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
            prev = -1;
            for (int x = W - 1; x >= 0; --x) {
                int cur = row[x];
                int nv = max((int)irow[x], min(cur, prev));
                if (nv != cur) { row[x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
        }
        __syncthreads();
        if (threadIdx.x < W) {
            const int x = threadIdx.x;
            int prev = -1;
            for (int y = 0; y < H; ++y) {
                int cur = psi[y * P + x];
                int nv = max((int)img[y * P + x], min(cur, prev));
                if (nv != cur) { psi[y * P + x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
            prev = -1;
            for (int y = H - 1; y >= 0; --y) {
                int cur = psi[y * P + x];
                int nv = max((int)img[y * P + x], min(cur, prev));
                if (nv != cur) { psi[y * P + x] = (uint8_t)nv; ch = 1; }
                prev = nv;
            }
        }
        if (ch) changed = 1;  // benign same-value race
        __syncthreads();
        if (!changed) break;
        __syncthreads();
    }
    uint8_t* dst = psi_out + (long)b * H * W;
    for (int i = threadIdx.x; i < H * W; i += NTB) {
        int y = i / W, x = i - y * W;
        dst[i] = psi[y * P + x];
    }
}

// --------------------------------------------------------------- levels
__device__ inline uint32_t find_root(const volatile uint32_t* lab, uint32_t x) {
    uint32_t p = lab[x];
    while (p != x) {
        x = p;
        p = lab[x];
    }
    return x;
}

__device__ inline void unite(uint32_t* lab, uint32_t a, uint32_t b) {
    for (;;) {
        a = find_root(lab, a);
        b = find_root(lab, b);
        if (a == b) return;
        if (a > b) { uint32_t t = a; a = b; b = t; }
        uint32_t old = atomicMin(&lab[b], a);
        if (old == b) return;
        b = old;
    }
}

__global__ __launch_bounds__(NTB) void level_kernel(const uint8_t* __restrict__ psi_g,
                                                    const int32_t* __restrict__ vmax,
                                                    int32_t* __restrict__ boxes, int H, int W) {
    __shared__ uint8_t psi[MAXH * MAXP];
    __shared__ uint32_t lab[MAXBH * MAXBW];
    __shared__ uint32_t area[MAXBH * MAXBW];
    __shared__ int red[NTB / 64 + 1];

    const int b = blockIdx.x / 255;
    const int L = blockIdx.x % 255;
    int32_t* box = boxes + ((long)b * 256 + L) * 4;
    if (L >= vmax[b]) {
        if (threadIdx.x < 4) box[threadIdx.x] = 0;
        return;
    }
    const int P = pitch_of(W);
    const int BH = (H + 1) / 2, BW = (W + 1) / 2, NB = BH * BW;
    const uint8_t* src = psi_g + (long)b * H * W;
    for (int i = threadIdx.x; i < H * W; i += NTB) {
        int y = i / W, x = i - y * W;
        psi[y * P + x] = src[i];
    }
    __syncthreads();
    auto F = [&](int y, int x) -> int {
        return ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) && (psi[y * P + x] > L);
    };
    // 1. block activity.
    for (int i = threadIdx.x; i < NB; i += NTB) {
        int by = i / BW, bx = i - by * BW;
        int y = 2 * by, x = 2 * bx;
        bool act = F(y, x) | F(y, x + 1) | F(y + 1, x) | F(y + 1, x + 1);
        lab[i] = act ? (uint32_t)i : INACT;
        area[i] = 0;
    }
    __syncthreads();
    // 2. union with the left, top-left, top and top-right blocks.
    for (int i = threadIdx.x; i < NB; i += NTB) {
        if (lab[i] == INACT) continue;
        int by = i / BW, bx = i - by * BW;
        int y = 2 * by, x = 2 * bx;
        int p00 = F(y, x), p01 = F(y, x + 1), p10 = F(y + 1, x), p11 = F(y + 1, x + 1);
        (void)p11;
        if (bx > 0 && (p00 | p10) && (F(y, x - 1) | F(y + 1, x - 1))) unite(lab, i, i - 1);
        if (by > 0) {
            if ((p00 | p01) && (F(y - 1, x) | F(y - 1, x + 1))) unite(lab, i, i - BW);
            if (bx > 0 && p00 && F(y - 1, x - 1)) unite(lab, i, i - BW - 1);
            if (bx + 1 < BW && p01 && F(y - 1, x + 2)) unite(lab, i, i - BW + 1);
        }
    }
    __syncthreads();
    // 3. flatten.
    for (int i = threadIdx.x; i < NB; i += NTB)
        if (lab[i] != INACT) lab[i] = find_root(lab, i);
    __syncthreads();
    // 4. window areas (half units) into the root's slot.
    {
        const int NWx = W + 1, NWin = (H + 1) * (W + 1);
        const int per = (NWin + NTB - 1) / NTB;
        const int w0 = threadIdx.x * per, w1 = min(NWin, w0 + per);
        uint32_t cur = INACT, acc = 0;
        for (int w = w0; w < w1; ++w) {
            int wy = w / NWx - 1, wx = w % NWx - 1;
            int f00 = F(wy, wx), f01 = F(wy, wx + 1), f10 = F(wy + 1, wx), f11 = F(wy + 1, wx + 1);
            int c = f00 + f01 + f10 + f11;
            if (c < 3) continue;
            int py = f00 ? wy : (f01 ? wy : wy + 1);
            int px = f00 ? wx : (f01 ? wx + 1 : (f10 ? wx : wx + 1));
            uint32_t r = lab[(py >> 1) * BW + (px >> 1)];
            if (r != cur) {
                if (cur != INACT && acc) atomicAdd(&area[cur], acc);
                cur = r;
                acc = 0;
            }
            acc += (uint32_t)(c - 2);
        }
        if (cur != INACT && acc) atomicAdd(&area[cur], acc);
    }
    __syncthreads();
    // 5. max area over roots.
    int ma = -1;
    for (int i = threadIdx.x; i < NB; i += NTB)
        if (lab[i] == (uint32_t)i) ma = max(ma, (int)area[i]);
    ma = block_max_i(ma, red);
    if (ma < 0) {  // no component (cannot happen for L < vmax)
        if (threadIdx.x < 4) box[threadIdx.x] = 0;
        return;
    }
    // 6. candidates: roots with the max area; their slot becomes a key.
    for (int i = threadIdx.x; i < NB; i += NTB)
        if (lab[i] == (uint32_t)i) area[i] = ((int)area[i] == ma) ? INACT : 0u;
    __syncthreads();
    // 7. key = 1 + raster index of the component's first pixel.
    for (int i = threadIdx.x; i < NB; i += NTB) {
        uint32_t r = lab[i];
        if (r == INACT || area[r] == 0) continue;
        int by = i / BW, bx = i - by * BW;
        int y = 2 * by, x = 2 * bx;
        int k;
        if (F(y, x)) k = y * W + x;
        else if (F(y, x + 1)) k = y * W + x + 1;
        else if (F(y + 1, x)) k = (y + 1) * W + x;
        else k = (y + 1) * W + x + 1;
        atomicMin(&area[r], (uint32_t)(k + 1));
    }
    __syncthreads();
    // 8. winner = candidate with the largest key (first in OpenCV's list).
    int best = 0;
    for (int i = threadIdx.x; i < NB; i += NTB)
        if (lab[i] == (uint32_t)i && area[i] != 0) best = max(best, (int)area[i]);
    best = block_max_i(best, red);
    const int fp = best - 1;
    const uint32_t wroot = lab[((fp / W) >> 1) * BW + ((fp % W) >> 1)];
    // 9. bbox of the winner.
    int x0 = W, y0 = H, x1 = -1, y1 = -1;
    for (int i = threadIdx.x; i < NB; i += NTB) {
        if (lab[i] != wroot) continue;
        int by = i / BW, bx = i - by * BW;
        for (int d = 0; d < 4; ++d) {
            int y = 2 * by + (d >> 1), x = 2 * bx + (d & 1);
            if (F(y, x)) {
                x0 = min(x0, x); y0 = min(y0, y);
                x1 = max(x1, x); y1 = max(y1, y);
            }
        }
    }
    x0 = block_min_i(x0, red);
    y0 = block_min_i(y0, red);
    x1 = block_max_i(x1, red);
    y1 = block_max_i(y1, red);
    if (threadIdx.x == 0) {
        box[0] = x0;
        box[1] = y0;
        box[2] = min(x1 + 1, W - 1);  // boundingRect: x + w, clamped (wsol_metrics.py:175-178)
        box[3] = min(y1 + 1, H - 1);
    }
}

// ------------------------------------------------------------ accumulate
__global__ void accumulate_kernel(const int32_t* __restrict__ boxes,
                                  const int32_t* __restrict__ vmax, const double* __restrict__ taus,
                                  int T, const int32_t* __restrict__ gt,
                                  const int32_t* __restrict__ ngt, int G,
                                  const int32_t* __restrict__ top1,
                                  const int32_t* __restrict__ top5,
                                  const double* __restrict__ iou_thr, int n_iou,
                                  int32_t* __restrict__ counters, double* __restrict__ best_iou,
                                  int B) {
    long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (long)B * T) return;
    const int b = (int)(id / T), i = (int)(id % T);
    const int vm = vmax[b];
    // thresh = int(threshold * np.max(scoremap_image))  (wsol_metrics.py:158)
    const int thr = (int)(taus[i] * (double)vm);
    int a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    if (thr < vm) {
        const int32_t* bx = boxes + ((long)b * 256 + thr) * 4;
        a0 = bx[0]; a1 = bx[1]; a2 = bx[2]; a3 = bx[3];
    }
    // calculate_multiple_iou (wsol_metrics.py:77-124), max over GT boxes.
    double best = 0.0;
    const int ng = ngt[b];
    for (int g = 0; g < ng; ++g) {
        const int32_t* q = gt + ((long)b * G + g) * 4;
        long mnx = max(a0, q[0]), mny = max(a1, q[1]);
        long mxx = min(a2, q[2]), mxy = min(a3, q[3]);
        long inter = max(0L, mxx - mnx + 1) * max(0L, mxy - mny + 1);
        long area_a = (long)(a2 - a0 + 1) * (a3 - a1 + 1);
        long area_b = (long)(q[2] - q[0] + 1) * (q[3] - q[1] + 1);
        long den = area_a + area_b - inter;
        double iou = den <= 0 ? 0.0 : (double)inter / (double)den;
        if (g == 0 || iou > best) best = iou;
    }
    if (best_iou) best_iou[id] = best;
    for (int j = 0; j < n_iou; ++j) {
        if (best >= iou_thr[j]) {
            atomicAdd(&counters[(0 * n_iou + j) * T + i], 1);
            if (top1[b]) atomicAdd(&counters[(1 * n_iou + j) * T + i], 1);
            if (top5[b]) atomicAdd(&counters[(2 * n_iou + j) * T + i], 1);
        }
    }
}

}  // namespace

extern "C" size_t tcam_bbox_ws_bytes(int B, int H, int W) {
    return (size_t)B * H * W;  // psi (uint8)
}

extern "C" int tcam_bbox_levels(const uint8_t* cam_u8, int32_t* boxes, int32_t* vmax,
                                void* ws, int B, int H, int W, void* stream) {
    TCAM_REQUIRE(cam_u8 && boxes && vmax && ws && B > 0);
    TCAM_REQUIRE(H > 0 && W > 0 && H <= MAXH && W <= MAXW && pitch_of(W) <= MAXP);
    hipStream_t st = as_stream(stream);
    uint8_t* psi = (uint8_t*)ws;
    fill_kernel<<<B, NTB, 0, st>>>(cam_u8, psi, vmax, H, W);
    TCAM_CHECK_LAUNCH();
    level_kernel<<<B * 255, NTB, 0, st>>>(psi, vmax, boxes, H, W);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_box_accumulate(const int32_t* boxes, const int32_t* vmax, const double* taus,
                                   int T, const int32_t* gt, const int32_t* ngt, int G,
                                   const int32_t* top1, const int32_t* top5,
                                   const double* iou_thr, int n_iou, int32_t* counters,
                                   double* best_iou, int B, void* stream) {
    TCAM_REQUIRE(boxes && vmax && taus && gt && ngt && top1 && top5 && iou_thr && counters);
    TCAM_REQUIRE(T > 0 && G > 0 && n_iou > 0 && B > 0);
    long total = (long)B * T;
    accumulate_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        boxes, vmax, taus, T, gt, ngt, G, top1, top5, iou_thr, n_iou, counters, best_iou, B);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
