// BoxAcc v2 (--box_v2_metric True) on the GPU: compute_bboxes_from_scoremaps with
// multi_contour_eval=True (metrics/wsol_metrics.py:155-181) keeps the boundingRect of EVERY
// contour cv2.findContours(u8 > thr, RETR_TREE, CHAIN_APPROX_SIMPLE) returns, and
// BoxEvaluator.accumulate scores a tau by the best IoU over those boxes
// (wsol_metrics.py:342-368).  parseit.py:684-689 turns box_v2_metric into
// multi_contour_eval = multi_iou_eval = True.
//
// The contour boxes, characterised (pinned against the border-following oracle,
// oracle/contours.c, on random and smooth masks in tests/test_bbox_oracle.py):
//  * one outer contour per 8-connected foreground component C: boundingRect = bbox(C), so the
//    box is [x0, y0, min(x1 + 1, W - 1), min(y1 + 1, H - 1)] (x + w, y + h clamped,
//    wsol_metrics.py:175-178);
//  * one hole contour per 4-connected background component that does not touch the frame
//    (findContours pads with zeros): the hole border runs through the foreground pixels
//    4-adjacent to the hole, so its boundingRect is bbox(hole) grown by one pixel on every
//    side — [hx0 - 1, hy0 - 1, min(hx1 + 2, W - 1), min(hy1 + 2, H - 1)].
// OpenCV's list order (only the compatibility list needs it): a contour's discovery key is
// the raster index of its component's first pixel; an outer contour's parent is the hole
// holding the pixel left of its first pixel (or the frame), a hole's parent is the
// component holding the pixel left of its first pixel; the list is the pre-order of that
// tree with siblings in decreasing key order (cvInsertNodeIntoTree prepends).
//
// Kernels:
//  u8_levels_kernel   one workgroup per frame: vmax = max(u8); the binary image {u8 > L}
//                     only changes where u8 takes the value L + 1, so the levels computed
//                     are {v - 1 : v present}, and canon[L] names the computed level each
//                     L < vmax shares its image with.
//  multi_level_kernel one workgroup per (frame, chunk of levels), each with its own
//                     scratch slot (union-find parents + per-root x0 / x1 / y1 in global
//                     memory, L2-resident): per level a bitmap in LDS, parents initialised
//                     to the pixel's run start inside its 32-pixel word, lock-free
//                     union-find (hooks toward the smaller index, so a root is its
//                     component's first pixel, y0 = root / W), run-wise bbox atomics, then
//                     per root the box and its IoU against the GT boxes (fp64, the +1
//                     inclusive convention of calculate_multiple_iou), max-reduced.
//  multi_accumulate   one thread per (frame, tau): thr = int(tau * vmax) as the reference,
//                     the canonical level's max IoU (or the [0,0,0,0] box above vmax), the
//                     BoxEvaluator counters.
// Every access to the union-find arrays is an agent-scope atomic (no stale vector-L1 line
// can be read after another wave's CAS).
#include "common.h"

namespace {

constexpr int MT = 1024;           // threads per workgroup
constexpr int MAX_HW = 320;        // frames up to 320 x 320
constexpr int MWPR = MAX_HW / 32;  // bitmap words per row
constexpr int MAX_G = 64;          // GT boxes per frame held in LDS

__device__ __forceinline__ int ald(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// root of x; parents only ever point to smaller indices (par[x] <= x), path halving
__device__ int uf_find(int* par, int x) {
    int cur = ald(par + x);
    if (cur != x) {
        int prev = x, nxt;
        while (cur > (nxt = ald(par + cur))) {
            ast(par + prev, nxt);
            prev = cur;
            cur = nxt;
        }
    }
    return cur;
}

// hook the larger root under the smaller one (CAS on a root's self-parent)
__device__ void uf_unite(int* par, int a, int b) {
    int ar = uf_find(par, a), br = uf_find(par, b);
    while (ar != br) {
        if (ar < br) {
            const int old = atomicCAS(par + br, br, ar);
            if (old == br) return;
            br = old;
        } else {
            const int old = atomicCAS(par + ar, ar, br);
            if (old == ar) return;
            ar = old;
        }
    }
}

struct Scratch {
    int* par;
    int* x0;
    int* x1;
    int* y1;
};

__device__ __forceinline__ int bm_bit(const uint32_t* bm, int wpr, int y, int x) {
    return (bm[y * wpr + (x >> 5)] >> (x & 31)) & 1;
}

// The components of {u8 > L} (foreground 8-connected, background 4-connected) with their
// bounding boxes; on return (after a barrier) every root p has par[p] == p and x0 / x1 / y1
// hold its box (y0 = p / W).
__device__ void label_level(const uint8_t* __restrict__ u8, int L, int H, int W, uint32_t* bm,
                            const Scratch& s) {
    const int tid = threadIdx.x;
    const int wpr = (W + 31) >> 5;
    const int HW = H * W;
    // 1. bitmap (bits beyond W stay 0 and are never read as pixels)
    for (int w = tid; w < H * wpr; w += MT) {
        const int y = w / wpr, x0 = (w - y * wpr) * 32;
        uint32_t bits = 0;
        const uint8_t* row = u8 + (long)y * W;
        for (int e = 0; e < 32; ++e) {
            const int x = x0 + e;
            if (x < W && (int)row[x] > L) bits |= 1u << e;
        }
        bm[w] = bits;
    }
    __syncthreads();
    // 2. parents = the pixel's run start inside its word; empty boxes
    for (int p = tid; p < HW; p += MT) {
        const int y = p / W, x = p - y * W;
        const uint32_t wd = bm[y * wpr + (x >> 5)];
        const int c = (wd >> (x & 31)) & 1;
        const uint32_t other = (c ? ~wd : wd) & ((2u << (x & 31)) - 1u);   // other colour <= x
        const int start = other ? (32 - __builtin_clz(other)) : 0;       // first bit after it
        ast(s.par + p, y * W + (x & ~31) + start);
        ast(s.x0 + p, W);
        ast(s.x1 + p, -1);
        ast(s.y1 + p, -1);
    }
    __threadfence();
    __syncthreads();
    // 3. unions: the run across a word boundary, and the row above (8-neighbourhood for the
    // foreground, 4 for the background), skipping links a neighbour already made
    for (int p = tid; p < HW; p += MT) {
        const int y = p / W, x = p - y * W;
        const int c = bm_bit(bm, wpr, y, x);
        const int cw = x > 0 ? bm_bit(bm, wpr, y, x - 1) : -1;
        if ((x & 31) == 0 && x > 0 && cw == c) uf_unite(s.par, p, p - 1);
        if (y == 0) continue;
        const int cn = bm_bit(bm, wpr, y - 1, x);
        const int cnw = x > 0 ? bm_bit(bm, wpr, y - 1, x - 1) : -1;
        if (c) {
            const int cne = x + 1 < W ? bm_bit(bm, wpr, y - 1, x + 1) : 0;
            if (cn) {
                // W and NW both set: W already joined NW, which is in N's run
                if (!(cw == 1 && cnw == 1)) uf_unite(s.par, p, p - W);
            } else {
                if (cnw == 1 && cw != 1) uf_unite(s.par, p, p - W - 1);
                if (cne) uf_unite(s.par, p, p - W + 1);
            }
        } else if (!cn && !(cw == 0 && cnw == 0)) {
            uf_unite(s.par, p, p - W);
        }
    }
    __threadfence();
    __syncthreads();
    // 4. boxes: one thread per row run (its start), the run's end from the bitmap
    for (int p = tid; p < HW; p += MT) {
        const int y = p / W, x = p - y * W;
        const int c = bm_bit(bm, wpr, y, x);
        if (x > 0 && bm_bit(bm, wpr, y, x - 1) == c) continue;
        int j = x >> 5;
        uint32_t m = c ? ~bm[y * wpr + j] : bm[y * wpr + j];
        m &= ~0u << (x & 31);
        while (!m && ++j < wpr) m = c ? ~bm[y * wpr + j] : bm[y * wpr + j];
        const int xe = min(W - 1, (m ? 32 * j + __builtin_ctz(m) : 32 * wpr) - 1);
        const int r = uf_find(s.par, p);
        atomicMin(s.x0 + r, x);
        atomicMax(s.x1 + r, xe);
        atomicMax(s.y1 + r, y);
    }
    __threadfence();
    __syncthreads();
}

// the contour box of root r, or false for a background component touching the frame
__device__ __forceinline__ bool root_box(const Scratch& s, const uint32_t* bm, int r, int H,
                                         int W, int& hole, int (&b)[4]) {
    const int wpr = (W + 31) >> 5;
    const int y0 = r / W, x0 = ald(s.x0 + r), x1 = ald(s.x1 + r), y1 = ald(s.y1 + r);
    hole = !bm_bit(bm, wpr, y0, r - y0 * W);
    if (hole) {
        if (x0 == 0 || y0 == 0 || x1 == W - 1 || y1 == H - 1) return false;
        b[0] = x0 - 1;
        b[1] = y0 - 1;
        b[2] = min(x1 + 2, W - 1);
        b[3] = min(y1 + 2, H - 1);
    } else {
        b[0] = x0;
        b[1] = y0;
        b[2] = min(x1 + 1, W - 1);
        b[3] = min(y1 + 1, H - 1);
    }
    return true;
}

// calculate_multiple_iou (wsol_metrics.py:77-124) of one box, max over the GT boxes
__device__ __forceinline__ double max_iou(const int (&a)[4], const int* gt, int ng) {
    double best = 0.0;
    for (int g = 0; g < ng; ++g) {
        const int* q = gt + 4 * g;
        const long mnx = max(a[0], q[0]), mny = max(a[1], q[1]);
        const long mxx = min(a[2], q[2]), mxy = min(a[3], q[3]);
        const long inter = max(0L, mxx - mnx + 1) * max(0L, mxy - mny + 1);
        const long area_a = (long)(a[2] - a[0] + 1) * (a[3] - a[1] + 1);
        const long area_b = (long)(q[2] - q[0] + 1) * (q[3] - q[1] + 1);
        const long den = area_a + area_b - inter;
        const double iou = den <= 0 ? 0.0 : (double)inter / (double)den;
        if (g == 0 || iou > best) best = iou;
    }
    return best;
}

__global__ __launch_bounds__(256) void u8_levels_kernel(const uint8_t* __restrict__ cam_u8,
                                                        int HW, int32_t* __restrict__ vmax,
                                                        int32_t* __restrict__ canon,
                                                        int32_t* __restrict__ lev_list,
                                                        int32_t* __restrict__ nlev) {
    __shared__ int hist[257];
    __shared__ int cnt;
    const int b = blockIdx.x, tid = threadIdx.x;
    hist[tid] = 0;
    if (tid == 0) {
        hist[256] = 0;
        cnt = 0;
    }
    __syncthreads();
    const uint8_t* u = cam_u8 + (long)b * HW;
    for (int i = tid; i < HW; i += 256) atomicOr(&hist[u[i]], 1);
    __syncthreads();
    int vm = 0;
    for (int v = 255; v > 0; --v)
        if (hist[v]) { vm = v; break; }
    if (tid == 0) vmax[b] = vm;
    // canon[L] = (smallest present value >= L + 1) - 1, for L < vmax
    const int L = tid;
    int c = -1;
    if (L < vm) {
        int v = L + 1;
        while (!hist[v]) ++v;
        c = v - 1;
    }
    canon[b * 256 + L] = c;
    // the computed levels in decreasing order (any order works; the list is per frame)
    if (L < vm && hist[L + 1]) lev_list[b * 256 + atomicAdd(&cnt, 1)] = L;
    __syncthreads();
    if (tid == 0) nlev[b] = cnt;
}

__global__ __launch_bounds__(MT) void multi_level_kernel(
    const uint8_t* __restrict__ cam_u8, const int32_t* __restrict__ gt,
    const int32_t* __restrict__ ngt, int G, const int32_t* __restrict__ lev_list,
    const int32_t* __restrict__ nlev, double* __restrict__ iou_out, int H, int W, int chunks,
    int* __restrict__ scratch) {
    __shared__ uint32_t bm[MAX_HW * MWPR];
    __shared__ int gbox[4 * MAX_G];
    __shared__ unsigned long long best_bits;
    const int b = blockIdx.x / chunks, chunk = blockIdx.x % chunks;
    const int nl = nlev[b];
    if (chunk >= nl) return;
    const int HW = H * W, tid = threadIdx.x;
    int* base = scratch + (long)blockIdx.x * 4 * HW;
    const Scratch s{base, base + HW, base + 2 * HW, base + 3 * HW};
    const int ng = min(ngt[b], MAX_G);
    for (int i = tid; i < 4 * ng; i += MT) gbox[i] = gt[(long)b * G * 4 + i];
    const uint8_t* u8 = cam_u8 + (long)b * HW;
    for (int li = chunk; li < nl; li += chunks) {
        const int L = lev_list[b * 256 + li];
        if (tid == 0) best_bits = 0ull;
        label_level(u8, L, H, W, bm, s);
        double best = 0.0;
        for (int p = tid; p < HW; p += MT) {
            if (ald(s.par + p) != p) continue;
            int hole, box[4];
            if (!root_box(s, bm, p, H, W, hole, box)) continue;
            best = fmax(best, max_iou(box, gbox, ng));
        }
        // IoU >= 0: the bit pattern orders like the value
        atomicMax(&best_bits, (unsigned long long)__double_as_longlong(best));
        __syncthreads();
        if (tid == 0) iou_out[b * 256 + L] = __longlong_as_double((long long)best_bits);
        __syncthreads();
    }
}

// one frame, one level: every contour as (is_hole, key, parent key, x0, y0, x1, y1, 0)
__global__ __launch_bounds__(MT) void contour_records_kernel(const uint8_t* __restrict__ u8,
                                                             int L, int H, int W,
                                                             int* __restrict__ scratch,
                                                             int32_t* __restrict__ rec, int cap,
                                                             int32_t* __restrict__ count) {
    __shared__ uint32_t bm[MAX_HW * MWPR];
    const int HW = H * W, tid = threadIdx.x;
    const Scratch s{scratch, scratch + HW, scratch + 2 * HW, scratch + 3 * HW};
    if (tid == 0) *count = 0;
    label_level(u8, L, H, W, bm, s);
    for (int p = tid; p < HW; p += MT) {
        if (ald(s.par + p) != p) continue;
        int hole, box[4];
        if (!root_box(s, bm, p, H, W, hole, box)) continue;
        int parent = -1;
        if (p % W > 0) {
            const int q = uf_find(s.par, p - 1);   // the component left of the first pixel
            if (hole) {
                parent = q;
            } else {
                int h2, b2[4];
                if (root_box(s, bm, q, H, W, h2, b2)) parent = q;   // a hole, not the frame
            }
        }
        const int k = atomicAdd(count, 1);
        if (k < cap) {
            int32_t* r = rec + 8 * (long)k;
            r[0] = hole; r[1] = p; r[2] = parent;
            r[3] = box[0]; r[4] = box[1]; r[5] = box[2]; r[6] = box[3]; r[7] = 0;
        }
    }
}

__global__ void multi_accumulate_kernel(const double* __restrict__ iou_tab,
                                        const int32_t* __restrict__ canon,
                                        const int32_t* __restrict__ vmax,
                                        const double* __restrict__ taus, int T,
                                        const int32_t* __restrict__ gt,
                                        const int32_t* __restrict__ ngt, int G,
                                        const int32_t* __restrict__ top1,
                                        const int32_t* __restrict__ top5,
                                        const double* __restrict__ iou_thr, int n_iou,
                                        int32_t* __restrict__ counters,
                                        double* __restrict__ best_iou, int B) {
    const long id = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (long)B * T) return;
    const int b = (int)(id / T), i = (int)(id % T);
    const int vm = vmax[b];
    // thresh = int(threshold * np.max(scoremap_image))  (wsol_metrics.py:158)
    const int thr = (int)(taus[i] * (double)vm);
    double best;
    if (thr < vm) {
        best = iou_tab[b * 256 + canon[b * 256 + thr]];
    } else {
        // no contour: the box [0, 0, 0, 0] (wsol_metrics.py:167-168)
        const int zero[4] = {0, 0, 0, 0};
        best = max_iou(zero, gt + (long)b * G * 4, ngt[b]);
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

__global__ void flag_count_kernel(const int32_t* __restrict__ flags, int B,
                                  int32_t* __restrict__ acc) {
    int v = 0;
    for (int i = threadIdx.x; i < B; i += 64) v += flags[i] != 0;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (threadIdx.x == 0) acc[0] += v;
}

int multi_chunks(int B) {
    const int c = 256 / (B > 0 ? B : 1);
    return c < 1 ? 1 : (c > 255 ? 255 : c);
}

size_t lev_bytes(int B) { return ((size_t)B * (256 + 256 + 1) * sizeof(int32_t) + 255) / 256 * 256; }

}  // namespace

extern "C" size_t tcam_bbox_multi_ws_bytes(int B, int H, int W) {
    // canon (B x 256) | lev_list (B x 256) | nlev (B) | per-workgroup scratch (4 x H*W int32)
    return lev_bytes(B) + (size_t)B * multi_chunks(B) * 4 * H * W * sizeof(int32_t);
}

extern "C" int tcam_bbox_multi_iou(const uint8_t* cam_u8, const int32_t* gt, const int32_t* ngt,
                                   int G, double* iou, int32_t* vmax, int32_t* canon, void* ws,
                                   int B, int H, int W, void* stream) {
    TCAM_REQUIRE(cam_u8 && gt && ngt && iou && vmax && canon && ws && B > 0 && G > 0);
    TCAM_REQUIRE(G <= MAX_G && H > 0 && W > 0 && H <= MAX_HW && W <= MAX_HW);
    hipStream_t st = as_stream(stream);
    int32_t* lev_list = (int32_t*)ws;
    int32_t* nlev = lev_list + (size_t)B * 256;
    int* scratch = (int*)((char*)ws + lev_bytes(B));
    const int chunks = multi_chunks(B);
    u8_levels_kernel<<<B, 256, 0, st>>>(cam_u8, H * W, vmax, canon, lev_list, nlev);
    TCAM_CHECK_LAUNCH();
    multi_level_kernel<<<B * chunks, MT, 0, st>>>(cam_u8, gt, ngt, G, lev_list, nlev, iou, H, W,
                                                  chunks, scratch);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_box_accumulate_multi(const double* iou, const int32_t* canon,
                                         const int32_t* vmax, const double* taus, int T,
                                         const int32_t* gt, const int32_t* ngt, int G,
                                         const int32_t* top1, const int32_t* top5,
                                         const double* iou_thr, int n_iou, int32_t* counters,
                                         double* best_iou, int B, void* stream) {
    TCAM_REQUIRE(iou && canon && vmax && taus && gt && ngt && top1 && top5 && iou_thr &&
                 counters);
    TCAM_REQUIRE(T > 0 && G > 0 && n_iou > 0 && B > 0);
    const long total = (long)B * T;
    multi_accumulate_kernel<<<cdiv(total, 256), 256, 0, as_stream(stream)>>>(
        iou, canon, vmax, taus, T, gt, ngt, G, top1, top5, iou_thr, n_iou, counters, best_iou,
        B);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" size_t tcam_bbox_contours_ws_bytes(int H, int W) {
    return (size_t)4 * H * W * sizeof(int32_t);
}

extern "C" int tcam_bbox_contours(const uint8_t* cam_u8, int level, int32_t* records, int cap,
                                  int32_t* count, void* ws, int H, int W, void* stream) {
    TCAM_REQUIRE(cam_u8 && records && count && ws && cap > 0 && level >= 0 && level < 256);
    TCAM_REQUIRE(H > 0 && W > 0 && H <= MAX_HW && W <= MAX_HW);
    contour_records_kernel<<<1, MT, 0, as_stream(stream)>>>(cam_u8, level, H, W, (int*)ws,
                                                             records, cap, count);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

extern "C" int tcam_flag_count(const int32_t* flags, int B, int32_t* acc, void* stream) {
    TCAM_REQUIRE(flags && acc && B > 0);
    flag_count_kernel<<<1, 64, 0, as_stream(stream)>>>(flags, B, acc);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}
