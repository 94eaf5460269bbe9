/*
 * TEST INFRASTRUCTURE ONLY (oracle): C restatement of the OpenCV 4.5.x
 * routines behind compute_bboxes_from_scoremaps (reference
 * dlib/metrics/wsol_metrics.py:127-197):
 *
 *   cv2.threshold(u8, thresh, 255, THRESH_BINARY)      -> u8 > thresh
 *   cv2.findContours(bin, RETR_TREE, CHAIN_APPROX_SIMPLE)
 *       imgproc/src/contours.cpp: cv::findContours pads the image with a
 *       1-pixel zero border (copyMakeBorder) and runs the Suzuki-Abe border
 *       follower cvFindNextContour / icvFetchContourEx with offset (-1,-1);
 *       contours are linked into a tree (cvInsertNodeIntoTree PREPENDS to
 *       the parent's child list) and returned in pre-order
 *       (cvTreeToNodeSeq).
 *   cv2.contourArea(c)    shapedescr.cpp: |shoelace| / 2 over the points.
 *   cv2.boundingRect(c)   (x, y, w, h) of the point set.
 *   max(contours, key=contourArea): the FIRST contour of maximal area.
 *
 * cv2 (opencv-python 4.1.2 / 4.5.5, dependencies/requirements.txt:52-54) is
 * not installed in this image, so this restatement is pinned only by the
 * analytic known-answer tests in tests/test_bbox_oracle.py ("parity
 * unpinned" against OpenCV binaries).
 *
 * Labels: the original uses 7-bit labels (nbd, nbd|0x80) that wrap and
 * resolves the LNBD contour through a per-label list + rectangle test;
 * here labels are unique ints (+id for a visited border pixel, -id for a
 * "right-bound" pixel), which selects the same LNBD contour directly.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int64_t area2;          /* 2 * contourArea (exact) */
    int x0, y0, x1, y1;     /* bounding rect, inclusive extremes */
    int is_hole;
    int parent;             /* index in output order, -1 = frame */
    int npts;               /* CHAIN_APPROX_SIMPLE vertex count */
} oc_contour;

typedef struct {
    int is_hole, parent;    /* parent = discovery id, -1 frame */
    int first_child, next_sibling;
    int64_t area2;
    int x0, y0, x1, y1, npts;
    int pts_off;
} node_t;

static const int code_dx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static const int code_dy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

/* icvFetchContourEx with CHAIN_APPROX_SIMPLE (method = 1). */
static void fetch_contour(int32_t* img, int step, int i0, int px, int py, int is_hole,
                          int lab, node_t* nd, int* pts, int* npts_total, int max_pts) {
    int deltas[16];
    deltas[0] = 1; deltas[1] = -step + 1; deltas[2] = -step; deltas[3] = -step - 1;
    deltas[4] = -1; deltas[5] = step - 1; deltas[6] = step; deltas[7] = step + 1;
    for (int k = 0; k < 8; ++k) deltas[8 + k] = deltas[k];
    int s, s_end, prev_s, i1 = 0, i3, i4 = 0;
    int rx = px, rw = px, ry = py, rh = py;  /* rect.x, .width(as max), .y, .height */
    int npts = 0;
    int64_t a2 = 0;
    int fx = 0, fy = 0, lx = 0, ly = 0;   /* first / last written point */
    nd->pts_off = *npts_total;
#define WRITE_PT(X, Y)                                                     \
    do {                                                                   \
        if (npts == 0) { fx = (X); fy = (Y); }                             \
        else a2 += (int64_t)lx * (Y) - (int64_t)ly * (X);                  \
        lx = (X); ly = (Y);                                                \
        if (*npts_total < max_pts) {                                       \
            pts[2 * (*npts_total)] = (X); pts[2 * (*npts_total) + 1] = (Y); \
        }                                                                  \
        ++*npts_total; ++npts;                                             \
    } while (0)

    s_end = s = is_hole ? 0 : 4;
    do {
        s = (s - 1) & 7;
        i1 = i0 + deltas[s];
    } while (img[i1] == 0 && s != s_end);

    if (s == s_end) { /* single pixel domain */
        img[i0] = -lab;
        WRITE_PT(px, py);
    } else {
        i3 = i0;
        prev_s = s ^ 4;
        for (;;) {
            s_end = s;
            if (s > 15) s = 15;
            while (s < 15) {
                i4 = i3 + deltas[++s];
                if (img[i4] != 0) break;
            }
            s &= 7;
            if ((unsigned)(s - 1) < (unsigned)s_end) img[i3] = -lab;
            else if (img[i3] == 1) img[i3] = lab;
            if (s != prev_s) {
                WRITE_PT(px, py);
                if (px < rx) rx = px; else if (px > rw) rw = px;
                if (py < ry) ry = py; else if (py > rh) rh = py;
            }
            prev_s = s;
            px += code_dx[s];
            py += code_dy[s];
            if (i4 == i0 && i3 == i1) break;
            i3 = i4;
            s = (s + 4) & 7;
        }
    }
    /* close the polygon (contourArea starts from prev = last point) */
    if (npts > 0) a2 += (int64_t)lx * fy - (int64_t)ly * fx;
    nd->area2 = a2 < 0 ? -a2 : a2;
    nd->x0 = rx; nd->x1 = rw; nd->y0 = ry; nd->y1 = rh;
    nd->npts = npts;
#undef WRITE_PT
}

/*
 * bin: (H, W) u8, nonzero = foreground.  Returns the number of contours
 * written to `out` in OpenCV's RETR_TREE output order (coordinates of the
 * unpadded image), or -1 if max_out is too small.  pts (optional) receives
 * the CHAIN_APPROX_SIMPLE vertices, contour after contour, in DISCOVERY
 * order offsets (use oc_contour_points to fetch by output index).
 */
static node_t* g_nodes = 0;
static int g_nnodes = 0;
static int* g_order = 0;

int oc_find_contours(const uint8_t* bin, int H, int W, oc_contour* out, int max_out,
                     int* pts, int max_pts) {
    const int PW = W + 2, PH = H + 2;
    int32_t* img = (int32_t*)calloc((size_t)PW * PH, sizeof(int32_t));
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) img[(y + 1) * PW + x + 1] = bin[y * W + x] ? 1 : 0;
    int cap = 1024, n = 0, npts_total = 0;
    node_t* nodes = (node_t*)malloc(sizeof(node_t) * cap);
    int frame_first_child = -1;
    /* cvFindNextContour scan over rows 1..H, cols 1..W of the padded image */
    int lnbd_x = 0;
    for (int y = 1; y < PH - 1; ++y) {
        int prev = 0;
        lnbd_x = 0;
        for (int x = 1; x < PW - 1; ++x) {
            int p = img[y * PW + x];
            if (p == prev) continue;
            int is_hole = 0;
            int found = 0;
            if (!(prev == 0 && p == 1)) {
                if (p != 0 || prev < 1) goto resume_scan;
                if (prev != 0 && prev != 1) lnbd_x = x - 1;
                is_hole = 1;
            }
            {
                int parent; /* -1 = frame */
                if (lnbd_x <= 0) {
                    parent = -1;
                } else {
                    int lv = img[y * PW + lnbd_x];
                    int id = (lv < 0 ? -lv : lv) - 2;
                    parent = id;
                    if (nodes[id].is_hole == is_hole) parent = nodes[id].parent;
                }
                int ox = x - is_hole;
                lnbd_x = x - is_hole;
                if (n == cap) {
                    cap *= 2;
                    nodes = (node_t*)realloc(nodes, sizeof(node_t) * cap);
                }
                node_t* nd = &nodes[n];
                nd->is_hole = is_hole;
                nd->parent = parent;
                nd->first_child = -1;
                nd->next_sibling = -1;
                fetch_contour(img, PW, y * PW + ox, ox - 1, y - 1, is_hole, n + 2, nd, pts,
                              &npts_total, max_pts);
                /* cvInsertNodeIntoTree: prepend to the parent's children */
                if (parent < 0) {
                    nd->next_sibling = frame_first_child;
                    frame_first_child = n;
                } else {
                    nd->next_sibling = nodes[parent].first_child;
                    nodes[parent].first_child = n;
                }
                ++n;
                found = 1;
            }
            if (found) {
                /* the next call restarts at x + 1 with prev = img[x] */
                prev = img[y * PW + x];
                continue;
            }
        resume_scan:
            prev = p;
            if (prev != 0 && prev != 1) lnbd_x = x;
        }
    }
    free(img);
    /* pre-order traversal (cvTreeToNodeSeq) */
    int* order = (int*)malloc(sizeof(int) * (n + 1));
    int* idx_of = (int*)malloc(sizeof(int) * (n + 1));
    int* stack = (int*)malloc(sizeof(int) * (n + 1));
    int no = 0, sp = 0;
    /* iterative pre-order: visit node, then its children, then siblings */
    int cur = frame_first_child;
    while (cur >= 0 || sp > 0) {
        if (cur < 0) { cur = stack[--sp]; continue; }
        order[no] = cur;
        idx_of[cur] = no;
        ++no;
        if (nodes[cur].next_sibling >= 0) stack[sp++] = nodes[cur].next_sibling;
        cur = nodes[cur].first_child;
    }
    int ret = n;
    if (n > max_out) {
        ret = -1;
    } else {
        for (int i = 0; i < n; ++i) {
            node_t* nd = &nodes[order[i]];
            out[i].area2 = nd->area2;
            out[i].x0 = nd->x0; out[i].y0 = nd->y0; out[i].x1 = nd->x1; out[i].y1 = nd->y1;
            out[i].is_hole = nd->is_hole;
            out[i].parent = nd->parent < 0 ? -1 : idx_of[nd->parent];
            out[i].npts = nd->npts;
        }
    }
    free(stack);
    free(g_nodes);
    free(g_order);
    g_nodes = nodes;
    g_nnodes = n;
    g_order = order;
    free(idx_of);
    return ret;
}

/* Vertices of output contour i of the last oc_find_contours call. */
int oc_contour_points(int i, const int* pts, int* dst, int max_dst) {
    if (!g_nodes || i < 0 || i >= g_nnodes) return -1;
    node_t* nd = &g_nodes[g_order[i]];
    int k = nd->npts < max_dst ? nd->npts : max_dst;
    memcpy(dst, pts + 2 * nd->pts_off, sizeof(int) * 2 * k);
    return nd->npts;
}

/*
 * scoremap2bbox for a list of integer thresholds (wsol_metrics.py:155-181,
 * multi_contour_eval=False): boxes[t] = [x0, y0, min(x0+w, W-1),
 * min(y0+h, H-1)] of max(contours, key=contourArea), or [0,0,0,0].
 */
int oc_boxes_for_thresholds(const uint8_t* u8, int H, int W, const int* thr, int T,
                            int* boxes, int* ncontours) {
    uint8_t* bin = (uint8_t*)malloc((size_t)H * W);
    int cap = H * W + 8;
    oc_contour* cs = (oc_contour*)malloc(sizeof(oc_contour) * cap);
    for (int t = 0; t < T; ++t) {
        for (int i = 0; i < H * W; ++i) bin[i] = u8[i] > thr[t];
        int n = oc_find_contours(bin, H, W, cs, cap, 0, 0);
        if (ncontours) ncontours[t] = n;
        int* b = boxes + 4 * t;
        if (n <= 0) {
            b[0] = b[1] = b[2] = b[3] = 0;
            continue;
        }
        int best = 0;
        for (int i = 1; i < n; ++i)
            if (cs[i].area2 > cs[best].area2) best = i;
        b[0] = cs[best].x0;
        b[1] = cs[best].y0;
        b[2] = cs[best].x1 + 1 < W - 1 ? cs[best].x1 + 1 : W - 1;
        b[3] = cs[best].y1 + 1 < H - 1 ? cs[best].y1 + 1 : H - 1;
    }
    free(cs);
    free(bin);
    return 0;
}
