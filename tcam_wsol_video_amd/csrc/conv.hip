// Implicit-GEMM convolution on the fp32 MFMA pipe of gfx950.
//
//   out[b, m, p] = act( sum_k  Wt[k, m] * X[k, (b, p)]  + bias[m]  (+ res) )
//
// GEMM view: M = Cout, N = B * Hout * Wout (frames x output pixels; NCHW so p
// is contiguous), K = KH * KW * Ctot ordered TAP-MAJOR: k = (kh*KW + kw) *
// Ctot + c, c running over the concatenated source channels.  X is never
// materialised: the B-operand tile is gathered straight from the NCHW
// sources (im2col on the fly), including the decoder's nearest-x2 upsample
// and skip concat (unet/decoder.py:41-57) and the bottleneck's conv3 +
// downsample pair (resnet.py:214-232), which become one GEMM over a
// concatenated K.  BN is folded into Wt/bias on the host (eval mode).
//
// Weight contract (tcam_hip.h): Wt is (roundup(K, 32), roundup(Cout, 128))
// row-major, zero padded, so A-tile loads need no bounds checks.
//
// Fast path (every source's C % 16 == 0): each 16-row half of a 32-deep
// K-step lies inside one tap and one source, so its spatial offset and
// padding mask are computed once per half per thread and the gathered
// elements of a thread are one fixed stride apart.  Padding / out-of-image taps use buffer loads whose
// offset is pushed past num_records: the hardware returns 0, no branches.
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact k-ordered fp32 fma chain
// (cdna_hip_programming.md §3); results differ from PyTorch CPU only by
// summation order.
//
// Tiling: BM x BN block tile, BK = 32, 256 threads = 4 waves, each wave a
// (TM*32) x (TN*32) sub-tile.  Operand tiles are staged in LDS (double
// buffered, one barrier per K-step); global loads for step t+1 are issued
// before the MFMAs of step t and written to LDS after them.  Blocks that
// share an N tile (same input patch) are mapped onto one XCD (T1 remap).
#include "common.h"

namespace {

constexpr int BK = 32;
constexpr int NT = 256;
constexpr int MPAD = 128;
constexpr uint32_t OOB = 0x80000000u;  // > any num_records: buffer load returns 0

typedef __amdgpu_buffer_rsrc_t rsrc_t;

struct Src {
    const float* ptr;
    int C, H, W, stride, up2;
    uint32_t bytes;
};

struct ConvP {
    Src s[2];
    int c0;        // channels of source 0
    int Ctot;
    const float* wt;
    int ldw;       // = roundup(Cout, 128)
    const float* bias;
    const float* res;
    float* out;
    int Cout, Hout, Wout, pad, relu, KS;
    int K, N, HWo;
    int mtiles, ntiles, nblocks;
};

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float bload(rsrc_t rsrc, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, (int)off, 0, 0));
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5, T1): consecutive
// logical ids land on the same XCD (blocks b and b+8 share one).
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <int BM, int BN, int WM, bool FAST, int STAGES>
__global__ __launch_bounds__(NT, STAGES == 1 ? 4 : 2) void conv_mfma_kernel(ConvP p) {
    constexpr int WN = 4 / WM;
    constexpr int WTM = BM / WM;
    constexpr int WTN = BN / WN;
    constexpr int TM = WTM / 32;
    constexpr int TN = WTN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile too small");
    constexpr int A_F4 = BM * BK / 4;
    constexpr int A_PER_T = (A_F4 + NT - 1) / NT;
    constexpr int B_PER_T = BK * BN / NT;
    constexpr int B_RSTEP = NT / BN;

    // STAGES = 2: double-buffered LDS, one barrier per K-step.
    // STAGES = 1: one LDS stage (half the LDS -> twice the blocks per CU),
    // two barriers per K-step; the register prefetch of step t+1 overlaps
    // the HBM latency in both.
    __shared__ float As[STAGES][BK][BM];
    __shared__ float Bs[STAGES][BK][BN];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;

    const int lb = xcd_remap(blockIdx.x, p.nblocks);
    const int m0 = (lb % p.mtiles) * BM;
    const int n0 = (lb / p.mtiles) * BN;

    const int bcol = tid % BN;
    const int brow0 = tid / BN;
    const int n = n0 + bcol;
    const bool nvalid = n < p.N;
    int img = 0, oh = 0, ow = 0;
    if (nvalid) {
        img = n / p.HWo;
        int hw = n - img * p.HWo;
        oh = hw / p.Wout;
        ow = hw - oh * p.Wout;
    }
    const rsrc_t rs0 = make_rsrc(p.s[0].ptr, p.s[0].bytes);
    const rsrc_t rs1 = make_rsrc(p.s[1].ptr, p.s[1].bytes);

    float4 areg[A_PER_T];
    float breg[B_PER_T];

    auto load_tile = [&](int kt) {
        const int kbase = kt * BK;
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
            int f = tid + i * NT;
            if (A_F4 % NT == 0 || f < A_F4) {
                int kr = f / (BM / 4);
                int mc = (f % (BM / 4)) * 4;
                areg[i] = *reinterpret_cast<const float4*>(p.wt + (long)(kbase + kr) * p.ldw + m0 + mc);
            }
        }
        if constexpr (FAST) {
            // Each 16-row half of the K-step lies inside one tap and one
            // source (every source's C % 16 == 0): offset and padding mask
            // are computed once per half, the half's elements are one
            // channel-plane stride apart.
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int kh0 = kbase + hf * 16;
                const int tap = kh0 / p.Ctot;
                int c = kh0 - tap * p.Ctot;
                const int kh = tap / p.KS, kw = tap - (tap / p.KS) * p.KS;
                const int si = c < p.c0 ? 0 : 1;
                if (si) c -= p.c0;
                const Src& s = p.s[si];
                const int iy = oh * s.stride - p.pad + kh;
                const int ix = ow * s.stride - p.pad + kw;
                const bool ok = nvalid && kh0 < p.K && (unsigned)iy < (unsigned)(s.H << s.up2) &&
                                (unsigned)ix < (unsigned)(s.W << s.up2);
                const uint32_t plane = (uint32_t)s.H * s.W * 4u;
                uint32_t off = ((((uint32_t)img * s.C + c + brow0) * s.H + (iy >> s.up2)) * s.W +
                                (ix >> s.up2)) * 4u;
                off = ok ? off : OOB;
                const uint32_t step = ok ? plane * B_RSTEP : 0u;
                const rsrc_t rs = si ? rs1 : rs0;
#pragma unroll
                for (int j = 0; j < B_PER_T / 2; ++j)
                    breg[hf * (B_PER_T / 2) + j] = bload(rs, off + j * step);
            }
        } else {
#pragma unroll
            for (int j = 0; j < B_PER_T; ++j) {
                const int k = kbase + brow0 + j * B_RSTEP;
                const int tap = k / p.Ctot;
                int c = k - tap * p.Ctot;
                const int kh = tap / p.KS, kw = tap - kh * p.KS;
                const int si = c < p.c0 ? 0 : 1;
                if (si) c -= p.c0;
                const Src& s = p.s[si];
                const int iy = oh * s.stride - p.pad + kh;
                const int ix = ow * s.stride - p.pad + kw;
                const bool ok = nvalid && k < p.K && (unsigned)iy < (unsigned)(s.H << s.up2) &&
                                (unsigned)ix < (unsigned)(s.W << s.up2);
                uint32_t off = ((((uint32_t)img * s.C + c) * s.H + (iy >> s.up2)) * s.W +
                                (ix >> s.up2)) * 4u;
                breg[j] = bload(si ? rs1 : rs0, ok ? off : OOB);
            }
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
            int f = tid + i * NT;
            if (A_F4 % NT == 0 || f < A_F4) {
                int kr = f / (BM / 4);
                int mc = (f % (BM / 4)) * 4;
                *reinterpret_cast<float4*>(&As[buf][kr][mc]) = areg[i];
            }
        }
#pragma unroll
        for (int j = 0; j < B_PER_T; ++j) Bs[buf][brow0 + j * B_RSTEP][bcol] = breg[j];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = (p.K + BK - 1) / BK;
    load_tile(0);
    store_tile(0);
    __syncthreads();

    const int h = lane >> 5, l32 = lane & 31;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = STAGES == 1 ? 0 : (kt & 1);
        if (kt + 1 < nk) load_tile(kt + 1);
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            float a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) a[i] = As[cur][2 * s + h][wm * WTM + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < TN; ++j) b[j] = Bs[cur][2 * s + h][wn * WTN + j * 32 + l32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if constexpr (STAGES == 1) {
            __syncthreads();
            if (kt + 1 < nk) {
                store_tile(0);
                __syncthreads();
            }
        } else {
            if (kt + 1 < nk) store_tile(cur ^ 1);
            __syncthreads();
        }
    }

    // Epilogue: bias (+ residual) (+ ReLU), NCHW store.
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nn = n0 + wn * WTN + j * 32 + l32;
        if (nn >= p.N) continue;
        const int im = nn / p.HWo;
        const int hw = nn - im * p.HWo;
        const long obase = (long)im * p.Cout * p.HWo + hw;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= p.Cout) continue;
                float v = acc[i][j][r] + p.bias[m];
                const long o = obase + (long)m * p.HWo;
                if (p.res) v += p.res[o];
                if (p.relu) v = relu_nan(v);
                p.out[o] = v;
            }
        }
    }
}

template <int BM, int BN, int WM, int STAGES>
int launch(ConvP p, bool fast, hipStream_t st) {
    p.mtiles = (p.Cout + BM - 1) / BM;
    p.ntiles = (p.N + BN - 1) / BN;
    p.nblocks = p.mtiles * p.ntiles;
    if (fast) conv_mfma_kernel<BM, BN, WM, true, STAGES><<<p.nblocks, NT, 0, st>>>(p);
    else conv_mfma_kernel<BM, BN, WM, false, STAGES><<<p.nblocks, NT, 0, st>>>(p);
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

// Tile table: (BM, BN, LDS stages).  Blocks per CU follow from LDS (64 KiB
// double-buffered 128x128 -> 2, 32 KiB -> 4) and VGPRs.
struct TileCfg { int bm, bn, stages, per_cu; double eff; };
constexpr TileCfg kTiles[] = {
    {128, 128, 2, 2, 1.00}, {128, 64, 2, 3, 0.93}, {64, 128, 2, 3, 0.90}, {64, 64, 2, 5, 0.80},
    {32, 128, 2, 4, 0.75},  {128, 128, 1, 4, 0.95}, {128, 64, 1, 5, 0.90}, {64, 128, 1, 5, 0.88},
    {64, 64, 1, 8, 0.78},   {32, 128, 1, 6, 0.72}};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);
int g_force_tile = -1;

int launch_tile(int id, ConvP& p, bool fast, hipStream_t st) {
    switch (id) {
        case 0: return launch<128, 128, 2, 2>(p, fast, st);
        case 1: return launch<128, 64, 2, 2>(p, fast, st);
        case 2: return launch<64, 128, 2, 2>(p, fast, st);
        case 3: return launch<64, 64, 2, 2>(p, fast, st);
        case 4: return launch<32, 128, 1, 2>(p, fast, st);
        case 5: return launch<128, 128, 2, 1>(p, fast, st);
        case 6: return launch<128, 64, 2, 1>(p, fast, st);
        case 7: return launch<64, 128, 2, 1>(p, fast, st);
        case 8: return launch<64, 64, 2, 1>(p, fast, st);
        default: return launch<32, 128, 1, 1>(p, fast, st);
    }
}

// Measured on MI355X (scripts/tune_conv.py, profiles/round1_tune_conv.txt):
// the 32x128 single-stage tile (8 waves / SIMD) is the fastest or within 2 %
// on every fast-path layer of ResNet50-TCAM; the generic path (stem, Cin=3)
// prefers 64x64.
int choose_tile(const ConvP& p, bool fast) {
    if (fast) return 9;
    return 8;
}

// Wave-count model kept for shapes outside the measured set.
int choose_tile_model(const ConvP& p) {
    double best = 1e30;
    int bi = 0;
    for (int i = 0; i < kNumTiles; ++i) {
        const TileCfg& c = kTiles[i];
        if (c.bm > 32 && p.Cout <= c.bm / 2) continue;  // mostly empty M tiles
        if (c.bm == 32 && p.Cout > 64) continue;
        long nb = (long)((p.Cout + c.bm - 1) / c.bm) * ((p.N + c.bn - 1) / c.bn);
        long slots = 256L * c.per_cu;
        long waves = (nb + slots - 1) / slots;
        double t = (double)waves * c.bm * c.bn * c.per_cu / c.eff;
        if (t < best) { best = t; bi = i; }
    }
    return bi;
}

}  // namespace

extern "C" int tcam_conv_weight_dims(int K, int Cout, int* Kpad, int* Mpad) {
    TCAM_REQUIRE(K > 0 && Cout > 0 && Kpad && Mpad);
    *Kpad = (K + BK - 1) / BK * BK;
    *Mpad = (Cout + MPAD - 1) / MPAD * MPAD;
    return TCAM_OK;
}

extern "C" int tcam_conv2d(const tcam_conv_src* srcs, int nsrc, int B, const float* wt,
                           const float* bias, const float* residual, float* out, int Cout,
                           int Hout, int Wout, int KH, int KW, int pad, int relu,
                           void* stream) {
    TCAM_REQUIRE(srcs && (nsrc == 1 || nsrc == 2) && B > 0 && wt && bias && out);
    TCAM_REQUIRE(KH == KW && KH >= 1 && KH <= 7);
    TCAM_REQUIRE(Cout > 0 && Hout > 0 && Wout > 0);
    TCAM_REQUIRE(((uintptr_t)wt & 15) == 0);
    ConvP p{};
    bool fast = true;
    int ctot = 0;
    for (int i = 0; i < nsrc; ++i) {
        const tcam_conv_src& s = srcs[i];
        TCAM_REQUIRE(s.ptr && s.C > 0 && s.H > 0 && s.W > 0 && s.stride >= 1);
        long bytes = (long)B * s.C * s.H * s.W * 4;
        TCAM_REQUIRE(bytes < (long)OOB);  // 32-bit buffer offsets
        p.s[i] = Src{s.ptr, s.C, s.H, s.W, s.stride, s.up2 ? 1 : 0, (uint32_t)bytes};
        if (s.C % 16) fast = false;
        ctot += s.C;
    }
    if (nsrc == 1) p.s[1] = p.s[0];
    p.c0 = srcs[0].C;
    p.Ctot = ctot;
    p.wt = wt;
    p.ldw = (Cout + MPAD - 1) / MPAD * MPAD;
    p.bias = bias;
    p.res = residual;
    p.out = out;
    p.Cout = Cout;
    p.Hout = Hout;
    p.Wout = Wout;
    p.pad = pad;
    p.relu = relu;
    p.KS = KH;
    p.K = ctot * KH * KW;
    p.HWo = Hout * Wout;
    long N = (long)B * Hout * Wout;
    TCAM_REQUIRE(N < (1L << 31));
    p.N = (int)N;
    const int id = (g_force_tile >= 0 && g_force_tile < kNumTiles) ? g_force_tile : choose_tile(p, fast);
    return launch_tile(id, p, fast, as_stream(stream));
}

// Tuning hook (scripts/tune_conv.py): force a tile config id, -1 = auto.
extern "C" int tcam_conv_force_tile(int id) {
    g_force_tile = id;
    return kNumTiles;
}
