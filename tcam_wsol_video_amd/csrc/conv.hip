// Implicit-GEMM convolution on the fp32 MFMA pipe of gfx950.
//
//   out[b, m, p] = act( sum_k  Wt[k, m] * X[k, (b, p)]  + bias[m]  (+ res) )
//
// GEMM view: M = Cout, N = B * Hout * Wout (frames x output pixels, NCHW so
// p is contiguous), K = sum_src C_src * KH * KW.  X is never materialised:
// the B-operand tile is gathered straight from the NCHW sources (im2col on
// the fly), including the decoder's nearest-x2 upsample and skip concat
// (unet/decoder.py:41-57) and the bottleneck's conv3 + downsample pair
// (resnet.py:214-232), which become one GEMM over a concatenated K.
// BN is folded into Wt/bias on the host (eval mode, base/model.py:141-160).
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact k-ordered fp32 fma chain
// (cdna_hip_programming.md §3), so results differ from PyTorch CPU only by
// summation order.
//
// Tiling: BM x BN block tile, BK = 16, 256 threads = 4 waves, each wave a
// (TM*32) x (TN*32) sub-tile of 32x32x2 MFMAs.  Both operand tiles are staged
// in LDS (double buffered, one barrier per K-step); global loads for step
// t+1 are issued before the MFMAs of step t and written to LDS after them.
#include "common.h"

namespace {

constexpr int BK = 16;
constexpr int NT = 256;

struct Src {
    const float* ptr;
    int C, H, W, stride, up2;
};

struct ConvP {
    Src s0, s1;
    int c0;       // channels of source 0
    int B;
    const float* wt;
    const float* bias;
    const float* res;
    float* out;
    int Cout, Hout, Wout, pad, relu;
    int K, N, HWo;
};

template <int KS>
__device__ __forceinline__ float gather_x(const ConvP& p, int k, int img,
                                          int oh, int ow, bool nvalid) {
    constexpr int KHW = KS * KS;
    if (!nvalid || k >= p.K) return 0.f;
    int ci = k / KHW;
    int r = k - ci * KHW;
    int kh = r / KS;
    int kw = r - kh * KS;
    const Src& s = (ci < p.c0) ? p.s0 : p.s1;
    if (ci >= p.c0) ci -= p.c0;
    int iy = oh * s.stride - p.pad + kh;
    int ix = ow * s.stride - p.pad + kw;
    int Hv = s.H << s.up2, Wv = s.W << s.up2;
    if ((unsigned)iy >= (unsigned)Hv || (unsigned)ix >= (unsigned)Wv) return 0.f;
    iy >>= s.up2;
    ix >>= s.up2;
    return s.ptr[(((long)img * s.C + ci) * s.H + iy) * s.W + ix];
}

template <int BM, int BN, int WM, int KS>
__global__ __launch_bounds__(NT) void conv_mfma_kernel(ConvP p) {
    constexpr int WN = 4 / WM;
    constexpr int WTM = BM / WM;  // wave tile rows
    constexpr int WTN = BN / WN;  // wave tile cols
    constexpr int TM = WTM / 32;
    constexpr int TN = WTN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile too small");
    constexpr int A_F4 = BM * BK / 4;              // float4 per A tile
    constexpr int A_PER_T = (A_F4 + NT - 1) / NT;
    constexpr int B_PER_T = BK * BN / NT;           // gathered floats / thread
    constexpr int B_RSTEP = NT / BN;                // row step between them

    __shared__ float As[2][BK][BM];
    __shared__ float Bs[2][BK][BN];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;

    const int mtiles = (p.Cout + BM - 1) / BM;
    const int m0 = (blockIdx.x % mtiles) * BM;
    const int n0 = (blockIdx.x / mtiles) * BN;

    // This thread's fixed B column.
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

    float4 areg[A_PER_T];
    float breg[B_PER_T];

    auto load_tile = [&](int kt) {
        const int kbase = kt * BK;
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
            int f = tid + i * NT;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (f < A_F4) {
                int kr = f / (BM / 4);
                int mc = (f % (BM / 4)) * 4;
                int k = kbase + kr, m = m0 + mc;
                if (k < p.K && m < p.Cout)
                    v = *reinterpret_cast<const float4*>(p.wt + (long)k * p.Cout + m);
            }
            areg[i] = v;
        }
#pragma unroll
        for (int j = 0; j < B_PER_T; ++j) {
            int k = kbase + brow0 + j * B_RSTEP;
            breg[j] = gather_x<KS>(p, k, img, oh, ow, nvalid);
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_PER_T; ++i) {
            int f = tid + i * NT;
            if (f < A_F4) {
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
        const int cur = kt & 1;
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
        if (kt + 1 < nk) store_tile(cur ^ 1);
        __syncthreads();
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
                if (p.relu) v = fmaxf(v, 0.f);
                p.out[o] = v;
            }
        }
    }
}

template <int BM, int BN, int WM>
int launch_ks(const ConvP& p, int KS, hipStream_t st) {
    const int mtiles = (p.Cout + BM - 1) / BM;
    const int ntiles = (p.N + BN - 1) / BN;
    dim3 grid(mtiles * ntiles);
    switch (KS) {
        case 1: conv_mfma_kernel<BM, BN, WM, 1><<<grid, NT, 0, st>>>(p); break;
        case 3: conv_mfma_kernel<BM, BN, WM, 3><<<grid, NT, 0, st>>>(p); break;
        case 7: conv_mfma_kernel<BM, BN, WM, 7><<<grid, NT, 0, st>>>(p); break;
        default: return TCAM_E_ARG;
    }
    TCAM_CHECK_LAUNCH();
    return TCAM_OK;
}

}  // namespace

extern "C" int tcam_conv2d(const tcam_conv_src* srcs, int nsrc, int B,
                           const float* wt, const float* bias,
                           const float* residual, float* out, int Cout,
                           int Hout, int Wout, int KH, int KW, int pad,
                           int relu, void* stream) {
    TCAM_REQUIRE(srcs && (nsrc == 1 || nsrc == 2) && B > 0 && wt && bias && out);
    TCAM_REQUIRE(KH == KW && (KH == 1 || KH == 3 || KH == 7));
    TCAM_REQUIRE(Cout > 0 && (Cout % 4) == 0 && Hout > 0 && Wout > 0);
    TCAM_REQUIRE(((uintptr_t)wt & 15) == 0);
    ConvP p{};
    auto mk = [](const tcam_conv_src& s) {
        Src r{s.ptr, s.C, s.H, s.W, s.stride, s.up2 ? 1 : 0};
        return r;
    };
    for (int i = 0; i < nsrc; ++i) {
        const tcam_conv_src& s = srcs[i];
        // Taps are bounds-checked per element in the kernel.
        TCAM_REQUIRE(s.ptr && s.C > 0 && s.H > 0 && s.W > 0 && s.stride >= 1);
    }
    p.s0 = mk(srcs[0]);
    p.c0 = srcs[0].C;
    if (nsrc == 2) p.s1 = mk(srcs[1]);
    else { p.s1 = p.s0; }
    const int Ctot = srcs[0].C + (nsrc == 2 ? srcs[1].C : 0);
    p.B = B;
    p.wt = wt;
    p.bias = bias;
    p.res = residual;
    p.out = out;
    p.Cout = Cout;
    p.Hout = Hout;
    p.Wout = Wout;
    p.pad = pad;
    p.relu = relu;
    p.K = Ctot * KH * KW;
    p.HWo = Hout * Wout;
    long N = (long)B * Hout * Wout;
    TCAM_REQUIRE(N < (1L << 31));
    p.N = (int)N;
    hipStream_t st = as_stream(stream);
    if (Cout >= 128) return launch_ks<128, 128, 2>(p, KH, st);
    if (Cout >= 64) return launch_ks<64, 128, 2>(p, KH, st);
    return launch_ks<32, 128, 1>(p, KH, st);
}
