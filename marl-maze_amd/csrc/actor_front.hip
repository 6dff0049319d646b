// actor_front.hip -- fused Actor front-end for gfx950: the 23 feature
// embeddings (networks.py:51-65), Q/K/V projections, softmax attention over
// the 23 tokens and the residual (networks.py:67-82), forward and backward.
//
// Why fused: per sample the front-end is a chain of 23x20 / 23x23 matrices.
// As library calls it becomes batched GEMMs with 10..23-wide tiles plus
// [B,23,40] split/cat copies -- the dominant cost of the PPO update.  Here a
// 32-lane group owns one sample, lane i = token i (23 of 32 lanes active):
// its embedding t_i and q_i stay in registers; every token's k, v (and in the
// backward q, P, dS, dctx) sit in LDS and are read as wave-wide broadcasts
// with 16-byte reads; the Q/K/V weights are staged once per workgroup in LDS.
// fp32 throughout (fmaf accumulation; the reference's op order per element:
// logits / sqrt(10), softmax = exp(x - max) / sum).
//
// Forward : x [B, ldx] -> h [B, 460] = t + softmax(q k^T / sqrt(10)) v
// Backward: persistent grid; each workgroup accumulates the weight gradients
//           of the rows it owns in registers (fixed entry -> thread map, so the
//           sum order is deterministic) and writes ONE partial row of
//           kGradLen floats; the caller sums the partial rows.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "marlmaze.h"

namespace mm {

constexpr int kTok = 23;            // FEATURE_AMOUNT
constexpr int kEmb = 20;            // EMBEDDING_DIM
constexpr int kKq = 10;             // kq_dim
constexpr int kPin = 4;             // max feature width (networks.py:8)
constexpr int kRowF = kTok * kEmb;  // 460
constexpr float kSqrtKq = 3.16227766016838f;  // f32(np.sqrt(10)): the reference divides by it

// gradient partial layout: [wq 10x20 | wk 10x20 | wv 20x20 | wp 23x20x4 | bp 23x20]
constexpr int kGQ = 0, kGK = 200, kGV = 400, kGP = 800, kGB = 800 + kTok * kEmb * kPin;
constexpr int kGradLen = kGB + kTok * kEmb;  // 3100

__constant__ int c_dims[kTok] = {4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 2, 2, 1, 4, 1, 1, 1, 1, 1, 1, 2};
__constant__ int c_starts_fixed[kTok] = {0,  4,  8,  12, 16, 20, 24, 28, 32, 36, 40, 44,
                                         48, 50, 52, 53, 57, 58, 59, 60, 61, 62, 63};

struct FrontW {
    const float* wp;  // [23][20][4] per-token projection weights, zero beyond d_i
    const float* bp;  // [23][20]
    const float* wq;  // [10][20]  (nn.Linear weight: [out, in])
    const float* wk;  // [10][20]
    const float* wv;  // [20][20]
};

struct WLds {  // Q/K/V weights: [40][20] = rows of wq, wk, wv
    float w[2 * kKq + kEmb][kEmb];
};

__device__ __forceinline__ void stage_w(const FrontW& W, WLds& s) {
    for (int e = threadIdx.x; e < (2 * kKq + kEmb) * kEmb; e += blockDim.x) {
        const int r = e / kEmb, c = e % kEmb;
        s.w[r][c] = r < kKq ? W.wq[e] : (r < 2 * kKq ? W.wk[e - kKq * kEmb] : W.wv[e - 2 * kKq * kEmb]);
    }
}

// x slice of token i (zero beyond d_i)
__device__ __forceinline__ float4 xslice(const float* __restrict__ xr, int i, bool parity) {
    const int d = c_dims[i];
    const int s = parity ? 0 : c_starts_fixed[i];
    return make_float4(xr[s], d > 1 ? xr[s + 1] : 0.f, d > 2 ? xr[s + 2] : 0.f, d > 3 ? xr[s + 3] : 0.f);
}

// Token embedding t_i = W_i x_i + b_i (Projection; quirk Q1 when parity)
__device__ __forceinline__ void embed(const FrontW& W, float4 xv, int i, float t[kEmb]) {
    const float4* wi = reinterpret_cast<const float4*>(W.wp) + i * kEmb;
#pragma unroll
    for (int c = 0; c < kEmb; c++) {
        const float4 w = wi[c];
        float acc = w.x * xv.x;
        acc = fmaf(w.y, xv.y, acc);
        acc = fmaf(w.z, xv.z, acc);
        acc = fmaf(w.w, xv.w, acc);
        t[c] = acc + W.bp[i * kEmb + c];
    }
}

// o[a] = sum_b w[r0 + a][b] t[b]
template <int OUT>
__device__ __forceinline__ void matvec(const WLds& s, int r0, const float t[kEmb], float o[OUT]) {
#pragma unroll
    for (int a = 0; a < OUT; a++) {
        const float4* w4 = reinterpret_cast<const float4*>(s.w[r0 + a]);
        float acc = 0.f;
#pragma unroll
        for (int b = 0; b < kEmb / 4; b++) {
            const float4 w = w4[b];
            acc = fmaf(w.x, t[4 * b], acc);
            acc = fmaf(w.y, t[4 * b + 1], acc);
            acc = fmaf(w.z, t[4 * b + 2], acc);
            acc = fmaf(w.w, t[4 * b + 3], acc);
        }
        o[a] = acc;
    }
}

template <int N>
__device__ __forceinline__ float dot4(const float* a, const float* __restrict__ b_lds) {  // N % 2 == 0
    float acc = 0.f;
    if constexpr (N % 4 == 0) {
        const float4* b4 = reinterpret_cast<const float4*>(b_lds);
#pragma unroll
        for (int k = 0; k < N / 4; k++) {
            const float4 v = b4[k];
            acc = fmaf(a[4 * k], v.x, acc);
            acc = fmaf(a[4 * k + 1], v.y, acc);
            acc = fmaf(a[4 * k + 2], v.z, acc);
            acc = fmaf(a[4 * k + 3], v.w, acc);
        }
    } else {
        const float2* b2 = reinterpret_cast<const float2*>(b_lds);
#pragma unroll
        for (int k = 0; k < N / 2; k++) {
            const float2 v = b2[k];
            acc = fmaf(a[2 * k], v.x, acc);
            acc = fmaf(a[2 * k + 1], v.y, acc);
        }
    }
    return acc;
}

template <int N>
__device__ __forceinline__ void axpy4(float* acc, float p, const float* __restrict__ v_lds) {  // acc += p * v
    if constexpr (N % 4 == 0) {
        const float4* v4 = reinterpret_cast<const float4*>(v_lds);
#pragma unroll
        for (int k = 0; k < N / 4; k++) {
            const float4 v = v4[k];
            acc[4 * k] = fmaf(p, v.x, acc[4 * k]);
            acc[4 * k + 1] = fmaf(p, v.y, acc[4 * k + 1]);
            acc[4 * k + 2] = fmaf(p, v.z, acc[4 * k + 2]);
            acc[4 * k + 3] = fmaf(p, v.w, acc[4 * k + 3]);
        }
    } else {
        const float2* v2 = reinterpret_cast<const float2*>(v_lds);
#pragma unroll
        for (int k = 0; k < N / 2; k++) {
            const float2 v = v2[k];
            acc[2 * k] = fmaf(p, v.x, acc[2 * k]);
            acc[2 * k + 1] = fmaf(p, v.y, acc[2 * k + 1]);
        }
    }
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
constexpr int kFwdRows = 8;  // samples per 256-thread workgroup

__global__ __launch_bounds__(256) void k_front_fwd(FrontW W, const float* __restrict__ x, int ldx, int B,
                                                   int parity, float* __restrict__ h) {
    __shared__ __attribute__((aligned(16))) float Ks[kFwdRows][kTok][kKq];
    __shared__ __attribute__((aligned(16))) float Vs[kFwdRows][kTok][kEmb];
    __shared__ __attribute__((aligned(16))) WLds Ws;
    stage_w(W, Ws);
    __syncthreads();
    const int g = threadIdx.x >> 5;  // sample slot in the workgroup
    const int i = threadIdx.x & 31;  // token
    const int row = blockIdx.x * kFwdRows + g;
    const bool act = (i < kTok) && (row < B);
    float t[kEmb], q[kKq];
    if (act) {
        embed(W, xslice(x + (size_t)row * ldx, i, parity != 0), i, t);
        float k[kKq], v[kEmb];
        matvec<kKq>(Ws, 0, t, q);
        matvec<kKq>(Ws, kKq, t, k);
        matvec<kEmb>(Ws, 2 * kKq, t, v);
#pragma unroll
        for (int a = 0; a < kKq; a++) Ks[g][i][a] = k[a];
#pragma unroll
        for (int a = 0; a < kEmb; a++) Vs[g][i][a] = v[a];
    }
    __syncthreads();
    if (!act) return;
    float s[kTok];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kTok; j++) {
        s[j] = dot4<kKq>(q, Ks[g][j]) / kSqrtKq;
        mx = fmaxf(mx, s[j]);
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < kTok; j++) {
        s[j] = expf(s[j] - mx);
        sum += s[j];
    }
    float out[kEmb];
#pragma unroll
    for (int c = 0; c < kEmb; c++) out[c] = 0.f;
#pragma unroll
    for (int j = 0; j < kTok; j++) axpy4<kEmb>(out, s[j] / sum, Vs[g][j]);
    float* o = h + (size_t)row * kRowF + i * kEmb;
#pragma unroll
    for (int c = 0; c < kEmb; c += 4)
        *reinterpret_cast<float4*>(o + c) =
            make_float4(t[c] + out[c], t[c + 1] + out[c + 1], t[c + 2] + out[c + 2], t[c + 3] + out[c + 3]);
}

// ---------------------------------------------------------------------------
// backward (persistent, in-kernel weight-gradient reduction)
// ---------------------------------------------------------------------------
constexpr int kBwdRows = 4;      // samples per iteration of a 128-thread workgroup
constexpr int kBwdThreads = 128;
constexpr int kQkvQuads = (2 * kKq + kEmb) * (kEmb / 4);  // 200 (row a, columns 4b..4b+3) of [40 x 20]
constexpr int kPQuads = kTok * kEmb;                      // 460 (token i, channel c) x 4 inputs
constexpr int kQ1 = (kQkvQuads + kBwdThreads - 1) / kBwdThreads;  // 2
constexpr int kP1 = (kPQuads + kBwdThreads - 1) / kBwdThreads;    // 4

struct BwdLds {
    float Q[kBwdRows][kTok][kKq];
    float K[kBwdRows][kTok][kKq];
    float V[kBwdRows][kTok][kEmb];
    float T[kBwdRows][kTok][kEmb];
    float C[kBwdRows][kTok][kEmb];     // dctx = dh
    float P[kBwdRows][kTok][kTok + 1];
    float S[kBwdRows][kTok][kTok + 1];  // dS
    float G[kBwdRows][kTok][2 * kKq + kEmb];  // [dq | dk | dv] per token
    float D[kBwdRows][kTok][kEmb];     // dt
    float X[kBwdRows][kTok][kPin];     // token input slices
};

__global__ __launch_bounds__(kBwdThreads) void k_front_bwd(FrontW W, const float* __restrict__ x, int ldx, int B,
                                                           int parity, const float* __restrict__ dh,
                                                           float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) BwdLds L;
    __shared__ __attribute__((aligned(16))) WLds Ws;
    stage_w(W, Ws);
    const int g = threadIdx.x >> 5;
    const int i = threadIdx.x & 31;
    // weight-gradient accumulators owned by this thread
    float aq[kQ1][4], ap[kP1][4], ab[kP1];
#pragma unroll
    for (int u = 0; u < kQ1; u++) aq[u][0] = aq[u][1] = aq[u][2] = aq[u][3] = 0.f;
#pragma unroll
    for (int u = 0; u < kP1; u++) {
        ap[u][0] = ap[u][1] = ap[u][2] = ap[u][3] = 0.f;
        ab[u] = 0.f;
    }
    const int iters = (B + kBwdRows - 1) / kBwdRows;
    for (int it = blockIdx.x; it < iters; it += gridDim.x) {
        const int row = it * kBwdRows + g;
        const bool act = (i < kTok) && (row < B);
        __syncthreads();  // previous iteration's readers are done with L
        float t[kEmb], q[kKq], dctx[kEmb];
        if (i < kTok) {
            if (act) {
                const float4 xv = xslice(x + (size_t)row * ldx, i, parity != 0);
                *reinterpret_cast<float4*>(L.X[g][i]) = xv;
                embed(W, xv, i, t);
                float k[kKq], v[kEmb];
                matvec<kKq>(Ws, 0, t, q);
                matvec<kKq>(Ws, kKq, t, k);
                matvec<kEmb>(Ws, 2 * kKq, t, v);
                const float* dhi = dh + (size_t)row * kRowF + i * kEmb;
#pragma unroll
                for (int c = 0; c < kEmb; c += 4) {
                    const float4 d4 = *reinterpret_cast<const float4*>(dhi + c);
                    dctx[c] = d4.x;
                    dctx[c + 1] = d4.y;
                    dctx[c + 2] = d4.z;
                    dctx[c + 3] = d4.w;
                }
#pragma unroll
                for (int a = 0; a < kKq; a++) {
                    L.Q[g][i][a] = q[a];
                    L.K[g][i][a] = k[a];
                }
#pragma unroll
                for (int c = 0; c < kEmb; c++) {
                    L.V[g][i][c] = v[c];
                    L.T[g][i][c] = t[c];
                    L.C[g][i][c] = dctx[c];
                }
            } else {  // padding rows contribute nothing to the weight gradients
                *reinterpret_cast<float4*>(L.X[g][i]) = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int a = 0; a < kKq; a++) L.Q[g][i][a] = L.K[g][i][a] = 0.f;
#pragma unroll
                for (int c = 0; c < kEmb; c++) L.V[g][i][c] = L.T[g][i][c] = L.C[g][i][c] = 0.f;
            }
        }
        __syncthreads();
        if (act) {
            float p[kTok];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = dot4<kKq>(q, L.K[g][j]) / kSqrtKq;
                mx = fmaxf(mx, p[j]);
            }
            float sum = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = expf(p[j] - mx);
                sum += p[j];
            }
            float dp[kTok];
            float rs = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = p[j] / sum;
                dp[j] = dot4<kEmb>(dctx, L.V[g][j]);  // dP_ij = dctx_i . v_j
                rs = fmaf(dp[j], p[j], rs);
            }
            float dq[kKq];
#pragma unroll
            for (int a = 0; a < kKq; a++) dq[a] = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                const float ds = (p[j] * (dp[j] - rs)) / kSqrtKq;  // softmax backward, then / sqrt(10)
                L.P[g][i][j] = p[j];
                L.S[g][i][j] = ds;
                axpy4<kKq>(dq, ds, L.K[g][j]);
            }
#pragma unroll
            for (int a = 0; a < kKq; a++) L.G[g][i][a] = dq[a];
        } else if (i < kTok) {
#pragma unroll
            for (int j = 0; j < kTok; j++) L.P[g][i][j] = L.S[g][i][j] = 0.f;
#pragma unroll
            for (int a = 0; a < kKq; a++) L.G[g][i][a] = 0.f;
        }
        __syncthreads();
        if (i < kTok) {
            // dv_i = sum_j P_ji dctx_j ; dk_i = sum_j dS_ji q_j
            float dv[kEmb], dk[kKq];
#pragma unroll
            for (int c = 0; c < kEmb; c++) dv[c] = 0.f;
#pragma unroll
            for (int a = 0; a < kKq; a++) dk[a] = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                axpy4<kEmb>(dv, L.P[g][j][i], L.C[g][j]);
                axpy4<kKq>(dk, L.S[g][j][i], L.Q[g][j]);
            }
#pragma unroll
            for (int a = 0; a < kKq; a++) L.G[g][i][kKq + a] = dk[a];
#pragma unroll
            for (int c = 0; c < kEmb; c++) L.G[g][i][2 * kKq + c] = dv[c];
            // dt_i = dctx_i (residual) + Wq^T dq + Wk^T dk + Wv^T dv
            float dt[kEmb];
#pragma unroll
            for (int b = 0; b < kEmb; b++) dt[b] = L.C[g][i][b];
#pragma unroll
            for (int r = 0; r < 2 * kKq + kEmb; r++) {
                const float gr = (r < kKq) ? L.G[g][i][r] : (r < 2 * kKq ? dk[r - kKq] : dv[r - 2 * kKq]);
                axpy4<kEmb>(dt, gr, Ws.w[r]);
            }
#pragma unroll
            for (int c = 0; c < kEmb; c++) L.D[g][i][c] = dt[c];
        }
        __syncthreads();
        // weight gradients of this iteration's rows, fixed thread -> entry map
#pragma unroll
        for (int u = 0; u < kQ1; u++) {
            const int e = threadIdx.x + u * kBwdThreads;  // quad over [40 x 20]
            if (e < kQkvQuads) {
                const int r = e / (kEmb / 4), c4 = e % (kEmb / 4);
                for (int gg = 0; gg < kBwdRows; gg++)
#pragma unroll
                    for (int j = 0; j < kTok; j++) {
                        const float gr = L.G[gg][j][r];
                        const float4 tv = reinterpret_cast<const float4*>(L.T[gg][j])[c4];
                        aq[u][0] = fmaf(gr, tv.x, aq[u][0]);
                        aq[u][1] = fmaf(gr, tv.y, aq[u][1]);
                        aq[u][2] = fmaf(gr, tv.z, aq[u][2]);
                        aq[u][3] = fmaf(gr, tv.w, aq[u][3]);
                    }
            }
        }
#pragma unroll
        for (int u = 0; u < kP1; u++) {
            const int e = threadIdx.x + u * kBwdThreads;  // (token, channel)
            if (e < kPQuads) {
                const int tk = e / kEmb, c = e % kEmb;
#pragma unroll
                for (int gg = 0; gg < kBwdRows; gg++) {
                    const float d = L.D[gg][tk][c];
                    const float4 xv = *reinterpret_cast<const float4*>(L.X[gg][tk]);
                    ap[u][0] = fmaf(d, xv.x, ap[u][0]);
                    ap[u][1] = fmaf(d, xv.y, ap[u][1]);
                    ap[u][2] = fmaf(d, xv.z, ap[u][2]);
                    ap[u][3] = fmaf(d, xv.w, ap[u][3]);
                    ab[u] += d;
                }
            }
        }
    }
    float* out = partial + (size_t)blockIdx.x * kGradLen;
#pragma unroll
    for (int u = 0; u < kQ1; u++) {
        const int e = threadIdx.x + u * kBwdThreads;
        if (e < kQkvQuads) {
            const int r = e / (kEmb / 4), c4 = e % (kEmb / 4);
            *reinterpret_cast<float4*>(out + kGQ + r * kEmb + 4 * c4) =
                make_float4(aq[u][0], aq[u][1], aq[u][2], aq[u][3]);
        }
    }
#pragma unroll
    for (int u = 0; u < kP1; u++) {
        const int e = threadIdx.x + u * kBwdThreads;
        if (e < kPQuads) {
            *reinterpret_cast<float4*>(out + kGP + e * kPin) = make_float4(ap[u][0], ap[u][1], ap[u][2], ap[u][3]);
            out[kGB + e] = ab[u];
        }
    }
}

}  // namespace mm

using namespace mm;

extern "C" int mm_actor_front_fwd(const float* wp, const float* bp, const float* wq, const float* wk,
                                  const float* wv, const float* x, int ldx, int B, int parity, float* h,
                                  void* stream) {
    if (!wp || !bp || !wq || !wk || !wv || !x || !h || B < 0 || ldx < MM_OBS_DIM) return MM_E_ARG;
    if (B == 0) return 0;
    FrontW W{wp, bp, wq, wk, wv};
    hipLaunchKernelGGL(k_front_fwd, dim3((B + kFwdRows - 1) / kFwdRows), dim3(256), 0, (hipStream_t)stream, W, x,
                       ldx, B, parity, h);
    return (int)hipGetLastError();
}

extern "C" int mm_actor_front_grad_len(void) { return kGradLen; }

extern "C" int mm_actor_front_bwd(const float* wp, const float* bp, const float* wq, const float* wk,
                                  const float* wv, const float* x, int ldx, int B, int parity, const float* dh,
                                  float* partial, int grid, void* stream) {
    if (!wp || !bp || !wq || !wk || !wv || !x || !dh || !partial || B < 0 || ldx < MM_OBS_DIM || grid <= 0)
        return MM_E_ARG;
    FrontW W{wp, bp, wq, wk, wv};
    hipLaunchKernelGGL(k_front_bwd, dim3(grid), dim3(kBwdThreads), 0, (hipStream_t)stream, W, x, ldx, B, parity, dh,
                       partial);
    return (int)hipGetLastError();
}
