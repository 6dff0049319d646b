// actor_front.hip -- fused Actor front-end for gfx950: the 23 feature
// embeddings (networks.py:51-65), Q/K/V projections, softmax attention over
// the 23 tokens and the residual (networks.py:67-82), forward and backward.
//
// Why fused: per sample the front-end is a chain of 23x20 / 23x23 matrices.
// As library calls it becomes batched GEMMs with 10..23-wide tiles (the
// dominant cost of the PPO update before this kernel) plus [B,23,40]
// split/cat copies.  Here one 32-lane group owns one sample, lane i = token i
// (23 of 32 lanes active): its embedding, q, k, v stay in registers, the other
// tokens' k and v are read from LDS as wave-wide broadcasts, the weights
// (1.2 K floats, identical for every lane) come through the scalar cache.
// Arithmetic is fp32 in the reference's order per element (dot products in
// increasing index order, logits / sqrt(10), softmax = exp(x - max) / sum).
//
// Forward  : x [B, 65] -> h [B, 460] (= t + softmax(q k^T / sqrt10) v, flattened)
// Backward : dh [B, 460] -> dT [B, 23, 20] (grad of the embeddings, residual +
//            attention paths), dQ/dK [B, 23, 10], dV [B, 23, 20] and the
//            recomputed embeddings T [B, 23, 20]; the weight gradients are then
//            reductions over all B*23 tokens, done as GEMMs by the caller.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "marlmaze.h"

namespace mm {

constexpr int kTok = 23;    // FEATURE_AMOUNT
constexpr int kEmb = 20;    // EMBEDDING_DIM
constexpr int kKq = 10;     // kq_dim
constexpr int kPin = 4;     // max feature width (networks.py:8)
constexpr int kRowF = kTok * kEmb;  // 460

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

// Token embedding t_i = W_i x[s_i : s_i + d_i] + b_i  (Projection, Q1 quirk when parity)
__device__ __forceinline__ void embed(const FrontW& W, const float* __restrict__ x, int i, bool parity,
                                      float t[kEmb]) {
    const int d = c_dims[i];
    const int s = parity ? 0 : c_starts_fixed[i];
    float xv[kPin];
#pragma unroll
    for (int k = 0; k < kPin; k++) xv[k] = (k < d) ? x[s + k] : 0.f;
    const float* wi = W.wp + i * kEmb * kPin;
#pragma unroll
    for (int c = 0; c < kEmb; c++) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < kPin; k++)
            if (k < d) acc = __fadd_rn(acc, __fmul_rn(wi[c * kPin + k], xv[k]));
        t[c] = __fadd_rn(acc, W.bp[i * kEmb + c]);
    }
}

template <int OUT>
__device__ __forceinline__ void matvec(const float* w, const float t[kEmb], float o[OUT]) {
#pragma unroll
    for (int a = 0; a < OUT; a++) {
        float acc = 0.f;
#pragma unroll
        for (int b = 0; b < kEmb; b++) acc = __fadd_rn(acc, __fmul_rn(w[a * kEmb + b], t[b]));
        o[a] = acc;
    }
}

constexpr int kFwdRows = 8;  // samples per 256-thread workgroup

// Q/K/V weights staged once per workgroup in LDS (read as broadcasts: every
// lane of a wave reads the same word), so they do not occupy scalar registers.
struct WLds {
    float q[kKq * kEmb];
    float k[kKq * kEmb];
    float v[kEmb * kEmb];
};

__device__ __forceinline__ void stage_w(const FrontW& W, WLds& s) {
    for (int e = threadIdx.x; e < kKq * kEmb; e += blockDim.x) {
        s.q[e] = W.wq[e];
        s.k[e] = W.wk[e];
    }
    for (int e = threadIdx.x; e < kEmb * kEmb; e += blockDim.x) s.v[e] = W.wv[e];
}

__global__ __launch_bounds__(256) void k_front_fwd(FrontW W, const float* __restrict__ x, int ldx, int B,
                                                   int parity, float* __restrict__ h) {
    __shared__ float Ks[kFwdRows][kTok][kKq];
    __shared__ float Vs[kFwdRows][kTok][kEmb];
    __shared__ WLds Ws;
    stage_w(W, Ws);
    __syncthreads();
    const int g = threadIdx.x >> 5;  // sample slot in the block
    const int i = threadIdx.x & 31;  // token
    const int row = blockIdx.x * kFwdRows + g;
    const bool act = (i < kTok) && (row < B);
    float t[kEmb], q[kKq];
    if (act) {
        embed(W, x + (size_t)row * ldx, i, parity != 0, t);
        float k[kKq], v[kEmb];
        matvec<kKq>(Ws.q, t, q);
        matvec<kKq>(Ws.k, t, k);
        matvec<kEmb>(Ws.v, t, v);
#pragma unroll
        for (int a = 0; a < kKq; a++) Ks[g][i][a] = k[a];
#pragma unroll
        for (int a = 0; a < kEmb; a++) Vs[g][i][a] = v[a];
    }
    __syncthreads();
    if (!act) return;
    const float inv = 3.16227766016838f;  // f32(np.sqrt(10)): the reference divides by it
    float s[kTok];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < kTok; j++) {
        float acc = 0.f;
#pragma unroll
        for (int a = 0; a < kKq; a++) acc = __fadd_rn(acc, __fmul_rn(q[a], Ks[g][j][a]));
        s[j] = __fdiv_rn(acc, inv);
        mx = fmaxf(mx, s[j]);
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < kTok; j++) {
        s[j] = expf(__fsub_rn(s[j], mx));
        sum = __fadd_rn(sum, s[j]);
    }
    float out[kEmb];
#pragma unroll
    for (int c = 0; c < kEmb; c++) out[c] = 0.f;
#pragma unroll
    for (int j = 0; j < kTok; j++) {
        const float p = __fdiv_rn(s[j], sum);
#pragma unroll
        for (int c = 0; c < kEmb; c++) out[c] = __fadd_rn(out[c], __fmul_rn(p, Vs[g][j][c]));
    }
    float* o = h + (size_t)row * kRowF + i * kEmb;
#pragma unroll
    for (int c = 0; c < kEmb; c += 4)
        *reinterpret_cast<float4*>(o + c) = make_float4(__fadd_rn(t[c], out[c]), __fadd_rn(t[c + 1], out[c + 1]),
                                                        __fadd_rn(t[c + 2], out[c + 2]),
                                                        __fadd_rn(t[c + 3], out[c + 3]));
}

constexpr int kBwdRows = 4;  // samples per 128-thread workgroup

__global__ __launch_bounds__(128) void k_front_bwd(FrontW W, const float* __restrict__ x, int ldx, int B, int parity,
                                                   const float* __restrict__ dh, float* __restrict__ dT,
                                                   float* __restrict__ dQ, float* __restrict__ dK,
                                                   float* __restrict__ dV, float* __restrict__ Tout) {
    __shared__ float Qs[kBwdRows][kTok][kKq];
    __shared__ float Ks[kBwdRows][kTok][kKq];
    __shared__ float Vs[kBwdRows][kTok][kEmb];
    __shared__ float Ps[kBwdRows][kTok][kTok + 1];
    __shared__ float Ss[kBwdRows][kTok][kTok + 1];  // dS
    __shared__ float Cs[kBwdRows][kTok][kEmb];      // dctx
    __shared__ WLds Ws;
    stage_w(W, Ws);
    __syncthreads();
    const int g = threadIdx.x >> 5;
    const int i = threadIdx.x & 31;
    const int row = blockIdx.x * kBwdRows + g;
    const bool act = (i < kTok) && (row < B);
    float t[kEmb], q[kKq], k[kKq], dctx[kEmb];
    if (act) {
        embed(W, x + (size_t)row * ldx, i, parity != 0, t);
        float v[kEmb];
        matvec<kKq>(Ws.q, t, q);
        matvec<kKq>(Ws.k, t, k);
        matvec<kEmb>(Ws.v, t, v);
#pragma unroll
        for (int a = 0; a < kKq; a++) {
            Qs[g][i][a] = q[a];
            Ks[g][i][a] = k[a];
        }
#pragma unroll
        for (int a = 0; a < kEmb; a++) Vs[g][i][a] = v[a];
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
        for (int c = 0; c < kEmb; c++) Cs[g][i][c] = dctx[c];
    }
    __syncthreads();
    const float inv = 3.16227766016838f;
    float dq[kKq];
    if (act) {
        float p[kTok];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < kTok; j++) {
            float acc = 0.f;
#pragma unroll
            for (int a = 0; a < kKq; a++) acc = __fadd_rn(acc, __fmul_rn(q[a], Ks[g][j][a]));
            p[j] = __fdiv_rn(acc, inv);
            mx = fmaxf(mx, p[j]);
        }
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < kTok; j++) {
            p[j] = expf(__fsub_rn(p[j], mx));
            sum = __fadd_rn(sum, p[j]);
        }
        // dP_ij = dctx_i . v_j ; softmax backward ; / sqrt10
        float dp[kTok];
        float rs = 0.f;
#pragma unroll
        for (int j = 0; j < kTok; j++) {
            p[j] = __fdiv_rn(p[j], sum);
            float acc = 0.f;
#pragma unroll
            for (int c = 0; c < kEmb; c++) acc = __fadd_rn(acc, __fmul_rn(dctx[c], Vs[g][j][c]));
            dp[j] = acc;
            rs = __fadd_rn(rs, __fmul_rn(dp[j], p[j]));
        }
#pragma unroll
        for (int a = 0; a < kKq; a++) dq[a] = 0.f;
#pragma unroll
        for (int j = 0; j < kTok; j++) {
            const float ds = __fdiv_rn(__fmul_rn(p[j], __fsub_rn(dp[j], rs)), inv);
            Ps[g][i][j] = p[j];
            Ss[g][i][j] = ds;
#pragma unroll
            for (int a = 0; a < kKq; a++) dq[a] = __fadd_rn(dq[a], __fmul_rn(ds, Ks[g][j][a]));
        }
    }
    __syncthreads();
    if (!act) return;
    // dv_i = sum_j P_ji dctx_j ; dk_i = sum_j dS_ji q_j
    float dv[kEmb], dk[kKq];
#pragma unroll
    for (int c = 0; c < kEmb; c++) dv[c] = 0.f;
#pragma unroll
    for (int a = 0; a < kKq; a++) dk[a] = 0.f;
#pragma unroll
    for (int j = 0; j < kTok; j++) {
        const float pj = Ps[g][j][i];
        const float sj = Ss[g][j][i];
#pragma unroll
        for (int c = 0; c < kEmb; c++) dv[c] = __fadd_rn(dv[c], __fmul_rn(pj, Cs[g][j][c]));
#pragma unroll
        for (int a = 0; a < kKq; a++) dk[a] = __fadd_rn(dk[a], __fmul_rn(sj, Qs[g][j][a]));
    }
    // dt_i = dh_i (residual) + Wq^T dq + Wk^T dk + Wv^T dv
    float dt[kEmb];
#pragma unroll
    for (int b = 0; b < kEmb; b++) {
        float acc = dctx[b];
#pragma unroll
        for (int a = 0; a < kKq; a++) acc = __fadd_rn(acc, __fmul_rn(Ws.q[a * kEmb + b], dq[a]));
#pragma unroll
        for (int a = 0; a < kKq; a++) acc = __fadd_rn(acc, __fmul_rn(Ws.k[a * kEmb + b], dk[a]));
#pragma unroll
        for (int a = 0; a < kEmb; a++) acc = __fadd_rn(acc, __fmul_rn(Ws.v[a * kEmb + b], dv[a]));
        dt[b] = acc;
    }
    const size_t tok = (size_t)row * kTok + i;
#pragma unroll
    for (int c = 0; c < kEmb; c += 4) {
        *reinterpret_cast<float4*>(dT + tok * kEmb + c) = make_float4(dt[c], dt[c + 1], dt[c + 2], dt[c + 3]);
        *reinterpret_cast<float4*>(dV + tok * kEmb + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
        *reinterpret_cast<float4*>(Tout + tok * kEmb + c) = make_float4(t[c], t[c + 1], t[c + 2], t[c + 3]);
    }
#pragma unroll
    for (int a = 0; a < kKq; a += 2) {
        *reinterpret_cast<float2*>(dQ + tok * kKq + a) = make_float2(dq[a], dq[a + 1]);
        *reinterpret_cast<float2*>(dK + tok * kKq + a) = make_float2(dk[a], dk[a + 1]);
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

extern "C" int mm_actor_front_bwd(const float* wp, const float* bp, const float* wq, const float* wk,
                                  const float* wv, const float* x, int ldx, int B, int parity, const float* dh,
                                  float* dT, float* dQ, float* dK, float* dV, float* T, void* stream) {
    if (!wp || !bp || !wq || !wk || !wv || !x || !dh || !dT || !dQ || !dK || !dV || !T || B < 0 ||
        ldx < MM_OBS_DIM)
        return MM_E_ARG;
    if (B == 0) return 0;
    FrontW W{wp, bp, wq, wk, wv};
    hipLaunchKernelGGL(k_front_bwd, dim3((B + kBwdRows - 1) / kBwdRows), dim3(128), 0, (hipStream_t)stream, W, x,
                       ldx, B, parity, dh, dT, dQ, dK, dV, T);
    return (int)hipGetLastError();
}
