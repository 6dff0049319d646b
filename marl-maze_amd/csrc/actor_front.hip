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
//           kGradLen floats; the caller sums the partial rows.  Sized for two
//           256-thread workgroups per CU (grid = 2 x CUs).
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

// Weights read by every lane alike go through the scalar cache: a pointer in
// the constant address space makes the uniform loads s_load_dword* into SGPRs
// that the FMAs take as their scalar operand (no LDS traffic, no VGPRs).
typedef const __attribute__((address_space(4))) float cfloat;
__device__ __forceinline__ cfloat* as_const(const float* p) { return (cfloat*)p; }

// o[a] = sum_b w[a][b] t[b], w = [OUT][20] row-major in global memory (scalar loads)
template <int OUT>
__device__ __forceinline__ void matvec_s(const float* w, const float t[kEmb], float o[OUT]) {
    cfloat* ws = as_const(w);
#pragma unroll
    for (int a = 0; a < OUT; a++) {
        float acc = 0.f;
#pragma unroll
        for (int b = 0; b < kEmb; b++) acc = fmaf(ws[a * kEmb + b], t[b], acc);
        o[a] = acc;
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
// 256 threads = 8 samples per iteration (32-lane group g = sample, lane i =
// token).  LDS per sample (floats): attention phase {K 23x10 | Q 23x10 |
// V 23x20 | P 23x23 | dS 23x23}; after a barrier the same words hold the
// weight-gradient operands {G = [dq|dk|dv] 23x40 | T 23x20 | dT 23x20 | X 23x4}.
// dctx rows are re-read from global (L1/L2) rather than staged.  With the
// Q/K/V weights that is 66.5 KB per workgroup: two workgroups (8 waves) per CU.
constexpr int kBwdRows = 8;
constexpr int kBwdThreads = 256;
constexpr int kOffK = 0, kOffQ = 230, kOffV = 460, kOffP = 920, kOffS = 1449;  // attention phase
constexpr int kOffG = 0, kOffT = 920, kOffD = 1380, kOffX = 1840;               // weight-gradient phase
constexpr int kSampleF = 1980;  // floats per sample (>= 1978 and >= 1932; multiple of 4)
constexpr int kQkvQuads = (2 * kKq + kEmb) * (kEmb / 4);  // 200 (row a, columns 4b..4b+3) of [40 x 20]
constexpr int kPQuads = kTok * kEmb;                      // 460 (token i, channel c) x 4 inputs
constexpr int kP1 = (kPQuads + kBwdThreads - 1) / kBwdThreads;  // 2

__global__ __launch_bounds__(kBwdThreads, 2) void k_front_bwd(FrontW W, const float* __restrict__ x, int ldx, int B,
                                                              int parity, const float* __restrict__ dh,
                                                              float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float sm[kBwdRows * kSampleF];
    const int g = threadIdx.x >> 5;
    const int i = threadIdx.x & 31;
    float* my = sm + g * kSampleF;
    // weight-gradient accumulators, fixed entry map (deterministic sums):
    //   dW_qkv [40 x 20] as 50 4x4 tiles x 5 token classes (j mod 5): thread t < 250
    //   dW_p / db_p: (token, 4 channels) units: thread t < 115
    const int qt = threadIdx.x / 5, qc = threadIdx.x % 5;  // tile (rows 4*(qt/5).., cols 4*(qt%5)..), token class
    const int qr0 = 4 * (qt / 5), qc0 = 4 * (qt % 5);
    float aq[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++) aq[a][0] = aq[a][1] = aq[a][2] = aq[a][3] = 0.f;
    const int ptk = threadIdx.x / 5, pc0 = 4 * (threadIdx.x % 5);  // token, first channel
    float ap[4][4], ab[4];
#pragma unroll
    for (int a = 0; a < 4; a++) ap[a][0] = ap[a][1] = ap[a][2] = ap[a][3] = ab[a] = 0.f;
    const int iters = (B + kBwdRows - 1) / kBwdRows;
    for (int it = blockIdx.x; it < iters; it += gridDim.x) {
        const int row0 = it * kBwdRows;
        const int nrow = min(kBwdRows, B - row0);
        const int row = row0 + g;
        const bool act = (i < kTok) && (g < nrow);
        __syncthreads();  // previous iteration's weight-gradient readers are done
        float dctx[kEmb];
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        const float* dhr = dh + (size_t)row * kRowF;
        if (act) {  // phase 1: embedding, q/k/v
            xv = xslice(x + (size_t)row * ldx, i, parity != 0);
            float t[kEmb], q[kKq], k[kKq], v[kEmb];
            embed(W, xv, i, t);
            matvec_s<kKq>(W.wq, t, q);
            matvec_s<kKq>(W.wk, t, k);
            matvec_s<kEmb>(W.wv, t, v);
#pragma unroll
            for (int c = 0; c < kEmb; c += 4) {
                const float4 d4 = *reinterpret_cast<const float4*>(dhr + i * kEmb + c);
                dctx[c] = d4.x;
                dctx[c + 1] = d4.y;
                dctx[c + 2] = d4.z;
                dctx[c + 3] = d4.w;
            }
#pragma unroll
            for (int a = 0; a < kKq; a += 2) {
                *reinterpret_cast<float2*>(my + kOffK + i * kKq + a) = make_float2(k[a], k[a + 1]);
                *reinterpret_cast<float2*>(my + kOffQ + i * kKq + a) = make_float2(q[a], q[a + 1]);
            }
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(my + kOffV + i * kEmb + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
        }
        __syncthreads();
        float dq[kKq];
        if (act) {  // phase 2: softmax row i, dP, dS, dq
            float q[kKq];
#pragma unroll
            for (int a = 0; a < kKq; a += 2) {
                const float2 q2 = *reinterpret_cast<const float2*>(my + kOffQ + i * kKq + a);
                q[a] = q2.x;
                q[a + 1] = q2.y;
            }
            float p[kTok];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = dot4<kKq>(q, my + kOffK + j * kKq) / kSqrtKq;
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
                dp[j] = dot4<kEmb>(dctx, my + kOffV + j * kEmb);  // dP_ij = dctx_i . v_j
                rs = fmaf(dp[j], p[j], rs);
            }
#pragma unroll
            for (int a = 0; a < kKq; a++) dq[a] = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                const float ds = (p[j] * (dp[j] - rs)) / kSqrtKq;  // softmax backward, then / sqrt(10)
                my[kOffP + i * kTok + j] = p[j];
                my[kOffS + i * kTok + j] = ds;
                axpy4<kKq>(dq, ds, my + kOffK + j * kKq);
            }
        }
        __syncthreads();
        float dk[kKq], dv[kEmb], dt[kEmb], t[kEmb];
        if (act) {  // phase 3: dv_i = sum_j P_ji dctx_j, dk_i = sum_j dS_ji q_j, dt_i
#pragma unroll
            for (int c = 0; c < kEmb; c++) dv[c] = 0.f;
#pragma unroll
            for (int a = 0; a < kKq; a++) dk[a] = 0.f;
#pragma unroll 4
            for (int j = 0; j < kTok; j++) {
                const float pj = my[kOffP + j * kTok + i];
                const float sj = my[kOffS + j * kTok + i];
                const float4* cj = reinterpret_cast<const float4*>(dhr + j * kEmb);
#pragma unroll
                for (int c = 0; c < kEmb / 4; c++) {
                    const float4 v = cj[c];
                    dv[4 * c] = fmaf(pj, v.x, dv[4 * c]);
                    dv[4 * c + 1] = fmaf(pj, v.y, dv[4 * c + 1]);
                    dv[4 * c + 2] = fmaf(pj, v.z, dv[4 * c + 2]);
                    dv[4 * c + 3] = fmaf(pj, v.w, dv[4 * c + 3]);
                }
                axpy4<kKq>(dk, sj, my + kOffQ + j * kKq);
            }
            // dt_i = dctx_i (residual) + Wq^T dq + Wk^T dk + Wv^T dv (scalar-loaded weights)
            cfloat* wq = as_const(W.wq);
            cfloat* wk = as_const(W.wk);
            cfloat* wv = as_const(W.wv);
#pragma unroll
            for (int b = 0; b < kEmb; b++) dt[b] = dctx[b];
#pragma unroll
            for (int r = 0; r < kKq; r++)
#pragma unroll
                for (int b = 0; b < kEmb; b++) dt[b] = fmaf(dq[r], wq[r * kEmb + b], dt[b]);
#pragma unroll
            for (int r = 0; r < kKq; r++)
#pragma unroll
                for (int b = 0; b < kEmb; b++) dt[b] = fmaf(dk[r], wk[r * kEmb + b], dt[b]);
#pragma unroll
            for (int r = 0; r < kEmb; r++)
#pragma unroll
                for (int b = 0; b < kEmb; b++) dt[b] = fmaf(dv[r], wv[r * kEmb + b], dt[b]);
        }
        __syncthreads();  // attention-phase words are dead: reuse them for the gradient operands
        if (act) {
            embed(W, xv, i, t);  // recomputed rather than held in registers through phases 2-3
            float* G = my + kOffG + i * (2 * kKq + kEmb);
#pragma unroll
            for (int a = 0; a < kKq; a += 2) {
                *reinterpret_cast<float2*>(G + a) = make_float2(dq[a], dq[a + 1]);
                *reinterpret_cast<float2*>(G + kKq + a) = make_float2(dk[a], dk[a + 1]);
            }
#pragma unroll
            for (int c = 0; c < kEmb; c += 4) {
                *reinterpret_cast<float4*>(G + 2 * kKq + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
                *reinterpret_cast<float4*>(my + kOffT + i * kEmb + c) = make_float4(t[c], t[c + 1], t[c + 2], t[c + 3]);
                *reinterpret_cast<float4*>(my + kOffD + i * kEmb + c) =
                    make_float4(dt[c], dt[c + 1], dt[c + 2], dt[c + 3]);
            }
            *reinterpret_cast<float4*>(my + kOffX + i * kPin) = xv;
        }
        __syncthreads();
        // phase 4: weight gradients of this iteration's nrow samples (4x4 register tiles)
        if (threadIdx.x < 250) {
            for (int gg = 0; gg < nrow; gg++) {
                const float* sg = sm + gg * kSampleF;
                for (int j = qc; j < kTok; j += 5) {
                    const float4 gv = *reinterpret_cast<const float4*>(sg + kOffG + j * (2 * kKq + kEmb) + qr0);
                    const float4 tv = *reinterpret_cast<const float4*>(sg + kOffT + j * kEmb + qc0);
                    const float gr[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                    for (int a = 0; a < 4; a++) {
                        aq[a][0] = fmaf(gr[a], tv.x, aq[a][0]);
                        aq[a][1] = fmaf(gr[a], tv.y, aq[a][1]);
                        aq[a][2] = fmaf(gr[a], tv.z, aq[a][2]);
                        aq[a][3] = fmaf(gr[a], tv.w, aq[a][3]);
                    }
                }
            }
        }
        if (threadIdx.x < kTok * (kEmb / 4)) {
            for (int gg = 0; gg < nrow; gg++) {
                const float* sg = sm + gg * kSampleF;
                const float4 dv4 = *reinterpret_cast<const float4*>(sg + kOffD + ptk * kEmb + pc0);
                const float4 xq = *reinterpret_cast<const float4*>(sg + kOffX + ptk * kPin);
                const float d[4] = {dv4.x, dv4.y, dv4.z, dv4.w};
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    ap[a][0] = fmaf(d[a], xq.x, ap[a][0]);
                    ap[a][1] = fmaf(d[a], xq.y, ap[a][1]);
                    ap[a][2] = fmaf(d[a], xq.z, ap[a][2]);
                    ap[a][3] = fmaf(d[a], xq.w, ap[a][3]);
                    ab[a] += d[a];
                }
            }
        }
    }
    // reduce the 5 token classes of dW_qkv through LDS, then write the partial row
    __syncthreads();
    float* red = sm;  // [250][16]
    if (threadIdx.x < 250) {
#pragma unroll
        for (int a = 0; a < 4; a++)
            *reinterpret_cast<float4*>(red + threadIdx.x * 16 + 4 * a) =
                make_float4(aq[a][0], aq[a][1], aq[a][2], aq[a][3]);
    }
    __syncthreads();
    float* out = partial + (size_t)blockIdx.x * kGradLen;
    for (int e = threadIdx.x; e < (2 * kKq + kEmb) * kEmb; e += kBwdThreads) {
        const int r = e / kEmb, c = e % kEmb;
        const int tile = (r / 4) * 5 + c / 4, within = (r % 4) * 4 + (c % 4);
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 5; k++) acc += red[(tile * 5 + k) * 16 + within];
        out[kGQ + e] = acc;
    }
    if (threadIdx.x < kTok * (kEmb / 4)) {
#pragma unroll
        for (int a = 0; a < 4; a++) {
            const int e = ptk * kEmb + pc0 + a;
            *reinterpret_cast<float4*>(out + kGP + e * kPin) = make_float4(ap[a][0], ap[a][1], ap[a][2], ap[a][3]);
            out[kGB + e] = ab[a];
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
