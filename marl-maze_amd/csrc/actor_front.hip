// actor_front.hip -- fused Actor front-end for gfx950: the 23 feature
// embeddings (networks.py:51-65), Q/K/V projections, softmax attention over
// the 23 tokens and the residual (networks.py:67-82), forward and backward.
//
// Why fused: per sample the front-end is a chain of 23x20 / 23x23 matrices.
// As library calls it becomes batched GEMMs with 10..23-wide tiles plus
// [B,23,40] split/cat copies.  Here a 32-lane group owns one sample, lane i =
// token i (23 of 32 lanes active): its own vectors stay in registers, every
// token's k, v (and in the backward q, P, dS) sit in LDS and are read as
// broadcasts.  fp32 throughout (fmaf accumulation; the reference's op order
// per element: logits / sqrt(10), softmax = exp(x - max) * (1 / sum)).
//
// Linear-map folding.  Token i's input is a <= 4-wide slice x_i, and
//   t_i = Wp_i x_i + b_i,   [q|k|v]_i = Wqkv t_i = (Wqkv Wp_i) x_i + Wqkv b_i,
// so k_front_prep folds A_i = Wqkv Wp_i [40x4] and c_i = Wqkv b_i once per
// call (parameters are fixed within a forward/backward), and the kernels
// form q, k, v with 4 FMAs per output instead of 20.  In the backward the
// gradient of t_i is only needed for dWp_i = sum dt x^T and dbp_i = sum dt, and
// dt = dctx + Wqkv^T g (g = [dq|dk|dv]), so the kernel accumulates
// E_i = sum g x^T, F_i = sum dctx x^T, e_i = sum g, f_i = sum dctx and
// k_front_combine applies Wqkv^T once at the end.  The same sums give the
// attention weights' gradient: dWqkv = sum_s,i g t_i^T with t_i = Wp_i x_i +
// b_i, so dWqkv = sum_i (E_i Wp_i^T + e_i b_i^T) -- formed once in
// k_front_combine (92k FMAs per call) instead of 18.4k FMAs per sample.
//
// Workspace (k_front_prep): [Wp 23x20x4 | bp 23x20 | A 23x40x4 | c 23x40 | Wqkv 40x20 | A^T 23x4x40]
// Forward : x [B, ldx] -> h [B, 460] = t + softmax(q k^T / sqrt(10)) v
// Backward: persistent grid of 256-thread workgroups (8 samples per
//           iteration, two workgroups per CU); fixed entry -> thread maps, so
//           every sum has a fixed order (deterministic).  Each workgroup writes
//           one partial row; k_front_sum adds the rows, k_front_combine forms
//           the parameter gradients.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "marlmaze.h"

namespace mm {

// loop-unroll build knobs of the backward (tools/front_variants.sh; the defaults are the measured best)
#ifndef FRONT_P3_UNROLL
#define FRONT_P3_UNROLL 4
#endif
#ifndef FRONT_EF_UNROLL
#define FRONT_EF_UNROLL 2
#endif
#ifndef FRONT_EF_ROWS
#define FRONT_EF_ROWS 4
#endif

constexpr int kTok = 23;            // FEATURE_AMOUNT
constexpr int kEmb = 20;            // EMBEDDING_DIM
constexpr int kKq = 10;             // kq_dim
constexpr int kQkv = 2 * kKq + kEmb;  // 40 rows of [wq; wk; wv]
constexpr int kPin = 4;             // max feature width (networks.py:8)
constexpr int kRowF = kTok * kEmb;  // 460
constexpr float kSqrtKq = 3.16227766016838f;  // f32(np.sqrt(10)): the reference divides by it
constexpr float kRSqrtKq = 0.316227766016838f;  // RN(1 / kSqrtKq)

// x / sqrt(10): reciprocal product plus one fma residual correction (Markstein),
// which lands on the correctly rounded quotient -- 3 VALU ops instead of a
// full IEEE division sequence
__device__ __forceinline__ float div_sqrt_kq(float x) {
    const float q = x * kRSqrtKq;
    return fmaf(fmaf(-q, kSqrtKq, x), kRSqrtKq, q);
}

// workspace (floats)
constexpr int kWsWP = 0;                          // [23][20][4], zero beyond d_i
constexpr int kWsBP = kWsWP + kTok * kEmb * kPin;  // [23][20]
constexpr int kWsA = kWsBP + kTok * kEmb;          // [23][40][4]
constexpr int kWsC = kWsA + kTok * kQkv * kPin;    // [23][40]
constexpr int kWsW = kWsC + kTok * kQkv;           // [40][20]
constexpr int kWsAT = kWsW + kQkv * kEmb;          // [23][4][40]: A column-major (the forward's staged tables)
constexpr int kWsLen = kWsAT + kTok * kPin * kQkv;  // 11380

// backward partial row (floats)
constexpr int kGd = kQkv + kEmb;                    // 60 rows per token: g (40) then dctx (20)
constexpr int kPEF = 0;                             // [23][60][4]: E_i (rows 0-39), F_i (rows 40-59)
constexpr int kPef = kPEF + kTok * kGd * kPin;      // [23][60]: e_i, f_i
constexpr int kPartLen = kPef + kTok * kGd;         // 6900

// final gradient layout: [wq 10x20 | wk 10x20 | wv 20x20 | wp 23x20x4 | bp 23x20]
constexpr int kGP = kQkv * kEmb, kGB = kGP + kTok * kEmb * kPin;
constexpr int kGradLen = kGB + kTok * kEmb;  // 3100

__constant__ int c_dims[kTok] = {4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 2, 2, 1, 4, 1, 1, 1, 1, 1, 1, 2};
__constant__ int c_starts_fixed[kTok] = {0,  4,  8,  12, 16, 20, 24, 28, 32, 36, 40, 44,
                                         48, 50, 52, 53, 57, 58, 59, 60, 61, 62, 63};

struct ProjPtrs {  // the 23 Linear(d_i -> 20) modules' parameters (nn.Linear layout [20][d_i], [20])
    const float* w[kTok];
    const float* b[kTok];
};

// x slice of token i (zero beyond d_i)
__device__ __forceinline__ float4 xslice(const float* __restrict__ xr, int i, bool parity) {
    const int d = c_dims[i];
    const int s = parity ? 0 : c_starts_fixed[i];
    // four unconditional loads inside the slice (clamped index), zeros selected past d (no exec-masked
    // loads)
    const float v0 = xr[s], v1 = xr[s + min(1, d - 1)], v2 = xr[s + min(2, d - 1)], v3 = xr[s + min(3, d - 1)];
    return make_float4(v0, d > 1 ? v1 : 0.f, d > 2 ? v2 : 0.f, d > 3 ? v3 : 0.f);
}

typedef __attribute__((ext_vector_type(2))) float f32x2;

// o[r] = M[r] . xv + c[r] for the rows r of a [R][4] matrix (per-lane rows;
// M and c 16-byte aligned, R % 4 == 0)
template <int R>
__device__ __forceinline__ void affine4(const float* __restrict__ M, const float* __restrict__ c, float4 xv,
                                        float o[R]) {
    const float4* m4 = reinterpret_cast<const float4*>(M);
    const float4* c4 = reinterpret_cast<const float4*>(c);
#pragma unroll
    for (int r4 = 0; r4 < R / 4; r4++) {
        const float4 cv = c4[r4];
        const float cc[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float4 w = m4[4 * r4 + u];
            float acc = w.x * xv.x;
            acc = fmaf(w.y, xv.y, acc);
            acc = fmaf(w.z, xv.z, acc);
            acc = fmaf(w.w, xv.w, acc);
            o[4 * r4 + u] = acc + cc[u];
        }
    }
}

// affine4 over a column-major (transposed) [4][R] matrix: rows r, r + 1 of each column are adjacent, so
// every step is one packed FMA on aligned pairs (the [R][4] form needs two moves per packed FMA to pair
// up rows).  Same per-element order as affine4 (mul, three fmas, + c): bit-identical results.
template <int R>
__device__ __forceinline__ void affine4t(const float* __restrict__ MT, const float* __restrict__ c, float4 xv,
                                         float o[R]) {
    const f32x2 x0 = {xv.x, xv.x}, x1 = {xv.y, xv.y}, x2 = {xv.z, xv.z}, x3 = {xv.w, xv.w};
    const float4* m0 = reinterpret_cast<const float4*>(MT);
    const float4* m1 = reinterpret_cast<const float4*>(MT + R);
    const float4* m2 = reinterpret_cast<const float4*>(MT + 2 * R);
    const float4* m3 = reinterpret_cast<const float4*>(MT + 3 * R);
    const float4* c4 = reinterpret_cast<const float4*>(c);
#pragma unroll
    for (int r4 = 0; r4 < R / 4; r4++) {
        const float4 a = m0[r4], b = m1[r4], d = m2[r4], e = m3[r4], cv = c4[r4];
        f32x2 lo = f32x2{a.x, a.y} * x0, hi = f32x2{a.z, a.w} * x0;
        lo = __builtin_elementwise_fma(f32x2{b.x, b.y}, x1, lo);
        hi = __builtin_elementwise_fma(f32x2{b.z, b.w}, x1, hi);
        lo = __builtin_elementwise_fma(f32x2{d.x, d.y}, x2, lo);
        hi = __builtin_elementwise_fma(f32x2{d.z, d.w}, x2, hi);
        lo = __builtin_elementwise_fma(f32x2{e.x, e.y}, x3, lo);
        hi = __builtin_elementwise_fma(f32x2{e.z, e.w}, x3, hi);
        lo = lo + f32x2{cv.x, cv.y};
        hi = hi + f32x2{cv.z, cv.w};
        o[4 * r4] = lo.x;
        o[4 * r4 + 1] = lo.y;
        o[4 * r4 + 2] = hi.x;
        o[4 * r4 + 3] = hi.y;
    }
}

// token embedding t_i = Wp_i x_i + b_i (Projection; quirk Q1 when parity)
__device__ __forceinline__ void embed(const float* __restrict__ ws, float4 xv, int i, float t[kEmb]) {
    affine4<kEmb>(ws + kWsWP + i * kEmb * kPin, ws + kWsBP + i * kEmb, xv, t);
}

// [q|k|v] of token i from its input slice (folded maps)
__device__ __forceinline__ void qkv_of(const float* __restrict__ ws, float4 xv, int i, float o[kQkv]) {
    affine4<kQkv>(ws + kWsA + i * kQkv * kPin, ws + kWsC + i * kQkv, xv, o);
}

// A sample's 32 lanes are half of one wavefront, and a wavefront's LDS
// accesses execute in program order, so hand-offs between the lanes of one
// sample need only a compiler-level ordering point, not a workgroup barrier.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a . b over N (even) values, b in LDS: two interleaved accumulators (even / odd k) on packed FMAs
// (v_pk_fma_f32: two FMAs per instruction, half the dependent chain), summed at the end.  The
// summation order is not the reference's (torch's CPU einsum order is not reproducible anyway; the
// front-end is held to fp64 / torch within 1e-5).
template <int N>
__device__ __forceinline__ float dot4(const float* a, const float* __restrict__ b_lds) {  // N % 2 == 0
    f32x2 acc = {0.f, 0.f};
    if constexpr (N % 4 == 0) {
        const float4* b4 = reinterpret_cast<const float4*>(b_lds);
#pragma unroll
        for (int k = 0; k < N / 4; k++) {
            const float4 v = b4[k];
            acc = __builtin_elementwise_fma(f32x2{a[4 * k], a[4 * k + 1]}, f32x2{v.x, v.y}, acc);
            acc = __builtin_elementwise_fma(f32x2{a[4 * k + 2], a[4 * k + 3]}, f32x2{v.z, v.w}, acc);
        }
    } else {
        const float2* b2 = reinterpret_cast<const float2*>(b_lds);
#pragma unroll
        for (int k = 0; k < N / 2; k++) {
            const float2 v = b2[k];
            acc = __builtin_elementwise_fma(f32x2{a[2 * k], a[2 * k + 1]}, f32x2{v.x, v.y}, acc);
        }
    }
    return acc.x + acc.y;
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
// prep: workspace from the parameters (one workgroup per token)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_front_prep(ProjPtrs P, const float* __restrict__ wq,
                                                    const float* __restrict__ wk, const float* __restrict__ wv,
                                                    float* __restrict__ ws) {
    __shared__ float W[kQkv][kEmb];
    __shared__ float Wp[kEmb][kPin];
    __shared__ float bp[kEmb];
    const int i = blockIdx.x;
    const int d = c_dims[i];
    const float* wi = P.w[0];
    const float* bi = P.b[0];
#pragma unroll
    for (int k = 1; k < kTok; k++)  // uniform select (no dynamic indexing of the argument struct)
        if (k == i) {
            wi = P.w[k];
            bi = P.b[k];
        }
    for (int e = threadIdx.x; e < kQkv * kEmb; e += blockDim.x) {
        const int r = e / kEmb;
        const float w = r < kKq ? wq[e] : (r < 2 * kKq ? wk[e - kKq * kEmb] : wv[e - 2 * kKq * kEmb]);
        W[r][e % kEmb] = w;
        if (i == 0) ws[kWsW + e] = w;
    }
    for (int e = threadIdx.x; e < kEmb * kPin; e += blockDim.x) {
        const int c = e / kPin, k = e % kPin;
        const float w = k < d ? wi[c * d + k] : 0.f;
        Wp[c][k] = w;
        ws[kWsWP + i * kEmb * kPin + e] = w;
    }
    for (int c = threadIdx.x; c < kEmb; c += blockDim.x) {
        bp[c] = bi[c];
        ws[kWsBP + i * kEmb + c] = bi[c];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kQkv * kPin; e += blockDim.x) {  // A_i = Wqkv Wp_i
        const int r = e / kPin, k = e % kPin;
        float acc = 0.f;
        for (int c = 0; c < kEmb; c++) acc = fmaf(W[r][c], Wp[c][k], acc);
        ws[kWsA + i * kQkv * kPin + e] = acc;
        ws[kWsAT + i * kQkv * kPin + k * kQkv + r] = acc;
    }
    for (int r = threadIdx.x; r < kQkv; r += blockDim.x) {  // c_i = Wqkv b_i
        float acc = 0.f;
        for (int c = 0; c < kEmb; c++) acc = fmaf(W[r][c], bp[c], acc);
        ws[kWsC + i * kQkv + r] = acc;
    }
}

// ---------------------------------------------------------------------------
// forward (persistent: the per-token tables are staged in LDS once per workgroup)
// ---------------------------------------------------------------------------
constexpr int kFwdRows = 8;  // samples per iteration of a 256-thread workgroup
constexpr int kTabF = kQkv * kPin + kQkv + kEmb * kPin + kEmb;  // 300 floats per token: A^T | c | Wp^T | bp
// (A and Wp column-major, [4][40] and [4][20], for affine4t; 300 dwords = 75 16-byte quads, odd: a wave's
// per-token 16-byte reads are bank-conflict free)

// all of a thread's table loads are issued before its LDS writes (one L2
// round trip per workgroup instead of one per element); 256 threads
__device__ __forceinline__ void stage_tables(const float* __restrict__ ws, float* tab) {
    constexpr int kN = kTok * kTabF, kPer = (kN + 255) / 256;
    float v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int e = threadIdx.x + 256 * u;
        const int i = e / kTabF, f = e % kTabF;
        int src;
        if (f < kQkv * kPin) src = kWsAT + i * kQkv * kPin + f;  // A^T
        else if (f < kQkv * kPin + kQkv) src = kWsC + i * kQkv + f - kQkv * kPin;
        else if (f < kQkv * kPin + kQkv + kEmb * kPin) {
            const int g = f - kQkv * (kPin + 1);  // Wp^T[k][c] = Wp[c][k]
            src = kWsWP + i * kEmb * kPin + (g % kEmb) * kPin + g / kEmb;
        } else src = kWsBP + i * kEmb + f - kQkv * (kPin + 1) - kEmb * kPin;
        v[u] = e < kN ? ws[src] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const int e = threadIdx.x + 256 * u;
        if (e < kN) tab[e] = v[u];
    }
}

__global__ __launch_bounds__(256) void k_front_fwd(const float* __restrict__ ws, const float* __restrict__ x,
                                                   int ldx, int B, int parity, float* __restrict__ h) {
    __shared__ __attribute__((aligned(16))) float tab[kTok * kTabF];
    __shared__ __attribute__((aligned(16))) float Ks[kFwdRows][kTok][kKq];
    __shared__ __attribute__((aligned(16))) float Vs[kFwdRows][kTok][kEmb];
    stage_tables(ws, tab);
    __syncthreads();
    const int g = threadIdx.x >> 5;  // sample slot in the workgroup
    const int i = threadIdx.x & 31;  // token
    const float* ti = tab + (i < kTok ? i : 0) * kTabF;
    const int groups = (B + kFwdRows - 1) / kFwdRows;
    for (int grp = blockIdx.x; grp < groups; grp += gridDim.x) {
        const int row = grp * kFwdRows + g;
        const bool act = (i < kTok) && (row < B);
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (act) xv = xslice(x + (size_t)row * ldx, i, parity != 0);
        wave_sync();  // previous iteration's K, V readers (this wavefront) are done
        float q[kKq];
        if (act) {
            float o[kQkv];
            affine4t<kQkv>(ti, ti + kQkv * kPin, xv, o);
#pragma unroll
            for (int a = 0; a < kKq; a++) q[a] = o[a];
            // 8- and 16-byte LDS writes (rows of 40 and 80 bytes) instead of 30 4-byte ones
#pragma unroll
            for (int a = 0; a < kKq; a += 2)
                *reinterpret_cast<float2*>(&Ks[g][i][a]) = make_float2(o[kKq + a], o[kKq + a + 1]);
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(&Vs[g][i][c]) =
                    make_float4(o[2 * kKq + c], o[2 * kKq + c + 1], o[2 * kKq + c + 2], o[2 * kKq + c + 3]);
        }
        wave_sync();
        if (act) {
            float s[kTok];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                s[j] = div_sqrt_kq(dot4<kKq>(q, Ks[g][j]));
                mx = fmaxf(mx, s[j]);
            }
            float sum0 = 0.f, sum1 = 0.f;  // even / odd j: two short chains (the backward recomputes the same way)
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                s[j] = expf(s[j] - mx);
                if (j & 1) sum1 += s[j];
                else sum0 += s[j];
            }
            const float sum = sum0 + sum1;
            float out[kEmb];
#pragma unroll
            for (int c = 0; c < kEmb; c++) out[c] = 0.f;
            const float inv = 1.f / sum;  // torch's softmax scales by the reciprocal of the sum
#pragma unroll
            for (int j = 0; j < kTok; j++) axpy4<kEmb>(out, s[j] * inv, Vs[g][j]);
            float t[kEmb];
            affine4t<kEmb>(ti + kQkv * (kPin + 1), ti + kQkv * (kPin + 1) + kEmb * kPin, xv, t);
            float* o = h + (size_t)row * kRowF + i * kEmb;
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(o + c) =
                    make_float4(t[c] + out[c], t[c + 1] + out[c + 1], t[c + 2] + out[c + 2], t[c + 3] + out[c + 3]);
        }
    }
}

// ---------------------------------------------------------------------------
// forward, two query rows per lane (k_front_fwd2)
// ---------------------------------------------------------------------------
// k_front_fwd is bound by LDS data return, not by the VALU: every lane reads
// all 23 k_j / v_j rows (690 floats) for its one query row, and a broadcast
// read costs the same return bandwidth as a gather.  Here 16 lanes own a
// sample and lane l owns query rows l and l + 12 (lane 11: row 11 only), so
// each k_j / v_j read feeds two rows: per sample 12 x 690 instead of
// 23 x 690 floats of K/V reads (the per-token table reads, 300 floats per
// token, are unchanged).  Same arithmetic per row as k_front_fwd (dot4 /
// axpy4 order, even/odd softmax sums), so h is bit-identical to it.
constexpr int kF2Lanes = 16;                // lanes per sample
constexpr int kF2Half = 12;                 // lane l owns rows l and l + 12
constexpr int kF2Rows = 256 / kF2Lanes;     // 16 samples per workgroup iteration

__global__ __launch_bounds__(256, 2) void k_front_fwd2(const float* __restrict__ ws, const float* __restrict__ x,
                                                       int ldx, int B, int parity, float* __restrict__ h) {
    __shared__ __attribute__((aligned(16))) float tab[kTok * kTabF];
    __shared__ __attribute__((aligned(16))) float Ks[kF2Rows][kTok][kKq];
    __shared__ __attribute__((aligned(16))) float Vs[kF2Rows][kTok][kEmb];
    stage_tables(ws, tab);
    __syncthreads();
    const int g = threadIdx.x >> 4;  // sample slot in the workgroup
    const int l = threadIdx.x & 15;
    const bool own0 = l < kF2Half, own1 = l + kF2Half < kTok;
    const int i0 = own0 ? l : 0, i1 = own1 ? l + kF2Half : 0;  // rows (clamped: lane 11's second row is a
                                                              // discarded copy of row 0)
    const float* ta = tab + i0 * kTabF;
    const float* tb = tab + i1 * kTabF;
    const int groups = (B + kF2Rows - 1) / kF2Rows;
    for (int grp = blockIdx.x; grp < groups; grp += gridDim.x) {
        const int row = grp * kF2Rows + g;
        const bool act = own0 && (row < B);
        float4 xa = make_float4(0.f, 0.f, 0.f, 0.f), xb = xa;
        if (act) {
            const float* xr = x + (size_t)row * ldx;
            xa = xslice(xr, i0, parity != 0);
            xb = xslice(xr, i1, parity != 0);
        }
        wave_sync();  // previous iteration's K, V readers (this wavefront) are done
        float qa[kKq], qb[kKq];
        if (act) {
            float o[kQkv];
            affine4t<kQkv>(ta, ta + kQkv * kPin, xa, o);
#pragma unroll
            for (int a = 0; a < kKq; a++) qa[a] = o[a];
#pragma unroll
            for (int a = 0; a < kKq; a += 2)
                *reinterpret_cast<float2*>(&Ks[g][i0][a]) = make_float2(o[kKq + a], o[kKq + a + 1]);
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(&Vs[g][i0][c]) =
                    make_float4(o[2 * kKq + c], o[2 * kKq + c + 1], o[2 * kKq + c + 2], o[2 * kKq + c + 3]);
            affine4t<kQkv>(tb, tb + kQkv * kPin, xb, o);
#pragma unroll
            for (int a = 0; a < kKq; a++) qb[a] = o[a];
            if (own1) {
#pragma unroll
                for (int a = 0; a < kKq; a += 2)
                    *reinterpret_cast<float2*>(&Ks[g][i1][a]) = make_float2(o[kKq + a], o[kKq + a + 1]);
#pragma unroll
                for (int c = 0; c < kEmb; c += 4)
                    *reinterpret_cast<float4*>(&Vs[g][i1][c]) =
                        make_float4(o[2 * kKq + c], o[2 * kKq + c + 1], o[2 * kKq + c + 2], o[2 * kKq + c + 3]);
            }
        }
        wave_sync();
        if (act) {
            float sa[kTok], sb[kTok];
            float mxa = -INFINITY, mxb = -INFINITY;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                sa[j] = div_sqrt_kq(dot4<kKq>(qa, Ks[g][j]));
                sb[j] = div_sqrt_kq(dot4<kKq>(qb, Ks[g][j]));
                mxa = fmaxf(mxa, sa[j]);
                mxb = fmaxf(mxb, sb[j]);
            }
            float suma0 = 0.f, suma1 = 0.f, sumb0 = 0.f, sumb1 = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                sa[j] = expf(sa[j] - mxa);
                sb[j] = expf(sb[j] - mxb);
                if (j & 1) {
                    suma1 += sa[j];
                    sumb1 += sb[j];
                } else {
                    suma0 += sa[j];
                    sumb0 += sb[j];
                }
            }
            const float inva = 1.f / (suma0 + suma1), invb = 1.f / (sumb0 + sumb1);
            float oa[kEmb], ob[kEmb];
#pragma unroll
            for (int c = 0; c < kEmb; c++) oa[c] = ob[c] = 0.f;
            // partly unrolled: fully unrolled, the compiler hoists all 23 v_j reads (460 registers) and spills;
            // sa / sb are then indexed by the wave-uniform j (register-relative moves, no scratch)
#pragma unroll 4
            for (int j = 0; j < kTok; j++) {  // one v_j read, two rows
                const float4* v4 = reinterpret_cast<const float4*>(Vs[g][j]);
                const float pa = sa[j] * inva, pb = sb[j] * invb;
#pragma unroll
                for (int k = 0; k < kEmb / 4; k++) {
                    const float4 v = v4[k];
                    oa[4 * k] = fmaf(pa, v.x, oa[4 * k]);
                    oa[4 * k + 1] = fmaf(pa, v.y, oa[4 * k + 1]);
                    oa[4 * k + 2] = fmaf(pa, v.z, oa[4 * k + 2]);
                    oa[4 * k + 3] = fmaf(pa, v.w, oa[4 * k + 3]);
                    ob[4 * k] = fmaf(pb, v.x, ob[4 * k]);
                    ob[4 * k + 1] = fmaf(pb, v.y, ob[4 * k + 1]);
                    ob[4 * k + 2] = fmaf(pb, v.z, ob[4 * k + 2]);
                    ob[4 * k + 3] = fmaf(pb, v.w, ob[4 * k + 3]);
                }
            }
            float t[kEmb];
            float* hr = h + (size_t)row * kRowF;
            affine4t<kEmb>(ta + kQkv * (kPin + 1), ta + kQkv * (kPin + 1) + kEmb * kPin, xa, t);
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(hr + i0 * kEmb + c) =
                    make_float4(t[c] + oa[c], t[c + 1] + oa[c + 1], t[c + 2] + oa[c + 2], t[c + 3] + oa[c + 3]);
            if (own1) {
                affine4t<kEmb>(tb + kQkv * (kPin + 1), tb + kQkv * (kPin + 1) + kEmb * kPin, xb, t);
#pragma unroll
                for (int c = 0; c < kEmb; c += 4)
                    *reinterpret_cast<float4*>(hr + i1 * kEmb + c) =
                        make_float4(t[c] + ob[c], t[c + 1] + ob[c + 1], t[c + 2] + ob[c + 2], t[c + 3] + ob[c + 3]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// backward (persistent, in-kernel weight-gradient reduction)
// ---------------------------------------------------------------------------
// LDS per sample (floats): attention phase {K 23x10 | Q 23x10 | V 23x20 |
// P 23x23 | dS 23x23}; after a barrier the same words hold the reduction
// operands {G = [dq|dk|dv] 23x40 | (unused 23x20) | dctx 23x20 | X 23x4}; the V rows
// carry dctx in phase 3.  63 KB per workgroup: two workgroups (8 waves) per CU.
constexpr int kBwdRows = 8;
constexpr int kBwdThreads = 256;
constexpr int kOffK = 0, kOffQ = 230, kOffV = 460, kOffP = 920, kOffS = 1449;  // attention phase
constexpr int kOffG = 0, kOffD = 1380, kOffX = 1840;  // reduction phase
constexpr int kSampleF = 1980;  // floats per sample (>= 1978 and >= 1932; multiple of 4)
// E/F work units: (token, kEFR consecutive rows of [g|dctx]); kEFR = FRONT_EF_ROWS (4: 345 units, two per
// thread for 89 of 256 threads; 2: 690 units, three per thread for 178 -- a shorter critical thread)
constexpr int kEFR = FRONT_EF_ROWS;
static_assert(kEFR == 2 || kEFR == 4, "FRONT_EF_ROWS is 2 or 4");
constexpr int kEFPerTok = kGd / kEFR;                                    // units per token
constexpr int kEFUnits = kTok * kEFPerTok;                               // 345 / 690
constexpr int kEFU = (kEFUnits + kBwdThreads - 1) / kBwdThreads;         // units per thread (2 / 3)

// phase 4b of the backward: E/F (+= [g|dctx] x^T) and e/f (+= [g|dctx]) per token over the iteration's
// samples; thread t owns units t, t + 256, ... (token u / kEFPerTok, rows kEFR (u % kEFPerTok) ..), fixed
// order.  Accumulators held as aligned pairs: E rows (cols 0-1, 2-3) and e (row pairs), so every update is
// a packed FMA / add with the g value broadcast by op_sel (no pairing moves); per element the same fmaf /
// add order as the scalar form
struct EFAcc {
    f32x2 e[kEFU][kEFR][2];  // [unit][row a][column pair]
    f32x2 s[kEFU][kEFR / 2];  // [unit][row pair]
};

template <int kStride = kSampleF, int kG = kOffG, int kD = kOffD, int kX = kOffX>
__device__ __forceinline__ void ef_accumulate(const float* sm, int nrow, EFAcc& acc) {
#pragma unroll
    for (int u = 0; u < kEFU; u++) {
        const int unit = threadIdx.x + u * kBwdThreads;
        if (unit < kEFUnits) {
            const int tk = unit / kEFPerTok, r0 = kEFR * (unit % kEFPerTok);
            const int off = r0 < kQkv ? kG + tk * kQkv + r0 : kD + tk * kEmb + (r0 - kQkv);
#pragma unroll FRONT_EF_UNROLL
            for (int gg = 0; gg < nrow; gg++) {
                const float* sg = sm + gg * kStride;
                float gr[kEFR];
                if constexpr (kEFR == 4) {
                    const float4 gv = *reinterpret_cast<const float4*>(sg + off);
                    gr[0] = gv.x, gr[1] = gv.y, gr[2] = gv.z, gr[3] = gv.w;
                } else {
                    const float2 gv = *reinterpret_cast<const float2*>(sg + off);
                    gr[0] = gv.x, gr[1] = gv.y;
                }
                const float4 xq = *reinterpret_cast<const float4*>(sg + kX + tk * kPin);
                const f32x2 x01 = {xq.x, xq.y}, x23 = {xq.z, xq.w};
#pragma unroll
                for (int a = 0; a < kEFR; a++) {
                    const f32x2 ga = {gr[a], gr[a]};
                    acc.e[u][a][0] = __builtin_elementwise_fma(ga, x01, acc.e[u][a][0]);
                    acc.e[u][a][1] = __builtin_elementwise_fma(ga, x23, acc.e[u][a][1]);
                }
#pragma unroll
                for (int a = 0; a < kEFR / 2; a++) acc.s[u][a] += f32x2{gr[2 * a], gr[2 * a + 1]};
            }
        }
    }
}

__device__ __forceinline__ void ef_zero(EFAcc& acc) {
#pragma unroll
    for (int u = 0; u < kEFU; u++) {
#pragma unroll
        for (int a = 0; a < kEFR; a++) acc.e[u][a][0] = acc.e[u][a][1] = f32x2{0.f, 0.f};
#pragma unroll
        for (int a = 0; a < kEFR / 2; a++) acc.s[u][a] = f32x2{0.f, 0.f};
    }
}

__device__ __forceinline__ void ef_write(float* partial, const EFAcc& acc) {
    float* out = partial + (size_t)blockIdx.x * kPartLen;
#pragma unroll
    for (int u = 0; u < kEFU; u++) {
        const int unit = threadIdx.x + u * kBwdThreads;
        if (unit < kEFUnits) {
            const int tk = unit / kEFPerTok, r0 = kEFR * (unit % kEFPerTok);
#pragma unroll
            for (int a = 0; a < kEFR; a++) {
                *reinterpret_cast<float4*>(out + kPEF + (tk * kGd + r0 + a) * kPin) =
                    make_float4(acc.e[u][a][0].x, acc.e[u][a][0].y, acc.e[u][a][1].x, acc.e[u][a][1].y);
                out[kPef + tk * kGd + r0 + a] = (a & 1) ? acc.s[u][a / 2].y : acc.s[u][a / 2].x;
            }
        }
    }
}

__global__ __launch_bounds__(kBwdThreads, 2) void k_front_bwd(const float* __restrict__ ws,
                                                              const float* __restrict__ x, int ldx, int B,
                                                              int parity, const float* __restrict__ dh,
                                                              float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float sm[kBwdRows * kSampleF];
    const int g = threadIdx.x >> 5;
    const int i = threadIdx.x & 31;
    float* my = sm + g * kSampleF;
    // E/F/e/f: thread t owns units t, t + 256, ... (ef_accumulate)
    EFAcc ef;
    ef_zero(ef);
    const int iters = (B + kBwdRows - 1) / kBwdRows;
    for (int it = blockIdx.x; it < iters; it += gridDim.x) {
        const int row0 = it * kBwdRows;
        const int nrow = min(kBwdRows, B - row0);
        const int row = row0 + g;
        const bool act = (i < kTok) && (g < nrow);
        __syncthreads();  // previous iteration's reduction readers are done
        float dctx[kEmb];
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        const float* dhr = dh + (size_t)row * kRowF;
        if (act) {  // phase 1: q/k/v (folded maps), own dctx row
            xv = xslice(x + (size_t)row * ldx, i, parity != 0);
            float o[kQkv];
            qkv_of(ws, xv, i, o);
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
                *reinterpret_cast<float2*>(my + kOffQ + i * kKq + a) = make_float2(o[a], o[a + 1]);
                *reinterpret_cast<float2*>(my + kOffK + i * kKq + a) = make_float2(o[kKq + a], o[kKq + a + 1]);
            }
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(my + kOffV + i * kEmb + c) =
                    make_float4(o[2 * kKq + c], o[2 * kKq + c + 1], o[2 * kKq + c + 2], o[2 * kKq + c + 3]);
        }
        wave_sync();
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
                p[j] = div_sqrt_kq(dot4<kKq>(q, my + kOffK + j * kKq));
                mx = fmaxf(mx, p[j]);
            }
            float sum0 = 0.f, sum1 = 0.f;  // as the forward: even / odd j
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = expf(p[j] - mx);
                if (j & 1) sum1 += p[j];
                else sum0 += p[j];
            }
            const float sum = sum0 + sum1;
            float dp[kTok];
            float rs0 = 0.f, rs1 = 0.f;
            const float inv = 1.f / sum;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = p[j] * inv;
                dp[j] = dot4<kEmb>(dctx, my + kOffV + j * kEmb);  // dP_ij = dctx_i . v_j
                if (j & 1) rs1 = fmaf(dp[j], p[j], rs1);
                else rs0 = fmaf(dp[j], p[j], rs0);
            }
            const float rs = rs0 + rs1;
#pragma unroll
            for (int a = 0; a < kKq; a++) dq[a] = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                const float ds = div_sqrt_kq(p[j] * (dp[j] - rs));  // softmax backward, then / sqrt(10)
                my[kOffP + i * kTok + j] = p[j];
                my[kOffS + i * kTok + j] = ds;
                axpy4<kKq>(dq, ds, my + kOffK + j * kKq);
            }
            // v is dead once this wave's dP loop is done (a sample's 32 lanes are
            // one wavefront, so its LDS accesses stay in program order): the V
            // rows now carry dctx for phase 3
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(my + kOffV + i * kEmb + c) =
                    make_float4(dctx[c], dctx[c + 1], dctx[c + 2], dctx[c + 3]);
        }
        wave_sync();
        float dk[kKq], dv[kEmb];
        if (act) {  // phase 3: dv_i = sum_j P_ji dctx_j, dk_i = sum_j dS_ji q_j
#pragma unroll
            for (int c = 0; c < kEmb; c++) dv[c] = 0.f;
#pragma unroll
            for (int a = 0; a < kKq; a++) dk[a] = 0.f;
#pragma unroll FRONT_P3_UNROLL
            for (int j = 0; j < kTok; j++) {
                const float pj = my[kOffP + j * kTok + i];
                const float sj = my[kOffS + j * kTok + i];
                const float4* cj = reinterpret_cast<const float4*>(my + kOffV + j * kEmb);
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
        }
        wave_sync();  // attention-phase words of this sample are dead: reuse them for the reduction operands
        if (act) {
            float* G = my + kOffG + i * kQkv;
#pragma unroll
            for (int a = 0; a < kKq; a += 2) {
                *reinterpret_cast<float2*>(G + a) = make_float2(dq[a], dq[a + 1]);
                *reinterpret_cast<float2*>(G + kKq + a) = make_float2(dk[a], dk[a + 1]);
            }
#pragma unroll
            for (int c = 0; c < kEmb; c += 4) {
                *reinterpret_cast<float4*>(G + 2 * kKq + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
                *reinterpret_cast<float4*>(my + kOffD + i * kEmb + c) =
                    make_float4(dctx[c], dctx[c + 1], dctx[c + 2], dctx[c + 3]);
            }
            *reinterpret_cast<float4*>(my + kOffX + i * kPin) = xv;
        }
        __syncthreads();
        ef_accumulate(sm, nrow, ef);
    }
    ef_write(partial, ef);
}

// ---------------------------------------------------------------------------
// backward on the MFMA (k_front_bwd_mfma): the per-sample attention products
// run as 16x16x16 bf16 MFMA tiles with the exact three-way split (six products
// per fp32 product, as csrc/x3mlp.hip), tokens padded 23 -> 32, d_k 10 -> 16,
// d_v 20 -> 32.  One wavefront per sample (two samples per wave per
// iteration).  Accumulator tiles feed the next products directly: a C tile
// (lane l holds rows 4 (l >> 4) + g, column l & 15) is the B operand of a
// 16x16x16 MFMA whose k runs over its rows, and its transpose is an A
// operand -- so
//   S   = Q K^T          (A: Q rows, B: K rows; computed in-lane)
//   dP  = dctx V^T       (A: dctx rows from dh, B: V rows in-lane)
//   dV^T = dctx^T P      (B = the P tiles themselves)
//   dK^T = Q^T dS        (B = the dS tiles)
//   dQ  = dS K           (A = dS re-read through a 4-KiB LDS transpose)
// and every q/k/v operand value is formed in the lane that needs it from the
// folded maps (4 FMAs each).  Softmax and dS = P (dP - rowsum(P dP)) / sqrt(10)
// act on the C tiles (row reductions across 16 lanes).  The per-token
// gradients g = [dq | dk | dv], dctx and x go to the same LDS rows as in
// k_front_bwd, whose E/F accumulation phase follows unchanged.
//
// Measured (tools/bench_front.py, 419,430 rows; tools/pmc_front.sh): 2.70 ms
// against k_front_bwd's 1.85 ms, so it is not the default.  It executes 2,196
// VALU instructions per sample against the VALU kernel's 1,213: the exact
// three-way split of every operand value (~700 per sample) and the 32 x 32
// padding of the 23 x 23 attention (softmax and dS on 1,024 entries instead
// of 529) cost more VALU than the 168 MFMAs per sample save.
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// 4 fp32 -> three bf16 planes (x = hi + mid + lo exactly), hardware RNE conversions
__device__ __forceinline__ void split4(const float* v, s16x4 (&p)[3]) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
    typedef __attribute__((ext_vector_type(2))) float f2;
    uint32_t h[2], m[2], l[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const float x0 = v[2 * k], x1 = v[2 * k + 1];
        h[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){x0, x1}, bf2));
        const float r0 = x0 - __uint_as_float(h[k] << 16), r1 = x1 - __uint_as_float(h[k] & 0xFFFF0000u);
        m[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){r0, r1}, bf2));
        const float s0 = r0 - __uint_as_float(m[k] << 16), s1 = r1 - __uint_as_float(m[k] & 0xFFFF0000u);
        l[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){s0, s1}, bf2));
    }
    p[0] = __builtin_bit_cast(s16x4, make_uint2(h[0], h[1]));
    p[1] = __builtin_bit_cast(s16x4, make_uint2(m[0], m[1]));
    p[2] = __builtin_bit_cast(s16x4, make_uint2(l[0], l[1]));
}

// acc += A B over one k-block of 16 (fp32-class: the six partial products >= 2^-16 |ab|, small terms first)
__device__ __forceinline__ f32x4_t mma16x3(const s16x4 (&a)[3], const s16x4 (&b)[3], f32x4_t acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[0], b[0], acc, 0, 0, 0);
    return acc;
}

constexpr int kMmaPitch = 32;  // dS transpose buffer row pitch (floats)
constexpr int kMG = 0, kMD = kTok * kQkv, kMX = kMD + kTok * kEmb;  // reduction operands per sample
constexpr int kMmaSample = kMX + kTok * kPin;                       // 1,472 floats (>= the 32 x 32 transpose)
static_assert(kMmaSample >= 32 * kMmaPitch, "the dS transpose lives in the sample's region");

__global__ __launch_bounds__(kBwdThreads, 2) void k_front_bwd_mfma(const float* __restrict__ ws,
                                                                   const float* __restrict__ x, int ldx, int B,
                                                                   int parity, const float* __restrict__ dh,
                                                                   float* __restrict__ partial) {
    // per sample: the reduction operands G [23][40] | dctx [23][20] | x [23][4] (the first 1,024 floats
    // serve as the sample's dS transpose buffer before G is written); the folded maps A | c staged once
    __shared__ __attribute__((aligned(16))) float sm[kBwdRows * kMmaSample];
    __shared__ __attribute__((aligned(16))) float tA[kTok * kQkv * kPin];
    __shared__ __attribute__((aligned(16))) float tC[kTok * kQkv];
    {
        constexpr int kN = kTok * kQkv * kPin + kTok * kQkv, kPer = (kN + kBwdThreads - 1) / kBwdThreads;
        float v[kPer];
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            const int e = threadIdx.x + kBwdThreads * u;
            v[u] = e < kN ? ws[e < kTok * kQkv * kPin ? kWsA + e : kWsC + e - kTok * kQkv * kPin] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            const int e = threadIdx.x + kBwdThreads * u;
            if (e < kTok * kQkv * kPin) tA[e] = v[u];
            else if (e < kN) tC[e - kTok * kQkv * kPin] = v[u];
        }
    }
    const int wave = threadIdx.x >> 6;
    EFAcc ef;
    ef_zero(ef);
    const float* const fA = tA;  // folded maps [23][40][4] (LDS)
    const float* const fC = tC;  // [23][40]
    // output r (0-9 q, 10-19 k, 20-39 v) of token t for input slice xv; 0 for padding tokens
    auto qkv = [&](int t, int r, float4 xv) -> float {
        if (t >= kTok) return 0.f;
        const float4 w = *reinterpret_cast<const float4*>(fA + (t * kQkv + r) * kPin);
        float acc = w.x * xv.x;
        acc = fmaf(w.y, xv.y, acc);
        acc = fmaf(w.z, xv.z, acc);
        acc = fmaf(w.w, xv.w, acc);
        return acc + fC[t * kQkv + r];
    };
    const int iters = (B + kBwdRows - 1) / kBwdRows;
    for (int it = blockIdx.x; it < iters; it += gridDim.x) {
        const int row0 = it * kBwdRows;
        const int nrow = min(kBwdRows, B - row0);
        __syncthreads();  // previous iteration's reduction readers are done
#pragma unroll 1
        for (int half = 0; half < 2; half++) {
            const int slot = 2 * wave + half;  // this wave's sample of the iteration
            if (slot >= nrow) break;           // wave-uniform
            // lane indices recomputed per sample behind an opaque copy: otherwise the compiler hoists every
            // lane-dependent table address out of the loop and spills them
            int lane = threadIdx.x & 63;
            asm volatile("" : "+v"(lane));
            const int c16 = lane & 15, q4 = lane >> 4;
            const int row = row0 + slot;
            const float* xr = x + (size_t)row * ldx;
            const float* dhr = dh + (size_t)row * kRowF;
            float* my = sm + slot * kMmaSample;
            float* const tbuf = my;  // dS transpose (dead before G is written: one wave, LDS in program order)
            // the 23 token input slices -> the sample's X rows (also the reduction's operand), then every
            // q/k/v value reads its slice from LDS
            const float* const X = my + kMX;
            if (lane < kTok) *reinterpret_cast<float4*>(my + kMX + lane * kPin) = xslice(xr, lane, parity != 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            auto xk = [&](int tok) {
                return tok < kTok ? *reinterpret_cast<const float4*>(X + tok * kPin) : make_float4(0.f, 0.f, 0.f, 0.f);
            };
            float4 xrow[2] = {xk(c16), xk(c16 + 16)};
            // ---- S = Q K^T (d_k 10 -> one k-block of 16) ----
            s16x4 aq[2][3], bk[2][3];
#pragma unroll
            for (int t = 0; t < 2; t++) {
                float v[4], w[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int k = 4 * q4 + e;
                    v[e] = k < kKq ? qkv(c16 + 16 * t, k, xrow[t]) : 0.f;
                    w[e] = k < kKq ? qkv(c16 + 16 * t, kKq + k, xrow[t]) : 0.f;
                }
                split4(v, aq[t]);
                split4(w, bk[t]);
            }
            f32x4_t P[2][2];
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < 2; tj++) P[ti][tj] = mma16x3(aq[ti], bk[tj], f32x4_t{0.f, 0.f, 0.f, 0.f});
            __builtin_amdgcn_sched_barrier(0);  // (register pressure: no hoisting across sections)
            // ---- dP = dctx V^T (d_v 20 -> two k-blocks); dS later overwrites it in place ----
            f32x4_t dP[2][2];
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < 2; tj++) dP[ti][tj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kb = 0; kb < 2; kb++) {
                const int d0 = 16 * kb + 4 * q4;  // this lane's 4 d's
                s16x4 ad[2][3], bv[2][3];
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    const int tok = c16 + 16 * t;
                    float v[4] = {0.f, 0.f, 0.f, 0.f}, w[4];
                    if (tok < kTok && d0 < kEmb) {
                        const float4 d4 = *reinterpret_cast<const float4*>(dhr + tok * kEmb + d0);
                        v[0] = d4.x; v[1] = d4.y; v[2] = d4.z; v[3] = d4.w;
                    }
#pragma unroll
                    for (int e = 0; e < 4; e++) w[e] = d0 + e < kEmb ? qkv(tok, 2 * kKq + d0 + e, xrow[t]) : 0.f;
                    split4(v, ad[t]);
                    split4(w, bv[t]);
                }
#pragma unroll
                for (int ti = 0; ti < 2; ti++)
#pragma unroll
                    for (int tj = 0; tj < 2; tj++) dP[ti][tj] = mma16x3(ad[ti], bv[tj], dP[ti][tj]);
            }
            __builtin_amdgcn_sched_barrier(0);  // (register pressure: no hoisting across sections)
            // ---- softmax rows (the reference's order: / sqrt(10), exp(x - max), * (1 / sum)) and dS ----
#pragma unroll
            for (int ti = 0; ti < 2; ti++) {
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const bool rowok = 16 * ti + 4 * q4 + g < kTok;
                    float s[2];
                    float mx = -INFINITY;
#pragma unroll
                    for (int tj = 0; tj < 2; tj++) {
                        s[tj] = (16 * tj + c16 < kTok) ? div_sqrt_kq(P[ti][tj][g]) : -INFINITY;
                        mx = fmaxf(mx, s[tj]);
                    }
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 16));
                    float sum = 0.f;
#pragma unroll
                    for (int tj = 0; tj < 2; tj++) {
                        s[tj] = (16 * tj + c16 < kTok) ? expf(s[tj] - mx) : 0.f;
                        sum += s[tj];
                    }
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 16);
                    const float inv = 1.f / sum;
                    float rs = 0.f;
#pragma unroll
                    for (int tj = 0; tj < 2; tj++) {
                        const float p = rowok ? s[tj] * inv : 0.f;
                        P[ti][tj][g] = p;
                        rs = fmaf(dP[ti][tj][g], p, rs);
                    }
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) rs += __shfl_xor(rs, o, 16);
#pragma unroll
                    for (int tj = 0; tj < 2; tj++)
                        dP[ti][tj][g] = div_sqrt_kq(P[ti][tj][g] * (dP[ti][tj][g] - rs));  // = dS
                }
            }
            f32x4_t (&dS)[2][2] = dP;
            __builtin_amdgcn_sched_barrier(0);
            {
                {
                }
            }
            // ---- dS through LDS (row-major [i][j]) for dQ's A operand ----
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < 2; tj++)
#pragma unroll
                    for (int g = 0; g < 4; g++) tbuf[(16 * ti + 4 * q4 + g) * kMmaPitch + 16 * tj + c16] = dS[ti][tj][g];
            __builtin_amdgcn_sched_barrier(0);  // (register pressure: no hoisting across sections)
            // ---- dV^T = dctx^T P  (rows d, columns j; k = i) ----
            f32x4_t dVt[2][2];
#pragma unroll
            for (int td = 0; td < 2; td++)
#pragma unroll
                for (int tj = 0; tj < 2; tj++) dVt[td][tj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            // ---- dK^T = Q^T dS  (rows k, columns j; k-dim = i) ----
            f32x4_t dKt[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ib = 0; ib < 2; ib++) {
                s16x4 bp[2][3], bs[2][3];
#pragma unroll
                for (int tj = 0; tj < 2; tj++) {
                    const float pv[4] = {P[ib][tj][0], P[ib][tj][1], P[ib][tj][2], P[ib][tj][3]};
                    const float sv[4] = {dS[ib][tj][0], dS[ib][tj][1], dS[ib][tj][2], dS[ib][tj][3]};
                    split4(pv, bp[tj]);
                    split4(sv, bs[tj]);
                }
#pragma unroll
                for (int td = 0; td < 2; td++) {
                    const int d = 16 * td + c16;
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        const int i = 16 * ib + 4 * q4 + e;
                        v[e] = (i < kTok && d < kEmb) ? dhr[i * kEmb + d] : 0.f;
                    }
                    s16x4 a[3];
                    split4(v, a);
#pragma unroll
                    for (int tj = 0; tj < 2; tj++) dVt[td][tj] = mma16x3(a, bp[tj], dVt[td][tj]);
                }
                {
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        v[e] = c16 < kKq ? qkv(16 * ib + 4 * q4 + e, c16, xk(16 * ib + 4 * q4 + e)) : 0.f;
                    s16x4 a[3];
                    split4(v, a);
#pragma unroll
                    for (int tj = 0; tj < 2; tj++) dKt[tj] = mma16x3(a, bs[tj], dKt[tj]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // (register pressure: no hoisting across sections)
            // ---- dQ = dS K  (rows i, columns k; k-dim = j) ----
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            f32x4_t dQ[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int jb = 0; jb < 2; jb++) {
                float w[4];
#pragma unroll
                for (int e = 0; e < 4; e++)
                    w[e] = c16 < kKq ? qkv(16 * jb + 4 * q4 + e, kKq + c16, xk(16 * jb + 4 * q4 + e)) : 0.f;
                s16x4 b[3];
                split4(w, b);
#pragma unroll
                for (int ti = 0; ti < 2; ti++) {
                    const float4 r4 = *reinterpret_cast<const float4*>(tbuf + (16 * ti + c16) * kMmaPitch + 16 * jb +
                                                                       4 * q4);
                    const float v[4] = {r4.x, r4.y, r4.z, r4.w};
                    s16x4 a[3];
                    split4(v, a);
                    dQ[ti] = mma16x3(a, b, dQ[ti]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // (register pressure: no hoisting across sections)
            // ---- the reduction operands of this sample: G = [dq | dk | dv], dctx, x ----
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int i = 16 * ti + 4 * q4 + g;
                    if (i < kTok && c16 < kKq) my[kMG + i * kQkv + c16] = dQ[ti][g];
                }
#pragma unroll
            for (int tj = 0; tj < 2; tj++) {
                const int j = 16 * tj + c16;
                if (j < kTok) {
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        const int k = 4 * q4 + g;
                        if (k < kKq) my[kMG + j * kQkv + kKq + k] = dKt[tj][g];
                    }
#pragma unroll
                    for (int td = 0; td < 2; td++) {
                        const int d0 = 16 * td + 4 * q4;
                        if (d0 < kEmb)
                            *reinterpret_cast<float4*>(my + kMG + j * kQkv + 2 * kKq + d0) =
                                make_float4(dVt[td][tj][0], dVt[td][tj][1], dVt[td][tj][2], dVt[td][tj][3]);
                    }
                }
            }
            for (int e = lane; e < kTok * kEmb / 4; e += 64)
                *reinterpret_cast<float4*>(my + kMD + 4 * e) = *reinterpret_cast<const float4*>(dhr + 4 * e);
        }
        __syncthreads();
        ef_accumulate<kMmaSample, kMG, kMD, kMX>(sm, nrow, ef);
    }
    ef_write(partial, ef);
}

// sum of the partial rows: workgroup = 64 columns x 16 row classes (r mod 16);
// each thread sums its class in row order, then the 16 class sums are added in
// class order (fixed order: deterministic)
constexpr int kSumCols = 64, kSumClasses = 16;

__global__ __launch_bounds__(kSumCols * kSumClasses) void k_front_sum(const float* __restrict__ partial, int rows,
                                                                      float* __restrict__ red) {
    __shared__ float acc_s[kSumClasses][kSumCols];
    const int c = threadIdx.x % kSumCols, k = threadIdx.x / kSumCols;
    const int e = blockIdx.x * kSumCols + c;
    float acc = 0.f;
    if (e < kPartLen)
        for (int r = k; r < rows; r += kSumClasses) acc += partial[(size_t)r * kPartLen + e];
    acc_s[k][c] = acc;
    __syncthreads();
    if (k == 0 && e < kPartLen) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < kSumClasses; q++) t += acc_s[q][c];
        red[e] = t;
    }
}

// parameter gradients: dWqkv = sum_i E_i Wp_i^T + e_i b_i^T; dWp_i = F_i + Wqkv^T E_i,
// dbp_i = f_i + Wqkv^T e_i (fixed summation order)
// destinations of the parameter gradients in the modules' own layouts (nn.Linear [out][in], [out]):
// the update writes them straight into the .grad storage (no copies out of a packed buffer)
struct FrontGradPtrs {
    float* wq;
    float* wk;
    float* wv;
    float* wp[kTok];  // [20][d_i]
    float* bp[kTok];  // [20]
};

// SCATTER = false: the packed layout grad [kGradLen]; true: the per-parameter destinations dst
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_front_combine(const float* __restrict__ ws, const float* __restrict__ red,
                                                       float* __restrict__ grad, FrontGradPtrs dst) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGradLen) return;
    auto put = [&](float v) {
        if (!SCATTER) {
            grad[e] = v;
        } else if (e < kGP) {
            const int r = e / kEmb, c = e % kEmb;
            float* d = r < kKq ? dst.wq + r * kEmb : r < 2 * kKq ? dst.wk + (r - kKq) * kEmb : dst.wv + (r - 2 * kKq) * kEmb;
            d[c] = v;
        } else if (e < kGB) {
            const int f = e - kGP, tk = f / (kEmb * kPin), c = (f / kPin) % kEmb, k = f % kPin;
            if (k < c_dims[tk]) dst.wp[tk][c * c_dims[tk] + k] = v;
        } else {
            const int f = e - kGB;
            dst.bp[f / kEmb][f % kEmb] = v;
        }
    };
    const float* W = ws + kWsW;  // [40][20]
    if (e < kGP) {
        const int r = e / kEmb, c = e % kEmb;
        float acc = 0.f;
        for (int tk = 0; tk < kTok; tk++) {
            const float* Wp = ws + kWsWP + (tk * kEmb + c) * kPin;  // Wp_i[c][0..3] (zero beyond d_i)
            const float* E = red + kPEF + (tk * kGd + r) * kPin;    // E_i[r][0..3]
#pragma unroll
            for (int a = 0; a < kPin; a++) acc = fmaf(E[a], Wp[a], acc);
            acc = fmaf(red[kPef + tk * kGd + r], ws[kWsBP + tk * kEmb + c], acc);  // e_i[r] b_i[c]
        }
        put(acc);
    } else if (e < kGB) {
        const int f = e - kGP, tk = f / (kEmb * kPin), c = (f / kPin) % kEmb, k = f % kPin;
        float acc = red[kPEF + (tk * kGd + kQkv + c) * kPin + k];  // F_i[c][k]
        for (int r = 0; r < kQkv; r++) acc = fmaf(W[r * kEmb + c], red[kPEF + (tk * kGd + r) * kPin + k], acc);
        put(acc);
    } else {
        const int f = e - kGB, tk = f / kEmb, c = f % kEmb;
        float acc = red[kPef + tk * kGd + kQkv + c];  // f_i[c]
        for (int r = 0; r < kQkv; r++) acc = fmaf(W[r * kEmb + c], red[kPef + tk * kGd + r], acc);
        put(acc);
    }
}

}  // namespace mm

using namespace mm;

extern "C" int mm_actor_front_ws_len(void) { return kWsLen; }
extern "C" int mm_actor_front_grad_len(void) { return kGradLen; }
extern "C" int mm_actor_front_partial_len(void) { return kPartLen; }

extern "C" int mm_actor_front_prep(const float* const* wproj, const float* const* bproj, const float* wq,
                                   const float* wk, const float* wv, float* ws, void* stream) {
    if (!wproj || !bproj || !wq || !wk || !wv || !ws) return MM_E_ARG;
    ProjPtrs P;
    for (int i = 0; i < kTok; i++) {
        if (!wproj[i] || !bproj[i]) return MM_E_ARG;
        P.w[i] = wproj[i];
        P.b[i] = bproj[i];
    }
    hipLaunchKernelGGL(k_front_prep, dim3(kTok), dim3(256), 0, (hipStream_t)stream, P, wq, wk, wv, ws);
    return (int)hipGetLastError();
}

static int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
    return cus[dev];
}

extern "C" int mm_actor_front_fwd_ex(const float* ws, const float* x, int ldx, int B, int parity, float* h,
                                     int algo, void* stream) {
    if (!ws || !x || !h || B < 0 || ldx < MM_OBS_DIM) return MM_E_ARG;
    if (algo != MM_FRONT_FWD_ROW1 && algo != MM_FRONT_FWD_ROW2) return MM_E_ARG;
    if (B == 0) return 0;
    if (algo == MM_FRONT_FWD_ROW2) {
        const int groups = (B + kF2Rows - 1) / kF2Rows;
        const int grid = groups < 2 * cu_count() ? groups : 2 * cu_count();  // two workgroups per CU (72 KB LDS)
        hipLaunchKernelGGL(k_front_fwd2, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B, parity, h);
    } else {
        const int groups = (B + kFwdRows - 1) / kFwdRows;
        const int grid = groups < 3 * cu_count() ? groups : 3 * cu_count();  // three workgroups per CU
        hipLaunchKernelGGL(k_front_fwd, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B, parity, h);
    }
    return (int)hipGetLastError();
}

extern "C" int mm_actor_front_fwd(const float* ws, const float* x, int ldx, int B, int parity, float* h,
                                  void* stream) {
    return mm_actor_front_fwd_ex(ws, x, ldx, B, parity, h, MM_FRONT_FWD_ROW1, stream);
}

static int front_bwd(const float* ws, const float* x, int ldx, int B, int parity, const float* dh, float* partial,
                     int grid, float* red, float* grad, const FrontGradPtrs* dst, int algo, void* stream) {
    if (!ws || !x || !dh || !partial || !red || (!grad && !dst) || B < 0 || ldx < MM_OBS_DIM || grid <= 0)
        return MM_E_ARG;
    if (algo != MM_FRONT_BWD_MFMA && algo != MM_FRONT_BWD_VALU) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (algo == MM_FRONT_BWD_MFMA)
        hipLaunchKernelGGL(k_front_bwd_mfma, dim3(grid), dim3(kBwdThreads), 0, s, ws, x, ldx, B, parity, dh, partial);
    else
        hipLaunchKernelGGL(k_front_bwd, dim3(grid), dim3(kBwdThreads), 0, s, ws, x, ldx, B, parity, dh, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_front_sum, dim3((kPartLen + kSumCols - 1) / kSumCols), dim3(kSumCols * kSumClasses), 0, s,
                       partial, grid, red);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    if (grad)
        hipLaunchKernelGGL(k_front_combine<false>, dim3((kGradLen + 255) / 256), dim3(256), 0, s, ws, red, grad,
                           FrontGradPtrs{});
    else
        hipLaunchKernelGGL(k_front_combine<true>, dim3((kGradLen + 255) / 256), dim3(256), 0, s, ws, red, nullptr, *dst);
    return (int)hipGetLastError();
}

extern "C" int mm_actor_front_bwd_ex(const float* ws, const float* x, int ldx, int B, int parity, const float* dh,
                                     float* partial, int grid, float* red, float* grad, int algo, void* stream) {
    if (!grad) return MM_E_ARG;
    return front_bwd(ws, x, ldx, B, parity, dh, partial, grid, red, grad, nullptr, algo, stream);
}

extern "C" int mm_actor_front_bwd_to(const float* ws, const float* x, int ldx, int B, int parity, const float* dh,
                                     float* partial, int grid, float* red, float* const* wproj_grad,
                                     float* const* bproj_grad, float* wq_grad, float* wk_grad, float* wv_grad,
                                     int algo, void* stream) {
    if (!wproj_grad || !bproj_grad || !wq_grad || !wk_grad || !wv_grad) return MM_E_ARG;
    FrontGradPtrs d;
    d.wq = wq_grad;
    d.wk = wk_grad;
    d.wv = wv_grad;
    for (int i = 0; i < kTok; i++) {
        if (!wproj_grad[i] || !bproj_grad[i]) return MM_E_ARG;
        d.wp[i] = wproj_grad[i];
        d.bp[i] = bproj_grad[i];
    }
    return front_bwd(ws, x, ldx, B, parity, dh, partial, grid, red, nullptr, &d, algo, stream);
}

extern "C" int mm_actor_front_bwd(const float* ws, const float* x, int ldx, int B, int parity, const float* dh,
                                  float* partial, int grid, float* red, float* grad, void* stream) {
    return mm_actor_front_bwd_ex(ws, x, ldx, B, parity, dh, partial, grid, red, grad, MM_FRONT_BWD_VALU, stream);
}
