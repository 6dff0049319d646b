// actor_front.hip -- fused Actor front-end for gfx950: the 23 feature
// embeddings (networks.py:51-65), Q/K/V projections, softmax attention over
// the 23 tokens and the residual (networks.py:67-82), forward and backward.
//
// Why fused: per sample the front-end is a chain of 23x20 / 23x23 matrices.
// As library calls it becomes batched GEMMs with 10..23-wide tiles plus
// [B,23,40] split/cat copies.  Here a 32-lane group owns one sample, lane i =
// token i (23 of 32 lanes active): its own vectors stay in registers, every
// token's k, v (and in the backward q, P, dS) sit in LDS and are read as
// broadcasts.  fp32 throughout (fmaf accumulation; the softmax as exp2 of the
// scaled logits on v_exp_f32 and v_rcp_f32 for 1 / sum by default -- ~1 ulp
// each -- or the reference's steps, logits / sqrt(10), expf(x - max) * (1 / sum),
// with FRONT_FWD_FAST_SOFTMAX=0 / FRONT_MFMA_FAST_SOFTMAX=0).
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

constexpr float kLog2eRsqrtKq = 1.44269504088896341f * 0.316227766016838f;  // log2(e) / sqrt(10)

// The forward's softmax steps.  FRONT_FWD_FAST_SOFTMAX=1 (default): scores kept as raw q.k, exponent
// exp2(q.k log2(e) / sqrt(10) - max) on v_exp_f32 (one fma + one exp instead of the division and the
// libm expf sequence), v_rcp_f32 for 1 / sum (~1 ulp each; h stays within ~3e-7 relative of the
// reference's steps, the same form as k_front_bwd_mfma's backward).  0: the reference's steps
// (x / sqrt(10), expf, 1 / sum).
#ifndef FRONT_FWD_FAST_SOFTMAX
#define FRONT_FWD_FAST_SOFTMAX 1
#endif
__device__ __forceinline__ float fwd_score(float qk) {
#if FRONT_FWD_FAST_SOFTMAX
    return qk;
#else
    return div_sqrt_kq(qk);
#endif
}
__device__ __forceinline__ float fwd_exp(float s, float mx) {
#if FRONT_FWD_FAST_SOFTMAX
    return __builtin_amdgcn_exp2f(fmaf(s, kLog2eRsqrtKq, -mx * kLog2eRsqrtKq));
#else
    return expf(s - mx);
#endif
}
__device__ __forceinline__ float fwd_rcp(float sum) {
#if FRONT_FWD_FAST_SOFTMAX
    return __builtin_amdgcn_rcpf(sum);
#else
    return 1.f / sum;
#endif
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
// up rows).  Same per-element order as affine4 (mul, three fmas, + c): bit-identical results.  Rows
// [LO, HI) only when given (multiples of 4).
template <int R, int LO = 0, int HI = R>
__device__ __forceinline__ void affine4t(const float* __restrict__ MT, const float* __restrict__ c, float4 xv,
                                         float o[R]) {
    const f32x2 x0 = {xv.x, xv.x}, x1 = {xv.y, xv.y}, x2 = {xv.z, xv.z}, x3 = {xv.w, xv.w};
    const float4* m0 = reinterpret_cast<const float4*>(MT);
    const float4* m1 = reinterpret_cast<const float4*>(MT + R);
    const float4* m2 = reinterpret_cast<const float4*>(MT + 2 * R);
    const float4* m3 = reinterpret_cast<const float4*>(MT + 3 * R);
    const float4* c4 = reinterpret_cast<const float4*>(c);
#pragma unroll
    for (int r4 = LO / 4; r4 < HI / 4; r4++) {
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

// acc += p * v; N % 4 == 0: packed FMAs on aligned accumulator pairs with p broadcast (per element the
// same fmaf as the scalar form: bit-identical, half the instructions)
template <int N>
__device__ __forceinline__ void axpy4(float* acc, float p, const float* __restrict__ v_lds) {
    if constexpr (N % 4 == 0) {
        const float4* v4 = reinterpret_cast<const float4*>(v_lds);
        const f32x2 pp = {p, p};
#pragma unroll
        for (int k = 0; k < N / 4; k++) {
            const float4 v = v4[k];
            const f32x2 lo = __builtin_elementwise_fma(pp, f32x2{v.x, v.y}, f32x2{acc[4 * k], acc[4 * k + 1]});
            const f32x2 hi = __builtin_elementwise_fma(pp, f32x2{v.z, v.w}, f32x2{acc[4 * k + 2], acc[4 * k + 3]});
            acc[4 * k] = lo.x;
            acc[4 * k + 1] = lo.y;
            acc[4 * k + 2] = hi.x;
            acc[4 * k + 3] = hi.y;
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

// k rows of the forward's K image, padded from 10 to kKqP = 12 floats (48 bytes): every row starts
// 16-byte aligned, so a q.k_j reads one row as two ds_read_b128 + one ds_read_b64 (10 LDS cycles per
// wave) -- at the unpadded 40-byte pitch every other row is only 8-byte aligned and the compiler reads
// all rows as ds_read2_b64 pairs (20 cycles).  The forward is bound by LDS cycles (per wave-iteration
// of two samples ~1,280 LDS cycles against ~650 VALU instructions), so this is the K share of that.
#ifndef FRONT_FWD_KPITCH
#define FRONT_FWD_KPITCH 12
#endif
constexpr int kKqP = FRONT_FWD_KPITCH;
static_assert(kKqP == 10 || kKqP == 12, "FRONT_FWD_KPITCH is 10 or 12");
__device__ __forceinline__ void store_krow(float* kr, const float* k) {
    if constexpr (kKqP == 12) {
        *reinterpret_cast<float4*>(kr) = make_float4(k[0], k[1], k[2], k[3]);
        *reinterpret_cast<float4*>(kr + 4) = make_float4(k[4], k[5], k[6], k[7]);
        *reinterpret_cast<float2*>(kr + 8) = make_float2(k[8], k[9]);
    } else {
#pragma unroll
        for (int a = 0; a < kKq; a += 2) *reinterpret_cast<float2*>(kr + a) = make_float2(k[a], k[a + 1]);
    }
}
// q . k_j: the same packed-pair order as dot4<10> (pairs (0,1) .. (8,9) into one f32x2 accumulator), so
// h is bit-identical at either pitch
__device__ __forceinline__ float dot_krow(const float* q, const float* __restrict__ kr) {
    if constexpr (kKq == 10 && kKqP == 12) {
        const float4 v0 = *reinterpret_cast<const float4*>(kr);
        const float4 v1 = *reinterpret_cast<const float4*>(kr + 4);
        const float2 v2 = *reinterpret_cast<const float2*>(kr + 8);
        f32x2 acc = {0.f, 0.f};
        acc = __builtin_elementwise_fma(f32x2{q[0], q[1]}, f32x2{v0.x, v0.y}, acc);
        acc = __builtin_elementwise_fma(f32x2{q[2], q[3]}, f32x2{v0.z, v0.w}, acc);
        acc = __builtin_elementwise_fma(f32x2{q[4], q[5]}, f32x2{v1.x, v1.y}, acc);
        acc = __builtin_elementwise_fma(f32x2{q[6], q[7]}, f32x2{v1.z, v1.w}, acc);
        acc = __builtin_elementwise_fma(f32x2{q[8], q[9]}, f32x2{v2.x, v2.y}, acc);
        return acc.x + acc.y;
    } else {
        return dot4<kKq>(q, kr);
    }
}

// H16: h stored as fp16 (the fp16 networks' update: their first trunk GEMM and its weight gradient round h to
// fp16 anyway), rounded to nearest from the same fp32 values
template <bool H16 = false>
__global__ __launch_bounds__(256) void k_front_fwd(const float* __restrict__ ws, const float* __restrict__ x,
                                                   int ldx, int B, int parity, void* __restrict__ hv) {
    __shared__ __attribute__((aligned(16))) float tab[kTok * kTabF];
    __shared__ __attribute__((aligned(16))) float Ks[kFwdRows][kTok][kKqP];
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
            // 16- and 8-byte LDS writes (k rows padded to 48 bytes, v rows of 80) instead of 30 4-byte ones
            store_krow(&Ks[g][i][0], o + kKq);
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
                s[j] = fwd_score(dot_krow(q, Ks[g][j]));
                mx = fmaxf(mx, s[j]);
            }
            float sum0 = 0.f, sum1 = 0.f;  // even / odd j: two short chains (the backward recomputes the same way)
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                s[j] = fwd_exp(s[j], mx);
                if (j & 1) sum1 += s[j];
                else sum0 += s[j];
            }
            const float sum = sum0 + sum1;
            float out[kEmb];
#pragma unroll
            for (int c = 0; c < kEmb; c++) out[c] = 0.f;
            const float inv = fwd_rcp(sum);  // torch's softmax scales by the reciprocal of the sum
#pragma unroll
            for (int j = 0; j < kTok; j++) axpy4<kEmb>(out, s[j] * inv, Vs[g][j]);
            float t[kEmb];
            affine4t<kEmb>(ti + kQkv * (kPin + 1), ti + kQkv * (kPin + 1) + kEmb * kPin, xv, t);
            if constexpr (H16) {
                typedef __attribute__((ext_vector_type(4))) _Float16 h4;
                _Float16* o = static_cast<_Float16*>(hv) + (size_t)row * kRowF + i * kEmb;
#pragma unroll
                for (int c = 0; c < kEmb; c += 4)
                    *reinterpret_cast<h4*>(o + c) = h4{(_Float16)(t[c] + out[c]), (_Float16)(t[c + 1] + out[c + 1]),
                                                       (_Float16)(t[c + 2] + out[c + 2]), (_Float16)(t[c + 3] + out[c + 3])};
            } else {
                float* o = static_cast<float*>(hv) + (size_t)row * kRowF + i * kEmb;
#pragma unroll
                for (int c = 0; c < kEmb; c += 4)
                    *reinterpret_cast<float4*>(o + c) =
                        make_float4(t[c] + out[c], t[c + 1] + out[c + 1], t[c + 2] + out[c + 2], t[c + 3] + out[c + 3]);
            }
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
    __shared__ __attribute__((aligned(16))) float Ks[kF2Rows][kTok][kKqP];
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
            store_krow(&Ks[g][i0][0], o + kKq);
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(&Vs[g][i0][c]) =
                    make_float4(o[2 * kKq + c], o[2 * kKq + c + 1], o[2 * kKq + c + 2], o[2 * kKq + c + 3]);
            affine4t<kQkv>(tb, tb + kQkv * kPin, xb, o);
#pragma unroll
            for (int a = 0; a < kKq; a++) qb[a] = o[a];
            if (own1) {
                store_krow(&Ks[g][i1][0], o + kKq);
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
                sa[j] = fwd_score(dot_krow(qa, Ks[g][j]));
                sb[j] = fwd_score(dot_krow(qb, Ks[g][j]));
                mxa = fmaxf(mxa, sa[j]);
                mxb = fmaxf(mxb, sb[j]);
            }
            float suma0 = 0.f, suma1 = 0.f, sumb0 = 0.f, sumb1 = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                sa[j] = fwd_exp(sa[j], mxa);
                sb[j] = fwd_exp(sb[j], mxb);
                if (j & 1) {
                    suma1 += sa[j];
                    sumb1 += sb[j];
                } else {
                    suma0 += sa[j];
                    sumb0 += sb[j];
                }
            }
            const float inva = fwd_rcp(suma0 + suma1), invb = fwd_rcp(sumb0 + sumb1);
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
// forward on the fp32 MFMA (k_front_fwd_mfma)
// ---------------------------------------------------------------------------
// k_front_fwd spends its time on LDS cycles, not on arithmetic: every lane
// reads all 23 k_j / v_j rows of its sample as broadcasts, ~1,100 LDS cycles
// per wavefront and two samples against ~650 VALU instructions.  Here the two
// products run on v_mfma_f32_32x32x2_f32 (an exact fp32 fmaf chain per output,
// no operand split), one sample at a time on the whole wavefront:
//   S^T   = K Q^T    [j][i], k = a (10: five steps, no padding)
//   ctx^T = V^T P^T  [c][i], k = j (23 -> 24: twelve steps), accumulated onto t^T
// Phase 1 is k_front_fwd's (lane = token, the wavefront's two samples in its
// two halves, folded maps from the staged tables).  The MFMA operands then come
// from registers: lane half 1 needs the other sample's q / k / t values of its
// token, one v_permlane32_swap per register pair (lanes 32-63 of the first
// operand trade with lanes 0-31 of the second), so sample 0's k-step e pairs
// a = 5 + e (lanes 0-31) with a = e (lanes 32-63), and the same for sample 1.
// The S^T C tile (lane l: column i = l & 31, register r: row j = (r & 3) +
// 8 (r >> 2) + 4 (l >> 5)) is the B operand of the second product as it stands
// (k-step r, k-lane l >> 5 = row j of register r); its A operand V^T reads
// v_j[c] from LDS (V image [32][20] per sample, rows 23-31 zero) with lanes
// c = l & 31 on consecutive words.  The result's lane holds token i's
// columns c = 4 (l >> 5) + 0..3, 8 + .., 16 + .. (lanes 0-31): 16-byte stores.
// LDS per workgroup: the tables (27.6 KB) and eight V images (20 KB), three
// workgroups per CU.  The softmax is k_front_fwd's (fwd_score / fwd_exp /
// fwd_rcp), over the 8 + 4 register rows of the lane and its partner lane.
constexpr int kFMRows = 8;  // samples per workgroup iteration: two per wavefront
// waves per SIMD the register budget is cut for (2: 256 VGPRs, 222 used, two workgroups per CU; 3: 168,
// with spills, three per CU as the LDS allows)
#ifndef FRONT_FM_WAVES
#define FRONT_FM_WAVES 3
#endif
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

__device__ __forceinline__ f32x16_t mfma32(float a, float b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// v_permlane32_swap(a, b): s0 = {a of lanes 0-31, b of lanes 0-31}, s1 = {a of lanes 32-63, b of lanes 32-63}
// -- with the wavefront's sample 0 in lanes 0-31 and sample 1 in lanes 32-63, s0 holds sample 0's a (low
// lanes) and b (high lanes), s1 sample 1's
__device__ __forceinline__ void swap32(float a, float b, float& s0, float& s1) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    s0 = __uint_as_float(r[0]);
    s1 = __uint_as_float(r[1]);
}

// 1 (default): the wavefront's two samples' MFMA chains interleaved; 0: one after the other
#ifndef FRONT_FM_ILP
#define FRONT_FM_ILP 1
#endif
// ctx^T = V^T P^T: 1 (default) on the x2 f16 MFMA (v_mfma_f32_32x32x16_f16: hi hi, hi lo, lo hi, two k-steps of
// 16 rows j: 6 MFMAs of 32 cycles per sample instead of 12 f32 ones of 64), 0 on the fp32 MFMA
#ifndef FRONT_FM_PV
#define FRONT_FM_PV 1
#endif
static_assert(FRONT_FM_PV == 0 || FRONT_FM_ILP == 1, "the x2 PV product is built in the interleaved form");
// the V image's scale: v 2^-8 is split, the result scaled back by 2^8 (both exact), so fp16's range covers
// |v| < 2^24 and the hi plane stays normal down to |v| = 2^-6
constexpr float kFMVs = 1.f / 256.f, kFMVsInv = 256.f;
constexpr float kFMLo = 2048.f, kFMLoInv = 1.f / 2048.f;  // x2: x = hi + 2^-11 lo
typedef _Float16 fm_f16x8 __attribute__((ext_vector_type(8)));
typedef short fm_s4 __attribute__((ext_vector_type(4)));

// x2 split of two values (x s): hi = RN16(x s), lo = RN16(2^11 (x s - hi)), as x3mlp.hip's pair2
__device__ __forceinline__ void fm_pair2(float x0, float x1, float s, uint32_t& h, uint32_t& l) {
    typedef __attribute__((ext_vector_type(2))) _Float16 h2;
    const f32x2 v = f32x2{x0, x1} * s;
    const h2 hv = __builtin_convertvector(v, h2);
    const f32x2 r = (v - __builtin_convertvector(hv, f32x2)) * kFMLo;
    h = __builtin_bit_cast(uint32_t, hv);
    l = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h2));
}

// 4 x 16-bit of a [row][col] LDS image, transposed across each 16-lane group (ds_read_b64_tr_b16)
__device__ __forceinline__ fm_s4 fm_tr(const uint16_t* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) fm_s4*)(p));
}

// softmax over the rows j of the S^T tile's column i: registers r < 12 of both lane halves (j = 23, register
// 11 of the high half, and j >= 24 are padding); p = P^T's registers
__device__ __forceinline__ void fm_softmax(f32x16_t& S, int hh, float (&p)[12]) {
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 12; r++) {
        S[r] = fwd_score(S[r]);
        if (r < 11 || hh == 0) mx = fmaxf(mx, S[r]);
    }
    float m0, m1;
    swap32(mx, mx, m0, m1);
    mx = fmaxf(m0, m1);
    float sum0 = 0.f, sum1 = 0.f;
#pragma unroll
    for (int r = 0; r < 12; r++) {
        p[r] = (r < 11 || hh == 0) ? fwd_exp(S[r], mx) : 0.f;
        if (r & 1) sum1 += p[r];
        else sum0 += p[r];
    }
    float s0, s1;
    swap32(sum0 + sum1, sum0 + sum1, s0, s1);
    const float inv = fwd_rcp(s0 + s1);
#pragma unroll
    for (int r = 0; r < 12; r++) p[r] *= inv;
}

// h row `row`, token tok: this lane's column quads 4 hh, 8 + 4 hh (and 16 on lanes 0-31) of ctx^T + t^T
template <bool H16>
__device__ __forceinline__ void fm_store(void* hv, int row, int tok, int hh, const f32x16_t& acc) {
    if (tok >= kTok) return;
    const int nq = hh ? 2 : 3;
    if constexpr (H16) {
        typedef __attribute__((ext_vector_type(4))) _Float16 h4;
        _Float16* hr = static_cast<_Float16*>(hv) + (size_t)row * kRowF + tok * kEmb + 4 * hh;
#pragma unroll
        for (int m = 0; m < 3; m++)
            if (m < nq)
                *reinterpret_cast<h4*>(hr + 8 * m) = h4{(_Float16)acc[4 * m], (_Float16)acc[4 * m + 1],
                                                       (_Float16)acc[4 * m + 2], (_Float16)acc[4 * m + 3]};
    } else {
        float* hr = static_cast<float*>(hv) + (size_t)row * kRowF + tok * kEmb + 4 * hh;
#pragma unroll
        for (int m = 0; m < 3; m++)
            if (m < nq)
                *reinterpret_cast<float4*>(hr + 8 * m) =
                    make_float4(acc[4 * m], acc[4 * m + 1], acc[4 * m + 2], acc[4 * m + 3]);
    }
}

template <bool H16 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FRONT_FM_WAVES))) void k_front_fwd_mfma(const float* __restrict__ ws, const float* __restrict__ x,
                                                        int ldx, int B, int parity, void* __restrict__ hv) {
    __shared__ __attribute__((aligned(16))) float tab[kTok * kTabF];
#if FRONT_FM_PV
    // V image as x2 fp16 planes [plane][slot][32 rows][20] (rows 23-31 zero), plus a pad: the transposed reads
    // of columns 20-31 run past a row's end (into the next row, past the last one into the pad) and reach only
    // rows c >= 20 of the result
    constexpr int kVpN = kFMRows * 32 * kEmb + 16;
    __shared__ __attribute__((aligned(16))) uint16_t Vp[2][kVpN];
    for (int e = threadIdx.x; e < kVpN; e += 256) Vp[0][e] = Vp[1][e] = 0;
#else
    __shared__ __attribute__((aligned(16))) float Vs[kFMRows][32][kEmb];
    for (int e = threadIdx.x; e < kFMRows * 32 * kEmb; e += 256) (&Vs[0][0][0])[e] = 0.f;
#endif
    stage_tables(ws, tab);
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    const int hh = (threadIdx.x >> 5) & 1;  // lane half: phase 1's sample, the MFMAs' k-lane
    const int tok = threadIdx.x & 31;       // phase 1's token; the MFMA results' column i
    const int groups = (B + kFMRows - 1) / kFMRows;
    for (int grp = blockIdx.x; grp < groups; grp += gridDim.x) {
        const int row0 = grp * kFMRows + 2 * wave;  // the wavefront's samples row0, row0 + 1
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tok < kTok && row0 + hh < B) xv = xslice(x + (size_t)(row0 + hh) * ldx, tok, parity != 0);
        // ---- phase 1: q | k | v and t of token tok of sample hh (padding tokens and samples past B: the
        // maps of token 0 at x = 0, finite values that no stored result depends on) ----
        // the table address behind an opaque copy: the tables are loop-invariant, and hoisted out of the loop
        // their 300 words per lane spill
        // (padding lanes 23-31 read token tok - 16's table: their 16-byte reads then fill the bank quads the
        // other lanes of their ds_read_b128 lane group leave free -- token 0's, the obvious choice, shares
        // a quad with token 16 in lane group {4-11, 16-19, 28-31}: 2-way conflicts on every table read)
        int toff = (tok < kTok ? tok : tok - 16) * kTabF;
        asm volatile("" : "+v"(toff));
        const float* tl = tab + toff;
        float o[kQkv], t[kEmb];
        // table reads in groups of at most ten 16-byte reads, each group's values consumed before the next is
        // issued (scheduling barriers): issued all at once, the 75 reads per lane need 300 registers
#define FM_SB __builtin_amdgcn_sched_barrier(0)
        affine4t<kQkv, 0, 8>(tl, tl + kQkv * kPin, xv, o);
        FM_SB;
        affine4t<kQkv, 8, 16>(tl, tl + kQkv * kPin, xv, o);
        FM_SB;
        affine4t<kQkv, 16, 20>(tl, tl + kQkv * kPin, xv, o);
        // MFMA operands per sample s: q / k at k-step e (a = 5 + e on lanes 0-31, a = e on lanes 32-63) and
        // t in the C layout of ctx^T (register 4 m + u: c = 8 m + 4 hh + u for m < 2, 16 + u for m = 2 on
        // lanes 0-31)
        float qs[2][5], ks[2][5], ts[2][12];
#pragma unroll
        for (int e = 0; e < 5; e++) {
            swap32(o[5 + e], o[e], qs[0][e], qs[1][e]);
            swap32(o[kKq + 5 + e], o[kKq + e], ks[0][e], ks[1][e]);
        }
        FM_SB;
        affine4t<kQkv, 20, 28>(tl, tl + kQkv * kPin, xv, o);
        FM_SB;
        affine4t<kQkv, 28, 36>(tl, tl + kQkv * kPin, xv, o);
        FM_SB;
        affine4t<kQkv, 36, 40>(tl, tl + kQkv * kPin, xv, o);
        wave_sync();  // the previous iteration's V readers (this wavefront) are done
        if (tok < kTok) {
#if FRONT_FM_PV
            uint32_t vh[kEmb / 2], vl[kEmb / 2];
#pragma unroll
            for (int k = 0; k < kEmb / 2; k++) fm_pair2(o[2 * kKq + 2 * k], o[2 * kKq + 2 * k + 1], kFMVs, vh[k], vl[k]);
            uint2* dh = reinterpret_cast<uint2*>(&Vp[0][((2 * wave + hh) * 32 + tok) * kEmb]);  // 40-byte rows
            uint2* dl = reinterpret_cast<uint2*>(&Vp[1][((2 * wave + hh) * 32 + tok) * kEmb]);
#pragma unroll
            for (int k = 0; k < kEmb / 4; k++) {
                dh[k] = make_uint2(vh[2 * k], vh[2 * k + 1]);
                dl[k] = make_uint2(vl[2 * k], vl[2 * k + 1]);
            }
#else
            float4* vr = reinterpret_cast<float4*>(&Vs[2 * wave + hh][tok][0]);
#pragma unroll
            for (int c = 0; c < kEmb / 4; c++)
                vr[c] = make_float4(o[2 * kKq + 4 * c], o[2 * kKq + 4 * c + 1], o[2 * kKq + 4 * c + 2],
                                    o[2 * kKq + 4 * c + 3]);
#endif
        }
        FM_SB;
        const float* tt = tl + kQkv * (kPin + 1);
        affine4t<kEmb, 0, 8>(tt, tt + kEmb * kPin, xv, t);
        FM_SB;
        affine4t<kEmb, 8, 16>(tt, tt + kEmb * kPin, xv, t);
        FM_SB;
        affine4t<kEmb, 16, 20>(tt, tt + kEmb * kPin, xv, t);
#undef FM_SB
#pragma unroll
        for (int m = 0; m < 2; m++)
#pragma unroll
            for (int u = 0; u < 4; u++) swap32(t[8 * m + u], t[8 * m + 4 + u], ts[0][4 * m + u], ts[1][4 * m + u]);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            float dummy;
            swap32(t[16 + u], t[16 + u], dummy, ts[1][8 + u]);
            ts[0][8 + u] = t[16 + u];
        }
        wave_sync();  // the V images are written
#if FRONT_FM_ILP
        // both samples' chains side by side (independent MFMA accumulators and softmax chains: each wave keeps
        // its own matrix pipe and VALU busy while the other chain waits); a sample past B is computed on the
        // finite phase-1 values and not stored
        if (row0 < B) {  // wavefront-uniform
            f32x16_t S[2] = {{}, {}};
#pragma unroll
            for (int e = 0; e < 5; e++) {
                S[0] = mfma32(ks[0][e], qs[0][e], S[0]);
                S[1] = mfma32(ks[1][e], qs[1][e], S[1]);
            }
            float p[2][12];
#pragma unroll
            for (int s = 0; s < 2; s++) fm_softmax(S[s], hh, p[s]);
            f32x16_t acc[2] = {{}, {}};
#if FRONT_FM_PV
            // B = P^T: k-step t takes the S^T registers 8t .. 8t + 7 as they stand (element e of lane half hh is
            // row j = 16 t + 8 (e >> 2) + 4 hh + (e & 3)), split into the x2 planes; A = V^T: the same rows j of
            // column c = lane & 31, two transposed 4-row reads per plane (lane 4q + p of a 16-lane group: row q of
            // the block, columns 4p .. 4p + 3).  acc = t^T 2^-8 + hi hi, accx = hi lo + lo hi; h = 2^8 (acc +
            // 2^-11 accx)
            f32x16_t accx[2] = {{}, {}};
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int r = 0; r < 12; r++) acc[s][r] = ts[s][r] * kFMVs;
            const int lane = threadIdx.x & 63;
            const int voff = (2 * wave * 32 + 4 * hh + ((lane >> 2) & 3)) * kEmb + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
#pragma unroll
            for (int t = 0; t < 2; t++) {
                fm_f16x8 bh[2], bl[2];
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    uint32_t h4[4], l4[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int r = 8 * t + 2 * k;
                        if (r < 12) fm_pair2(p[s][r], p[s][r + 1], 1.f, h4[k], l4[k]);
                        else h4[k] = l4[k] = 0u;
                    }
                    bh[s] = __builtin_bit_cast(fm_f16x8, make_uint4(h4[0], h4[1], h4[2], h4[3]));
                    bl[s] = __builtin_bit_cast(fm_f16x8, make_uint4(l4[0], l4[1], l4[2], l4[3]));
                }
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int o0 = voff + (s * 32 + 16 * t) * kEmb;
                    fm_s4 a0 = fm_tr(&Vp[0][o0]), a1 = fm_tr(&Vp[0][o0 + 8 * kEmb]);
                    fm_s4 c0 = fm_tr(&Vp[1][o0]), c1 = fm_tr(&Vp[1][o0 + 8 * kEmb]);
                    const fm_f16x8 ah = __builtin_bit_cast(fm_f16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
                    const fm_f16x8 al = __builtin_bit_cast(fm_f16x8, __builtin_shufflevector(c0, c1, 0, 1, 2, 3, 4, 5, 6, 7));
                    accx[s] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[s], accx[s], 0, 0, 0);
                    accx[s] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[s], accx[s], 0, 0, 0);
                    acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[s], acc[s], 0, 0, 0);
                }
            }
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int r = 0; r < 12; r++) acc[s][r] = fmaf(accx[s][r], kFMLoInv, acc[s][r]) * kFMVsInv;
#else
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int r = 0; r < 12; r++) acc[s][r] = ts[s][r];
            const float* vb0 = &Vs[2 * wave][0][0] + tok;
#pragma unroll
            for (int r = 0; r < 12; r++) {
                const int j = (r & 3) + 8 * (r >> 2) + 4 * hh;
                acc[0] = mfma32(vb0[j * kEmb], p[0][r], acc[0]);
                acc[1] = mfma32(vb0[32 * kEmb + j * kEmb], p[1][r], acc[1]);
            }
#endif
            fm_store<H16>(hv, row0, tok, hh, acc[0]);
            if (row0 + 1 < B) fm_store<H16>(hv, row0 + 1, tok, hh, acc[1]);
        }
#else
        // one sample at a time (a rolled loop: the second sample's operands move into the first's registers at
        // the end of the first pass; unrolled, the two chains interleave and spill)
#pragma unroll 1
        for (int s = 0; s < 2; s++) {
            const int row = row0 + s;
            if (row >= B) break;  // wavefront-uniform
            f32x16_t S = {};
#pragma unroll
            for (int e = 0; e < 5; e++) S = mfma32(ks[0][e], qs[0][e], S);
            float p[12];
            fm_softmax(S, hh, p);
            // ctx^T + t^T: A = V^T (v_j[c], c = l & 31: words past c = 19 are the next row's, finite, and only
            // reach rows c >= 20 of the result), B = P^T (register r)
            const float* vb = &Vs[2 * wave + s][0][0] + tok;
            f32x16_t acc = {};
#pragma unroll
            for (int r = 0; r < 12; r++) acc[r] = ts[0][r];
#pragma unroll
            for (int r = 0; r < 12; r++) {
                const int j = (r & 3) + 8 * (r >> 2) + 4 * hh;
                acc = mfma32(vb[j * kEmb], p[r], acc);
            }
            fm_store<H16>(hv, row, tok, hh, acc);
#pragma unroll
            for (int e = 0; e < 5; e++) qs[0][e] = qs[1][e], ks[0][e] = ks[1][e];
#pragma unroll
            for (int r = 0; r < 12; r++) ts[0][r] = ts[1][r];
        }
#endif
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
// backward on the fp32 MFMA (k_front_bwd_mfma)
// ---------------------------------------------------------------------------
// The per-sample attention products run as v_mfma_f32_16x16x4_f32 tiles
// (fp32 operands, an exact fmaf chain per output: no operand split), tokens
// padded 23 -> 32.  One wavefront per sample, two samples per wave per
// iteration.  The attention is held TRANSPOSED, S^T [j][i] (C tile: lane l
// holds rows j = 4 (l >> 4) + g, column i = l & 15), so a softmax row (over j
// for query i) is 8 values in the lane plus the 4 lane groups of 16 (two
// permlane swaps).  Products (k = the summed index):
//   S^T  = K Q^T          k = a: A = k rows, B = q rows      (QKV in LDS)
//   dP^T = V dctx^T       k = c: A = v rows (LDS), B = dctx (dh)
//   dQ^T = K^T dS^T       k = j: B = the dS^T C tiles themselves (register g of
//                         a tile is the B operand whose k-lane q4 is row 4 q4 + g)
//   dV   = P^T dctx       k = i: A = P^T rows through a 4.5-KiB LDS transpose
//   dK   = dS^T Q         k = i: A = dS^T rows through the same buffer
// Phase 1 (one lane per token, both samples of the wave at once) forms every
// token's q|k|v once from the folded maps into LDS (QKV [32][44]: q at 0, k at
// 12, v at 24, zero pads and padding tokens), so operands load as aligned
// float4 (one per 4 MFMAs) or from a zero pad (no exec-masked loads); the
// region is reused for the transposes once the operands are in registers, then
// for the reduction operands G = [dq | dk | dv], dctx and x of k_front_bwd,
// whose E/F accumulation phase follows (dctx read from dh).  4 KB of LDS per
// sample plus the folded maps staged once (18.8 KB): 51 KB per 8-sample
// workgroup, three workgroups per CU.  The softmax runs on
// exp2 / rcp (v_exp_f32, v_rcp_f32: ~1 ulp; the reference's
// exp(x / sqrt(10) - max) * (1 / sum) within ~3e-7 relative).
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr int kQp = 44;                      // QKV row pitch (floats): [32 tokens][44]
constexpr int kQO = 0, kKO = 12, kVO = 24;   // q | 0 0 | k | 0 0 | v
constexpr int kTp = 36;                      // transpose buffer T [i][j], pitch 36 (query-major, rows i < 24)
// per sample: QKV [23][44], then T [23][36], then the reduction operands G [23][40] | x [23][4] (dctx is
// read from dh).  The padding tokens' rows 23-31 of QKV and T are read past the rows written -- the next
// words of the workgroup's LDS, zeroed at the start, finite ever after: every product keeps them out of
// the results (S^T and dP^T rows / columns >= 23 are masked out of the softmax, P and dS are 0 there)
constexpr int kMG = 0, kMX = kTok * kQkv;
constexpr int kMSample = kMX + kTok * kPin;  // 1,012 floats per sample
static_assert(kTok * kQp <= kMSample && 24 * kTp <= kMSample, "QKV and T live in the sample's region");
// zeroed words after the last sample's region, so that its padding rows read this kernel's own data (words
// of another kernel could hold anything, and a huge finite value times the zero weight it gets is not 0)
constexpr int kMPad = ((32 * kQp > 32 * kTp ? 32 * kQp : 32 * kTp) - kMSample + 3) & ~3;
// LDS bank swizzles of the per-sample chain (MI355X LDS: ds_read_b32 serves lanes 0-31 and 32-63 in one
// cycle each when their 32 banks are distinct).  The chain's b32 reads touch 16 rows x 2 k-lanes per group;
// with row pitches that are multiples of 4 (the float4 writes need them) rows r and r + 8 share banks, and
// the transposed reads of T (dQ) put 4 lanes on a bank.  So the column index is XORed with a row-dependent
// value below 4 (a permutation inside each float4: the float4 writes permute their components instead):
//   QKV, q | k words (< 24): bit 1 flipped on rows with bit 3 set -- the S^T operand reads conflict-free;
//   T: k ^ L(r), L(r) = (r & 1) | 2 ((r >> 3) & 1) -- the dQ column reads conflict-free.
// Modelled per access (lane groups and bank rules of MI355X_MICROARCH.md): 108 -> 28 extra LDS cycles per
// sample over the chain's 156.  Measured (419,430 rows, tools/ab_libs.py, profiles/r05_front_bwd_swizzle.txt):
// SQ_LDS_BANK_CONFLICT 98.2M -> 64.6M, but the swizzle's selects and XORed addresses add 9% VALU
// instructions in a kernel bound by issue and dependency waits, not by LDS: 1,151 us plain, 1,166 us q|k
// only (bit 0), 1,204 us both (bits 0 + 1).  So FRONT_SWZ=0 (plain) is the default; 1 / 2 / 3 select them.
#ifndef FRONT_SWZ
#define FRONT_SWZ 0
#endif
__device__ __forceinline__ int qk_sw(int r) { return (FRONT_SWZ & 1) ? 2 * ((r >> 3) & 1) : 0; }
__device__ __forceinline__ int t_sw(int r) { return (FRONT_SWZ & 2) ? ((r & 1) | (((r >> 3) & 1) << 1)) : 0; }
// the swizzled column c16 of T's row kh_row(s, q4) (L of that row: bit 0 = s's for s < 4, q4's for s >= 4;
// bit 1 = q4's bit 1 for s < 4, 0 for the rows 16-23)
__device__ __forceinline__ int t_col(int s, int c16, int q4) {
    if constexpr ((FRONT_SWZ & 2) == 0) return c16;
    return s < 4 ? c16 ^ ((s & 1) | (q4 & 2)) : c16 ^ (q4 & 1);
}
// a C tile's four registers to words dst[g ^ x] (x < 4): the halves by address (two 8-byte writes), the
// pairs inside them by select
__device__ __forceinline__ void t_store(float* dst, const f32x4_t& v, int x) {
    const bool sw = x & 1;
    float2* d2 = reinterpret_cast<float2*>(dst);
    const int h = (x >> 1) & 1;
    d2[h] = sw ? make_float2(v[1], v[0]) : make_float2(v[0], v[1]);
    d2[h ^ 1] = sw ? make_float2(v[3], v[2]) : make_float2(v[2], v[3]);
}

#ifndef FRONT_MFMA_FAST_SOFTMAX  // 1: exp2 / rcp / * (1 / sqrt(10)); 0: the reference's steps (12% slower)
#define FRONT_MFMA_FAST_SOFTMAX 1
#endif

__device__ __forceinline__ f32x4_t mfma4(float a, float b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// the k = i steps of dV and dK: i = 4 q4 + s over the first 16 tokens (s < 4), then 16 + q4 + 4 (s - 4):
// two steps cover tokens 16-23 (token 23 is padding: P^T and dS^T are 0 there)
constexpr int kKH = 6;
__device__ __forceinline__ int kh_row(int s, int q4) { return s < 4 ? 4 * q4 + s : 16 + q4 + 4 * (s - 4); }

__device__ __forceinline__ float f4at(const float4& v, int e) {
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

// sum / max over the four 16-lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48): the same value in every lane
// (each swap pairs the lower group's value with the upper's, in that order)
__device__ __forceinline__ float xq_sum(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ float xq_max(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}


// dP^T's B operand of one sample (dh row grow): rows 16 t + c16 (zero past token 22), columns 4 q4 .. 4 q4 + 3
// and 16 + q4
__device__ __forceinline__ void dp_operands(const float* __restrict__ dh, long grow, int c16, int q4, float4 (&df)[2],
                                            float (&dt)[2]) {
    const float* dhr = dh + grow * kRowF;
#pragma unroll
    for (int t = 0; t < 2; t++) {
        const int r = 16 * t + c16, rc = min(r, kTok - 1);
        df[t] = *reinterpret_cast<const float4*>(dhr + rc * kEmb + 4 * q4);
        dt[t] = dhr[rc * kEmb + 16 + q4];
        if (r >= kTok) df[t] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r >= kTok) dt[t] = 0.f;
    }
}

constexpr int kTabS = kQkv * kPin + kQkv + 4;  // staged folded map per token: A^T [4][40] | c [40] | pad; 204 words:
                                               // 16 lanes' 16-byte reads of 16 tokens hit disjoint banks

// E/F phase of k_front_bwd_mfma, with the dctx rows read from dh (L2-resident: the samples' dP operands were
// just read from them) instead of LDS.  Units 0-229: G rows (token u / 10, rows 4 (u % 10)); 230-344: dctx
// rows (token (u - 230) / 5, rows 40 + 4 ((u - 230) % 5)).  Thread t owns units t and t + 256, so at most one
// dctx unit, whose rows for all the iteration's samples are loaded up front (ef2_prefetch, before the barrier)
static_assert(kEFR == 4, "k_front_bwd_mfma's E/F units are 4 rows");
constexpr int kEF2G = kTok * kQkv / 4;  // 230 G units
// samples per workgroup iteration (two per wavefront): 8 -> 256 threads, two E/F units for 89 of them, three
// workgroups per CU (51 KB of LDS each).  12 -> 384 threads, every E/F unit its own thread (half the E/F
// critical path), two workgroups per CU on LDS and registers -- measured 1.54x slower: a 6-wave workgroup
// spreads its waves 2-2-1-1 over the SIMDs, and the second one then finds no SIMD pair free, so only one
// workgroup per CU runs
#ifndef FRONT_MFMA_ROWS
#define FRONT_MFMA_ROWS 8
#endif
constexpr int kMRows = FRONT_MFMA_ROWS;
constexpr int kMThreads = 32 * kMRows;
constexpr int kMPerCU = kMRows == 12 ? 2 : 3;
static_assert(kMRows == 8 || kMRows == 12, "FRONT_MFMA_ROWS is 8 or 12");
constexpr int kMEFU = (kEFUnits + kMThreads - 1) / kMThreads;  // E/F units per thread (1 / 2)
struct EFAccM {
    f32x2 e[kMEFU][4][2];  // [unit][row a][column pair]
    f32x2 s[kMEFU][2];     // [unit][row pair]
};

__device__ __forceinline__ void ef2_unit(int unit, int& tk, int& r0) {
    if (unit < kEF2G) {
        tk = unit / (kQkv / 4);
        r0 = 4 * (unit % (kQkv / 4));
    } else {
        tk = (unit - kEF2G) / (kEmb / 4);
        r0 = kQkv + 4 * ((unit - kEF2G) % (kEmb / 4));
    }
}

// the dctx rows of samples g0 .. g0 + kEFPf - 1 (kEFPf at a time: 48 registers for 12 samples would cost the
// third wave per SIMD)
constexpr int kEFPf = kMRows == 12 ? 6 : kMRows;
__device__ __forceinline__ void ef2_prefetch(const float* __restrict__ dh0, int nrow, int g0, float4 (&fp)[kEFPf]) {
    const int fu = threadIdx.x < kEF2G ? threadIdx.x + kMThreads : threadIdx.x;
    int tk, r0;
    ef2_unit(fu, tk, r0);
    const bool has = fu < kEFUnits;
#pragma unroll
    for (int u = 0; u < kEFPf; u++) {
        const int gg = g0 + u;
        fp[u] = (has && gg < nrow) ? *reinterpret_cast<const float4*>(dh0 + (size_t)gg * kRowF + tk * kEmb + r0 - kQkv)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

template <int kStride, int kG, int kX>
__device__ __forceinline__ void ef2_accumulate(const float* sm, const float* __restrict__ dh0, int nrow,
                                               float4 (&fp)[kEFPf], EFAccM& acc) {
#pragma unroll
    for (int g0 = 0; g0 < kMRows; g0 += kEFPf) {
        if (g0 > 0) ef2_prefetch(dh0, nrow, g0, fp);
#pragma unroll
        for (int u = 0; u < kMEFU; u++) {
            const int unit = threadIdx.x + u * kMThreads;
            if (unit < kEFUnits) {
                int tk, r0;
                ef2_unit(unit, tk, r0);
                const bool lds = unit < kEF2G;
#pragma unroll
                for (int v = 0; v < kEFPf; v++) {
                    const int gg = g0 + v;
                    if (gg < nrow) {
                        const float* sg = sm + gg * kStride;
                        // the G row read unconditionally (for a dctx unit, r0 >= 40, the address is still inside
                        // the sample's region) and selected by value: as a conditional read, the compiler split
                        // it into four exec-masked 4-byte reads and moves per unit and sample
                        const float4 lv = *reinterpret_cast<const float4*>(sg + kG + tk * kQkv + r0);
                        const float4 gv = lds ? lv : fp[v];
                        const float gr[4] = {gv.x, gv.y, gv.z, gv.w};
                        const float4 xq = *reinterpret_cast<const float4*>(sg + kX + tk * kPin);
                        const f32x2 x01 = {xq.x, xq.y}, x23 = {xq.z, xq.w};
#pragma unroll
                        for (int a = 0; a < 4; a++) {
                            const f32x2 ga = {gr[a], gr[a]};
                            acc.e[u][a][0] = __builtin_elementwise_fma(ga, x01, acc.e[u][a][0]);
                            acc.e[u][a][1] = __builtin_elementwise_fma(ga, x23, acc.e[u][a][1]);
                        }
#pragma unroll
                        for (int a = 0; a < 2; a++) acc.s[u][a] += f32x2{gr[2 * a], gr[2 * a + 1]};
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ void ef2_zero(EFAccM& acc) {
#pragma unroll
    for (int u = 0; u < kMEFU; u++) {
#pragma unroll
        for (int a = 0; a < 4; a++) acc.e[u][a][0] = acc.e[u][a][1] = f32x2{0.f, 0.f};
        acc.s[u][0] = acc.s[u][1] = f32x2{0.f, 0.f};
    }
}

__device__ __forceinline__ void ef2_write(float* partial, const EFAccM& acc) {
    float* out = partial + (size_t)blockIdx.x * kPartLen;
#pragma unroll
    for (int u = 0; u < kMEFU; u++) {
        const int unit = threadIdx.x + u * kMThreads;
        if (unit < kEFUnits) {
            int tk, r0;
            ef2_unit(unit, tk, r0);
#pragma unroll
            for (int a = 0; a < 4; a++) {
                *reinterpret_cast<float4*>(out + kPEF + (tk * kGd + r0 + a) * kPin) =
                    make_float4(acc.e[u][a][0].x, acc.e[u][a][0].y, acc.e[u][a][1].x, acc.e[u][a][1].y);
                out[kPef + tk * kGd + r0 + a] = (a & 1) ? acc.s[u][a / 2].y : acc.s[u][a / 2].x;
            }
        }
    }
}

// issue priority of the per-sample chain: 1 (default) its MFMA blocks at s_setprio 1, so a wave entering
// one keeps the SIMD's matrix pipe fed while the co-resident waves' VALU phases fill in (419,430 rows, A/B on
// one box, 7 rounds: 1,206 -> 1,165 us); 2 the softmax (VALU) block at s_setprio 1 instead (1,189 us); 0 none
#ifndef FRONT_PRIO
#define FRONT_PRIO 1
#endif
__device__ __forceinline__ void front_prio(int phase) {  // phase 0: MFMA block starts; 1: softmax starts; 2: chain ends
    if constexpr (FRONT_PRIO == 1) {
        if (phase == 0) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    } else if constexpr (FRONT_PRIO == 2) {
        if (phase == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }
}

__global__ __launch_bounds__(kMThreads) __attribute__((amdgpu_waves_per_eu(3))) void k_front_bwd_mfma(const float* __restrict__ ws,
                                                                   const float* __restrict__ x, int ldx, int B,
                                                                   int parity, const float* __restrict__ dh,
                                                                   float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float sm[kMRows * kMSample + kMPad];
    __shared__ __attribute__((aligned(16))) float tab[kTok * kTabS];
    const int wave = threadIdx.x >> 6;
    for (int e = threadIdx.x; e < kMRows * kMSample + kMPad; e += kMThreads) sm[e] = 0.f;  // (see kMSample)
    // the folded maps once per workgroup (each lane's q|k|v reads them every iteration)
    for (int e = threadIdx.x; e < kTok * (kQkv * kPin + kQkv); e += kMThreads) {
        const int t = e / (kQkv * kPin + kQkv), f = e % (kQkv * kPin + kQkv);
        tab[t * kTabS + f] = f < kQkv * kPin ? ws[kWsAT + t * kQkv * kPin + f] : ws[kWsC + t * kQkv + f - kQkv * kPin];
    }
    EFAccM ef;
    ef2_zero(ef);
    const int iters = (B + kMRows - 1) / kMRows;
    const int tok = threadIdx.x & 31, hs = 2 * wave + ((threadIdx.x >> 5) & 1);
    for (int it = blockIdx.x; it < iters; it += gridDim.x) {
        const int row0 = it * kMRows;
        const int nrow = min(kMRows, B - row0);
        __syncthreads();  // previous iteration's reduction readers are done
        // ---- phase 1: lane (half h, token t) forms q|k|v of token t of sample 2 wave + h ----
        float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (hs < nrow) {
            float4* q = reinterpret_cast<float4*>(sm + hs * kMSample + tok * kQp);
            if (tok < kTok) {
                xv = xslice(x + (size_t)(row0 + hs) * ldx, tok, parity != 0);
                float o[kQkv];
#ifdef FRONT_DIAG_NO_P1LOAD  // timing diagnostic (wrong results): no folded-map table loads
#pragma unroll
                for (int r = 0; r < kQkv; r++) o[r] = xv.x * (r + 1) + xv.y;
#else
                affine4t<kQkv>(tab + tok * kTabS, tab + tok * kTabS + kQkv * kPin, xv, o);
#endif
                // q | k: the two halves of each float4 trade places on swizzled rows (see qk_sw): two 8-byte
                // writes at swapped offsets, no value selects
                float2* q2 = reinterpret_cast<float2*>(q);
                const int x = qk_sw(tok) >> 1, y = x ^ 1;
                q2[0 + x] = make_float2(o[0], o[1]), q2[0 + y] = make_float2(o[2], o[3]);
                q2[2 + x] = make_float2(o[4], o[5]), q2[2 + y] = make_float2(o[6], o[7]);
                q2[4 + x] = make_float2(o[8], o[9]), q2[4 + y] = make_float2(0.f, 0.f);
                q2[6 + x] = make_float2(o[10], o[11]), q2[6 + y] = make_float2(o[12], o[13]);
                q2[8 + x] = make_float2(o[14], o[15]), q2[8 + y] = make_float2(o[16], o[17]);
                q2[10 + x] = make_float2(o[18], o[19]), q2[10 + y] = make_float2(0.f, 0.f);
#pragma unroll
                for (int c = 0; c < kEmb / 4; c++)
                    q[6 + c] = make_float4(o[20 + 4 * c], o[21 + 4 * c], o[22 + 4 * c], o[23 + 4 * c]);
            }
        }
        wave_sync();
#ifndef FRONT_HALF_UNROLL  // 2: both samples' chains in one body (156 VGPRs) measured 1% slower
#define FRONT_HALF_UNROLL 1
#endif
#pragma unroll FRONT_HALF_UNROLL
        for (int half = 0; half < 2; half++) {
            const int slot = 2 * wave + half;
            if (slot >= nrow) break;  // wave-uniform
            // lane indices recomputed per sample behind an opaque copy (no hoisted, spilled lane addresses)
            int lane = threadIdx.x & 63;
            asm volatile("" : "+v"(lane));
            const int c16 = lane & 15, q4 = (lane >> 4) & 3;
            const float* dhr = dh + (size_t)(row0 + slot) * kRowF;
            float* my = sm + slot * kMSample;
            const float* QKV = my;
            float4 df[2];
            float dt[2];
#if defined(FRONT_DIAG_NO_DH)  // timing diagnostic (wrong results): no dh loads for dP
            df[0] = df[1] = make_float4(1.f, 2.f, 3.f, 4.f), dt[0] = dt[1] = 1.f;
#else
            dp_operands(dh, row0 + slot, c16, q4, df, dt);
#endif
            front_prio(0);
            // ---- S^T = K Q^T: tiles [J][I]; k = a = q4 + 4 e, three steps over a < 12 (d_k 10: a = 10, 11
            // read the zero pads) ----
            f32x4_t S[2][2];
            {
                float kf[2][3], qf[2][3];
#pragma unroll
                for (int t = 0; t < 2; t++)
#pragma unroll
                    for (int e = 0; e < 3; e++) {
                        const int qx = q4 ^ qk_sw(c16);  // rows 16 t + c16: bit 3 is c16's; (k ^ x) = 4 (k >> 2) + (q4 ^ x)
                        kf[t][e] = QKV[(16 * t + c16) * kQp + kKO + 4 * e + qx];
                        qf[t][e] = QKV[(16 * t + c16) * kQp + kQO + 4 * e + qx];
                    }
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int I = 0; I < 2; I++) {
                        f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int e = 0; e < 3; e++) acc = mfma4(kf[J][e], qf[I][e], acc);
                        S[J][I] = acc;
                    }
            }
            // ---- dP^T = V dctx^T; k = c: 4 q4 + e (c < 16, float4 operands), then 16 + q4 ----
            f32x4_t dP[2][2];
            {
                float4 vf[2];
                float vt[2];
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    const int r = 16 * t + c16;
                    vf[t] = *reinterpret_cast<const float4*>(QKV + r * kQp + kVO + 4 * q4);
                    vt[t] = QKV[r * kQp + kVO + 16 + q4];
                }
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int I = 0; I < 2; I++) {
                        f32x4_t acc = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int e = 0; e < 4; e++) acc = mfma4(f4at(vf[J], e), f4at(df[I], e), acc);
                        dP[J][I] = mfma4(vt[J], dt[I], acc);
                    }
            }
            // operands of dK (B: q of rows i = kh_row(s, q4), column c16) and dQ^T (A: k of rows j = kh_row(s, q4),
            // column c16; 0 for the padding token 23, whose dS^T row in T is never written), from the zero pads for
            // c16 >= 10; read before the QKV words are reused
            float qb[kKH], ka[kKH];
            {
                const int ca = min(c16, kKq);
#pragma unroll
                for (int s = 0; s < kKH; s++) {
                    // rows kh_row(s, q4): bit 3 is q4's bit 1 for s < 4, 0 for s >= 4 (rows 16-23)
                    const int r = kh_row(s, q4), cx = s < 4 ? ca ^ qk_sw(4 * q4) : ca;
                    qb[s] = QKV[r * kQp + kQO + cx];
                    ka[s] = r < kTok ? QKV[r * kQp + kKO + cx] : 0.f;
                }
            }
            // ---- softmax over j per query column i, then dS^T = P (dP - rowsum(P dP)) / sqrt(10) in place
            // of dP^T; padding rows j (k = 0, so S = 0) are kept out of the max and the sum.  exp2 / rcp
            // (~1 ulp) by default; FRONT_MFMA_FAST_SOFTMAX=0 takes the reference's rounding steps (x /
            // sqrt(10), expf, 1 / sum, as k_front_bwd) -- the gradients' distance to fp64 is the same ----
            front_prio(1);
#pragma unroll
            for (int I = 0; I < 2; I++) {
                float mx = -INFINITY;
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int g = 0; g < 4; g++) {
#if !FRONT_MFMA_FAST_SOFTMAX
                        S[J][I][g] = div_sqrt_kq(S[J][I][g]);
#endif
                        if (16 * J + 4 * q4 + g < kTok) mx = fmaxf(mx, S[J][I][g]);
                    }
                mx = xq_max(mx);
                float sum = 0.f;
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int g = 0; g < 4; g++) {
#if FRONT_MFMA_FAST_SOFTMAX
                        float e = __builtin_amdgcn_exp2f((S[J][I][g] - mx) * kLog2eRsqrtKq);
#else
                        float e = expf(S[J][I][g] - mx);
#endif
                        e = 16 * J + 4 * q4 + g < kTok ? e : 0.f;
                        S[J][I][g] = e;
                        sum += e;
                    }
                // P = 0 in the padding columns i (their dctx rows are not read as zeros below)
#if FRONT_MFMA_FAST_SOFTMAX
                const float inv = 16 * I + c16 < kTok ? __builtin_amdgcn_rcpf(xq_sum(sum)) : 0.f;
#else
                const float inv = 16 * I + c16 < kTok ? 1.f / xq_sum(sum) : 0.f;
#endif
                float rs = 0.f;
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int g = 0; g < 4; g++) {
                        const float p = S[J][I][g] * inv;
                        S[J][I][g] = p;
                        rs = fmaf(dP[J][I][g], p, rs);
                    }
                rs = xq_sum(rs);
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int g = 0; g < 4; g++)
#if FRONT_MFMA_FAST_SOFTMAX
                        dP[J][I][g] = (S[J][I][g] * (dP[J][I][g] - rs)) * kRSqrtKq;
#else
                        dP[J][I][g] = div_sqrt_kq(S[J][I][g] * (dP[J][I][g] - rs));
#endif
            }
            f32x4_t (&P)[2][2] = S;
            f32x4_t (&dS)[2][2] = dP;
            front_prio(0);
            wave_sync();  // the QKV words are dead: the transpose buffer
            // T [i][j] (query-major, rows i < 24, pitch kTp): a C tile's four registers g are consecutive j, so a
            // lane stores them as one 16-byte write (P and dS are 0 in the padding rows and columns)
            float* T = my;
            // ---- dV = P^T dctx: rows j, columns c (20 -> 32); k = i = kh_row(s, q4) ----
#pragma unroll
            for (int I = 0; I < 2; I++)
                if (16 * I + c16 < 24)
#pragma unroll
                    for (int J = 0; J < 2; J++)
                        t_store(T + (16 * I + c16) * kTp + 16 * J + 4 * q4, P[J][I], t_sw(c16));
            wave_sync();
            f32x4_t dV[2][2];
#pragma unroll
            for (int J = 0; J < 2; J++)
#pragma unroll
                for (int C = 0; C < 2; C++) dV[J][C] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < kKH; s++) {
                // k = i = kh_row(s, q4): P^T rows j, column i; dctx rows i (P^T is 0 in the columns i >= 23, whose
                // clamped rows are finite; columns c >= 20 repeat column 19: those dV columns are not kept)
                const int i = kh_row(s, q4);
                float pa[2];
#pragma unroll
                for (int J = 0; J < 2; J++) pa[J] = T[i * kTp + 16 * J + t_col(s, c16, q4)];
                const float* dr = dhr + min(i, kTok - 1) * kEmb;
                const float db[2] = {dr[c16], dr[min(16 + c16, kEmb - 1)]};
#pragma unroll
                for (int J = 0; J < 2; J++)
#pragma unroll
                    for (int C = 0; C < 2; C++) dV[J][C] = mfma4(pa[J], db[C], dV[J][C]);
            }
            wave_sync();  // P^T reads done: dS^T into the same buffer
#pragma unroll
            for (int I = 0; I < 2; I++)
                if (16 * I + c16 < 24)
#pragma unroll
                    for (int J = 0; J < 2; J++)
                        t_store(T + (16 * I + c16) * kTp + 16 * J + 4 * q4, dS[J][I], t_sw(c16));
            wave_sync();
            // ---- dK = dS^T Q: rows j, columns a (10 of 16); k = i = kh_row(s, q4) ----
            // ---- dQ^T = K^T dS^T: rows a = 4 q4 + g (10 of 16), columns i; k = j = kh_row(s, q4): B = dS^T rows
            // j from T (six steps over j < 24 instead of eight over the accumulator tiles' j < 32) ----
            f32x4_t dK[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
            f32x4_t dQ[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int s = 0; s < kKH; s++) {
                const int i = kh_row(s, q4);
#pragma unroll
                for (int J = 0; J < 2; J++) dK[J] = mfma4(T[i * kTp + 16 * J + t_col(s, c16, q4)], qb[s], dK[J]);
#pragma unroll
                for (int I = 0; I < 2; I++) {  // (query rows i >= 24 hold other words: their dQ columns are not kept)
                    // word (row, i ^ L(row)): rows 16 I + c16 (L is c16's); i = 4 q4 + s (s < 4: the row base is a
                    // multiple of 4, so the XOR applies to the whole index) or 16 + 4 (s - 4) + q4
                    const int rb = (16 * I + c16) * kTp;
                    const float tv = s < 4 ? T[(rb + 4 * q4 + t_sw(c16)) ^ s] : T[rb + 16 + 4 * (s - 4) + (q4 ^ t_sw(c16))];
                    dQ[I] = mfma4(ka[s], tv, dQ[I]);
                }
            }
            front_prio(2);
            wave_sync();  // T is dead: the reduction operands G = [dq | dk | dv] and dctx
#pragma unroll
            for (int I = 0; I < 2; I++) {  // dq rows a = 4 q4 .. 4 q4 + 3 of token i: one 16-byte write (a = 10, 11
                                            // are 0 -- k's zero pad -- and rewritten with dk below)
                const int i = 16 * I + c16;
                if (i < kTok && q4 < 3)
                    *reinterpret_cast<float4*>(my + kMG + i * kQkv + 4 * q4) =
                        make_float4(dQ[I][0], dQ[I][1], dQ[I][2], dQ[I][3]);
            }
#pragma unroll
            for (int J = 0; J < 2; J++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int j = 16 * J + 4 * q4 + g;
                    if (j < kTok) {
                        if (c16 < kKq) my[kMG + j * kQkv + kKq + c16] = dK[J][g];
#pragma unroll
                        for (int C = 0; C < 2; C++)
                            if (16 * C + c16 < kEmb) my[kMG + j * kQkv + 2 * kKq + 16 * C + c16] = dV[J][C][g];
                    }
                }
        }
        float4 fp[kEFPf];
        ef2_prefetch(dh + (size_t)row0 * kRowF, nrow, 0, fp);
        // the X rows (the reduction's x operand; phase 1's lanes hold them), now that both samples' QKV words are dead
        if (hs < nrow && tok < kTok) *reinterpret_cast<float4*>(sm + hs * kMSample + kMX + tok * kPin) = xv;
        __syncthreads();
#ifndef FRONT_DIAG_NO_EF  // timing diagnostic (wrong results): no E/F accumulation
        ef2_accumulate<kMSample, kMG, kMX>(sm, dh + (size_t)row0 * kRowF, nrow, fp, ef);
#endif
    }
    ef2_write(partial, ef);
}

// sum of the partial rows: workgroup = 64 columns x 16 row classes (r mod 16);
// each thread sums its class in row order, then the 16 class sums are added in
// class order (fixed order: deterministic).  In fp64: the parameter gradients
// are differences of these sums (dbp_i = f_i + Wqkv^T e_i nearly cancels under
// quirk Q1, where every row of a feature sees the same few inputs), so their
// rounding must stay far below the gradients' own size.
constexpr int kSumCols = 64, kSumClasses = 16;

__global__ __launch_bounds__(kSumCols * kSumClasses) void k_front_sum(const float* __restrict__ partial, int rows,
                                                                      double* __restrict__ red) {
    __shared__ double acc_s[kSumClasses][kSumCols];
    const int c = threadIdx.x % kSumCols, k = threadIdx.x / kSumCols;
    const int e = blockIdx.x * kSumCols + c;
    double acc = 0.0;
    if (e < kPartLen) {  // 8 rows' loads in flight per batch; the additions in row order (as one row at a time)
        int r = k;
        for (; r + 7 * kSumClasses < rows; r += 8 * kSumClasses) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; i++) v[i] = partial[(size_t)(r + i * kSumClasses) * kPartLen + e];
#pragma unroll
            for (int i = 0; i < 8; i++) acc += (double)v[i];
        }
        for (; r < rows; r += kSumClasses) acc += (double)partial[(size_t)r * kPartLen + e];
    }
    acc_s[k][c] = acc;
    __syncthreads();
    if (k == 0 && e < kPartLen) {
        double t = 0.0;
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
__global__ __launch_bounds__(256) void k_front_combine(const float* __restrict__ ws, const double* __restrict__ red,
                                                       float* __restrict__ grad, FrontGradPtrs dst) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGradLen) return;
    auto put = [&](double vd) {
        const float v = (float)vd;
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
        double acc = 0.0;
        for (int tk = 0; tk < kTok; tk++) {
            const float* Wp = ws + kWsWP + (tk * kEmb + c) * kPin;  // Wp_i[c][0..3] (zero beyond d_i)
            const double* E = red + kPEF + (tk * kGd + r) * kPin;   // E_i[r][0..3]
#pragma unroll
            for (int a = 0; a < kPin; a++) acc = fma(E[a], (double)Wp[a], acc);
            acc = fma(red[kPef + tk * kGd + r], (double)ws[kWsBP + tk * kEmb + c], acc);  // e_i[r] b_i[c]
        }
        put(acc);
    } else if (e < kGB) {
        const int f = e - kGP, tk = f / (kEmb * kPin), c = (f / kPin) % kEmb, k = f % kPin;
        double acc = red[kPEF + (tk * kGd + kQkv + c) * kPin + k];  // F_i[c][k]
        for (int r = 0; r < kQkv; r++) acc = fma((double)W[r * kEmb + c], red[kPEF + (tk * kGd + r) * kPin + k], acc);
        put(acc);
    } else {
        const int f = e - kGB, tk = f / kEmb, c = f % kEmb;
        double acc = red[kPef + tk * kGd + kQkv + c];  // f_i[c]
        for (int r = 0; r < kQkv; r++) acc = fma((double)W[r * kEmb + c], red[kPef + tk * kGd + r], acc);
        put(acc);
    }
}

}  // namespace mm

using namespace mm;

extern "C" int mm_actor_front_ws_len(void) { return kWsLen; }
extern "C" int mm_actor_front_grad_len(void) { return kGradLen; }
static int cu_count() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 256;
    return cus[dev];
}

extern "C" int mm_actor_front_partial_len(void) { return kPartLen; }

// the persistent grid of the backward for B samples: every workgroup resident at once (MFMA kernel: kMRows
// samples per iteration, kMPerCU workgroups per CU; VALU kernel: 8 samples, two per CU)
extern "C" int mm_actor_front_bwd_grid(int B, int algo) {
    if (B < 0 || (algo != MM_FRONT_BWD_MFMA && algo != MM_FRONT_BWD_VALU)) return MM_E_ARG;
    const int rows = algo == MM_FRONT_BWD_MFMA ? kMRows : kBwdRows;
    const int per_cu = algo == MM_FRONT_BWD_MFMA ? kMPerCU : 2;
    const int groups = (B + rows - 1) / rows;
    const int cap = per_cu * cu_count();
    return groups < 1 ? 1 : (groups < cap ? groups : cap);
}

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


extern "C" int mm_actor_front_fwd_ex(const float* ws, const float* x, int ldx, int B, int parity, float* h,
                                     int algo, void* stream) {
    if (!ws || !x || !h || B < 0 || ldx < MM_OBS_DIM) return MM_E_ARG;
    if (algo != MM_FRONT_FWD_ROW1 && algo != MM_FRONT_FWD_ROW2 && algo != MM_FRONT_FWD_MFMA) return MM_E_ARG;
    if (B == 0) return 0;
    if (algo == MM_FRONT_FWD_MFMA) {
        const int groups = (B + kFMRows - 1) / kFMRows;
        const int cap = FRONT_FM_WAVES * cu_count();  // workgroups per CU = waves per SIMD (48 KB of LDS each)
        const int grid = groups < cap ? groups : cap;
        hipLaunchKernelGGL(k_front_fwd_mfma<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B,
                           parity, (void*)h);
    } else if (algo == MM_FRONT_FWD_ROW2) {
        const int groups = (B + kF2Rows - 1) / kF2Rows;
        const int grid = groups < 2 * cu_count() ? groups : 2 * cu_count();  // two workgroups per CU (72 KB LDS)
        hipLaunchKernelGGL(k_front_fwd2, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B, parity, h);
    } else {
        const int groups = (B + kFwdRows - 1) / kFwdRows;
        const int grid = groups < 3 * cu_count() ? groups : 3 * cu_count();  // three workgroups per CU
        hipLaunchKernelGGL(k_front_fwd<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B, parity,
                           (void*)h);
    }
    return (int)hipGetLastError();
}

extern "C" int mm_actor_front_fwd_h16_ex(const float* ws, const float* x, int ldx, int B, int parity, void* h,
                                         int algo, void* stream) {
    if (!ws || !x || !h || B < 0 || ldx < MM_OBS_DIM || ((uintptr_t)h & 7)) return MM_E_ARG;
    if (algo != MM_FRONT_FWD_ROW1 && algo != MM_FRONT_FWD_MFMA) return MM_E_ARG;
    if (B == 0) return 0;
    if (algo == MM_FRONT_FWD_MFMA) {
        const int groups = (B + kFMRows - 1) / kFMRows;
        const int cap = FRONT_FM_WAVES * cu_count();
        const int grid = groups < cap ? groups : cap;
        hipLaunchKernelGGL(k_front_fwd_mfma<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B,
                           parity, h);
    } else {
        const int groups = (B + kFwdRows - 1) / kFwdRows;
        const int grid = groups < 3 * cu_count() ? groups : 3 * cu_count();
        hipLaunchKernelGGL(k_front_fwd<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B, parity,
                           h);
    }
    return (int)hipGetLastError();
}

extern "C" int mm_actor_front_fwd_h16(const float* ws, const float* x, int ldx, int B, int parity, void* h,
                                      void* stream) {
    return mm_actor_front_fwd_h16_ex(ws, x, ldx, B, parity, h, MM_FRONT_FWD_ROW1, stream);
}

extern "C" int mm_actor_front_fwd(const float* ws, const float* x, int ldx, int B, int parity, float* h,
                                  void* stream) {
    return mm_actor_front_fwd_ex(ws, x, ldx, B, parity, h, MM_FRONT_FWD_ROW1, stream);
}

static int front_bwd(const float* ws, const float* x, int ldx, int B, int parity, const float* dh, float* partial,
                     int grid, float* red, float* grad, const FrontGradPtrs* dst, int algo, void* stream) {
    if (!ws || !x || !dh || !partial || !red || (!grad && !dst) || B < 0 || ldx < MM_OBS_DIM || grid <= 0)
        return MM_E_ARG;
    if ((uintptr_t)red & 7) return MM_E_ARG;  // red holds the fp64 sums: 2 x mm_actor_front_partial_len() floats
    if (algo != MM_FRONT_BWD_MFMA && algo != MM_FRONT_BWD_VALU) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    double* red64 = reinterpret_cast<double*>(red);
    if (algo == MM_FRONT_BWD_MFMA)
        hipLaunchKernelGGL(k_front_bwd_mfma, dim3(grid), dim3(kMThreads), 0, s, ws, x, ldx, B, parity, dh, partial);
    else
        hipLaunchKernelGGL(k_front_bwd, dim3(grid), dim3(kBwdThreads), 0, s, ws, x, ldx, B, parity, dh, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_front_sum, dim3((kPartLen + kSumCols - 1) / kSumCols), dim3(kSumCols * kSumClasses), 0, s,
                       partial, grid, red64);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    if (grad)
        hipLaunchKernelGGL(k_front_combine<false>, dim3((kGradLen + 255) / 256), dim3(256), 0, s, ws, red64, grad,
                           FrontGradPtrs{});
    else
        hipLaunchKernelGGL(k_front_combine<true>, dim3((kGradLen + 255) / 256), dim3(256), 0, s, ws, red64, nullptr, *dst);
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
