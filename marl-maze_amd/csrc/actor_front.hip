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
// Workspace (k_front_prep): [Wp 23x20x4 | bp 23x20 | A 23x40x4 | c 23x40 | Wqkv 40x20]
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
constexpr int kWsLen = kWsW + kQkv * kEmb;         // 7700

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
    return make_float4(xr[s], d > 1 ? xr[s + 1] : 0.f, d > 2 ? xr[s + 2] : 0.f, d > 3 ? xr[s + 3] : 0.f);
}

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
constexpr int kTabF = kQkv * kPin + kQkv + kEmb * kPin + kEmb;  // 300 floats per token: A | c | Wp | bp
// (300 dwords = 75 16-byte quads, odd: a wave's per-token 16-byte reads are bank-conflict free)

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
        if (f < kQkv * kPin) src = kWsA + i * kQkv * kPin + f;
        else if (f < kQkv * kPin + kQkv) src = kWsC + i * kQkv + f - kQkv * kPin;
        else if (f < kQkv * kPin + kQkv + kEmb * kPin) src = kWsWP + i * kEmb * kPin + f - kQkv * (kPin + 1);
        else src = kWsBP + i * kEmb + f - kQkv * (kPin + 1) - kEmb * kPin;
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
            affine4<kQkv>(ti, ti + kQkv * kPin, xv, o);
#pragma unroll
            for (int a = 0; a < kKq; a++) {
                q[a] = o[a];
                Ks[g][i][a] = o[kKq + a];
            }
#pragma unroll
            for (int c = 0; c < kEmb; c++) Vs[g][i][c] = o[2 * kKq + c];
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
            float sum = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                s[j] = expf(s[j] - mx);
                sum += s[j];
            }
            float out[kEmb];
#pragma unroll
            for (int c = 0; c < kEmb; c++) out[c] = 0.f;
            const float inv = 1.f / sum;  // torch's softmax scales by the reciprocal of the sum
#pragma unroll
            for (int j = 0; j < kTok; j++) axpy4<kEmb>(out, s[j] * inv, Vs[g][j]);
            float t[kEmb];
            affine4<kEmb>(ti + kQkv * (kPin + 1), ti + kQkv * (kPin + 1) + kEmb * kPin, xv, t);
            float* o = h + (size_t)row * kRowF + i * kEmb;
#pragma unroll
            for (int c = 0; c < kEmb; c += 4)
                *reinterpret_cast<float4*>(o + c) =
                    make_float4(t[c] + out[c], t[c + 1] + out[c + 1], t[c + 2] + out[c + 2], t[c + 3] + out[c + 3]);
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
constexpr int kEFUnits = kTok * (kGd / 4);           // 345 (token, 4 rows of [g|dctx])

__global__ __launch_bounds__(kBwdThreads, 2) void k_front_bwd(const float* __restrict__ ws,
                                                              const float* __restrict__ x, int ldx, int B,
                                                              int parity, const float* __restrict__ dh,
                                                              float* __restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float sm[kBwdRows * kSampleF];
    const int g = threadIdx.x >> 5;
    const int i = threadIdx.x & 31;
    float* my = sm + g * kSampleF;
    // E/F/e/f: thread t owns units t and t + 256 (token u / 15, rows 4 (u % 15) ..)
    float ae[2][4][4], as[2][4];
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int a = 0; a < 4; a++) ae[u][a][0] = ae[u][a][1] = ae[u][a][2] = ae[u][a][3] = as[u][a] = 0.f;
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
            float sum = 0.f;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = expf(p[j] - mx);
                sum += p[j];
            }
            float dp[kTok];
            float rs = 0.f;
            const float inv = 1.f / sum;
#pragma unroll
            for (int j = 0; j < kTok; j++) {
                p[j] = p[j] * inv;
                dp[j] = dot4<kEmb>(dctx, my + kOffV + j * kEmb);  // dP_ij = dctx_i . v_j
                rs = fmaf(dp[j], p[j], rs);
            }
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
#pragma unroll 4
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
        // phase 4b: E/F (+= [g|dctx] x^T) and e/f (+= [g|dctx]) per token
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int unit = threadIdx.x + u * kBwdThreads;
            if (unit < kEFUnits) {
                const int tk = unit / (kGd / 4), r0 = 4 * (unit % (kGd / 4));
                const int off = r0 < kQkv ? kOffG + tk * kQkv + r0 : kOffD + tk * kEmb + (r0 - kQkv);
                for (int gg = 0; gg < nrow; gg++) {
                    const float* sg = sm + gg * kSampleF;
                    const float4 gv = *reinterpret_cast<const float4*>(sg + off);
                    const float4 xq = *reinterpret_cast<const float4*>(sg + kOffX + tk * kPin);
                    const float gr[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                    for (int a = 0; a < 4; a++) {
                        ae[u][a][0] = fmaf(gr[a], xq.x, ae[u][a][0]);
                        ae[u][a][1] = fmaf(gr[a], xq.y, ae[u][a][1]);
                        ae[u][a][2] = fmaf(gr[a], xq.z, ae[u][a][2]);
                        ae[u][a][3] = fmaf(gr[a], xq.w, ae[u][a][3]);
                        as[u][a] += gr[a];
                    }
                }
            }
        }
    }
    float* out = partial + (size_t)blockIdx.x * kPartLen;
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int unit = threadIdx.x + u * kBwdThreads;
        if (unit < kEFUnits) {
            const int tk = unit / (kGd / 4), r0 = 4 * (unit % (kGd / 4));
#pragma unroll
            for (int a = 0; a < 4; a++) {
                *reinterpret_cast<float4*>(out + kPEF + (tk * kGd + r0 + a) * kPin) =
                    make_float4(ae[u][a][0], ae[u][a][1], ae[u][a][2], ae[u][a][3]);
                out[kPef + tk * kGd + r0 + a] = as[u][a];
            }
        }
    }
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
__global__ __launch_bounds__(256) void k_front_combine(const float* __restrict__ ws, const float* __restrict__ red,
                                                       float* __restrict__ grad) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGradLen) return;
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
        grad[e] = acc;
    } else if (e < kGB) {
        const int f = e - kGP, tk = f / (kEmb * kPin), c = (f / kPin) % kEmb, k = f % kPin;
        float acc = red[kPEF + (tk * kGd + kQkv + c) * kPin + k];  // F_i[c][k]
        for (int r = 0; r < kQkv; r++) acc = fmaf(W[r * kEmb + c], red[kPEF + (tk * kGd + r) * kPin + k], acc);
        grad[e] = acc;
    } else {
        const int f = e - kGB, tk = f / kEmb, c = f % kEmb;
        float acc = red[kPef + tk * kGd + kQkv + c];  // f_i[c]
        for (int r = 0; r < kQkv; r++) acc = fmaf(W[r * kEmb + c], red[kPef + tk * kGd + r], acc);
        grad[e] = acc;
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

extern "C" int mm_actor_front_fwd(const float* ws, const float* x, int ldx, int B, int parity, float* h,
                                  void* stream) {
    if (!ws || !x || !h || B < 0 || ldx < MM_OBS_DIM) return MM_E_ARG;
    if (B == 0) return 0;
    const int groups = (B + kFwdRows - 1) / kFwdRows;
    const int grid = groups < 3 * cu_count() ? groups : 3 * cu_count();  // three workgroups per CU
    hipLaunchKernelGGL(k_front_fwd, dim3(grid), dim3(256), 0, (hipStream_t)stream, ws, x, ldx, B, parity, h);
    return (int)hipGetLastError();
}

extern "C" int mm_actor_front_bwd(const float* ws, const float* x, int ldx, int B, int parity, const float* dh,
                                  float* partial, int grid, float* red, float* grad, void* stream) {
    if (!ws || !x || !dh || !partial || !red || !grad || B < 0 || ldx < MM_OBS_DIM || grid <= 0) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_front_bwd, dim3(grid), dim3(kBwdThreads), 0, s, ws, x, ldx, B, parity, dh, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_front_sum, dim3((kPartLen + kSumCols - 1) / kSumCols), dim3(kSumCols * kSumClasses), 0, s,
                       partial, grid, red);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_front_combine, dim3((kGradLen + 255) / 256), dim3(256), 0, s, ws, red, grad);
    return (int)hipGetLastError();
}
