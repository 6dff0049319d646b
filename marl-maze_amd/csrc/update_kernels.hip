// update_kernels.hip -- the small reductions and the optimizer step of the PPO
// update (PPO.py:58-85), so that one minibatch step is a fixed set of
// hand-written launches with no framework glue between them:
//
//   mm_colsum       bias gradients: column sums of the GEMM engine's per-16-row
//                   tile sums (nn.Linear's db = sum_m dY[m, :], networks.py:35-41,
//                   87-106 under autograd)
//   mm_mse_loss     the critic loss nn.MSELoss()(V, rtg) (PPO.py:78-80): per-
//                   workgroup partial sums of (V - rtg)^2 and dV = 2 (V - rtg) / M
//   mm_losses_final the two losses from the partial sums: [actor, critic]
//   mm_clip_adam    clip_grad_norm_(params, max_grad) + Adam.step() per network
//                   (PPO.py:74-85) over flat parameter / gradient / moment buffers
//
// Every sum has a fixed order (deterministic, bit-reproducible run to run).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "marlmaze.h"

namespace mm {

// column sums of a row-major [R, N] f32 matrix.  A workgroup = 64 columns x 4
// row lanes over one slab of rows; each lane sums its rows (stride 4, ascending)
// in two alternating accumulators, the 4 lanes are added in order.
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ x, long R, int N, long rps,
                                                float* __restrict__ out) {
    __shared__ float red[4][64];
    const int rl = threadIdx.x >> 6, c = blockIdx.y * 64 + (threadIdx.x & 63);
    const long r0 = (long)blockIdx.x * rps, r1 = min(R, r0 + rps);
    float a0 = 0.f, a1 = 0.f;
    if (c < N) {
        long r = r0 + rl;
#pragma unroll 4
        for (; r + 4 < r1; r += 8) {
            a0 += x[r * N + c];
            a1 += x[(r + 4) * N + c];
        }
        if (r < r1) a0 += x[r * N + c];
    }
    red[rl][threadIdx.x & 63] = a0 + a1;
    __syncthreads();
    if (rl == 0 && c < N) {
        const int k = threadIdx.x & 63;
        out[(long)blockIdx.x * N + c] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    }
}

// fixed-order tree sum of one value per thread (256 threads); the result in every thread
template <class T>
__device__ __forceinline__ T block_sum256(T v, T* red) {
    red[threadIdx.x] = v;
    __syncthreads();
#pragma unroll
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    const T r = red[0];
    __syncthreads();
    return r;
}

constexpr int kMseThreads = 256;

// (V - rtg)^2 partial sums per workgroup and dV = (V - rtg) * (2 / M): torch's
// mse_loss backward (grad = (input - target) * norm, norm = 2 / numel)
__global__ __launch_bounds__(kMseThreads) void k_mse_loss(const float* __restrict__ v, const float* __restrict__ rtg,
                                                          int M, float norm, float* __restrict__ dv,
                                                          float* __restrict__ partial) {
    __shared__ float red[kMseThreads];
    const int i = blockIdx.x * kMseThreads + threadIdx.x;
    float sq = 0.f;
    if (i < M) {
        const float d = v[i] - rtg[i];
        sq = d * d;
        if (dv) dv[i] = d * norm;
    }
    const float s = block_sum256(sq, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// out[0] = -sum(ppo partials) / M (the actor loss), out[1] = sum(mse partials) / M
__global__ __launch_bounds__(256) void k_losses_final(const float* __restrict__ pp, int npp,
                                                      const float* __restrict__ mp, int nmp, int M,
                                                      float* __restrict__ out) {
    __shared__ float red[256];
    float a = 0.f, c = 0.f;
    for (int j = threadIdx.x; j < npp; j += 256) a += pp[j];
    for (int j = threadIdx.x; j < nmp; j += 256) c += mp[j];
    a = block_sum256(a, red);
    c = block_sum256(c, red);
    if (threadIdx.x == 0) {
        out[0] = -a / (float)M;
        out[1] = c / (float)M;
    }
}

// ---- clip_grad_norm_ + Adam ----
constexpr int kMaxSeg = 4;
constexpr int kNormBlocks = 64;  // partial sums of squares per segment

struct AdamSegs {
    mm_adam_seg_t s[kMaxSeg];
};

// sum of squares of each segment's gradient in kNormBlocks fp64 partials (grid (kNormBlocks, nseg))
__global__ __launch_bounds__(256) void k_gnorm_partial(AdamSegs segs, double* __restrict__ ws) {
    __shared__ double red[256];
    const mm_adam_seg_t& sg = segs.s[blockIdx.y];
    double acc = 0.0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < sg.n; i += (long)kNormBlocks * 256) {
        const double g = (double)(sg.grad[i] * sg.grad_scale);
        acc += g * g;
    }
    acc = block_sum256(acc, red);
    if (threadIdx.x == 0) ws[blockIdx.y * kNormBlocks + blockIdx.x] = acc;
}

// grid (X, nseg): each workgroup reduces its segment's partials (fixed order), forms
// clip_grad_norm_'s coefficient min(1, max_norm / (norm + 1e-6)) and runs Adam
// (torch's single-tensor rule: exp_avg.lerp_(g, 1 - b1); exp_avg_sq * b2 +
// (1 - b2) g g; p -= step_size exp_avg / (sqrt(exp_avg_sq) / sqrt(bc2) + eps))
// on its elements with the clipped gradient
__global__ __launch_bounds__(256) void k_clip_adam(AdamSegs segs, const double* __restrict__ ws, float beta1,
                                                   float beta2, float eps, float* __restrict__ norms) {
    __shared__ double red[256];
    const mm_adam_seg_t& sg = segs.s[blockIdx.y];
    const double part = threadIdx.x < kNormBlocks ? ws[blockIdx.y * kNormBlocks + threadIdx.x] : 0.0;
    const double tot = block_sum256(part, red);
    const float norm = (float)sqrt(tot);
    float coef = 1.f;
    if (sg.max_norm > 0.f) coef = fminf(sg.max_norm / (norm + 1e-6f), 1.f);
    if (blockIdx.x == 0 && threadIdx.x == 0 && norms) norms[blockIdx.y] = norm;
    const float omb1 = 1.f - beta1, omb2 = 1.f - beta2, ss = sg.step_size, bc2 = sg.bc2_sqrt;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < sg.n; i += (long)gridDim.x * 256) {
        const float g = (sg.grad[i] * sg.grad_scale) * coef;
        float m = sg.exp_avg[i];
        m = m + omb1 * (g - m);
        float v = sg.exp_avg_sq[i];
        v = v * beta2 + (omb2 * g) * g;
        const float denom = sqrtf(v) / bc2 + eps;
        sg.exp_avg[i] = m;
        sg.exp_avg_sq[i] = v;
        sg.param[i] = sg.param[i] + (-ss) * (m / denom);
    }
}

// ---- several reductions in one launch (the update's bias gradients and weight-gradient partials
// are reduced together at the end of a backward: per-launch latency, not bandwidth, is their cost) ----
constexpr int kMaxMulti = 16;
struct ColsumSegs {
    mm_colsum_seg_t s[kMaxMulti];
    int G[kMaxMulti];          // slabs
    long rps[kMaxMulti];       // rows per slab
    int blk1[kMaxMulti + 1];   // pass-1 workgroup prefix (G x column blocks)
    int blk2[kMaxMulti + 1];   // pass-2 workgroup prefix (column blocks)
    long woff[kMaxMulti];      // partials offset in ws (floats)
    int nseg;
};

// one workgroup of k_colsum's body: rows r0 .. r1 of x [R, N], columns 64 cb .. (fixed order, as k_colsum)
__device__ __forceinline__ void colsum_block(const float* __restrict__ x, long r0, long r1, int N, int cb,
                                             float* __restrict__ out, float (*red)[64]) {
    const int rl = threadIdx.x >> 6, c = cb * 64 + (threadIdx.x & 63);
    float a0 = 0.f, a1 = 0.f;
    if (c < N) {
        long r = r0 + rl;
#pragma unroll 4
        for (; r + 4 < r1; r += 8) {
            a0 += x[r * N + c];
            a1 += x[(r + 4) * N + c];
        }
        if (r < r1) a0 += x[r * N + c];
    }
    red[rl][threadIdx.x & 63] = a0 + a1;
    __syncthreads();
    if (rl == 0 && c < N) {
        const int k = threadIdx.x & 63;
        out[c] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    }
}

__device__ __forceinline__ int seg_of(const int* pre, int nseg, int b) {
    int k = 0;
    while (k + 1 < nseg && b >= pre[k + 1]) k++;
    return k;
}

__global__ __launch_bounds__(256) void k_colsum_multi1(ColsumSegs cs, float* __restrict__ ws) {
    __shared__ float red[4][64];
    const int k = seg_of(cs.blk1, cs.nseg, blockIdx.x);
    const mm_colsum_seg_t& sg = cs.s[k];
    const int b = blockIdx.x - cs.blk1[k], G = cs.G[k];
    const int slab = b % G, cb = b / G;
    const long r0 = slab * cs.rps[k], r1 = min(sg.R, r0 + cs.rps[k]);
    colsum_block(sg.x, r0, r1, sg.N, cb, ws + cs.woff[k] + (long)slab * sg.N, red);
}

__global__ __launch_bounds__(256) void k_colsum_multi2(ColsumSegs cs, const float* __restrict__ ws) {
    __shared__ float red[4][64];
    const int k = seg_of(cs.blk2, cs.nseg, blockIdx.x);
    const mm_colsum_seg_t& sg = cs.s[k];
    colsum_block(ws + cs.woff[k], 0, cs.G[k], sg.N, blockIdx.x - cs.blk2[k], sg.out, red);
}

struct WsumSegs {
    mm_wsum_seg_t s[kMaxMulti];
    int blk[kMaxMulti + 1];  // workgroup prefix: ceil(n / 16) each
    int nseg;
};

// out[e] = sum over s of x[s * n + e]: 16 groups of slices, each summed in order, then the groups in order
// (the order of csrc/x3mlp.hip's k_wg_reduce: identical results)
__global__ __launch_bounds__(256) void k_wsum_multi(WsumSegs ws) {
    __shared__ float red[16][17];
    const int k = seg_of(ws.blk, ws.nseg, blockIdx.x);
    const mm_wsum_seg_t& sg = ws.s[k];
    const int el = threadIdx.x & 15, g = threadIdx.x >> 4;
    const long e = (blockIdx.x - ws.blk[k]) * 16L + el, n = sg.n;
    const int S = sg.S, per = (S + 15) / 16, s0 = g * per, s1 = min(S, s0 + per);
    float a = 0.f;
    if (e < n) {
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = s0 + i < s1 ? sg.x[(long)(s0 + i) * n + e] : 0.f;
#pragma unroll
        for (int i = 0; i < 16; i++) a += v[i];
        for (int t = s0 + 16; t < s1; t++) a += sg.x[(long)t * n + e];  // S > 256
    }
    red[g][el] = a;
    __syncthreads();
    if (g == 0 && e < n) {
        float t = red[0][el];
#pragma unroll
        for (int q = 1; q < 16; q++) t += red[q][el];
        sg.out[e] = t;
    }
}

// k_wsum_multi with 4 consecutive elements per lane (16-byte loads: a wave reads 4 slices x 256 contiguous
// bytes per instruction instead of 4 x 64) for segments whose n is a multiple of 4 on 16-byte aligned
// partials; per element the same additions in the same order (bit-identical)
__global__ __launch_bounds__(256) void k_wsum_multi4(WsumSegs ws) {
    __shared__ float4 red[16][16];
    const int k = seg_of(ws.blk, ws.nseg, blockIdx.x);
    const mm_wsum_seg_t& sg = ws.s[k];
    const int el = threadIdx.x & 15, g = threadIdx.x >> 4;
    const long e = ((blockIdx.x - ws.blk[k]) * 16L + el) * 4, n = sg.n;
    const int S = sg.S, per = (S + 15) / 16, s0 = g * per, s1 = min(S, s0 + per);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < n) {
        float4 v[16];
#pragma unroll
        for (int i = 0; i < 16; i++)
            v[i] = s0 + i < s1 ? *reinterpret_cast<const float4*>(sg.x + (long)(s0 + i) * n + e)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < 16; i++) a.x += v[i].x, a.y += v[i].y, a.z += v[i].z, a.w += v[i].w;
        for (int t = s0 + 16; t < s1; t++) {  // S > 256
            const float4 u = *reinterpret_cast<const float4*>(sg.x + (long)t * n + e);
            a.x += u.x, a.y += u.y, a.z += u.z, a.w += u.w;
        }
    }
    red[g][el] = a;
    __syncthreads();
    if (g == 0 && e < n) {
        float4 t = red[0][el];
#pragma unroll
        for (int q = 1; q < 16; q++) t.x += red[q][el].x, t.y += red[q][el].y, t.z += red[q][el].z, t.w += red[q][el].w;
        *reinterpret_cast<float4*>(sg.out + e) = t;
    }
}

}  // namespace mm

using namespace mm;

static bool colsum_plan(const mm_colsum_seg_t* segs, int nseg, ColsumSegs& cs, long& wlen) {
    if (!segs || nseg <= 0 || nseg > kMaxMulti) return false;
    cs.nseg = nseg;
    cs.blk1[0] = cs.blk2[0] = 0;
    wlen = 0;
    for (int k = 0; k < nseg; k++) {
        const mm_colsum_seg_t& g = segs[k];
        if (!g.x || !g.out || g.R <= 0 || g.N <= 0) return false;
        cs.s[k] = g;
        long G = g.R / 8;  // slabs of >= 8 rows, at most 256 (as marlmaze.x3.colsum)
        G = G < 1 ? 1 : G > 256 ? 256 : G;
        const long rps = (g.R + G - 1) / G;
        cs.G[k] = (int)((g.R + rps - 1) / rps);
        cs.rps[k] = rps;
        const int cb = (g.N + 63) / 64;
        cs.blk1[k + 1] = cs.blk1[k] + cs.G[k] * cb;
        cs.blk2[k + 1] = cs.blk2[k] + cb;
        cs.woff[k] = wlen;
        wlen += (long)cs.G[k] * g.N;
    }
    return true;
}

extern "C" long mm_colsum_multi_ws_len(const mm_colsum_seg_t* segs, int nseg) {
    ColsumSegs cs;
    long wlen;
    return colsum_plan(segs, nseg, cs, wlen) ? wlen : MM_E_ARG;
}

extern "C" int mm_colsum_multi(const mm_colsum_seg_t* segs, int nseg, float* ws, void* stream) {
    ColsumSegs cs;
    long wlen;
    if (!colsum_plan(segs, nseg, cs, wlen) || !ws) return MM_E_ARG;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_colsum_multi1, dim3(cs.blk1[nseg]), dim3(256), 0, st, cs, ws);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_colsum_multi2, dim3(cs.blk2[nseg]), dim3(256), 0, st, cs, (const float*)ws);
    return (int)hipGetLastError();
}

extern "C" int mm_wsum_multi(const mm_wsum_seg_t* segs, int nseg, void* stream) {
    if (!segs || nseg <= 0 || nseg > kMaxMulti) return MM_E_ARG;
    WsumSegs w;
    w.nseg = nseg;
    w.blk[0] = 0;
    bool v4 = true;  // every segment n % 4 == 0 with 16-byte aligned partials and output
    for (int k = 0; k < nseg; k++) {
        if (!segs[k].x || !segs[k].out || segs[k].S <= 0 || segs[k].n <= 0) return MM_E_ARG;
        v4 = v4 && !(segs[k].n & 3) && !((uintptr_t)segs[k].x & 15) && !((uintptr_t)segs[k].out & 15);
    }
    for (int k = 0; k < nseg; k++) {
        w.s[k] = segs[k];
        w.blk[k + 1] = w.blk[k] + (int)((segs[k].n + (v4 ? 63 : 15)) / (v4 ? 64 : 16));
    }
    if (v4)
        hipLaunchKernelGGL(k_wsum_multi4, dim3(w.blk[nseg]), dim3(256), 0, (hipStream_t)stream, w);
    else
        hipLaunchKernelGGL(k_wsum_multi, dim3(w.blk[nseg]), dim3(256), 0, (hipStream_t)stream, w);
    return (int)hipGetLastError();
}

extern "C" int mm_colsum(const float* x, long R, int N, float* part, int G, float* out, void* stream) {
    if (!x || !out || R <= 0 || N <= 0 || G <= 0 || (G > 1 && !part)) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    const int cb = (N + 63) / 64;
    if (G > R) G = (int)R;
    if (G == 1) {
        hipLaunchKernelGGL(k_colsum, dim3(1, cb), dim3(256), 0, s, x, R, N, R, out);
        return (int)hipGetLastError();
    }
    const long rps = (R + G - 1) / G;
    const int g = (int)((R + rps - 1) / rps);  // slabs actually holding rows
    hipLaunchKernelGGL(k_colsum, dim3(g, cb), dim3(256), 0, s, x, R, N, rps, part);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_colsum, dim3(1, cb), dim3(256), 0, s, (const float*)part, (long)g, N, (long)g, out);
    return (int)hipGetLastError();
}

extern "C" int mm_mse_loss_partials(int M) { return (M + kMseThreads - 1) / kMseThreads; }

extern "C" int mm_mse_loss(const float* v, const float* rtg, int M, float* dv, float* partial, void* stream) {
    if (!v || !rtg || !partial || M <= 0) return MM_E_ARG;
    hipLaunchKernelGGL(k_mse_loss, dim3(mm_mse_loss_partials(M)), dim3(kMseThreads), 0, (hipStream_t)stream, v, rtg,
                       M, (float)(2.0 / (double)M), dv, partial);
    return (int)hipGetLastError();
}

extern "C" int mm_losses_final(const float* ppo_partial, int n_ppo, const float* mse_partial, int n_mse, int M,
                               float* out, void* stream) {
    if (!ppo_partial || !mse_partial || !out || n_ppo <= 0 || n_mse <= 0 || M <= 0) return MM_E_ARG;
    hipLaunchKernelGGL(k_losses_final, dim3(1), dim3(256), 0, (hipStream_t)stream, ppo_partial, n_ppo, mse_partial,
                       n_mse, M, out);
    return (int)hipGetLastError();
}

extern "C" long mm_clip_adam_ws_len(int nseg) { return (long)nseg * kNormBlocks * 2; }

extern "C" int mm_clip_adam(const mm_adam_seg_t* segs, int nseg, float beta1, float beta2, float eps, float* ws,
                            float* norms, void* stream) {
    if (!segs || nseg <= 0 || nseg > kMaxSeg || !ws || ((uintptr_t)ws & 7)) return MM_E_ARG;
    AdamSegs a{};
    long nmax = 0;
    for (int k = 0; k < nseg; k++) {
        const mm_adam_seg_t& s = segs[k];
        if (s.n < 0 || (s.n > 0 && (!s.param || !s.grad || !s.exp_avg || !s.exp_avg_sq)) || !(s.bc2_sqrt > 0.f) ||
            !(s.grad_scale > 0.f))
            return MM_E_ARG;
        a.s[k] = s;
        nmax = s.n > nmax ? s.n : nmax;
    }
    if (nmax == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    double* wsd = reinterpret_cast<double*>(ws);
    hipLaunchKernelGGL(k_gnorm_partial, dim3(kNormBlocks, nseg), dim3(256), 0, st, a, wsd);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    // about 4 elements per thread of the largest segment, at most 1,024 workgroups per segment
    long blocks = (nmax + 1023) / 1024;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_clip_adam, dim3((unsigned)blocks, nseg), dim3(256), 0, st, a, (const double*)wsd, beta1,
                       beta2, eps, norms);
    return (int)hipGetLastError();
}
