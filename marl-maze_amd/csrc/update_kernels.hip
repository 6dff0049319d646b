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

}  // namespace mm

using namespace mm;

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
