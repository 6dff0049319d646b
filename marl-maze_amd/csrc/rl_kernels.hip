// rl_kernels.hip -- PPO rollout-side kernels for MI355X (gfx950).
//
//   k_gae     PPO.get_GAEs (PPO.py:193-203) over a time-major [T, N] rollout,
//             one lane per maze column: the reverse recursion is sequential in
//             t by definition, the N columns are independent, and the [T, N]
//             layout makes every step's loads/stores one coalesced row.
//             fp32, no FMA contraction, the reference's operation order:
//               delta_t = (r_t + f32(g*V_{t+1}) * (1-d_{t+1})) - V_t
//               A_t     = delta_t + f32(f32(g*lam) * A_{t+1})   (0 if d_t)
//             (the d_{t+1} mask drops V_{L-1} from delta_{L-2}: quirk Q7).
//   k_sample  PPO.get_action (PPO.py:170-186) for every agent row: masked
//             categorical move + Bernoulli mark, per-agent and joint log-prob,
//             counter-based Philox4x32-10 draws.
//   k_head_sample  the actor's two heads (networks.py:38-41) fused with
//             k_sample's draw: last hidden layer -> actions, log-probs.
//   k_ppo_loss / k_ppo_loss_bwd  the update's policy side (PPO.py:62-72 with
//             get_log_probs PPO.py:154-168): per-agent masked log-softmax of
//             the move logits + masked Bernoulli mark log-prob, joint log-prob,
//             ratio, clipped surrogate and its mean; the backward writes the
//             gradient of the loss w.r.t. the six head logits of each agent
//             row directly (torch's min() splits a tie's gradient in half, as
//             here).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "marlmaze.h"

namespace mm {

__global__ void k_gae(const float* __restrict__ rew, const float* __restrict__ val, const uint8_t* __restrict__ done,
                      const float* __restrict__ last_val, int T, int N, float g, float gl, float* __restrict__ adv,
                      float* __restrict__ rtg) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float a = 0.f;
    // state carried from t+1: value and done flag
    float v_next = last_val ? last_val[i] : 0.f;
    bool have_next = last_val != nullptr;  // false: segment end == episode end
    bool d_next = false;
    for (int t = T - 1; t >= 0; t--) {
        const size_t k = (size_t)t * N + i;
        const float r = rew[k];
        const float v = val[k];
        // without a bootstrap value the segment end IS an episode end (done=1),
        // so the reference's d_{t+1} mask also applies to delta_{T-2} (Q7)
        const bool d = done[k] != 0 || (t == T - 1 && !last_val);
        float delta;
        if (d || !have_next) {
            // the reference's `t+1 == len(ep)` branch: delta = r - V
            delta = __fsub_rn(r, v);
        } else {
            float boot = __fmul_rn(g, v_next);
            if (d_next) boot = __fmul_rn(boot, 0.f);
            delta = __fsub_rn(__fadd_rn(r, boot), v);
        }
        const float scale = d ? 0.f : gl;
        a = __fadd_rn(delta, __fmul_rn(scale, a));
        adv[k] = a;
        if (rtg) rtg[k] = __fadd_rn(a, v);  // b_rtgs = b_advs + b_vals (PPO.py:46)
        v_next = v;
        d_next = d;
        have_next = true;
    }
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// One agent row of PPO.get_action (PPO.py:170-186): masked categorical move,
// Bernoulli mark; returns the per-agent log-prob.  The draws are Philox of
// counter (offset, row): the same row gets the same numbers in k_sample and
// k_head_sample.
__device__ __forceinline__ float sample_row(const float ml[5], float kl, const uint8_t* __restrict__ mk, int row,
                                            uint64_t seed, uint64_t offset, int& move, int& mark) {
    const uint4 rnd = philox(make_uint4((uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)row, 0u),
                             make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    float l[5];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        l[j] = mk[j] ? ml[j] : -INFINITY;  // masked_fill(~mask, -inf)
        mx = fmaxf(mx, l[j]);
    }
    float p[5], sum = 0.f;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        p[j] = mk[j] ? expf(l[j] - mx) : 0.f;
        sum += p[j];
    }
    // inverse-CDF draw over the allowed moves
    const float target = u01(rnd.x) * sum;
    int mv = -1, last = -1;
    float c = 0.f;
#pragma unroll
    for (int j = 0; j < 5; j++) {
        if (!mk[j]) continue;
        last = j;
        c += p[j];
        if (mv < 0 && target < c) mv = j;
    }
    if (mv < 0) mv = last;
    float lp;
    if (mv < 0) {  // no legal move: the reference's Categorical is undefined (NaN)
        mv = 4;
        lp = NAN;
    } else {
        lp = (l[mv] - mx) - logf(sum);  // Categorical.log_prob = logit - logsumexp
    }
    // mark ~ Bernoulli(sigmoid(mark_logit)) if allowed else 0 (PPO.py:179-181)
    int mk5 = 0;
    float pm = 0.f;
    if (mk[5]) {
        pm = 1.f / (1.f + expf(-kl));
        mk5 = u01(rnd.y) < pm ? 1 : 0;
    }
    lp += logf(mk5 ? pm : 1.f - pm);
    move = mv;
    mark = mk5;
    return lp;
}

// One thread per maze: rows 2i (agent 0) and 2i+1 (agent 1).
__global__ void k_sample(const float* __restrict__ ml, const float* __restrict__ kl, const uint8_t* __restrict__ masks,
                         int M, uint64_t seed, uint64_t offset, int8_t* __restrict__ act, float* __restrict__ logp,
                         float* __restrict__ joint) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int nm = (M + 1) / 2;
    if (i >= nm) return;
    float jl = 0.f;
#pragma unroll
    for (int a = 0; a < 2; a++) {
        const int row = 2 * i + a;
        if (row >= M) break;
        float l[5];
#pragma unroll
        for (int j = 0; j < 5; j++) l[j] = ml[(size_t)row * 5 + j];
        int move, mark;
        const float lp = sample_row(l, kl[row], masks + (size_t)row * MM_MASK_DIM, row, seed, offset, move, mark);
        act[2 * row] = (int8_t)move;
        act[2 * row + 1] = (int8_t)mark;
        if (logp) logp[row] = lp;
        jl += lp;
    }
    if (joint) joint[i] = jl;
}

// ---------------------------------------------------------------------------
// fused policy head + sampler
// ---------------------------------------------------------------------------
// logits = h W^T + b for the concatenated heads W = [move_head; mark_head]
// [6, K] (networks.py:38-41), then sample_row -- the logits never leave the
// registers.  8 lanes per row (each lane a 4-column stride of the row, so a
// row's 8 lanes read 128 contiguous bytes per step), 32 rows = 16 mazes per
// 256-thread workgroup; head weights staged in LDS.
constexpr int kHsLanes = 8;
constexpr int kHsRows = 32;
constexpr int kHsMaxK = 1024;

__global__ __launch_bounds__(kHsLanes* kHsRows) void k_head_sample(const float* __restrict__ h, int ldh, int K,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ b,
                                                                   const uint8_t* __restrict__ masks, int M,
                                                                   uint64_t seed, uint64_t offset,
                                                                   int8_t* __restrict__ act, float* __restrict__ logp,
                                                                   float* __restrict__ joint,
                                                                   float* __restrict__ logits) {
    __shared__ __attribute__((aligned(16))) float W[6 * kHsMaxK];
    // loads batched ahead of the LDS writes: one L2 round trip, not one per element
    constexpr int kB = 8;
    for (int e0 = threadIdx.x; e0 < 6 * K; e0 += kB * blockDim.x) {
        float t[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int e = e0 + u * blockDim.x;
            t[u] = e < 6 * K ? w[e] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int e = e0 + u * blockDim.x;
            if (e < 6 * K) W[e] = t[u];
        }
    }
    __syncthreads();
    const int j = threadIdx.x % kHsLanes;
    const int row = blockIdx.x * kHsRows + threadIdx.x / kHsLanes;
    const bool valid = row < M;
    float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (valid) {
        const float* hr = h + (size_t)row * ldh;
        for (int c = 4 * j; c < K; c += 4 * kHsLanes) {
            const float4 hv = *reinterpret_cast<const float4*>(hr + c);
#pragma unroll
            for (int o = 0; o < 6; o++) {
                const float4 wv = *reinterpret_cast<const float4*>(W + o * K + c);
                acc[o] = fmaf(hv.x, wv.x, acc[o]);
                acc[o] = fmaf(hv.y, wv.y, acc[o]);
                acc[o] = fmaf(hv.z, wv.z, acc[o]);
                acc[o] = fmaf(hv.w, wv.w, acc[o]);
            }
        }
    }
#pragma unroll
    for (int o = 0; o < 6; o++) {  // butterfly over the row's 8 lanes: every lane holds the sums
#pragma unroll
        for (int d = kHsLanes / 2; d > 0; d >>= 1) acc[o] += __shfl_xor(acc[o], d);
    }
    float lp = 0.f;
    if (valid && j == 0) {
        float l[5];
#pragma unroll
        for (int o = 0; o < 5; o++) l[o] = acc[o] + b[o];
        const float kl = acc[5] + b[5];
        int move, mark;
        lp = sample_row(l, kl, masks + (size_t)row * MM_MASK_DIM, row, seed, offset, move, mark);
        act[2 * row] = (int8_t)move;
        act[2 * row + 1] = (int8_t)mark;
        if (logp) logp[row] = lp;
        if (logits) {
#pragma unroll
            for (int o = 0; o < 5; o++) logits[(size_t)row * 6 + o] = l[o];
            logits[(size_t)row * 6 + 5] = kl;
        }
    }
    // joint log-prob of maze row/2: rows 2i and 2i+1 are adjacent 8-lane groups
    const float other = __shfl_down(lp, kHsLanes);
    if (joint && valid && j == 0 && (row & 1) == 0) joint[row >> 1] = lp + (row + 1 < M ? other : 0.f);
}

// per agent row: log pi(a | z) for the masked move logits z[0:5] and the
// masked mark logit z[5] (PPO.py:154-168, torch's op order in fp32); also the
// gradient d log pi / d z when grad != null
__device__ __forceinline__ float row_logp(const float* z, const uint8_t* mk, int move, int mark, float* grad) {
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 5; j++)
        if (mk[j]) mx = fmaxf(mx, z[j]);
    float se = 0.f;
    float e[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
        e[j] = mk[j] ? expf(z[j] - mx) : 0.f;
        se += e[j];
    }
    const float lse = logf(se);
    const float lpm = mk[move] ? (z[move] - mx) - lse : -INFINITY;  // log_softmax(masked)[move]
    // mark: p = sigmoid(masked logit); log(p) or log(1 - p)
    const float k = mk[5] ? z[5] : -INFINITY;
    const float p = 1.f / (1.f + expf(-k));
    const float pm = mark ? p : 1.f - p;
    if (grad) {
        const float inv = 1.f / se;
#pragma unroll
        for (int j = 0; j < 5; j++) grad[j] = mk[j] ? ((j == move ? 1.f : 0.f) - e[j] * inv) : 0.f;
        grad[5] = mk[5] ? (mark ? 1.f - p : -p) : 0.f;
    }
    return lpm + logf(pm);
}

constexpr int kLossThreads = 256;

// one thread per sample (two agent rows); per-workgroup partial sums of the
// clipped surrogate (fixed order: deterministic), coef[i] = d(-mean term)/d logp_i
__global__ __launch_bounds__(kLossThreads) void k_ppo_loss(const float* __restrict__ z, const uint8_t* __restrict__ mk,
                                                           const int8_t* __restrict__ act,
                                                           const float* __restrict__ old_lp,
                                                           const float* __restrict__ adv, int M, float clip,
                                                           float* __restrict__ coef, float* __restrict__ partial) {
    __shared__ float red[kLossThreads];
    const int i = blockIdx.x * kLossThreads + threadIdx.x;
    float term = 0.f;
    if (i < M) {
        float lp = 0.f;
#pragma unroll
        for (int a = 0; a < 2; a++) {
            const int r = 2 * i + a;
            lp += row_logp(z + (size_t)r * 6, mk + (size_t)r * 6, act[2 * r], act[2 * r + 1], nullptr);
        }
        const float ratio = expf(lp - old_lp[i]);
        const float A = adv[i];
        const float s1 = ratio * A;
        const float rc = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip);
        const float s2 = rc * A;
        term = fminf(s1, s2);
        // torch.min backward: the smaller input gets the gradient, a tie splits it;
        // clamp passes it only inside [1 - clip, 1 + clip]
        const bool inside = ratio >= 1.f - clip && ratio <= 1.f + clip;
        float dd;
        if (s1 < s2) dd = A;
        else if (s1 > s2) dd = inside ? A : 0.f;
        else dd = 0.5f * A + (inside ? 0.5f * A : 0.f);
        coef[i] = -dd * ratio / (float)M;
    }
    red[threadIdx.x] = term;
    __syncthreads();
    for (int w = kLossThreads / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void k_ppo_loss_bwd(const float* __restrict__ z, const uint8_t* __restrict__ mk,
                                                      const int8_t* __restrict__ act, const float* __restrict__ coef,
                                                      const float* __restrict__ dloss, int M,
                                                      float* __restrict__ dz) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;  // agent row
    if (r >= 2 * M) return;
    float g[6];
    row_logp(z + (size_t)r * 6, mk + (size_t)r * 6, act[2 * r], act[2 * r + 1], g);
    const float c = coef[r >> 1] * dloss[0];
#pragma unroll
    for (int j = 0; j < 6; j++) dz[(size_t)r * 6 + j] = c * g[j];
}

}  // namespace mm

using namespace mm;

extern "C" int mm_gae(const float* reward, const float* value, const uint8_t* done, const float* last_value, int T,
                      int N, float gamma, float gamma_lambda, float* adv, float* rtg, void* stream) {
    if (!reward || !value || !done || !adv || T < 0 || N < 0) return MM_E_ARG;
    if (T == 0 || N == 0) return 0;
    hipLaunchKernelGGL(k_gae, dim3((N + 255) / 256), dim3(256), 0, (hipStream_t)stream, reward, value, done,
                       last_value, T, N, gamma, gamma_lambda, adv, rtg);
    return (int)hipGetLastError();
}

extern "C" int mm_sample(const float* move_logits, const float* mark_logits, const uint8_t* masks, int M,
                         uint64_t seed, uint64_t offset, int8_t* actions, float* logp, float* joint_logp,
                         void* stream) {
    if (!move_logits || !mark_logits || !masks || !actions || M < 0) return MM_E_ARG;
    if (M == 0) return 0;
    const int nm = (M + 1) / 2;
    hipLaunchKernelGGL(k_sample, dim3((nm + 255) / 256), dim3(256), 0, (hipStream_t)stream, move_logits, mark_logits,
                       masks, M, seed, offset, actions, logp, joint_logp);
    return (int)hipGetLastError();
}

extern "C" int mm_head_sample(const float* h, int ldh, int K, const float* w, const float* b, const uint8_t* masks,
                              int M, uint64_t seed, uint64_t offset, int8_t* actions, float* logp, float* joint_logp,
                              float* logits, void* stream) {
    if (!h || !w || !b || !masks || !actions || M < 0 || K <= 0 || (K & 3) || K > kHsMaxK || ldh < K || (ldh & 3) ||
        ((uintptr_t)h & 15))
        return MM_E_ARG;
    if (M == 0) return 0;
    hipLaunchKernelGGL(k_head_sample, dim3((M + kHsRows - 1) / kHsRows), dim3(kHsLanes * kHsRows), 0,
                       (hipStream_t)stream, h, ldh, K, w, b, masks, M, seed, offset, actions, logp, joint_logp,
                       logits);
    return (int)hipGetLastError();
}

extern "C" int mm_ppo_loss_partials(int M) { return (M + kLossThreads - 1) / kLossThreads; }

extern "C" int mm_ppo_loss(const float* heads, const uint8_t* masks, const int8_t* actions, const float* old_logp,
                           const float* adv, int M, float clip, float* coef, float* partial, void* stream) {
    if (!heads || !masks || !actions || !old_logp || !adv || !coef || !partial || M <= 0) return MM_E_ARG;
    hipLaunchKernelGGL(k_ppo_loss, dim3(mm_ppo_loss_partials(M)), dim3(kLossThreads), 0, (hipStream_t)stream, heads,
                       masks, actions, old_logp, adv, M, clip, coef, partial);
    return (int)hipGetLastError();
}

extern "C" int mm_ppo_loss_bwd(const float* heads, const uint8_t* masks, const int8_t* actions, const float* coef,
                               const float* dloss, int M, float* dheads, void* stream) {
    if (!heads || !masks || !actions || !coef || !dloss || !dheads || M <= 0) return MM_E_ARG;
    hipLaunchKernelGGL(k_ppo_loss_bwd, dim3((2 * M + 255) / 256), dim3(256), 0, (hipStream_t)stream, heads, masks,
                       actions, coef, dloss, M, dheads);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// split-K partial sum (networks._split_k_wgrad): out[j] = sum_s x[s, j] (s in
// order) + addend[j].  Replaces a torch reduction over the leading dim of the
// [S, N*K] batched-GEMM partials plus the add of the remainder rows' GEMM.
// ---------------------------------------------------------------------------
namespace mm {
__global__ __launch_bounds__(256) void k_sum_leading4(const float4* __restrict__ x, int S, long n4,
                                                     const float4* __restrict__ addend, float4* __restrict__ out) {
    for (long j = blockIdx.x * 256L + threadIdx.x; j < n4; j += (long)gridDim.x * 256) {
        float4 a = x[j];
        for (int s = 1; s < S; s++) {
            const float4 b = x[(long)s * n4 + j];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        if (addend) {
            const float4 b = addend[j];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        out[j] = a;
    }
}

__global__ __launch_bounds__(256) void k_sum_leading1(const float* __restrict__ x, int S, long n,
                                                     const float* __restrict__ addend, float* __restrict__ out) {
    for (long j = blockIdx.x * 256L + threadIdx.x; j < n; j += (long)gridDim.x * 256) {
        float a = x[j];
        for (int s = 1; s < S; s++) a += x[(long)s * n + j];
        if (addend) a += addend[j];
        out[j] = a;
    }
}
}  // namespace mm

extern "C" int mm_sum_leading(const float* x, int S, long n, const float* addend, float* out, void* stream) {
    if (!x || !out || S <= 0 || n <= 0) return MM_E_ARG;
    const bool v4 = (n % 4 == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)out % 16 == 0) &&
                    (!addend || (uintptr_t)addend % 16 == 0);
    const long units = v4 ? n / 4 : n;
    const int grid = (int)((units + 255) / 256 < 4096 ? (units + 255) / 256 : 4096);
    if (v4)
        hipLaunchKernelGGL(mm::k_sum_leading4, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<const float4*>(x), S, units, reinterpret_cast<const float4*>(addend),
                           reinterpret_cast<float4*>(out));
    else
        hipLaunchKernelGGL(mm::k_sum_leading1, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, S, units, addend,
                           out);
    return (int)hipGetLastError();
}
