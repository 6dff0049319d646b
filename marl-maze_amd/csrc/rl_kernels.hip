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
//   k_gae_walk  the same, bit-identical, for few columns and long T (whole-
//             episode batches): parallel across episodes, one lane per
//             (column, chunk) running the episodes that end in its chunk.
//   k_gae_scan  the same recursion as an affine-map suffix scan (wavefront
//             shuffles + LDS): parallel inside episodes, reassociated (fp32
//             rounding differs; within 1e-5 relative).
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

#include <algorithm>

#include "marlmaze.h"
#include "policy_device.h"

namespace mm {

struct GaeArgs {
    const float* rew;
    const float* val;
    const uint8_t* done;
    const float* lv;  // last_value [N] or null
    int T, N;
    float g, gl;
    float* adv;
    float* rtg;  // or null
};

// delta_t of one position in the reference's operation order (header): `d` =
// this transition ends the episode, `have_next` = a value exists at t+1 (the
// next position or the bootstrap), `d_next` = the transition at t+1 ended its
// episode (quirk Q7's mask)
__device__ __forceinline__ float gae_delta(float r, float v, bool d, bool have_next, float v_next, bool d_next,
                                           float g) {
    if (d || !have_next) return __fsub_rn(r, v);  // the reference's `t+1 == len(ep)` branch
    float boot = __fmul_rn(g, v_next);
    if (d_next) boot = __fmul_rn(boot, 0.f);
    return __fsub_rn(__fadd_rn(r, boot), v);
}

// without a bootstrap value the segment end IS an episode end (done = 1)
__device__ __forceinline__ bool gae_end_at(const GaeArgs& a, int n, int t) {
    return a.done[(size_t)t * a.N + n] != 0 || (t == a.T - 1 && !a.lv);
}

// Reverse sweep of column n over t = t_hi .. t_lo calling f(t, delta_t, d_t,
// V_t) (f returns false to stop before position t).  The loads of kGaeU
// positions are issued together: the sweep is latency-bound (one HBM round
// trip per block instead of one per position).
constexpr int kGaeU = 16;
template <class F>
__device__ __forceinline__ void gae_sweep(const GaeArgs& a, int n, int t_hi, int t_lo, F&& f) {
    float v_next;
    bool d_next, have_next;
    if (t_hi + 1 < a.T) {
        v_next = a.val[(size_t)(t_hi + 1) * a.N + n];
        d_next = gae_end_at(a, n, t_hi + 1);
        have_next = true;
    } else {
        v_next = a.lv ? a.lv[n] : 0.f;
        d_next = false;
        have_next = a.lv != nullptr;
    }
    for (int tb = t_hi; tb >= t_lo; tb -= kGaeU) {
        float r[kGaeU], v[kGaeU];
        uint8_t dd[kGaeU];
#pragma unroll
        for (int u = 0; u < kGaeU; u++) {
            const int t = tb - u;
            if (t >= t_lo) {
                const size_t k = (size_t)t * a.N + n;
                r[u] = a.rew[k];
                v[u] = a.val[k];
                dd[u] = a.done[k];
            }
        }
#pragma unroll
        for (int u = 0; u < kGaeU; u++) {
            const int t = tb - u;
            if (t < t_lo) break;
            const bool d = dd[u] != 0 || (t == a.T - 1 && !a.lv);
            const float delta = gae_delta(r[u], v[u], d, have_next, v_next, d_next, a.g);
            if (!f(t, delta, d, v[u])) return;
            v_next = v[u];
            d_next = d;
            have_next = true;
        }
    }
}

__device__ __forceinline__ void gae_store(const GaeArgs& a, int n, int t, float adv, float v) {
    const size_t k = (size_t)t * a.N + n;
    a.adv[k] = adv;
    if (a.rtg) a.rtg[k] = __fadd_rn(adv, v);  // b_rtgs = b_advs + b_vals (PPO.py:46)
}

// one lane per maze column (many columns, short T): A_t = delta_t + f32(gl * A_{t+1}), 0-scaled at d_t
__global__ void k_gae(GaeArgs a) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= a.N) return;
    float acc = 0.f;
    gae_sweep(a, n, a.T - 1, 0, [&](int t, float delta, bool d, float v) {
        acc = __fadd_rn(delta, __fmul_rn(d ? 0.f : a.gl, acc));
        gae_store(a, n, t, acc, v);
        return true;
    });
}

// Few columns, long T (the reference's whole-episode batches: T up to tens of
// thousands): the column is cut into chunks of Lc positions, one lane per
// (column, chunk), and each lane owns the episodes that END in its chunk.  It
// runs each of them backward from its end to the position after the previous
// episode's end -- the same serial recursion, in the same order, as k_gae, so
// the result is bit-identical; the parallelism is across episodes (the
// recursion restarts at every done, PPO.py:201).  The longest episode bounds
// the time (<= max_timestep steps).
__global__ void k_gae_walk(GaeArgs a, int Lc, int nch) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)a.N * nch) return;
    const int n = (int)(gid % a.N), j = (int)(gid / a.N);  // neighbouring lanes: neighbouring columns
    const int t0 = j * Lc, t1 = min(a.T, t0 + Lc);
    for (int e = t1 - 1; e >= t0; e--) {
        if (!gae_end_at(a, n, e) && e != a.T - 1) continue;  // (T-1 with a bootstrap: the fragment's end)
        float acc = 0.f;
        gae_sweep(a, n, e, 0, [&](int t, float delta, bool d, float v) {
            if (t < e && d) return false;  // the previous episode's end: this episode is done
            acc = __fadd_rn(delta, __fmul_rn(d ? 0.f : a.gl, acc));
            gae_store(a, n, t, acc, v);
            return true;
        });
    }
}

// Long T, parallel INSIDE episodes (not bit-exact: the recursion is
// reassociated).  A_t = delta_t + c_t A_{t+1} is an affine map of A_{t+1}, and
// maps compose associatively, (P1, Q1) o (P2, Q2) = (P1 P2, P1 Q2 + Q1).  One
// workgroup per column; thread i owns a contiguous chunk (thread order = time
// order) and composes its chunk's map; a suffix scan of the maps with
// wavefront shuffles (then across the 4 wavefronts through LDS) gives every
// thread the advantage just after its chunk; a second sweep writes A_t.
__global__ __launch_bounds__(256) void k_gae_scan(GaeArgs a) {
    __shared__ float sP[4], sQ[4];
    const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (a.T + 255) / 256;
    const int t0 = min(a.T, tid * per), t1 = min(a.T, t0 + per);
    float P = 1.f, Q = 0.f;  // A(t0) = P A(t1) + Q
    if (t1 > t0)
        gae_sweep(a, n, t1 - 1, t0, [&](int, float delta, bool d, float) {
            const float c = d ? 0.f : a.gl;
            Q = __fadd_rn(delta, __fmul_rn(c, Q));
            P = __fmul_rn(c, P);
            return true;
        });
    // suffix scan inside the wavefront: lane l -> the map of lanes l .. 63
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float Pn = __shfl_down(P, off), Qn = __shfl_down(Q, off);
        if (lane + off < 64) {
            Q = __fadd_rn(__fmul_rn(P, Qn), Q);
            P = __fmul_rn(P, Pn);
        }
    }
    if (lane == 0) {
        sP[w] = P;
        sQ[w] = Q;
    }
    __syncthreads();
    float carry = 0.f;  // A at the start of wavefront w + 1's chunks (A after the column's end = 0)
    for (int ww = 3; ww > w; ww--) carry = __fadd_rn(__fmul_rn(sP[ww], carry), sQ[ww]);
    const float P1 = __shfl_down(P, 1), Q1 = __shfl_down(Q, 1);
    float acc = lane < 63 ? __fadd_rn(__fmul_rn(P1, carry), Q1) : carry;  // A(t1)
    if (t1 > t0)
        gae_sweep(a, n, t1 - 1, t0, [&](int t, float delta, bool d, float v) {
            acc = __fadd_rn(delta, __fmul_rn(d ? 0.f : a.gl, acc));
            gae_store(a, n, t, acc, v);
            return true;
        });
}

// Philox4x32-10 and sample_row (one agent row of PPO.get_action): policy_device.h, shared with the fused
// trunk + heads + sampler of x3mlp.hip.

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
                                                                   const uint64_t* __restrict__ offset_dev,
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
        const uint64_t off = offset + (offset_dev ? *offset_dev : 0ull);  // a device base: graph replays advance it
        lp = sample_row(l, kl, masks + (size_t)row * MM_MASK_DIM, row, seed, off, move, mark);
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

// The heads alone (the update's forward, networks.py:38-41): logits [M, 6] = h W^T + b with k_head_sample's
// arithmetic per row -- the same lanes, per-lane fma order and butterfly -- so the update's logits equal the
// rollout's bit for bit at the same parameters (the PPO ratio is exactly 1 before the first step).  A
// streaming GEMV (443 MB of h per 419,430-row minibatch): NS (= ceil(K / 32)) 16-byte loads per lane all in
// flight, through a buffer resource (columns past K and rows past M read zeros: no exec-masked loads), head
// weights zero-padded in LDS.  NS = 0: a runtime loop for other widths.
// H16: h is fp16 (the f16 networks' stored activations; exact in fp32, so the arithmetic is unchanged)
template <int NS, bool H16 = false>
__global__ __launch_bounds__(kHsLanes* kHsRows) void k_heads_fwd(const float* __restrict__ h, int ldh, int K,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ b, int M,
                                                                 float* __restrict__ logits) {
    constexpr int kSpan = NS > 0 ? 32 * NS : kHsMaxK;  // W row pitch (zero past K)
    __shared__ __attribute__((aligned(16))) float W[6 * kSpan];
    constexpr int kB = 8;
    for (int e0 = threadIdx.x; e0 < 6 * kSpan; e0 += kB * blockDim.x) {
        float t[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int e = e0 + u * blockDim.x, o = e / kSpan, c = e - o * kSpan;
            t[u] = (e < 6 * kSpan && c < K) ? w[o * K + c] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int e = e0 + u * blockDim.x;
            if (e < 6 * kSpan) W[e] = t[u];
        }
    }
    __syncthreads();
    const int j = threadIdx.x % kHsLanes;
    const int row = blockIdx.x * kHsRows + threadIdx.x / kHsLanes;
    float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (NS > 0) {
        // gfx9 buffer resource word 3 0x00020000: 32-bit data format, raw addressing
        constexpr uint32_t esz = H16 ? 2u : 4u;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)h, (short)0, (int)((size_t)M * ldh * esz), 0x00020000);
        float4 hv[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int c = 4 * j + 32 * s;
            const uint32_t off = (row < M && c < K) ? esz * ((uint32_t)row * (uint32_t)ldh + (uint32_t)c) : 0x80000000u;
            if constexpr (H16) {
                typedef __attribute__((ext_vector_type(2))) unsigned int u2;
                typedef __attribute__((ext_vector_type(4))) _Float16 h4;
                // (the whole vector cast at once: __builtin_bit_cast of a vector ELEMENT (v.y) compiled to the
                // first element's bits with this clang -- tests/test_gpu_f16_act.py caught it)
                const u2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
                const h4 hh = __builtin_bit_cast(h4, v);
                hv[s] = make_float4((float)hh.x, (float)hh.y, (float)hh.z, (float)hh.w);
            } else {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
                hv[s] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                                    __uint_as_float(v[3]));
            }
        }
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int c = 4 * j + 32 * s;
#pragma unroll
            for (int o = 0; o < 6; o++) {
                const float4 wv = *reinterpret_cast<const float4*>(W + o * kSpan + c);
                acc[o] = fmaf(hv[s].x, wv.x, acc[o]);
                acc[o] = fmaf(hv[s].y, wv.y, acc[o]);
                acc[o] = fmaf(hv[s].z, wv.z, acc[o]);
                acc[o] = fmaf(hv[s].w, wv.w, acc[o]);
            }
        }
    } else if (row < M) {
        const float* hr = h + (size_t)row * ldh;
        for (int c = 4 * j; c < K; c += 4 * kHsLanes) {
            const float4 hv = *reinterpret_cast<const float4*>(hr + c);
#pragma unroll
            for (int o = 0; o < 6; o++) {
                const float4 wv = *reinterpret_cast<const float4*>(W + o * kSpan + c);
                acc[o] = fmaf(hv.x, wv.x, acc[o]);
                acc[o] = fmaf(hv.y, wv.y, acc[o]);
                acc[o] = fmaf(hv.z, wv.z, acc[o]);
                acc[o] = fmaf(hv.w, wv.w, acc[o]);
            }
        }
    }
#pragma unroll
    for (int o = 0; o < 6; o++) {
#pragma unroll
        for (int d = kHsLanes / 2; d > 0; d >>= 1) acc[o] += __shfl_xor(acc[o], d);
    }
    // lane j < 6 of the row writes logit j: a row's 24 bytes, the workgroup's 32 rows contiguous
    float v = acc[0];
#pragma unroll
    for (int o = 1; o < 6; o++) v = j == o ? acc[o] : v;
    if (row < M && j < 6) logits[(size_t)row * 6 + j] = v + b[j];
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


// ---------------------------------------------------------------------------
// The critic's value, fused (networks.py:87-102 forward, inference only): V = w2 . ReLU(W1 ReLU(W0 x + b0) + b1)
// + b2 for x [M, K0], hidden widths 64 and 64, in ONE launch on the fp32 MFMA (v_mfma_f32_16x16x4_f32: an exact
// fmaf chain per output, no operand split).  A wavefront owns 16 rows at a time, no LDS staging of the weights:
// each lane holds its 4 x ceil(K0 / 4) W0 values and 4 x 16 W1 values in registers.  Persistent: one resident
// wavefront per SIMD loads the weights (50 KB, L2-resident) ONCE and then walks the row tiles blockIdx.x,
// + gridDim.x, ..., with the next tile's x values loaded while the current tile's MFMAs run.  (The first form,
// one wavefront per 16-row tile, re-read the 50 KB of weights per tile: 3.5 GB of L2 reads for the rollout's
// batched 1.1M rows, 1.14 ms.)  The hidden rows go through 4 KB of LDS into the A-operand layout of layer 1; the
// value head is a cross-lane dot product in a fixed order.  Per row the same operations in the same order as
// the one-tile form: bit-identical values.
// ---------------------------------------------------------------------------
constexpr int kCvH = 64;       // hidden width (PPO's Critic: hidden_sizes [64, 64])
constexpr int kCvMaxK = 132;   // K0 limit (the reference's 2 x 65 observations = 130): 33 k-steps in registers
constexpr int kCvMaxS = kCvMaxK / 4;
constexpr int kCvHp = kCvH + 4;  // LDS row pitch of the hidden rows (64 banks: conflict-free A reads)

typedef __attribute__((ext_vector_type(4))) float cv_f32x4;

// this lane's x values of row tile `tile` (MFMA 16x16x4 A operand: row c16, k = 4 s + q); zeros past K0, rows past
// M clamped (computed, never stored), a tile past the last one: zeros (not used)
__device__ __forceinline__ void cv_load_x(const float* __restrict__ x, int ldx, int K0, int S0, int M, int ntiles,
                                          int tile, int c16, int q, float (&xa)[kCvMaxS]) {
    const bool tv = tile < ntiles;
    const int xr = min(tile * 16 + c16, M - 1);
#pragma unroll
    for (int s = 0; s < kCvMaxS; s++) {
        const int k = 4 * s + q;
        xa[s] = (tv && s < S0 && k < K0) ? x[(size_t)xr * ldx + k] : 0.f;
    }
}

__global__ __launch_bounds__(64) void k_critic_value(const float* __restrict__ x, int ldx, int K0, int M,
                                                     const float* __restrict__ w0, const float* __restrict__ b0,
                                                     const float* __restrict__ w1, const float* __restrict__ b1,
                                                     const float* __restrict__ w2, const float* __restrict__ b2,
                                                     float* __restrict__ v) {
    __shared__ float hs[16 * kCvHp];
    const int lane = threadIdx.x, c16 = lane & 15, q = lane >> 4;
    const int S0 = (K0 + 3) >> 2;
    const int ntiles = (M + 15) / 16;
    int tile = blockIdx.x;
    float xa[kCvMaxS], wa[4][kCvMaxS], wb[4][kCvH / 4];
    cv_load_x(x, ldx, K0, S0, M, ntiles, tile, c16, q, xa);
#pragma unroll
    for (int s = 0; s < kCvMaxS; s++) {
        const int k = 4 * s + q;
        const bool ok = s < S0 && k < K0;
#pragma unroll
        for (int t = 0; t < 4; t++) wa[t][s] = ok ? w0[(size_t)(16 * t + c16) * K0 + k] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < kCvH / 4; s++)
#pragma unroll
        for (int t = 0; t < 4; t++) wb[t][s] = w1[(16 * t + c16) * kCvH + 4 * s + q];
    float bias0[4], bias1[4], wv[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        bias0[t] = b0[16 * t + c16];
        bias1[t] = b1[16 * t + c16];
        wv[t] = w2[16 * t + c16];
    }
    const float bv = b2[0];
    for (; tile < ntiles; tile += gridDim.x) {  // wave-uniform
        // layer 0, with the next tile's x loads in flight
        cv_f32x4 h[4];
#pragma unroll
        for (int t = 0; t < 4; t++) h[t] = cv_f32x4{0.f, 0.f, 0.f, 0.f};
        float xn[kCvMaxS];
        cv_load_x(x, ldx, K0, S0, M, ntiles, tile + gridDim.x, c16, q, xn);
#pragma unroll
        for (int s = 0; s < kCvMaxS; s++)
            if (s < S0) {  // wave-uniform
#pragma unroll
                for (int t = 0; t < 4; t++) h[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s], wa[t][s], h[t], 0, 0, 0);
            }
        // bias + ReLU; lane holds rows 4 q + g, column 16 t + c16 -> LDS, read back as layer 1's A operand
        __syncthreads();  // the previous tile's layer-1 reads of hs are done
#pragma unroll
        for (int t = 0; t < 4; t++) {
#pragma unroll
            for (int g = 0; g < 4; g++) hs[(4 * q + g) * kCvHp + 16 * t + c16] = fmaxf(h[t][g] + bias0[t], 0.f);
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; t++) h[t] = cv_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kCvH / 4; s++) {
            const float a = hs[c16 * kCvHp + 4 * s + q];
#pragma unroll
            for (int t = 0; t < 4; t++) h[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, wb[t][s], h[t], 0, 0, 0);
        }
        // value head: V[row] = b2 + sum_j ReLU(h1 + b1)[row][j] w2[j]: this lane's 4 rows x its 4 columns, then
        // the sum over the 16 lanes sharing the rows -- a fixed order
        float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 4; t++) {
#pragma unroll
            for (int g = 0; g < 4; g++) part[g] = fmaf(fmaxf(h[t][g] + bias1[t], 0.f), wv[t], part[g]);
        }
#pragma unroll
        for (int g = 0; g < 4; g++) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) part[g] += __shfl_xor(part[g], o);
        }
        if (c16 == 0) {
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int r = tile * 16 + 4 * q + g;
                if (r < M) v[r] = part[g] + bv;
            }
        }
#pragma unroll
        for (int s = 0; s < kCvMaxS; s++) xa[s] = xn[s];
    }
}

}  // namespace mm

using namespace mm;

extern "C" int mm_gae_ex(const float* reward, const float* value, const uint8_t* done, const float* last_value,
                         int T, int N, float gamma, float gamma_lambda, float* adv, float* rtg, int algo,
                         void* stream) {
    if (!reward || !value || !done || !adv || T < 0 || N < 0 || algo < MM_GAE_AUTO || algo > MM_GAE_SCAN)
        return MM_E_ARG;
    if (T == 0 || N == 0) return 0;
    const GaeArgs a{reward, value, done, last_value, T, N, gamma, gamma_lambda, adv, rtg};
    hipStream_t s = (hipStream_t)stream;
    // measured (tools/bench_gae.py): one lane per column wins from a few hundred columns up (T = 400, 4,096
    // columns: 55 us vs 1.7 ms walked); below that the serial column of one lane is latency-bound and the
    // episode-parallel walk wins (T = 15,600, 1 column: 0.49 vs 2.05 ms)
    if (algo == MM_GAE_AUTO) algo = (N >= 256 || T <= 2 * kGaeU) ? MM_GAE_COLUMN : MM_GAE_WALK;
    if (algo == MM_GAE_COLUMN) {
        hipLaunchKernelGGL(k_gae, dim3((N + 255) / 256), dim3(256), 0, s, a);
    } else if (algo == MM_GAE_WALK) {
        // chunks of >= 16 positions, enough of them for ~16k lanes
        const long want = (long)T * N / 16384;
        const int Lc = (int)std::max<long>(16, std::min<long>(want, T));
        const int nch = (T + Lc - 1) / Lc;
        const long lanes = (long)N * nch;
        hipLaunchKernelGGL(k_gae_walk, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, s, a, Lc, nch);
    } else {
        hipLaunchKernelGGL(k_gae_scan, dim3(N), dim3(256), 0, s, a);
    }
    return (int)hipGetLastError();
}

extern "C" int mm_gae(const float* reward, const float* value, const uint8_t* done, const float* last_value, int T,
                      int N, float gamma, float gamma_lambda, float* adv, float* rtg, void* stream) {
    return mm_gae_ex(reward, value, done, last_value, T, N, gamma, gamma_lambda, adv, rtg, MM_GAE_AUTO, stream);
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

extern "C" int mm_head_sample_ex(const float* h, int ldh, int K, const float* w, const float* b,
                                 const uint8_t* masks, int M, uint64_t seed, uint64_t offset,
                                 const uint64_t* offset_dev, int8_t* actions, float* logp, float* joint_logp,
                                 float* logits, void* stream) {
    if (!h || !w || !b || !masks || !actions || M < 0 || K <= 0 || (K & 3) || K > kHsMaxK || ldh < K || (ldh & 3) ||
        ((uintptr_t)h & 15))
        return MM_E_ARG;
    if (M == 0) return 0;
    hipLaunchKernelGGL(k_head_sample, dim3((M + kHsRows - 1) / kHsRows), dim3(kHsLanes * kHsRows), 0,
                       (hipStream_t)stream, h, ldh, K, w, b, masks, M, seed, offset, offset_dev, actions, logp,
                       joint_logp, logits);
    return (int)hipGetLastError();
}

extern "C" int mm_head_sample(const float* h, int ldh, int K, const float* w, const float* b, const uint8_t* masks,
                              int M, uint64_t seed, uint64_t offset, int8_t* actions, float* logp, float* joint_logp,
                              float* logits, void* stream) {
    return mm_head_sample_ex(h, ldh, K, w, b, masks, M, seed, offset, nullptr, actions, logp, joint_logp, logits,
                             stream);
}

extern "C" int mm_heads_fwd(const float* h, int ldh, int K, const float* w, const float* b, int M, float* logits,
                            void* stream) {
    if (!h || !w || !b || !logits || M < 0 || K <= 0 || (K & 3) || K > kHsMaxK || ldh < K || (ldh & 3) ||
        ((uintptr_t)h & 15) || (size_t)M * ldh * 4 >= 0x80000000ull)
        return MM_E_ARG;
    if (M == 0) return 0;
    const dim3 grid((M + kHsRows - 1) / kHsRows), block(kHsLanes * kHsRows);
    if ((K + 31) / 32 == 9)  // the actor's 264-wide last hidden layer
        hipLaunchKernelGGL(k_heads_fwd<9>, grid, block, 0, (hipStream_t)stream, h, ldh, K, w, b, M, logits);
    else
        hipLaunchKernelGGL(k_heads_fwd<0>, grid, block, 0, (hipStream_t)stream, h, ldh, K, w, b, M, logits);
    return (int)hipGetLastError();
}

// the same over fp16 h [M, ldh] (K = 257..288: the actor's 264-wide layer only)
extern "C" int mm_heads_fwd_h16(const void* h, int ldh, int K, const float* w, const float* b, int M, float* logits,
                                void* stream) {
    if (!h || !w || !b || !logits || M < 0 || (K & 3) || (K + 31) / 32 != 9 || ldh < K || (ldh & 3) ||
        ((uintptr_t)h & 7) || (size_t)M * ldh * 2 >= 0x80000000ull)
        return MM_E_ARG;
    if (M == 0) return 0;
    const dim3 grid((M + kHsRows - 1) / kHsRows), block(kHsLanes * kHsRows);
    hipLaunchKernelGGL((k_heads_fwd<9, true>), grid, block, 0, (hipStream_t)stream, static_cast<const float*>(h), ldh,
                       K, w, b, M, logits);
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

extern "C" int mm_critic_value(const float* x, int ldx, int K0, int M, int H0, int H1, const float* w0, const float* b0,
                               const float* w1, const float* b1, const float* w2, const float* b2, float* v,
                               void* stream) {
    if (!x || !w0 || !b0 || !w1 || !b1 || !w2 || !b2 || !v || M < 0 || K0 <= 0 || K0 > mm::kCvMaxK || ldx < K0)
        return MM_E_ARG;
    if (H0 != mm::kCvH || H1 != mm::kCvH) return MM_E_ARG;  // the reference critic's [64, 64]
    if (M == 0) return 0;
    // persistent: as many one-wavefront workgroups as are resident at once (the occupancy the compiler's register
    // count allows, times the CUs), or one per row tile when there are fewer tiles
    static int resident[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return MM_E_ARG;
    if (!resident[dev]) {
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)mm::k_critic_value, 64, 0) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 4;
        resident[dev] = cus * per_cu;
    }
    const int tiles = (M + 15) / 16;
    const int grid = tiles < resident[dev] ? tiles : resident[dev];
    hipLaunchKernelGGL(mm::k_critic_value, dim3(grid), dim3(64), 0, (hipStream_t)stream, x, ldx, K0, M, w0, b0, w1,
                       b1, w2, b2, v);
    return (int)hipGetLastError();
}
