// policy_device.h -- device code of PPO.get_action (PPO.py:170-186) shared by rl_kernels.hip (k_sample,
// k_head_sample) and x3mlp.hip (k_trunk3's fused heads + sampler): the same draws and the same arithmetic
// in every kernel that samples an action.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace mm {

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


}  // namespace mm
