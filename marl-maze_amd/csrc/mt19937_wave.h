// mt19937_wave.h -- CPython-compatible MT19937 for one maze per wavefront.
//
// The reference draws every maze-generation random number from CPython's
// global `random` (maze.py:172,188,189,232-233,242,245,255).  Each maze owns
// its own stream (random.seed(seed_i) semantics, continued across resets).
// State layout = random.getstate()[1]: 624 words + the index, so a Python
// RNG state can be handed to / taken from the device unchanged.
//
// Generation runs one maze per 64-lane wavefront with the 624-word state in
// LDS.  The twist is split into 10 chunks of 64 lanes processed in order:
// chunk c reads words [64c, 64c+64) and their k+1 / k+-397 partners, then
// writes; every word a chunk reads is either not yet rewritten (k+1, k+397)
// or rewritten by an EARLIER chunk (k-227), exactly as the sequential loop
// of genrand_uint32 orders them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mm {

constexpr int kMtN = 624;
constexpr int kMtM = 397;

// Block = one wavefront: __syncthreads() is a wave barrier + LDS fence.
__device__ __forceinline__ void mt_twist_wave(uint32_t* mt, int lane) {
#pragma unroll 1
    for (int base = 0; base < kMtN; base += 64) {
        const int k = base + lane;
        uint32_t v = 0;
        if (k < kMtN) {
            const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % kMtN] & 0x7fffffffu);
            const uint32_t src = (k < kMtN - kMtM) ? mt[k + kMtM] : mt[k - (kMtN - kMtM)];
            v = src ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        __syncthreads();
        if (k < kMtN) mt[k] = v;
        __syncthreads();
    }
}

// Wave-uniform generator: every lane holds the same `idx` and reads the same
// LDS word (broadcast).  Must be called from wave-uniform control flow.
struct WaveRng {
    uint32_t* mt;  // LDS [624]
    int idx;       // 0..624
    int lane;

    __device__ __forceinline__ uint32_t u32() {
        if (idx >= kMtN) {
            mt_twist_wave(mt, lane);
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    // random.random(): 53-bit double
    __device__ __forceinline__ double random() {
        const uint32_t a = u32() >> 5, b = u32() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    // Random._randbelow_with_getrandbits(n), n >= 1
    __device__ __forceinline__ int below(uint32_t n) {
        const int k = 32 - __clz(n);  // n.bit_length()
        uint32_t r = u32() >> (32 - k);
        while (r >= n) r = u32() >> (32 - k);
        return (int)r;
    }
    // random.randint(a, b)
    __device__ __forceinline__ int randint(int a, int b) { return a + below((uint32_t)(b - a + 1)); }
};

// init_genrand + init_by_array (CPython random_seed for a non-negative int),
// one thread per maze, in place on the maze's global state row.
__device__ __forceinline__ void mt_seed_thread(uint32_t* st, uint64_t seed) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int klen = key[1] ? 2 : 1;
    uint32_t prev = 19650218u;
    st[0] = prev;
    for (int i = 1; i < kMtN; i++) {
        prev = 1812433253u * (prev ^ (prev >> 30)) + (uint32_t)i;
        st[i] = prev;
    }
    int i = 1, j = 0;
    prev = st[0];
    for (int k = (kMtN > klen ? kMtN : klen); k; k--) {
        const uint32_t v = (st[i] ^ ((prev ^ (prev >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        st[i] = v;
        prev = v;
        i++;
        j++;
        if (i >= kMtN) {
            st[0] = st[kMtN - 1];
            prev = st[0];
            i = 1;
        }
        if (j >= klen) j = 0;
    }
    for (int k = kMtN - 1; k; k--) {
        const uint32_t v = (st[i] ^ ((prev ^ (prev >> 30)) * 1566083941u)) - (uint32_t)i;
        st[i] = v;
        prev = v;
        i++;
        if (i >= kMtN) {
            st[0] = st[kMtN - 1];
            prev = st[0];
            i = 1;
        }
    }
    st[0] = 0x80000000u;
    st[kMtN] = kMtN;  // index: next draw twists
}

}  // namespace mm
