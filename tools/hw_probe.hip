// hw_probe.hip -- two hardware assumptions the weight-gradient kernels rest on, tested directly on gfx950
// (round-5 root-cause work on the intermittent k_wgrad_rect results):
//
//  P1  vmcnt counts buffer loads in issue order, also when a later load is out of range (offset past
//      num_records: no memory access) -- a later load completing first would let `s_waitcnt vmcnt(N)` pass
//      while an older load's registers still hold their previous contents.
//  P2  an MFMA has read its A/B operands once it has issued: a DS read or VALU write of those registers
//      right after it (LLVM inserts no wait states for this; only SrcC WAR is padded) cannot change the
//      product.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_var/hw_probe tools/hw_probe.hip
// Every asm block pads its own hazards (s_nop 4 after an SGPR written by VALU before a VMEM reads it,
// s_nop 2 before an MFMA reads a just-written VGPR) and drains its loads (vmcnt(0) / lgkmcnt(0)) before it
// ends; no address depends on a value under test.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#ifndef P6_NWR
#define P6_NWR 2
#endif

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__host__ __device__ inline uint32_t pattern(uint32_t i) { return i * 2654435761u + 12345u; }

__global__ void k_fill(uint32_t* p, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = pattern(i);
}

// buffer descriptor in SGPRs (word 3 0x00020000: 32-bit format, raw addressing), made uniform
__device__ inline i32x4 make_desc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    i32x4 d;
    d.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    d.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xFFFF));
    d.z = __builtin_amdgcn_readfirstlane((int)bytes);
    d.w = __builtin_amdgcn_readfirstlane(0x00020000);
    return d;
}

// P1.  mode 0: second load in range, random (control); 1: second load out of range on every lane;
// 2: out of range on odd lanes; 3: second load in range at a hot address (L2 hit);
// 4: eight out-of-range loads after the slow one, vmcnt(8); 5: the FIRST load out of range on odd lanes
// (its in-range lanes checked), the second in range; 6: the second load out of range on lanes 56-63 only
// (one 16-lane group partly out of range, as k_wgrad_rect's last B piece at K = 264).
// A lane counts the iterations whose first load's register still held the sentinel (or a wrong value)
// after the wait that should cover it.
__global__ void k_p1(const uint32_t* src, uint32_t nwords, int iters, int mode, unsigned long long* bad,
                     unsigned long long* checks) {
    const i32x4 rs = make_desc(src, nwords * 4u);
    uint32_t h = 0x9E3779B9u ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2246822519u);
    unsigned long long nb = 0;
    for (int it = 0; it < iters; it++) {
        h ^= h << 13;
        h ^= h >> 17;
        h ^= h << 5;
        const uint32_t idx = h % nwords;
        const uint32_t o1 = idx * 4u;
        uint32_t o2;
        const uint32_t r2 = ((h * 747796405u) % nwords) * 4u;
        const bool odd = threadIdx.x & 1;
        uint32_t o1x = o1;
        if (mode == 0 || mode == 5) o2 = r2;
        else if (mode == 2) o2 = odd ? 0x80000000u : r2;
        else if (mode == 3) o2 = 64u * 4u;
        else if (mode == 6) o2 = (threadIdx.x & 63) >= 56 ? 0x80000000u : r2;
        else o2 = 0x80000000u;
        if (mode == 5 && odd) o1x = 0x80000000u;
        uint32_t a, b, c;
        if (mode == 4) {
            uint32_t b1, b2, b3, b4, b5, b6, b7;
            asm volatile(
                "s_nop 4\n\t"
                "v_mov_b32 %0, 0xdeadbeef\n\t"
                "buffer_load_dword %0, %10, %12, 0 offen\n\t"
                "buffer_load_dword %1, %11, %12, 0 offen\n\t"
                "buffer_load_dword %2, %11, %12, 0 offen offset:4\n\t"
                "buffer_load_dword %3, %11, %12, 0 offen offset:8\n\t"
                "buffer_load_dword %4, %11, %12, 0 offen offset:12\n\t"
                "buffer_load_dword %5, %11, %12, 0 offen offset:16\n\t"
                "buffer_load_dword %6, %11, %12, 0 offen offset:20\n\t"
                "buffer_load_dword %7, %11, %12, 0 offen offset:24\n\t"
                "buffer_load_dword %8, %11, %12, 0 offen offset:28\n\t"
                "s_waitcnt vmcnt(8)\n\t"
                "v_mov_b32 %9, %0\n\t"
                "s_waitcnt vmcnt(0)\n\t"
                : "=&v"(a), "=&v"(b), "=&v"(b1), "=&v"(b2), "=&v"(b3), "=&v"(b4), "=&v"(b5), "=&v"(b6), "=&v"(b7),
                  "=&v"(c)
                : "v"(o1x), "v"(o2), "s"(rs)
                : "memory");
        } else {
            asm volatile(
                "s_nop 4\n\t"
                "v_mov_b32 %0, 0xdeadbeef\n\t"
                "buffer_load_dword %0, %3, %5, 0 offen\n\t"
                "buffer_load_dword %1, %4, %5, 0 offen\n\t"
                "s_waitcnt vmcnt(1)\n\t"
                "v_mov_b32 %2, %0\n\t"
                "s_waitcnt vmcnt(0)\n\t"
                : "=&v"(a), "=&v"(b), "=&v"(c)
                : "v"(o1x), "v"(o2), "s"(rs)
                : "memory");
        }
        (void)b;
        const uint32_t want = o1x == o1 ? pattern(idx) : 0u;  // an out-of-range lane reads 0
        nb += (c != want) || (a != want);
    }
    atomicAdd(bad, nb);
    atomicAdd(checks, (unsigned long long)iters);
}

// P2.  Every wave: acc += A . B with A = B = 1 (fp16), 32 per element per product; right after the MFMA
// its B register is overwritten (mode 0: ds_read_b128 of 2.0s, 16x16x32; mode 1: v_pk_mov of 2.0s,
// 16x16x16, 64-bit operands), then B is restored and padded before the next MFMA.  A product that read
// the new B would add 64 (mode 0) / 32 (mode 1, k = 16: 16 vs 32) instead.  `hog` MFMAs into independent
// accumulators just before keep the XDL pipe busy, so the tested MFMA waits to start.
template <int HOG>
__global__ void k_p2(int iters, int mode, unsigned long long* bad, unsigned long long* checks) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[2][64 * 4];
    const int lane = threadIdx.x & 63;
    const uint32_t one2 = 0x3C003C00u, two2 = 0x40004000u;  // fp16 pairs (1, 1) and (2, 2)
    if (threadIdx.x < 64) {
        for (int j = 0; j < 4; j++) {
            lds[0][lane * 4 + j] = one2;
            lds[1][lane * 4 + j] = two2;
        }
    }
    __syncthreads();
    const uint32_t aold = (uint32_t)(uintptr_t)&lds[0][lane * 4];
    const uint32_t anew = (uint32_t)(uintptr_t)&lds[1][lane * 4];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    f32x4 h0 = acc, h1 = acc, h2 = acc, h3 = acc;
    u32x4 a4 = {one2, one2, one2, one2}, b4 = a4;
    f32x2 a2 = __builtin_bit_cast(f32x2, (uint2){one2, one2}), b2 = a2;
    const f32x2 t2 = __builtin_bit_cast(f32x2, (uint2){two2, two2});
    const f32x2 o2 = a2;
    for (int it = 0; it < iters; it++) {
        if (mode == 0) {
            asm volatile(
                "s_nop 2\n\t"
                ".if %8\n\t"
                "v_mfma_f32_16x16x32_f16 %1, %5, %5, %1\n\t"
                "v_mfma_f32_16x16x32_f16 %2, %5, %5, %2\n\t"
                "v_mfma_f32_16x16x32_f16 %3, %5, %5, %3\n\t"
                "v_mfma_f32_16x16x32_f16 %4, %5, %5, %4\n\t"
                ".endif\n\t"
                "v_mfma_f32_16x16x32_f16 %0, %5, %6, %0\n\t"
                "ds_read_b128 %6, %7\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "ds_read_b128 %6, %9\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "s_nop 7\n\t"
                "s_nop 7\n\t"
                : "+v"(acc), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(a4), "+v"(b4)
                : "v"(anew), "i"(HOG), "v"(aold)
                : "memory");
        } else {
            asm volatile(
                "s_nop 2\n\t"
                ".if %8\n\t"
                "v_mfma_f32_16x16x16_f16 %1, %5, %5, %1\n\t"
                "v_mfma_f32_16x16x16_f16 %2, %5, %5, %2\n\t"
                "v_mfma_f32_16x16x16_f16 %3, %5, %5, %3\n\t"
                "v_mfma_f32_16x16x16_f16 %4, %5, %5, %4\n\t"
                ".endif\n\t"
                "v_mfma_f32_16x16x16_f16 %0, %5, %6, %0\n\t"
                "v_pk_mov_b32 %6, %7, %7 op_sel:[0,1]\n\t"
                "v_pk_mov_b32 %6, %9, %9 op_sel:[0,1]\n\t"
                "s_nop 7\n\t"
                "s_nop 7\n\t"
                : "+v"(acc), "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3), "+v"(a2), "+v"(b2)
                : "v"(t2), "i"(HOG), "v"(o2)
                : "memory");
        }
    }
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    const float want = (mode == 0 ? 32.f : 16.f) * iters;
    unsigned long long nb = 0;
    for (int g = 0; g < 4; g++) nb += acc[g] != want;
    atomicAdd(bad, nb);
    atomicAdd(checks, 4ull);
    (void)h0;
}

// P3.  Eight buffer_load_dword back to back (random addresses: HBM misses), then -- with no wait -- the
// registers they read are rewritten: mode 0 the descriptor's num_records by SALU (s_mov_b32 s42, 0);
// mode 1 the same by VALU (v_readfirstlane_b32 s42 of a zero); mode 2 the address VGPRs by VALU (an
// out-of-range offset); mode 3 the same as mode 0 after 32 wait states (control).  A load that read its
// operands after the rewrite returns 0 instead of the pattern.  Counts per (load index, quarter-wave).
__global__ void k_p3(const uint32_t* src, uint32_t nwords, int iters, int mode, unsigned long long* bad) {
    const uint64_t base = (uint64_t)src;
    const int b0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const int b1 = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFF));
    const int b2 = __builtin_amdgcn_readfirstlane((int)(nwords * 4u));
    const int b3 = __builtin_amdgcn_readfirstlane(0x00020000);
    uint32_t h = 0x85EBCA6Bu ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2246822519u);
    uint32_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t zero = (uint32_t)iters >> 31;  // 0, opaque
    for (int it = 0; it < iters; it++) {
        uint32_t idx[8], o[8], d[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            h ^= h << 13;
            h ^= h >> 17;
            h ^= h << 5;
            idx[j] = h % nwords;
            o[j] = idx[j] * 4u;
        }
#define P3_LOADS                                                                                           \
    "s_mov_b32 s40, %16\n\ts_mov_b32 s41, %17\n\ts_mov_b32 s42, %18\n\ts_mov_b32 s43, %19\n\ts_nop 4\n\t" \
    "buffer_load_dword %0, %8, s[40:43], 0 offen\n\t"                                                      \
    "buffer_load_dword %1, %9, s[40:43], 0 offen\n\t"                                                      \
    "buffer_load_dword %2, %10, s[40:43], 0 offen\n\t"                                                     \
    "buffer_load_dword %3, %11, s[40:43], 0 offen\n\t"                                                     \
    "buffer_load_dword %4, %12, s[40:43], 0 offen\n\t"                                                     \
    "buffer_load_dword %5, %13, s[40:43], 0 offen\n\t"                                                     \
    "buffer_load_dword %6, %14, s[40:43], 0 offen\n\t"                                                     \
    "buffer_load_dword %7, %15, s[40:43], 0 offen\n\t"
#define P3_OUT                                                                                              \
    : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6]), "=&v"(d[7]), \
      "+v"(o[0]), "+v"(o[1]), "+v"(o[2]), "+v"(o[3]), "+v"(o[4]), "+v"(o[5]), "+v"(o[6]), "+v"(o[7])         \
    : "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(zero)                                                        \
    : "s40", "s41", "s42", "s43", "memory"
        if (mode == 0) {
            asm volatile(P3_LOADS "s_mov_b32 s42, 0\n\ts_waitcnt vmcnt(0)\n\t" P3_OUT);
        } else if (mode == 1) {
            asm volatile(P3_LOADS "v_readfirstlane_b32 s42, %20\n\ts_waitcnt vmcnt(0)\n\t" P3_OUT);
        } else if (mode == 2) {
            asm volatile(P3_LOADS
                         "v_mov_b32 %8, 0x80000000\n\tv_mov_b32 %9, 0x80000000\n\tv_mov_b32 %10, 0x80000000\n\t"
                         "v_mov_b32 %11, 0x80000000\n\tv_mov_b32 %12, 0x80000000\n\tv_mov_b32 %13, 0x80000000\n\t"
                         "v_mov_b32 %14, 0x80000000\n\tv_mov_b32 %15, 0x80000000\n\ts_waitcnt vmcnt(0)\n\t" P3_OUT);
        } else {
            asm volatile(P3_LOADS "s_nop 15\n\ts_nop 15\n\ts_mov_b32 s42, 0\n\ts_waitcnt vmcnt(0)\n\t" P3_OUT);
        }
#undef P3_LOADS
#undef P3_OUT
#pragma unroll
        for (int j = 0; j < 8; j++) cnt[j] += d[j] != pattern(idx[j]);
    }
    const int qw = (threadIdx.x & 63) >> 4;
    for (int j = 0; j < 8; j++)
        if (cnt[j]) atomicAdd(bad + 4 * j + qw, (unsigned long long)cnt[j]);
}

// P4.  The k_wgrad_rect signature (zeros in lanes 48-63 of a load whose address VGPR was written by VALU
// just before): the address VGPR A is rewritten by v_mov right after (mode 0) nothing, (1) an
// s_waitcnt vmcnt(0) for a buffer_load whose DESTINATION was A (its data, as an offset, is out of range),
// (2) a ds_write_b128 that read A as data, (3) the same as 1 with 4 wait states between the wait and the
// v_mov (control) -- then A is the address of a buffer_load.  A load that used a stale A returns 0.
// Counts per quarter-wave; all offsets stay inside the buffer or past num_records (no fault possible).
__global__ void k_p4(const uint32_t* src, uint32_t nwords, int iters, int mode, unsigned long long* bad) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[256 * 4];
    const uint64_t base = (uint64_t)src;
    const int b0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const int b1 = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFF));
    const int b2 = __builtin_amdgcn_readfirstlane((int)(nwords * 4u));
    const int b3 = __builtin_amdgcn_readfirstlane(0x00020000);
    const int lane = threadIdx.x & 63;
    const uint32_t ldsa = (uint32_t)(uintptr_t)&lds[(threadIdx.x & 255) * 4];
    uint32_t h = 0x27D4EB2Fu ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    unsigned long long nb = 0;
    for (int it = 0; it < iters; it++) {
        h ^= h << 13;
        h ^= h >> 17;
        h ^= h << 5;
        // coalesced: a wave reads 64 consecutive words at a random (wave-uniform) row
        const uint32_t row = (uint32_t)__builtin_amdgcn_readfirstlane((int)(h % (nwords / 64 - 1)));
        const uint32_t off = (row * 64u + lane) * 4u;
        const uint32_t offb = ((row + 1) * 64u + lane) * 4u;  // the first load's source: data words (floats)
        uint32_t a, d, x0, x1, x2;
        if (mode == 0) {
            asm volatile(
                "s_mov_b32 s40, %5\n\ts_mov_b32 s41, %6\n\ts_mov_b32 s42, %7\n\ts_mov_b32 s43, %8\n\ts_nop 4\n\t"
                "v_mov_b32 %0, %9\n\t"
                "buffer_load_dword %1, %0, s[40:43], 0 offen\n\t"
                "s_waitcnt vmcnt(0)\n\t"
                : "=&v"(a), "=&v"(d), "=&v"(x0), "=&v"(x1), "=&v"(x2)
                : "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(off), "v"(offb), "v"(ldsa)
                : "s40", "s41", "s42", "s43", "memory");
        } else if (mode == 1 || mode == 3) {
            asm volatile(
                "s_mov_b32 s40, %5\n\ts_mov_b32 s41, %6\n\ts_mov_b32 s42, %7\n\ts_mov_b32 s43, %8\n\ts_nop 4\n\t"
                "buffer_load_dword %0, %10, s[40:43], 0 offen\n\t"
                "s_waitcnt vmcnt(0)\n\t"
                ".if %12\n\ts_nop 3\n\t.endif\n\t"
                "v_mov_b32 %0, %9\n\t"
                "buffer_load_dword %1, %0, s[40:43], 0 offen\n\t"
                "s_waitcnt vmcnt(0)\n\t"
                : "=&v"(a), "=&v"(d), "=&v"(x0), "=&v"(x1), "=&v"(x2)
                : "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(off), "v"(offb), "v"(ldsa), "i"(0)
                : "s40", "s41", "s42", "s43", "memory");
            if (mode == 3) { /* control variant compiled below */ }
        } else {
            // v[100:103] carry float data; ds_write_b128 reads them, then v100 is rewritten and used as the address
            asm volatile(
                "s_mov_b32 s40, %5\n\ts_mov_b32 s41, %6\n\ts_mov_b32 s42, %7\n\ts_mov_b32 s43, %8\n\ts_nop 4\n\t"
                "v_mov_b32 v100, 0x3f800000\n\tv_mov_b32 v101, 0x3f800000\n\tv_mov_b32 v102, 0x3f800000\n\t"
                "v_mov_b32 v103, 0x3f800000\n\t"
                "ds_write_b128 %11, v[100:103]\n\t"
                "v_mov_b32 v100, %9\n\t"
                "buffer_load_dword %1, v100, s[40:43], 0 offen\n\t"
                "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
                : "=&v"(a), "=&v"(d), "=&v"(x0), "=&v"(x1), "=&v"(x2)
                : "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(off), "v"(offb), "v"(ldsa)
                : "s40", "s41", "s42", "s43", "v100", "v101", "v102", "v103", "memory");
        }
        (void)x0;
        (void)x1;
        (void)x2;
        (void)a;
        nb += d != pattern(row * 64u + lane);
        if (d != pattern(row * 64u + lane)) atomicAdd(bad + (lane >> 4), 1ull);
    }
    (void)nb;
}

// P5.  The k_wgrad_rect staging burst: three groups of 8 buffer_load_dword (16-lane groups read 64
// contiguous bytes, the group's 8 loads 384 B apart), issued back to back, then vmcnt(0).  mode 0: all in
// range (control); 1: the third group out of range on every lane; 2: the third group out of range on lanes
// 56-63; 3: the first group out of range on lanes 6-15 of every 16-lane group (k_wgrad_rect's dY pieces at
// N = 6).  Counts the in-range lanes of loads #1, #3 (group 1) and #9, #11 (group 2) whose value is wrong,
// per quarter-wave.
__global__ void k_p5(const uint32_t* src, uint32_t nwords, int iters, int mode, unsigned long long* bad) {
    const uint64_t base = (uint64_t)src;
    const int b0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const int b1 = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFF));
    const int b2 = __builtin_amdgcn_readfirstlane((int)(nwords * 4u));
    const int b3 = __builtin_amdgcn_readfirstlane(0x00020000);
    const int lane = threadIdx.x & 63;
    uint32_t h = 0x165667B1u ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    unsigned long long nb[4] = {0, 0, 0, 0};
    const uint32_t nblk = nwords / 1024 - 2;  // 4 KB blocks: a group reads 8 rows of 96 words
    for (int it = 0; it < iters; it++) {
        h ^= h << 13;
        h ^= h >> 17;
        h ^= h << 5;
        const uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane((int)(h % nblk));
        const uint32_t w0 = blk * 1024u + lane, w1 = blk * 1024u + 64u + lane, w2 = (blk + 1) * 1024u + lane;
        uint32_t a0 = w0 * 4u, a1 = w1 * 4u, a2 = w2 * 4u;
        const bool oob0 = mode == 3 && (lane & 15) >= 6;
        if (oob0) a0 = 0x80000000u;
        if (mode == 1 || (mode == 2 && lane >= 56)) a2 = 0x80000000u;
        uint32_t f0, f1, f2, f3;
        asm volatile(
            "s_mov_b32 s40, %7\n\ts_mov_b32 s41, %8\n\ts_mov_b32 s42, %9\n\ts_mov_b32 s43, %10\n\ts_nop 4\n\t"
            "buffer_load_dword v100, %4, s[40:43], 0 offen\n\t"
            "buffer_load_dword v101, %4, s[40:43], 0 offen offset:384\n\t"
            "buffer_load_dword v102, %4, s[40:43], 0 offen offset:768\n\t"
            "buffer_load_dword v103, %4, s[40:43], 0 offen offset:1152\n\t"
            "buffer_load_dword v104, %4, s[40:43], 0 offen offset:1536\n\t"
            "buffer_load_dword v105, %4, s[40:43], 0 offen offset:1920\n\t"
            "buffer_load_dword v106, %4, s[40:43], 0 offen offset:2304\n\t"
            "buffer_load_dword v107, %4, s[40:43], 0 offen offset:2688\n\t"
            "buffer_load_dword v108, %5, s[40:43], 0 offen\n\t"
            "buffer_load_dword v109, %5, s[40:43], 0 offen offset:384\n\t"
            "buffer_load_dword v110, %5, s[40:43], 0 offen offset:768\n\t"
            "buffer_load_dword v111, %5, s[40:43], 0 offen offset:1152\n\t"
            "buffer_load_dword v112, %5, s[40:43], 0 offen offset:1536\n\t"
            "buffer_load_dword v113, %5, s[40:43], 0 offen offset:1920\n\t"
            "buffer_load_dword v114, %5, s[40:43], 0 offen offset:2304\n\t"
            "buffer_load_dword v115, %5, s[40:43], 0 offen offset:2688\n\t"
            "buffer_load_dword v116, %6, s[40:43], 0 offen\n\t"
            "buffer_load_dword v117, %6, s[40:43], 0 offen offset:384\n\t"
            "buffer_load_dword v118, %6, s[40:43], 0 offen offset:768\n\t"
            "buffer_load_dword v119, %6, s[40:43], 0 offen offset:1152\n\t"
            "buffer_load_dword v120, %6, s[40:43], 0 offen offset:1536\n\t"
            "buffer_load_dword v121, %6, s[40:43], 0 offen offset:1920\n\t"
            "buffer_load_dword v122, %6, s[40:43], 0 offen offset:2304\n\t"
            "buffer_load_dword v123, %6, s[40:43], 0 offen offset:2688\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            "v_mov_b32 %0, v100\n\tv_mov_b32 %1, v102\n\tv_mov_b32 %2, v108\n\tv_mov_b32 %3, v110\n\t"
            : "=&v"(f0), "=&v"(f1), "=&v"(f2), "=&v"(f3)
            : "v"(a0), "v"(a1), "v"(a2), "s"(b0), "s"(b1), "s"(b2), "s"(b3)
            : "s40", "s41", "s42", "s43", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108",
              "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120",
              "v121", "v122", "v123", "memory");
        const int qw = lane >> 4;
        if (!oob0) nb[qw] += (f0 != pattern(w0)) + (f1 != pattern(w0 + 192));
        nb[qw] += (f2 != pattern(w1)) + (f3 != pattern(w1 + 192));
    }
    for (int q = 0; q < 4; q++)
        if (nb[q]) atomicAdd(bad + q, nb[q]);
}

// P6.  The k_wgrad_rect staging tail under LDS contention: odd waves stream ds_read_b128 (as the MFMA phase
// of the other waves does); even waves, per iteration: fill the address registers v[110:117] with float data
// (1.0f: out of range as an offset), issue two ds_write_b128 (left in flight), compute the eight addresses
// into v[110:117] by VALU (v_mov + v_add chain, as hipcc emits), issue eight buffer_load_dword, wait, and
// compare.  A load that used a stale address returns 0.  Counts per load index x quarter-wave.
__global__ __launch_bounds__(512) void k_p6(const uint32_t* src, uint32_t nwords, int iters, int nwr,
                                            unsigned long long* bad) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[8192];
    const uint64_t base = (uint64_t)src;
    const int b0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const int b1 = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFF));
    const int b2 = __builtin_amdgcn_readfirstlane((int)(nwords * 4u));
    const int b3 = __builtin_amdgcn_readfirstlane(0x00020000);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 8192; i += 512) lds[i] = i;
    __syncthreads();
    if (wave & 1) {  // LDS contention
        uint32_t a = (uint32_t)(uintptr_t)&lds[(lane * 4 + wave * 256) & 8191];
        u32x4 acc = {0, 0, 0, 0};
        for (int it = 0; it < iters * 8; it++) {
            u32x4 v;
            asm volatile("ds_read_b128 %0, %1\n\tds_read_b128 %0, %1 offset:1024\n\tds_read_b128 %0, %1 offset:2048\n\t"
                         "ds_read_b128 %0, %1 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(v) : "v"(a) : "memory");
            acc += v;
        }
        if (acc.x == 0x12345678u) bad[8 * 4] = acc.y;  // keep the loop
        return;
    }
    const uint32_t wa = (uint32_t)(uintptr_t)&lds[(lane * 4 + wave * 512) & 8191];
    uint32_t h = 0x9E3779B1u ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2246822519u);
    const uint32_t nrow = nwords / 264 - 8;
    unsigned long long nb[8][4] = {};
    for (int it = 0; it < iters; it++) {
        h ^= h << 13;
        h ^= h >> 17;
        h ^= h << 5;
        const uint32_t row = (uint32_t)__builtin_amdgcn_readfirstlane((int)(h % nrow));
        const uint32_t o0 = (row * 264u + lane) * 4u;  // 8 rows of 264 words, lanes on consecutive words
        uint32_t d0, d1, d2, d3, d4, d5, d6, d7;
        asm volatile(
            "s_mov_b32 s40, %9\n\ts_mov_b32 s41, %10\n\ts_mov_b32 s42, %11\n\ts_mov_b32 s43, %12\n\t"
            "v_mov_b32 v110, 0x3f800000\n\tv_mov_b32 v111, 0x3f800000\n\tv_mov_b32 v112, 0x3f800000\n\t"
            "v_mov_b32 v113, 0x3f800000\n\tv_mov_b32 v114, 0x3f800000\n\tv_mov_b32 v115, 0x3f800000\n\t"
            "v_mov_b32 v116, 0x3f800000\n\tv_mov_b32 v117, 0x3f800000\n\t"
            "v_mov_b32 v100, %8\n\tv_mov_b32 v101, %8\n\tv_mov_b32 v102, %8\n\tv_mov_b32 v103, %8\n\t"
            "s_nop 4\n\t"
            "ds_write_b128 %13, v[100:103]\n\t"
            ".if %15 > 1\n\tds_write_b128 %13, v[100:103] offset:1024\n\t.endif\n\t"
            ".if %15 > 2\n\tds_write_b128 %13, v[100:103] offset:2048\n\tds_write_b128 %13, v[100:103] offset:3072\n\t.endif\n\t"
            "v_mov_b32 v110, %14\n\t"
            "v_add_u32 v111, 0x420, v110\n\t"
            "v_add_u32 v112, 0x420, v111\n\t"
            "v_add_u32 v113, 0x420, v112\n\t"
            "v_add_u32 v114, 0x420, v113\n\t"
            "v_add_u32 v115, 0x420, v114\n\t"
            "v_add_u32 v116, 0x420, v115\n\t"
            "v_add_u32 v117, 0x420, v116\n\t"
            "buffer_load_dword %0, v110, s[40:43], 0 offen\n\t"
            "buffer_load_dword %1, v111, s[40:43], 0 offen\n\t"
            "buffer_load_dword %2, v112, s[40:43], 0 offen\n\t"
            "buffer_load_dword %3, v113, s[40:43], 0 offen\n\t"
            "buffer_load_dword %4, v114, s[40:43], 0 offen\n\t"
            "buffer_load_dword %5, v115, s[40:43], 0 offen\n\t"
            "buffer_load_dword %6, v116, s[40:43], 0 offen\n\t"
            "buffer_load_dword %7, v117, s[40:43], 0 offen\n\t"
            "s_waitcnt vmcnt(0) lgkmcnt(0)\n\t"
            : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(d4), "=&v"(d5), "=&v"(d6), "=&v"(d7)
            : "v"(h), "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(wa), "v"(o0), "i"(P6_NWR)
            : "s40", "s41", "s42", "s43", "v100", "v101", "v102", "v103", "v110", "v111", "v112", "v113", "v114",
              "v115", "v116", "v117", "memory");
        const uint32_t w = row * 264u + lane;
        const uint32_t d[8] = {d0, d1, d2, d3, d4, d5, d6, d7};
#pragma unroll
        for (int j = 0; j < 8; j++) nb[j][lane >> 4] += d[j] != pattern(w + 264u * j);
    }
    for (int j = 0; j < 8; j++)
        for (int q = 0; q < 4; q++)
            if (nb[j][q]) atomicAdd(bad + 4 * j + q, nb[j][q]);
    (void)nwr;
}

// P7.  The k_wgrad_rect register reuse: eight buffer_load_dword whose address VGPRs v[110:117] are the
// DESTINATIONS of the next eight buffer_load_dword (the next piece slot), issued right behind them --
// LLVM pads one wait state only when the two loads are adjacent.  Odd waves keep the texture path busy
// with random loads.  A load that read its address after the later load claimed the register gets a
// wrong value; counts per load index x quarter-wave.  PAD: wait states between the two groups.
template <int PAD>
__global__ __launch_bounds__(512) void k_p7(const uint32_t* src, uint32_t nwords, int iters, unsigned long long* bad) {
    const uint64_t base = (uint64_t)src;
    const int b0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const int b1 = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFF));
    const int b2 = __builtin_amdgcn_readfirstlane((int)(nwords * 4u));
    const int b3 = __builtin_amdgcn_readfirstlane(0x00020000);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t h = 0x2545F491u ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    const uint32_t nrow = nwords / 264 - 16;
    if (wave & 1) {  // texture-path contention: random dword loads
        uint32_t acc = 0;
        const volatile uint32_t* vs = src;
        for (int it = 0; it < iters * 4; it++) {
            h ^= h << 13;
            h ^= h >> 17;
            h ^= h << 5;
            acc += vs[h % nwords];
        }
        if (acc == 0x12345678u) bad[40] = acc;
        return;
    }
    unsigned long long nb[8][4] = {};
    for (int it = 0; it < iters; it++) {
        h ^= h << 13;
        h ^= h >> 17;
        h ^= h << 5;
        const uint32_t row = (uint32_t)__builtin_amdgcn_readfirstlane((int)(h % nrow));
        const uint32_t o0 = (row * 264u + lane) * 4u, o1 = ((row + 8) * 264u + lane) * 4u;
        uint32_t d0, d1, d2, d3, d4, d5, d6, d7;
        asm volatile(
            "s_mov_b32 s40, %8\n\ts_mov_b32 s41, %9\n\ts_mov_b32 s42, %10\n\ts_mov_b32 s43, %11\n\t"
            "v_mov_b32 v110, %12\n\t"
            "v_add_u32 v111, 0x420, v110\n\tv_add_u32 v112, 0x420, v111\n\tv_add_u32 v113, 0x420, v112\n\t"
            "v_add_u32 v114, 0x420, v113\n\tv_add_u32 v115, 0x420, v114\n\tv_add_u32 v116, 0x420, v115\n\t"
            "v_add_u32 v117, 0x420, v116\n\t"
            "v_mov_b32 v120, %13\n\t"
            "v_add_u32 v121, 0x420, v120\n\tv_add_u32 v122, 0x420, v121\n\tv_add_u32 v123, 0x420, v122\n\t"
            "v_add_u32 v124, 0x420, v123\n\tv_add_u32 v125, 0x420, v124\n\tv_add_u32 v126, 0x420, v125\n\t"
            "v_add_u32 v127, 0x420, v126\n\t"
            "s_nop 4\n\t"
            "buffer_load_dword %0, v110, s[40:43], 0 offen\n\t"
            "buffer_load_dword %1, v111, s[40:43], 0 offen\n\t"
            "buffer_load_dword %2, v112, s[40:43], 0 offen\n\t"
            "buffer_load_dword %3, v113, s[40:43], 0 offen\n\t"
            "buffer_load_dword %4, v114, s[40:43], 0 offen\n\t"
            "buffer_load_dword %5, v115, s[40:43], 0 offen\n\t"
            "buffer_load_dword %6, v116, s[40:43], 0 offen\n\t"
            "buffer_load_dword %7, v117, s[40:43], 0 offen\n\t"
            ".rept %14\n\ts_nop 0\n\t.endr\n\t"
            "buffer_load_dword v111, v120, s[40:43], 0 offen\n\t"
            "buffer_load_dword v110, v121, s[40:43], 0 offen\n\t"
            "buffer_load_dword v113, v122, s[40:43], 0 offen\n\t"
            "buffer_load_dword v112, v123, s[40:43], 0 offen\n\t"
            "buffer_load_dword v115, v124, s[40:43], 0 offen\n\t"
            "buffer_load_dword v114, v125, s[40:43], 0 offen\n\t"
            "buffer_load_dword v117, v126, s[40:43], 0 offen\n\t"
            "buffer_load_dword v116, v127, s[40:43], 0 offen\n\t"
            "s_waitcnt vmcnt(0)\n\t"
            : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(d4), "=&v"(d5), "=&v"(d6), "=&v"(d7)
            : "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(o0), "v"(o1), "i"(PAD)
            : "s40", "s41", "s42", "s43", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v120",
              "v121", "v122", "v123", "v124", "v125", "v126", "v127", "memory");
        const uint32_t w = row * 264u + lane;
        const uint32_t d[8] = {d0, d1, d2, d3, d4, d5, d6, d7};
#pragma unroll
        for (int j = 0; j < 8; j++) nb[j][lane >> 4] += d[j] != pattern(w + 264u * j);
    }
    for (int j = 0; j < 8; j++)
        for (int q = 0; q < 4; q++)
            if (nb[j][q]) atomicAdd(bad + 4 * j + q, nb[j][q]);
}

// P8.  k_wgrad_rect's destination order: eight buffer_load_dword into v[100:107] with the rows 264 words
// apart, issued in the order the compiler emits for the staging pieces -- ORDER 0: odd register of each
// 64-bit pair first (v101, v100, v103, v102, ...); 1: even first (v100, v101, ...); 2: eight loads into
// the even registers v100, v102, ... v114 (no pair written by two loads).  Odd waves keep the texture
// path busy.  Counts lanes whose value is wrong, per load x quarter-wave.
template <int ORDER>
__global__ __launch_bounds__(512) void k_p8(const uint32_t* src, uint32_t nwords, int iters, unsigned long long* bad) {
    const uint64_t base = (uint64_t)src;
    const int b0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    const int b1 = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFF));
    const int b2 = __builtin_amdgcn_readfirstlane((int)(nwords * 4u));
    const int b3 = __builtin_amdgcn_readfirstlane(0x00020000);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t h = 0x2545F491u ^ ((blockIdx.x * blockDim.x + threadIdx.x) * 2654435761u);
    const uint32_t nrow = nwords / 264 - 16;
    if (wave & 1) {  // texture-path contention: random dword loads
        uint32_t acc = 0;
        const volatile uint32_t* vs = src;
        for (int it = 0; it < iters * 4; it++) {
            h ^= h << 13;
            h ^= h >> 17;
            h ^= h << 5;
            acc += vs[h % nwords];
        }
        if (acc == 0x12345678u) bad[40] = acc;
        return;
    }
    unsigned long long nb[8][4] = {};
    for (int it = 0; it < iters; it++) {
        h ^= h << 13;
        h ^= h >> 17;
        h ^= h << 5;
        const uint32_t row = (uint32_t)__builtin_amdgcn_readfirstlane((int)(h % nrow));
        const uint32_t o0 = (row * 264u + lane) * 4u;
        uint32_t d0, d1, d2, d3, d4, d5, d6, d7;
#define P8_ADDR                                                                                              \
    "s_mov_b32 s40, %8\n\ts_mov_b32 s41, %9\n\ts_mov_b32 s42, %10\n\ts_mov_b32 s43, %11\n\t"               \
    "v_mov_b32 v120, %12\n\t"                                                                               \
    "v_add_u32 v121, 0x420, v120\n\tv_add_u32 v122, 0x420, v121\n\tv_add_u32 v123, 0x420, v122\n\t"         \
    "v_add_u32 v124, 0x420, v123\n\tv_add_u32 v125, 0x420, v124\n\tv_add_u32 v126, 0x420, v125\n\t"         \
    "v_add_u32 v127, 0x420, v126\n\ts_nop 4\n\t"
#define P8_OPS                                                                                               \
    : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3), "=v"(d4), "=v"(d5), "=v"(d6), "=v"(d7)                        \
    : "s"(b0), "s"(b1), "s"(b2), "s"(b3), "v"(o0)                                                            \
    : "s40", "s41", "s42", "s43", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108",   \
      "v110", "v112", "v114", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "memory"
        if constexpr (ORDER == 0)
            asm volatile(P8_ADDR
                         "buffer_load_dword v101, v120, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v100, v121, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v103, v122, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v102, v123, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v105, v124, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v104, v125, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v107, v126, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v106, v127, s[40:43], 0 offen\n\t"
                         "s_waitcnt vmcnt(0)\n\t"
                         "v_mov_b32 %0, v101\n\tv_mov_b32 %1, v100\n\tv_mov_b32 %2, v103\n\tv_mov_b32 %3, v102\n\t"
                         "v_mov_b32 %4, v105\n\tv_mov_b32 %5, v104\n\tv_mov_b32 %6, v107\n\tv_mov_b32 %7, v106\n\t" P8_OPS);
        else if constexpr (ORDER == 1)
            asm volatile(P8_ADDR
                         "buffer_load_dword v100, v120, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v101, v121, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v102, v122, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v103, v123, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v104, v124, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v105, v125, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v106, v126, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v107, v127, s[40:43], 0 offen\n\t"
                         "s_waitcnt vmcnt(0)\n\t"
                         "v_mov_b32 %0, v100\n\tv_mov_b32 %1, v101\n\tv_mov_b32 %2, v102\n\tv_mov_b32 %3, v103\n\t"
                         "v_mov_b32 %4, v104\n\tv_mov_b32 %5, v105\n\tv_mov_b32 %6, v106\n\tv_mov_b32 %7, v107\n\t" P8_OPS);
        else
            asm volatile(P8_ADDR
                         "buffer_load_dword v100, v120, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v102, v121, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v104, v122, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v106, v123, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v108, v124, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v110, v125, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v112, v126, s[40:43], 0 offen\n\t"
                         "buffer_load_dword v114, v127, s[40:43], 0 offen\n\t"
                         "s_waitcnt vmcnt(0)\n\t"
                         "v_mov_b32 %0, v100\n\tv_mov_b32 %1, v102\n\tv_mov_b32 %2, v104\n\tv_mov_b32 %3, v106\n\t"
                         "v_mov_b32 %4, v108\n\tv_mov_b32 %5, v110\n\tv_mov_b32 %6, v112\n\tv_mov_b32 %7, v114\n\t" P8_OPS);
#undef P8_ADDR
#undef P8_OPS
        const uint32_t w = row * 264u + lane;
        const uint32_t d[8] = {d0, d1, d2, d3, d4, d5, d6, d7};
#pragma unroll
        for (int j = 0; j < 8; j++) nb[j][lane >> 4] += d[j] != pattern(w + 264u * j);
    }
    for (int j = 0; j < 8; j++)
        for (int q = 0; q < 4; q++)
            if (nb[j][q]) atomicAdd(bad + 4 * j + q, nb[j][q]);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const int which = argc > 2 ? atoi(argv[2]) : 31;  // bit k: probe P(k+1)
    const uint32_t nwords = 256u << 20;  // 1 GiB: random loads miss L2 (and mostly the TLB)
    uint32_t* src;
    CK(hipMalloc(&src, (size_t)nwords * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, src, nwords);
    unsigned long long *d, h[2];
    CK(hipMalloc(&d, 16));
    const char* p1n[] = {"in-range/in-range (control)", "in-range then OOB (all lanes)", "in-range then OOB (odd lanes)",
                         "miss then L2-hit", "in-range then 8 x OOB, vmcnt(8)", "first load OOB on odd lanes",
                         "second OOB on lanes 56-63"};
    for (int mode = 0; mode < 7 && (which & 1); mode++) {
        CK(hipMemset(d, 0, 16));
        hipLaunchKernelGGL(k_p1, dim3(2048), dim3(256), 0, 0, src, nwords, iters, mode, d, d + 1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
        printf("P1 vmcnt order, %-34s: %llu stale of %llu lane-checks\n", p1n[mode], h[0], h[1]);
        fflush(stdout);
    }
    const char* p2n[] = {"ds_read_b128 over B (16x16x32)", "v_pk_mov over B (16x16x16)"};
    for (int mode = 0; mode < 2 && (which & 2); mode++)
        for (int hog = 0; hog < 2; hog++) {
            CK(hipMemset(d, 0, 16));
            // 8 waves per workgroup, 4 workgroups per CU worth of grid: several waves per SIMD contend
            if (hog)
                hipLaunchKernelGGL(k_p2<1>, dim3(1024), dim3(512), 0, 0, iters, mode, d, d + 1);
            else
                hipLaunchKernelGGL(k_p2<0>, dim3(1024), dim3(512), 0, 0, iters, mode, d, d + 1);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
            printf("P2 MFMA SrcB WAR, %-30s hog %d: %llu wrong of %llu accumulator values\n", p2n[mode], hog, h[0],
                   h[1]);
            fflush(stdout);
        }
    {
        unsigned long long* db;
        CK(hipMalloc(&db, 32 * 8));
        const char* p3n[] = {"SALU rewrites num_records", "VALU (readfirstlane) rewrites num_records", "VALU rewrites the addresses",
                             "control: SALU rewrite after 32 wait states"};
        for (int mode = 0; mode < 4 && (which & 4); mode++) {
            CK(hipMemset(db, 0, 32 * 8));
            hipLaunchKernelGGL(k_p3, dim3(2048), dim3(256), 0, 0, src, nwords, iters / 4 + 1, mode, db);
            CK(hipDeviceSynchronize());
            unsigned long long hb[32];
            CK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
            unsigned long long tot = 0;
            for (int i = 0; i < 32; i++) tot += hb[i];
            printf("P3 operand read after issue, %-44s: %llu wrong of %llu lane-loads; per load index x quarter-wave:",
                   p3n[mode], tot, (unsigned long long)2048 * 256 * (iters / 4 + 1) * 8);
            for (int j = 0; j < 8; j++) printf(" [%llu %llu %llu %llu]", hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
            printf("\n");
            fflush(stdout);
        }
        CK(hipFree(db));
    }
    {
        // a small descriptor range: float data read as an offset (1.0f = 0x3f800000) is past num_records
        const uint32_t nsmall = 1u << 20;
        unsigned long long* db;
        CK(hipMalloc(&db, 4 * 8));
        const char* p4n[] = {"v_mov then load (RAW)", "load dest -> vmcnt(0) -> v_mov -> load", "ds_write_b128 data -> v_mov -> load"};
        for (int mode = 0; mode < 3 && (which & 8); mode++) {
            CK(hipMemset(db, 0, 4 * 8));
            hipLaunchKernelGGL(k_p4, dim3(2048), dim3(512), 0, 0, src, nsmall, iters, mode, db);
            CK(hipDeviceSynchronize());
            unsigned long long hb[4];
            CK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
            printf("P4 stale address VGPR, %-40s: wrong per quarter-wave [%llu %llu %llu %llu] of %llu loads each\n", p4n[mode],
                   hb[0], hb[1], hb[2], hb[3], (unsigned long long)2048 * 512 / 4 * iters);
            fflush(stdout);
        }
        CK(hipFree(db));
    }
    {
        unsigned long long* db;
        CK(hipMalloc(&db, 4 * 8));
        const char* p5n[] = {"all in range (control)", "third group OOB (all lanes)", "third group OOB (lanes 56-63)",
                             "first group OOB (lanes 6-15 of each 16)"};
        for (int mode = 0; mode < 4 && (which & 16); mode++) {
            CK(hipMemset(db, 0, 4 * 8));
            hipLaunchKernelGGL(k_p5, dim3(2048), dim3(512), 0, 0, src, nwords, iters, mode, db);
            CK(hipDeviceSynchronize());
            unsigned long long hb[4];
            CK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
            printf("P5 staging burst, %-40s: wrong in-range values per quarter-wave [%llu %llu %llu %llu]\n", p5n[mode],
                   hb[0], hb[1], hb[2], hb[3]);
            fflush(stdout);
        }
        CK(hipFree(db));
    }
    if (which & 32) {
        unsigned long long* db;
        CK(hipMalloc(&db, 40 * 8));
        CK(hipMemset(db, 0, 40 * 8));
        hipLaunchKernelGGL(k_p6, dim3(1024), dim3(512), 0, 0, src, nwords, iters, P6_NWR, db);
        CK(hipDeviceSynchronize());
        unsigned long long hb[40];
        CK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
        unsigned long long tot = 0;
        for (int i = 0; i < 32; i++) tot += hb[i];
        printf("P6 staging tail under LDS contention (%d ds_write_b128 in flight): %llu wrong of %llu lane-loads;"
               " per load x quarter-wave:", P6_NWR, tot, (unsigned long long)1024 * 256 * iters * 8);
        for (int j = 0; j < 8; j++) printf(" [%llu %llu %llu %llu]", hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
        printf("\n");
        fflush(stdout);
        CK(hipFree(db));
    }
    if (which & 64) {
        unsigned long long* db;
        CK(hipMalloc(&db, 48 * 8));
        for (int pad = 0; pad < 2; pad++) {
            CK(hipMemset(db, 0, 48 * 8));
            if (pad)
                hipLaunchKernelGGL(k_p7<8>, dim3(1024), dim3(512), 0, 0, src, nwords, iters, db);
            else
                hipLaunchKernelGGL(k_p7<0>, dim3(1024), dim3(512), 0, 0, src, nwords, iters, db);
            CK(hipDeviceSynchronize());
            unsigned long long hb[48];
            CK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
            unsigned long long tot = 0;
            for (int i = 0; i < 32; i++) tot += hb[i];
            printf("P7 address VGPRs reused as the next loads' destinations, %d wait states between: %llu wrong of "
                   "%llu lane-loads; per load x quarter-wave:", pad ? 8 : 0, tot, (unsigned long long)1024 * 256 * iters * 8);
            for (int j = 0; j < 8; j++) printf(" [%llu %llu %llu %llu]", hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
            printf("\n");
            fflush(stdout);
        }
        CK(hipFree(db));
    }
    if (which & 128) {
        unsigned long long* db;
        CK(hipMalloc(&db, 48 * 8));
        const char* names[3] = {"odd register of each pair first", "even first", "even registers only"};
        for (int order = 0; order < 3; order++) {
            CK(hipMemset(db, 0, 48 * 8));
            if (order == 0) hipLaunchKernelGGL(k_p8<0>, dim3(1024), dim3(512), 0, 0, src, nwords, iters, db);
            else if (order == 1) hipLaunchKernelGGL(k_p8<1>, dim3(1024), dim3(512), 0, 0, src, nwords, iters, db);
            else hipLaunchKernelGGL(k_p8<2>, dim3(1024), dim3(512), 0, 0, src, nwords, iters, db);
            CK(hipDeviceSynchronize());
            unsigned long long hb[48];
            CK(hipMemcpy(hb, db, sizeof(hb), hipMemcpyDeviceToHost));
            unsigned long long tot = 0;
            for (int i = 0; i < 32; i++) tot += hb[i];
            printf("P8 eight dword loads, destinations %s: %llu wrong of %llu lane-loads; per load x quarter-wave:",
                   names[order], tot, (unsigned long long)1024 * 256 * iters * 8);
            for (int j = 0; j < 8; j++) printf(" [%llu %llu %llu %llu]", hb[4 * j], hb[4 * j + 1], hb[4 * j + 2], hb[4 * j + 3]);
            printf("\n");
            fflush(stdout);
        }
        CK(hipFree(db));
    }
    CK(hipFree(src));
    CK(hipFree(d));
    return 0;
}
