// x3mlp.hip -- fp32-accurate GEMMs of the actor MLP on gfx950's bf16 MFMA,
// operands pre-split into bf16 planes and stored in MFMA fragment order.
//
// Arithmetic (as gemm_x3.hip): every fp32 x is split exactly into three bf16
// parts x = hi + mid + lo (hi = RN(x), mid = RN(x - hi), lo = RN(x - hi -
// mid)); a product keeps the six partial products >= 2^-16 |ab| (hh, hm, mh,
// mm, hl, lh), each exact in the fp32 MFMA accumulator.  6 bf16 MFMAs per
// fp32 product: 2,500 / 6 = 417 TFLOP/s of fp32-class peak vs 157 for the
// f32 MFMA.
//
// What is new here: the split happens ONCE, in the producer (the previous
// GEMM's epilogue, or mm_x3_tp_pack for weights and the front-end output),
// into the "TP" layout below.  The GEMM main loop then has no VALU work at
// all: operand tiles go HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4,
// one 1-KiB wave-instruction per fragment tile), double-buffered, and the
// waves only issue ds_read_b128 + MFMA.
//
// TP layout of a logical [R, C] fp32 matrix (R padded to 256, C to 32):
//   block (rt, ks) = rows 16 rt .. +15, cols 32 ks .. +31, 3 KiB contiguous:
//   [plane 3][chunk c 4][row r 16][8 bf16], element j of chunk c = column
//   32 ks + kcol(c, j), kcol(c, j) = 4 c + j (j < 4) or 16 + 4 c + (j - 4):
//   the MFMA takes any order of k inside a step as long as both operands use
//   it, and this one lets a 16-lane group read a row's 64 contiguous bytes
//   (the fp32 A source below) instead of 16-byte pieces 32 bytes apart.
// so lane l of a 16x16x32 MFMA operand fragment (row l & 15, k 8 (l >> 4) ..
// +7) reads the 16 bytes at l * 16 of a plane block: lane-linear, conflict
// free, and exactly the image one global_load_lds_dwordx4 writes.
// Padding rows / columns hold zeros (the packers and epilogues write them).
//
// Precision template P (MM_PREC_*): P_X3 is the above; P_F16 keeps ONE fp16
// plane per operand (round-to-nearest), one f16 MFMA per product: the fp16
// actor/critic of BASELINE configs[4].  Storage stays fp32 (activations,
// gradients, master weights); an A-operand scale (a power of two, exact)
// keeps small gradients out of the fp16 subnormal range and the epilogue
// multiplies by its inverse (cscale).  The TP layout of P_F16 is the same
// with one plane (1 KiB blocks).
//
// k_wgrad: the weight gradient dW [N, K] = sum_m dY[m, n] X[m, k] of every
// nn.Linear in the update (networks.py:35-41, 87-106 under autograd).  The
// reduction runs over the M rows, which both operands store row-major, so each
// workgroup stages a 32-row step of dY and X into LDS already transposed into
// fragment order (one thread: one column x 8 rows -> split -> 16-byte LDS
// writes), waves own contiguous runs of output tiles (A fragments reused
// along a run), and the row slices' partials are summed in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "marlmaze.h"
#include "policy_device.h"

namespace mm {
namespace x3 {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

enum { P_X3 = MM_PREC_X3, P_F16 = MM_PREC_F16, P_X2 = MM_PREC_X2 };
template <int P>
struct Prec {
    static constexpr int kPlanes = P == P_X3 ? 3 : P == P_X2 ? 2 : 1;
    static constexpr int kBlk = 512 * kPlanes;  // uint16 per (rt, ks) block
    static constexpr bool kScaled = P != P_X3;  // operand scales / the output's cscale apply
};
constexpr float kX2Lo = 2048.f;         // P_X2: lo = RN16(2^11 (x - hi))
constexpr float kX2LoInv = 1.f / 2048.f;

// Range guard of the fp16-plane precisions.  P_X2 (x s = hi + 2^-11 lo) and P_F16 (x s rounded) hold every
// operand value as fp16 planes: |x s| >= 65520 rounds hi to inf (lo then to -inf), and every output that
// value reaches becomes inf or NaN, where the fp32 reference stays finite.  The kernels therefore check
// their OUTPUT accumulators, not their inputs (cheaper -- an output tile is a few values per lane -- and
// exact: an out-of-range operand always reaches a non-finite accumulator, an in-range one never does):
// a lane whose accumulators hold an inf / NaN (exponent field all ones) ORs bit 0 into g_range_flag.  mm_gemm_range_flag reads and clears the flag, stream-ordered,
// and the caller redoes the work at x3 (bf16x3: fp32's range).  (A non-finite INPUT also raises it: the
// redo then reproduces fp32's inf / NaN.)  The flag is written by vector atomics only.
__device__ unsigned int g_range_flag;

template <int P>
__device__ __forceinline__ void range_acc(uint32_t& rm, const f32x4& a) {  // rm: the largest |bits| (no compares)
    if constexpr (P != P_X3) {
#pragma unroll
        for (int g = 0; g < 4; g++) rm = max(rm, __float_as_uint(a[g]) & 0x7FFFFFFFu);
    }
    (void)rm;
    (void)a;
}
// the epilogues' form: a wave-wide mask in SGPRs (v_cmp_class + s_or), no VGPR held over the columns
template <int P>
__device__ __forceinline__ void range_val(uint64_t& rb, float x) {
    if constexpr (P != P_X3) rb |= __builtin_amdgcn_ballot_w64(!__builtin_isfinite(x));
    (void)rb;
    (void)x;
}
template <int P>
__device__ __forceinline__ void range_note_wave(uint64_t rb) {
    if constexpr (P != P_X3) {
        if (rb != 0 && (threadIdx.x & 63) == 0)
            __hip_atomic_fetch_or(&g_range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    (void)rb;
}
template <int P>
__device__ __forceinline__ void range_note(uint32_t rm) {
    if constexpr (P != P_X3) {  // an exponent field of all ones: inf or NaN
        if (rm >= 0x7F800000u) __hip_atomic_fetch_or(&g_range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    (void)rm;
}

constexpr int kBlk = 1536;  // uint16 per (rt, ks) block of P_X3: 3 planes x 512
constexpr int kRowPad = 256;

__host__ __device__ inline int rup(int x, int m) { return (x + m - 1) / m * m; }

// column (inside a 32-wide k-step) of element j of fragment chunk c
__host__ __device__ inline int kcol(int c, int j) { return j < 4 ? 4 * c + j : 12 + 4 * c + j; }

__device__ __forceinline__ uint32_t bf16_rn(float x) {  // round-to-nearest-even (finite x)
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ void split3(float x, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
    hi = bf16_rn(x);
    const float r1 = x - __uint_as_float(hi << 16);
    mid = bf16_rn(r1);
    const float r2 = r1 - __uint_as_float(mid << 16);
    lo = bf16_rn(r2);
}

// 8 consecutive fp32 -> three 16-byte plane pieces
__device__ __forceinline__ void split8(const float* v, uint4& h, uint4& m, uint4& l) {
    uint32_t hh[8], mm_[8], ll[8];
#pragma unroll
    for (int j = 0; j < 8; j++) split3(v[j], hh[j], mm_[j], ll[j]);
    h = make_uint4(hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16), hh[4] | (hh[5] << 16), hh[6] | (hh[7] << 16));
    m = make_uint4(mm_[0] | (mm_[1] << 16), mm_[2] | (mm_[3] << 16), mm_[4] | (mm_[5] << 16),
                   mm_[6] | (mm_[7] << 16));
    l = make_uint4(ll[0] | (ll[1] << 16), ll[2] | (ll[3] << 16), ll[4] | (ll[5] << 16), ll[6] | (ll[7] << 16));
}

// x * s -> fp16 (round to nearest even), two values packed
__device__ __forceinline__ uint32_t f16x2_rn(float x0, float x1) {
    typedef __attribute__((ext_vector_type(2))) _Float16 h2;
    const h2 h = __builtin_convertvector((__attribute__((ext_vector_type(2))) float){x0, x1}, h2);
    return __builtin_bit_cast(uint32_t, h);
}

__device__ __forceinline__ uint4 f16x8_rn(const float* v, float s) {
    return make_uint4(f16x2_rn(v[0] * s, v[1] * s), f16x2_rn(v[2] * s, v[3] * s), f16x2_rn(v[4] * s, v[5] * s),
                      f16x2_rn(v[6] * s, v[7] * s));
}

// P_X2: two values x s -> (hi, lo) fp16 pairs, hi = RN16(x s), lo = RN16(2^11 (x s - hi)).  x s - hi is exact
// (hi is the nearest fp16 to x s: Sterbenz), the 2^11 is exact, so lo carries the next 11 significand bits
// and x s = hi + 2^-11 lo to 2^-22 relative while hi is normal (|x s| >= 2^-14).
__device__ __forceinline__ void pair2(float x0, float x1, float s, uint32_t& h, uint32_t& l) {
    typedef __attribute__((ext_vector_type(2))) float f2;
    typedef __attribute__((ext_vector_type(2))) _Float16 h2;
    const f2 v = f2{x0, x1} * s;
    const h2 hv = __builtin_convertvector(v, h2);
    const f2 r = (v - __builtin_convertvector(hv, f2)) * kX2Lo;
    h = __builtin_bit_cast(uint32_t, hv);
    l = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h2));
}

// 8 values -> the two 16-byte P_X2 plane pieces
__device__ __forceinline__ void pair8(const float* v, float s, uint4& h, uint4& l) {
    uint32_t hh[4], ll[4];
#pragma unroll
    for (int k = 0; k < 4; k++) pair2(v[2 * k], v[2 * k + 1], s, hh[k], ll[k]);
    h = make_uint4(hh[0], hh[1], hh[2], hh[3]);
    l = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// the 8 values of one fragment piece -> the P planes (16 bytes each) at dst, dst + 64, ... (uint4 units)
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l);

template <int P>
__device__ __forceinline__ void store_piece(const float* v, float s, uint4* dst) {
    if constexpr (P == P_X3) {  // the hardware bf16 conversions (split2): ~4 VALU per value, not ~20
        uint32_t h[4], m[4], l[4];
#pragma unroll
        for (int k = 0; k < 4; k++) split2(v[2 * k], v[2 * k + 1], h[k], m[k], l[k]);
        dst[0] = make_uint4(h[0], h[1], h[2], h[3]);
        dst[64] = make_uint4(m[0], m[1], m[2], m[3]);
        dst[128] = make_uint4(l[0], l[1], l[2], l[3]);
    } else if constexpr (P == P_X2) {
        uint4 h, l;
        pair8(v, s, h, l);
        dst[0] = h;
        dst[64] = l;
    } else {
        dst[0] = f16x8_rn(v, s);
    }
}

// one fragment product, the precision's MFMAs (P_X3: the six partial products, small terms first; P_X2:
// hi hi into acc, the cross terms hi lo + lo hi into accx -- combined by x2_combine before the epilogue)
template <int P>
__device__ __forceinline__ f32x4 mma(const bf16x8* a, const bf16x8* b, f32x4 acc, f32x4& accx) {
    if constexpr (P == P_X2) {
#define MM_H8(x) __builtin_bit_cast(f16x8, x)
        accx = __builtin_amdgcn_mfma_f32_16x16x32_f16(MM_H8(a[1]), MM_H8(b[0]), accx, 0, 0, 0);
        accx = __builtin_amdgcn_mfma_f32_16x16x32_f16(MM_H8(a[0]), MM_H8(b[1]), accx, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(MM_H8(a[0]), MM_H8(b[0]), acc, 0, 0, 0);
#undef MM_H8
        return acc;
    }
    (void)accx;
    if constexpr (P == P_X3) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
    } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[0]), __builtin_bit_cast(f16x8, b[0]),
                                                     acc, 0, 0, 0);
    }
    return acc;
}

// P_X2: the product = hi hi + 2^-11 (hi lo + lo hi), one rounding (the scaling by 2^-11 is exact)
template <int P>
__device__ __forceinline__ f32x4 x2_combine(f32x4 acc, f32x4 accx) {
    if constexpr (P == P_X2) {
#pragma unroll
        for (int g = 0; g < 4; g++) acc[g] = fmaf(accx[g], kX2LoInv, acc[g]);
    }
    (void)accx;
    return acc;
}

// fp32 [R, C] (row-major, leading dimension ld; trans: element (i, j) at
// X[j * ld + i]) -> TP.  One thread per (rt, ks, c, r) 8-element piece.
template <int P>
__global__ __launch_bounds__(256) void k_tp_pack(const float* __restrict__ X, int R, int C, int ld, int trans,
                                                 int nks, long total, uint16_t* __restrict__ tp) {
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        const int l = (int)(e & 63);  // lane-linear position inside a plane block
        const long blk = e >> 6;      // (rt, ks)
        const int ks = (int)(blk % nks);
        const int rt = (int)(blk / nks);
        const int row = 16 * rt + (l & 15), c = l >> 4;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int col = 32 * ks + kcol(c, j);
            v[j] = (row < R && col < C) ? (trans ? X[(size_t)col * ld + row] : X[(size_t)row * ld + col]) : 0.f;
        }
        store_piece<P>(v, 1.f, reinterpret_cast<uint4*>(tp + blk * Prec<P>::kBlk) + l);
    }
}

// several packs in one launch (the update packs every weight of a network before its backward):
// the pieces of all segments laid end to end, each piece packed as by k_tp_pack
constexpr int kMaxPackSegs = 16;
struct PackSegs {
    mm_pack_seg_t s[kMaxPackSegs];
    long pre[kMaxPackSegs + 1];  // piece prefix
    int nks[kMaxPackSegs];
    int nseg;
};

template <int P>
__global__ __launch_bounds__(256) void k_tp_pack_multi(PackSegs ps) {
    const long total = ps.pre[ps.nseg];
    for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
        int k = 0;
        while (k + 1 < ps.nseg && t >= ps.pre[k + 1]) k++;
        const mm_pack_seg_t& g = ps.s[k];
        const long e = t - ps.pre[k];
        const int l = (int)(e & 63);
        const long blk = e >> 6;
        const int nks = ps.nks[k], ks = (int)(blk % nks), rt = (int)(blk / nks);
        const int row = 16 * rt + (l & 15), c = l >> 4;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int col = 32 * ks + kcol(c, j);
            v[j] = (row < g.R && col < g.C) ? (g.trans ? g.X[(size_t)col * g.ld + row] : g.X[(size_t)row * g.ld + col])
                                            : 0.f;
        }
        store_piece<P>(v, 1.f, reinterpret_cast<uint4*>(g.tp + blk * Prec<P>::kBlk) + l);
    }
}

#ifndef X3_WAVES
#define X3_WAVES 16
#endif
constexpr int kWaves = X3_WAVES;  // the streaming kernel's waves per workgroup (one row tile each)
constexpr int kThreads = 64 * kWaves;
constexpr int kBM = 16 * kWaves;  // rows per workgroup: one row tile per wave
static_assert(kBM <= kRowPad, "A row blocks must stay inside the TP row padding");
// per precision: P_X2 holds two accumulator sets (17 column tiles: 136 registers), so its workgroups are
// 8 waves (two per SIMD, 256 registers each) instead of 16
template <int P>
struct SW {
    static constexpr int kWaves = P == P_X2 ? 8 : ::mm::x3::kWaves;
    static constexpr int kThreads = 64 * kWaves;
    static constexpr int kBM = 16 * kWaves;
};

template <int NT, int P = P_X3>
struct Cfg {
    static constexpr int kPiecesB = Prec<P>::kPlanes * NT;      // 1-KiB B pieces per k-step
    static constexpr int kPerWaveB = (kPiecesB + SW<P>::kWaves - 1) / SW<P>::kWaves;
    static constexpr int kStageB = NT * Prec<P>::kBlk;          // uint16 per B stage
    static constexpr int kEpiLen = kWaves * 16 * 36 * 2;         // uint16: the waves' TP epilogue slices
    static constexpr int kLen0 = kStageB > kEpiLen ? kStageB : kEpiLen;  // stage buffer 0 doubles as epilogue
    static_assert((kLen0 + kStageB) * 2 <= 160 * 1024, "LDS");
};

// ReLU bit masks in accumulator order: for row tile rt, lane l, 3 words; bit
// 4 c + g = (value at row 16 rt + 4 (l >> 4) + g, column 16 c + (l & 15)) > 0.
// A forward GEMM with relu writes them (mbits_out); the input-gradient GEMM of
// the next layer, whose output has the same [M, N] tiling, reads them
// (mbits_in) to apply the ReLU backward without touching the fp32 activations.
constexpr int kMaskWords = 3;  // 96 bits >= 4 * NT for NT <= 24

struct Epi {
    const float* bias;       // [N] or null
    const float* mask;       // fp32 [M, ldm] or null: out *= (mask > 0) (the ReLU-backward of the layer below)
    const uint32_t* mbits_in;  // or null: out *= bit (one column block, N <= 272)
    uint32_t* mbits_out;       // or null: bit = (out > 0) after bias / ReLU
    float* c;                // fp32 [M, ldc] or null
    uint16_t* ctp;           // TP of the output or null (needs one column block)
    float* colsum;           // EM_BWD, or null: per row tile column sums of the output [rows / 16][N]
    int ldc, ldm, relu, cnks;  // cnks = TP column blocks of the output (ceil(N / 32))
    float cscale;              // P_F16: out = acc * cscale before bias (the inverse of the A scale)
    int bufok;                 // fp32 c (and colsum) addressable through buffer resources (< 2^31 bytes)
    int c16;                   // c holds fp16 [M, ldc] (EM_FWD16 / EM_BWD16: P_F16's stored activations / gradients)
    float oscale;              // EM_BWD16: c = fp16(out * oscale) (the input gradient pre-scaled for its consumers)
};

// B piece i (column tile i / planes, plane i % planes) of k-step ks -> LDS (one 1-KiB LDS-DMA)
template <int P>
__device__ __forceinline__ void dma_b(const uint16_t* Bg, int nks, int ks, int i, uint16_t* dst, int lane) {
    constexpr int np = Prec<P>::kPlanes;
    const int ct = i / np, p = i - np * ct;
    const uint4* src = reinterpret_cast<const uint4*>(Bg + ((size_t)ct * nks + ks) * Prec<P>::kBlk + p * 512);
    __builtin_amdgcn_global_load_lds(src + lane, dst, 16, 0, 0);
}

// x -> (hi, mid, lo) with the hardware round-to-nearest-even conversion
// (v_cvt_pk_bf16_f32), two values at a time; same values as split3
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf2;
    const bf2 hb = __builtin_convertvector((__attribute__((ext_vector_type(2))) float){x0, x1}, bf2);
    h = __builtin_bit_cast(uint32_t, hb);
    const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xFFFF0000u);
    const bf2 mb = __builtin_convertvector((__attribute__((ext_vector_type(2))) float){r0, r1}, bf2);
    m = __builtin_bit_cast(uint32_t, mb);
    const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xFFFF0000u);
    const bf2 lb = __builtin_convertvector((__attribute__((ext_vector_type(2))) float){s0, s1}, bf2);
    l = __builtin_bit_cast(uint32_t, lb);
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2v;
constexpr uint32_t kBufOOB = 0x80000000u;  // an offset past every buffer (num_records < 2^31)


// A operand sources.  A wave owns one row tile; per k-step each lane needs the
// 8 values (row 16 rt + (l & 15), k 32 ks + 8 (l >> 4) .. +7) as three bf16x8.
struct ASrcTP {  // pre-split TP planes: three lane-linear 1-KiB loads
    typedef bf16x8 Raw[3];
    const uint16_t* A;  // the wave's row tile
    int nks;
    __device__ void init(const uint16_t* base, int rt, int nks_, int, int, int, float) {
        nks = nks_;
        A = base + (size_t)rt * nks * kBlk;
    }
    __device__ __forceinline__ void load(int ks, Raw& r, int lane) const {
        const uint4* p = reinterpret_cast<const uint4*>(A + (size_t)ks * kBlk);
#pragma unroll
        for (int q = 0; q < 3; q++) r[q] = __builtin_bit_cast(bf16x8, p[64 * q + lane]);
    }
    template <int P>
    __device__ __forceinline__ void frag(const Raw& r, bf16x8 (&a)[3]) const {
        static_assert(P == P_X3, "pre-split TP A operands are bf16x3");
#pragma unroll
        for (int q = 0; q < 3; q++) a[q] = r[q];
    }
};

// a lane's 8 fp32 A values of one k-step (r[0]: k 4c..4c+3, r[1]: k 16+4c..: kcol order) -> its fragment
// planes: split (P_X3), hi / lo pairs of x s (P_X2), or rounded after scaling (P_F16)
template <int P>
__device__ __forceinline__ void frag_f32(const float4 (&r)[2], float scale, bf16x8 (&a)[3]) {
    if constexpr (P == P_X3) {
        uint32_t h[4], m[4], l[4];
        split2(r[0].x, r[0].y, h[0], m[0], l[0]);
        split2(r[0].z, r[0].w, h[1], m[1], l[1]);
        split2(r[1].x, r[1].y, h[2], m[2], l[2]);
        split2(r[1].z, r[1].w, h[3], m[3], l[3]);
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
        a[1] = __builtin_bit_cast(bf16x8, make_uint4(m[0], m[1], m[2], m[3]));
        a[2] = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
    } else if constexpr (P == P_X2) {
        uint32_t h[4], l[4];
        pair2(r[0].x, r[0].y, scale, h[0], l[0]);
        pair2(r[0].z, r[0].w, scale, h[1], l[1]);
        pair2(r[1].x, r[1].y, scale, h[2], l[2]);
        pair2(r[1].z, r[1].w, scale, h[3], l[3]);
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
        a[1] = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
    } else {
        const float s = scale;
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(f16x2_rn(r[0].x * s, r[0].y * s), f16x2_rn(r[0].z * s, r[0].w * s),
                                                     f16x2_rn(r[1].x * s, r[1].y * s), f16x2_rn(r[1].z * s, r[1].w * s)));
    }
}

// fp32 row-major [M, lda]: VW = 4 (16-byte loads; lda % 4 == 0) or 2 (8-byte
// loads: lda, K even, e.g. the critic's [M, 130] observations), split (P_X3)
// or rounded after scaling (P_F16) in registers
template <int VW>
struct ASrcF32V {
    typedef float4 Raw[2];
    __amdgpu_buffer_rsrc_t rs;  // A [M, lda] (the host keeps M lda 4 < 2^31: row chunks)
    uint32_t roff;              // this lane's row (clamped inside the matrix), column 4 (l >> 4), bytes
    int K, kq;
    float scale;
    __device__ void init(const float* base, int rt, int, int M, int lda, int K_, float scale_) {
        const int lane = threadIdx.x & 63;
        const int r = min(16 * rt + (lane & 15), M - 1);  // rows past M: computed, never stored
        K = K_;
        scale = scale_;
        kq = 4 * (lane >> 4);
        rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)((size_t)M * lda * 4), 0x00020000);
        roff = 4u * ((uint32_t)r * (uint32_t)lda + (uint32_t)kq);
    }
    // columns past K: an out-of-range offset reads zeros (no exec-masked conditional loads)
    __device__ __forceinline__ void load(int ks, Raw& r, int) const {
        const int k = 32 * ks + kq;  // kcol(c, 0..3) = 4c.., kcol(c, 4..7) = 16 + 4c..
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t o = roff + 4u * (32 * ks + 16 * h);
            if constexpr (VW == 4) {
                const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, k + 16 * h < K ? o : kBufOOB, 0, 0);
                r[h] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                                   __uint_as_float(v.w));
            } else {
                const u32x2v x = __builtin_amdgcn_raw_buffer_load_b64(rs, k + 16 * h < K ? o : kBufOOB, 0, 0);
                const u32x2v y = __builtin_amdgcn_raw_buffer_load_b64(rs, k + 16 * h + 2 < K ? o + 8 : kBufOOB, 0, 0);
                r[h] = make_float4(__uint_as_float(x.x), __uint_as_float(x.y), __uint_as_float(y.x),
                                   __uint_as_float(y.y));
            }
        }
    }
    template <int P>
    __device__ __forceinline__ void frag(const Raw& r, bf16x8 (&a)[3]) const {
        frag_f32<P>(r, scale, a);
    }
};
typedef ASrcF32V<4> ASrcF32;
typedef ASrcF32V<2> ASrcF32U;

// fp16 row-major [M, lda] (P_F16 at scale 1: the f16 networks' stored front-end output h, K = 460, which the
// B-resident kernel does not take): the lane's two 8-byte runs of 4 halves ARE its fragment, no conversion
struct ASrcF16V {
    typedef u32x2v Raw[2];
    __amdgpu_buffer_rsrc_t rs;
    uint32_t roff;  // this lane's row (clamped inside the matrix), column 4 (l >> 4), bytes
    int K, kq;
    __device__ void init(const unsigned short* base, int rt, int, int M, int lda, int K_, float) {
        const int lane = threadIdx.x & 63;
        const int r = min(16 * rt + (lane & 15), M - 1);  // rows past M: computed, never stored
        K = K_;
        kq = 4 * (lane >> 4);
        rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)((size_t)M * lda * 2), 0x00020000);
        roff = 2u * ((uint32_t)r * (uint32_t)lda + (uint32_t)kq);
    }
    __device__ __forceinline__ void load(int ks, Raw& r, int) const {  // columns past K: zeros (out of range)
        const int k = 32 * ks + kq;
#pragma unroll
        for (int h = 0; h < 2; h++)
            r[h] = __builtin_amdgcn_raw_buffer_load_b64(rs, k + 16 * h < K ? roff + 2u * (32 * ks + 16 * h) : kBufOOB, 0, 0);
    }
    template <int P>
    __device__ __forceinline__ void frag(const Raw& r, bf16x8 (&a)[3]) const {
        static_assert(P == P_F16, "fp16 A: P_F16");
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(r[0].x, r[0].y, r[1].x, r[1].y));
    }
};

// One k-step on stage buffer `cur`: split this step's A (raw -> fragments),
// prefetch the next step's raw A (registers) and B pieces (the other buffer;
// the DMA issues spread over the column loop), the 6 x NT MFMAs, one barrier.
template <int NT, int P, class AS>
__device__ __forceinline__ void k_step(f32x4 (&acc)[NT], f32x4 (&accx)[NT], const AS& as, const typename AS::Raw& raw,
                                       typename AS::Raw& rawn, const uint16_t* Bg, int nks, int ks,
                                       const uint16_t* cur, uint16_t* nxt, int wave, int lane) {
    using C = Cfg<NT, P>;
    constexpr int np = Prec<P>::kPlanes;
    const bool more = ks + 1 < nks;
    bf16x8 a[3];
    as.template frag<P>(raw, a);
#ifndef X3_NO_ALOAD  // diagnostic builds (tools/x3_variants.sh) only
    as.load(more ? ks + 1 : ks, rawn, lane);
#endif
    const bf16x8* b8 = reinterpret_cast<const bf16x8*>(cur) + lane;
#pragma unroll
    for (int c = 0; c < NT; c++) {
#ifndef X3_NO_DMA
        if (more && c < C::kPerWaveB) {
#else
        if (false) {
#endif
            const int i = wave + SW<P>::kWaves * c;
            if (i < C::kPiecesB) dma_b<P>(Bg, nks, ks + 1, i, nxt + i * 512, lane);
        }
        bf16x8 b[3];
#pragma unroll
        for (int q = 0; q < np; q++) b[q] = b8[(c * np + q) * 64];
        acc[c] = mma<P>(a, b, acc[c], accx[c]);
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // vmcnt(0): this wave's next-stage pieces and A loads landed; the barrier: every
                      // wave's, and stage `cur` is no longer read
    __builtin_amdgcn_sched_barrier(0);
}

// Epilogue modes (template parameter EM, so each kernel carries only its own
// epilogue and the main loop keeps its registers):
//   EM_F32:  fp32 out (+ bias)(ReLU)(* (fp32 mask > 0))
//   EM_FWD:  fp32 out (+ bias)(ReLU) and the ReLU bit mask (mbits_out)
//   EM_BWD:  fp32 out * bits (mbits_in): the input gradient through the ReLU below
//   EM_TP:   TP out (+ bias)(ReLU)(* (fp32 mask > 0))
// Accumulators acc[c]: lane l holds rows 4 (l >> 4) + g, column 16 c + (l & 15).
// fp32 rows are stored straight from the accumulators (16 lanes = 64 contiguous
// bytes of a row); no workgroup barrier.
//   EM_FWD16: EM_FWD with fp16 out (P_F16: the update's activations stored at the operand precision --
//             the next GEMM rounds them to fp16 anyway -- half the bytes of every activation read / write)
//   EM_BWD16: EM_BWD with fp16 out * oscale (P_F16: the input gradient stored pre-scaled, as its consumers'
//             operands; the column sums stay those of the fp32 values)
enum { EM_F32 = 0, EM_FWD = 1, EM_BWD = 2, EM_TP = 3, EM_FWD16 = 4, EM_BWD16 = 5 };
constexpr bool em_fwd(int em) { return em == EM_FWD || em == EM_FWD16; }
constexpr bool em_bwd(int em) { return em == EM_BWD || em == EM_BWD16; }
constexpr bool em_16(int em) { return em == EM_FWD16 || em == EM_BWD16; }

template <int NT, int EM, int P>
__device__ __forceinline__ void epilogue_f32(const f32x4 (&acc)[NT], int rt, int M, int N, int col0, const Epi& ep,
                                             const float* sbias, int lane) {
    uint64_t rb = 0;  // the range guard (range_val), noted at the end
    const int rq = 4 * (lane >> 4);  // first of this lane's four rows (within the tile)
    const float* sb = sbias + (lane & 15);  // one base register, column c at immediate offset 64 c
    uint32_t bits[kMaskWords] = {0u, 0u, 0u};
    if (EM == EM_BWD) {
        const uint32_t* mb = ep.mbits_in + ((size_t)rt * 64 + lane) * kMaskWords;
#pragma unroll
        for (int w = 0; w < kMaskWords; w++) bits[w] = mb[w];
    }
#pragma unroll
    for (int c = 0; c < NT; c++) {
        const int col = col0 + 16 * c + (lane & 15);
        // the unit's bias sits in LDS: a global load here would make every column
        // wait (vmcnt) for the previous columns' stores
        const float bv = (EM != EM_BWD && ep.bias) ? sb[16 * c] : 0.f;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int row = 16 * rt + rq + g, bit = 4 * c + g;
            float x = acc[c][g];
            range_val<P>(rb, x);
            if (Prec<P>::kScaled) x *= ep.cscale;
            if (EM == EM_BWD) {
                if (!((bits[bit >> 5] >> (bit & 31)) & 1u)) x = 0.f;
            } else {
                x += bv;
                if (ep.relu) x = fmaxf(x, 0.f);
            }
            if (EM == EM_FWD && x > 0.f && col < N && row < M) bits[bit >> 5] |= 1u << (bit & 31);
            if (row >= M || col >= N) continue;
            if (EM == EM_F32 && ep.mask && !(ep.mask[(size_t)row * ep.ldm + col] > 0.f)) x = 0.f;
            ep.c[(size_t)row * ep.ldc + col] = x;
        }
        if (EM == EM_BWD && ep.colsum) {  // the bias gradient's partial: this tile's 16-row column sums
            float cs = 0.f;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int row = 16 * rt + rq + g;
                if (row < M && ((bits[(4 * c + g) >> 5] >> ((4 * c + g) & 31)) & 1u))
                    cs += Prec<P>::kScaled ? acc[c][g] * ep.cscale : acc[c][g];
            }
            cs += __shfl_xor(cs, 16);
            cs += __shfl_xor(cs, 32);
            if (lane < 16 && col < N && 16 * rt < M) ep.colsum[(size_t)rt * N + col] = cs;
        }
        __builtin_amdgcn_sched_barrier(0);  // one column at a time: bounded live values
    }
    if (EM == EM_FWD) {
        uint32_t* mb = ep.mbits_out + ((size_t)rt * 64 + lane) * kMaskWords;
#pragma unroll
        for (int w = 0; w < kMaskWords; w++) mb[w] = bits[w];
    }
    range_note_wave<P>(rb);
}

// TP output through a 2-KiB wave-private LDS slice, 32 columns at a time, where
// each lane picks up the 8 consecutive values of its fragment-order piece.
template <int NT>
__device__ __forceinline__ void epilogue_tp(const f32x4 (&acc)[NT], float* slice, int rt, int M, int N,
                                            const Epi& ep, int lane) {
    const int rq = 4 * (lane >> 4);
    const int rr = lane & 15, row = 16 * rt + rr, ch = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < (16 * NT + 31) / 32; ks++) {
        if (ks >= ep.cnks) break;  // the output is narrower than the tile block
        // tiles 2 ks, 2 ks + 1 -> slice [16 rows][32 cols] (stride 36 floats: conflict-free writes)
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int c = 2 * ks + h;
#pragma unroll
            for (int g = 0; g < 4; g++)
                slice[(rq + g) * 36 + 16 * h + (lane & 15)] = c < NT ? acc[c < NT ? c : 0][g] : 0.f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float4 v0 = *reinterpret_cast<const float4*>(slice + rr * 36 + kcol(ch, 0));
        const float4 v1 = *reinterpret_cast<const float4*>(slice + rr * 36 + kcol(ch, 4));
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int col = 32 * ks + kcol(ch, j);
            float x = 0.f;
            if (col < N && row < M) {
                x = v[j] + (ep.bias ? ep.bias[col] : 0.f);
                if (ep.relu) x = fmaxf(x, 0.f);
                if (ep.mask && !(ep.mask[(size_t)row * ep.ldm + col] > 0.f)) x = 0.f;
            }
            v[j] = x;
        }
        uint4 h, m, l;
        split8(v, h, m, l);
        uint4* dst = reinterpret_cast<uint4*>(ep.ctp + ((size_t)rt * ep.cnks + ks) * kBlk) + lane;
        dst[0] = h;
        dst[64] = m;
        dst[128] = l;
        __builtin_amdgcn_wave_barrier();  // the slice is rewritten next round
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int ks = (16 * NT + 31) / 32; ks < ep.cnks; ks++) {  // columns beyond the block: zeros
        uint4* dst = reinterpret_cast<uint4*>(ep.ctp + ((size_t)rt * ep.cnks + ks) * kBlk) + lane;
        dst[0] = dst[64] = dst[128] = make_uint4(0, 0, 0, 0);
    }
}

// C[M, N] = A[M, K] . B[N, K]^T, B in TP, A from source AS.  Workgroup: 16
// waves, 256 rows x 16 NT columns; wave w owns row tile w and all NT column
// tiles.  A is private to a wave: straight from HBM to registers, one k-step
// ahead.  B (the weights) is shared: LDS-DMA into a double-buffered stage, the
// DMA issues spread over the MFMA stream.  One barrier per k-step; four waves
// per SIMD hide the LDS latency of the B fragment reads.  Persistent over
// 256-row units.
// Epilogue of one row tile x ctn column tiles (global tiles tg0 .. tg0 + ctn - 1; tg0 even), all stores
// through buffer resources: rows past M fall past num_records and are dropped by the hardware, so there is
// one code path with no per-element branches or 64-bit address arithmetic (lane offsets per row, the
// column tile at an immediate offset); only a tile crossing N selects an out-of-range offset for its
// lanes past N.  ReLU bits: bit 4 c + g of the tile-local words = bit 4 (tg0 + c) + g of the row tile's
// mask, i.e. local byte m is global byte tg0 / 2 + m -- each block writes (EM_FWD) and reads (EM_BWD)
// whole bytes of its own tiles.  Bits of rows past M are left unspecified (every reader masks by row);
// columns past N compute to exact zeros (zero B rows and bias) and record 0.
template <int P, int CT, int EM>
__device__ __forceinline__ void bres_epilogue(const f32x4 (&acc)[CT], int rt, int tg0, int ctn, int M, int N,
                                              const Epi& ep, __amdgpu_buffer_rsrc_t crs,
                                              __amdgpu_buffer_rsrc_t srs, const float* sb, int lane) {
    constexpr int NW = (4 * CT + 31) / 32;  // local mask words
    uint64_t rb = 0;  // the range guard (range_val), noted at the end
    int rq = 4 * (lane >> 4);
    asm volatile("" : "+v"(rq));  // offsets formed here, not hoisted over the main loop and held
    const int row0 = 16 * rt + rq, cl = lane & 15;
    constexpr uint32_t esz = em_16(EM) ? 2u : 4u;  // bytes per output element
    uint32_t voff[4];
#pragma unroll
    for (int g = 0; g < 4; g++) voff[g] = esz * ((uint32_t)(row0 + g) * (uint32_t)ep.ldc + (uint32_t)cl);
    const int soff = 16 * (int)esz * tg0;  // bytes: the block's first column tile
    uint32_t lbits[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) lbits[w] = 0u;
    if (em_bwd(EM)) {
        const uint8_t* mi =
            reinterpret_cast<const uint8_t*>(ep.mbits_in + ((size_t)rt * 64 + lane) * kMaskWords) + tg0 / 2;
#pragma unroll
        for (int m = 0; m < (CT + 1) / 2; m++)
            if (2 * m < ctn) lbits[m >> 2] |= (uint32_t)mi[m] << (8 * (m & 3));
        if (16 * rt + 16 > M) {  // the last row tile: rows past M masked out (their bits are unspecified)
            uint32_t rmask = 0u;
#pragma unroll
            for (int g = 0; g < 4; g++) rmask |= (row0 + g < M ? 1u : 0u) << g;
#pragma unroll
            for (int w = 0; w < NW; w++) lbits[w] &= rmask * 0x11111111u;
        }
    }
    const float* sbl = sb + cl;
#pragma unroll
    for (int c = 0; c < CT; c++) {
        if (c >= ctn || 16 * (tg0 + c) >= N) continue;  // wave-uniform (continue: the loop stays unrolled)
        const int col = 16 * (tg0 + c) + cl;
        const bool part = 16 * (tg0 + c) + 16 > N;  // wave-uniform: a tile crossing N
        const float bv = (!em_bwd(EM) && ep.bias) ? sbl[16 * c] : 0.f;
        float cs = 0.f;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int bit = 4 * c + g;
            float x = acc[c][g];
            range_val<P>(rb, x);
            if (Prec<P>::kScaled) x *= ep.cscale;
            if (em_bwd(EM)) {
                const bool on = (lbits[bit >> 5] >> (bit & 31)) & 1u;
                if (!on) x = 0.f;
                cs += x;
            } else {
                x += bv;
                if (ep.relu) x = fmaxf(x, 0.f);
                if (em_fwd(EM)) lbits[bit >> 5] |= (x > 0.f ? 1u : 0u) << (bit & 31);
            }
            uint32_t o = voff[g] + 16u * esz * c;
            if (part && col >= N) o = kBufOOB;
#ifdef BRES_NO_STORE  // diagnostic builds only
            if (x == 1234.5f)
#endif
            if constexpr (em_16(EM)) {
                // round to nearest; past 65504 it is inf: the range guard sees it
                const _Float16 h = (_Float16)(EM == EM_BWD16 ? x * ep.oscale : x);
                range_val<P>(rb, (float)h);
                __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), crs, o, soff, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), crs, o, soff, 0);
            }
        }
        if (em_bwd(EM) && ep.colsum) {  // the bias gradient's partial: this tile's 16-row column sums
            cs += __shfl_xor(cs, 16);
            cs += __shfl_xor(cs, 32);
            const uint32_t so = (lane < 16 && col < N) ? 4u * ((uint32_t)rt * (uint32_t)N + (uint32_t)col) : kBufOOB;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cs), srs, so, 0, 0);
        }
    }
    if (em_fwd(EM)) {
        uint8_t* mb = reinterpret_cast<uint8_t*>(ep.mbits_out + ((size_t)rt * 64 + lane) * kMaskWords) + tg0 / 2;
#pragma unroll
        for (int m = 0; m < (CT + 1) / 2; m++)
            if (2 * m < ctn) mb[m] = (uint8_t)(lbits[m >> 2] >> (8 * (m & 3)));
    }
    range_note_wave<P>(rb);
}

#ifdef X3_STAMPS  // diagnostic builds only (tools/x3_stamps.sh): per-wave phase clocks of k_x3nt
__device__ unsigned long long g_x3_stamps[256 * 16 * kWaves * 8];
#define X3_STAMP(it, slot, val)                                                                       \
    do {                                                                                              \
        if (lane == 0 && blockIdx.x < 256 && (it) < 16)                                               \
            g_x3_stamps[((blockIdx.x * 16 + (it)) * kWaves + wave) * 8 + (slot)] = (val);             \
    } while (0)
#else
#define X3_STAMP(it, slot, val) \
    do {                        \
    } while (0)
#endif

template <int NT, int P, class AS, class AT, int EM>
__global__ __launch_bounds__(SW<P>::kThreads) void k_x3nt(const AT* __restrict__ A, int lda, float ascale,
                                                   const uint16_t* __restrict__ B, int M, int N, int K, int nks,
                                                   int nrb, int ncb, Epi ep) {
    using C = Cfg<NT, P>;
    static_assert(EM != EM_TP || P == P_X3, "TP outputs are bf16x3");
    // two distinct LDS objects: the compiler's alias scopes then let a B read of
    // one stage run while the DMA into the other is in flight
    __shared__ float sbias[16 * NT];  // the unit's bias columns (EM_F32 / EM_FWD); first: small LDS offsets
    __shared__ __attribute__((aligned(16))) uint16_t sB0[C::kLen0];
    __shared__ __attribute__((aligned(16))) uint16_t sB1[C::kStageB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // (unused when !ep.bufok: then the ranges below are not consulted)
    const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)ep.c, (short)0, (int)((size_t)M * ep.ldc * (EM == EM_FWD16 ? 2 : 4)), 0x00020000);
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)ep.colsum, (short)0, (int)((size_t)((M + 15) / 16) * N * 4), 0x00020000);
    // workgroup g takes units g, g + G, ...  XCD-aware unit order: units u and
    // u + 8 (one XCD) are the column blocks of one row block, so its A is shared
    // through that XCD's L2
    const int nunits = ((nrb + 7) / 8) * 8 * ncb;
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        const int xcd = u & 7, slot = u >> 3;
        const int rb = (slot / ncb) * 8 + xcd, cb = slot % ncb;
        if (rb >= nrb) continue;  // workgroup-uniform
        const int rt = rb * SW<P>::kWaves + wave;  // this wave's row tile
        const int it = (u - (int)blockIdx.x) / (int)gridDim.x;
        (void)it;
        X3_STAMP(it, 0, __builtin_amdgcn_s_memtime());
        X3_STAMP(it, 4, __builtin_amdgcn_s_memrealtime());
        AS as;
        as.init(A, rt, nks, M, lda, K, ascale);
        const uint16_t* Bg = B + (size_t)cb * NT * nks * Prec<P>::kBlk;
        if (EM != EM_BWD && EM != EM_TP && ep.bias && threadIdx.x < 16 * NT) {  // visible after the prologue barrier
            int t = threadIdx.x;
            asm volatile("" : "+v"(t));  // recomputed per unit, not a loop-invariant address held (spilled) across it
            const int col = cb * 16 * NT + t;
            sbias[t] = col < N ? ep.bias[col] : 0.f;
        }

        f32x4 acc[NT], accx[NT];
#pragma unroll
        for (int c = 0; c < NT; c++) acc[c] = accx[c] = f32x4{0.f, 0.f, 0.f, 0.f};

        typename AS::Raw r0, r1;
        for (int i = wave; i < C::kPiecesB; i += SW<P>::kWaves) dma_b<P>(Bg, nks, 0, i, sB0 + i * 512, lane);
        as.load(0, r0, lane);
        __syncthreads();
        X3_STAMP(it, 1, __builtin_amdgcn_s_memtime());
        // k-steps in pairs so the two stage buffers are compile-time distinct
        // (no wait of a B fragment read on the other buffer's DMA)
        int ks = 0;
        for (; ks + 1 < nks; ks += 2) {
            k_step<NT, P>(acc, accx, as, r0, r1, Bg, nks, ks, sB0, sB1, wave, lane);
            k_step<NT, P>(acc, accx, as, r1, r0, Bg, nks, ks + 1, sB1, sB0, wave, lane);
        }
        if (ks < nks) k_step<NT, P>(acc, accx, as, r0, r1, Bg, nks, ks, sB0, sB1, wave, lane);
#pragma unroll
        for (int c = 0; c < NT; c++) acc[c] = x2_combine<P>(acc[c], accx[c]);
        X3_STAMP(it, 2, __builtin_amdgcn_s_memtime());

        // ---- epilogue (after the last k-step's barrier both stage buffers are free) ----
        if constexpr (EM == EM_TP) {
            epilogue_tp<NT>(acc, reinterpret_cast<float*>(sB0) + wave * 16 * 36, rt, M, N, ep, lane);
        } else if constexpr (EM == EM_FWD16) {  // (the host requires bufok)
            bres_epilogue<P, NT, EM>(acc, rt, cb * NT, NT, M, N, ep, crs, srs, sbias, lane);
        } else {
            if (ep.bufok && !ep.mask)  // buffer stores, one code path (bres_epilogue; tiles cb NT .. : even when bits)
                bres_epilogue<P, NT, EM>(acc, rt, cb * NT, NT, M, N, ep, crs, srs, sbias, lane);
            else
                epilogue_f32<NT, EM, P>(acc, rt, M, N, cb * 16 * NT, ep, sbias, lane);
        }
        // the next unit's DMA overwrites the epilogue slices: LDS reads done everywhere
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((15 << 0) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0) only
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        X3_STAMP(it, 3, __builtin_amdgcn_s_memtime());
        X3_STAMP(it, 5, __builtin_amdgcn_s_memrealtime());
    }
}

// ---------------------------------------------------------------------------
// The actor trunk's three ReLU layers in ONE launch for small M (the rollout's per-step forward at BASELINE
// configs[1]: 4,096 mazes = 8,192 rows; networks.py:35-36 under torch.no_grad, PPO.py:170-186):
//   h3 = relu(relu(relu(h0 W0^T + b0) W1^T + b1) W2^T + b2)
// At that size each layer on k_x3nt is a chain of k-steps at its launch floor (~13.6 us each, 160
// workgroups).  Here one workgroup owns 16 RT rows through all three layers.  The unit's h0 rows and each
// hidden layer's output stay in LDS, already in the precision's fragment planes (TP order, converted ONCE:
// h0 at staging, each hidden layer in its producer's epilogue), so a wave's A fragment is one lane-linear
// ds_read_b128 per plane and no wave repeats another's conversion.  Wave w owns the column-tile pair
// (2w, 2w + 1) -- one 32-column TP block of the output -- and tile 16 (N <= 272) is split by row tiles
// over waves 0, 5, 2 (SIMDs 0, 1, 2: no SIMD carries a whole third tile); the weight
// fragments come straight from the TP planes in L2 into registers, D k-steps ahead.  Only h0 is read from
// HBM and only h3 written.  Bit-identical to three k_x3nt launches (EM_F32, ReLU): the same conversion of
// the same fp32 values (store_piece = frag_f32 per value), the same MFMA sequence per output tile in k
// order (mma), the same epilogue arithmetic.  The weight-fragment loads follow the k_wgrad_rect rule
// (DESIGN.md section 4): their VGPR offsets are advanced in place and held live until consumed.
// ---------------------------------------------------------------------------
constexpr int kTrWaves = 8;
constexpr int kTrMaxN = 272;   // 17 column tiles: pairs 0..7 to waves 0..7, tile 16's row tiles to waves 0, 5, 2
constexpr int kTrMaxK0 = 512;  // padded width of the staged h0
constexpr int kTrSlice = 16 * 36;  // floats: a wave's [16 rows][32 columns] epilogue slice (stride 36)
struct TrunkArgs {
    const float* h0;
    const uint16_t* w[3];  // TP [N_l, K_l] in the precision P (K_1 = N_0, K_2 = N_1)
    const float* b[3];     // [N_l] or null
    float* out;            // fp32 [M, ldc]
    int lda, ldc, M, K0;
    int N[3];
    int bx;  // uint16 offset of the second activation buffer (bufH) from the first (bufX)
    // the fused heads + sampler (k_trunk3<.., HS = true>: k_head_sample's arithmetic on the LDS-resident h3)
    const float* hw;  // [6, N2] = [move_head.weight; mark_head.weight]
    const float* hb;  // [6]
    const uint8_t* masks;
    uint64_t seed, offset;
    const uint64_t* offset_dev;
    int8_t* act;
    float* logp;
    float* joint;
    float* logits;
    int hoff;  // float offset (from the LDS base) of the h3 rows, stride N2 + 4
};

#ifdef X3_STAMPS  // diagnostic builds only (tools/trunk_stamps.py): per-wave phase clocks of k_trunk3
__device__ unsigned long long g_tr_stamps[1024 * kTrWaves * 10];
#define TR_STAMP(slot, val)                                                                      \
    do {                                                                                         \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024)                                        \
            g_tr_stamps[(blockIdx.x * kTrWaves + (threadIdx.x >> 6)) * 10 + (slot)] = (val);     \
    } while (0)
#else
#define TR_STAMP(slot, val) \
    do {                    \
    } while (0)
#endif

// the column tile of a wave's accumulator slot c: 2 w, 2 w + 1, then 16 (one row tile of it, on waves 0, 5, 2)
__device__ __forceinline__ int trunk_tile(int wave, int c) { return c < 2 ? 2 * wave + c : 16; }
// the row tile of tile 16 on wave w (-1: none)
__device__ __forceinline__ int trunk_r16(int w) { return w == 0 ? 0 : w == 5 ? 1 : w == 2 ? 2 : -1; }

// one layer: dst = relu(src W^T + b) for the unit's 16 RT rows.  src: TP blocks (rt, ks) of the layer
// input in LDS (nks = ceil(K / 32) per row tile); dst: the same for the output (dstL), or the global output
// rows (dstL null).  NC: the wave's tiles; D: the weight prefetch depth in k-steps, nks % D == 0 -- both
// compile-time, and the k-loop is branch-free (groups of D steps, the last one peeled): branches in it made
// the compiler's wait counting fall back to waiting for every load in flight at each step.
template <int P, int RT, int D, int NC>
__device__ __forceinline__ void trunk_layer_n(const uint16_t* src, int K, const uint16_t* W, int N, const float* sb,
                                              uint16_t* dstL, float* slice, float* h3s, const TrunkArgs& ta, int m0,
                                              int wave, int lane, uint32_t& rm, int stamp) {
    constexpr int np = Prec<P>::kPlanes;
    constexpr uint32_t kBS = 2u * Prec<P>::kBlk;  // bytes per TP block (16 rows x 32 k, all planes)
    const int nks = rup(K, 32) / 32, tiles = (N + 15) / 16;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)W, (short)0, (int)((uint32_t)tiles * nks * kBS), 0x00020000);
    // slot s holds the fragments of the k-steps s, s + D, ...; ob[s][c]: the lane's byte offset of its
    // fragment piece in block (tile, next k-step of the slot), advanced in place after each use
    uint32_t ob[D][NC];
#pragma unroll
    for (int s = 0; s < D; s++)
#pragma unroll
        for (int c = 0; c < NC; c++) ob[s][c] = ((uint32_t)trunk_tile(wave, c) * nks + s) * kBS + 16u * lane;
    bf16x8 bq[D][NC][3];
    auto issue = [&](int s) {
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int p = 0; p < np; p++)
                bq[s][c][p] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, ob[s][c] + 1024u * p, 0, 0));
    };
    auto advance = [&](int s) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < NC; c++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(ob[s][c]) : "s"((uint32_t)D * kBS));
    };
    const bf16x8* const a8 = reinterpret_cast<const bf16x8*>(src) + lane;
    f32x4 acc[NC][RT], accx[NC][RT];
#pragma unroll
    for (int c = 0; c < NC; c++)
#pragma unroll
        for (int rt = 0; rt < RT; rt++) acc[c][rt] = accx[c][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // slot 2 (tile 16) covers one row tile r2 (trunk_r16); its A fragment picked by per-lane selects (from
    // threadIdx, not the wave-uniform value: a uniform select became a branch)
    static_assert(RT <= 3, "tile 16's row tiles: waves 0, 5, 2");
    const int r2 = trunk_r16(wave);
    const int r2v = trunk_r16((int)(threadIdx.x >> 6));
    // A fragments one k-step ahead (the last step re-reads its own block: no branch in the loop)
    bf16x8 an[RT][3];
    auto load_a = [&](int ks) {
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int q = 0; q < np; q++) an[rt][q] = a8[((rt * nks + ks) * np + q) * 64];
    };
    load_a(0);
    auto compute = [&](int ks, int s) {
        bf16x8 a[RT][3];
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int q = 0; q < np; q++) a[rt][q] = an[rt][q];
        load_a(min(ks + 1, nks - 1));
#pragma unroll
        for (int c = 0; c < (NC < 2 ? NC : 2); c++)
#pragma unroll
            for (int rt = 0; rt < RT; rt++) acc[c][rt] = mma<P>(a[rt], bq[s][c], acc[c][rt], accx[c][rt]);
        if constexpr (NC == 3) {
            bf16x8 a2[3];
#pragma unroll
            for (int q = 0; q < np; q++) {
                a2[q] = a[0][q];
#pragma unroll
                for (int rt = 1; rt < RT; rt++) a2[q] = r2v == rt ? a[rt][q] : a2[q];
            }
            acc[2][0] = mma<P>(a2, bq[s][2], acc[2][0], accx[2][0]);
        }
    };
#pragma unroll
    for (int s = 0; s < D; s++) issue(s);
    const int G = nks / D;
    for (int g = 0; g + 1 < G; g++) {
#pragma unroll
        for (int s = 0; s < D; s++) {
            compute(g * D + s, s);
            advance(s);
            issue(s);
        }
    }
#pragma unroll
    for (int s = 0; s < D; s++) compute((G - 1) * D + s, s);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < D; s++)
#pragma unroll
        for (int c = 0; c < NC; c++) asm volatile("" ::"v"(ob[s][c]));  // held to here (all loads consumed)
    TR_STAMP(stamp, __builtin_amdgcn_s_memtime());
    (void)stamp;
    // epilogue: the k_x3nt arithmetic (x2_combine; cscale 1; + bias; ReLU)
    const int rq = 4 * (lane >> 4);
    float x[NC][RT][4];
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const float bv = sb[16 * trunk_tile(wave, c) + (lane & 15)];
#pragma unroll
        for (int rt = 0; rt < (c < 2 ? RT : 1); rt++) {
            const f32x4 v = x2_combine<P>(acc[c][rt], accx[c][rt]);
            range_acc<P>(rm, v);
#pragma unroll
            for (int g = 0; g < 4; g++) x[c][rt][g] = fmaxf(v[g] + bv, 0.f);
        }
    }
    if (!dstL) {  // the last layer: fp32 rows of the output (16 lanes: 64 contiguous bytes of a row), and / or
                  // the unit's rows in LDS for the fused heads (h3s, rows of N + 4 floats)
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int col = 16 * trunk_tile(wave, c) + (lane & 15);
#pragma unroll
            for (int rt = 0; rt < (c < 2 ? RT : 1); rt++)
#pragma unroll
                for (int g = 0; g < 4; g++) {
                    const int rl = 16 * (c < 2 ? rt : r2) + rq + g, row = m0 + rl;
                    if (h3s && col < N) h3s[rl * (N + 4) + col] = x[c][rt][g];
                    if (ta.out && row < ta.M && col < N) ta.out[(size_t)row * ta.ldc + col] = x[c][rt][g];
                }
        }
        return;
    }
    // a hidden layer: each owned 32-column block (tile pair) through an fp32 slice into fragment order,
    // converted once (store_piece), into the next layer's input blocks; a missing tile of a pair is zeros.
    // x2 / x3: the slice is the destination block itself (2 KiB of fp32 fit its np KiB; the block is this
    // wave's until the layer's barrier), 32 floats a row with the float4 groups XOR-swizzled by row / 2 (a
    // 16-row column read then touches distinct banks); f16: the wave's own slice (rows of 36 floats).
    const int nksD = rup(N, 32) / 32, rr = lane & 15, ch = lane >> 4;
    auto sidx = [&](int row, int col) {
        return np >= 2 ? row * 32 + ((((col >> 2) ^ ((row >> 1) & 7))) << 2) + (col & 3) : row * 36 + col;
    };
    // slots c0, c1 (-1: no tile) of the wave's row tile rs -> block (rt, ks)
    auto put_block = [&](int ks, int rt, int rs, int c0, int c1) {
        uint16_t* const blk = dstL + (size_t)(rt * nksD + ks) * np * 512;
        float* const sl = np >= 2 ? reinterpret_cast<float*>(blk) : slice;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            sl[sidx(rq + g, lane & 15)] = c0 >= 0 ? x[c0 >= 0 ? c0 : 0][rs][g] : 0.f;
            sl[sidx(rq + g, 16 + (lane & 15))] = c1 >= 0 ? x[c1 >= 0 ? c1 : 0][rs][g] : 0.f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float4 v0 = *reinterpret_cast<const float4*>(sl + sidx(rr, kcol(ch, 0)));
        const float4 v1 = *reinterpret_cast<const float4*>(sl + sidx(rr, kcol(ch, 4)));
        const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // (in place: every lane has read the block before it is overwritten)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        store_piece<P>(v, 1.f, reinterpret_cast<uint4*>(blk) + lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the slice is rewritten next
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
        if (NC >= 1) put_block(wave, rt, rt, 0, NC >= 2 ? 1 : -1);
    if (NC >= 3) put_block(8, r2, 0, 2, -1);
    (void)nksD;
}

template <int P, int RT, int D>
__device__ __forceinline__ void trunk_layer(const uint16_t* src, int K, const uint16_t* W, int N, const float* sb,
                                            uint16_t* dstL, float* slice, float* h3s, const TrunkArgs& ta, int m0,
                                            int wave, int lane, uint32_t& rm, int stamp) {
    const int tiles = (N + 15) / 16, nks = rup(K, 32) / 32;
    // wave-uniform: slots 0, 1 = tiles 2 w, 2 w + 1; slot 2 = one row tile of tile 16 (N > 256)
    const int nc = 2 * wave >= tiles ? 0 : 2 * wave + 1 >= tiles ? 1 : (trunk_r16(wave) >= 0 && trunk_r16(wave) < RT && tiles > 16) ? 3 : 2;
    if (nks % D == 0) {
        if (nc == 3) trunk_layer_n<P, RT, D, 3>(src, K, W, N, sb, dstL, slice, h3s, ta, m0, wave, lane, rm, stamp);
        else if (nc == 2) trunk_layer_n<P, RT, D, 2>(src, K, W, N, sb, dstL, slice, h3s, ta, m0, wave, lane, rm, stamp);
        else if (nc == 1) trunk_layer_n<P, RT, D, 1>(src, K, W, N, sb, dstL, slice, h3s, ta, m0, wave, lane, rm, stamp);
    } else {  // (shapes other than the actor's: no prefetch beyond the next k-step)
        if (nc == 3) trunk_layer_n<P, RT, 1, 3>(src, K, W, N, sb, dstL, slice, h3s, ta, m0, wave, lane, rm, stamp);
        else if (nc == 2) trunk_layer_n<P, RT, 1, 2>(src, K, W, N, sb, dstL, slice, h3s, ta, m0, wave, lane, rm, stamp);
        else if (nc == 1) trunk_layer_n<P, RT, 1, 1>(src, K, W, N, sb, dstL, slice, h3s, ta, m0, wave, lane, rm, stamp);
    }
}

// HS: the actor's heads + the action draw fused after the last layer (PPO.py:170-186 with networks.py:38-41):
// k_head_sample's per-row arithmetic -- 8 lanes a row, the same fma order and butterfly, sample_row -- on the
// unit's h3 rows in LDS, so the draws, log-probs and logits equal the unfused trunk + k_head_sample's bit for
// bit; h3 is then written to HBM only when asked (ta.out)
template <int P, int RT, int D, bool HS>
__global__ __launch_bounds__(64 * kTrWaves) void k_trunk3(TrunkArgs ta) {
    constexpr int np = Prec<P>::kPlanes;
    constexpr int kIt = (RT * (kTrMaxK0 / 32) * 64 + 64 * kTrWaves - 1) / (64 * kTrWaves);  // h0 pieces per thread (max)
    constexpr int kHw = (6 * kTrMaxN + 64 * kTrWaves - 1) / (64 * kTrWaves);              // head weights per thread
    extern __shared__ __attribute__((aligned(16))) float tls[];
    float* const sbias = tls;                       // [3][kTrMaxN], zero past N
    float* const shw = tls + 3 * kTrMaxN;           // [6][N2]: the head weights (HS)
    float* const slices = shw + 6 * kTrMaxN;        // f16: [waves][kTrSlice] (x2 / x3 convert in place)
    uint16_t* const bufX = reinterpret_cast<uint16_t*>(slices + (np == 1 ? kTrWaves * kTrSlice : 0));  // h0, then layer 1's output
    uint16_t* const bufH = bufX + ta.bx;                                                 // layer 0's output
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int m0 = blockIdx.x * 16 * RT;
    TR_STAMP(0, __builtin_amdgcn_s_memtime());
    TR_STAMP(8, __builtin_amdgcn_s_memrealtime());
    {  // the unit's h0 rows as TP blocks (zero past M and past K0 up to the 32-column padding): every load
       // issued first, branch-free (out-of-range pieces read zeros through the buffer range check), their
       // offsets held until the data is consumed (the k_wgrad_rect rule)
        const int nks0 = rup(ta.K0, 32) / 32, npc = RT * nks0 * 64;
        const int nrows = min(16 * RT, ta.M - m0);
        const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(ta.h0 + (size_t)m0 * ta.lda), (short)0, (int)((uint32_t)nrows * ta.lda * 4u), 0x00020000);
        uint32_t off[kIt][2];
        float4 v[kIt][2];
#pragma unroll
        for (int j = 0; j < kIt; j++) {
            const int i = threadIdx.x + 64 * kTrWaves * j, l = i & 63, blk = i >> 6;  // blk = rt nks0 + ks
            const int rt = blk / nks0, ks = blk - nks0 * rt;
            const int row = 16 * rt + (l & 15), k0 = 32 * ks + 4 * (l >> 4);
#pragma unroll
            for (int h = 0; h < 2; h++)
                off[j][h] = (i < npc && row < nrows && k0 + 16 * h < ta.K0) ? 4u * ((uint32_t)row * ta.lda + k0 + 16 * h)
                                                                           : kBufOOB;
        }
#pragma unroll
        for (int j = 0; j < kIt; j++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const u32x4v d = __builtin_amdgcn_raw_buffer_load_b128(hrs, off[j][h], 0, 0);
                v[j][h] = make_float4(__uint_as_float(d.x), __uint_as_float(d.y), __uint_as_float(d.z),
                                      __uint_as_float(d.w));
            }
        // the biases: thread t < 272 loads column t of each layer's (zero past N_l, or for a null bias), in
        // flight together with h0
        const uint32_t boff = 4u * threadIdx.x;
        float bv[3];
#pragma unroll
        for (int l = 0; l < 3; l++) {
            const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)ta.b[l], (short)0, ta.b[l] ? 4 * ta.N[l] : 0, 0x00020000);
            bv[l] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, boff, 0, 0));
        }
        if (threadIdx.x < kTrMaxN) {
#pragma unroll
            for (int l = 0; l < 3; l++) sbias[kTrMaxN * l + threadIdx.x] = bv[l];
        }
        asm volatile("" ::"v"(boff));
        if constexpr (HS) {  // the head weights [6, N2], flat (k_head_sample's layout)
            const __amdgpu_buffer_rsrc_t wrs =
                __builtin_amdgcn_make_buffer_rsrc((void*)ta.hw, (short)0, 4 * 6 * ta.N[2], 0x00020000);
            uint32_t woff[kHw];
            float wv[kHw];
#pragma unroll
            for (int u = 0; u < kHw; u++) woff[u] = 4u * (threadIdx.x + 64 * kTrWaves * u);
#pragma unroll
            for (int u = 0; u < kHw; u++) wv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wrs, woff[u], 0, 0));
#pragma unroll
            for (int u = 0; u < kHw; u++) {
                const int e = threadIdx.x + 64 * kTrWaves * u;
                if (e < 6 * kTrMaxN) shw[e] = wv[u];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < kHw; u++) asm volatile("" ::"v"(woff[u]));
        }
#pragma unroll
        for (int j = 0; j < kIt; j++) {
            const int i = threadIdx.x + 64 * kTrWaves * j;
            if (i < npc) {
                const float e[8] = {v[j][0].x, v[j][0].y, v[j][0].z, v[j][0].w, v[j][1].x, v[j][1].y, v[j][1].z, v[j][1].w};
                store_piece<P>(e, 1.f, reinterpret_cast<uint4*>(bufX + (size_t)(i >> 6) * np * 512) + (i & 63));
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < kIt; j++)
#pragma unroll
            for (int h = 0; h < 2; h++) asm volatile("" ::"v"(off[j][h]));
    }
    __syncthreads();
    TR_STAMP(1, __builtin_amdgcn_s_memtime());
    float* const slice = slices + wave * kTrSlice;
    uint32_t rm = 0;  // the range guard (range_acc)
    trunk_layer<P, RT, D>(bufX, ta.K0, ta.w[0], ta.N[0], sbias, bufH, slice, nullptr, ta, m0, wave, lane, rm, 2);
    __syncthreads();
    TR_STAMP(3, __builtin_amdgcn_s_memtime());
    trunk_layer<P, RT, D>(bufH, ta.N[0], ta.w[1], ta.N[1], sbias + kTrMaxN, bufX, slice, nullptr, ta, m0, wave, lane,
                          rm, 4);
    __syncthreads();
    TR_STAMP(5, __builtin_amdgcn_s_memtime());
    float* const h3s = HS ? tls + ta.hoff : nullptr;  // (bufH, free in the last layer, or a region of its own)
    trunk_layer<P, RT, D>(bufX, ta.N[1], ta.w[2], ta.N[2], sbias + 2 * kTrMaxN, nullptr, slice, h3s, ta, m0, wave,
                          lane, rm, 6);
    range_note<P>(rm);
    if constexpr (HS) {  // k_head_sample's body on the LDS rows: 8 lanes a row, 16 RT rows (waves 0 .. 2 RT - 1)
        __syncthreads();
        constexpr int kL = 8;
        const int K = ta.N[2], sh = K + 4;
        if (threadIdx.x < kL * 16 * RT) {  // wave-uniform
            const int j = threadIdx.x % kL, rl = threadIdx.x / kL, row = m0 + rl;
            const bool valid = row < ta.M;
            float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (valid) {
                const float* hr = h3s + rl * sh;
                for (int c = 4 * j; c < K; c += 4 * kL) {
                    const float4 hv = *reinterpret_cast<const float4*>(hr + c);
#pragma unroll
                    for (int o = 0; o < 6; o++) {
                        const float4 wv = *reinterpret_cast<const float4*>(shw + o * K + c);
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
                for (int d = kL / 2; d > 0; d >>= 1) acc[o] += __shfl_xor(acc[o], d);
            }
            float lp = 0.f;
            if (valid && j == 0) {
                float l[5];
#pragma unroll
                for (int o = 0; o < 5; o++) l[o] = acc[o] + ta.hb[o];
                const float kl = acc[5] + ta.hb[5];
                int move, mark;
                const uint64_t off = ta.offset + (ta.offset_dev ? *ta.offset_dev : 0ull);
                lp = sample_row(l, kl, ta.masks + (size_t)row * MM_MASK_DIM, row, ta.seed, off, move, mark);
                ta.act[2 * row] = (int8_t)move;
                ta.act[2 * row + 1] = (int8_t)mark;
                if (ta.logp) ta.logp[row] = lp;
                if (ta.logits) {
#pragma unroll
                    for (int o = 0; o < 5; o++) ta.logits[(size_t)row * 6 + o] = l[o];
                    ta.logits[(size_t)row * 6 + 5] = kl;
                }
            }
            const float other = __shfl_down(lp, kL);  // rows 2i, 2i + 1: adjacent 8-lane groups (m0 even)
            if (ta.joint && valid && j == 0 && (row & 1) == 0) ta.joint[row >> 1] = lp + (row + 1 < ta.M ? other : 0.f);
        }
    }
    TR_STAMP(7, __builtin_amdgcn_s_memtime());
    TR_STAMP(9, __builtin_amdgcn_s_memrealtime());
}

// Backward of the actor heads into the last hidden layer (networks.py:38-41 +
// the ReLU of :36): dY[m, n] = (sum_j dz[m, j] W[j, n]) * bit(m, n), W [J, N]
// the concatenated head weights, bits the last forward GEMM's ReLU mask.  Same
// tile map as the GEMM epilogue (one wave per 16-row tile, lane l: rows
// 4 (l >> 4) + g, columns 16 c + (l & 15)), so the mask bits line up; also the
// per-tile column sums (the last layer's bias gradient, before the final sum).
// D16: dY stored fp16 as fp16(dY * oscale) (P_F16's pre-scaled input gradients; the sums stay fp32)
constexpr int kHeadsMaxJ = 8;
template <int NT, bool D16 = false>
__global__ __launch_bounds__(256) void k_heads_bwd(const float* __restrict__ dz, int J, const float* __restrict__ W,
                                                   const uint32_t* __restrict__ bits, int M, int N,
                                                   float* __restrict__ dy, float* __restrict__ colsum,
                                                   float oscale = 1.f) {
    __shared__ float sw[kHeadsMaxJ][16 * NT];
    {  // loads batched ahead of the LDS writes (one L2 round trip per workgroup); 256 threads
        constexpr int kN = kHeadsMaxJ * 16 * NT, kPer = (kN + 255) / 256;
        float t[kPer];
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            const int e = threadIdx.x + 256 * u, j = e / (16 * NT), n = e % (16 * NT);
            t[u] = (e < kN && j < J && n < N) ? W[(size_t)j * N + n] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kPer; u++) {
            const int e = threadIdx.x + 256 * u;
            if (e < kN) sw[e / (16 * NT)][e % (16 * NT)] = t[u];
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int rt = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (16 * rt >= M) return;
    const int rq = 4 * (lane >> 4);
    uint64_t rb = 0;  // D16: the range guard of the fp16 stores
    float z[4][kHeadsMaxJ];
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int row = 16 * rt + rq + g;
#pragma unroll
        for (int j = 0; j < kHeadsMaxJ; j++) z[g][j] = (row < M && j < J) ? dz[(size_t)row * J + j] : 0.f;
    }
    uint32_t b[kMaskWords];
#pragma unroll
    for (int w = 0; w < kMaskWords; w++) b[w] = bits[((size_t)rt * 64 + lane) * kMaskWords + w];
#pragma unroll
    for (int c = 0; c < NT; c++) {
        const int col = 16 * c + (lane & 15);
        float cs = 0.f;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int row = 16 * rt + rq + g, bit = 4 * c + g;
            float x = 0.f;
#pragma unroll
            for (int j = 0; j < kHeadsMaxJ; j++) x = fmaf(z[g][j], sw[j][col], x);
            if (!((b[bit >> 5] >> (bit & 31)) & 1u)) x = 0.f;
            if (row < M && col < N) {
                if constexpr (D16) {
                    const _Float16 h = (_Float16)(x * oscale);
                    range_val<P_F16>(rb, (float)h);
                    reinterpret_cast<_Float16*>(dy)[(size_t)row * N + col] = h;
                } else {
                    dy[(size_t)row * N + col] = x;
                }
                cs += x;
            }
        }
        cs += __shfl_xor(cs, 16);
        cs += __shfl_xor(cs, 32);
        if (lane < 16 && col < N) colsum[(size_t)rt * N + col] = cs;
    }
    if constexpr (D16) range_note_wave<P_F16>(rb);
}


// ---------------------------------------------------------------------------
// Weight gradient (see the header): dW [N, K] = cscale * sum_m (dscale dY[m, n]) X[m, k].
// Work unit = (row slice s, column block cb of <= 17 tiles); 8 waves; per
// 32-row step every thread loads (operand, column, 8-row chunk) pieces for the
// NEXT step into registers while the waves run the current step's MFMAs from
// LDS; then it converts them into the fragment images (bf16x3 split or scaled
// fp16) with one 16-byte LDS write per plane.  Wave w owns the contiguous run
// of output tiles w * TPW .. (row-major over (n-tile, k-tile)), so its A
// fragment is re-read only when the run crosses an n-tile.  Each unit writes
// its partial [N, K] to ws[s]; mm_sum_leading sums the slices in order.
// ---------------------------------------------------------------------------
constexpr int kWgWaves = 8;
constexpr int kWgThreads = 64 * kWgWaves;
constexpr int kWgMaxT = 17;                                             // tiles per side of a unit
constexpr int kWgPer = (64 * 2 * kWgMaxT + kWgThreads - 1) / kWgThreads;  // pieces per thread and step

template <int P, int TPW>
__global__ __launch_bounds__(kWgThreads) void k_wgrad(const float* __restrict__ dy, int lddy, float dscale,
                                                      const float* __restrict__ x, int ldx, int M, int N, int K,
                                                      int TN, int NTK, int tpw, int rows, int nslices, int ncb,
                                                      float cscale, float* __restrict__ ws) {
    constexpr int kB = Prec<P>::kBlk;
    constexpr int np = Prec<P>::kPlanes;
    // two image sets [A: TN tiles | B: NTK tiles] (dynamic LDS): step st's MFMAs read set st & 1 while the
    // waves convert step st + 1 into the other set -- one barrier per step
    extern __shared__ __attribute__((aligned(16))) uint16_t img[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware: units u and u + 8 (one XCD) are the column blocks of one slice (its dY rows shared in L2)
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int s = (slot / ncb) * 8 + xcd, cb = slot % ncb;
    if (s >= nslices) return;  // the whole workgroup
    const int m_begin = s * rows, nrows = min(M, m_begin + rows) - m_begin;
    const int col0 = cb * NTK * 16;
    const int wA = TN * 16, wB = NTK * 16;  // staged columns per operand
    const int itemsA = 4 * wA, items = itemsA + 4 * wB;  // itemsA = 64 TN: a piece's operand is wave-uniform
    const int set = (TN + NTK) * kB;                     // uint16 per image set
    const float* const baseA = dy + (size_t)m_begin * lddy;
    const float* const baseB = x + (size_t)m_begin * ldx + col0;

    // loop-invariant per piece q: first row inside a step (8c), element offset of (8c, column) from the
    // operand's slice base, validity, and the LDS destination of its fragment piece
    int r8[kWgPer], goff[kWgPer], loff[kWgPer];
    bool ok[kWgPer];
#pragma unroll
    for (int q = 0; q < kWgPer; q++) {
        const int e = threadIdx.x + kWgThreads * q;
        const bool isA = e < itemsA;
        const int e2 = isA ? e : e - itemsA, w = isA ? wA : wB;
        const int c = e2 / w, j = e2 - c * w;  // 8-row chunk, column: consecutive threads, consecutive columns
        ok[q] = e < items && (isA ? j < N : col0 + j < K);
        r8[q] = 8 * c;
        goff[q] = ok[q] ? 8 * c * (isA ? lddy : ldx) + j : 0;
        loff[q] = (isA ? 0 : TN * kB) + (j >> 4) * kB + c * 128 + (j & 15) * 8;
    }

    float raw[kWgPer][8];
    auto load_piece = [&](int q, int r0) {  // rows r0 + 8c .. + 7 of the slice
        const bool isA = threadIdx.x + kWgThreads * q < itemsA;  // wave-uniform
        const int ld = isA ? lddy : ldx;
        const float* rowp = (isA ? baseA : baseB) + (size_t)r0 * ld;  // uniform
        int o = goff[q];
        asm volatile("" : "+v"(o));  // per step: not 40 loop-invariant addresses held in registers
        const int lim = nrows - r0 - r8[q];
#pragma unroll
        for (int i = 0; i < 8; i++) {
#ifdef WG_NO_GLOAD  // diagnostic builds only: no global loads
            raw[q][i] = ok[q] ? (float)(r0 + i) : 0.f;
#else
            raw[q][i] = (ok[q] && i < lim) ? rowp[o + i * ld] : 0.f;
#endif
        }
    };
    auto store_piece_q = [&](int q, uint16_t* dst_set) {
        if (threadIdx.x + kWgThreads * q < items) {
            const bool isA = threadIdx.x + kWgThreads * q < itemsA;
            store_piece<P>(raw[q], isA ? dscale : 1.f, reinterpret_cast<uint4*>(dst_set + loff[q]));
        }
    };
    auto lds_barrier = [&]() {  // LDS writes visible, no wait for the register prefetch (vmcnt)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((15 << 0) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0) only
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    f32x4 acc[TPW], accx[TPW];
#pragma unroll
    for (int u = 0; u < TPW; u++) acc[u] = accx[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    // wave w: the run of tiles w * tpw .. + tpw - 1 (row-major over (n-tile, k-tile)), balanced
    const int ntiles = TN * NTK, first = wave * tpw, last = min(ntiles, first + tpw);
    const int tn0 = first / NTK, tk0 = first - tn0 * NTK;
    const int nsteps = (nrows + 31) / 32;
#pragma unroll
    for (int q = 0; q < kWgPer; q++) load_piece(q, 0);
#pragma unroll
    for (int q = 0; q < kWgPer; q++) store_piece_q(q, img);
    if (nsteps > 1) {
#pragma unroll
        for (int q = 0; q < kWgPer; q++) load_piece(q, 32);
    }
    lds_barrier();
    // the conversion of the next step's pieces is spread over the tile loop (VALU beside the MFMAs)
    constexpr int kEvery = TPW >= kWgPer ? TPW / kWgPer : 1;
    for (int st = 0; st < nsteps; st++) {
        const uint16_t* cur = img + (st & 1) * set;
        uint16_t* nxt = img + ((st + 1) & 1) * set;
        const bool more = st + 1 < nsteps;
        int tn = tn0, tk = tk0, curtn = -1;
        bf16x8 a[3], b[3];
#pragma unroll
        for (int u = 0; u < TPW; u++) {
#ifndef WG_NO_MFMA  // diagnostic builds only
            if (first + u < last) {
                if (tn != curtn) {
                    curtn = tn;
                    const bf16x8* pa = reinterpret_cast<const bf16x8*>(cur + tn * kB) + lane;
#pragma unroll
                    for (int q = 0; q < np; q++) a[q] = pa[64 * q];
                }
                const bf16x8* pb = reinterpret_cast<const bf16x8*>(cur + TN * kB + tk * kB) + lane;
#pragma unroll
                for (int q = 0; q < np; q++) b[q] = pb[64 * q];
                acc[u] = mma<P>(a, b, acc[u], accx[u]);
            }
            if (++tk == NTK) {
                tk = 0;
                tn++;
            }
#endif
            if (more && u % kEvery == 0 && u / kEvery < kWgPer) store_piece_q(u / kEvery, nxt);
        }
        if (more) {
#pragma unroll
            for (int q = TPW / kEvery; q < kWgPer; q++) store_piece_q(q, nxt);  // (TPW < kWgPer)
            if (st + 2 < nsteps) {
#pragma unroll
                for (int q = 0; q < kWgPer; q++) load_piece(q, 32 * (st + 2));  // a whole step ahead
            }
        }
        lds_barrier();  // set st & 1 read by every wave, set (st + 1) & 1 written
    }
    float* out = ws + (size_t)s * N * K;
    int tn = tn0, tk = tk0;
    uint32_t rm = 0;  // the range guard (range_acc)
#pragma unroll
    for (int u = 0; u < TPW; u++) {
        acc[u] = x2_combine<P>(acc[u], accx[u]);
        range_acc<P>(rm, acc[u]);  // (tiles past `last` were never accumulated: zeros)
        if (first + u < last) {
            const int col = col0 + 16 * tk + (lane & 15);
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int row = 16 * tn + 4 * (lane >> 4) + g;
                if (row < N && col < K) out[(size_t)row * K + col] = acc[u][g] * cscale;
            }
        }
        if (++tk == NTK) {
            tk = 0;
            tn++;
        }
    }
    range_note<P>(rm);
}

// Structured form of k_wgrad for the shapes the actor and critic use (TN, NTK
// compile-time): wave w owns the rectangle of n-tiles RN w .. RN w + RN - 1
// by all NTK k-tiles (its RN A fragments held in registers, each B fragment
// read once and used RN times, the next k-tile's B fragments read while the
// current ones feed the MFMAs), plus its share of the leftover n-tiles
// (TN - 8 RN rows of NTK tiles, dealt round-robin: A and B read per tile).
// No runtime branch in the MFMA loop.  Staging, double-buffered images,
// partials and the reduction are those of k_wgrad.
// a staged value from its dword: fp32 (esz 4), or the fp16 half at bit offset sh (esz 2) -- selects, no branch
__device__ __forceinline__ float wg_val16(uint32_t d, uint32_t sh, bool h16) {
    const float h = (float)__builtin_bit_cast(_Float16, (unsigned short)(d >> sh));
    return h16 ? h : __uint_as_float(d);
}

// XB: bytes per X element -- 4 (fp32) or 2 (fp16: P_F16's stored activations, and the heads' x3 weight
// gradient over them; fp16 values are exact in fp32, so the staging is that of their fp32 values)
// AB: bytes per dY element -- 4, or 2 (P_F16's input gradients stored fp16 and pre-scaled: dscale 1)
template <int P, int TN, int NTK, int XB = 4, int AB = 4>
__global__ __launch_bounds__(kWgThreads) void k_wgrad_rect(const float* __restrict__ dy, int lddy, float dscale,
                                                           const float* __restrict__ x, int ldx, int M, int N, int K,
                                                           int rows, int nslices, int ncb, float cscale,
                                                           float* __restrict__ ws) {
    static_assert(XB == 4 || (XB == 2 && P != P_X2), "fp16 X: P_F16 / P_X3");
    static_assert(AB == 4 || (AB == 2 && P == P_F16), "fp16 dY: P_F16");
    constexpr bool k16 = XB == 2 || AB == 2;  // some operand fp16: dword loads + half selects
    constexpr int kB = Prec<P>::kBlk;
    constexpr int np = Prec<P>::kPlanes;
    constexpr int RN = TN / kWgWaves;                               // n-tiles per wave in the rectangle
    constexpr int kRem = (TN - kWgWaves * RN) * NTK;                // leftover tiles
    constexpr int EX = (kRem + kWgWaves - 1) / kWgWaves;            // leftover tiles per wave (max)
    constexpr int kSet = (TN + NTK) * kB;                           // uint16 per image set
    constexpr int itemsA = 64 * TN, items = itemsA + 64 * NTK;      // staged pieces per step
    constexpr int kPer = (items + kWgThreads - 1) / kWgThreads;
    extern __shared__ __attribute__((aligned(16))) uint16_t img[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int s = (slot / ncb) * 8 + xcd, cb = slot % ncb;
    if (s >= nslices) return;  // the whole workgroup
    const int m_begin = s * rows, nrows = min(M, m_begin + rows) - m_begin;
    const int col0 = cb * NTK * 16;
    const void* const baseA = reinterpret_cast<const char*>(dy) + (size_t)m_begin * lddy * AB;
    const void* const baseB = reinterpret_cast<const char*>(x) + ((size_t)m_begin * ldx + col0) * XB;

    // loads through one buffer resource per piece slot q over the slice's rows (loop-invariant, built once),
    // the step's row offset added to the lane's VGPR offset -- no per-element branch or 64-bit address.
    // EVERY OFFSET IS IN RANGE: lanes whose column is past N / K read the slice's first element (their
    // values only reach output rows >= N / columns >= K, which are never stored: an MFMA output element
    // depends on its own A row and B column only), and the rows past the slice in its last, partial step
    // read it too and are zeroed by a select.  (The round-4 forms, with out-of-range offsets or without,
    // returned zeros in the last quarter-wave of some loads; the cause was operand registers rewritten
    // while the loads were in flight: see the pinned operands below.)
    int loff[kPer], r8q[kPer], ldq[kPer];
    uint32_t voff[kPer], eszq[kPer];  // eszq: bytes per element of the slot's operand (wave-uniform)
    uint32_t hsh[kPer];               // XB 2, B slots: the bit offset of the lane's half in its dword
    bool h16q[kPer];
    __amdgpu_buffer_rsrc_t rsq[kPer];
#pragma unroll
    for (int q = 0; q < kPer; q++) {
        const int e = threadIdx.x + kWgThreads * q;
        const bool isA = e < itemsA;
        const int e2 = isA ? e : e - itemsA, w = isA ? 16 * TN : 16 * NTK;
        const int c = e2 / w, j = e2 - c * w;
        const bool ok = e < items && (isA ? j < N : col0 + j < K);
        // fp16 X (XB 2): every load is a dword (one instruction form for A and B slots, no branch between
        // load forms -- two forms merged at a branch made the compiler wait on each batch); the lane takes
        // the half (j & 1) of the dword holding its element (ldx even: rows stay dword-aligned)
        voff[q] = ok ? (isA ? (uint32_t)AB * (uint32_t)(8 * c * lddy + j) & ~3u
                            : (uint32_t)XB * (uint32_t)(8 * c * ldx + j) & ~3u)
                     : 0u;
        h16q[q] = isA ? AB == 2 : XB == 2;  // per lane (from threadIdx, not readfirstlane): a select, not a branch
        hsh[q] = (h16q[q] && ok) ? 16u * (uint32_t)(j & 1) : 0u;
        loff[q] = (isA ? 0 : TN * kB) + (j >> 4) * kB + c * 128 + (j & 15) * 8;
        r8q[q] = 8 * c;
        // wave-uniform (itemsA = 64 TN), made scalar: a resource built from a divergent value becomes a
        // readfirstlane waterfall loop per load
        const bool isAu = __builtin_amdgcn_readfirstlane(threadIdx.x + kWgThreads * q) < itemsA;
        ldq[q] = isAu ? lddy : ldx;
        eszq[q] = isAu ? (uint32_t)AB : (uint32_t)XB;
        rsq[q] = __builtin_amdgcn_make_buffer_rsrc(isAu ? (void*)baseA : (void*)baseB, (short)0,
                                                   (int)(nrows * ldq[q] * eszq[q]), 0x00020000);
    }
    float raw[kPer][8];
#ifndef WG_OLDFORM
    // Every operand register of a staging load stays untouched until that load has completed (DESIGN.md
    // section 4, "The k_wgrad_rect zeros": a buffer load reads the operands of its last quarter-wave after
    // the wave has gone on, and a register rewritten in that window -- the compiler reuses a load's address
    // or offset register as soon as the load has issued -- gave lanes 48-63 zeros).  So: the lane's VGPR
    // offset ob[q] is advanced IN PLACE one step at a time, just before the next batch (by then the
    // previous batch has landed: its values were converted and stored); the row strides i ld are scalar
    // offsets built once; ob, the strides and the resources are held live to the end of the kernel.
    // x2 (235 VGPRs of accumulators and pieces): one VGPR offset per slot plus eight scalar row offsets
    // i ld 4; x3 / f16 (VGPR room, and the scalar form spilled SGPRs in the f16 kernels -- a reloaded
    // spill is a fresh temporary, rewritten right after the load): one VGPR offset per (slot, row i),
    // each advanced in place.  tools/check_wgrad_operands.py checks the ISA of every instantiation.
    constexpr bool kSOff = P == P_X2;  // (x2 never has fp16 operands)
    constexpr int kNv = kSOff ? 1 : 8;
    uint32_t ob[kPer][kNv], sri[kPer][8];
#pragma unroll
    for (int q = 0; q < kPer; q++) {
#pragma unroll
        for (int i = 0; i < kNv; i++) ob[q][i] = voff[q] + eszq[q] * (uint32_t)(i * ldq[q]);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr (kSOff) asm volatile("s_mul_i32 %0, %1, %2" : "=s"(sri[q][i]) : "s"(ldq[q]), "n"(4 * i));
            else sri[q][i] = 0u;
        }
    }
    auto hold_operands = [&]() {
#pragma unroll
        for (int q = 0; q < kPer; q++) {
            asm volatile("" ::"s"(rsq[q]));
#pragma unroll
            for (int i = 0; i < kNv; i++) asm volatile("" ::"v"(ob[q][i]));
            if constexpr (kSOff) {
#pragma unroll
                for (int i = 0; i < 8; i++) asm volatile("" ::"s"(sri[q][i]));
            }
        }
    };
    auto load_piece = [&](int q, int r0) {  // rows r0 + 8c .. + 7 of the slice; r0 = 0, 32, 64, .. in turn
        const int ld = ldq[q];
        if (r0 > 0) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < kNv; i++)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(ob[q][i]) : "s"(32 * (int)eszq[q] * ld));
        }
        if (r0 + 32 <= nrows) {  // a whole step inside the slice (wave-uniform)
#pragma unroll
            for (int i = 0; i < 8; i++) {
#ifdef WG_NO_GLOAD  // diagnostic builds only: no global loads
                raw[q][i] = (float)(r0 + i);
#else
                {
                    const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(rsq[q], ob[q][kSOff ? 0 : i], sri[q][i], 0);
                    raw[q][i] = __uint_as_float(d);  // (fp16 X: the dword's bits; converted where consumed)
                }
#endif
            }
        } else {  // the slice's last, partial step: rows past the slice read its first element, zeroed; these
                  // loads' offsets are temporaries, so they are waited for here (once per slice at most; the
                  // previous batch has landed -- it was converted and stored just before -- so nothing is in
                  // flight while the temporaries live: the markers let tools/check_wgrad_operands.py skip them)
            asm volatile(";;wg-partial-begin");
            const int lim = nrows - r0 - r8q[q];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t o = i < lim ? ob[q][0] + eszq[q] * i * ld : 0u;
                const uint32_t d = __builtin_amdgcn_raw_buffer_load_b32(rsq[q], o, 0, 0);
                raw[q][i] = i < lim ? __uint_as_float(d) : 0.f;  // (fp16 X: bits, converted where consumed; 0 -> 0)
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
            asm volatile(";;wg-partial-end");
        }
    };
#else  // diagnostic builds: the round-4 form (offsets recomputed per batch, registers reused by the compiler)
    auto hold_operands = [&]() {};
    auto load_piece = [&](int q, int r0) {  // rows r0 + 8c .. + 7 of the slice
        const int ld = ldq[q];
        uint32_t o = voff[q] + 4u * (uint32_t)(r0 * ld);
        asm volatile("" : "+v"(o));
        if (r0 + 32 <= nrows) {  // a whole step inside the slice (wave-uniform)
#pragma unroll
            for (int i = 0; i < 8; i++) {
#ifdef WG_NO_GLOAD  // diagnostic builds only: no global loads
                raw[q][i] = (float)(r0 + i);
#else
                raw[q][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsq[q], o + 4u * i * ld, 0, 0));
#endif
            }
        } else {  // the slice's last, partial step: rows past the slice read its first element, zeroed
            const int lim = nrows - r0 - r8q[q];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const float v =
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsq[q], i < lim ? o + 4u * i * ld : 0u, 0, 0));
                raw[q][i] = i < lim ? v : 0.f;
            }
        }
    };
#endif
    auto store_piece_q = [&](int q, uint16_t* dst_set) {
        if (threadIdx.x + kWgThreads * q < items) {
            const bool isA = threadIdx.x + kWgThreads * q < itemsA;
            if constexpr (k16) {  // the fp16 halves of the loaded dwords, here where they are consumed (a
                                  // conversion right after the load would wait for it there)
                float v[8];
#pragma unroll
                for (int i = 0; i < 8; i++) v[i] = wg_val16(__float_as_uint(raw[q][i]), hsh[q], h16q[q]);
                store_piece<P>(v, isA ? dscale : 1.f, reinterpret_cast<uint4*>(dst_set + loff[q]));
            } else {
                store_piece<P>(raw[q], isA ? dscale : 1.f, reinterpret_cast<uint4*>(dst_set + loff[q]));
            }
        }
    };
    auto lds_barrier = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((15 << 0) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0) only
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto frag = [&](const uint16_t* tile, bf16x8 (&f)[3]) {
        const bf16x8* p = reinterpret_cast<const bf16x8*>(tile) + lane;
#pragma unroll
        for (int q = 0; q < np; q++) f[q] = p[64 * q];
    };

    f32x4 acc[RN * NTK + EX], accx[RN * NTK + EX];
#pragma unroll
    for (int u = 0; u < RN * NTK + EX; u++) acc[u] = accx[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nsteps = (nrows + 31) / 32;
#pragma unroll
    for (int q = 0; q < kPer; q++) load_piece(q, 0);
#pragma unroll
    for (int q = 0; q < kPer; q++) store_piece_q(q, img);
    if (nsteps > 1) {
#pragma unroll
        for (int q = 0; q < kPer; q++) load_piece(q, 32);
    }
    lds_barrier();
    // conversion of the next step's pieces: piece q at slot q * kEvery of the tile loop (VALU beside the
    // MFMAs), the rest after it
    constexpr int kSlots = (RN > 0 ? NTK : 0) + EX;
    constexpr int kEvery = kSlots >= kPer ? kSlots / kPer : 1;
    // fp16 (cheap conversion, short MFMA phase): all after the MFMAs, so the loads issued at the end of the
    // previous step get the whole MFMA phase to arrive (measured: 264 x 460 415 -> 366 us; x3: 765 -> 788)
#if !defined(WG_NO_MFMA) && !defined(WG_CONV_LATE)
    constexpr int kDone = P != P_X3 ? 0 : ((kSlots + kEvery - 1) / kEvery < kPer ? (kSlots + kEvery - 1) / kEvery : kPer);
#else
    constexpr int kDone = 0;
#endif
    // Ping-pong (x2 / f16, whose conversion runs after the MFMAs): waves 4-7 -- each sharing its SIMD with one
    // of waves 0-3 -- convert and stage the next step's pieces BEFORE their MFMAs, waves 0-3 after theirs, so
    // on every SIMD one wave's MFMAs overlap the other's conversion VALU instead of both waves running the
    // same phase at once.  The two halves touch different image sets (cur is read, nxt written), and each
    // wave's loads still get one MFMA phase to arrive.  Measured slower (tools/ab_libs.py, 419,430 rows:
    // x2 264 x 264 295 -> 311 us, 264 x 460 484 -> 532 us, f16 264 x 460 352 -> 368 us; x3 unchanged), so
    // WG_PINGPONG=0 (every wave MFMAs first) is the default.
#ifndef WG_PINGPONG
#define WG_PINGPONG 0
#endif
    const bool conv_first = WG_PINGPONG && kDone == 0 && wave >= kWgWaves / 2;
    for (int st = 0; st < nsteps; st++) {
        const uint16_t* cur = img + (st & 1) * kSet;
        uint16_t* nxt = img + ((st + 1) & 1) * kSet;
        const bool more = st + 1 < nsteps;
        auto conv_at = [&](int slot) {
            if (kDone > 0 && more && slot % kEvery == 0 && slot / kEvery < kPer) store_piece_q(slot / kEvery, nxt);
        };
        auto stage_next = [&]() {  // the next step's pieces into nxt, then the loads of the step after it
            if (more) {
#pragma unroll
                for (int q = kDone; q < kPer; q++) store_piece_q(q, nxt);
                if (st + 2 < nsteps) {
#pragma unroll
                    for (int q = 0; q < kPer; q++) load_piece(q, 32 * (st + 2));
                }
            }
        };
        if (conv_first) stage_next();
#ifndef WG_NO_MFMA
        if constexpr (RN > 0) {
            bf16x8 a[RN][3], b[2][3];
#pragma unroll
            for (int r = 0; r < RN; r++) frag(cur + (RN * wave + r) * kB, a[r]);
            frag(cur + TN * kB, b[0]);
#pragma unroll
            for (int tk = 0; tk < NTK; tk++) {
                if (tk + 1 < NTK) frag(cur + (TN + tk + 1) * kB, b[(tk + 1) & 1]);  // next k-tile, ahead
#pragma unroll
                for (int r = 0; r < RN; r++)
                    acc[r * NTK + tk] = mma<P>(a[r], b[tk & 1], acc[r * NTK + tk], accx[r * NTK + tk]);
                conv_at(tk);
            }
        }
#pragma unroll
        for (int e = 0; e < EX; e++) {
            int j = wave + kWgWaves * e;  // leftover tile j (clamped: a duplicate, not stored)
            j = j < kRem ? j : kRem - 1;
            const int tn = kWgWaves * RN + j / NTK, tk = j % NTK;
            bf16x8 a1[3], b1[3];
            frag(cur + tn * kB, a1);
            frag(cur + (TN + tk) * kB, b1);
            acc[RN * NTK + e] = mma<P>(a1, b1, acc[RN * NTK + e], accx[RN * NTK + e]);
            conv_at((RN > 0 ? NTK : 0) + e);
        }
#endif
        if (!conv_first) stage_next();
        lds_barrier();
    }
    hold_operands();
    uint32_t rm = 0;  // the range guard (range_acc; the clamped duplicate leftover tiles included: same data)
#pragma unroll
    for (int u = 0; u < RN * NTK + EX; u++) {
        acc[u] = x2_combine<P>(acc[u], accx[u]);
        range_acc<P>(rm, acc[u]);
    }
    range_note<P>(rm);
    float* out = ws + (size_t)s * N * K;
    auto put = [&](const f32x4& v, int tn, int tk) {
        const int col = col0 + 16 * tk + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int row = 16 * tn + 4 * (lane >> 4) + g;
            if (row < N && col < K) out[(size_t)row * K + col] = v[g] * cscale;
        }
    };
#pragma unroll
    for (int r = 0; r < RN; r++)
#pragma unroll
        for (int tk = 0; tk < NTK; tk++) put(acc[r * NTK + tk], RN * wave + r, tk);
#pragma unroll
    for (int e = 0; e < EX; e++) {
        const int j = wave + kWgWaves * e;
        if (j < kRem) put(acc[RN * NTK + e], kWgWaves * RN + j / NTK, j % NTK);
    }
}

// k_wgrad_dma (round 6): k_wgrad_rect<P_X2, TN, NTK> with the staging taken off the registers and the dY
// conversion moved under the MFMAs.
//
// Why (419,430 rows, 264 x 264; phase-removed builds timed by tools/bench_wgrad_dma.py): k_wgrad_rect takes
// ~300 us.  Alone, its MFMA phase takes ~96 us (the x2 floor, 3 f16 MFMAs per product), the operand streaming
// ~132 us (5.3 TB/s) and the conversion to fp16 planes ~71 us; the kernel runs them one after the other per
// 32-row step, with one step of loads in flight in registers.
//
// Here: (1) the raw fp32 rows go HBM -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) into TWO raw stages,
// [A: 32 rows x 16 TN][B: 32 rows x 16 NTK] row-major, so two steps' bytes are in flight.  Rows past the
// slice read past the resource's num_records and land as zeros; columns past N / K read finite neighbours
// that reach only output rows / columns that are never stored.  (2) One fragment image (k_wgrad_rect's
// layout).  Its A part (the TN dY tiles, 2/3 of the image) is needed only for the waves' A fragments, which
// they load into registers at the start of a step (the leftover tiles' one A fragment included); after a
// barrier the A part is free, and the next step's dY pieces are converted into it between the MFMAs of this
// step, which read only the B part.  The X pieces (1/3) are converted after the MFMAs.  Per step: A
// fragments; [wait for this wave's DMAs of the next step; barrier]; MFMAs + the dY conversion; barrier; the X
// conversion; barrier; the freed raw stage takes the DMA of the step after next.
//
// The DMA is inline asm (dma16): the compiler then sees no LDS write it cannot place, and inserts none of
// its own vmcnt waits before LDS accesses (through the stage pointers it made every conversion wait for
// every DMA in flight: vmcnt(0), one step of prefetch).  The kernel waits for its DMAs itself, by count.
// Operand rule: an in-flight DMA's offset VGPR is never rewritten (one offset set per
// raw stage, advanced in place by two steps after its previous DMA was waited for); its resource SGPRs are
// held for the whole kernel.  The MFMA order per output tile and the images are k_wgrad_rect's: the same
// partials, bit for bit.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t lds) {
    uint32_t save;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(save)
                 : "v"(voff), "s"(r), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// pair2 (x s -> the x2 (hi, lo) fp16 pair of two values) in NON-packed instructions, for conversions that
// run beside MFMAs: packed f32 VALU (v_pk_mul_f32 / v_pk_fma_f32, which the compiler SLP-forms from pair2's
// vector arithmetic) costs ~22-26 extra cycles per instruction next to an MFMA (MI355X_MICROARCH.md), plain
// VOP3 / VOP3P-mix instructions do not.  Same values as pair2: hi = RN16(x s); x s - hi exactly by one
// v_fma_mix_f32 reading hi's halves (x s is exact, s a power of two; the difference is exact, Sterbenz);
// times 2^11 exactly; RN16.  SCALED = false: s = 1 (no multiplies).
template <bool SCALED>
__device__ __forceinline__ void pair2_plain(float x0, float x1, float s, uint32_t& h, uint32_t& l) {
    float y0, y1;
    if constexpr (SCALED) {
        asm("v_mul_f32 %0, %4, %6\n\t"
            "v_mul_f32 %1, %5, %6\n\t"
            "v_cvt_pk_f16_f32 %2, %0, %1\n\t"
            "v_fma_mix_f32 %0, %4, %6, -%2 op_sel_hi:[0,0,1]\n\t"
            "v_fma_mix_f32 %1, %5, %6, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
            "v_mul_f32 %0, 0x45000000, %0\n\t"
            "v_mul_f32 %1, 0x45000000, %1\n\t"
            "v_cvt_pk_f16_f32 %3, %0, %1"
            : "=&v"(y0), "=&v"(y1), "=&v"(h), "=&v"(l)
            : "v"(x0), "v"(x1), "v"(s));
    } else {
        asm("v_cvt_pk_f16_f32 %2, %4, %5\n\t"
            "v_fma_mix_f32 %0, %4, 1.0, -%2 op_sel_hi:[0,0,1]\n\t"
            "v_fma_mix_f32 %1, %5, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
            "v_mul_f32 %0, 0x45000000, %0\n\t"
            "v_mul_f32 %1, 0x45000000, %1\n\t"
            "v_cvt_pk_f16_f32 %3, %0, %1"
            : "=&v"(y0), "=&v"(y1), "=&v"(h), "=&v"(l)
            : "v"(x0), "v"(x1));
        (void)s;
    }
}
template <bool SCALED>
__device__ __forceinline__ void store_piece_x2_plain(const float* v, float s, uint4* dst) {
    uint32_t hh[4], ll[4];
#pragma unroll
    for (int k = 0; k < 4; k++) pair2_plain<SCALED>(v[2 * k], v[2 * k + 1], s, hh[k], ll[k]);
    dst[0] = make_uint4(hh[0], hh[1], hh[2], hh[3]);
    dst[64] = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

template <int P, int TN, int NTK>
__global__ __launch_bounds__(kWgThreads) void k_wgrad_dma(const float* __restrict__ dy, int lddy, float dscale,
                                                          const float* __restrict__ x, int ldx, int M, int N, int K,
                                                          int rows, int nslices, int ncb, float cscale,
                                                          float* __restrict__ ws) {
    static_assert(P == P_X2, "k_wgrad_dma: the x2 weight gradients (fp32 operands)");
    constexpr int kB = Prec<P>::kBlk;
    constexpr int np = Prec<P>::kPlanes;
    constexpr int RN = TN / kWgWaves;
    constexpr int kRem = (TN - kWgWaves * RN) * NTK;
    constexpr int EX = (kRem + kWgWaves - 1) / kWgWaves;
    static_assert(RN > 0 && (kRem == 0 || TN - kWgWaves * RN == 1), "leftover tiles of one n-tile (one A fragment)");
    constexpr int kWA = 16 * TN, kWB = 16 * NTK;            // raw row widths (floats)
    constexpr int kRawA = 32 * kWA, kRaw = 32 * (kWA + kWB);  // floats
    constexpr int kImg = (TN + NTK) * kB;                   // uint16 per image
    constexpr int kInsA = kRawA / 256, kIns = kRaw / 256;   // 1-KiB DMA instructions per stage
    constexpr int kInsW = (kIns + kWgWaves - 1) / kWgWaves;  // per wave (max)
    constexpr int kInsWmin = kIns / kWgWaves;                // per wave (min)
    constexpr int itemsA = 64 * TN, itemsB = 64 * NTK;
    constexpr int kPerA = (itemsA + kWgThreads - 1) / kWgThreads, kPerB = (itemsB + kWgThreads - 1) / kWgThreads;
    static_assert((2 * kRaw * 4 + kImg * 2) <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float raw0[kRaw];
    __shared__ __attribute__((aligned(16))) float raw1[kRaw];
    __shared__ __attribute__((aligned(16))) uint16_t img[kImg];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int s = (slot / ncb) * 8 + xcd, cb = slot % ncb;
    if (s >= nslices) return;  // the whole workgroup
    const int m_begin = s * rows, nrows = min(M, m_begin + rows) - m_begin;
    const int col0 = cb * NTK * 16;
    __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(dy + (size_t)m_begin * lddy), (short)0, (int)(nrows * lddy * 4), 0x00020000);
    __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + (size_t)m_begin * ldx + col0), (short)0, (int)((nrows * ldx - col0) * 4), 0x00020000);
    asm volatile("" : "+s"(rsA));
    asm volatile("" : "+s"(rsB));

    // this wave's DMA instructions i = wave + 8 k: the lane's byte offset in the step of each offset set
    uint32_t ob[2][kInsW];
#pragma unroll
    for (int k = 0; k < kInsW; k++) {
        const int i = wave + kWgWaves * k;
        const int p = 64 * i + lane;
        const bool isA = i < kInsA;
        const int e = isA ? p : p - kRawA / 4;
        const int w4 = isA ? kWA / 4 : kWB / 4;
        const int r = e / w4, c4 = e - r * w4;
        const int ld = isA ? lddy : ldx;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            ob[t][k] = (uint32_t)(((32 * t + r) * ld + 4 * c4) * 4);
            asm volatile("" : "+v"(ob[t][k]));
        }
    }
    const uint32_t stepA = 2u * 32u * (uint32_t)lddy * 4u, stepB = 2u * 32u * (uint32_t)ldx * 4u;
    auto issue = [&](auto tc, int st) {  // the DMA of step st into raw stage T (offset set T)
        constexpr int T = decltype(tc)::value;
#ifdef WG_NO_DMA  // diagnostic builds only (wrong results): no loads
        return;
#endif
        const uint32_t base = lds_addr(T ? raw1 : raw0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < kInsW; k++) {
            const int i = wave + kWgWaves * k;  // wave-uniform
            if (i < kIns) {
                if (st >= 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(ob[T][k]) : "s"(i < kInsA ? stepA : stepB));
                dma16(i < kInsA ? rsA : rsB, ob[T][k], base + 1024u * (uint32_t)i);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    // this wave's DMAs of the stage converted next have landed; only the later stage's may be in flight
    auto wait_stage = [&](bool later_in_flight) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (later_in_flight) {
            if (wave < kIns % kWgWaves || kIns % kWgWaves == 0) {
                __builtin_amdgcn_s_waitcnt(0x0F70 | (kInsW & 15) | ((kInsW >> 4) << 14));
            } else {
                __builtin_amdgcn_s_waitcnt(0x0F70 | (kInsWmin & 15) | ((kInsWmin >> 4) << 14));
            }
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
    };
    auto barrier = [&]() {  // LDS writes visible to the workgroup (the DMAs: waited for above)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((15 << 0) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    // piece q of an operand: (8-row chunk c, column j) of this thread -> its raw words and image destination
    auto piece_conv = [&](const float* stage, bool isA, int e) {
#ifdef WG_NO_CONV  // diagnostic builds only (wrong results): no conversion
        return;
#endif
        const int w = isA ? kWA : kWB;
        const int c = e / w, j = e - c * w;
        const float* src = stage + (isA ? 0 : kRawA) + 8 * c * w + j;
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = src[i * w];
        const int loff = (isA ? 0 : TN * kB) + (j >> 4) * kB + c * 128 + (j & 15) * 8;
#ifdef WG_PACKED_CONV  // A/B: the packed-f32 form (store_piece)
        store_piece<P>(v, isA ? dscale : 1.f, reinterpret_cast<uint4*>(img + loff));
#else
        if (isA) store_piece_x2_plain<true>(v, dscale, reinterpret_cast<uint4*>(img + loff));
        else store_piece_x2_plain<false>(v, 1.f, reinterpret_cast<uint4*>(img + loff));
#endif
    };
    auto convA = [&](const float* stage, int q) {
        const int e = threadIdx.x + kWgThreads * q;
        if (e < itemsA) piece_conv(stage, true, e);
    };
    auto convB = [&](const float* stage) {
#pragma unroll
        for (int q = 0; q < kPerB; q++) {
            const int e = threadIdx.x + kWgThreads * q;
            if (e < itemsB) piece_conv(stage, false, e);
        }
    };
    auto frag = [&](const uint16_t* tile, bf16x8 (&f)[3]) {
        const bf16x8* p = reinterpret_cast<const bf16x8*>(tile) + lane;
#pragma unroll
        for (int q = 0; q < np; q++) f[q] = p[64 * q];
    };

    f32x4 acc[RN * NTK + EX], accx[RN * NTK + EX];
#pragma unroll
    for (int u = 0; u < RN * NTK + EX; u++) acc[u] = accx[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nsteps = (nrows + 31) / 32;
    constexpr std::integral_constant<int, 0> c0{};
    constexpr std::integral_constant<int, 1> c1{};
    issue(c0, 0);
    if (nsteps > 1) issue(c1, 1);
    wait_stage(nsteps > 1);
    barrier();
#pragma unroll
    for (int q = 0; q < kPerA; q++) convA(raw0, q);
    convB(raw0);
    barrier();
    if (nsteps > 2) issue(c0, 2);
    // WG_SPLIT_CONV=1: the dY pieces of the next step go between the MFMAs (piece q after k-tile kAtStride (q +
    // 1) - 1), the image's A part freed by a barrier after the A fragments are loaded.  Measured (419,430 rows):
    // 264 x 264 296-300 us against 282 us with the whole conversion after the MFMAs (0, the default); 264 x 460
    // 465 against 467 -- the conversion's VALU did not hide under the MFMAs (non-packed instructions or not)
#ifndef WG_SPLIT_CONV
#define WG_SPLIT_CONV 0
#endif
    constexpr bool kSplit = WG_SPLIT_CONV != 0;
    constexpr int kAtStride = NTK / (kPerA + 1) > 0 ? NTK / (kPerA + 1) : 1;
    auto step = [&](auto tc, int st) {  // step st; raw stage 1 - T holds step st + 1 (T = st & 1)
        constexpr int T = decltype(tc)::value;
        constexpr std::integral_constant<int, 1 - T> cn{};
        const float* nxt = T ? raw0 : raw1;
        const bool more = st + 1 < nsteps;
        bf16x8 a[RN][3], ax[3], b[2][3];
#pragma unroll
        for (int r = 0; r < RN; r++) frag(img + (RN * wave + r) * kB, a[r]);
        if constexpr (EX > 0) frag(img + kWgWaves * RN * kB, ax);  // the leftover tiles' n-tile
        frag(img + TN * kB, b[0]);
        if constexpr (kSplit) {
            if (more) wait_stage(st + 2 < nsteps);  // step st + 1's DMAs (this wave) landed
            barrier();  // every wave holds its A fragments: the image's A part is free; step st + 1's raw visible
        }
#ifndef WG_NO_MFMA
#pragma unroll
        for (int tk = 0; tk < NTK; tk++) {
            if (tk + 1 < NTK) frag(img + (TN + tk + 1) * kB, b[(tk + 1) & 1]);
#pragma unroll
            for (int r = 0; r < RN; r++)
                acc[r * NTK + tk] = mma<P>(a[r], b[tk & 1], acc[r * NTK + tk], accx[r * NTK + tk]);
            if constexpr (kSplit) {
#pragma unroll
                for (int q = 0; q < kPerA; q++)
                    if (tk == kAtStride * (q + 1) - 1 && more) convA(nxt, q);
            }
        }
#pragma unroll
        for (int e = 0; e < EX; e++) {
            int j = wave + kWgWaves * e;
            j = j < kRem ? j : kRem - 1;
            const int tk = j % NTK;
            bf16x8 b1[3];
            frag(img + (TN + tk) * kB, b1);
            acc[RN * NTK + e] = mma<P>(ax, b1, acc[RN * NTK + e], accx[RN * NTK + e]);
        }
#else
        if (more && kSplit) {
#pragma unroll
            for (int q = 0; q < kPerA; q++) convA(nxt, q);
        }
#endif
        if (more) {
            if constexpr (!kSplit) wait_stage(st + 2 < nsteps);  // step st + 1's DMAs (this wave) landed
            barrier();  // the MFMAs' reads of the image are done (and, unsplit, step st + 1's raw is visible)
            if constexpr (!kSplit) {
#pragma unroll
                for (int q = 0; q < kPerA; q++) convA(nxt, q);
            }
            convB(nxt);
            barrier();  // the image holds step st + 1; raw stage 1 - T is free
            if (st + 3 < nsteps) issue(cn, st + 3);
        }
    };
    for (int st = 0; st < nsteps; st += 2) {
        step(c0, st);
        if (st + 1 < nsteps) step(c1, st + 1);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // (every issued DMA was waited for before its conversion)
#pragma unroll
    for (int t = 0; t < 2; t++)
#pragma unroll
        for (int k = 0; k < kInsW; k++) asm volatile("" ::"v"(ob[t][k]));
    asm volatile("" ::"s"(rsA), "s"(rsB), "s"(stepA), "s"(stepB));
    uint32_t rm = 0;
#pragma unroll
    for (int u = 0; u < RN * NTK + EX; u++) {
        acc[u] = x2_combine<P>(acc[u], accx[u]);
        range_acc<P>(rm, acc[u]);
    }
    range_note<P>(rm);
    float* out = ws + (size_t)s * N * K;
    auto put = [&](const f32x4& v, int tn, int tk) {
        const int col = col0 + 16 * tk + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const int row = 16 * tn + 4 * (lane >> 4) + g;
            if (row < N && col < K) out[(size_t)row * K + col] = v[g] * cscale;
        }
    };
#pragma unroll
    for (int r = 0; r < RN; r++)
#pragma unroll
        for (int tk = 0; tk < NTK; tk++) put(acc[r * NTK + tk], RN * wave + r, tk);
#pragma unroll
    for (int e = 0; e < EX; e++) {
        const int j = wave + kWgWaves * e;
        if (j < kRem) put(acc[RN * NTK + e], kWgWaves * RN + j / NTK, j % NTK);
    }
}

// out[e] = sum over the row slices s of ws[s][e]: 16 groups of consecutive slices per element, each group's
// loads all in flight (the plain per-element loop over S = 256 slices was latency-bound: ~90 us), the
// groups then summed in order -- a fixed order, so the result is deterministic
__global__ __launch_bounds__(256) void k_wg_reduce(const float* __restrict__ ws, int S, long n,
                                                   float* __restrict__ out) {
    __shared__ float red[16][17];
    const int el = threadIdx.x & 15, g = threadIdx.x >> 4;
    const long e = blockIdx.x * 16L + el;
    const int per = (S + 15) / 16, s0 = g * per, s1 = min(S, s0 + per);
    float a = 0.f;
    if (e < n) {
        float v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = s0 + i < s1 ? ws[(long)(s0 + i) * n + e] : 0.f;
#pragma unroll
        for (int i = 0; i < 16; i++) a += v[i];
        for (int t = s0 + 16; t < s1; t++) a += ws[(long)t * n + e];  // S > 256
    }
    red[g][el] = a;
    __syncthreads();
    if (g == 0 && e < n) {
        float t = red[0][el];
#pragma unroll
        for (int k = 1; k < 16; k++) t += red[k][el];
        out[e] = t;
    }
}


// ---------------------------------------------------------------------------
// k_bres: C[M, N] = A[M, K] . B[N, K]^T with a column block of B RESIDENT in
// LDS for the whole launch (the forward and input-gradient GEMMs of the actor
// and critic, K <= 288 for x3).  Why (tools/x3_stamps.py on k_x3nt, 264 x 264,
// M = 419,430): k_x3nt streams B through LDS one k-step at a time, so its 16
// waves meet at a barrier every k-step and split A, read B and issue MFMAs in
// lock-step: 12.2k cycles per k-step against 6.5k of MFMA work, plus 15k of
// prologue and 21k of epilogue per 256-row unit that no other wave overlaps.
// Here each workgroup loads its block of B once (LDS-DMA), and after one
// barrier its waves run independently: a wave owns 32 rows (two row tiles)
// x <= CT column tiles at a time, loads and splits its own A (fp32, one
// k-step ahead), reads B fragments from LDS (each feeds both row tiles) and
// writes its outputs -- one wave's loads and stores overlap the others'
// MFMAs, and nothing waits for the slowest wave.
//
// Column blocks: B of a tile over the whole K is planes x (32-wide steps x 1
// KiB + a final 16-wide step x 512 B when K % 32 is 1..16, on the 16x16x16
// MFMA); the block is as many tiles as fit 160 KiB (x3, K = 264: 6 tiles ->
// 17 = 6 + 6 + 5; f16: all 17).  Workgroups of one XCD split over the blocks
// in proportion to their tiles, and the XCD takes every 8th 32-row unit, so
// the blocks re-reading a unit's A rows do it through the same L2.  Waves
// whose block is wider than CT take the sub-blocks of a unit in turn (A again
// from L1 / L2).
#ifndef BRES_WAVES
#define BRES_WAVES 12
#endif
#ifndef BRES_BPREF
#define BRES_BPREF 0
#endif
// waves per workgroup (one workgroup per CU: the B block fills LDS).  12 (168 registers per wave: no spills,
// the epilogue's row offsets and both A buffers held) measured 5-8% faster than 16 (128 registers, spilling)
// and than 8 (tools/bres_variants.sh + tools/bench_gemm_ab.py)
constexpr int kBresWaves = BRES_WAVES;

struct BresPlan {
    int xcds;   // XCDs the grid spreads over (8, or 1)
    int nblk;   // column blocks
    int ctb;    // column tiles of the widest block (the LDS the launch reserves)
    int tiles;  // column tiles of the output
    int tstart[9];  // block b: column tiles tstart[b] .. tstart[b + 1] - 1 (starts even when ReLU bits are involved)
    int nfull;  // 32-wide k-steps
    int half;   // 1: a final 16-wide k-step
    int first[9];  // per XCD: block b's workgroups are first[b] .. first[b + 1] - 1
};
constexpr int kBresMaxBlk = 8;

// A through a buffer resource: a load whose offset is past the buffer's end returns zeros, so the
// columns past K cost one select of the offset -- no branch, and no wait on the loaded value (a select
// on the value, or two load forms merged at a branch, made the compiler wait for each k-step's loads
// at the end of the step that issued them: no prefetch at all)

struct BresA {
    __amdgpu_buffer_rsrc_t rsrc;  // A: base, num_records = M lda 4 bytes
    uint32_t roff[2];             // this lane's row of row tile r (r < RT), + 4 kq bytes
};

// A for one 32-wide k-step: row tile r's lane row, columns k = 32 ks + 4 (l >> 4) .. +3 and +16 .. +19;
// zeros at columns >= K
template <int RT, int VW>
__device__ __forceinline__ void bres_load(const BresA& as, int ks, int K, int kq, float4 (&raw)[RT][2]) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int kk = 32 * ks + kq + 16 * h;
#pragma unroll
        for (int r = 0; r < RT; r++) {
            if constexpr (VW == 16) {  // fp16 A: the 4 halves k .. k + 3 as 8 bytes; r[.][0] packs both halves'
                const uint32_t o = as.roff[r] + 2u * (32 * ks + 16 * h);
                const u32x2v v = __builtin_amdgcn_raw_buffer_load_b64(as.rsrc, kk < K ? o : kBufOOB, 0, 0);
                if (h == 0) raw[r][0].x = __uint_as_float(v.x), raw[r][0].y = __uint_as_float(v.y);
                else raw[r][0].z = __uint_as_float(v.x), raw[r][0].w = __uint_as_float(v.y);
                raw[r][1] = make_float4(0.f, 0.f, 0.f, 0.f);
                continue;
            }
            const uint32_t o = as.roff[r] + 4u * (32 * ks + 16 * h);
            if constexpr (VW == 4) {
                const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(as.rsrc, kk < K ? o : kBufOOB, 0, 0);
                raw[r][h] = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                                        __uint_as_float(v.w));
            } else {
                const u32x2v a = __builtin_amdgcn_raw_buffer_load_b64(as.rsrc, kk < K ? o : kBufOOB, 0, 0);
                const u32x2v b = __builtin_amdgcn_raw_buffer_load_b64(as.rsrc, kk + 2 < K ? o + 8 : kBufOOB, 0, 0);
                raw[r][h] = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(b.x),
                                        __uint_as_float(b.y));
            }
        }
    }
}

// 8 fp32 -> the precision's A fragment planes (P_X3: exact three-way split; P_F16: x * s rounded)
template <int P, int VW>
__device__ __forceinline__ void bres_frag(const float4 (&r)[2], float s, bf16x8 (&a)[3]) {
    if constexpr (VW == 16) {  // fp16 A (P_F16, scale 1): the loaded halves are the fragment
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(__float_as_uint(r[0].x), __float_as_uint(r[0].y),
                                                     __float_as_uint(r[0].z), __float_as_uint(r[0].w)));
        return;
    }
#ifdef BRES_NO_SPLIT  // diagnostic builds only: the raw bits as fragments (no split VALU; outputs wrong)
    a[0] = __builtin_bit_cast(bf16x8, make_uint4(__float_as_uint(r[0].x), __float_as_uint(r[0].y),
                                                 __float_as_uint(r[1].x), __float_as_uint(r[1].y)));
    a[1] = __builtin_bit_cast(bf16x8, make_uint4(__float_as_uint(r[0].z), __float_as_uint(r[0].w),
                                                 __float_as_uint(r[1].z), __float_as_uint(r[1].w)));
    a[2] = a[0];
    return;
#endif
    if constexpr (P == P_X3) {
        uint32_t h[4], m[4], l[4];
        split2(r[0].x, r[0].y, h[0], m[0], l[0]);
        split2(r[0].z, r[0].w, h[1], m[1], l[1]);
        split2(r[1].x, r[1].y, h[2], m[2], l[2]);
        split2(r[1].z, r[1].w, h[3], m[3], l[3]);
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
        a[1] = __builtin_bit_cast(bf16x8, make_uint4(m[0], m[1], m[2], m[3]));
        a[2] = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
    } else if constexpr (P == P_X2) {
        uint32_t h[4], l[4];
        pair2(r[0].x, r[0].y, s, h[0], l[0]);
        pair2(r[0].z, r[0].w, s, h[1], l[1]);
        pair2(r[1].x, r[1].y, s, h[2], l[2]);
        pair2(r[1].z, r[1].w, s, h[3], l[3]);
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
        a[1] = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
    } else {
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(f16x2_rn(r[0].x * s, r[0].y * s), f16x2_rn(r[0].z * s, r[0].w * s),
                                                     f16x2_rn(r[1].x * s, r[1].y * s), f16x2_rn(r[1].z * s, r[1].w * s)));
    }
}

// the final 16-wide step: the 4 values k = 4 (l >> 4) .. +3 (the j < 4 half of a TP piece)
template <int P, int VW>
__device__ __forceinline__ void bres_frag16(const float4& r, float s, uint2 (&a)[3]) {
    if constexpr (VW == 16) {  // fp16 A: the j < 4 half is the first 8 bytes
        a[0] = make_uint2(__float_as_uint(r.x), __float_as_uint(r.y));
        return;
    }
    if constexpr (P == P_X3) {
        uint32_t h[2], m[2], l[2];
        split2(r.x, r.y, h[0], m[0], l[0]);
        split2(r.z, r.w, h[1], m[1], l[1]);
        a[0] = make_uint2(h[0], h[1]);
        a[1] = make_uint2(m[0], m[1]);
        a[2] = make_uint2(l[0], l[1]);
    } else if constexpr (P == P_X2) {
        uint32_t h[2], l[2];
        pair2(r.x, r.y, s, h[0], l[0]);
        pair2(r.z, r.w, s, h[1], l[1]);
        a[0] = make_uint2(h[0], h[1]);
        a[1] = make_uint2(l[0], l[1]);
    } else {
        a[0] = make_uint2(f16x2_rn(r.x * s, r.y * s), f16x2_rn(r.z * s, r.w * s));
    }
}

template <int P>
__device__ __forceinline__ f32x4 mma16(const uint2 (&a)[3], const uint2* b, f32x4 acc, f32x4& accx) {
    typedef __attribute__((ext_vector_type(4))) short s4;
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    if constexpr (P == P_X2) {
#define MM_H4(x) __builtin_bit_cast(h4, x)
        accx = __builtin_amdgcn_mfma_f32_16x16x16f16(MM_H4(a[1]), MM_H4(b[0]), accx, 0, 0, 0);
        accx = __builtin_amdgcn_mfma_f32_16x16x16f16(MM_H4(a[0]), MM_H4(b[1]), accx, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16f16(MM_H4(a[0]), MM_H4(b[0]), acc, 0, 0, 0);
#undef MM_H4
        return acc;
    }
    (void)accx;
    if constexpr (P == P_X3) {
#define MM_B16(x) __builtin_bit_cast(s4, x)
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(MM_B16(a[2]), MM_B16(b[0]), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(MM_B16(a[0]), MM_B16(b[2]), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(MM_B16(a[1]), MM_B16(b[1]), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(MM_B16(a[1]), MM_B16(b[0]), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(MM_B16(a[0]), MM_B16(b[1]), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(MM_B16(a[0]), MM_B16(b[0]), acc, 0, 0, 0);
#undef MM_B16
    } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h4, a[0]), __builtin_bit_cast(h4, b[0]), acc, 0,
                                                     0, 0);
    }
    return acc;
}

// Epilogue of one row tile x ctn column tiles (global tiles tg0 .. tg0 + ctn - 1; tg0 even).  ReLU bits:
// bit 4 c + g of the tile-local word = bit 4 (tg0 + c) + g of the row tile's mask, i.e. local byte m is
// global byte tg0 / 2 + m -- each block writes (EM_FWD) and reads (EM_BWD) whole bytes of its own tiles.
// one 32-wide k-step: cur -> fragments, step ks + 1 -> nxt (past the last step: offsets past K, zeros),
// the CT column tiles' MFMAs for both row tiles (each B fragment read feeds both)
template <int P, int CT, int RT, int VW, int D = 1>
__device__ __forceinline__ void bres_step(f32x4 (&acc)[RT][CT], f32x4 (&accx)[RT][CT], const float4 (&cur)[RT][2],
                                          float4 (&nxt)[RT][2],
                                          const BresA& as, int ks, int K, int kq, int ctb, int c0, int ctn,
                                          float ascale, const uint16_t* sF, int lane) {
    constexpr int np = Prec<P>::kPlanes;
    bf16x8 a[RT][3];
#pragma unroll
    for (int r = 0; r < RT; r++) bres_frag<P, VW>(cur[r], ascale, a[r]);
    bres_load<RT, VW>(as, ks + D, K, kq, nxt);  // D steps ahead (past the last step: zeros)
    int boff = ((ks * ctb + c0) * np) * 64 + lane;  // bf16x8 units
    asm volatile("" : "+v"(boff));                  // one base per step (not 18 hoisted addresses)
    const bf16x8* bp = reinterpret_cast<const bf16x8*>(sF) + boff;
#if BRES_BPREF
    // column c + 1's B fragments read while column c's MFMAs run
    bf16x8 bb[2][3];
#pragma unroll
    for (int q = 0; q < np; q++) bb[0][q] = bp[q * 64];
#pragma unroll
    for (int c = 0; c < CT; c++) {
        if (c < ctn) {  // wave-uniform (a guard, not a break: the loop stays fully unrolled, acc in registers)
            if (c + 1 < CT && c + 1 < ctn) {
#pragma unroll
                for (int q = 0; q < np; q++) bb[(c + 1) & 1][q] = bp[((c + 1) * np + q) * 64];
            }
#pragma unroll
            for (int r = 0; r < RT; r++) acc[r][c] = mma<P>(a[r], bb[c & 1], acc[r][c], accx[r][c]);
        }
    }
#else
#pragma unroll
    for (int c = 0; c < CT; c++) {
        if (c < ctn) {  // wave-uniform (a guard, not a break: the loop stays fully unrolled, acc in registers)
            bf16x8 bb[3];
#ifdef BRES_NO_BREAD  // diagnostic builds only: B fragments from the A registers (no LDS reads; outputs wrong)
#pragma unroll
            for (int q = 0; q < np; q++) bb[q] = a[0][(q + c) % 3];
#else
#pragma unroll
            for (int q = 0; q < np; q++) bb[q] = bp[(c * np + q) * 64];
#endif
#pragma unroll
            for (int r = 0; r < RT; r++) acc[r][c] = mma<P>(a[r], bb, acc[r][c], accx[r][c]);
        }
    }
#endif
}

template <int P, int CT, int RT, int EM, int VW>
__global__ __launch_bounds__(64 * kBresWaves) void k_bres(const float* __restrict__ A, int lda, float ascale,
                                                   const uint16_t* __restrict__ B, int M, int N, int K, int nks,
                                                   BresPlan pl, Epi ep) {
    static_assert(EM == EM_F32 || em_fwd(EM) || em_bwd(EM), "row-major outputs");
    static_assert(VW != 16 || P == P_F16, "fp16 A: P_F16");
    constexpr int np = Prec<P>::kPlanes;
    extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int X = pl.xcds, x = (int)blockIdx.x % X, wi = (int)blockIdx.x / X;
    X3_STAMP(0, 0, __builtin_amdgcn_s_memtime());
    X3_STAMP(0, 4, __builtin_amdgcn_s_memrealtime());
    if (wi >= pl.first[pl.nblk]) return;  // a surplus workgroup: uniform, before any barrier
    int b = 0;
    while (b + 1 < pl.nblk && wi >= pl.first[b + 1]) b++;
    const int t0 = pl.tstart[b], ctb = pl.tstart[b + 1] - t0;
    const int nfull = pl.nfull, half = pl.half;
    uint16_t* sF = smem;                               // [nfull][ctb][np][512]: a step's pieces at immediate offsets
    uint16_t* sT = smem + (size_t)ctb * nfull * np * 512;  // [ctb][np][256]: the 16-wide step
    float* sbias = reinterpret_cast<float*>(sT + ctb * np * 256 * half);

    // ---- the block of B -> LDS, once ----
    const int nF = ctb * nfull * np;
    for (int p = wave; p < nF; p += kBresWaves) {
        const int q = p % np, cks = p / np, c = cks % ctb, ks = cks / ctb;
        const uint4* src =
            reinterpret_cast<const uint4*>(B + ((size_t)(t0 + c) * nks + ks) * Prec<P>::kBlk + q * 512);
        __builtin_amdgcn_global_load_lds(src + lane, sF + (size_t)p * 512, 16, 0, 0);
    }
    if (half) {
        for (int p = wave; p < ctb * np; p += kBresWaves) {
            const int q = p % np, c = p / np;
            const uint2* src =
                reinterpret_cast<const uint2*>(B + ((size_t)(t0 + c) * nks + nfull) * Prec<P>::kBlk + q * 512);
            reinterpret_cast<uint2*>(sT + p * 256)[lane] = src[2 * lane];
        }
    }
    if (!em_bwd(EM) && ep.bias)
        for (int t = threadIdx.x; t < ctb * 16; t += 64 * kBresWaves) {
            const int col = 16 * t0 + t;
            sbias[t] = col < N ? ep.bias[col] : 0.f;
        }
    __syncthreads();  // vmcnt(0) + barrier: every wave's DMA pieces and writes landed
    X3_STAMP(0, 1, __builtin_amdgcn_s_memtime());

    // ---- independent waves ----
    // the workgroup takes groups of 16 consecutive 32-row units (512 rows, one per wave): groups
    // x + X (wb + nW t) for t = 0, 1, ...  -- each CU's loads and stores stay inside one ~0.5 MB stretch
    // of A and C at a time (scattering a workgroup's waves over the matrix measured ~2x slower)
    const int nu = (M + 16 * RT - 1) / (16 * RT);
    const int nW = pl.first[b + 1] - pl.first[b], wb = wi - pl.first[b];
    const int nsb = (ctb + CT - 1) / CT;
    const int kq = 4 * (lane >> 4);
    // gfx9 buffer resource word 3 0x00020000: 32-bit data format, raw (stride 0) addressing
    constexpr uint32_t aesz = VW == 16 ? 2u : 4u;  // VW 16: A is fp16 [M, lda]
    const __amdgpu_buffer_rsrc_t arsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)((size_t)M * lda * aesz), 0x00020000);
    const __amdgpu_buffer_rsrc_t crs =  // C [M, ldc]: rows past M past num_records
        __builtin_amdgcn_make_buffer_rsrc((void*)ep.c, (short)0, (int)((size_t)M * ep.ldc * (em_16(EM) ? 2 : 4)),
                                          0x00020000);
    const __amdgpu_buffer_rsrc_t srs =  // colsum [ceil(M / 16), N]
        __builtin_amdgcn_make_buffer_rsrc((void*)ep.colsum, (short)0, (int)((size_t)((M + 15) / 16) * N * 4),
                                          0x00020000);
    for (int t = 0;; t++) {
        const int u = (x + X * (wb + nW * t)) * kBresWaves + wave;
        if (u >= nu) break;
        BresA as;
        as.rsrc = arsrc;
#pragma unroll
        for (int r = 0; r < RT; r++) {
#ifdef BRES_ROW0  // diagnostic builds only: every unit reads the first 32 rows (A L2-resident; outputs wrong)
            const int row = min(16 * r + (lane & 15), M - 1);
#else
            const int row = min(16 * (RT * u + r) + (lane & 15), M - 1);  // rows past M: computed, not stored
#endif
            as.roff[r] = aesz * ((uint32_t)row * (uint32_t)lda + (uint32_t)kq);
        }
        for (int s = 0; s < nsb; s++) {
            const int c0 = s * CT, ctn = min(CT, ctb - c0);
            f32x4 acc[RT][CT], accx[RT][CT];  // accx: P_X2's cross terms (unused otherwise)
#pragma unroll
            for (int r = 0; r < RT; r++)
#pragma unroll
                for (int c = 0; c < CT; c++) acc[r][c] = accx[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
            // A register buffers: step ks splits cur and loads a later step into another buffer, so the
            // loads stay in flight over whole steps (one buffer made the compiler copy at the loop end,
            // waiting for the loads it had just issued).  RT = 2 (x3): two buffers, one step ahead; RT = 1
            // (f16, bound by its A loads): three buffers, two steps ahead.
            uint2 a4[RT][3];
            if constexpr (RT == 1) {
                float4 rA[RT][2], rB[RT][2], rC[RT][2];
                bres_load<RT, VW>(as, 0, K, kq, rA);
                bres_load<RT, VW>(as, 1, K, kq, rB);
                int ks = 0;
                for (; ks + 3 <= nfull; ks += 3) {
                    bres_step<P, CT, RT, VW, 2>(acc, accx, rA, rC, as, ks, K, kq, ctb, c0, ctn, ascale, sF, lane);
                    bres_step<P, CT, RT, VW, 2>(acc, accx, rB, rA, as, ks + 1, K, kq, ctb, c0, ctn, ascale, sF, lane);
                    bres_step<P, CT, RT, VW, 2>(acc, accx, rC, rB, as, ks + 2, K, kq, ctb, c0, ctn, ascale, sF, lane);
                }
                const int rem = nfull - ks;  // A holds step ks, B step ks + 1
                if (rem >= 1) bres_step<P, CT, RT, VW, 2>(acc, accx, rA, rC, as, ks, K, kq, ctb, c0, ctn, ascale, sF, lane);
                if (rem >= 2) bres_step<P, CT, RT, VW, 2>(acc, accx, rB, rA, as, ks + 1, K, kq, ctb, c0, ctn, ascale, sF, lane);
                if (half) {  // step nfull is in A (rem 0), B (rem 1) or C (rem 2)
#pragma unroll
                    for (int r = 0; r < RT; r++)
                        bres_frag16<P, VW>(rem == 0 ? rA[r][0] : rem == 1 ? rB[r][0] : rC[r][0], ascale, a4[r]);
                }
            } else {
                float4 rawA[RT][2], rawB[RT][2];
                bres_load<RT, VW>(as, 0, K, kq, rawA);
                int ks = 0;
                for (; ks + 2 <= nfull; ks += 2) {
                    bres_step<P, CT, RT, VW>(acc, accx, rawA, rawB, as, ks, K, kq, ctb, c0, ctn, ascale, sF, lane);
                    bres_step<P, CT, RT, VW>(acc, accx, rawB, rawA, as, ks + 1, K, kq, ctb, c0, ctn, ascale, sF, lane);
                }
                const bool odd = ks < nfull;
                if (odd) bres_step<P, CT, RT, VW>(acc, accx, rawA, rawB, as, ks, K, kq, ctb, c0, ctn, ascale, sF, lane);
                if (half) {
#pragma unroll
                    for (int r = 0; r < RT; r++) bres_frag16<P, VW>(odd ? rawB[r][0] : rawA[r][0], ascale, a4[r]);
                }
            }
            if (half) {
                const uint2* bp = reinterpret_cast<const uint2*>(sT) + (size_t)(c0 * np) * 64 + lane;
#pragma unroll
                for (int c = 0; c < CT; c++) {
                    if (c < ctn) {
                        uint2 bb[3];
#pragma unroll
                        for (int q = 0; q < np; q++) bb[q] = bp[(c * np + q) * 64];
#pragma unroll
                        for (int r = 0; r < RT; r++) acc[r][c] = mma16<P>(a4[r], bb, acc[r][c], accx[r][c]);
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < RT; r++)
#pragma unroll
                for (int c = 0; c < CT; c++) acc[r][c] = x2_combine<P>(acc[r][c], accx[r][c]);
#pragma unroll
            for (int r = 0; r < RT; r++)
                bres_epilogue<P, CT, EM>(acc[r], RT * u + r, t0 + c0, ctn, M, N, ep, crs, srs, sbias + 16 * c0, lane);
        }
        X3_STAMP(1 + t, 2, __builtin_amdgcn_s_memtime());  // end of unit t
    }
    X3_STAMP(0, 3, __builtin_amdgcn_s_memtime());
    X3_STAMP(0, 5, __builtin_amdgcn_s_memrealtime());
}

}  // namespace x3
}  // namespace mm

using namespace mm::x3;

#ifdef X3_STAMPS
extern "C" int mm_x3_stamps_read(unsigned long long* out, long n) {
    const long cap = (long)(sizeof(g_x3_stamps) / sizeof(g_x3_stamps[0]));
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x3_stamps), (n < cap ? n : cap) * sizeof(unsigned long long), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int mm_trunk_stamps_read(unsigned long long* out, long n) {
    const long cap = (long)(sizeof(g_tr_stamps) / sizeof(g_tr_stamps[0]));
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tr_stamps), (n < cap ? n : cap) * sizeof(unsigned long long), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int mm_x3_stamps_clear() {
    static unsigned long long zero[256 * 16 * kWaves * 8];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_x3_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess
               ? 0 : -1;
}
#endif

extern "C" long mm_x3_tp_len(int R, int C) { return (long)(rup(R, kRowPad) / 16) * (rup(C, 32) / 32) * kBlk; }

extern "C" long mm_gemm_tp_len(int prec, int R, int C) {
    if (prec != MM_PREC_X3 && prec != MM_PREC_F16 && prec != MM_PREC_X2) return MM_E_ARG;
    return mm_x3_tp_len(R, C) / 3 * (prec == MM_PREC_X3 ? 3 : prec == MM_PREC_X2 ? 2 : 1);
}

extern "C" long mm_x3_mbits_len(int M) { return (long)(rup(M, kRowPad) / 16) * 64 * kMaskWords; }

extern "C" int mm_gemm_tp_pack(int prec, const float* X, int R, int C, int ld, int trans, uint16_t* tp,
                               void* stream) {
    if (!X || !tp || R <= 0 || C <= 0 || ld < (trans ? R : C)) return MM_E_ARG;
    if ((uintptr_t)tp & 15) return MM_E_ARG;
    const int nks = rup(C, 32) / 32;
    const long total = (long)(rup(R, kRowPad) / 16) * nks * 64;
    const int grid = (int)std::min<long>((total + 255) / 256, 256L * 64);
    if (prec == MM_PREC_X3)
        hipLaunchKernelGGL(k_tp_pack<P_X3>, dim3(grid), dim3(256), 0, (hipStream_t)stream, X, R, C, ld, trans, nks,
                           total, tp);
    else if (prec == MM_PREC_F16)
        hipLaunchKernelGGL(k_tp_pack<P_F16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, X, R, C, ld, trans, nks,
                           total, tp);
    else if (prec == MM_PREC_X2)
        hipLaunchKernelGGL(k_tp_pack<P_X2>, dim3(grid), dim3(256), 0, (hipStream_t)stream, X, R, C, ld, trans, nks,
                           total, tp);
    else
        return MM_E_ARG;
    return (int)hipGetLastError();
}

extern "C" int mm_gemm_tp_pack_multi(int prec, const mm_pack_seg_t* segs, int nseg, void* stream) {
    if (!segs || nseg <= 0 || nseg > kMaxPackSegs) return MM_E_ARG;
    PackSegs ps;
    ps.nseg = nseg;
    ps.pre[0] = 0;
    for (int k = 0; k < nseg; k++) {
        const mm_pack_seg_t& g = segs[k];
        if (!g.X || !g.tp || g.R <= 0 || g.C <= 0 || g.ld < (g.trans ? g.R : g.C) || ((uintptr_t)g.tp & 15))
            return MM_E_ARG;
        ps.s[k] = g;
        ps.nks[k] = rup(g.C, 32) / 32;
        ps.pre[k + 1] = ps.pre[k] + (long)(rup(g.R, kRowPad) / 16) * ps.nks[k] * 64;
    }
    const int grid = (int)std::min<long>((ps.pre[nseg] + 255) / 256, 256L * 64);
    if (prec == MM_PREC_X3)
        hipLaunchKernelGGL(k_tp_pack_multi<P_X3>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ps);
    else if (prec == MM_PREC_F16)
        hipLaunchKernelGGL(k_tp_pack_multi<P_F16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ps);
    else if (prec == MM_PREC_X2)
        hipLaunchKernelGGL(k_tp_pack_multi<P_X2>, dim3(grid), dim3(256), 0, (hipStream_t)stream, ps);
    else
        return MM_E_ARG;
    return (int)hipGetLastError();
}

extern "C" int mm_x3_tp_pack(const float* X, int R, int C, int ld, int trans, uint16_t* tp, void* stream) {
    return mm_gemm_tp_pack(MM_PREC_X3, X, R, C, ld, trans, tp, stream);
}

static int persistent_grid() {  // one 16-wave workgroup per CU
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    return cus;
}

template <int NT, int P, class AS, class AT>
static int launch_nt(const AT* a, int lda, float ascale, const uint16_t* b, int M, int N, int K, int ncb,
                     const Epi& ep, hipStream_t s) {
    constexpr int kT = SW<P>::kThreads;
    const int nks = rup(K, 32) / 32;
    const int nrb = rup(M, SW<P>::kBM) / SW<P>::kBM;
    const int grid = std::min(rup(nrb, 8) * ncb, persistent_grid() * (P == P_X2 ? 2 : 1));
    if (ep.ctp && ep.c) return MM_E_ARG;  // one output form per launch
    if constexpr (P == P_X3) {
        if (ep.ctp) {
            hipLaunchKernelGGL((k_x3nt<NT, P, AS, AT, EM_TP>), dim3(grid), dim3(kT), 0, s, a, lda, ascale, b, M,
                               N, K, nks, nrb, ncb, ep);
            return (int)hipGetLastError();
        }
    } else if (ep.ctp) {
        return MM_E_ARG;
    }
    if (ep.c16) {  // fp16 activations out: P_F16's forward with bits, through the buffer-store epilogue
        if constexpr (P == P_F16) {
            if (!ep.mbits_out || !ep.bufok) return MM_E_ARG;
            hipLaunchKernelGGL((k_x3nt<NT, P, AS, AT, EM_FWD16>), dim3(grid), dim3(kT), 0, s, a, lda, ascale, b, M, N,
                               K, nks, nrb, ncb, ep);
            return (int)hipGetLastError();
        }
        return MM_E_ARG;
    }
    if (ep.mbits_out)
        hipLaunchKernelGGL((k_x3nt<NT, P, AS, AT, EM_FWD>), dim3(grid), dim3(kT), 0, s, a, lda, ascale, b, M, N,
                           K, nks, nrb, ncb, ep);
    else if (ep.mbits_in)
        hipLaunchKernelGGL((k_x3nt<NT, P, AS, AT, EM_BWD>), dim3(grid), dim3(kT), 0, s, a, lda, ascale, b, M, N,
                           K, nks, nrb, ncb, ep);
    else
        hipLaunchKernelGGL((k_x3nt<NT, P, AS, AT, EM_F32>), dim3(grid), dim3(kT), 0, s, a, lda, ascale, b, M, N,
                           K, nks, nrb, ncb, ep);
    return (int)hipGetLastError();
}

template <int P, class AS, class AT>
static int dispatch_nt(const AT* a, int lda, float ascale, const uint16_t* b_tp, int M, int N, int K, const Epi& ep,
                       hipStream_t s) {
    // column tiling: one block of <= 17 tiles, or several blocks of 15 (B rows are padded to 256)
    const int tiles = (N + 15) / 16;
    int NT, ncb;
    if (tiles <= 1) { NT = 1; ncb = 1; }
    else if (tiles <= 4) { NT = 4; ncb = 1; }
    else if (tiles <= 8) { NT = 8; ncb = 1; }
    else if (tiles <= 17) { NT = 17; ncb = 1; }
    else { NT = 15; ncb = (tiles + 14) / 15; }
    // few rows (the rollout's 4,096-8,192-row calls, the reference's 3,000-sample minibatches): too few
    // 256-row units to fill the chip, so the columns are split into 4-tile blocks (x5 workgroups at N =
    // 264).  Needs the buffer-store epilogue when bits are involved (it writes whole mask bytes per block).
    const int nrb = rup(M, SW<P>::kBM) / SW<P>::kBM;
    if (tiles > 4 && !ep.ctp && (ep.bufok || (!ep.mbits_in && !ep.mbits_out)) && 2L * nrb * ncb <= persistent_grid()) {
        NT = 4;
        ncb = (tiles + 3) / 4;
    }
    if (ncb * NT * 16 > rup(N, kRowPad)) return MM_E_ARG;  // B TP row padding would be overrun
    if (ep.ctp && ncb != 1) return MM_E_ARG;
    switch (NT) {
        case 1: return launch_nt<1, P, AS>(a, lda, ascale, b_tp, M, N, K, ncb, ep, s);
        case 4: return launch_nt<4, P, AS>(a, lda, ascale, b_tp, M, N, K, ncb, ep, s);
        case 8: return launch_nt<8, P, AS>(a, lda, ascale, b_tp, M, N, K, ncb, ep, s);
        case 15: return launch_nt<15, P, AS>(a, lda, ascale, b_tp, M, N, K, ncb, ep, s);
        default: return launch_nt<17, P, AS>(a, lda, ascale, b_tp, M, N, K, ncb, ep, s);
    }
}

// 8-byte-row A sources serve only narrow outputs (the critic's first layer)
template <int P>
static int dispatch_nt_u(const float* a, int lda, float ascale, const uint16_t* b_tp, int M, int N, int K,
                         const Epi& ep, hipStream_t s) {
    const int tiles = (N + 15) / 16;
    if (tiles <= 1) return launch_nt<1, P, ASrcF32U>(a, lda, ascale, b_tp, M, N, K, 1, ep, s);
    if (tiles <= 4) return launch_nt<4, P, ASrcF32U>(a, lda, ascale, b_tp, M, N, K, 1, ep, s);
    return MM_E_ARG;
}

// ---- k_bres dispatch ----
static int g_gemm_algo = -1;  // MM_GEMM_*; -1: not read from the environment yet
static bool bres_enabled() {
    if (g_gemm_algo < 0) {
        const char* e = getenv("MARLMAZE_GEMM_BRES");
        g_gemm_algo = (e && e[0] == '0') ? MM_GEMM_STREAM : MM_GEMM_AUTO;
    }
    return g_gemm_algo == MM_GEMM_AUTO;
}

extern "C" int mm_gemm_nt_algo(int algo) {
    bres_enabled();
    const int prev = g_gemm_algo;
    if (algo == MM_GEMM_AUTO || algo == MM_GEMM_STREAM) g_gemm_algo = algo;
    return prev;
}

constexpr int kBresMinRows = 16384;
// the B-resident kernel's row threshold: kBresMinRows, or MARLMAZE_BRES_MIN_ROWS (A/B runs of the small-M
// calls: the rollout's 4,096-8,192-row GEMMs)
static int bres_min_rows() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("MARLMAZE_BRES_MIN_ROWS");
        v = e ? atoi(e) : kBresMinRows;
        if (v < 1) v = 1;
    }
    return v;
}
// wave units: C_NARROW two row tiles x 6 column tiles (acc 48 registers; each B fragment read feeds two
// tiles) -- x3, and f16 up to 6 tiles; C_WIDE (f16) one row tile x up to 17 column tiles (acc 68: the
// whole 264-wide output per wave, A read once)
// C_PAIR (x2): one row tile x up to 9 column tiles (two accumulator sets: 72 registers), the widest block
// two B planes leave room for at K = 264
enum { C_NARROW = 0, C_WIDE = 1, C_PAIR = 2 };
template <int C>
struct BresCfg {
    static constexpr int CT = C == C_NARROW ? 6 : C == C_WIDE ? 17 : 9, RT = C == C_NARROW ? 2 : 1;
};

// The column blocks and the per-XCD workgroup split (see k_bres); false: the shape does not fit.
static bool bres_plan(int prec, int M, int N, int K, int lda, int ldc, bool bits, BresPlan& pl, int& cfg) {
    // A and C through buffer resources (num_records < 2^31, in-range offsets < 2^31 = kBufOOB)
    if (M < bres_min_rows() || (size_t)M * lda * 4 >= ((size_t)1 << 31) || (size_t)(M + 16) * ldc * 4 >= ((size_t)1 << 31))
        return false;
    const int np = prec == MM_PREC_X3 ? 3 : prec == MM_PREC_X2 ? 2 : 1;
    const int tiles = (N + 15) / 16;
    const int nks = rup(K, 32) / 32, rem = K % 32;
    pl.half = rem != 0 && rem <= 16;
    pl.nfull = nks - pl.half;
    const long tile_bytes = (long)np * (pl.nfull * 1024L + pl.half * 512L) + 64;  // + the bias columns
    int cmax = (int)((160L * 1024) / tile_bytes);
    if (prec == MM_PREC_X2) cmax = std::min(cmax, BresCfg<C_PAIR>::CT);  // one sub-block per wave
    if (cmax < 1 || pl.nfull < 1) return false;
    // blocks: as few as fit, then the narrowest widest block; every block but the last holds e tiles, and
    // with ReLU bits e is even (blocks start at even tiles: whole mask bytes per block) -- x3 at K = 264:
    // 6 + 6 + 5, x2: 8 + 9
    int nblk = 0, e_best = 0, ctb = 0;
    for (int nb = (tiles + cmax - 1) / cmax; nb <= kBresMaxBlk && !nblk; nb++) {
        if (nb == 1) {
            nblk = 1;
            ctb = e_best = tiles;
            break;
        }
        for (int e = cmax; e >= 1; e--) {
            if (bits && (e & 1)) continue;
            const int last = tiles - e * (nb - 1);
            if (last < 1 || last > cmax) continue;
            const int wmax = std::max(e, last);
            if (!nblk || wmax < ctb) {
                nblk = nb;
                ctb = wmax;
                e_best = e;
            }
        }
    }
    if (!nblk) return false;
    if (nblk > 1 && std::min(e_best, tiles - e_best * (nblk - 1)) < 4 && prec != MM_PREC_X2)
        return false;  // A re-read per block: x3 at K = 460 (3 tiles) measured slower
    // f16 / x2 at K = 460 (blocks re-reading A of 460 columns): the streaming kernel measured faster (f16
    // 0.81x; x2, four 4-5-tile blocks: 568 vs 462 us at 419,430 rows -- BRES_X2_WIDE_K=1 builds that form)
#ifndef BRES_X2_WIDE_K
#define BRES_X2_WIDE_K 0
#endif
    if (prec != MM_PREC_X3 && nblk > 1 && K > 288 && (prec != MM_PREC_X2 || !BRES_X2_WIDE_K)) return false;
    cfg = prec == MM_PREC_X2 ? C_PAIR : (prec == MM_PREC_F16 && ctb > BresCfg<C_NARROW>::CT) ? C_WIDE : C_NARROW;
    pl.nblk = nblk;
    pl.ctb = ctb;
    pl.tiles = tiles;
    for (int bk = 0; bk <= kBresMaxBlk; bk++) pl.tstart[bk] = std::min(tiles, bk * e_best);
    pl.tstart[nblk] = tiles;
    const int G = persistent_grid();
    pl.xcds = G % 8 == 0 ? 8 : 1;
    const int per = G / pl.xcds;
    if (per < nblk) return false;
    // workgroups per block in proportion to its tiles: greedy on the largest tiles-per-workgroup
    // (equal counts per block, so that the blocks sweep the row groups in step for L2 reuse of A, measured
    // 3% slower at x2 264 x 264, round 6)
    int w[kBresMaxBlk];
    for (int bk = 0; bk < nblk; bk++) w[bk] = 1;
    for (int left = per - nblk; left > 0; left--) {
        int best = 0;
        for (int bk = 1; bk < nblk; bk++) {
            const int tb = pl.tstart[bk + 1] - pl.tstart[bk], tbest = pl.tstart[best + 1] - pl.tstart[best];
            if ((long)tb * w[best] > (long)tbest * w[bk]) best = bk;
        }
        w[best]++;
    }
    pl.first[0] = 0;
    for (int bk = 0; bk < nblk; bk++) pl.first[bk + 1] = pl.first[bk] + w[bk];
    for (int bk = nblk + 1; bk <= kBresMaxBlk; bk++) pl.first[bk] = pl.first[nblk];
    return true;
}

template <int P, int C, int EM, int VW>
static int launch_bres(const float* a, int lda, float ascale, const uint16_t* b, int M, int N, int K,
                       const BresPlan& pl, const Epi& ep, hipStream_t s) {
    constexpr int CT = BresCfg<C>::CT, RT = BresCfg<C>::RT;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k_bres<P, CT, RT, EM, VW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess)
            return MM_E_ARG;
        attr = true;
    }
    constexpr int np = Prec<P>::kPlanes;
    const size_t lds = (size_t)pl.ctb * np * (pl.nfull * 1024 + pl.half * 512) + (size_t)pl.ctb * 16 * 4;
    hipLaunchKernelGGL((k_bres<P, CT, RT, EM, VW>), dim3(persistent_grid()), dim3(64 * kBresWaves), lds, s, a, lda, ascale, b,
                       M, N, K, rup(K, 32) / 32, pl, ep);
    return (int)hipGetLastError();
}

template <int P, int C, int VW>
static int dispatch_bres_c(const float* a, int lda, float ascale, const uint16_t* b, int M, int N, int K,
                           const BresPlan& pl, const Epi& ep, hipStream_t s) {
    if (ep.c16) {
        if constexpr (P == P_F16) {
            if (ep.mbits_out) return launch_bres<P, C, EM_FWD16, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
            if (ep.mbits_in) return launch_bres<P, C, EM_BWD16, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
        }
        return MM_E_ARG;
    }
    if (ep.mbits_out) return launch_bres<P, C, EM_FWD, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
    if (ep.mbits_in) return launch_bres<P, C, EM_BWD, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
    return launch_bres<P, C, EM_F32, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
}

template <int P, int VW>
static int dispatch_bres(const float* a, int lda, float ascale, const uint16_t* b, int M, int N, int K,
                         const BresPlan& pl, int cfg, const Epi& ep, hipStream_t s) {
    if constexpr (P == P_X2) {
        (void)cfg;
        return dispatch_bres_c<P, C_PAIR, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
    } else {
        if constexpr (P == P_F16)
            if (cfg == C_WIDE) return dispatch_bres_c<P, C_WIDE, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
        return dispatch_bres_c<P, C_NARROW, VW>(a, lda, ascale, b, M, N, K, pl, ep, s);
    }
}

static int check_common(const uint16_t* b_tp, int M, int N, int K, const float* mask, int ldm, float* c, int ldc,
                        uint16_t* c_tp) {
    if (!b_tp || M < 0 || N <= 0 || K <= 0 || (!c && !c_tp)) return MM_E_ARG;
    if (c && (ldc < N || ((uintptr_t)c & 3))) return MM_E_ARG;
    if (mask && ldm < N) return MM_E_ARG;
    if (((uintptr_t)b_tp | (uintptr_t)c_tp) & 15) return MM_E_ARG;
    return 0;
}

// C = A . B^T (+bias)(ReLU)(* (mask > 0)): A TP of [M, K], B TP of [N, K];
// outputs fp32 c [M, ldc] and/or TP ctp of [M, N].
extern "C" int mm_x3_nt(const uint16_t* a_tp, const uint16_t* b_tp, int M, int N, int K, const float* bias, int relu,
                        const float* mask, int ldm, float* c, int ldc, uint16_t* c_tp, void* stream) {
    int e = check_common(b_tp, M, N, K, mask, ldm, c, ldc, c_tp);
    if (e) return e;
    if (!a_tp || ((uintptr_t)a_tp & 15)) return MM_E_ARG;
    if (M == 0) return 0;
    Epi ep{bias, mask, nullptr, nullptr, c, c_tp, nullptr, ldc, ldm, relu, rup(N, 32) / 32, 1.f,
           c && (size_t)(M + 16) * ldc * 4 < ((size_t)1 << 31), 0, 1.f};
    return dispatch_nt<P_X3, ASrcTP>(a_tp, 0, 1.f, b_tp, M, N, K, ep, (hipStream_t)stream);
}

static int gemm_nt_f32a(int prec, const float* a, int lda, float ascale, const uint16_t* b_tp, int M, int N, int K,
                        const float* bias, int relu, const float* mask, int ldm, const uint32_t* mbits_in,
                        uint32_t* mbits_out, float* colsum, float cscale, float* c, int ldc, uint16_t* c_tp,
                        void* stream, int flags = 0, float oscale = 1.f) {
    int e = check_common(b_tp, M, N, K, mask, ldm, c, ldc, c_tp);
    if (e) return e;
    if (prec != MM_PREC_X3 && prec != MM_PREC_F16 && prec != MM_PREC_X2) return MM_E_ARG;
    const bool a16 = flags & MM_GEMM_A_F16, c16 = flags & MM_GEMM_C_F16;
    if (flags & ~(MM_GEMM_A_F16 | MM_GEMM_C_F16)) return MM_E_ARG;
    // fp16 activations (P_F16 only): A fp16 at scale 1 on the B-resident kernel; C fp16 for the forward with bits
    if ((a16 || c16) && (prec != MM_PREC_F16 || mask || c_tp)) return MM_E_ARG;
    if (a16 && (ascale != 1.f || (K & 3) || (lda & 3) || ((uintptr_t)a & 7))) return MM_E_ARG;
    if (c16 && ((!mbits_out && !mbits_in) || ((uintptr_t)c & 1))) return MM_E_ARG;
    if (prec == MM_PREC_X3 && (ascale != 1.f || cscale != 1.f)) return MM_E_ARG;  // the split is exact: no scaling
    const bool v4 = !a16 && !(K & 3) && !(lda & 3) && !((uintptr_t)a & 15);
    const bool v2 = !a16 && !(K & 1) && !(lda & 1) && !((uintptr_t)a & 7);
    if (!a || lda < K || !(v4 || v2 || a16) || (!v4 && !a16 && N > 64)) return MM_E_ARG;  // 8-byte rows: narrow outputs only
    if ((mbits_in || mbits_out) && (N > 16 * 17 || c_tp || mask || (mbits_in && mbits_out))) return MM_E_ARG;
    if (mbits_in && (bias || relu)) return MM_E_ARG;  // the input-gradient form: no bias, no ReLU of its own
    if (colsum && (!mbits_in || !c)) return MM_E_ARG;
    if (M == 0) return 0;
    // the kernels address A and C through buffer resources (num_records < 2^31 bytes): larger calls run
    // in row chunks of a multiple of 256 rows (whole row tiles of the bit masks and column sums)
    const size_t wmax = std::max(std::max((size_t)lda, (size_t)ldc), std::max((size_t)ldm, (size_t)N));
    const size_t cap = ((((size_t)1 << 31) - 1) / (4 * wmax) - 32) / kRowPad * kRowPad;
    if ((size_t)M > cap) {
        if (cap < (size_t)kRowPad || c_tp) return MM_E_ARG;
        for (size_t m0 = 0; m0 < (size_t)M; m0 += cap) {
            const int mr = (int)std::min(cap, (size_t)M - m0);
            const size_t rt0 = m0 / 16;
            const float* am = reinterpret_cast<const float*>(reinterpret_cast<const char*>(a) + m0 * lda * (a16 ? 2 : 4));
            float* cm = reinterpret_cast<float*>(reinterpret_cast<char*>(c) + m0 * ldc * (c16 ? 2 : 4));
            const int rc = gemm_nt_f32a(prec, am, lda, ascale, b_tp, mr, N, K, bias, relu,
                                        mask ? mask + m0 * ldm : nullptr, ldm,
                                        mbits_in ? mbits_in + rt0 * 64 * kMaskWords : nullptr,
                                        mbits_out ? mbits_out + rt0 * 64 * kMaskWords : nullptr,
                                        colsum ? colsum + rt0 * N : nullptr, cscale, cm, ldc, nullptr, stream, flags,
                                        oscale);
            if (rc) return rc;
        }
        return 0;
    }
    Epi ep{bias, mask, mbits_in, mbits_out, c, c_tp, colsum, ldc, ldm, relu, rup(N, 32) / 32, cscale, c != nullptr,
           c16 ? 1 : 0, oscale};
    hipStream_t s = (hipStream_t)stream;
    BresPlan pl;
    int cfg = C_NARROW;
    if (a16 || (c16 && mbits_in)) {  // fp16 A, or fp16 input gradients: the B-resident kernel, or for fp16 A
                                      // where it does not fit (K = 460) the streaming kernel with ASrcF16V
        if (!bres_plan(prec, M, N, K, lda, ldc, mbits_in || mbits_out, pl, cfg)) {
            if (a16 && !(c16 && mbits_in))
                return dispatch_nt<P_F16, ASrcF16V>(reinterpret_cast<const unsigned short*>(a), lda, 1.f, b_tp, M, N,
                                                    K, ep, s);
            return MM_E_ARG;
        }
        return a16 ? dispatch_bres<P_F16, 16>(a, lda, 1.f, b_tp, M, N, K, pl, cfg, ep, s)
                   : (v4 ? dispatch_bres<P_F16, 4>(a, lda, ascale, b_tp, M, N, K, pl, cfg, ep, s)
                         : dispatch_bres<P_F16, 2>(a, lda, ascale, b_tp, M, N, K, pl, cfg, ep, s));
    }
    if (!mask && !c_tp && bres_enabled() && bres_plan(prec, M, N, K, lda, ldc, mbits_in || mbits_out, pl, cfg)) {
        if (prec == MM_PREC_X3)
            return v4 ? dispatch_bres<P_X3, 4>(a, lda, 1.f, b_tp, M, N, K, pl, cfg, ep, s)
                      : dispatch_bres<P_X3, 2>(a, lda, 1.f, b_tp, M, N, K, pl, cfg, ep, s);
        if (prec == MM_PREC_X2)
            return v4 ? dispatch_bres<P_X2, 4>(a, lda, ascale, b_tp, M, N, K, pl, cfg, ep, s)
                      : dispatch_bres<P_X2, 2>(a, lda, ascale, b_tp, M, N, K, pl, cfg, ep, s);
        return v4 ? dispatch_bres<P_F16, 4>(a, lda, ascale, b_tp, M, N, K, pl, cfg, ep, s)
                  : dispatch_bres<P_F16, 2>(a, lda, ascale, b_tp, M, N, K, pl, cfg, ep, s);
    }
    if (prec == MM_PREC_X3)
        return v4 ? dispatch_nt<P_X3, ASrcF32>(a, lda, 1.f, b_tp, M, N, K, ep, s)
                  : dispatch_nt_u<P_X3>(a, lda, 1.f, b_tp, M, N, K, ep, s);
    if (prec == MM_PREC_X2)
        return v4 ? dispatch_nt<P_X2, ASrcF32>(a, lda, ascale, b_tp, M, N, K, ep, s)
                  : dispatch_nt_u<P_X2>(a, lda, ascale, b_tp, M, N, K, ep, s);
    return v4 ? dispatch_nt<P_F16, ASrcF32>(a, lda, ascale, b_tp, M, N, K, ep, s)
              : dispatch_nt_u<P_F16>(a, lda, ascale, b_tp, M, N, K, ep, s);
}

// The same with A fp32 row-major [M, lda] (K % 4 == 0, lda % 4 == 0, 16-byte
// aligned), split into bf16 planes in registers inside the GEMM.
extern "C" int mm_x3_nt_f32a(const float* a, int lda, const uint16_t* b_tp, int M, int N, int K, const float* bias,
                             int relu, const float* mask, int ldm, const uint32_t* mbits_in, uint32_t* mbits_out,
                             float* colsum, float* c, int ldc, uint16_t* c_tp, void* stream) {
    if (!a || (K & 3) || (lda & 3) || ((uintptr_t)a & 15)) return MM_E_ARG;
    return gemm_nt_f32a(MM_PREC_X3, a, lda, 1.f, b_tp, M, N, K, bias, relu, mask, ldm, mbits_in, mbits_out, colsum,
                        1.f, c, ldc, c_tp, stream);
}

extern "C" int mm_gemm_nt(int prec, const float* a, int lda, float ascale, const uint16_t* b_tp, int M, int N, int K,
                          const float* bias, int relu, const uint32_t* mbits_in, uint32_t* mbits_out, float* colsum,
                          float cscale, float* c, int ldc, void* stream) {
    if (!c) return MM_E_ARG;
    return gemm_nt_f32a(prec, a, lda, ascale, b_tp, M, N, K, bias, relu, nullptr, 0, mbits_in, mbits_out, colsum,
                        cscale, c, ldc, nullptr, stream);
}

extern "C" int mm_gemm_nt_h(int prec, int flags, const void* a, int lda, float ascale, const uint16_t* b_tp, int M,
                            int N, int K, const float* bias, int relu, const uint32_t* mbits_in, uint32_t* mbits_out,
                            float* colsum, float cscale, float oscale, void* c, int ldc, void* stream) {
    if (!c) return MM_E_ARG;
    return gemm_nt_f32a(prec, static_cast<const float*>(a), lda, ascale, b_tp, M, N, K, bias, relu, nullptr, 0,
                        mbits_in, mbits_out, colsum, cscale, static_cast<float*>(c), ldc, nullptr, stream, flags,
                        oscale);
}

// ---- the fused small-M trunk (k_trunk3) ----
// row tiles per workgroup: 2 (MARLMAZE_TRUNK_RT=3: 3 where the LDS holds them -- fewer workgroups
// re-reading the weights from L2, but each one's k-loops 1.27x longer: 25.3 vs 22.3 us at 8,192 rows, x2).  Weight fragments D
// k-steps ahead: 1 for x2 / x3, 3 for f16 (its k-steps are 3x shorter); MARLMAZE_TRUNK_D=1 or 3 forces one.
static int trunk_env(const char* name) {
    const char* e = getenv(name);
    return e ? atoi(e) : 0;
}

// LDS: the biases, the f16 kernels' epilogue slices, then two activation buffers of TP blocks (uint16):
// bufX = h0 / layer 1's output, bufH = layer 0's output
static void trunk_bufs(int prec, int RT, int K0, int N0, int N1, int& bx, size_t& lds) {
    const int np = prec == MM_PREC_X3 ? 3 : prec == MM_PREC_X2 ? 2 : 1;
    const int nx = std::max(rup(K0, 32), rup(N1, 32)) / 32, nh = rup(N0, 32) / 32;
    bx = RT * nx * np * 512;
    lds = (size_t)(9 * kTrMaxN + (np == 1 ? kTrWaves * kTrSlice : 0)) * 4 + (size_t)RT * (nx + nh) * np * 1024;
}

// the fused heads' h3 rows (16 RT rows of N2 + 4 floats): in bufH when it holds them (free during the last
// layer), else in a region appended to the LDS; hoff in floats from the LDS base
static void trunk_h3(int prec, int RT, int K0, int N0, int N1, int N2, int& hoff, size_t& lds) {
    const int np = prec == MM_PREC_X3 ? 3 : prec == MM_PREC_X2 ? 2 : 1;
    int bx;
    trunk_bufs(prec, RT, K0, N0, N1, bx, lds);
    const size_t need = (size_t)16 * RT * (N2 + 4) * 4, hbytes = (size_t)RT * (rup(N0, 32) / 32) * np * 1024;
    const size_t bufx = (size_t)(9 * kTrMaxN + (np == 1 ? kTrWaves * kTrSlice : 0)) * 4;
    if (need <= hbytes) {
        hoff = (int)((bufx + (size_t)bx * 2) / 4);
    } else {
        hoff = (int)(lds / 4);
        lds += need;
    }
}

static int trunk_pick_rt(int prec, int K0, int N0, int N1) {
    int bx;
    size_t lds;
    if (trunk_env("MARLMAZE_TRUNK_RT") == 3) {
        trunk_bufs(prec, 3, K0, N0, N1, bx, lds);
        if (lds <= 160 * 1024) return 3;
    }
    trunk_bufs(prec, 2, K0, N0, N1, bx, lds);
    return lds <= 160 * 1024 ? 2 : 0;
}

extern "C" int mm_trunk3_ok(int prec, int M, int K0, int N0, int N1, int N2, int lda) {
    if (prec != MM_PREC_X3 && prec != MM_PREC_F16 && prec != MM_PREC_X2) return 0;
    if (M < 0 || K0 <= 0 || (K0 & 3) || (lda & 3) || lda < K0 || rup(K0, 32) > kTrMaxK0) return 0;
    if (N0 <= 0 || N1 <= 0 || N2 <= 0 || N0 > kTrMaxN || N1 > kTrMaxN || N2 > kTrMaxN) return 0;
    return trunk_pick_rt(prec, K0, N0, N1) ? 1 : 0;
}

template <int P, int RT, int D, bool HS = false>
static int launch_trunk(const TrunkArgs& ta, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k_trunk3<P, RT, D, HS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024) != hipSuccess)
            return MM_E_ARG;
        attr = true;
    }
    hipLaunchKernelGGL((k_trunk3<P, RT, D, HS>), dim3((ta.M + 16 * RT - 1) / (16 * RT)), dim3(64 * kTrWaves), lds, s,
                       ta);
    return (int)hipGetLastError();
}

template <int P>
static int launch_trunk_p(TrunkArgs& ta, int RT, hipStream_t s) {
    const int de = trunk_env("MARLMAZE_TRUNK_D");
    const int d = de == 1 || de == 3 ? de : P == P_F16 ? 3 : 1;
    size_t lds;
    trunk_bufs(P, RT, ta.K0, ta.N[0], ta.N[1], ta.bx, lds);
    if (RT == 3) return d == 3 ? launch_trunk<P, 3, 3>(ta, lds, s) : launch_trunk<P, 3, 1>(ta, lds, s);
    return d == 3 ? launch_trunk<P, 2, 3>(ta, lds, s) : launch_trunk<P, 2, 1>(ta, lds, s);
}

extern "C" int mm_trunk3(int prec, const float* h0, int lda, int M, int K0, const uint16_t* w0, const float* b0,
                         int N0, const uint16_t* w1, const float* b1, int N1, const uint16_t* w2, const float* b2,
                         int N2, float* out, int ldc, void* stream) {
    if (!mm_trunk3_ok(prec, M, K0, N0, N1, N2, lda) || !h0 || !out || !w0 || !w1 || !w2 || ldc < N2) return MM_E_ARG;
    if (((uintptr_t)h0 & 15) || (((uintptr_t)w0 | (uintptr_t)w1 | (uintptr_t)w2) & 15) || ((uintptr_t)out & 3))
        return MM_E_ARG;
    if (M == 0) return 0;
    TrunkArgs ta{h0, {w0, w1, w2}, {b0, b1, b2}, out, lda, ldc, M, K0, {N0, N1, N2}, 0,
                 nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
    const int RT = trunk_pick_rt(prec, K0, N0, N1);
    hipStream_t s = (hipStream_t)stream;
    if (prec == MM_PREC_X2) return launch_trunk_p<P_X2>(ta, RT, s);
    if (prec == MM_PREC_F16) return launch_trunk_p<P_F16>(ta, RT, s);
    return launch_trunk_p<P_X3>(ta, RT, s);
}

// the trunk + the actor heads + PPO.get_action in one launch (two row tiles a workgroup; D as mm_trunk3)
extern "C" int mm_trunk3_head_sample_ok(int prec, int M, int K0, int N0, int N1, int N2, int lda) {
    if (!mm_trunk3_ok(prec, M, K0, N0, N1, N2, lda) || (N2 & 3)) return 0;
    int hoff;
    size_t lds;
    trunk_h3(prec, 2, K0, N0, N1, N2, hoff, lds);
    return lds <= 160 * 1024 ? 1 : 0;
}

extern "C" int mm_trunk3_head_sample(int prec, const float* h0, int lda, int M, int K0, const uint16_t* w0,
                                     const float* b0, int N0, const uint16_t* w1, const float* b1, int N1,
                                     const uint16_t* w2, const float* b2, int N2, const float* head_w,
                                     const float* head_b, const uint8_t* masks, uint64_t seed, uint64_t offset,
                                     const uint64_t* offset_dev, int8_t* actions, float* logp, float* joint_logp,
                                     float* logits, float* h3, int ldh3, void* stream) {
    if (!mm_trunk3_head_sample_ok(prec, M, K0, N0, N1, N2, lda) || !h0 || !w0 || !w1 || !w2 || !head_w || !head_b ||
        !masks || !actions || (h3 && (ldh3 < N2 || ((uintptr_t)h3 & 3))))
        return MM_E_ARG;
    if (((uintptr_t)h0 & 15) || (((uintptr_t)w0 | (uintptr_t)w1 | (uintptr_t)w2) & 15)) return MM_E_ARG;
    if (M == 0) return 0;
    TrunkArgs ta{h0, {w0, w1, w2}, {b0, b1, b2}, h3, lda, ldh3, M, K0, {N0, N1, N2}, 0,
                 head_w, head_b, masks, seed, offset, offset_dev, actions, logp, joint_logp, logits, 0};
    size_t lds;
    trunk_bufs(prec, 2, K0, N0, N1, ta.bx, lds);
    trunk_h3(prec, 2, K0, N0, N1, N2, ta.hoff, lds);
    hipStream_t s = (hipStream_t)stream;
    if (prec == MM_PREC_X2) return launch_trunk<P_X2, 2, 1, true>(ta, lds, s);
    if (prec == MM_PREC_F16) return launch_trunk<P_F16, 2, 3, true>(ta, lds, s);
    return launch_trunk<P_X3, 2, 1, true>(ta, lds, s);
}

// dY = (dz W) * bits (the heads' backward through the last ReLU, bits from the
// last forward GEMM's mbits_out, N <= 272, J <= 8), and the per-16-row-tile
// column sums colsum [ceil(M / 16), N].
// the same with dY fp16 = fp16(dY * oscale) (P_F16's pre-scaled input gradients)
extern "C" int mm_x3_heads_bwd_h16(const float* dz, int J, const float* W, const uint32_t* bits, int M, int N,
                                   void* dy, float* colsum, float oscale, void* stream) {
    if (!dz || !W || !bits || !dy || !colsum || J <= 0 || J > kHeadsMaxJ || N <= 0 || N > 272 || M < 0)
        return MM_E_ARG;
    if (M == 0) return 0;
    const int nrt = (M + 15) / 16;
    hipLaunchKernelGGL((k_heads_bwd<17, true>), dim3((nrt + 3) / 4), dim3(256), 0, (hipStream_t)stream, dz, J, W, bits,
                       M, N, static_cast<float*>(dy), colsum, oscale);
    return (int)hipGetLastError();
}

extern "C" int mm_x3_heads_bwd(const float* dz, int J, const float* W, const uint32_t* bits, int M, int N, float* dy,
                               float* colsum, void* stream) {
    if (!dz || !W || !bits || !dy || !colsum || J <= 0 || J > kHeadsMaxJ || N <= 0 || N > 272 || M < 0)
        return MM_E_ARG;
    if (M == 0) return 0;
    const int nrt = (M + 15) / 16;
    hipLaunchKernelGGL(k_heads_bwd<17>, dim3((nrt + 3) / 4), dim3(256), 0, (hipStream_t)stream, dz, J, W, bits, M, N,
                       dy, colsum);
    return (int)hipGetLastError();
}

// ---- weight gradient ----
struct WgPlan {
    int TN, NTK, ncb, nslices, rows, TPW, tpw;  // TPW: the instantiation (>= tpw, the balanced run length)
};

static WgPlan wg_plan(int prec, int M, int N, int K) {
    WgPlan p;
    p.TN = (N + 15) / 16;
    const int tk_all = (K + 15) / 16;
    // column blocks: at most 20 tiles per wave (the register budget of 2 waves per SIMD) and two image sets
    // within 160 KiB of LDS; a slice's blocks share its dY rows through the XCD's L2
    p.ncb = (tk_all + kWgMaxT - 1) / kWgMaxT;
    const int kb = prec == MM_PREC_X3 ? 1536 : prec == MM_PREC_X2 ? 1024 : 512;
    auto fits = [&](int ncb) {
        const int ntk = (tk_all + ncb - 1) / ncb;
        return p.TN * ntk <= kWgWaves * 20 && 2 * (p.TN + ntk) * kb * 2 <= 160 * 1024;
    };
    while (!fits(p.ncb)) p.ncb++;
    p.NTK = (tk_all + p.ncb - 1) / p.ncb;
    p.tpw = (p.TN * p.NTK + kWgWaves - 1) / kWgWaves;
    static const int kTPW[] = {1, 2, 3, 5, 8, 12, 16, 20};
    p.TPW = 0;
    for (int t : kTPW)
        if (t >= p.tpw) {
            p.TPW = t;
            break;
        }
    // about one unit per CU: slices of whole 32-row steps (a floor of 512 rows per slice, to shrink the slices'
    // partials at BASELINE configs[1]'s 52,428-row minibatch, measured slower: 24.6 vs 23.5 ms per update)
    const int want = std::max(1, std::min((M + 31) / 32, persistent_grid() / p.ncb));
    p.rows = rup((M + want - 1) / want, 32);
    p.nslices = std::max(1, (M + p.rows - 1) / p.rows);
    return p;
}

__global__ void k_range_flag(uint32_t* out, int clear) {
    if (threadIdx.x == 0) {  // vector atomics on the flag (no scalar-cache writes)
        const uint32_t v = clear ? __hip_atomic_exchange(&g_range_flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : __hip_atomic_load(&g_range_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (out) out[0] = v;
    }
}

extern "C" int mm_gemm_range_flag(uint32_t* out, int clear, void* stream) {
    hipLaunchKernelGGL(k_range_flag, dim3(1), dim3(64), 0, (hipStream_t)stream, out, clear);
    return (int)hipGetLastError();
}

extern "C" long mm_gemm_wgrad_ws_len(int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0) return 0;
    long n = 0;  // the larger of the two precisions' plans
    for (int prec : {MM_PREC_X3, MM_PREC_F16, MM_PREC_X2}) {
        const WgPlan p = wg_plan(prec, M, N, K);
        n = std::max(n, (long)p.nslices * N * K);
    }
    return n;
}

template <int P>
static int launch_wgrad(const WgPlan& p, const float* dy, int lddy, float dscale, const float* x, int ldx, int M,
                        int N, int K, float cscale, float* ws, hipStream_t s) {
    const dim3 grid(rup(p.nslices, 8) * p.ncb), block(kWgThreads);
    const size_t lds = (size_t)2 * (p.TN + p.NTK) * Prec<P>::kBlk * sizeof(uint16_t);
#define MM_WG(T)                                                                                               \
    case T:                                                                                                    \
        {                                                                                                      \
            static bool attr = false;                                                                          \
            if (!attr) {                                                                                       \
                if (hipFuncSetAttribute((const void*)k_wgrad<P, T>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                        160 * 1024) != hipSuccess)                                             \
                    return MM_E_ARG;                                                                           \
                attr = true;                                                                                   \
            }                                                                                                  \
        }                                                                                                      \
        hipLaunchKernelGGL((k_wgrad<P, T>), grid, block, lds, s, dy, lddy, dscale, x, ldx, M, N, K, p.TN, p.NTK, \
                           p.tpw, p.rows, p.nslices, p.ncb, cscale, ws);                                       \
        break;
    switch (p.TPW) {
        MM_WG(1) MM_WG(2) MM_WG(3) MM_WG(5) MM_WG(8) MM_WG(12) MM_WG(16) MM_WG(20)
        default: return MM_E_ARG;
    }
#undef MM_WG
    return (int)hipGetLastError();
}

// the structured kernel for the (TN, NTK) blocks the actor and critic produce; 1 = no instantiation
template <int P, int TN, int NTK, int XB = 4, int AB = 4>
static int launch_rect_t(const WgPlan& p, const float* dy, int lddy, float dscale, const float* x, int ldx, int M,
                         int N, int K, float cscale, float* ws, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute((const void*)k_wgrad_rect<P, TN, NTK, XB, AB>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
            return MM_E_ARG;
        attr = true;
    }
    const size_t lds = (size_t)2 * (TN + NTK) * Prec<P>::kBlk * sizeof(uint16_t);
    hipLaunchKernelGGL((k_wgrad_rect<P, TN, NTK, XB, AB>), dim3(rup(p.nslices, 8) * p.ncb), dim3(kWgThreads), lds, s,
                       dy, lddy, dscale, x, ldx, M, N, K, p.rows, p.nslices, p.ncb, cscale, ws);
    return (int)hipGetLastError();
}

// the DMA-staged x2 kernel (k_wgrad_dma) for the actor trunk's two large shapes; MARLMAZE_WG_DMA=0 keeps
// k_wgrad_rect (A/B)
static int g_wgrad_algo = -1;
static bool wg_dma_enabled() {
    if (g_wgrad_algo < 0) {
        const char* e = getenv("MARLMAZE_WG_DMA");
        g_wgrad_algo = (e && e[0] == '0') ? MM_WGRAD_REG : MM_WGRAD_DMA;
    }
    return g_wgrad_algo == MM_WGRAD_DMA;
}

extern "C" int mm_gemm_wgrad_algo(int algo) {
    wg_dma_enabled();
    const int prev = g_wgrad_algo;
    if (algo == MM_WGRAD_DMA || algo == MM_WGRAD_REG) g_wgrad_algo = algo;
    return prev;
}

template <int TN, int NTK>
static int launch_dma_t(const WgPlan& p, const float* dy, int lddy, float dscale, const float* x, int ldx, int M,
                        int N, int K, float cscale, float* ws, hipStream_t s) {
    hipLaunchKernelGGL((k_wgrad_dma<P_X2, TN, NTK>), dim3(rup(p.nslices, 8) * p.ncb), dim3(kWgThreads), 0, s, dy,
                       lddy, dscale, x, ldx, M, N, K, p.rows, p.nslices, p.ncb, cscale, ws);
    return (int)hipGetLastError();
}

template <int P, int XB = 4, int AB = 4>
static int launch_rect_p(const WgPlan& p, const float* dy, int lddy, float dscale, const float* x, int ldx, int M,
                         int N, int K, float cscale, float* ws, hipStream_t s) {
    if constexpr (P == P_X2 && XB == 4 && AB == 4) {
        // 16-byte pieces: rows and bases 16-byte aligned (else the register-staged kernel)
        const bool al = (lddy % 4 == 0) && (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(dy) & 15) == 0) &&
                        ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
        if (wg_dma_enabled() && al) {
            if (p.TN == 17 && p.NTK == 9) return launch_dma_t<17, 9>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
            if (p.TN == 17 && p.NTK == 8) return launch_dma_t<17, 8>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
        }
    }
#define MM_WR(a, b)                                                                                              \
    if (p.TN == a && p.NTK == b)                                                                                 \
        return launch_rect_t<P, a, b, XB, AB>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
    if constexpr (XB == 2 && P == P_X3) {  // fp16 X at x3: the actor heads' weight gradient over h3 only
        MM_WR(1, 17)
    } else {
        MM_WR(17, 9) MM_WR(17, 8) MM_WR(1, 17) MM_WR(4, 9) MM_WR(4, 4) MM_WR(1, 4)
    }
#undef MM_WR
    return (XB == 2 || AB == 2) ? MM_E_ARG : 1;  // fp16 operands: no generic-kernel fallback
}

static int launch_wgrad_rect(int prec, const WgPlan& p, const float* dy, int lddy, float dscale, const float* x,
                             int ldx, int M, int N, int K, float cscale, float* ws, hipStream_t s, bool x16 = false,
                             bool a16 = false) {
    if (x16 || a16) {  // fp16 operands (X: P_F16 / P_X3; dY: P_F16): the structured kernel only
        if ((size_t)M * lddy * 4 >= ((size_t)1 << 31) || (size_t)M * ldx * 4 >= ((size_t)1 << 31)) return MM_E_ARG;
        if ((x16 && (ldx & 1)) || (a16 && (lddy & 1))) return MM_E_ARG;  // fp16 rows: dword-aligned
        if (prec == MM_PREC_X3) return a16 ? MM_E_ARG : launch_rect_p<P_X3, 2>(p, dy, lddy, 1.f, x, ldx, M, N, K, 1.f, ws, s);
        if (prec != MM_PREC_F16) return MM_E_ARG;
        if (a16 && x16) return launch_rect_p<P_F16, 2, 2>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
        if (a16) return launch_rect_p<P_F16, 4, 2>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
        return launch_rect_p<P_F16, 2>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
    }
#ifdef WG_GENERIC  // diagnostic builds: the generic kernel for every shape
    return 1;
#endif
    if ((size_t)M * lddy * 4 >= ((size_t)1 << 31) || (size_t)M * ldx * 4 >= ((size_t)1 << 31))
        return 1;  // loads through buffer resources (num_records < 2^31): the generic kernel
    return prec == MM_PREC_X3   ? launch_rect_p<P_X3>(p, dy, lddy, 1.f, x, ldx, M, N, K, 1.f, ws, s)
           : prec == MM_PREC_X2 ? launch_rect_p<P_X2>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s)
                                : launch_rect_p<P_F16>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
}

static int gemm_wgrad(int prec, const float* dy, int lddy, float dscale, const float* x, int ldx, int M, int N, int K,
                      float cscale, float* ws, float* dw, void* stream, int flags = 0) {
    if (M < 0 || N <= 0 || K <= 0 || N > 16 * kWgMaxT || lddy < N || ldx < K) return MM_E_ARG;
    if (flags & ~(MM_GEMM_B_F16 | MM_GEMM_A_F16)) return MM_E_ARG;
    const bool x16 = flags & MM_GEMM_B_F16, a16 = flags & MM_GEMM_A_F16;  // a16: dY fp16 (pre-scaled)
    if (prec != MM_PREC_X3 && prec != MM_PREC_F16 && prec != MM_PREC_X2) return MM_E_ARG;
    if (prec == MM_PREC_X3 && (dscale != 1.f || cscale != 1.f)) return MM_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (M == 0) return dw ? (int)hipMemsetAsync(dw, 0, sizeof(float) * (size_t)N * K, s) : MM_E_ARG;
    if (!dy || !x || !ws) return MM_E_ARG;
    const WgPlan p = wg_plan(prec, M, N, K);
    if (!p.TPW) return MM_E_ARG;
    int e = launch_wgrad_rect(prec, p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s, x16, a16);
    if (e == 1 && !x16 && !a16)
        e = prec == MM_PREC_X3   ? launch_wgrad<P_X3>(p, dy, lddy, 1.f, x, ldx, M, N, K, 1.f, ws, s)
            : prec == MM_PREC_X2 ? launch_wgrad<P_X2>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s)
                                 : launch_wgrad<P_F16>(p, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, s);
    if (e) return e;
    const long n = (long)N * K;
    if (!dw) return 0;  // mm_gemm_wgrad_partials: the caller reduces (mm_wsum_multi)
    hipLaunchKernelGGL(k_wg_reduce, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, s, ws, p.nslices, n, dw);
    return (int)hipGetLastError();
}

extern "C" int mm_gemm_wgrad(int prec, const float* dy, int lddy, float dscale, const float* x, int ldx, int M, int N,
                             int K, float cscale, float* ws, float* dw, void* stream) {
    if (!dw) return MM_E_ARG;
    return gemm_wgrad(prec, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, dw, stream);
}

extern "C" int mm_gemm_wgrad_h(int prec, int flags, const float* dy, int lddy, float dscale, const void* x, int ldx,
                               int M, int N, int K, float cscale, float* ws, float* dw, void* stream) {
    if (!dw) return MM_E_ARG;
    return gemm_wgrad(prec, dy, lddy, dscale, static_cast<const float*>(x), ldx, M, N, K, cscale, ws, dw, stream,
                      flags);
}

extern "C" int mm_gemm_wgrad_partials_h(int prec, int flags, const float* dy, int lddy, float dscale, const void* x,
                                        int ldx, int M, int N, int K, float cscale, float* ws, void* stream) {
    if (M <= 0) return MM_E_ARG;
    return gemm_wgrad(prec, dy, lddy, dscale, static_cast<const float*>(x), ldx, M, N, K, cscale, ws, nullptr, stream,
                      flags);
}

extern "C" int mm_gemm_a16_ok(int M, int N, int K, int lda, int ldc) {
    BresPlan pl;
    int cfg = C_NARROW;
    return bres_enabled() && bres_plan(MM_PREC_F16, M, N, K, lda, ldc, true, pl, cfg) ? 1 : 0;
}

extern "C" int mm_gemm_wgrad_slices(int prec, int M, int N, int K) {
    if (M <= 0 || N <= 0 || K <= 0 || (prec != MM_PREC_X3 && prec != MM_PREC_F16 && prec != MM_PREC_X2))
        return MM_E_ARG;
    const WgPlan p = wg_plan(prec, M, N, K);
    return p.TPW ? p.nslices : MM_E_ARG;
}

extern "C" int mm_gemm_wgrad_partials(int prec, const float* dy, int lddy, float dscale, const float* x, int ldx, int M,
                                      int N, int K, float cscale, float* ws, void* stream) {
    if (M <= 0) return MM_E_ARG;
    return gemm_wgrad(prec, dy, lddy, dscale, x, ldx, M, N, K, cscale, ws, nullptr, stream);
}
