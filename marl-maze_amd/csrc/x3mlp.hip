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
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "marlmaze.h"

namespace mm {
namespace x3 {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kBlk = 1536;  // uint16 per (rt, ks) block: 3 planes x 512
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

// fp32 [R, C] (row-major, leading dimension ld; trans: element (i, j) at
// X[j * ld + i]) -> TP.  One thread per (rt, ks, c, r) 8-element piece.
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
        uint4 h, m, lo;
        split8(v, h, m, lo);
        uint4* dst = reinterpret_cast<uint4*>(tp + blk * kBlk) + l;
        dst[0] = h;
        dst[64] = m;
        dst[128] = lo;
    }
}

constexpr int kWaves = 16;
constexpr int kThreads = 64 * kWaves;
constexpr int kBM = 16 * kWaves;  // rows per workgroup: one row tile per wave
static_assert(kBM <= kRowPad, "A row blocks must stay inside the TP row padding");

template <int NT>
struct Cfg {
    static constexpr int kPiecesB = 3 * NT;                     // 1-KiB B pieces per k-step
    static constexpr int kPerWaveB = (kPiecesB + kWaves - 1) / kWaves;
    static constexpr int kStageB = NT * kBlk;                   // uint16 per B stage
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
};

// B piece i (column tile i / 3, plane i % 3) of k-step ks -> LDS (one 1-KiB LDS-DMA)
__device__ __forceinline__ void dma_b(const uint16_t* Bg, int nks, int ks, int i, uint16_t* dst, int lane) {
    const int ct = i / 3, p = i - 3 * ct;
    const uint4* src = reinterpret_cast<const uint4*>(Bg + ((size_t)ct * nks + ks) * kBlk + p * 512);
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

// A operand sources.  A wave owns one row tile; per k-step each lane needs the
// 8 values (row 16 rt + (l & 15), k 32 ks + 8 (l >> 4) .. +7) as three bf16x8.
struct ASrcTP {  // pre-split TP planes: three lane-linear 1-KiB loads
    typedef bf16x8 Raw[3];
    const uint16_t* A;  // the wave's row tile
    int nks;
    __device__ void init(const uint16_t* base, int rt, int nks_, int, int, int) {
        nks = nks_;
        A = base + (size_t)rt * nks * kBlk;
    }
    __device__ __forceinline__ void load(int ks, Raw& r, int lane) const {
        const uint4* p = reinterpret_cast<const uint4*>(A + (size_t)ks * kBlk);
#pragma unroll
        for (int q = 0; q < 3; q++) r[q] = __builtin_bit_cast(bf16x8, p[64 * q + lane]);
    }
    __device__ __forceinline__ void frag(const Raw& r, bf16x8 (&a)[3]) const {
#pragma unroll
        for (int q = 0; q < 3; q++) a[q] = r[q];
    }
};

struct ASrcF32 {  // fp32 row-major [M, lda]: two 16-byte loads per lane, split in registers
    typedef float4 Raw[2];
    const float* row;  // this lane's row (clamped inside the matrix), column 8 (l >> 4)
    int K, ok;         // ok: the row exists
    __device__ void init(const float* base, int rt, int, int M, int lda, int K_) {
        const int lane = threadIdx.x & 63;
        const int r = 16 * rt + (lane & 15);
        ok = r < M;
        K = K_;
        row = base + (size_t)(ok ? r : 0) * lda + 4 * (lane >> 4);
    }
    __device__ __forceinline__ void load(int ks, Raw& r, int lane) const {
        const int k = 32 * ks + 4 * (lane >> 4);  // kcol(c, 0..3) = 4c.., kcol(c, 4..7) = 16 + 4c..
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        r[0] = (ok && k < K) ? *reinterpret_cast<const float4*>(row + 32 * ks) : z;
        r[1] = (ok && k + 16 < K) ? *reinterpret_cast<const float4*>(row + 32 * ks + 16) : z;
    }
    __device__ __forceinline__ void frag(const Raw& r, bf16x8 (&a)[3]) const {
        uint32_t h[4], m[4], l[4];
        split2(r[0].x, r[0].y, h[0], m[0], l[0]);
        split2(r[0].z, r[0].w, h[1], m[1], l[1]);
        split2(r[1].x, r[1].y, h[2], m[2], l[2]);
        split2(r[1].z, r[1].w, h[3], m[3], l[3]);
        a[0] = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
        a[1] = __builtin_bit_cast(bf16x8, make_uint4(m[0], m[1], m[2], m[3]));
        a[2] = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
    }
};

// One k-step on stage buffer `cur`: split this step's A (raw -> fragments),
// prefetch the next step's raw A (registers) and B pieces (the other buffer;
// the DMA issues spread over the column loop), the 6 x NT MFMAs, one barrier.
template <int NT, class AS>
__device__ __forceinline__ void k_step(f32x4 (&acc)[NT], const AS& as, const typename AS::Raw& raw,
                                       typename AS::Raw& rawn, const uint16_t* Bg, int nks, int ks,
                                       const uint16_t* cur, uint16_t* nxt, int wave, int lane) {
    using C = Cfg<NT>;
    const bool more = ks + 1 < nks;
    bf16x8 a[3];
    as.frag(raw, a);
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
            const int i = wave + kWaves * c;
            if (i < C::kPiecesB) dma_b(Bg, nks, ks + 1, i, nxt + i * 512, lane);
        }
        const bf16x8 bh = b8[(c * 3 + 0) * 64], bm = b8[(c * 3 + 1) * 64], bl = b8[(c * 3 + 2) * 64];
        // small terms first
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bh, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bl, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bm, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bh, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bm, acc[c], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bh, acc[c], 0, 0, 0);
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
enum { EM_F32 = 0, EM_FWD = 1, EM_BWD = 2, EM_TP = 3 };

template <int NT, int EM>
__device__ __forceinline__ void epilogue_f32(const f32x4 (&acc)[NT], int rt, int M, int N, int col0, const Epi& ep,
                                             const float* sbias, int lane) {
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
                if (row < M && ((bits[(4 * c + g) >> 5] >> ((4 * c + g) & 31)) & 1u)) cs += acc[c][g];
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
template <int NT, class AS, class AT, int EM>
__global__ __launch_bounds__(kThreads) void k_x3nt(const AT* __restrict__ A, int lda, const uint16_t* __restrict__ B,
                                                   int M, int N, int K, int nks, int nrb, int ncb, Epi ep) {
    using C = Cfg<NT>;
    // two distinct LDS objects: the compiler's alias scopes then let a B read of
    // one stage run while the DMA into the other is in flight
    __shared__ float sbias[16 * NT];  // the unit's bias columns (EM_F32 / EM_FWD); first: small LDS offsets
    __shared__ __attribute__((aligned(16))) uint16_t sB0[C::kLen0];
    __shared__ __attribute__((aligned(16))) uint16_t sB1[C::kStageB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // workgroup g takes units g, g + G, ...  XCD-aware unit order: units u and
    // u + 8 (one XCD) are the column blocks of one row block, so its A is shared
    // through that XCD's L2
    const int nunits = ((nrb + 7) / 8) * 8 * ncb;
    for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
        const int xcd = u & 7, slot = u >> 3;
        const int rb = (slot / ncb) * 8 + xcd, cb = slot % ncb;
        if (rb >= nrb) continue;  // workgroup-uniform
        const int rt = rb * kWaves + wave;  // this wave's row tile
        AS as;
        as.init(A, rt, nks, M, lda, K);
        const uint16_t* Bg = B + (size_t)cb * NT * nks * kBlk;
        if (EM != EM_BWD && EM != EM_TP && ep.bias && threadIdx.x < 16 * NT) {  // visible after the prologue barrier
            int t = threadIdx.x;
            asm volatile("" : "+v"(t));  // recomputed per unit, not a loop-invariant address held (spilled) across it
            const int col = cb * 16 * NT + t;
            sbias[t] = col < N ? ep.bias[col] : 0.f;
        }

        f32x4 acc[NT];
#pragma unroll
        for (int c = 0; c < NT; c++) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};

        typename AS::Raw r0, r1;
        for (int i = wave; i < C::kPiecesB; i += kWaves) dma_b(Bg, nks, 0, i, sB0 + i * 512, lane);
        as.load(0, r0, lane);
        __syncthreads();
        // k-steps in pairs so the two stage buffers are compile-time distinct
        // (no wait of a B fragment read on the other buffer's DMA)
        int ks = 0;
        for (; ks + 1 < nks; ks += 2) {
            k_step<NT>(acc, as, r0, r1, Bg, nks, ks, sB0, sB1, wave, lane);
            k_step<NT>(acc, as, r1, r0, Bg, nks, ks + 1, sB1, sB0, wave, lane);
        }
        if (ks < nks) k_step<NT>(acc, as, r0, r1, Bg, nks, ks, sB0, sB1, wave, lane);

        // ---- epilogue (after the last k-step's barrier both stage buffers are free) ----
        if (EM == EM_TP)
            epilogue_tp<NT>(acc, reinterpret_cast<float*>(sB0) + wave * 16 * 36, rt, M, N, ep, lane);
        else
            epilogue_f32<NT, EM>(acc, rt, M, N, cb * 16 * NT, ep, sbias, lane);
        // the next unit's DMA overwrites the epilogue slices: LDS reads done everywhere
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt((15 << 0) | (7 << 4) | (0 << 8) | (3 << 14));  // lgkmcnt(0) only
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Backward of the actor heads into the last hidden layer (networks.py:38-41 +
// the ReLU of :36): dY[m, n] = (sum_j dz[m, j] W[j, n]) * bit(m, n), W [J, N]
// the concatenated head weights, bits the last forward GEMM's ReLU mask.  Same
// tile map as the GEMM epilogue (one wave per 16-row tile, lane l: rows
// 4 (l >> 4) + g, columns 16 c + (l & 15)), so the mask bits line up; also the
// per-tile column sums (the last layer's bias gradient, before the final sum).
constexpr int kHeadsMaxJ = 8;
template <int NT>
__global__ __launch_bounds__(256) void k_heads_bwd(const float* __restrict__ dz, int J, const float* __restrict__ W,
                                                   const uint32_t* __restrict__ bits, int M, int N,
                                                   float* __restrict__ dy, float* __restrict__ colsum) {
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
                dy[(size_t)row * N + col] = x;
                cs += x;
            }
        }
        cs += __shfl_xor(cs, 16);
        cs += __shfl_xor(cs, 32);
        if (lane < 16 && col < N) colsum[(size_t)rt * N + col] = cs;
    }
}

}  // namespace x3
}  // namespace mm

using namespace mm::x3;

extern "C" long mm_x3_tp_len(int R, int C) { return (long)(rup(R, kRowPad) / 16) * (rup(C, 32) / 32) * kBlk; }

extern "C" long mm_x3_mbits_len(int M) { return (long)(rup(M, kRowPad) / 16) * 64 * kMaskWords; }

extern "C" int mm_x3_tp_pack(const float* X, int R, int C, int ld, int trans, uint16_t* tp, void* stream) {
    if (!X || !tp || R <= 0 || C <= 0 || ld < (trans ? R : C)) return MM_E_ARG;
    if ((uintptr_t)tp & 15) return MM_E_ARG;
    const int nks = rup(C, 32) / 32;
    const long total = (long)(rup(R, kRowPad) / 16) * nks * 64;
    const int grid = (int)std::min<long>((total + 255) / 256, 256L * 64);
    hipLaunchKernelGGL(k_tp_pack, dim3(grid), dim3(256), 0, (hipStream_t)stream, X, R, C, ld, trans, nks, total, tp);
    return (int)hipGetLastError();
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

template <int NT, class AS, class AT>
static int launch_nt(const AT* a, int lda, const uint16_t* b, int M, int N, int K, int ncb, const Epi& ep,
                     hipStream_t s) {
    const int nks = rup(K, 32) / 32;
    const int nrb = rup(M, kBM) / kBM;
    const int grid = std::min(rup(nrb, 8) * ncb, persistent_grid());
    if (ep.ctp && ep.c) return MM_E_ARG;  // one output form per launch
    if (ep.ctp)
        hipLaunchKernelGGL((k_x3nt<NT, AS, AT, EM_TP>), dim3(grid), dim3(kThreads), 0, s, a, lda, b, M, N, K, nks, nrb,
                           ncb, ep);
    else if (ep.mbits_out)
        hipLaunchKernelGGL((k_x3nt<NT, AS, AT, EM_FWD>), dim3(grid), dim3(kThreads), 0, s, a, lda, b, M, N, K, nks,
                           nrb, ncb, ep);
    else if (ep.mbits_in)
        hipLaunchKernelGGL((k_x3nt<NT, AS, AT, EM_BWD>), dim3(grid), dim3(kThreads), 0, s, a, lda, b, M, N, K, nks,
                           nrb, ncb, ep);
    else
        hipLaunchKernelGGL((k_x3nt<NT, AS, AT, EM_F32>), dim3(grid), dim3(kThreads), 0, s, a, lda, b, M, N, K, nks,
                           nrb, ncb, ep);
    return (int)hipGetLastError();
}

template <class AS, class AT>
static int dispatch_nt(const AT* a, int lda, const uint16_t* b_tp, int M, int N, int K, const Epi& ep,
                       hipStream_t s) {
    // column tiling: one block of <= 17 tiles, or several blocks of 15 (B rows are padded to 256)
    const int tiles = (N + 15) / 16;
    int NT, ncb;
    if (tiles <= 4) { NT = 4; ncb = 1; }
    else if (tiles <= 8) { NT = 8; ncb = 1; }
    else if (tiles <= 17) { NT = 17; ncb = 1; }
    else { NT = 15; ncb = (tiles + 14) / 15; }
    if (ncb * NT * 16 > rup(N, kRowPad)) return MM_E_ARG;  // B TP row padding would be overrun
    if (ep.ctp && ncb != 1) return MM_E_ARG;
    switch (NT) {
        case 4: return launch_nt<4, AS>(a, lda, b_tp, M, N, K, ncb, ep, s);
        case 8: return launch_nt<8, AS>(a, lda, b_tp, M, N, K, ncb, ep, s);
        case 15: return launch_nt<15, AS>(a, lda, b_tp, M, N, K, ncb, ep, s);
        default: return launch_nt<17, AS>(a, lda, b_tp, M, N, K, ncb, ep, s);
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
    Epi ep{bias, mask, nullptr, nullptr, c, c_tp, nullptr, ldc, ldm, relu, rup(N, 32) / 32};
    return dispatch_nt<ASrcTP>(a_tp, 0, b_tp, M, N, K, ep, (hipStream_t)stream);
}

// The same with A fp32 row-major [M, lda] (K % 4 == 0, lda % 4 == 0, 16-byte
// aligned), split into bf16 planes in registers inside the GEMM.
extern "C" int mm_x3_nt_f32a(const float* a, int lda, const uint16_t* b_tp, int M, int N, int K, const float* bias,
                             int relu, const float* mask, int ldm, const uint32_t* mbits_in, uint32_t* mbits_out,
                             float* colsum, float* c, int ldc, uint16_t* c_tp, void* stream) {
    int e = check_common(b_tp, M, N, K, mask, ldm, c, ldc, c_tp);
    if (e) return e;
    if (!a || (K & 3) || (lda & 3) || lda < K || ((uintptr_t)a & 15)) return MM_E_ARG;
    if ((mbits_in || mbits_out) && (N > 16 * 17 || c_tp || mask || (mbits_in && mbits_out))) return MM_E_ARG;
    if (mbits_in && (bias || relu)) return MM_E_ARG;  // the input-gradient form: no bias, no ReLU of its own
    if (colsum && (!mbits_in || !c)) return MM_E_ARG;
    if (M == 0) return 0;
    Epi ep{bias, mask, mbits_in, mbits_out, c, c_tp, colsum, ldc, ldm, relu, rup(N, 32) / 32};
    return dispatch_nt<ASrcF32>(a, lda, b_tp, M, N, K, ep, (hipStream_t)stream);
}

// dY = (dz W) * bits (the heads' backward through the last ReLU, bits from the
// last forward GEMM's mbits_out, N <= 272, J <= 8), and the per-16-row-tile
// column sums colsum [ceil(M / 16), N].
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
