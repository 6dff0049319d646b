// gemm_x3.hip -- fp32 GEMMs of the actor/critic MLP on gfx950's bf16 MFMA.
//
// gfx950 runs f32-input MFMA at 1/16 of the bf16 MFMA rate (157 vs 2,500
// TFLOP/s dense).  Each fp32 operand is split exactly into three bf16 parts,
// x = hi + mid + lo (hi = RN_bf16(x), mid = RN_bf16(x - hi), lo =
// RN_bf16(x - hi - mid); the subtractions are exact in fp32, and the three
// parts carry all 24 significand bits).  A product a*b is then the sum of nine
// bf16 products, each exact in the fp32 accumulator; the six whose magnitude
// is >= 2^-16 |a b| are kept (hi*hi, hi*mid, mid*hi, mid*mid, hi*lo, lo*hi),
// the dropped three are below 2^-23 |a b|, i.e. at the level of one fp32
// rounding.  Accumulation is fp32 (MFMA accumulators), as in an fp32 GEMM.
// Six bf16 MFMAs per fp32 product: 2,500 / 6 = 417 TFLOP/s of fp32-accurate
// peak against 157 for the f32 MFMA.
//
// Status: exact to fp32 level (max error vs fp64 2.4-2.8e-7 of sum|ab|, below the
// fp32 library GEMM's 2.7-3.5e-7), but at 78-85 TFLOP/s effective it does not
// yet beat the tuned fp32 hipBLASLt kernels (90-110 TFLOP/s) on the MLP
// shapes: the per-k-step restaging of B (pre-split planes, 1.5x the fp32
// bytes, re-read by every row block) and LDS bank conflicts dominate
// (rocprofv3: MFMA busy 22%, waits 62%).  Selected with MARLMAZE_GEMM=x3.
//
// Kernel: C[M, N] = A[M, K] . B[N, K]^T (+ bias[N]) (ReLU), all row-major fp32
// with K contiguous -- the layout of y = x W^T (nn.Linear forward) and, with
// B = W^T, of dX = dY W.  Workgroup = 8 waves, tile 256 rows x 16*NT
// columns, K in steps of 32 (one mfma_f32_16x16x32_bf16 k-step).  The fp32
// tiles are loaded, split and written to LDS as three bf16 planes; each wave
// owns 32 rows x 16*NT columns (2 x NT accumulator tiles).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "marlmaze.h"

namespace mm {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kGBK = 32;       // k per step
constexpr int kGLd = kGBK;  // bf16 per LDS row (64 B), 16-byte chunks XOR-swizzled by (row >> 1) & 3
// so that fragment reads and both staging writes are bank-conflict free

__device__ __forceinline__ int swz(int row, int chunk) { return row * kGLd + 8 * (chunk ^ ((row >> 1) & 3)); }

__device__ __forceinline__ uint32_t bf16_rn(float x) {  // round-to-nearest-even, finite x
    const uint32_t u = __float_as_uint(x);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

// x -> (hi, mid, lo) bf16 bit patterns
__device__ __forceinline__ void split3(float x, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
    hi = bf16_rn(x);
    const float r1 = x - __uint_as_float(hi << 16);
    mid = bf16_rn(r1);
    const float r2 = r1 - __uint_as_float(mid << 16);
    lo = bf16_rn(r2);
}

// lane l's 16x16x32 operand fragment of rows [16 t, 16 t + 16) of a plane:
// row l & 15, k = 8 (l >> 4) .. + 7
__device__ __forceinline__ bf16x8 frag(const uint16_t* __restrict__ plane, int t, int lane) {
    return *reinterpret_cast<const bf16x8*>(plane + swz(16 * t + (lane & 15), lane >> 4));
}

// B [N, K] fp32 -> pre-split tiles, once per GEMM: for column block cb and
// k-step ks, one contiguous block Bs[cb][ks][plane][n < BN][32] of bf16 (zero
// padded), so a workgroup's per-step copy is one linear, coalesced read.
__global__ __launch_bounds__(256) void k_split_b(const float* __restrict__ B, int N, int K, int BN, int nks,
                                                 int total, uint16_t* __restrict__ Bs) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int kk = e % kGBK, n = (e / kGBK) % BN, p = (e / (kGBK * BN)) % 3, ks = (e / (kGBK * BN * 3)) % nks,
              cb = e / (kGBK * BN * 3 * nks);
    const int gn = cb * BN + n, gk = ks * kGBK + kk;
    const float x = (gn < N && gk < K) ? B[(size_t)gn * K + gk] : 0.f;
    uint32_t h, m, l;
    split3(x, h, m, l);
    Bs[e] = (uint16_t)(p == 0 ? h : (p == 1 ? m : l));
}

// One workgroup: 4 waves x 32 rows = 128 rows, 16*NT columns.  LDS per
// workgroup = 3 bf16 planes of A (128 x 80 B) + of B (16 NT x 80 B) <= 80 KB,
// so two workgroups share a CU: their load/split phases and MFMA phases
// interleave (one barrier-synchronised workgroup cannot overlap them itself).
constexpr int kXWaves = 4;
constexpr int kXThreads = kXWaves * 64;
constexpr int kXBM = 32 * kXWaves;

template <int NT>
__global__ __launch_bounds__(kXThreads, 3) void k_gemm_x3(const float* __restrict__ A,
                                                          const uint16_t* __restrict__ Bs, int nks,
                                                          const float* __restrict__ bias, float* __restrict__ C,
                                                          int M, int N, int K, int relu) {
    constexpr int BN = 16 * NT;
    constexpr int AQ = kXBM * (kGBK / 4) / kXThreads;              // A float4 per thread per k-step (4)
    constexpr int BPIECES = 3 * BN * (kGBK / 8);                    // 16-byte B pieces per k-step
    __shared__ __attribute__((aligned(16))) uint16_t sA[3][kXBM * kGLd];
    __shared__ __attribute__((aligned(16))) uint16_t sB[3][BN * kGLd];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * kXBM;  // column blocks of one row block are adjacent
    const uint4* btiles = reinterpret_cast<const uint4*>(Bs) + (size_t)blockIdx.x * nks * (BPIECES);
    f32x4 acc[2][NT];
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int c = 0; c < NT; c++) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    float4 pa[AQ];  // next k-step's A (thread t: quads t + 256 i; row e / 8, k quad e % 8)
    auto load_a = [&](int k0) {
#pragma unroll
        for (int i = 0; i < AQ; i++) {
            const int e = threadIdx.x + i * kXThreads;
            const int gr = m0 + e / (kGBK / 4), gk = k0 + 4 * (e % (kGBK / 4));
            pa[i] = (gr < M && gk < K) ? *reinterpret_cast<const float4*>(A + (size_t)gr * K + gk)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    load_a(0);
    for (int k0 = 0; k0 < K; k0 += kGBK) {
        __syncthreads();  // previous step's fragment reads are done
#pragma unroll
        for (int i = 0; i < AQ; i++) {  // A: split into the three planes
            const int e = threadIdx.x + i * kXThreads;
            const int r = e / (kGBK / 4), kq = e % (kGBK / 4);
            uint32_t h0, m0_, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
            split3(pa[i].x, h0, m0_, l0);
            split3(pa[i].y, h1, m1, l1);
            split3(pa[i].z, h2, m2, l2);
            split3(pa[i].w, h3, m3, l3);
            const int o = swz(r, kq >> 1) + 4 * (kq & 1);
            *reinterpret_cast<uint2*>(sA[0] + o) = make_uint2(h0 | (h1 << 16), h2 | (h3 << 16));
            *reinterpret_cast<uint2*>(sA[1] + o) = make_uint2(m0_ | (m1 << 16), m2 | (m3 << 16));
            *reinterpret_cast<uint2*>(sA[2] + o) = make_uint2(l0 | (l1 << 16), l2 | (l3 << 16));
        }
        {  // B: this k-step's pre-split tile, one contiguous block (coalesced 16-byte pieces)
            const uint4* bt = btiles + (size_t)(k0 / kGBK) * BPIECES;
            for (int e = threadIdx.x; e < BPIECES; e += kXThreads) {
                const int p = e / (BN * (kGBK / 8)), n = (e / (kGBK / 8)) % BN, k8 = e % (kGBK / 8);
                *reinterpret_cast<uint4*>(sB[p] + swz(n, k8)) = bt[e];
            }
        }
        __syncthreads();
        if (k0 + kGBK < K) load_a(k0 + kGBK);  // next step's A in flight during the MFMAs
        bf16x8 a[2][3];
#pragma unroll
        for (int r = 0; r < 2; r++)
#pragma unroll
            for (int p = 0; p < 3; p++) a[r][p] = frag(sA[p], 2 * wave + r, lane);
#pragma unroll
        for (int c = 0; c < NT; c++) {
            const bf16x8 bh = frag(sB[0], c, lane), bm = frag(sB[1], c, lane), bl = frag(sB[2], c, lane);
#pragma unroll
            for (int r = 0; r < 2; r++) {  // small terms first
                acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][2], bh, acc[r][c], 0, 0, 0);
                acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], bl, acc[r][c], 0, 0, 0);
                acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][1], bm, acc[r][c], 0, 0, 0);
                acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][1], bh, acc[r][c], 0, 0, 0);
                acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], bm, acc[r][c], 0, 0, 0);
                acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[r][0], bh, acc[r][c], 0, 0, 0);
            }
        }
    }
    // epilogue: C/D map col = lane & 15, row = (lane >> 4) * 4 + reg
#pragma unroll
    for (int c = 0; c < NT; c++) {
        const int col = n0 + 16 * c + (lane & 15);
        if (col >= N) continue;
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 2; r++) {
#pragma unroll
            for (int g = 0; g < 4; g++) {
                const int row = m0 + 32 * wave + 16 * r + 4 * (lane >> 4) + g;
                if (row < M) {
                    float v = acc[r][c][g] + bv;
                    if (relu) v = v > 0.f ? v : 0.f;
                    C[(size_t)row * N + col] = v;
                }
            }
        }
    }
}

}  // namespace mm

using namespace mm;

// column block width: 144 (N <= 288, e.g. 264 -> 2 blocks) or 160 (460 -> 3 blocks)
static void x3_shape(int N, int K, int* BN, int* ncb, int* nks) {
    *BN = N <= 288 ? 16 * 9 : 16 * 10;
    *ncb = (N + *BN - 1) / *BN;
    *nks = (K + kGBK - 1) / kGBK;
}

extern "C" int mm_gemm_x3_bsplit_len(int N, int K) {
    int BN, ncb, nks;
    x3_shape(N, K, &BN, &ncb, &nks);
    return ncb * nks * 3 * BN * kGBK;  // uint16 elements
}

extern "C" int mm_gemm_x3(const float* A, const float* B, const float* bias, float* C, int M, int N, int K, int relu,
                          uint16_t* bsplit, void* stream) {
    if (!A || !B || !C || !bsplit || M < 0 || N <= 0 || K <= 0 || (K & 3)) return MM_E_ARG;
    if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)bsplit) & 15) return MM_E_ARG;
    if (M == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int gm = (M + kXBM - 1) / kXBM;
    int BN, ncb, nks;
    x3_shape(N, K, &BN, &ncb, &nks);
    const int total = ncb * nks * 3 * BN * kGBK;
    hipLaunchKernelGGL(k_split_b, dim3((total + 255) / 256), dim3(256), 0, s, B, N, K, BN, nks, total, bsplit);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    if (BN == 16 * 9) {
        hipLaunchKernelGGL(k_gemm_x3<9>, dim3(ncb, gm), dim3(kXThreads), 0, s, A, bsplit, nks, bias, C, M, N, K, relu);
    } else {
        hipLaunchKernelGGL(k_gemm_x3<10>, dim3(ncb, gm), dim3(kXThreads), 0, s, A, bsplit, nks, bias, C, M, N, K,
                           relu);
    }
    return (int)hipGetLastError();
}
