// Cycles per MFMA, back-to-back on one SIMD (one wave per SIMD, 4 independent accumulators):
// v_mfma_f32_16x16x16_f16 (the x2 / f16 GEMMs' instruction) against v_mfma_f32_16x16x32_f16 and the f32-input
// v_mfma_f32_16x16x4_f32.  Build and run: hipcc --offload-arch=gfx950 -O3 tools/mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) _Float16 h4;
typedef __attribute__((ext_vector_type(8))) _Float16 h8;

constexpr int kIters = 4096;

template <int KIND>
__global__ void k_rate(float* out, long long* cyc, float seed) {
    f4 acc[4] = {};
    h4 a4, b4;
    h8 a8, b8;
    for (int i = 0; i < 4; i++) a4[i] = (_Float16)(seed + threadIdx.x + i), b4[i] = (_Float16)(seed - i);
    for (int i = 0; i < 8; i++) a8[i] = (_Float16)(seed + threadIdx.x + i), b8[i] = (_Float16)(seed - i);
    float af = seed + threadIdx.x, bf = seed * 0.5f;
    const long long t0 = clock64();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if constexpr (KIND == 0) acc[j] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc[j], 0, 0, 0);
            else if constexpr (KIND == 1) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc[j], 0, 0, 0);
            else acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, acc[j], 0, 0, 0);
        }
    }
    const long long t1 = clock64();
    float s = 0.f;
    for (int j = 0; j < 4; j++) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, float* out, long long* cyc) {
    hipLaunchKernelGGL(k_rate<KIND>, dim3(1), dim3(64), 0, 0, out, cyc, 1.f);
    hipDeviceSynchronize();
    long long c = 0;
    hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-28s %.2f cycles per MFMA (clock64 ticks)\n", name, (double)c / (4.0 * kIters));
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 64 * 4);
    hipMalloc(&cyc, 8);
    for (int rep = 0; rep < 2; rep++) {
        run<0>("v_mfma_f32_16x16x16_f16", out, cyc);
        run<1>("v_mfma_f32_16x16x32_f16", out, cyc);
        run<2>("v_mfma_f32_16x16x4_f32", out, cyc);
    }
    return 0;
}
