// Probe: how does v_mfma_f32_16x16x32_bf16 round?  D = C + sum_k a_k * 1.0 with
// chosen a_k (bf16) and C (fp32), printed against the exact sum.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_build/mfma_round tools/mfma_round.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f4;

__device__ short bf(float x) { unsigned u = __float_as_uint(x); return (short)(u >> 16); }  // exact for our values

__global__ void probe(const float* vals, const float* cs, int ncase, float* out) {
    const int l = threadIdx.x;
    for (int t = 0; t < ncase; t++) {
        bf16x8 a, b;
        for (int j = 0; j < 8; j++) {
            a[j] = bf(vals[t * 32 + 8 * (l >> 4) + j]);
            b[j] = bf(1.0f);
        }
        f4 c = {cs[t], cs[t], cs[t], cs[t]};
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
        if (l == 0) out[t] = c[0];
    }
}

int main() {
    const int N = 12;
    float v[N * 32] = {0}, c[N] = {0};
    const float t26 = ldexpf(1.f, -26);
    const char* name[N];
    // a: group 0 = [1, 7 x 2^-26]
    name[0] = "[1, 7x2^-26] k0-7"; v[0] = 1.f; for (int k = 1; k < 8; k++) v[k] = t26;
    // b: 1 at k0, 7 tiny at k8..14
    name[1] = "1@k0, 7x2^-26 @k8-14"; v[32] = 1.f; for (int k = 8; k < 15; k++) v[32 + k] = t26;
    // c: negative of a
    name[2] = "-[1, 7x2^-26] k0-7"; v[64] = -1.f; for (int k = 1; k < 8; k++) v[64 + k] = -t26;
    // d: 1, -7 tiny in group 0
    name[3] = "[1, -7x2^-26] k0-7"; v[96] = 1.f; for (int k = 1; k < 8; k++) v[96 + k] = -t26;
    // e: 1 at k0, 3 tiny at k4..6 (group of 4?)
    name[4] = "1@k0, 3x2^-26 @k4-6"; v[128] = 1.f; for (int k = 4; k < 7; k++) v[128 + k] = t26;
    // f: 1 at k0, 3 tiny at k1..3
    name[5] = "1@k0, 3x2^-26 @k1-3"; v[160] = 1.f; for (int k = 1; k < 4; k++) v[160 + k] = t26;
    // g: 1 at k0, 1 tiny at k1: 2^-24*1.5 (=3*2^-25) exact sum 1+0.75ulp
    name[6] = "1@k0, 3*2^-25@k1"; v[192] = 1.f; v[193] = 3 * ldexpf(1.f, -25);
    // h: 1 at k0, 3*2^-25 at k16
    name[7] = "1@k0, 3*2^-25@k16"; v[224] = 1.f; v[224 + 16] = 3 * ldexpf(1.f, -25);
    // i: C = 1, products 7 x 2^-26 in group 0
    name[8] = "C=1, 7x2^-26 k0-6"; c[8] = 1.f; for (int k = 0; k < 7; k++) v[256 + k] = t26;
    // j: 1 at k0, 1 tiny 1.5*2^-24 at k8 (separate groups)
    name[9] = "1@k0, 3*2^-25@k8"; v[288] = 1.f; v[288 + 8] = 3 * ldexpf(1.f, -25);
    // k: 1 at k0, -3*2^-25 at k1  (exact 1 - 1.5*2^-24 = 1 - 1.5 ulp_below): RNE -> 1 - 2*2^-24
    name[10] = "1@k0, -3*2^-25@k1"; v[320] = 1.f; v[321] = -3 * ldexpf(1.f, -25);
    // l: 1 at k0, 2^-25 + 2^-26 spread k1,k2 (exact 1+0.75*2^-24... = 1 + 0.375 ulp) RNE->1
    name[11] = "1@k0, 2^-24@k1, 2^-24@k2"; v[352] = 1.f; v[353] = ldexpf(1.f, -24); v[354] = ldexpf(1.f, -24);
    float *dv, *dc, *dout;
    hipMalloc(&dv, sizeof v); hipMalloc(&dc, sizeof c); hipMalloc(&dout, N * 4);
    hipMemcpy(dv, v, sizeof v, hipMemcpyHostToDevice);
    hipMemcpy(dc, c, sizeof c, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dv, dc, N, dout);
    float o[N];
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    for (int t = 0; t < N; t++) {
        double ex = c[t];
        for (int k = 0; k < 32; k++) ex += v[t * 32 + k];
        const double ref = ex < 0 ? -1.0 : 1.0;
        printf("case %-26s got %+.4f  exact %+.4f  (x 2^-24, offset from %+.0f)\n", name[t],
               ((double)o[t] - ref) * 16777216.0, (ex - ref) * 16777216.0, ref);
    }
    return 0;
}
