// Probe: operand / accumulator layout of v_mfma_f64_16x16x4_f64 on gfx950 with
// exact integer data (C = A B for A 16x4, B 4x16), checked on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* C) {
    const int l = threadIdx.x;
    const double a = A[(l & 15) * 4 + (l >> 4)];   // A[row l&15][k l>>4]
    const double b = B[(l >> 4) * 16 + (l & 15)];  // B[k l>>4][col l&15]
    v4d acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];   // row (l>>4)+4r, col l&15
}
int main() {
    double hA[64], hB[64], hC[256], ref[256];
    for (int i = 0; i < 64; ++i) { hA[i] = (i * 7) % 13 - 6; hB[i] = (i * 5) % 11 - 5; }
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            double s = 0;
            for (int q = 0; q < 4; ++q) s += hA[i * 4 + q] * hB[q * 16 + j];
            ref[i * 16 + j] = s;
        }
    double *dA, *dB, *dC;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 2048);
    hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 2048, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
    printf("mfma_f64_16x16x4 layout: %d / 256 mismatches\n", bad);
    return bad != 0;
}
