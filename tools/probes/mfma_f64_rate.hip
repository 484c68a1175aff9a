// Issue rate of v_mfma_f64_16x16x4f64 on one SIMD: one wave, N independent
// accumulators, K rounds, s_memtime around the loop.  Also the dependent
// (single accumulator) chain.  Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mr mfma_f64_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ void k(double* out, unsigned long long* cyc, int rounds) {
    v4d acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = v4d{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    __syncthreads();
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < NACC; ++i) asm volatile("" : "+v"(acc[i]));
    unsigned long long t1 = __builtin_readcyclecounter();
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int NACC>
void run(int waves_per_cu) {
    double* o; unsigned long long* c;
    const int blocks = 256 * waves_per_cu, rounds = 200;
    hipMalloc(&o, blocks * 64 * 8); hipMalloc(&c, blocks * 8);
    hipLaunchKernelGGL(k<NACC>, dim3(blocks), dim3(64), 0, 0, o, c, rounds);
    hipDeviceSynchronize();
    unsigned long long* h = new unsigned long long[blocks];
    hipMemcpy(h, c, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < blocks; ++i) avg += h[i]; avg /= blocks;
    printf("NACC=%2d waves/CU=%d: %.1f cycles per MFMA per wave\n", NACC, waves_per_cu, avg / (rounds * NACC));
    hipFree(o); hipFree(c); delete[] h;
}
int main() {
    run<1>(1); run<4>(1); run<8>(1); run<16>(1); run<8>(4); run<8>(8);
    return 0;
}
