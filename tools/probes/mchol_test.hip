// Probe: msckf_mchol.h's MFMA partial Cholesky on random SPD matrices, one
// workgroup, against a host Cholesky.  Prints the max error of L, of the
// panel rows below the eliminated block and of the Schur complement.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "msckf_mchol.h"
using namespace msckf;

template <int NW, int TPW>
__global__ void __launch_bounds__(64 * NW) k_test(const double* A, int n, int nrow, int nelim, double* L, double* S) {
    extern __shared__ double lds[];
    auto load = [&](int i, int j) -> double { return (i < n && j < n) ? A[i * n + j] : (i == j ? 1.0 : 0.0); };
    auto out = [&](int i, int j, double v) { if (i < n && j < n) L[i * n + j] = v; };
    auto trail = [&](int i, int j, double v) { if (i < n && j < n) S[i * n + j] = v; };
    mchol_core<NW, TPW>(nrow, nrow, nelim, lds, load, out, trail, 0.0);
}

template <int NW, int TPW>
static int run(int nrow, int nelim) {
    const int n = 16 * nrow, m = 16 * nelim;
    std::vector<double> A(n * n), X(n * n);
    unsigned s = 12345;
    for (auto& x : X) { s = s * 1664525u + 1013904223u; x = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = i == j ? n : 0.0;
            for (int k = 0; k < n; ++k) v += X[i * n + k] * X[j * n + k];
            A[i * n + j] = v;
        }
    // host: Cholesky of the leading m x m, panel rows, Schur complement
    std::vector<double> H = A;
    for (int j = 0; j < m; ++j) {
        const double d = std::sqrt(H[j * n + j]);
        for (int i = j; i < n; ++i) H[i * n + j] /= (i == j ? 1.0 : d);
        H[j * n + j] = d;
        for (int i = j + 1; i < n; ++i)
            for (int k = j + 1; k <= i; ++k) H[i * n + k] -= H[i * n + j] * H[k * n + j];
    }
    double *dA, *dL, *dS;
    hipMalloc(&dA, n * n * 8); hipMalloc(&dL, n * n * 8); hipMalloc(&dS, n * n * 8);
    hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice);
    hipMemset(dL, 0, n * n * 8); hipMemset(dS, 0, n * n * 8);
    const size_t lds = mchol_lds_doubles(nrow) * 8;
    (void)hipFuncSetAttribute((const void*)k_test<NW, TPW>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL((k_test<NW, TPW>), dim3(1), dim3(64 * NW), lds, 0, dA, n, nrow, nelim, dL, dS);
    hipError_t e = hipDeviceSynchronize();
    std::vector<double> L(n * n), S(n * n);
    hipMemcpy(L.data(), dL, n * n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(S.data(), dS, n * n * 8, hipMemcpyDeviceToHost);
    double eL = 0, eP = 0, eS = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            if (j < m && i < m) eL = std::fmax(eL, std::fabs(L[i * n + j] - H[i * n + j]));
            else if (j < m) eP = std::fmax(eP, std::fabs(L[i * n + j] - H[i * n + j]));
            else eS = std::fmax(eS, std::fabs(S[i * n + j] - H[i * n + j]));
        }
    printf("mchol probe NW %d nrow %d nelim %d TPW %d (%s): max |dL| %.3e  panel %.3e  schur %.3e\n", NW, nrow, nelim, TPW,
           hipGetErrorString(e), eL, eP, eS);
    // first bad entries
    int shown = 0;
    for (int i = 0; i < n && shown < 8; ++i)
        for (int j = 0; j <= i && shown < 8; ++j) {
            const double ref = H[i * n + j], got = j < m ? L[i * n + j] : S[i * n + j];
            if (std::fabs(got - ref) > 1e-9 * (1 + std::fabs(ref))) { printf("  (%d,%d) got %.6g ref %.6g\n", i, j, got, ref); ++shown; }
        }
    // throughput: 2048 workgroups on the same matrix (identical writes)
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL((k_test<NW, TPW>), dim3(2048), dim3(64 * NW), lds, 0, dA, n, nrow, nelim, dL, dS);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("   2048 workgroups: %.3f ms (lds %zu B)\n", ms, lds);
    hipFree(dA); hipFree(dL); hipFree(dS);
    return 0;
}

int main() {
    run<16, 4>(6, 4);
    run<16, 7>(14, 12);
    run<16, 5>(12, 12);
    run<8, 3>(6, 4);
    run<8, 14>(14, 12);
    run<8, 10>(12, 12);
    run<4, 27>(14, 12);
    run<4, 20>(12, 12);
    return 0;
}
