// msckf_kalman.hip -- Cholesky-form EKF update (msckf.py:559-604) on the
// information A = H^T H, b = H^T r assembled by k_info.
//
// With P_cc = Lc Lc^T (cam block of P, PD), Vc = P[:, cams] Lc^-T and
// T = s2 I + Lc^T A Lc (PD for every PSD A -- no rank decisions), the
// reference's update (K = P H^T S^-1, dx = K r, P <- (I - K H) P) is
//     dx = Vc T^-1 Lc^T b
//     P+ = blockdiag(P_ii - Vc_i Vc_i^T, 0) + s2 W W^T,     W = Vc L_T^-T
// (P - Vc Vc^T vanishes outside the 21 x 21 IMU block.)  Stages, all fp64 and
// batched over filters:
//   A  k_kal_a   partial Cholesky of [P_cc P_ci; P_ic P_ii] over the cam
//                pivots: Lc, Vc_i = P_ic Lc^-T, S_ii = P_ii - Vc_i Vc_i^T
//   B  k_kal_b1  G = A Lc;   k_kal_b2  [T | c] = s2 I + Lc^T [G | b]
//   C  k_kal_c   Cholesky of T with the extra rows [Vc_i ; Lc ; c^T]
//                appended: their panel rows are W = [Vc_i ; Lc] L_T^-T and
//                y = L_T^-1 c (rows split over several workgroups per
//                filter, each refactoring T)
//   E  k_kal_e   P+ = blockdiag(S_ii, 0) + s2 W W^T and dx = W y
// A and C keep the matrix in registers as 4x4 tiles (one workgroup per
// filter); B and E are 64 x 64-tiled LDS GEMMs.
#include "msckf_common.h"
#include "msckf_launch.h"

namespace msckf {

constexpr int KW = 24;   // IMU block padded to a multiple of 4

__device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }

// ===========================================================================
// Register-tile partial Cholesky.  The lower tiles (ti, tl), tl < ncol,
// tl <= ti < nrow, enumerated column-major; tile t lives in thread t % NT,
// slot t / NT.  Eliminates tile columns 0..nelim-1 (4 pivots per step):
//   1. owners of the step's tile column dump it to LDS (double-buffered)
//   2. every thread factors the 4x4 diagonal tile (uniform) and transforms
//      panel rows (one row per thread): W = A_panel L_d^-T -> LDS + panel()
//   3. every tile right of the panel takes A -= W_i W_l^T from registers
// Two barriers per step.  Tiles in columns >= nelim end as the Schur
// complement and are handed to trail().  In the LDS column buffer each 4-row
// block takes RB = 18 doubles (144 B): consecutive lanes read consecutive
// blocks with ds_read_b128, and a 144-B stride spreads a 16-lane group over
// all 64 banks (a 128-B stride would put it on two).
// load(i, j) must be symmetric on the square part (diagonal tiles read both
// triangles).
// ===========================================================================
constexpr int RB = 18;   // doubles per 4-row block of the LDS column buffer

template <int NT, int TPL, class Load, class Panel, class Trail>
__device__ __forceinline__ bool rchol_core(int nrow, int ncol, int nelim, double* lds, Load load, Panel panel,
                                           Trail trail) {
    const int tid = threadIdx.x;
    const int ntiles = ncol * nrow - ncol * (ncol - 1) / 2;
    int crd[TPL], tlmax[TPL];
#pragma unroll
    for (int s = 0; s < TPL; ++s) {
        const int t = NT * s + tid;
        const int c = colmajor_col(t < ntiles ? t : 0, nrow);
        const int rem = (t < ntiles ? t : 0) - (c * nrow - c * (c - 1) / 2);
        crd[s] = t < ntiles ? ((c + rem) | (c << 16)) : -1;
        const int tm = NT * s + NT - 1 < ntiles - 1 ? NT * s + NT - 1 : ntiles - 1;
        tlmax[s] = NT * s < ntiles ? colmajor_col(tm, nrow) : -1;
    }
#define RTI(s) (crd[s] & 0xffff)
#define RTL(s) (crd[s] >> 16)
#define ROK(s) (crd[s] >= 0)
    double a[TPL][4][4];
#pragma unroll
    for (int s = 0; s < TPL; ++s) {
        const int i0 = 4 * RTI(s), j0 = 4 * RTL(s);
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) a[s][x][y] = ROK(s) ? load(i0 + x, j0 + y) : 0.0;
    }
    bool fail = false;
    for (int tj = 0; tj < nelim; ++tj) {
        double* buf = lds + (tj & 1) * RB * nrow;   // [nrow][RB]: rows 4 t + x at RB t + 4 x
#pragma unroll
        for (int s = 0; s < TPL; ++s) {
            if (!ROK(s) || RTL(s) != tj) continue;
            double* dst = buf + RB * RTI(s);
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) dst[4 * x + y] = a[s][x][y];
        }
        LDS_BARRIER();
        const double* dt = buf + RB * tj;
        const double l00 = sqrt(dt[0]);
        const double i00 = 1.0 / l00;
        const double l10 = dt[4] * i00, l20 = dt[8] * i00, l30 = dt[12] * i00;
        const double l11 = sqrt(dt[5] - l10 * l10);
        const double i11 = 1.0 / l11;
        const double l21 = (dt[9] - l20 * l10) * i11, l31 = (dt[13] - l30 * l10) * i11;
        const double l22 = sqrt(dt[10] - l20 * l20 - l21 * l21);
        const double i22 = 1.0 / l22;
        const double l32 = (dt[14] - l30 * l20 - l31 * l21) * i22;
        const double l33 = sqrt(dt[15] - l30 * l30 - l31 * l31 - l32 * l32);
        const double i33 = 1.0 / l33;
        if (!(l00 > 0.0) || !(l11 > 0.0) || !(l22 > 0.0) || !(l33 > 0.0)) { fail = true; break; }
        for (int r = 4 * tj + 4 + tid; r < 4 * nrow; r += NT) {
            double* row = buf + RB * (r >> 2) + 4 * (r & 3);
            const double w0 = row[0] * i00;
            const double w1 = (row[1] - w0 * l10) * i11;
            const double w2 = (row[2] - w0 * l20 - w1 * l21) * i22;
            const double w3 = (row[3] - w0 * l30 - w1 * l31 - w2 * l32) * i33;
            row[0] = w0; row[1] = w1; row[2] = w2; row[3] = w3;
            panel(r, 4 * tj, w0, w1, w2, w3);
        }
        if (tid < 4) {
            const int r = 4 * tj + tid;
            if (tid == 0) panel(r, 4 * tj, l00, 0.0, 0.0, 0.0);
            if (tid == 1) panel(r, 4 * tj, l10, l11, 0.0, 0.0);
            if (tid == 2) panel(r, 4 * tj, l20, l21, l22, 0.0);
            if (tid == 3) panel(r, 4 * tj, l30, l31, l32, l33);
        }
        LDS_BARRIER();
#pragma unroll
        for (int s = 0; s < TPL; ++s) {
            if (tlmax[s] <= tj) continue;   // slot entirely in finished columns
            if (!ROK(s) || RTL(s) <= tj) continue;
            const double* ri = buf + RB * RTI(s);
            const double* rl = buf + RB * RTL(s);
            double u[4][4], w[4][4];
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int c = 0; c < 4; ++c) { u[x][c] = ri[4 * x + c]; w[x][c] = rl[4 * x + c]; }
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y)
                    a[s][x][y] -= u[x][0] * w[y][0] + u[x][1] * w[y][1] + u[x][2] * w[y][2] + u[x][3] * w[y][3];
            asm volatile("" ::: "memory");
        }
    }
    if (!fail) {
#pragma unroll
        for (int s = 0; s < TPL; ++s) {
            if (!ROK(s) || RTL(s) < nelim) continue;
            const int i0 = 4 * RTI(s), j0 = 4 * RTL(s);
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) trail(i0 + x, j0 + y, a[s][x][y]);
        }
    }
#undef RTI
#undef RTL
#undef ROK
    return !fail;
}

__host__ __device__ constexpr int rchol_lds_doubles(int nrow) { return 2 * RB * nrow; }

// ---- stage A: [P_cc P_ci; P_ic P_ii] in index space [cams (Cp) | IMU (24)] ----
template <typename T, int NT, int TPL>
__global__ void __launch_bounds__(NT) k_kal_a(DevState<T> st, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    const int* info = ws.info + 4 * b;
    if (info[0] == 0) return;
    const int C = 6 * st.ncams[b], Cp = round4(C);
    const int nrow = (Cp + KW) / 4;
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax, Cpw = ws.Cp;
    KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* Vi = ws.Vi + (size_t)b * KW * Cpw;
    KT* Sii = ws.Sii + (size_t)b * KW * KW;
    auto map = [&](int i) { return i < C ? 21 + i : (i < Cp ? -1 : (i < Cp + 21 ? i - Cp : -1)); };
    auto load = [&](int i, int j) -> double {
        const int mi = map(i), mj = map(j);
        if (mi < 0 || mj < 0) return i == j ? 1.0 : 0.0;
        return (double)P[(size_t)mi * ld + mj];
    };
    auto panel = [&](int r, int c0, double w0, double w1, double w2, double w3) {
        KT* dst = r < Cp ? Lc + (size_t)r * Cpw + c0 : Vi + (size_t)(r - Cp) * Cpw + c0;
        dst[0] = w0; dst[1] = w1; dst[2] = w2; dst[3] = w3;
    };
    auto trail = [&](int i, int j, double v) { Sii[(i - Cp) * KW + (j - Cp)] = v; };
    const bool ok = rchol_core<NT, TPL>(nrow, nrow, Cp / 4, reinterpret_cast<double*>(smem_raw), load, panel, trail);
    if (!ok && threadIdx.x == 0) ws.info[4 * b + 3] = -1;
}

// ---- stage C: Cholesky of T (Cp) with extra rows [Vc_i (21); Lc (C); c^T] ----
// blockIdx.x = group g of extra-row tiles handled by this workgroup
template <typename T, int NT, int TPL>
__global__ void __launch_bounds__(NT) k_kal_c(DevState<T> st, UpdWs<T> ws, int ner) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.y, g = blockIdx.x;
    const int* info = ws.info + 4 * b;
    if (info[0] == 0) return;
    const int C = 6 * st.ncams[b], Cp = round4(C), nTc = Cp / 4;
    const int E = 21 + C + 1, ER = (E + 3) / 4;   // extra rows / extra tile rows
    const int e0 = g * ner;                       // first extra tile row of this group
    if (e0 >= ER) return;
    const int nr = ER - e0 < ner ? ER - e0 : ner;
    const int Cpw = ws.Cp, ldt = ws.Cmax + 1;
    const KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ldt;
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    const KT* Vi = ws.Vi + (size_t)b * KW * Cpw;
    KT* W = ws.W + (size_t)b * (st.Dmax + 1) * Cpw;
    auto load = [&](int i, int j) -> double {
        if (i < Cp) {   // T (lower stored), identity padding
            if (i >= C || j >= C) return i == j ? 1.0 : 0.0;
            return i >= j ? Tm[(size_t)i * ldt + j] : Tm[(size_t)j * ldt + i];
        }
        const int e = i - Cp + 4 * e0;
        if (j >= C) return 0.0;
        if (e < 21) return Vi[(size_t)e * Cpw + j];
        if (e < 21 + C) return j <= e - 21 ? Lc[(size_t)(e - 21) * Cpw + j] : 0.0;
        if (e == 21 + C) return Tm[(size_t)j * ldt + C];
        return 0.0;
    };
    auto panel = [&](int r, int c0, double w0, double w1, double w2, double w3) {
        if (r < Cp) return;
        const int e = r - Cp + 4 * e0;
        if (e >= E) return;
        KT* dst = W + (size_t)e * Cpw + c0;
        dst[0] = w0; dst[1] = w1; dst[2] = w2; dst[3] = w3;
    };
    auto trail = [](int, int, double) {};
    const bool ok = rchol_core<NT, TPL>(nTc + nr, nTc, nTc, reinterpret_cast<double*>(smem_raw), load, panel, trail);
    if (!ok && threadIdx.x == 0) ws.info[4 * b + 3] = -1;
}

// ===========================================================================
// 64 x 64 output tile, 256 threads (4 x 4 each), K in steps of 16 through LDS.
// A(i, k) and B(k, j) are accessors; *_KFAST says whether consecutive k are
// contiguous in memory for that operand (selects the coalesced load mapping).
// ===========================================================================
constexpr int GT = 64, GK = 16;

template <bool A_KFAST, bool B_KFAST, class FA, class FB>
__device__ __forceinline__ void gemm64(int m, int n, int kb, int ke, int i0, int j0, FA A, FB B, double acc[4][4]) {
    __shared__ __attribute__((aligned(16))) double sa[GK][GT + 4], sb[GK][GT + 4];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = 0;
    for (int k0 = kb; k0 < ke; k0 += GK) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q;
            int ii, kk, jj, k2;
            if (A_KFAST) { ii = e >> 4; kk = e & 15; } else { ii = e & 63; kk = e >> 6; }
            const int gi = i0 + ii, gk = k0 + kk;
            sa[kk][ii] = (gi < m && gk < ke) ? A(gi, gk) : 0.0;
            if (B_KFAST) { jj = e >> 4; k2 = e & 15; } else { jj = e & 63; k2 = e >> 6; }
            const int gj = j0 + jj, gk2 = k0 + k2;
            sb[k2][jj] = (gj < n && gk2 < ke) ? B(gk2, gj) : 0.0;
        }
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < GK; ++kk) {
            double av[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { av[u] = sa[kk][4 * ty + u]; bv[u] = sb[kk][4 * tx + u]; }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] += av[u] * bv[v];
        }
        __syncthreads();
    }
}

// ---- stage B1: G = A Lc (C x C) ----
template <typename T>
__global__ void __launch_bounds__(256) k_kal_b1(DevState<T> st, UpdWs<T> ws) {
    const int b = blockIdx.z;
    if (ws.info[4 * b] == 0) return;
    const int C = 6 * st.ncams[b];
    const int i0 = blockIdx.y * GT, j0 = blockIdx.x * GT;
    if (i0 >= C || j0 >= C) return;
    const int lda = ws.Cmax + 1, Cpw = ws.Cp;
    const KT* Am = ws.Hthin + (size_t)b * ws.Cmax * lda;
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* G = ws.G + (size_t)b * ws.Cmax * lda;
    double acc[4][4];
    gemm64<true, false>(C, C, j0 & ~(GK - 1), C, i0, j0,
                        [&](int i, int k) { return Am[(size_t)i * lda + k]; },
                        [&](int k, int j) { return k >= j ? Lc[(size_t)k * Cpw + j] : 0.0; }, acc);
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int i = i0 + 4 * ty + u, j = j0 + 4 * tx + v;
            if (i < C && j < C) G[(size_t)i * lda + j] = acc[u][v];
        }
}

// ---- stage B2: [T | c] = s2 I + Lc^T [G | b] (lower triangle of T, and c) ----
template <typename T>
__global__ void __launch_bounds__(256) k_kal_b2(DevState<T> st, Params<T> prm, UpdWs<T> ws) {
    const int b = blockIdx.z;
    if (ws.info[4 * b] == 0) return;
    const int C = 6 * st.ncams[b];
    const int i0 = blockIdx.y * GT, j0 = blockIdx.x * GT;
    if (i0 >= C || j0 > C) return;
    if (j0 > i0 + GT - 1 && !(C >= j0 && C < j0 + GT)) return;   // strictly upper and no c column
    const int ld = ws.Cmax + 1, Cpw = ws.Cp;
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    const KT* G = ws.G + (size_t)b * ws.Cmax * ld;
    const KT* Hb = ws.Hthin + (size_t)b * ws.Cmax * ld;   // b in column Cmax
    KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ld;
    double acc[4][4];
    gemm64<false, false>(C, C + 1, i0 & ~(GK - 1), C, i0, j0,
                         [&](int i, int k) { return k >= i ? Lc[(size_t)k * Cpw + i] : 0.0; },
                         [&](int k, int j) { return j < C ? G[(size_t)k * ld + j] : Hb[(size_t)k * ld + ws.Cmax]; },
                         acc);
    const double s2 = (double)prm.sigma2;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int i = i0 + 4 * ty + u, j = j0 + 4 * tx + v;
            if (i >= C) continue;
            if (j < C && j <= i) Tm[(size_t)i * ld + j] = acc[u][v] + (i == j ? s2 : 0.0);
            if (j == C) Tm[(size_t)i * ld + C] = acc[u][v];
        }
}

// ---- stage E: P+ = blockdiag(S_ii, 0) + s2 W W^T (lower tiles, mirrored), dx = W y ----
template <typename T>
__global__ void __launch_bounds__(256) k_kal_e(DevState<T> st, Params<T> prm, UpdWs<T> ws) {
    const int b = blockIdx.z;
    if (ws.info[4 * b] == 0 || ws.info[4 * b + 3] < 0) return;
    const int C = 6 * st.ncams[b], D = 21 + C;
    const int i0 = blockIdx.y * GT, j0 = blockIdx.x * GT;
    if (i0 >= D || j0 > D) return;
    if (j0 > i0 + GT - 1 && !(D >= j0 && D < j0 + GT)) return;
    const int Cpw = ws.Cp, ld = st.Dmax;
    const KT* W = ws.W + (size_t)b * (st.Dmax + 1) * Cpw;
    const KT* Sii = ws.Sii + (size_t)b * KW * KW;
    T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    KT* dx = ws.dx + (size_t)b * (st.Dmax + ws.Cmax);
    double acc[4][4];
    gemm64<true, true>(D, D + 1, 0, C, i0, j0, [&](int i, int k) { return W[(size_t)i * Cpw + k]; },
                       [&](int k, int j) { return W[(size_t)(j < D ? j : D) * Cpw + k]; }, acc);
    const double s2 = (double)prm.sigma2;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int i = i0 + 4 * ty + u, j = j0 + 4 * tx + v;
            if (i >= D) continue;
            if (j < D && j <= i) {
                double p = s2 * acc[u][v];
                if (i < 21 && j < 21) p += Sii[i * KW + j];
                P[(size_t)i * ld + j] = (T)p;
                P[(size_t)j * ld + i] = (T)p;
            }
            if (j == D) dx[i] = acc[u][v];
        }
}

// ===========================================================================
// Host side
// ===========================================================================
struct RcholCfg { int nt, tpl; };

static bool pick_rchol(int tiles, RcholCfg& c) {
    if (tiles <= 256 * 4) { c = {256, 4}; return true; }
    if (tiles <= 512 * 4) { c = {512, 4}; return true; }
    return false;
}

template <typename T, int NT, int TPL>
static void launch_a_cfg(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws, size_t lds) {
    hipLaunchKernelGGL((k_kal_a<T, NT, TPL>), dim3(st.B), dim3(NT), lds, s, st, ws);
}
template <typename T, int NT, int TPL>
static void launch_c_cfg(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws, int groups, int ner, size_t lds) {
    hipLaunchKernelGGL((k_kal_c<T, NT, TPL>), dim3(groups, st.B), dim3(NT), lds, s, st, ws, ner);
}

bool kalman_chol_supported(int Cmax) {
    const int Cp = (Cmax + 3) & ~3;
    const int nrowA = (Cp + KW) / 4;
    RcholCfg c;
    if (!pick_rchol(nrowA * (nrowA + 1) / 2, c)) return false;
    const int nTc = Cp / 4;
    return pick_rchol(nTc * (nTc + 1) / 2 + nTc, c);
}

template <typename T>
void launch_kalman_chol(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const UpdWs<T>& ws,
                        KernelTimer* kt) {
    const int Cp = ws.Cp, Cmax = ws.Cmax;
    // stage A
    {
        const int nrow = (Cp + KW) / 4;
        RcholCfg c;
        pick_rchol(nrow * (nrow + 1) / 2, c);
        const size_t lds = rchol_lds_doubles(nrow) * sizeof(double);
        kt->begin(s, "kalman_a");
        if (c.nt == 256) launch_a_cfg<T, 256, 4>(s, st, ws, lds);
        else launch_a_cfg<T, 512, 4>(s, st, ws, lds);
        kt->end(s);
    }
    const int tiles = (Cmax + GT - 1) / GT;
    kt->begin(s, "kalman_b");
    hipLaunchKernelGGL(k_kal_b1<T>, dim3(tiles, tiles, st.B), dim3(256), 0, s, st, ws);
    hipLaunchKernelGGL(k_kal_b2<T>, dim3((Cmax + 1 + GT - 1) / GT, tiles, st.B), dim3(256), 0, s, st, prm, ws);
    kt->end(s);
    // stage C: T tiles + as many extra-row tiles as fit, the rest in more groups
    {
        const int nTc = Cp / 4, Tt = nTc * (nTc + 1) / 2;
        const int ER = (21 + Cmax + 1 + 3) / 4;
        RcholCfg c{512, 4};
        if (Tt + ER * nTc <= 256 * 4) c = {256, 4};
        const int ner_max = (c.nt * c.tpl - Tt) / nTc;
        const int groups = (ER + ner_max - 1) / ner_max;
        const int ner = (ER + groups - 1) / groups;
        const size_t lds = rchol_lds_doubles(nTc + ner) * sizeof(double);
        kt->begin(s, "kalman_c");
        if (c.nt == 256) launch_c_cfg<T, 256, 4>(s, st, ws, groups, ner, lds);
        else launch_c_cfg<T, 512, 4>(s, st, ws, groups, ner, lds);
        kt->end(s);
    }
    const int dt = (st.Dmax + GT - 1) / GT, dt1 = (st.Dmax + 1 + GT - 1) / GT;
    kt->begin(s, "kalman_e");
    hipLaunchKernelGGL(k_kal_e<T>, dim3(dt1, dt, st.B), dim3(256), 0, s, st, prm, ws);
    kt->end(s);
}

template void launch_kalman_chol<float>(hipStream_t, const DevState<float>&, const Params<float>&,
                                        const UpdWs<float>&, KernelTimer*);
template void launch_kalman_chol<double>(hipStream_t, const DevState<double>&, const Params<double>&,
                                         const UpdWs<double>&, KernelTimer*);

}  // namespace msckf
