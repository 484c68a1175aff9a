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
//   B  k_kal_b   [T | c] = s2 I + Lc^T [A Lc | b] (fp64 MFMA accumulators)
//   C  k_kal_c1  Cholesky of T; k_kal_c2: W^T = L_T^-1 [Vc_i ; Lc]^T and
//                y = L_T^-1 c (MFMA blocked forward substitution)
//   E  k_kal_e1  P+ = blockdiag(S_ii, 0) + s2 W W^T and dx = W y
// Up to 32 cams A and C1 keep the matrix in registers as 4x4 tiles (one
// workgroup per filter); larger windows run A and C as blocked global-memory
// Choleskys (k_gchol_*) and B / E as 64 x 64-tiled GEMMs (k_kal_b1/b2, k_kal_e).
#include "msckf_common.h"
#include "msckf_launch.h"
#include "msckf_rchol.h"

#include <stdlib.h>

namespace msckf {

constexpr int KW = 24;   // IMU block padded to a multiple of 4

__device__ __forceinline__ int round4(int x) { return (x + 3) & ~3; }


typedef double v4d __attribute__((ext_vector_type(4)));

// Pivot floor of the P_cc factorisations (stage A): KALMAN_PIVOT_FLOOR x the
// largest cam-block variance.  The reference's (I - KH)P update (msckf.py:598-604,
// not Joseph form) leaves P_cc indefinite at rounding level after a few frames
// (smallest eigenvalue ~ -3e-10 x max diag on synthetic EuRoC-shaped streams);
// the reference never factors P, so a pivot at or below zero must not abort the
// update here.  Flooring it factors P_cc + E, E diagonal and ~1e-10 relative:
// the update moves by that much, far inside the 1e-6 parity tolerance.  Only
// pivots down to -PIVOT_FLOOR_NEG x the floor (-1e-6 x max diag) are floored
// (msckf_rchol.h): a NaN or a deeper negative pivot still fails with -3.
constexpr double KALMAN_PIVOT_FLOOR = 1e-10;

// largest of n diagonal entries M[(o + i)(ld + 1)]: workgroup reduction (all
// threads call; lds: >= 16 doubles of scratch, reused after)
template <typename T>
__device__ double diag_max(const T* M, int ld, int o, int n, double* lds) {
    double m = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmax(m, (double)M[(size_t)(o + i) * (ld + 1)]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = m;
    __syncthreads();
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = fmax(m, lds[w]);
    __syncthreads();
    return m;
}
template <typename T>
__device__ double pcc_pivot_floor(const T* P, int ld, int C, double* lds) {
    return diag_max(P, ld, 21, C, lds) * KALMAN_PIVOT_FLOOR;
}
// Stage C's pivots are floored at s2 (T = s2 I + Lc^T A Lc >= s2 I in exact
// arithmetic; a numerically degenerate A's rounding can push a computed pivot
// below it) down to -T_FLOOR_NEG x the largest diagonal entry of T: that covers
// rounding at any conditioning (golden stream s4: pivots of order -eps |T|), a
// pivot further below zero means a corrupted T and fails the update.
constexpr double T_FLOOR_NEG = 1e-9;

// ---- stage A: [P_cc P_ci; P_ic P_ii] in index space [cams (Cp) | IMU (24)] ----
template <typename T, int NT, int TPL, bool RETRY = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 ? 2 : 1))) k_kal_a(DevState<T> st, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    // launched before k_select (side stream): every filter is factored, the
    // status goes to afail only, and k_kal_c1 turns it into info[3] for the
    // filters that do update
    const int b = blockIdx.x;
    if (RETRY && ws.afail[b] == 0) return;   // factored on the first attempt
    const int C = 6 * st.ncams[b], Cp = round4(C);
    const int nrow = (Cp + KW) / 4;
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax, Cpw = ws.Cp;
    KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* Vi = ws.Vi + (size_t)b * KW * Cpw;
    KT* Sii = ws.Sii + (size_t)b * KW * KW;
    auto map = [&](int i) { return i < C ? 21 + i : (i < Cp ? -1 : (i < Cp + 21 ? i - Cp : -1)); };
    double shift = 0.0;   // retries: P_cc + shift I (see below)
    auto load = [&](int i, int j) -> double {
        const int mi = map(i), mj = map(j);
        if (mi < 0 || mj < 0) return i == j ? 1.0 : 0.0;
        return (double)P[(size_t)mi * ld + mj] + (i == j && i < C ? shift : 0.0);
    };
    auto panel = [&](int r, int c0, double w0, double w1, double w2, double w3) {
        KT* dst = r < Cp ? Lc + (size_t)r * Cpw + c0 : Vi + (size_t)(r - Cp) * Cpw + c0;
        dst[0] = w0; dst[1] = w1; dst[2] = w2; dst[3] = w3;
    };
    auto trail = [&](int i, int j, double v) { Sii[(i - Cp) * KW + (j - Cp)] = v; };
    const double floor = pcc_pivot_floor(P, ld, C, reinterpret_cast<double*>(smem_raw));
    // A P_cc that the reference's update (msckf.py:598-604) left indefinite at
    // rounding level can still defeat the pivot floor: a floored pivot whose
    // column is not small makes the following pivots large and negative (golden
    // stream s4 after its degenerate frame-3 update: smallest eigenvalue
    // -4e-9 x the largest variance, pivots -> -inf).  Such a filter is factored
    // again as P_cc + shift I, shift = 1e-8 then 1e-6 x the largest cam variance
    // (the update moves by about that much; a PD P_cc never gets here); a P_cc
    // that fails even then (a clearly negative eigenvalue, NaN) fails with -3.
    // The retries run in a second launch (RETRY: only the filters whose first
    // attempt failed do any work), so the first attempt's register allocation is
    // the one-shot kernel's.
    bool ok = false;
    for (int att = RETRY ? 1 : 0; att < (RETRY ? 3 : 1) && !ok; ++att) {
        if (att > 0) {
            shift = (att == 1 ? 1e-8 : 1e-6) * (floor / KALMAN_PIVOT_FLOOR);
            __syncthreads();   // the previous attempt's LDS panel reads are done
        }
        ok = rchol_core<NT, TPL>(nrow, nrow, Cp / 4, reinterpret_cast<double*>(smem_raw), load, panel, trail, floor);
    }
    if (threadIdx.x == 0) ws.afail[b] = ok ? 0 : 1;   // read by k_kal_c1
}

// ---- stage C (register-tile windows, C <= 192) ----
// C1: Cholesky of T alone (4x4 register tiles, one workgroup per filter), L_T
//     written over the G workspace (free after stage B).
// C2: W^T = L_T^-1 X^T with X = [Vc_i ; Lc ; c^T] (E = 22 + C rows) as a
//     blocked forward substitution on MFMA: wave w owns the 16-row tiles
//     ct = w + NW t of X and keeps the solved blocks Y'[K] (16 x 16, K < nT) in
//     registers -- in the MFMA result layout (row = lane/16 + 4 r, col =
//     lane%16) a solved block's r-th value is exactly the B operand of
//     k-step r, so no block is re-read.  Step J:
//         Y'[J] = Linv_JJ (X^T[J] - sum_{K<J} L_T[J, K] Y'[K])
//     with -L_T[J, 0:16J] staged in LDS ([col][row], 17-double rows) and the
//     16 x 16 inverses of the diagonal blocks formed once up front.  W^T is
//     stored row-major over k (coalesced), the layout k_kal_e1 reads.
template <typename T, int NT, int TPL>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 ? 2 : 1))) k_kal_c1(DevState<T> st, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    if (ws.info[4 * b] == 0) return;
    if (ws.afail[b]) {   // stage A failed (P_cc not PD): no update for this filter
        if (threadIdx.x == 0) ws.info[4 * b + 3] = -2;
        return;
    }
    const int C = 6 * st.ncams[b], Cp = round4(C), nTc = Cp / 4;
    const int ldt = ws.Cmax + 1;
    const KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ldt;
    KT* L = ws.G + (size_t)b * ws.Cmax * ldt;
    auto load = [&](int i, int j) -> double {
        if (i >= C || j >= C) return i == j ? 1.0 : 0.0;
        return i >= j ? Tm[(size_t)i * ldt + j] : Tm[(size_t)j * ldt + i];
    };
    auto panel = [&](int r, int c0, double w0, double w1, double w2, double w3) {
        if (r >= C) return;
        KT* dst = L + (size_t)r * ldt;
        const double w[4] = {w0, w1, w2, w3};
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (c0 + q < C && c0 + q <= r) dst[c0 + q] = w[q];
    };
    auto trail = [](int, int, double) {};
    // T = s2 I + Lc^T A Lc >= s2 I, so every exact pivot is >= s2; rounding in a
    // numerically degenerate A (a landmark millimetres from the camera: entries
    // ~1e9, cond(T) beyond 1/eps) can still push computed pivots below it.  They
    // are floored at s2 instead of failing the filter -- the reference's LU solve
    // (msckf.py:560-563) returns its own rounding noise there, without an error --
    // down to -T_FLOOR_NEG x max diag(T); a NaN or deeper pivot still fails.
    const double tmax = diag_max(Tm, ldt, 0, C, reinterpret_cast<double*>(smem_raw));
    const bool ok = rchol_core<NT, TPL>(nTc, nTc, nTc, reinterpret_cast<double*>(smem_raw), load, panel, trail, ws.s2,
                                        -T_FLOOR_NEG * tmax);
    if (!ok && threadIdx.x == 0) ws.info[4 * b + 3] = -1;
}

constexpr int C2S = 17;   // LDS row stride (doubles) of the staged L_T block row

template <typename T, int NW, int CT, int NTM>
__global__ void __launch_bounds__(64 * NW) k_kal_c2(DevState<T> st, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    constexpr int NT = 64 * NW;
    const int b = blockIdx.x;
    if (ws.info[4 * b] == 0 || ws.info[4 * b + 3] < 0) return;
    const int C = 6 * st.ncams[b], nT = (C + 15) / 16, E = 22 + C, nE = (E + 15) / 16;
    const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ldt = ws.Cmax + 1, Cpw = ws.Cp, ldw = st.Dmax + 1;
    const KT* L = ws.G + (size_t)b * ws.Cmax * ldt;
    const KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ldt;
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    const KT* Vi = ws.Vi + (size_t)b * KW * Cpw;
    KT* Wt = ws.W + (size_t)b * (st.Dmax + 1) * Cpw;
    double* LI = reinterpret_cast<double*>(smem_raw);   // [NTM][k][i] = Linv_JJ[i][k]
    double* img = LI + NTM * 256;                        // [col][C2S]: -L_T[16J + i][col]
    auto Lv = [&](int r, int k) -> double {   // L_T with identity padding beyond C
        if (r >= C || k >= C) return r == k ? 1.0 : 0.0;
        return k <= r ? L[(size_t)r * ldt + k] : 0.0;
    };
    // diagonal block inverses: the block and its reciprocal diagonal go to a
    // per-wave LDS scratch (img is free until the main loop), lane j < 16
    // solves column j by forward substitution in registers (the divisions off
    // the dependent chain), then stores it to LI
    for (int J = wv; J < nT; J += NW) {
        double* blk = img + wv * 272;   // 16 x 16 block + reciprocal diagonal
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = lane + 64 * q, i = e >> 4, k = e & 15;
            blk[e] = Lv(16 * J + i, 16 * J + k);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (lane < 16) blk[256 + lane] = 1.0 / blk[17 * lane];   // reciprocal diagonal, in parallel
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (lane < 16) {   // column lane of the inverse, kept in registers
            double x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                double sv = i == lane ? 1.0 : 0.0;
#pragma unroll
                for (int k = 0; k < i; ++k) sv -= k >= lane ? blk[16 * i + k] * x[k] : 0.0;
                x[i] = i < lane ? 0.0 : sv * blk[256 + i];
            }
            double* xj = LI + J * 256 + 16 * lane;   // Linv[i][lane] at xj[i]
#pragma unroll
            for (int i = 0; i < 16; ++i) xj[i] = x[i];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
    auto Xv = [&](int e, int j) -> double {   // X[e][j]
        if (j >= C) return 0.0;
        if (e < 21) return Vi[(size_t)e * Cpw + j];
        if (e < 21 + C) return j <= e - 21 ? Lc[(size_t)(e - 21) * Cpw + j] : 0.0;
        if (e == 21 + C) return Tm[(size_t)j * ldt + C];
        return 0.0;
    };
    v4d yk[CT][NTM];
    // -L_T[16J : 16J+16, 0 : 16J] is software-pipelined: block row J + 1 is
    // loaded into registers while step J runs its MFMAs, and stored to LDS
    // after step J's closing barrier
    constexpr int PFN = (256 * (NTM - 1) + NT - 1) / NT;
    double pf[PFN];
    auto fetch = [&](int J) {
        const int w = 16 * J;
#pragma unroll
        for (int q = 0; q < PFN; ++q) {
            const int e = tid + NT * q, i = e / w, col = e - i * w;
            pf[q] = e < 16 * w ? -Lv(16 * J + i, col) : 0.0;
        }
    };
    // block row J is staged in buffer J & 1, so a step needs no closing
    // barrier: a later step's put never overwrites a buffer another wave may
    // still read (measured equal to two barriers per step; four accumulator
    // chains instead of two: 1.42 vs 1.19 ms, profiles/r04/ab_c2_*)
    constexpr int IMGB = 16 * NTM * C2S;
    auto imgJ = [&](int J) { return img + (J & 1) * IMGB; };
    auto put = [&](int J) {
        const int w = 16 * J;
        double* im = imgJ(J);
#pragma unroll
        for (int q = 0; q < PFN; ++q) {
            const int e = tid + NT * q, i = e / w, col = e - i * w;
            if (e < 16 * w) im[col * C2S + i] = pf[q];
        }
    };
    __syncthreads();   // the diagonal-block scratch in img is dead
    if (nT > 1) fetch(1);
    v4d xn[CT];   // this lane's X^T[J] elements of each tile
#pragma unroll
    for (int t = 0; t < CT; ++t) {
        const int ct = wv + NW * t;
#pragma unroll
        for (int q = 0; q < 4; ++q) xn[t][q] = ct < nE ? Xv(16 * ct + lc, lr + 4 * q) : 0.0;
    }
#pragma unroll
    for (int J = 0; J < NTM; ++J) {
        if (J >= nT) continue;   // uniform; continue (not break) keeps the loop unrollable
        if (J > 0) put(J);
        __syncthreads();
        if (J + 1 < nT) fetch(J + 1);
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            const int ct = wv + NW * t;
            if (ct >= nE) continue;
            v4d a0 = xn[t], a1 = v4d{0.0, 0.0, 0.0, 0.0};
            if (J + 1 < nT) {   // X^T[J + 1] for the next step, loaded under this one
#pragma unroll
                for (int q = 0; q < 4; ++q) xn[t][q] = Xv(16 * ct + lc, 16 * (J + 1) + lr + 4 * q);
            }
            const double* im = imgJ(J);
#pragma unroll
            for (int K = 0; K < J; ++K) {
#pragma unroll
                for (int kc = 0; kc < 4; ++kc) {
                    const double av = im[(16 * K + 4 * kc + lr) * C2S + lc];
                    if (K & 1) a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, yk[t][K][kc], a1, 0, 0, 0);
                    else a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, yk[t][K][kc], a0, 0, 0, 0);
                }
            }
            a0 += a1;
            v4d y = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kc = 0; kc < 4; ++kc)
                y = __builtin_amdgcn_mfma_f64_16x16x4f64(LI[J * 256 + (4 * kc + lr) * 16 + lc], a0[kc], y, 0, 0, 0);
            yk[t][J] = y;
        }
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) {
        const int ct = wv + NW * t, col = 16 * ct + lc;
        if (ct >= nE || col >= E) continue;
#pragma unroll
        for (int J = 0; J < NTM; ++J) {
            if (J >= nT) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = 16 * J + lr + 4 * q;
                if (k < C) Wt[(size_t)k * ldw + col] = yk[t][J][q];
            }
        }
    }
}

// ===========================================================================
// Stages A and C for windows whose tiles do not fit in one workgroup's
// registers (Nmax > 36): the same partial Cholesky, in place on a row-major
// global workspace (rows < ncol: the square lower part; rows >= ncol: extra
// rows with ncol columns), right-looking and blocked by GNB = 64 pivots.  Each
// panel step is three launches over all filters: factor the GNB x GNB diagonal
// block (one wave per filter), the panel rows below it (one row per thread,
// many workgroups per filter), and the trailing update A -= W W^T on the
// matrix cores (64 x 64 fp64 MFMA tiles, gemm64 below).  The trailing matrix
// makes one round trip per GNB = 64 pivots instead of one per pivot.
// ===========================================================================
constexpr int GNB = 64;   // pivots per panel (50x400 / 80x1000 updates/s: 16: 24.1k / 4.98k, 32: 26.3k / 5.27k, 48: 26.8k / 5.21k, 64: 27.5k / 5.20k)

// stage 0 = A: [P_cc P_ci; P_ic P_ii] (N = C + 21 square, C pivots), at the
// start of the filter's workspace;
// stage 1 = C: T (C square) with the extra rows [Vc_i (21); Lc (C); c^T], after
// it (gchol_c_off): stage A's store writes the Vc_i / Lc rows and stage B2 the
// T / c rows straight into it, and stage E reads the solved extra rows (W) from
// it -- no copies in or out (round 6: k_gchol_c_load / c_store, 1.8 ms per
// 50x400 step, removed)
__host__ __device__ constexpr size_t gchol_c_off(int Cmax) { return (size_t)(Cmax + 21) * (Cmax + 21); }
template <int STAGE, typename T>
__device__ __forceinline__ bool gdims(const DevState<T>& st, const UpdWs<T>& ws, int b, KT*& A, int& nrow,
                                      int& ncol, int& nelim) {
    if (ws.info[4 * b] == 0 || ws.info[4 * b + 3] < 0) return false;
    const int C = 6 * st.ncams[b];
    A = ws.Wk + (size_t)b * ws.wk_stride + (STAGE == 0 ? 0 : gchol_c_off(ws.Cmax));
    if (STAGE == 0) { nrow = C + 21; ncol = C + 21; }
    else { nrow = C + 22 + C; ncol = C; }
    nelim = C;
    return true;
}

// 1. factor the diagonal block A[k:k+nb, k:k+nb] in place (one wave per
// filter).  Lane i holds row i in registers; per pivot j the pivot comes from
// lane j (readlane), lane i scales its L[i][j] and publishes it to a 64-double
// LDS column, and every lane updates its row right-looking, x[c] -= L[i][j]
// L[c][j] (c > j, the column read as an LDS broadcast) -- the element-wise
// right-looking order of the round-2 kernel (same operations, same results),
// without its per-element LDS read-modify-writes and three barriers per pivot
// (round 6).  The entries right of a
// lane's diagonal collect garbage from those updates and are never stored.
template <int STAGE, typename T>
__global__ void __launch_bounds__(64) k_gchol_diag(DevState<T> st, UpdWs<T> ws, int k) {
    const int b = blockIdx.x;
    KT* A;
    int nrow, ncol, nelim;
    if (!gdims<STAGE>(st, ws, b, A, nrow, ncol, nelim) || k >= nelim) return;
    const int ld = ncol, nb = nelim - k < GNB ? nelim - k : GNB;
    __shared__ double colj[2][GNB];
    __shared__ double lt[GNB * (GNB + 1) / 2];   // L_kk^T, packed by columns of L
    const int lane = threadIdx.x;
    // row lane of the block's lower part (zeros right of the diagonal and past nb),
    // every load in flight before the first use
    double x[GNB];
    {
        const KT* src = A + (size_t)(k + lane) * ld + k;
#pragma unroll
        for (int j = 0; j < GNB; ++j) x[j] = (lane < nb && j <= lane) ? src[j] : (j == lane ? 1.0 : 0.0);
    }
    // stage A: pivots floored as in k_kal_a (pcc_pivot_floor); stage C: at s2 down
    // to -T_FLOOR_NEG x max diag(T), as k_kal_c1 / k_kal_mchol (stage B2 keeps
    // diag(T) in ws.Tm: the matrix itself is factored in place)
    double floor = STAGE == 0 ? 0.0 : ws.s2, lo;
    if (STAGE == 0) {
        const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
        for (int i = lane; i < nelim; i += 64) floor = fmax(floor, (double)P[(size_t)(21 + i) * st.Dmax + 21 + i]);
        floor = wave_max(floor) * KALMAN_PIVOT_FLOOR;
        lo = -PIVOT_FLOOR_NEG * floor;
    } else {
        const int ldt = ws.Cmax + 1;
        const KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ldt;
        double tmax = 0.0;
        for (int i = lane; i < nelim; i += 64) tmax = fmax(tmax, (double)Tm[(size_t)i * ldt + i]);
        lo = -T_FLOOR_NEG * wave_max(tmax);
    }
    bool bad = false;
#pragma unroll
    for (int j = 0; j < GNB; ++j) {
        if (j >= nb || bad) continue;   // uniform
        const double piv = pivot_floored(lane_bcast(x[j], j), floor, lo);
        if (!(piv > 0.0)) {
            bad = true;
            continue;
        }
        const double l = sqrt(piv), inv = 1.0 / l;
        const double lij = lane == j ? l : x[j] * inv;
        x[j] = lij;
        double* cj = colj[j & 1];
        cj[lane] = lij;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
        for (int c = j + 1; c < GNB; ++c) x[c] -= lij * cj[c];
    }
    if (bad) {
        if (lane == 0) ws.info[4 * b + 3] = STAGE == 0 ? -2 : -1;
        return;
    }
    if (lane < nb) {
        KT* dst = A + (size_t)(k + lane) * ld + k;
#pragma unroll
        for (int j = 0; j < GNB; ++j)
            if (j <= lane) dst[j] = x[j];
    }
    // L_kk^-1 for k_gchol_trsm: L's columns to LDS (column j packed from its
    // diagonal down, unit rows past nb), then lane j solves column j of L Y = I
    // right-looking (each pivot's column read as an LDS broadcast run); Y goes
    // row-major into the G workspace, which stage B1 fills only after stage A
    // and stage B2 has consumed before stage C
    auto lcol = [](int j) { return j * GNB - j * (j - 1) / 2; };   // offset of L[j][j]
#pragma unroll
    for (int j = 0; j < GNB; ++j)
        if (j <= lane) lt[lcol(j) + lane - j] = x[j];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    double* rdg = colj[0];
    rdg[lane] = 1.0 / lt[lcol(lane)];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int i = 0; i < GNB; ++i) x[i] = i == lane ? 1.0 : 0.0;
#pragma unroll
    for (int i = 0; i < GNB; ++i) {
        const double yi = x[i] * rdg[i];
        x[i] = yi;
#pragma unroll
        for (int r = i + 1; r < GNB; ++r) x[r] -= yi * lt[lcol(i) + r - i];
    }
    KT* Li = ws.G + (size_t)b * ws.Cmax * (ws.Cmax + 1);
#pragma unroll
    for (int i = 0; i < GNB; ++i) Li[i * GNB + lane] = x[i];
}

// 2. panel rows i >= k + nb: A[i, k:k+nb] <- A[i, k:k+nb] L_kk^-T, one 64-row
// tile per workgroup on the matrix cores (gemm64 below) against the inverse
// k_gchol_diag left in the G workspace.  In place: a tile reads all of its rows'
// panel columns before its store.  (The round-2 kernel solved one row per
// thread from per-lane strided row reads: 0.66 ms per stage-C launch at 50x400.)
template <int STAGE, typename T>
__global__ void __launch_bounds__(256) k_gchol_trsm(DevState<T> st, UpdWs<T> ws, int k);

// stage A workspace in / out (grid-stride over the N x N lower part, blockIdx.y = filter)
template <typename T>
__global__ void __launch_bounds__(256) k_gchol_a_load(DevState<T> st, UpdWs<T> ws) {
    const Blk3 bk = xcd_blk3();
    const int b = bk.y;
    KT* A;
    int N, ncol, nelim;
    if (!gdims<0>(st, ws, b, A, N, ncol, nelim)) return;
    const int C = nelim;
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax;
    auto map = [&](int i) { return i < C ? 21 + i : i - C; };
    for (int e = bk.x * 256 + threadIdx.x; e < N * N; e += gridDim.x * 256) {
        const int i = e / N, j = e - i * N;
        if (j <= i) A[(size_t)i * N + j] = (KT)P[(size_t)map(i) * ld + map(j)];
    }
}

template <typename T>
__global__ void __launch_bounds__(256) k_gchol_a_store(DevState<T> st, UpdWs<T> ws) {
    const Blk3 bk = xcd_blk3();
    const int b = bk.y;
    KT* A;
    int N, ncol, nelim;
    if (!gdims<0>(st, ws, b, A, N, ncol, nelim)) return;
    const int C = nelim, Cpw = ws.Cp;
    KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* Vi = ws.Vi + (size_t)b * KW * Cpw;
    KT* Sii = ws.Sii + (size_t)b * KW * KW;
    KT* Xc = ws.Wk + (size_t)b * ws.wk_stride + gchol_c_off(ws.Cmax) + (size_t)C * C;   // stage C's extra rows (ld C)
    for (int e = bk.x * 256 + threadIdx.x; e < N * N; e += gridDim.x * 256) {
        const int i = e / N, j = e - i * N;
        if (j > i) {   // the zeros above Lc's diagonal, in stage C's Lc rows
            if (j < C) Xc[(size_t)(21 + i) * C + j] = 0.0;
            continue;
        }
        const KT v = A[(size_t)i * N + j];
        if (i < C) {
            Lc[(size_t)i * Cpw + j] = v;
            Xc[(size_t)(21 + i) * C + j] = v;
        } else if (j < C) {
            Vi[(size_t)(i - C) * Cpw + j] = v;
            Xc[(size_t)(i - C) * C + j] = v;
        } else {
            Sii[(i - C) * KW + (j - C)] = v;
        }
    }
}

// 3. trailing update A[i][j] -= sum_p W[i][p] W[j][p], p in [k, k+nb), for the
// lower part j <= i, j in [k+nb, ncol), i in [k+nb, nrow): 64 x 64 MFMA tiles
template <int STAGE, typename T>
__global__ void __launch_bounds__(256) k_gchol_update(DevState<T> st, UpdWs<T> ws, int k);

size_t kalman_global_ws_doubles(int Cmax) {   // per filter, 0 when the register-tile stages fit
    if (kalman_chol_supported(Cmax)) return 0;
    const size_t C = Cmax, N = C + 21, E = 21 + C + 1;
    const size_t a = N * N, c = (C + E) * C;
    return a + c;   // stage A's matrix, then stage C's (gchol_c_off)
}

// ===========================================================================
// 64 x 64 output tile on the matrix cores: 256 threads = 4 waves, wave w owns
// the 32 x 32 quarter (w >> 1, w & 1) as 2 x 2 v_mfma_f64_16x16x4 tiles; K in
// steps of 16 staged through LDS ([k][i] / [k][j], rows padded to 80 doubles so
// the two k-rows a 32-lane group reads land on disjoint banks).  A(i, k) and
// B(k, j) are accessors; *_KFAST says whether consecutive k are contiguous in
// memory for that operand (selects the coalesced load mapping).  store(i, j, v)
// receives every in-range output element once.
// ===========================================================================
constexpr int GT = 64, GK = 16;

// TM x TM output tile per 256-thread workgroup (TM = 64 or 128): the four waves in
// 2 x 2, each TM/2 square as (TM/32)^2 v_mfma_f64_16x16x4f64 blocks.
// Double-buffered K chunks: chunk c + 1's global loads are in flight (in
// registers) under chunk c's MFMAs, one barrier per chunk (round 6; the
// single-buffered loop exposed every chunk's load latency).
template <int TM, bool A_KFAST, bool B_KFAST, class FA, class FB, class FS>
__device__ __forceinline__ void gemm_tile(int m, int n, int kb, int ke, int i0, int j0, FA A, FB B, FS store) {
    constexpr int NBW = TM / 32, NLD = TM * GK / 256, PAD = TM + 16, HW = TM / 2;
    __shared__ __attribute__((aligned(16))) double sa[2][GK][PAD], sb[2][GK][PAD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1, lc = lane & 15, lr = lane >> 4;
    v4d acc[NBW][NBW];
#pragma unroll
    for (int mi = 0; mi < NBW; ++mi)
#pragma unroll
        for (int ni = 0; ni < NBW; ++ni) acc[mi][ni] = v4d{0.0, 0.0, 0.0, 0.0};
    double ra[NLD], rb[NLD];
    auto idx = [&](int q, bool kfast, int& r, int& kk) {
        const int e = tid + 256 * q;
        if (kfast) { r = e >> 4; kk = e & 15; } else { r = e % TM; kk = e / TM; }
    };
    auto gload = [&](int k0) {
#pragma unroll
        for (int q = 0; q < NLD; ++q) {
            int ii, kk, jj, k2;
            idx(q, A_KFAST, ii, kk);
            idx(q, B_KFAST, jj, k2);
            const int gi = i0 + ii, gk = k0 + kk;
            ra[q] = (gi < m && gk < ke) ? A(gi, gk) : 0.0;
            const int gj = j0 + jj, gk2 = k0 + k2;
            rb[q] = (gj < n && gk2 < ke) ? B(gk2, gj) : 0.0;
        }
    };
    auto sstore = [&](int bf) {
#pragma unroll
        for (int q = 0; q < NLD; ++q) {
            int ii, kk, jj, k2;
            idx(q, A_KFAST, ii, kk);
            idx(q, B_KFAST, jj, k2);
            sa[bf][kk][ii] = ra[q];
            sb[bf][k2][jj] = rb[q];
        }
    };
    if (kb < ke) {
        gload(kb);
        sstore(0);
    }
    __syncthreads();
    for (int k0 = kb, it = 0; k0 < ke; k0 += GK, ++it) {
        const int bf = it & 1;
        const bool more = k0 + GK < ke;   // uniform
        if (more) gload(k0 + GK);
#pragma unroll
        for (int kc = 0; kc < GK / 4; ++kc) {
            const int kr = 4 * kc + lr;
            double av[NBW], bv[NBW];
#pragma unroll
            for (int t = 0; t < NBW; ++t) {
                av[t] = sa[bf][kr][HW * wr + 16 * t + lc];
                bv[t] = sb[bf][kr][HW * wc + 16 * t + lc];
            }
#pragma unroll
            for (int mi = 0; mi < NBW; ++mi)
#pragma unroll
                for (int ni = 0; ni < NBW; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
        }
        if (more) sstore(bf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int mi = 0; mi < NBW; ++mi)
#pragma unroll
        for (int ni = 0; ni < NBW; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = i0 + HW * wr + 16 * mi + lr + 4 * r, j = j0 + HW * wc + 16 * ni + lc;
                if (i < m && j < n) store(i, j, acc[mi][ni][r]);
            }
}
template <bool A_KFAST, bool B_KFAST, class FA, class FB, class FS>
__device__ __forceinline__ void gemm64(int m, int n, int kb, int ke, int i0, int j0, FA A, FB B, FS store) {
    gemm_tile<64, A_KFAST, B_KFAST>(m, n, kb, ke, i0, j0, A, B, store);
}

template <int STAGE, typename T>
__global__ void __launch_bounds__(256) k_gchol_trsm(DevState<T> st, UpdWs<T> ws, int k) {
    const Blk3 bk = xcd_blk3();
    const int b = bk.y;
    KT* A;
    int nrow, ncol, nelim;
    if (!gdims<STAGE>(st, ws, b, A, nrow, ncol, nelim) || k >= nelim) return;
    const int ld = ncol, nb = nelim - k < GNB ? nelim - k : GNB;
    const int i0 = k + nb + bk.x * GT;
    if (i0 >= nrow) return;
    const KT* Li = ws.G + (size_t)b * ws.Cmax * (ws.Cmax + 1);   // L_kk^-1, row-major GNB x GNB
    gemm64<true, true>(nrow, nb, 0, nb, i0, 0,
                       [&](int i, int p) { return A[(size_t)i * ld + k + p]; },
                       [&](int p, int j) { return Li[j * GNB + p]; },
                       [&](int i, int j, double v) { A[(size_t)i * ld + k + j] = v; });
}

template <int STAGE, typename T>
__global__ void __launch_bounds__(256) k_gchol_update(DevState<T> st, UpdWs<T> ws, int k) {
    const Blk3 bk = xcd_blk3();
    const int b = bk.z;
    KT* A;
    int nrow, ncol, nelim;
    if (!gdims<STAGE>(st, ws, b, A, nrow, ncol, nelim) || k >= nelim) return;
    const int ld = ncol, k1 = k + (nelim - k < GNB ? nelim - k : GNB);
    const int i0 = k1 + bk.y * GT, j0 = k1 + bk.x * GT;
    if (i0 >= nrow || j0 >= ncol || i0 + GT - 1 < j0) return;   // outside, or entirely above the diagonal
    gemm64<true, true>(nrow, ncol, k, k1, i0, j0,
                       [&](int i, int p) { return A[(size_t)i * ld + p]; },
                       [&](int p, int j) { return A[(size_t)j * ld + p]; },
                       [&](int i, int j, double v) {
                           if (j <= i) A[(size_t)i * ld + j] -= v;
                       });
}

// ---- stage B1: G = A Lc (C x C) ----
template <typename T>
__global__ void __launch_bounds__(256) k_kal_b1(DevState<T> st, UpdWs<T> ws) {
    const Blk3 bk = xcd_blk3();
    const int b = bk.z;
    if (ws.info[4 * b] == 0) return;
    const int C = 6 * st.ncams[b];
    const int i0 = bk.y * GT, j0 = bk.x * GT;
    if (i0 >= C || j0 >= C) return;
    const int lda = ws.Cmax + 1, Cpw = ws.Cp;
    const KT* Am = ws.Hthin + (size_t)b * ws.Cmax * lda;
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* G = ws.G + (size_t)b * ws.Cmax * lda;
    gemm64<true, false>(C, C, j0 & ~(GK - 1), C, i0, j0,
                        [&](int i, int k) { return Am[(size_t)i * lda + k]; },
                        [&](int k, int j) { return k >= j ? Lc[(size_t)k * Cpw + j] : 0.0; },
                        [&](int i, int j, double v) { G[(size_t)i * lda + j] = v; });
}

// ---- stage B2: [T | c] = s2 I + Lc^T [G | b] (lower triangle of T, and c) ----
template <typename T>
__global__ void __launch_bounds__(256) k_kal_b2(DevState<T> st, Params<T> prm, UpdWs<T> ws) {
    const Blk3 bk = xcd_blk3();
    const int b = bk.z;
    if (ws.info[4 * b] == 0) return;
    const int C = 6 * st.ncams[b];
    const int i0 = bk.y * GT, j0 = bk.x * GT;
    if (i0 >= C || j0 > C) return;
    if (j0 > i0 + GT - 1 && !(C >= j0 && C < j0 + GT)) return;   // strictly upper and no c column
    const int ld = ws.Cmax + 1, Cpw = ws.Cp;
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    const KT* G = ws.G + (size_t)b * ws.Cmax * ld;
    const KT* Hb = ws.Hthin + (size_t)b * ws.Cmax * ld;   // b in column Cmax
    KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ld;   // its diagonal only: stage C's pivot bound (k_gchol_diag<1>)
    KT* Ac = ws.Wk + (size_t)b * ws.wk_stride + gchol_c_off(ws.Cmax);   // stage C's [T ; extra rows], ld C
    const double s2 = (double)prm.sigma2;
    gemm64<false, false>(C, C + 1, i0 & ~(GK - 1), C, i0, j0,
                         [&](int i, int k) { return k >= i ? Lc[(size_t)k * Cpw + i] : 0.0; },
                         [&](int k, int j) { return j < C ? G[(size_t)k * ld + j] : Hb[(size_t)k * ld + ws.Cmax]; },
                         [&](int i, int j, double v) {
                             if (j < C && j <= i) {
                                 const double t = v + (i == j ? s2 : 0.0);
                                 Ac[(size_t)i * C + j] = t;
                                 if (i == j) Tm[(size_t)i * ld + i] = t;
                             }
                             if (j == C) Ac[(size_t)(2 * C + 21) * C + i] = v;   // c^T: the last extra row
                         });
}

// ---- stage B, one workgroup per filter (production path when C <= 16 * NTM) ----
// Phase 1: the lower 16 x 16 tiles of G = A Lc -- phase 2 reads G[k][j] only
// for k >= 16 (j / 16) (T[i][j] = sum_k Lc[k][i] G[k][j], Lc[k][i] = 0 for
// k < i, i >= j), so the upper tiles are neither formed nor stored (round 5:
// 28 % of the phase's MFMAs and half of G's HBM round trip).  Wave w owns
// tiles w + NW s of the column-major lower enumeration: a K chunk k0 reaches
// the tile columns <= k0 / 16 (Lc lower triangular), i.e. a prefix of that
// enumeration, which the round-robin deal spreads evenly over the waves
// (46 tile-chunks on the busiest wave at 12 x 12 tiles, against 72 for the
// full grid on a 4 x 4 wave grid).
// Phase 2: lower tiles of T = s2 I + Lc^T G (wave w owns tiles w + NW s of the
// row-major lower enumeration) and c = Lc^T b.  K streams in chunks of 16 rows
// through double-buffered LDS images [k][col]; A is read from its stored lower
// triangle (row or column segments, see load()), Lc and G as row slices.  Chunks that
// meet only the zero upper triangle of Lc are skipped per tile.
__device__ __forceinline__ void lower_tile(int t, int& ti, int& tj) {
    int i = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
    while (i * (i + 1) / 2 > t) --i;
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    ti = i;
    tj = t - i * (i + 1) / 2;
}

template <typename T, int NW, int NTM>
__global__ void __launch_bounds__(64 * NW) k_kal_b(DevState<T> st, Params<T> prm, UpdWs<T> ws) {
    constexpr int TP2 = (NTM * (NTM + 1) / 2 + NW - 1) / NW;     // lower tiles per wave (both phases)
    constexpr int NT = 64 * NW, Q = (16 * 16 * NTM + NT - 1) / NT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    if (ws.info[4 * b] == 0) return;
    const int C = 6 * st.ncams[b], nT = (C + 15) / 16, Cq = 16 * nT;
    const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ld = ws.Cmax + 1, Cpw = ws.Cp;
    const KT* Am = ws.Hthin + (size_t)b * ws.Cmax * ld;   // b in column Cmax
    const KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* G = ws.G + (size_t)b * ws.Cmax * ld;
    KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ld;
    // LDS images [2 buf][2 op][16][CqS], then [2][16] b chunk.  Row strides
    // (ds_read_b64 banks are (a/4) % 64 per 32-lane half = two k rows of 16
    // doubles): phase 1 uses CqS = 17 (mod 32) -- its column-gathered writes
    // step 34 dwords across lanes (conflict-free on 32 write banks) and the two
    // rows of a read half overlap on 2 banks only (Cq + 2 overlapped 28 of
    // them for even nT); phase 2's writes are row-contiguous, so it takes
    // CqS = 16 (mod 32) and its read halves are disjoint.
    const int CqS1 = (Cq & ~31) + 17, CqS2 = (Cq & ~31) + 16;
    double* img = reinterpret_cast<double*>(smem_raw);
    double* bb = img + 4 * 16 * CqS1;
    // operand 0 = rows of X (A in phase 1, Lc in phase 2), operand 1 = rows of Y (Lc, G).
    // load() issues the next chunk's global reads into registers before the
    // MFMAs of the current one; put() writes them to the other LDS buffer after.
    // A is stored as its lower triangle only (k_info_fused): phase 1 gathers
    // the chunk's 16 x 16 column tiles left of / on the diagonal as row
    // segments A[k][c] and those right of it as column segments A[c][k] (16
    // lanes over k: 128 contiguous bytes of row c), so every read stays coalesced.
    double r0[Q], r1[Q], rb = 0.0;
    int pos[Q];
    auto load = [&](int ph, int k0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int e = tid + NT * q;
            int k, c;
            if (ph == 0) {
                const int jt = e >> 8, u = e & 255;
                const bool up = jt > (k0 >> 4);
                k = up ? (u & 15) : (u >> 4);
                c = 16 * jt + (up ? (u >> 4) : (u & 15));
            } else {
                k = e / Cq;
                c = e - k * Cq;
            }
            const int gk = k0 + k;
            pos[q] = k * (ph == 0 ? CqS1 : CqS2) + c;
            const bool in = e < 16 * Cq && gk < C && c < C;
            const double lcv = (in && c <= gk) ? Lc[(size_t)gk * Cpw + c] : 0.0;
            double ov;
            if (ph == 0) {
                ov = in ? Am[c <= gk ? (size_t)gk * ld + c : (size_t)c * ld + gk] : 0.0;
            } else {   // G row gk holds the lower tile columns <= gk / 16 only
                ov = (in && c < 16 * (gk / 16 + 1)) ? G[(size_t)gk * ld + c] : 0.0;
            }
            r0[q] = ph == 0 ? ov : lcv;
            r1[q] = ph == 0 ? lcv : ov;
        }
        if (ph == 1 && tid < 16) rb = k0 + tid < C ? Am[(size_t)(k0 + tid) * ld + ws.Cmax] : 0.0;
    };
    auto put = [&](int ph, int buf) {
        const int CqS = ph == 0 ? CqS1 : CqS2;
        double* i0 = img + (2 * buf) * 16 * CqS;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int e = tid + NT * q;
            if (e < 16 * Cq) {
                i0[pos[q]] = r0[q];
                i0[16 * CqS + pos[q]] = r1[q];
            }
        }
        if (ph == 1 && tid < 16) bb[buf * 16 + tid] = rb;
    };
    // ---- phase 1: the lower tiles of G = A Lc ----
    {
        const int CqS = CqS1;
        const int ntl = nT * (nT + 1) / 2;
        v4d acc[TP2];
        int gr[TP2], gc[TP2];
#pragma unroll
        for (int s = 0; s < TP2; ++s) {   // column-major lower enumeration
            const int t = wv + NW * s, tt = t < ntl ? t : 0;
            const int c = colmajor_col(tt, nT), r = c + tt - (c * nT - c * (c - 1) / 2);
            gr[s] = __builtin_amdgcn_readfirstlane(t < ntl ? r : -1);
            gc[s] = __builtin_amdgcn_readfirstlane(c);
            acc[s] = v4d{0.0, 0.0, 0.0, 0.0};
        }
        load(0, 0);
        put(0, 0);
        __syncthreads();
        for (int k0 = 0, it = 0; k0 < C; k0 += 16, ++it) {
            const int buf = it & 1;
            const bool more = k0 + 16 < C;
            if (more) load(0, k0 + 16);
            const double* i0 = img + (2 * buf) * 16 * CqS;
            const double* i1 = i0 + 16 * CqS;
#pragma unroll
            for (int kc = 0; kc < 4; ++kc) {
                const int kr = (4 * kc + lr) * CqS;
#pragma unroll
                for (int s = 0; s < TP2; ++s) {
                    // Lc[k][j] = 0 for j > k: column tile gc needs k >= 16 gc
                    if (gr[s] < 0 || k0 + 15 < 16 * gc[s]) continue;
                    acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(i0[kr + 16 * gr[s] + lc], i1[kr + 16 * gc[s] + lc],
                                                                  acc[s], 0, 0, 0);
                }
            }
            if (more) put(0, buf ^ 1);
            __syncthreads();
        }
#pragma unroll
        for (int s = 0; s < TP2; ++s) {
            if (gr[s] < 0) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * gr[s] + lr + 4 * r, j = 16 * gc[s] + lc;
                if (i < C && j < C) G[(size_t)i * ld + j] = acc[s][r];
            }
        }
        __syncthreads();   // G visible to the whole workgroup before phase 2 streams it
    }
    // ---- phase 2: T = s2 I + Lc^T G (lower), c = Lc^T b ----
    {
        const int CqS = CqS2;
        const int ntl = nT * (nT + 1) / 2;
        v4d acc[TP2];
        int ti[TP2], tj[TP2];
#pragma unroll
        for (int s = 0; s < TP2; ++s) {
            const int t = wv + NW * s;
            int x, y;
            lower_tile(t, x, y);
            ti[s] = __builtin_amdgcn_readfirstlane(t < ntl ? x : -1);
            tj[s] = __builtin_amdgcn_readfirstlane(y);
            acc[s] = v4d{0.0, 0.0, 0.0, 0.0};
        }
        double ca = 0.0;
        load(1, 0);
        put(1, 0);
        __syncthreads();
        for (int k0 = 0, it = 0; k0 < C; k0 += 16, ++it) {
            const int buf = it & 1;
            const bool more = k0 + 16 < C;
            if (more) load(1, k0 + 16);
            const double* i0 = img + (2 * buf) * 16 * CqS;
            const double* i1 = i0 + 16 * CqS;
#pragma unroll
            for (int kc = 0; kc < 4; ++kc) {
                const int kr = (4 * kc + lr) * CqS;
#pragma unroll
                for (int s = 0; s < TP2; ++s) {
                    // Lc[k][i] = 0 for i > k: row tile ti needs k >= 16 ti
                    if (ti[s] < 0 || k0 + 15 < 16 * ti[s]) continue;
                    acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(i0[kr + 16 * ti[s] + lc], i1[kr + 16 * tj[s] + lc],
                                                                  acc[s], 0, 0, 0);
                }
            }
            if (tid < C) {
#pragma unroll
                for (int k = 0; k < 16; ++k) ca += i0[k * CqS + tid] * bb[buf * 16 + k];
            }
            if (more) put(1, buf ^ 1);
            __syncthreads();
        }
        const double s2 = (double)prm.sigma2;
#pragma unroll
        for (int s = 0; s < TP2; ++s) {
            if (ti[s] < 0) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 16 * ti[s] + lr + 4 * r, j = 16 * tj[s] + lc;
                if (i < C && j <= i) Tm[(size_t)i * ld + j] = acc[s][r] + (i == j ? s2 : 0.0);
            }
        }
        if (tid < C) Tm[(size_t)tid * ld + C] = ca;
    }
}

// ---- stage E: P+ = blockdiag(S_ii, 0) + s2 W W^T (lower tiles, mirrored), dx = W y ----
template <typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) k_kal_e(DevState<T> st, Params<T> prm, UpdWs<T> ws) {
    constexpr int TE = 128;   // output tile (round 6: 64 -> 128, twice the operand reuse per chunk)
    const Blk3 bk = xcd_blk3();
    const int b = bk.z;
    if (ws.info[4 * b] == 0 || ws.info[4 * b + 3] < 0) return;
    const int C = 6 * st.ncams[b], D = 21 + C;
    const int i0 = bk.y * TE, j0 = bk.x * TE;
    if (i0 >= D || j0 > D) return;
    if (j0 > i0 + TE - 1 && !(D >= j0 && D < j0 + TE)) return;
    const int ld = st.Dmax;
    // W: stage C's solved extra rows [Vc_i ; Lc ; c^T] L_T^-T, in place after T (ld C)
    const KT* W = ws.Wk + (size_t)b * ws.wk_stride + gchol_c_off(ws.Cmax) + (size_t)C * C;
    const KT* Sii = ws.Sii + (size_t)b * KW * KW;
    T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    KT* dx = ws.dx + (size_t)b * (st.Dmax + ws.Cmax);
    const double s2 = (double)prm.sigma2;
    gemm_tile<TE, true, true>(D, D + 1, 0, C, i0, j0, [&](int i, int k) { return W[(size_t)i * C + k]; },
                       [&](int k, int j) { return W[(size_t)(j < D ? j : D) * C + k]; },
                       [&](int i, int j, double v) {
                           if (j < D && j <= i) {
                               double p = s2 * v;
                               if (i < 21 && j < 21) p += Sii[i * KW + j];
                               P[(size_t)i * ld + j] = (T)p;
                               P[(size_t)j * ld + i] = (T)p;
                           }
                           if (j == D) dx[i] = v;
                       });
}

// ---- stage E, one workgroup per filter (production path when D fits) ----
// 16 waves; wave w owns lower 16 x 16 tiles t = w + 16 s (s < TPW) of P+ as
// MFMA accumulators.  W streams once through double-buffered LDS in chunks of
// 16 columns ([k][row] images, so each MFMA operand is one ds_read_b64); the
// same chunks give dx = W y (thread i < D accumulates row i).
template <typename T, int NW, int TPW>
__global__ void __launch_bounds__(64 * NW) k_kal_e1(DevState<T> st, Params<T> prm, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    if (ws.info[4 * b] == 0 || ws.info[4 * b + 3] < 0) return;
    const int C = 6 * st.ncams[b], D = 21 + C, nT = (D + 15) / 16, Dp = 16 * nT;
    const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ntiles = nT * (nT + 1) / 2;
    const int Cpw = ws.Cp, ld = st.Dmax;
    const KT* W = ws.W + (size_t)b * (st.Dmax + 1) * Cpw;
    double* img = reinterpret_cast<double*>(smem_raw);   // [2][16][Dp] chunk images, then [2][16] y
    double* yb = img + 2 * 16 * Dp;
    int ti[TPW], tj[TPW];
#pragma unroll
    for (int s = 0; s < TPW; ++s) {   // row-major lower enumeration of the tile grid
        const int t = wv + NW * s;
        int i = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
        while (i * (i + 1) / 2 > t) --i;
        while ((i + 1) * (i + 2) / 2 <= t) ++i;
        ti[s] = __builtin_amdgcn_readfirstlane(t < ntiles ? i : -1);
        tj[s] = __builtin_amdgcn_readfirstlane(t - i * (i + 1) / 2);
    }
    v4d acc[TPW];
#pragma unroll
    for (int s = 0; s < TPW; ++s) acc[s] = v4d{0.0, 0.0, 0.0, 0.0};
    double dxa = 0.0, dxb = 0.0;
    // W[:, k0:k0+16] -> img[buf][k][row] and the y chunk; load() before the
    // current chunk's MFMAs, put() after them
    constexpr int NT = 64 * NW, Q = (16 * 16 * (NW * TPW <= 96 ? 13 : 15) + NT - 1) / NT;
    double rw[Q], ry = 0.0;
    // W^T as stage C2 stores it: row-major over k, leading dimension Dmax + 1
    const int ldw = st.Dmax + 1;
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int e = tid + NT * q;
            const int k = e / Dp, row = e - k * Dp;
            rw[q] = (e < 16 * Dp && row < D && k0 + k < C) ? W[(size_t)(k0 + k) * ldw + row] : 0.0;
        }
        if (tid < 16) ry = k0 + tid < C ? W[(size_t)(k0 + tid) * ldw + D] : 0.0;
    };
    auto put = [&](int buf) {
        double* im = img + buf * 16 * Dp;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int e = tid + NT * q;
            if (e < 16 * Dp) im[e] = rw[q];
        }
        if (tid < 16) yb[buf * 16 + tid] = ry;
    };
    load(0);
    put(0);
    __syncthreads();
    for (int k0 = 0, it = 0; k0 < C; k0 += 16, ++it) {
        const int buf = it & 1;
        const bool more = k0 + 16 < C;
        if (more) load(k0 + 16);
        const double* im = img + buf * 16 * Dp;
#pragma unroll
        for (int kc = 0; kc < 4; ++kc) {
            const double* kr = im + (4 * kc + lr) * Dp;
#pragma unroll
            for (int s = 0; s < TPW; ++s) {
                if (ti[s] < 0) continue;
                acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(kr[16 * ti[s] + lc], kr[16 * tj[s] + lc], acc[s], 0, 0, 0);
            }
        }
        if (tid < D) {
#pragma unroll
            for (int k = 0; k < 16; ++k) dxa += im[k * Dp + tid] * yb[buf * 16 + k];
        }
        if (NT + tid < D) {
#pragma unroll
            for (int k = 0; k < 16; ++k) dxb += im[k * Dp + NT + tid] * yb[buf * 16 + k];
        }
        if (more) put(buf ^ 1);
        __syncthreads();
    }
    const double s2 = (double)prm.sigma2;
    const KT* Sii = ws.Sii + (size_t)b * KW * KW;
    T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
        if (ti[s] < 0) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = 16 * ti[s] + lr + 4 * r, j = 16 * tj[s] + lc;
            if (i >= D || j >= D || j > i) continue;
            double p = s2 * acc[s][r];
            if (i < 21 && j < 21) p += Sii[i * KW + j];
            P[(size_t)i * ld + j] = (T)p;
            P[(size_t)j * ld + i] = (T)p;
        }
    }
    if (tid < D) ws.dx[(size_t)b * (st.Dmax + ws.Cmax) + tid] = dxa;
    if (NT + tid < D) ws.dx[(size_t)b * (st.Dmax + ws.Cmax) + NT + tid] = dxb;
}

// ===========================================================================
// Stages A and C1 on the matrix cores (round 4, k_kal_mchol): the partial
// Cholesky of rchol_core, 4 pivots per step, with the matrix held as 16 x 16
// fp64 MFMA accumulator blocks (result layout: lane l holds rows (l >> 4) + 4 i
// of column l & 15) spread round-robin over NW waves, and the trailing rank-4
// update of each block one v_mfma_f64_16x16x4f64:
//     C -= X A_d^-1 X^T = C + (X m) X^T,   m = -A_d^-1 e_(l >> 4),
// X = the step's four pivot columns, dumped to a double-buffered LDS panel by
// the lanes that own them (one barrier per step).  Every lane factors the 4 x 4
// A_d = L D L^T itself from the panel (one fp64 chain: hardware reciprocals
// with a Newton step, no division or square root), the Cholesky columns
// Y = X L_d^-T of the step (Lc / Vc_i in A, L_T in C1) are formed one panel row
// per thread and stored.  Pivot floors as rchol_core (stage A: rounding-level
// negatives; C1: T >= s2 I).  Stage A's shifted retries of a failed filter run
// in a small second launch over the failed filters only (found by one
// parallel scan of the failure flags).
// ===========================================================================
constexpr int MK_PS = 4;   // doubles per panel row (the step's four columns)

__device__ __forceinline__ double mk_rcp(double x) {   // 1 / x: hardware reciprocal + one Newton step
    const double r = __builtin_amdgcn_rcp(x);
    return r * fma(-x, r, 2.0);
}

__host__ __device__ constexpr int mk_lds_doubles(int NBR) { return 2 * 16 * NBR * MK_PS + 16; }

// One factorisation of filter b (stage A: P_cc + shift I).  Returns false on a
// failed pivot; all outputs written on success.
template <typename T, int NW, int NBR, int STAGE>
__device__ __forceinline__ bool mk_factor(const DevState<T>& st, const UpdWs<T>& ws, int b, double shift,
                                          double floor, double lo, double* pan0) {
    constexpr int NBLK = NBR * (NBR + 1) / 2, SL = (NBLK + NW - 1) / NW;
    const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = 6 * st.ncams[b], Cp = round4(C);
    const int nrows = STAGE == 0 ? Cp + KW : C;   // rows beyond: identity padding up to 16 NBR
    const int nsteps = Cp / 4;
    const int ld = st.Dmax, Cpw = ws.Cp, ldt = ws.Cmax + 1;
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    KT* Lc = ws.Lc + (size_t)b * Cpw * Cpw;
    KT* Vi = ws.Vi + (size_t)b * KW * Cpw;
    KT* Sii = ws.Sii + (size_t)b * KW * KW;
    const KT* Tm = ws.Tm + (size_t)b * ws.Cmax * ldt;
    KT* LT = ws.G + (size_t)b * ws.Cmax * ldt;
    // stage A index space [cams (Cp) | IMU (24)]: P row of index i (-1: padding)
    auto map = [&](int i) { return i < C ? 21 + i : (i < Cp ? -1 : (i < Cp + 21 ? i - Cp : -1)); };
    auto load = [&](int i, int j) -> double {
        if (STAGE == 0) {
            const int mi = map(i), mj = map(j);
            if (mi < 0 || mj < 0) return i == j ? 1.0 : 0.0;
            return (double)P[(size_t)mi * ld + mj] + (i == j && i < C ? shift : 0.0);
        } else {
            if (i >= C || j >= C) return i == j ? 1.0 : 0.0;
            return i >= j ? Tm[(size_t)i * ldt + j] : Tm[(size_t)j * ldt + i];
        }
    };
    // blocks of this wave: t = wv + NW j, column-major lower order
    int brow[SL], bcol[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) {
        const int t = wv + NW * j;
        int cb = 0, rem = t;
        while (cb < NBR && rem >= NBR - cb) { rem -= NBR - cb; ++cb; }
        brow[j] = t < NBLK ? cb + rem : -1;
        bcol[j] = t < NBLK ? cb : NBR;   // an empty slot matches no column
    }
    using v4d_t = double __attribute__((ext_vector_type(4)));
    v4d_t acc[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[j][q] = brow[j] >= 0 ? load(16 * brow[j] + lr + 4 * q, 16 * bcol[j] + lc) : 0.0;
    const double oh[4] = {lr == 0 ? 1.0 : 0.0, lr == 1 ? 1.0 : 0.0, lr == 2 ? 1.0 : 0.0, lr == 3 ? 1.0 : 0.0};
    for (int s = 0; s < nsteps; ++s) {
        const int KB = s >> 2, sc = s & 3, p0 = 4 * s;
        double* pan = pan0 + (s & 1) * 16 * NBR * MK_PS;
        // 1. the owners of columns p0 .. p0 + 3 dump them (rows of block column KB)
        if ((lc >> 2) == sc) {
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                if (bcol[j] != KB) continue;   // uniform
                double* d = pan + (16 * brow[j] + lr) * MK_PS + (lc & 3);
#pragma unroll
                for (int q = 0; q < 4; ++q) d[4 * q * MK_PS] = acc[j][q];
            }
        }
        __syncthreads();
        // 2. A_d = L D L^T (lower entries of the panel's rows p0 .. p0 + 3), floored pivots
        const double* ad = pan + p0 * MK_PS;
        const double a10 = ad[4], a20 = ad[8], a30 = ad[12];
        const double a21 = ad[9], a31 = ad[13], a32 = ad[14];
        const double d0 = pivot_floored(ad[0], floor, lo), e0 = mk_rcp(d0);
        const double l10 = a10 * e0, l20 = a20 * e0, l30 = a30 * e0;
        const double d1 = pivot_floored(ad[5] - l10 * a10, floor, lo), e1 = mk_rcp(d1);
        const double m21 = a21 - l20 * a10, m31 = a31 - l30 * a10;
        const double l21 = m21 * e1, l31 = m31 * e1;
        const double d2 = pivot_floored(ad[10] - l20 * a20 - l21 * m21, floor, lo), e2 = mk_rcp(d2);
        const double m32 = a32 - l30 * a20 - l31 * m21;
        const double l32 = m32 * e2;
        const double d3 = pivot_floored(ad[15] - l30 * a30 - l31 * m31 - l32 * m32, floor, lo), e3 = mk_rcp(d3);
        if (!(d0 > 0.0) || !(d1 > 0.0) || !(d2 > 0.0) || !(d3 > 0.0)) {   // uniform
            __syncthreads();   // every wave's panel reads are done before a retry's dumps
            return false;
        }
        // 3. Cholesky columns p0 .. p0 + 3: y = x L_u^-T D^-1/2, one panel row per thread
        {
            const int r = p0 + tid;
            if (r < nrows) {
                const double* x = pan + r * MK_PS;
                const double z0 = x[0], z1 = x[1] - l10 * z0, z2 = x[2] - l20 * z0 - l21 * z1;
                const double z3 = x[3] - l30 * z0 - l31 * z1 - l32 * z2;
                const int k = r - p0;   // rows of the diagonal block: zeros above the diagonal
                // the diagonal entries take the (possibly floored) pivot itself: z_k
                // of row p0 + k is the unfloored Schur value (a floored -1e-12 would
                // otherwise give L_kk = -1e-12 / sqrt(s2) instead of sqrt(s2))
                const double y0 = (k == 0 ? d0 : z0) * rchol_rsq(d0);
                const double y1 = k >= 1 ? (k == 1 ? d1 : z1) * rchol_rsq(d1) : 0.0;
                const double y2 = k >= 2 ? (k == 2 ? d2 : z2) * rchol_rsq(d2) : 0.0;
                const double y3 = k >= 3 ? (k == 3 ? d3 : z3) * rchol_rsq(d3) : 0.0;
                if (STAGE == 0) {
                    KT* dst = r < Cp ? Lc + (size_t)r * Cpw + p0 : Vi + (size_t)(r - Cp) * Cpw + p0;
                    dst[0] = y0; dst[1] = y1; dst[2] = y2; dst[3] = y3;
                } else {
                    KT* dst = LT + (size_t)r * ldt + p0;
                    dst[0] = y0;
                    if (p0 + 1 < C) dst[1] = y1;
                    if (p0 + 2 < C) dst[2] = y2;
                    if (p0 + 3 < C) dst[3] = y3;
                }
            }
        }
        // 4. m = -A_d^-1 e_lr (h = L^-1 e, u = D^-1 h, m = L^-T u), then the
        //    rank-4 update of every block right of the pivots
        const double h0 = oh[0];
        const double h1 = fma(-l10, h0, oh[1]);
        const double h2 = fma(-l21, h1, fma(-l20, h0, oh[2]));
        const double h3 = fma(-l32, h2, fma(-l31, h1, fma(-l30, h0, oh[3])));
        const double u0 = h0 * e0, u1 = h1 * e1, u2 = h2 * e2, u3 = h3 * e3;
        const double w2 = fma(-l32, u3, u2);
        const double w1 = fma(-l31, u3, fma(-l21, w2, u1));
        const double w0 = fma(-l30, u3, fma(-l20, w2, fma(-l10, w1, u0)));
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            if (brow[j] < 0 || bcol[j] < KB || (bcol[j] == KB && sc == 3)) continue;   // uniform
            const double* xr = pan + (16 * brow[j] + lc) * MK_PS;
            const double av = -(xr[0] * w0 + xr[1] * w1 + xr[2] * w2 + xr[3] * u3);
            const double bv = pan[(16 * bcol[j] + lc) * MK_PS + lr];
            acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[j], 0, 0, 0);
        }
    }
    if (STAGE == 0) {   // S_ii: the Schur complement left in rows / columns >= Cp (lower part)
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            if (brow[j] < 0 || 16 * bcol[j] + 15 < Cp) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int i = 16 * brow[j] + lr + 4 * q, c = 16 * bcol[j] + lc;
                if (i >= Cp && c >= Cp && c <= i && i < Cp + KW) Sii[(i - Cp) * KW + (c - Cp)] = acc[j][q];
            }
        }
    }
    __syncthreads();
    return true;
}

// one workgroup per filter (RETRY: stage A's shifted retries, a few
// workgroups looping over the filters whose first factorisation failed)
// two filters per CU: NW / 2 waves per SIMD each
__host__ __device__ constexpr int mk_wpe(int NW) { return NW <= 4 ? 2 : (NW <= 8 ? 4 : 8); }

template <typename T, int NW, int NBR, int STAGE, bool RETRY = false>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(mk_wpe(NW))))
k_kal_mchol(DevState<T> st, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    double* pan0 = reinterpret_cast<double*>(smem_raw);   // [2][16 NBR][MK_PS]
    double* red = pan0 + 2 * 16 * NBR * MK_PS;             // 16 doubles of reduction scratch
    const int tid = threadIdx.x;
    if (STAGE == 1) {
        const int b = blockIdx.x;
        if (ws.info[4 * b] == 0) return;
        if (ws.afail[b]) {   // stage A failed (P_cc not PD): no update for this filter
            if (tid == 0) ws.info[4 * b + 3] = -2;
            return;
        }
        // T = s2 I + Lc^T A Lc >= s2 I: pivots below s2 are rounding (k_kal_c1)
        const int C = 6 * st.ncams[b], ldt = ws.Cmax + 1;
        const double tmax = diag_max(ws.Tm + (size_t)b * ws.Cmax * ldt, ldt, 0, C, red);
        const bool ok = mk_factor<T, NW, NBR, 1>(st, ws, b, 0.0, ws.s2, -T_FLOOR_NEG * tmax, pan0);
        if (!ok && tid == 0) ws.info[4 * b + 3] = -1;
        return;
    }
    __shared__ int nfail, failed[64];
    auto failed_b = [&](int k) { return failed[k]; };
    if (RETRY) {   // the failed filters of this workgroup's share, found in one parallel pass
        if (tid == 0) nfail = 0;
        __syncthreads();
        for (int i = tid; blockIdx.x + (size_t)i * gridDim.x < (size_t)st.B; i += blockDim.x) {
            const int b = blockIdx.x + i * gridDim.x;
            if (ws.afail[b]) {
                const int k = atomicAdd(&nfail, 1);
                if (k < 64) failed[k] = b;
            }
        }
        __syncthreads();
        const int nf = nfail;
        for (int k = 0; k < nf; ++k) {
            // (more than 64 failures in one share: the rest are walked by scanning again)
            const int b = k < 64 ? failed[k] : -1;
            if (b < 0) break;
            const int C = 6 * st.ncams[b];
            const double floor = pcc_pivot_floor(st.P + (size_t)b * st.Dmax * st.Dmax, st.Dmax, C, red);
            bool ok = false;
            for (int att = 1; att < 3 && !ok; ++att) {
                const double shift = (att == 1 ? 1e-8 : 1e-6) * (floor / KALMAN_PIVOT_FLOOR);
                ok = mk_factor<T, NW, NBR, 0>(st, ws, b, shift, floor, -PIVOT_FLOOR_NEG * floor, pan0);
            }
            if (tid == 0) ws.afail[b] = ok ? 0 : 1;   // read by stage C
        }
        if (nf <= 64) return;
        __syncthreads();
    }
    for (int b = blockIdx.x; b < st.B; b += gridDim.x) {
        if (RETRY && ws.afail[b] == 0) continue;   // uniform
        if (RETRY) {   // the first 64 of the share were retried above: not again
            bool done = false;
            for (int k = 0; k < 64; ++k) done |= failed_b(k) == b;
            if (done) continue;   // uniform
        }
        const int C = 6 * st.ncams[b];
        const double floor = pcc_pivot_floor(st.P + (size_t)b * st.Dmax * st.Dmax, st.Dmax, C, red);
        bool ok = false;
        for (int att = RETRY ? 1 : 0; att < (RETRY ? 3 : 1) && !ok; ++att) {
            const double shift = att == 0 ? 0.0 : (att == 1 ? 1e-8 : 1e-6) * (floor / KALMAN_PIVOT_FLOOR);
            ok = mk_factor<T, NW, NBR, 0>(st, ws, b, shift, floor, -PIVOT_FLOOR_NEG * floor, pan0);
        }
        if (tid == 0) ws.afail[b] = ok ? 0 : 1;   // read by stage C
    }
}

// ===========================================================================
// Host side
// ===========================================================================
struct RcholCfg { int nt, tpl; };

static bool pick_rchol(int tiles, RcholCfg& c) {
    if (tiles <= 256 * 4) { c = {256, 4}; return true; }
    if (tiles <= 256 * 6) { c = {256, 6}; return true; }
    if (tiles <= 512 * 4) { c = {512, 4}; return true; }
    return false;
}

template <typename T, int NT, int TPL>
static void launch_a_cfg(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws, size_t lds) {
    hipLaunchKernelGGL((k_kal_a<T, NT, TPL>), dim3(st.B), dim3(NT), lds, s, st, ws);
    // near-singular P_cc: the shifted retries (only failed filters do work)
    hipLaunchKernelGGL((k_kal_a<T, NT, TPL, true>), dim3(st.B), dim3(NT), lds, s, st, ws);
}

// Host side of the blocked global-memory factorisation (large windows).
template <int STAGE, typename T>
static void launch_gchol(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws) {
    const int Cmax = ws.Cmax;
    const int nrow = STAGE == 0 ? Cmax + 21 : 2 * Cmax + 22, ncol = STAGE == 0 ? Cmax + 21 : Cmax;
    const int ld_chunks = (nrow * ncol + 256 * 64 - 1) / (256 * 64);
    if (STAGE == 0) hipLaunchKernelGGL(k_gchol_a_load<T>, dim3(ld_chunks, st.B), dim3(256), 0, s, st, ws);
    for (int k = 0; k < Cmax; k += GNB) {
        hipLaunchKernelGGL((k_gchol_diag<STAGE, T>), dim3(st.B), dim3(64), 0, s, st, ws, k);
        // grids for the rows / columns below / right of the panel: a filter's last panel
        // may hold fewer than GNB pivots (nb = min(GNB, C_b - k), C_b <= Cmax), so size
        // them for nb >= 1; blocks past a filter's matrix exit at once
        const int rows = nrow - k - 1;
        if (rows > 0)
            hipLaunchKernelGGL((k_gchol_trsm<STAGE, T>), dim3((rows + GT - 1) / GT, st.B), dim3(256), 0, s, st, ws, k);
        const int ti = (rows + GT - 1) / GT, tj = (ncol - k - 1 + GT - 1) / GT;
        if (rows > 0 && tj > 0)
            hipLaunchKernelGGL((k_gchol_update<STAGE, T>), dim3(tj, ti, st.B), dim3(256), 0, s, st, ws, k);
    }
    if (STAGE == 0) hipLaunchKernelGGL(k_gchol_a_store<T>, dim3(ld_chunks, st.B), dim3(256), 0, s, st, ws);
}

// Register-tile stages A / C1 / C2 and E1 up to 32 cams (C <= 192); larger
// windows run A and C as blocked global-memory Choleskys.
bool kalman_chol_supported(int Cmax) { return ((Cmax + 15) & ~15) <= 16 * 12; }

template <typename T, int NW, int TPW>
static void launch_e1(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const UpdWs<T>& ws, size_t lds) {
    lds_limit((const void*)k_kal_e1<T, NW, TPW>, 160 * 1024);
    hipLaunchKernelGGL((k_kal_e1<T, NW, TPW>), dim3(st.B), dim3(64 * NW), lds, s, st, prm, ws);
}

template <typename T, int NT, int TPL>
static void launch_c1(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws, size_t lds) {
    hipLaunchKernelGGL((k_kal_c1<T, NT, TPL>), dim3(st.B), dim3(NT), lds, s, st, ws);
}
template <typename T, int NW, int CT, int NTM>
static void launch_c2(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws) {
    // two staging buffers; the first also holds the diagonal-block scratch
    constexpr int IMG = 16 * NTM * C2S > NW * 272 ? 16 * NTM * C2S : NW * 272;
    const size_t lds = (NTM * 256 + 16 * NTM * C2S + IMG) * sizeof(double);
    lds_limit((const void*)k_kal_c2<T, NW, CT, NTM>, 160 * 1024);
    hipLaunchKernelGGL((k_kal_c2<T, NW, CT, NTM>), dim3(st.B), dim3(64 * NW), lds, s, st, ws);
}

template <typename T, int NW, int NTM>
static void launch_b(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const UpdWs<T>& ws, size_t lds) {
    lds_limit((const void*)k_kal_b<T, NW, NTM>, 160 * 1024);
    hipLaunchKernelGGL((k_kal_b<T, NW, NTM>), dim3(st.B), dim3(64 * NW), lds, s, st, prm, ws);
}

// k_kal_mchol launches: NBR = block rows (exact for the bench window, 12 / 13),
// four waves per filter (8 / 16 measured slower, §5.7)
template <typename T, int STAGE, int NBR>
static void launch_mk_nbr(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws) {
    constexpr int NW = 4;
    const size_t lds = mk_lds_doubles(NBR) * sizeof(double);
    hipLaunchKernelGGL((k_kal_mchol<T, NW, NBR, STAGE>), dim3(st.B), dim3(64 * NW), lds, s, st, ws);
    // stage A near-singular P_cc: shifted retries of the failed filters only
    // (64 workgroups walk the filter list; none do any work on a healthy batch)
    if constexpr (STAGE == 0)
        hipLaunchKernelGGL((k_kal_mchol<T, NW, NBR, STAGE, true>), dim3(st.B < 64 ? st.B : 64), dim3(64 * NW), lds, s,
                           st, ws);
}
template <typename T, int STAGE>
static void launch_mk(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws, int nbr) {
    // (smaller windows round up: their extra block rows are identity padding)
    if (nbr <= 8) launch_mk_nbr<T, STAGE, 8>(s, st, ws);
    else if (nbr <= 12) launch_mk_nbr<T, STAGE, 12>(s, st, ws);
    else if (nbr <= 13) launch_mk_nbr<T, STAGE, 13>(s, st, ws);
    else launch_mk_nbr<T, STAGE, 14>(s, st, ws);
}

// Batches large enough to fill the chip run stages A / C1 on the matrix cores
// (throughput: two filters per CU, VALU-light); a handful of filters (the
// drop-in per-frame path, B = 1) keeps the register tiles, whose 4-pivot
// steps have the shorter latency (B = 1, 20 cams, fp64: A 57 vs 68 us).
constexpr int MK_MIN_B = 64;
// MSCKF_KALMAN_CHOL=mfma / tiles (environment, read per launch) forces one
// path -- the parity tests run both on the same inputs.
template <typename T> static bool use_mk(const DevState<T>& st) {
    if (const char* e = getenv("MSCKF_KALMAN_CHOL")) {
        if (e[0] == 'm') return true;
        if (e[0] == 't') return false;
    }
    return st.B >= MK_MIN_B;
}

template <typename T>
void launch_kalman_a_reg(hipStream_t s, const DevState<T>& st, const UpdWs<T>& ws, KernelTimer* kt) {
    const int Cp = (ws.Cmax + 3) & ~3;
    if (use_mk(st)) {
        kt->begin(s, "kalman_a");
        launch_mk<T, 0>(s, st, ws, (Cp + KW + 15) / 16);
        kt->end(s);
        return;
    }
    const int nrow = (Cp + KW) / 4;   // stage A, 4x4 register tiles
    RcholCfg c;
    pick_rchol(nrow * (nrow + 1) / 2, c);
    const size_t lds = rchol_lds_doubles(nrow) * sizeof(double);
    kt->begin(s, "kalman_a");
    if (c.nt == 256 && c.tpl == 4) launch_a_cfg<T, 256, 4>(s, st, ws, lds);
    else if (c.nt == 256) launch_a_cfg<T, 256, 6>(s, st, ws, lds);
    else launch_a_cfg<T, 512, 4>(s, st, ws, lds);
    kt->end(s);
}

template <typename T>
void launch_kalman_chol(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const UpdWs<T>& ws,
                        KernelTimer* kt) {
    const int Cmax = ws.Cmax;
    const bool reg = kalman_chol_supported(Cmax);   // else large window: global-memory stages A and C
    const int Cq = (Cmax + 15) & ~15;
    if (!reg) {   // (register-tile stage A: launch_kalman_a_reg, on the side stream)
        kt->begin(s, "kalman_a");
        launch_gchol<0, T>(s, st, ws);
        kt->end(s);
    }
    kt->begin(s, "kalman_b");
    if (Cq <= 16 * 8) {
        launch_b<T, 8, 8>(s, st, prm, ws, (4 * 16 * (size_t)(Cq + 17) + 32) * sizeof(double));
    } else if (Cq <= 16 * 12) {
        launch_b<T, 16, 12>(s, st, prm, ws, (4 * 16 * (size_t)(Cq + 17) + 32) * sizeof(double));
    } else {   // large windows: 64 x 64 output tiles, one workgroup each
        const int tiles = (Cmax + GT - 1) / GT;
        hipLaunchKernelGGL(k_kal_b1<T>, dim3(tiles, tiles, st.B), dim3(256), 0, s, st, ws);
        hipLaunchKernelGGL(k_kal_b2<T>, dim3((Cmax + 1 + GT - 1) / GT, tiles, st.B), dim3(256), 0, s, st, prm, ws);
    }
    kt->end(s);
    kt->begin(s, "kalman_c");
    if (reg) {   // C1: Cholesky of T (register tiles); C2: MFMA forward substitution of the extra rows
        if (use_mk(st)) {
            launch_mk<T, 1>(s, st, ws, (Cmax + 15) / 16);
        } else {
            const int nTc = ((Cmax + 3) & ~3) / 4;
            RcholCfg c;
            pick_rchol(nTc * (nTc + 1) / 2, c);
            const size_t lds = rchol_lds_doubles(nTc) * sizeof(double);
            if (c.nt == 256 && c.tpl == 4) launch_c1<T, 256, 4>(s, st, ws, lds);
            else if (c.nt == 256) launch_c1<T, 256, 6>(s, st, ws, lds);
            else launch_c1<T, 512, 4>(s, st, ws, lds);
        }
        if (Cq <= 16 * 8) launch_c2<T, 7, 2, 8>(s, st, ws);
        else launch_c2<T, 13, 1, 12>(s, st, ws);
    } else {
        launch_gchol<1, T>(s, st, ws);
    }
    kt->end(s);
    kt->begin(s, "kalman_e");
    const int nTe = (st.Dmax + 15) / 16, tilesE = nTe * (nTe + 1) / 2;
    const size_t ldsE = (2 * 16 * 16 * (size_t)nTe + 32) * sizeof(double);
    if (reg && tilesE <= 16 * 6) {
        launch_e1<T, 16, 6>(s, st, prm, ws, ldsE);
    } else if (reg) {
        launch_e1<T, 8, 16>(s, st, prm, ws, ldsE);
    } else {   // large windows: one 64 x 64 tile per workgroup
        const int dt = (st.Dmax + 127) / 128, dt1 = (st.Dmax + 1 + 127) / 128;
        hipLaunchKernelGGL(k_kal_e<T>, dim3(dt1, dt, st.B), dim3(256), 0, s, st, prm, ws);
    }
    kt->end(s);
}

template void launch_kalman_a_reg<float>(hipStream_t, const DevState<float>&, const UpdWs<float>&, KernelTimer*);
template void launch_kalman_a_reg<double>(hipStream_t, const DevState<double>&, const UpdWs<double>&, KernelTimer*);
template void launch_kalman_chol<float>(hipStream_t, const DevState<float>&, const Params<float>&,
                                        const UpdWs<float>&, KernelTimer*);
template void launch_kalman_chol<double>(hipStream_t, const DevState<double>&, const Params<double>&,
                                         const UpdWs<double>&, KernelTimer*);

}  // namespace msckf
