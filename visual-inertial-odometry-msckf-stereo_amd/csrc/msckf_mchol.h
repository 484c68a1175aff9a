// msckf_mchol.h -- blocked partial Cholesky of a symmetric fp64 matrix on the
// matrix cores (v_mfma_f64_16x16x4f64), one workgroup per filter.  Shared by
// the Kalman stages A (P_cc with the IMU rows) and C1 (T), msckf_kalman.hip.
//
// The lower 16 x 16 tiles (ti >= tj, tj < ncol) of an nrow x ncol tile grid
// live in VGPRs as MFMA accumulators (f64 result layout: lane l holds rows
// (l >> 4) + 4 q, q = 0..3, of column l & 15), tile t in wave t % NW, slot
// t / NW.  Tile column k is eliminated in one step of 16 pivots:
//   1. the owners of column k dump its tiles to an LDS panel (row-major,
//      double-buffered by step parity);                          -- barrier
//   2. wave 0 factors the diagonal tile in the panel and inverts L_kk into
//      LDS (four elements per lane, right-looking sweeps);     -- barrier
//   3. the owners of the column's sub-diagonal tiles form W_i = X_ik L_kk^-T
//      (four MFMAs, B operand L_kk^-T from LDS) and write it over X_ik in the
//      panel;                                                    -- barrier
//   4. every tile right of the column takes A_ij -= W_i W_j^T (four MFMAs, both
//      operands read from the panel in the same lane pattern).
// 16 pivots per three barriers instead of 4 pivots per two (msckf_rchol.h),
// and the trailing update issues one MFMA per 16 x 16 x 4 block instead of
// 64 VALU FMAs per 4 x 4 register tile.
// out(i, j, v) receives every finished factor element (i >= j, j < 16 nelim);
// trail(i, j, v) every element of the tiles in columns >= nelim (the Schur
// complement), lower tiles only.  floor > 0: a pivot below floor (or NaN) is
// replaced by floor instead of failing (msckf_rchol.h, KALMAN_PIVOT_FLOOR).
#pragma once
#include "msckf_common.h"

namespace msckf {

constexpr int MC_PS = 17;   // panel row stride (doubles): odd, spreads a 16-row operand read over the banks

__host__ __device__ constexpr int mchol_lds_doubles(int nrow) { return 2 * 16 * nrow * MC_PS + 256 + 16; }

template <int NW, int TPW, class Load, class Out, class Trail>
__device__ __forceinline__ bool mchol_core(int nrow, int ncol, int nelim, double* lds, Load load, Out out,
                                           Trail trail, double floor) {
    typedef double v4d __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ntiles = ncol * nrow - ncol * (ncol - 1) / 2;
    int ti[TPW], tj[TPW];
#pragma unroll
    for (int s = 0; s < TPW; ++s) {
        const int t = wv + NW * s;
        const int tc = t < ntiles ? t : 0;
        const int c = colmajor_col(tc, nrow);
        const int r = c + (tc - (c * nrow - c * (c - 1) / 2));
        ti[s] = __builtin_amdgcn_readfirstlane(t < ntiles ? r : -1);
        tj[s] = __builtin_amdgcn_readfirstlane(t < ntiles ? c : -1);   // an empty slot matches no column
    }
    v4d acc[TPW];
#pragma unroll
    for (int s = 0; s < TPW; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q)
            acc[s][q] = ti[s] >= 0 ? load(16 * ti[s] + lr + 4 * q, 16 * tj[s] + lc) : 0.0;
    double* LI = lds + 2 * 16 * nrow * MC_PS;   // LI[c * 16 + i] = (L_kk^-1)[i][c] = (L_kk^-T)[c][i]
    int* flag = reinterpret_cast<int*>(LI + 256);
    if (tid == 0) flag[0] = 0;
    auto fl = [floor](double x) { return (floor > 0.0 && !(x >= floor)) ? floor : x; };
    for (int k = 0; k < nelim; ++k) {
        double* pan = lds + (k & 1) * 16 * nrow * MC_PS;
        // lane offsets, opaque per step: the tile addresses are formed where
        // they are used instead of being hoisted out of this loop (and spilled)
        int op = lc * MC_PS + lr;          // operand element (row lc, column lr) of a tile's panel rows
        int dp = lr * MC_PS + lc;          // result element (row lr, column lc)
        int olr = lr, olc = lc;            // for the output indices
        asm volatile("" : "+v"(op), "+v"(dp), "+v"(olr), "+v"(olc));
        // 1. dump tile column k
#pragma unroll
        for (int s = 0; s < TPW; ++s) {
            if (tj[s] != k) continue;   // uniform
            double* d = pan + 16 * ti[s] * MC_PS + dp;
#pragma unroll
            for (int q = 0; q < 4; ++q) d[4 * q * MC_PS] = acc[s][q];
        }
        __syncthreads();
        // 2. wave 0: L_kk in place in the panel (four elements (r, m) per lane,
        //    right-looking, every step's reads issued before its writes), then L_kk^-1
        if (wv == 0) {
            double* D = pan + 16 * k * MC_PS;
            bool bad = false;
#pragma unroll 1
            for (int j = 0; j < 16; ++j) {
                const double d = fl(D[j * MC_PS + j]);
                bad = bad || !(d > 0.0);
                const double l = sqrt(d), id = 1.0 / d, il = l * id;
                double nv[4];
                int at[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = lane + 64 * q, r = e >> 4, m = e & 15;
                    const double crj = D[r * MC_PS + j], cmj = D[m * MC_PS + j], cur = D[r * MC_PS + m];
                    at[q] = -1;
                    if (r >= m && m > j) { nv[q] = cur - crj * cmj * id; at[q] = r * MC_PS + m; }
                    else if (m == j && r > j) { nv[q] = crj * il; at[q] = r * MC_PS + m; }
                    else if (m == j && r == j) { nv[q] = l; at[q] = r * MC_PS + m; }
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (at[q] >= 0) D[at[q]] = nv[q];
            }
            // L_kk^-1 by the same right-looking sweep: element (r, c) of the
            // inverse accumulates e_r - sum_{p < r} L[r][p] Linv[p][c] and is
            // divided by L[r][r] when row r comes up (upper elements stay 0)
            double xa[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = lane + 64 * q, r = e >> 4, c = e & 15;
                xa[q] = r == c ? 1.0 : 0.0;
                if (c > r) LI[c * 16 + r] = 0.0;
            }
#pragma unroll 1
            for (int j = 0; j < 16; ++j) {
                const double ljj = D[j * MC_PS + j];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = lane + 64 * q, r = e >> 4, c = e & 15;
                    if (r == j && c <= j) {
                        xa[q] /= ljj;
                        LI[c * 16 + j] = xa[q];
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int e = lane + 64 * q, r = e >> 4, c = e & 15;
                    if (r > j && c <= j) xa[q] -= D[r * MC_PS + j] * LI[c * 16 + j];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = lane + 64 * q, r = e >> 4, m = e & 15;
                if (m <= r) out(16 * k + r, 16 * k + m, D[r * MC_PS + m]);
            }
            if (bad && lane == 0) flag[0] = 1;
        }
        __syncthreads();
        // 3. panel W_i = X_ik L_kk^-T for the sub-diagonal tiles of column k
#pragma unroll
        for (int s = 0; s < TPW; ++s) {
            if (tj[s] != k || ti[s] == k) continue;
            double* rows = pan + 16 * ti[s] * MC_PS;
            v4d w = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kc = 0; kc < 4; ++kc)
                w = __builtin_amdgcn_mfma_f64_16x16x4f64(rows[op + 4 * kc], LI[(4 * kc + lr) * 16 + lc], w,
                                                         0, 0, 0);   // B[k][n] = (L_kk^-T)[k][n] = (L_kk^-1)[n][k]
            // X_ik's rows are this wave's alone: its reads above precede these writes
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                rows[dp + 4 * q * MC_PS] = w[q];
                out(16 * ti[s] + olr + 4 * q, 16 * k + olc, w[q]);
            }
        }
        __syncthreads();
        // 4. trailing update of the tiles right of column k
#pragma unroll
        for (int s = 0; s < TPW; ++s) {
            if (ti[s] < 0 || tj[s] <= k) continue;   // (empty slots: ti = tj = -1)
            const double* ri = pan + 16 * ti[s] * MC_PS + op;
            const double* rj = pan + 16 * tj[s] * MC_PS + op;
#pragma unroll
            for (int kc = 0; kc < 4; ++kc)
                acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(-ri[4 * kc], rj[4 * kc], acc[s], 0, 0, 0);
        }
    }
    __syncthreads();
    const bool ok = flag[0] == 0;
    if (ok) {
#pragma unroll
        for (int s = 0; s < TPW; ++s) {
            if (ti[s] < 0 || tj[s] < nelim) continue;
#pragma unroll
            for (int q = 0; q < 4; ++q) trail(16 * ti[s] + lr + 4 * q, 16 * tj[s] + lc, acc[s][q]);
        }
    }
    return ok;
}

}  // namespace msckf
