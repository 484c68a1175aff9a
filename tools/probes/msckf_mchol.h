// msckf_mchol.h -- EXPERIMENT (not in the library; tools/probes/mchol_test.hip
// drives it): blocked partial Cholesky of a symmetric fp64 matrix on the
// matrix cores (v_mfma_f64_16x16x4f64), one workgroup per filter, tried as a
// replacement for the Kalman stages A and C1 (msckf_kalman.hip, msckf_rchol.h).
// Measured on MI355X, 2048 filters: C1-sized (192 x 192) 0.79 ms and A-sized
// 0.92 ms against 0.60 / 1.0 ms for the 4x4 register-tile kernels -- the
// serial 16 x 16 diagonal factor+inverse on one wave (~15k cycles per step)
// dominates, and the 16-wave workgroup holding the matrix in VGPRs leaves one
// workgroup per CU to hide it.  Kept for the record.
//
// The lower 16 x 16 tiles (ti >= tj, tj < ncol) of an nrow x ncol tile grid
// live in VGPRs as MFMA accumulators (f64 result layout: lane l holds rows
// (l >> 4) + 4 q, q = 0..3, of column l & 15), tile t in wave t % NW, slot
// t / NW.  Tile column k is eliminated in one step of 16 pivots:
//   1. the owners of column k dump its tiles to an LDS panel (row-major,
//      double-buffered by step parity);                          -- barrier
//   2. wave 0 factors the diagonal tile and inverts L_kk into LDS, in
//      registers (lane m holds column m; pivot columns by v_readlane);
//                                                                -- barrier
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
#include "../../visual-inertial-odometry-msckf-stereo_amd/csrc/msckf_common.h"

namespace msckf {

constexpr int MC_PS = 17;   // panel row stride (doubles): odd, spreads a 16-row operand read over the banks

__host__ __device__ constexpr int mchol_lds_doubles(int nrow) { return 2 * 16 * nrow * MC_PS + 256 + 16; }

// Step 2 of mchol_core (one wave): L_kk = chol(D) written over D's lower
// triangle and L_kk^-1 into LI (LI[c * 16 + i] = (L_kk^-1)[i][c]).  Lane m
// (lanes 16..63 repeat lanes 0..15) holds column m of the tile in registers
// (a[r] = A[r][m]); pivot column entries reach every lane by v_readlane, so
// the 16 pivots are a chain of register FMAs with no LDS round trip in it:
//   pivot j:  a[r] -= A[r][j] A[j][m] / d_j   (lanes m > j, rows r > j),
// A[r][j] read from lane r's a[j] (the rows above m are kept for that).
// Column m is scaled by 1 / sqrt(d_m) at the end, then inverted in place.
// Returns true if a pivot was not positive (after the floor).  Not inlined:
// the 16-register column and the unrolled broadcasts get a register
// allocation of their own instead of competing with the caller's
// accumulator tiles (inlined, the scheduler hoists the broadcasts and spills).
__device__ __forceinline__ double rsqrt_f64(double d) {   // 1 / sqrt(d), two Newton steps on v_rsq_f64
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

typedef __attribute__((address_space(3))) double lds_f64;   // ds_* accesses through the call

__device__ __noinline__ bool mchol_diag16(lds_f64* D, lds_f64* LI, double floor) {
    // lanes 16..63 repeat lanes 0..15 (column m & 15) and store nothing
    const int lane = threadIdx.x & 63, m = lane & 15;
    double a[16];
    double ilv = 1.0, dv = 1.0;   // lane j: 1 / sqrt(d_j) and d_j
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = D[r * MC_PS + m];
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        double d = lane_bcast(a[j], j);
        if (floor > 0.0 && !(d >= floor)) d = floor;
        bad = bad || !(d > 0.0);
        const double il = rsqrt_f64(d);
        ilv = m == j ? il : ilv;
        dv = m == j ? d : dv;
        const double t = m > j ? a[j] * (il * il) : 0.0;   // A[j][m] / d_j
#pragma unroll
        for (int r = j + 1; r < 16; ++r) a[r] = fma(-lane_bcast(a[j], r), t, a[r]);
    }
    // column m of L_kk: rows below m scaled, sqrt(d_m) = d_m / sqrt(d_m) on the
    // diagonal, zeros above (they start the substitution below)
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = r > m ? a[r] * ilv : (r == m ? dv * ilv : 0.0);
    if (lane < 16) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (r >= m) D[r * MC_PS + m] = a[r];
    }
    // L_kk^-1 by forward substitution, column m in place: x_i lands in a[i]
    // after the L[i][p] (lane p's a[i], p < i) have been broadcast; x_i = 0
    // for i < m falls out of the zeros above
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        double sacc = m == i ? 1.0 : 0.0;
#pragma unroll
        for (int p = 0; p < i; ++p) sacc = fma(-lane_bcast(a[i], p), a[p], sacc);
        a[i] = sacc * lane_bcast(ilv, i);
    }
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) LI[m * 16 + i] = a[i];
    }
    return bad;
}

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
        // 2. wave 0: L_kk and L_kk^-1 in registers, lane m < 16 holding column m
        //    of the tile (a[r] = A[r][m]); the column entries every pivot needs
        //    arrive by v_readlane (SGPRs), so the 16 pivots are a chain of
        //    register FMAs with no LDS round trip in it.
#ifndef MCHOL_TIMING_SKIP   // (tools/probes/mchol_test.hip: bit 0 diag, 1 panel, 2 trailing update)
#define MCHOL_TIMING_SKIP 0
#endif
        if (wv == 0 && !(MCHOL_TIMING_SKIP & 1)) {
            double* D = pan + 16 * k * MC_PS;
            if (mchol_diag16((lds_f64*)D, (lds_f64*)LI, floor) && lane == 0) flag[0] = 1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = lane + 64 * q, r = e >> 4, c = e & 15;
                if (c <= r) out(16 * k + r, 16 * k + c, D[r * MC_PS + c]);
            }
        }
        __syncthreads();
        // 3. panel W_i = X_ik L_kk^-T for the sub-diagonal tiles of column k
#pragma unroll
        for (int s = 0; s < TPW; ++s) {
            if (tj[s] != k || ti[s] == k || (MCHOL_TIMING_SKIP & 2)) continue;
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
            if (ti[s] < 0 || tj[s] <= k || (MCHOL_TIMING_SKIP & 4)) continue;   // (empty slots: ti = tj = -1)
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
