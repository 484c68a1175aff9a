// msckf_mchol.h -- workgroup (partial) Cholesky on fp64 MFMA tiles, used by
// the Kalman stages A and C1 (msckf_kalman.hip) when the matrix has at most
// 13 16-row blocks (n <= 208).
//
// The lower block triangle lives in the C/D layout of v_mfma_f64_16x16x4_f64
// (lane l: column 16 cb + (l & 15), rows 16 rb + (l >> 4) + 4 r, r = 0..3);
// wave w of the eight owns block rows w and w + 8.  Per 4-pivot step:
//   1. the owners of the step's four columns dump them to a double-buffered
//      row-major LDS panel; one barrier;
//   2. every lane factors the 4x4 diagonal (uniform) and picks its row of
//      L_d^-1 (its pivot column c = l >> 4);
//   3. every lane forms W[r][c] = (x L_d^-T)[c] for row r = 16 rb + (l & 15) of
//      every block row (the B operands; the owning wave also stores them as
//      L entries) and the A operands -W of its own rows;
//   4. every block right of the panel takes A -= W W^T as one MFMA (a block
//      column's own update is skipped after its last step).
// One barrier per step; fp64 MFMA runs at the fp64 vector rate on MI355X, so
// the gain over the 4x4 VALU tiles of rchol_core is in the instruction count
// (one MFMA per 16x16 block and step instead of 16 FMA-chains per 4x4 tile).
#pragma once
#include "msckf_common.h"

namespace msckf {

typedef double mc_v4d __attribute__((ext_vector_type(4)));
constexpr int MC_NW = 8;     // waves per workgroup
constexpr int MC_NBK = 13;   // block rows at most
__host__ __device__ constexpr int mchol_lds_doubles() { return 2 * 16 * MC_NBK * 4; }
__host__ __device__ constexpr bool mchol_fits(int n) { return n >= 1 && (n + 15) / 16 <= MC_NBK; }

// load(i, j): symmetric entry (identity outside the matrix);
// put(r, c, v): factor entry L[r][c], r >= c (the 4x4 diagonal tiles also get
//               their zero upper entries), for pivot columns c < 4 nelim;
// trail(i, j, v): Schur complement entries i >= j >= 4 nelim.
template <class Load, class Put, class Trail>
__device__ __forceinline__ bool mchol_core(int n, int nelim, double* lds, Load load, Put put, Trail trail) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nbk = (n + 15) >> 4;
    const int col_l = lane & 15, rg = lane >> 4;
    const int RB0 = w, RB1 = w + 8;
    mc_v4d a0[8], a1[MC_NBK];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        a0[c] = mc_v4d{0.0, 0.0, 0.0, 0.0};
        if (c <= RB0 && RB0 < nbk)
#pragma unroll
            for (int r = 0; r < 4; ++r) a0[c][r] = load(16 * RB0 + rg + 4 * r, 16 * c + col_l);
    }
#pragma unroll
    for (int c = 0; c < MC_NBK; ++c) {
        a1[c] = mc_v4d{0.0, 0.0, 0.0, 0.0};
        if (c <= RB1 && RB1 < nbk)
#pragma unroll
            for (int r = 0; r < 4; ++r) a1[c][r] = load(16 * RB1 + rg + 4 * r, 16 * c + col_l);
    }
    bool fail = false;
#pragma unroll
    for (int KB = 0; KB < MC_NBK; ++KB) {
        if (4 * KB >= nelim || fail) break;
        for (int sc = 0; sc < 4; ++sc) {
            const int j = 4 * KB + sc;
            if (j >= nelim) break;
            const int p0 = 4 * j;
            double* pb = lds + (j & 1) * (16 * MC_NBK * 4);
            // 1. dump the step's four columns of the owned blocks (RB, KB)
            if ((col_l >> 2) == sc) {
                const int cc = col_l & 3;
                if (KB < 8 && RB0 >= KB && RB0 < nbk) {
                    const mc_v4d v = a0[KB < 8 ? KB : 0];
#pragma unroll
                    for (int r = 0; r < 4; ++r) pb[4 * (16 * RB0 + rg + 4 * r) + cc] = v[r];
                }
                if (RB1 >= KB && RB1 < nbk) {
                    const mc_v4d v = a1[KB];
#pragma unroll
                    for (int r = 0; r < 4; ++r) pb[4 * (16 * RB1 + rg + 4 * r) + cc] = v[r];
                }
            }
            LDS_BARRIER();
            // 2. the 4x4 diagonal: L_d and the lane's row of L_d^-1
            const double* dt = pb + 4 * p0;
            const double l00 = sqrt(dt[0]), i00 = 1.0 / l00;
            const double l10 = dt[4] * i00, l20 = dt[8] * i00, l30 = dt[12] * i00;
            const double l11 = sqrt(dt[5] - l10 * l10), i11 = 1.0 / l11;
            const double l21 = (dt[9] - l20 * l10) * i11, l31 = (dt[13] - l30 * l10) * i11;
            const double l22 = sqrt(dt[10] - l20 * l20 - l21 * l21), i22 = 1.0 / l22;
            const double l32 = (dt[14] - l30 * l20 - l31 * l21) * i22;
            const double l33 = sqrt(dt[15] - l30 * l30 - l31 * l31 - l32 * l32), i33 = 1.0 / l33;
            if (!(l00 > 0.0) || !(l11 > 0.0) || !(l22 > 0.0) || !(l33 > 0.0)) { fail = true; break; }   // uniform
            const double v10 = -l10 * i00 * i11;
            const double v20 = (-l20 * i00 - l21 * v10) * i22, v21 = -l21 * i11 * i22;
            const double v30 = (-l30 * i00 - l31 * v10 - l32 * v20) * i33;
            const double v31 = (-l31 * i11 - l32 * v21) * i33, v32 = -l32 * i22 * i33;
            const double g0 = rg == 0 ? i00 : (rg == 1 ? v10 : (rg == 2 ? v20 : v30));
            const double g1 = rg == 0 ? 0.0 : (rg == 1 ? i11 : (rg == 2 ? v21 : v31));
            const double g2 = rg <= 1 ? 0.0 : (rg == 2 ? i22 : v32);
            const double g3 = rg == 3 ? i33 : 0.0;
            if (w == 0 && lane < 4) {   // the diagonal tile of L (zero upper entries)
                const double lrow[4][4] = {{l00, 0.0, 0.0, 0.0}, {l10, l11, 0.0, 0.0}, {l20, l21, l22, 0.0},
                                           {l30, l31, l32, l33}};
#pragma unroll
                for (int x = 0; x < 4; ++x)
                    if (lane == x)
#pragma unroll
                        for (int y = 0; y < 4; ++y) put(p0 + x, p0 + y, lrow[x][y]);
            }
            // 3. operands: W[r][c] of a block row (B), -W of the owned rows (A)
            auto wrow = [&](int RB) -> double {
                const double2 x01 = *reinterpret_cast<const double2*>(pb + 4 * (16 * RB + col_l));
                const double2 x23 = *reinterpret_cast<const double2*>(pb + 4 * (16 * RB + col_l) + 2);
                const double v = fma(x23.y, g3, fma(x23.x, g2, fma(x01.y, g1, x01.x * g0)));
                return (16 * RB + col_l <= p0 + 3 || RB >= nbk) ? 0.0 : v;
            };
            // the owning waves store their rows' W as L entries
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int RB = q == 0 ? RB0 : RB1;
                const int r = 16 * RB + col_l;
                if ((q == 0 ? KB < 8 : true) && RB >= KB && RB < nbk && r > p0 + 3 && r < n) put(r, p0 + rg, wrow(RB));
            }
            // 4. A -= W W^T on the owned blocks right of the panel (B operands
            //    formed per block column as needed: registers)
            if (KB < 8 && RB0 >= KB && RB0 < nbk) {
                const double av = -wrow(RB0);
#pragma unroll
                for (int c = KB; c < 8; ++c)
                    if (c <= RB0 && (c > KB || sc < 3)) a0[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, wrow(c), a0[c], 0, 0, 0);
            }
            if (RB1 >= KB && RB1 < nbk) {
                const double av = -wrow(RB1);
#pragma unroll
                for (int c = KB; c < MC_NBK; ++c)
                    if (c <= RB1 && (c > KB || sc < 3)) a1[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, wrow(c), a1[c], 0, 0, 0);
            }
        }
    }
    if (!fail) {
        const int e0 = 4 * nelim;
#pragma unroll
        for (int c = 0; c < 8; ++c)
            if (c <= RB0 && RB0 < nbk && 16 * RB0 + 15 >= e0 && 16 * c + 15 >= e0)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * RB0 + rg + 4 * r, jj = 16 * c + col_l;
                    if (i < n && jj >= e0 && i >= jj) trail(i, jj, a0[c][r]);
                }
#pragma unroll
        for (int c = 0; c < MC_NBK; ++c)
            if (c <= RB1 && RB1 < nbk && 16 * RB1 + 15 >= e0 && 16 * c + 15 >= e0)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = 16 * RB1 + rg + 4 * r, jj = 16 * c + col_l;
                    if (i < n && jj >= e0 && i >= jj) trail(i, jj, a1[c][r]);
                }
    }
    return !fail;
}

}  // namespace msckf
