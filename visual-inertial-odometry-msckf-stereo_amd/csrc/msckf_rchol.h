// msckf_rchol.h -- register-tile blocked partial Cholesky shared by the
// Kalman stages (msckf_kalman.hip) and the large-track gating kernel.
#pragma once
#include "msckf_common.h"

namespace msckf {

// ===========================================================================
// Register-tile partial Cholesky.  The lower tiles (ti, tl), tl < ncol,
// tl <= ti < nrow, enumerated column-major; tile t lives in thread t % NT,
// slot t / NT.  Eliminates tile columns 0..nelim-1 (4 pivots per step):
//   1. owners of the step's tile column dump it to LDS (double-buffered)
//      -- the diagonal tile's owner factors it (L_d and the reciprocal
//      diagonal to LDS: one fp64 sqrt / division chain per step, not one per
//      thread)
//   2. every thread reads L_d and transforms panel rows (one row per thread):
//      W = A_panel L_d^-T -> LDS + panel()
//   3. every tile right of the panel takes A -= W_i W_l^T from registers
// Two barriers per step.  Tiles in columns >= nelim end as the Schur
// complement and are handed to trail().  In the LDS column buffer each 4-row
// block takes RB = 18 doubles (144 B): consecutive lanes read consecutive
// blocks with ds_read_b128, and a 144-B stride spreads a 16-lane group over
// all 64 banks (a 128-B stride would put it on two).
// load(i, j) must be symmetric on the square part (diagonal tiles read both
// triangles).
// floor > 0: a pivot in [-PIVOT_FLOOR_NEG x floor, floor) is replaced by
// floor instead of failing -- the factorisation is then the exact one of
// A + E with E >= 0 diagonal, non-zero only at those pivots (a covariance that
// the reference's non-Joseph update, msckf.py:598-604, has left indefinite at
// rounding level; the reference never factors it, so it does not fail there
// either).  A NaN pivot or one further below zero is a corrupted covariance,
// not rounding: it still fails the factorisation.
// ===========================================================================
constexpr double PIVOT_FLOOR_NEG = 1e4;   // x floor: the deepest negative pivot still floored
// lo: the lowest pivot still floored (default -PIVOT_FLOOR_NEG x floor); NaN is never floored
__device__ __forceinline__ double pivot_floored(double x, double floor, double lo) {
    return (floor > 0.0 && x < floor && x >= lo) ? floor : x;
}
__device__ __forceinline__ double pivot_floored(double x, double floor) {
    return pivot_floored(x, floor, -PIVOT_FLOOR_NEG * floor);
}
constexpr int RB = 18;   // doubles per 4-row block of the LDS column buffer
// 1 / sqrt(x): the hardware reciprocal square root plus one Newton step (about
// 1 ulp); the pivot is x * rchol_rsq(x).  No square root or division on the
// diagonal factor's dependent chain, which every thread of the workgroup waits
// for once per step.  x <= 0 or NaN gives NaN or a zero pivot: the step fails.
__device__ __forceinline__ double rchol_rsq(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    return r * fma(-0.5 * x * r, r, 1.5);
}

// TILE_LOAD: load(i0, j0, tile) fills a whole 4x4 tile (rows i0.., cols j0..)
// instead of being called per element (lets a loader share operands).
template <int NT, int TPL, class Load, class Panel, class Trail, bool TILE_LOAD = false>
__device__ __forceinline__ bool rchol_core(int nrow, int ncol, int nelim, double* lds, Load load, Panel panel,
                                           Trail trail, double floor = 0.0, double floor_lo = 1.0) {
    // floor_lo > 0 (default): pivots down to -PIVOT_FLOOR_NEG x floor are floored
    const double lo = floor_lo > 0.0 ? -PIVOT_FLOOR_NEG * floor : floor_lo;
    auto fl = [floor, lo](double x) { return pivot_floored(x, floor, lo); };
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
        if constexpr (TILE_LOAD) {
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) a[s][x][y] = 0.0;
            if (ROK(s)) load(i0, j0, a[s]);
        } else {
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) a[s][x][y] = ROK(s) ? load(i0 + x, j0 + y) : 0.0;
        }
    }
    bool fail = false;
    double* fac = lds + 2 * RB * nrow;   // [2][16]: the step's diagonal factor (double-buffered)
    for (int tj = 0; tj < nelim; ++tj) {
        double* buf = lds + (tj & 1) * RB * nrow;   // [nrow][RB]: rows 4 t + x at RB t + 4 x
        double* fj = fac + 16 * (tj & 1);
#pragma unroll
        for (int s = 0; s < TPL; ++s) {
            if (!ROK(s) || RTL(s) != tj) continue;
            double* dst = buf + RB * RTI(s);
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) dst[4 * x + y] = a[s][x][y];
            if (RTI(s) == tj) {   // the diagonal tile's owner factors it once for everyone
                const double p0 = fl(a[s][0][0]), i00 = rchol_rsq(p0), l00 = p0 * i00;
                const double l10 = a[s][1][0] * i00, l20 = a[s][2][0] * i00, l30 = a[s][3][0] * i00;
                const double p1 = fl(a[s][1][1] - l10 * l10), i11 = rchol_rsq(p1), l11 = p1 * i11;
                const double l21 = (a[s][2][1] - l20 * l10) * i11, l31 = (a[s][3][1] - l30 * l10) * i11;
                const double p2 = fl(a[s][2][2] - l20 * l20 - l21 * l21), i22 = rchol_rsq(p2), l22 = p2 * i22;
                const double l32 = (a[s][3][2] - l30 * l20 - l31 * l21) * i22;
                const double p3 = fl(a[s][3][3] - l30 * l30 - l31 * l31 - l32 * l32), i33 = rchol_rsq(p3), l33 = p3 * i33;
                fj[0] = l00; fj[1] = l10; fj[2] = l20; fj[3] = l30;
                fj[4] = l11; fj[5] = l21; fj[6] = l31; fj[7] = l22;
                fj[8] = l32; fj[9] = l33; fj[10] = i00; fj[11] = i11;
                fj[12] = i22; fj[13] = i33;
            }
        }
        LDS_BARRIER();
        const double l00 = fj[0], l10 = fj[1], l20 = fj[2], l30 = fj[3];
        const double l11 = fj[4], l21 = fj[5], l31 = fj[6], l22 = fj[7];
        const double l32 = fj[8], l33 = fj[9], i00 = fj[10], i11 = fj[11];
        const double i22 = fj[12], i33 = fj[13];
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
            double w[4][4];
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int c = 0; c < 4; ++c) w[x][c] = rl[4 * x + c];
#pragma unroll
            for (int x = 0; x < 4; ++x) {   // one row of u at a time (register budget)
                double u[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) u[c] = ri[4 * x + c];
#pragma unroll
                for (int y = 0; y < 4; ++y)
                    a[s][x][y] -= u[0] * w[y][0] + u[1] * w[y][1] + u[2] * w[y][2] + u[3] * w[y][3];
                if (TPL > 4) asm volatile("" ::: "memory");
            }
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

__host__ __device__ constexpr int rchol_lds_doubles(int nrow) { return 2 * RB * nrow + 32; }

}  // namespace msckf
