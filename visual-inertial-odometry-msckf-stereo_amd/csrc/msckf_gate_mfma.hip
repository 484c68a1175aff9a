// msckf_gate_mfma.hip -- chi^2 gating of the fp32 contexts (msckf.py:606-614)
// on fp32 MFMA tiles: one wavefront per feature (M <= 41), and for the large
// tracks (41 < M <= 82) a 2- to 8-wave workgroup per feature (k_gate_mfma_wt).
//
// Same mathematics as k_gate_wave (msckf_kernels.hip): gamma = r0^T S^-1 r0
// is read off an LDL^T elimination of the rank-3 reduced saddle-point matrix
//     [[Y~, H_f~, r~], [H_f~^T, 0, 0], [r~^T, 0, 0]],   Y~ = Ht P Ht^T + s2 I,
// (3M range rows, the null rows adding |r_n|^2 / s2), with no projection
// formed.  What changes is the layout of the elimination:
//   * the matrix is held as 16x16 blocks in the C/D layout of
//     v_mfma_f32_16x16x4_f32 (lane l: column 16 cb + (l & 15), rows
//     16 rb + 4 (l >> 4) + i, i = 0..3), lower block triangle only;
//   * rows: the 3M range rows, unit padding pivots, and the four B rows
//     [H_f~^T ; r~^T] as the last four rows of the last block;
//   * each 4-pivot step, the owners of the four pivot columns dump them to a
//     row-major LDS panel, every lane factors the 4x4 diagonal (one reciprocal
//     per pivot), forms its MFMA operands (lane l: row 16 rb + (l & 15), pivot
//     column l >> 4 of W = A L_d^-T and of -W D^-1; rows of finished pivots
//     zeroed), and the whole trailing lower block triangle takes the rank-4
//     update as one v_mfma_f32_16x16x4_f32 per block;
//   * the Schur complement left in the B rows' 4x4 gives gamma as before.
// One MFMA replaces the 16 packed FMAs + operand fetches a 4x4 register tile
// needed, and no lanes idle on finished tiles of a triangular tile order.
// fp32 MFMA is exact f32 (an fmaf chain) on gfx950.
#include "msckf_common.h"
#include "msckf_launch.h"

#include <stdlib.h>

namespace msckf {

// Phase timing of the one-wave kernel (probe builds only, `make probe`:
// -DMSCKF_GATE_PROBE; tools/probes/gate_phases.py reads it): per class NB and
// scalar type, wave-cycle sums (s_memtime) of record fetch, Y pair blocks,
// assembly, elimination, finish, and the wave count.
#ifdef MSCKF_GATE_PROBE
__device__ unsigned long long g_gate_probe[2][9][8];   // [f32, f64][NB][phase]
#define GPROBE_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define GPROBE_ADDK(kind, NB, ph, dt) \
    do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_gate_probe[kind][NB][ph], (unsigned long long)(dt)); } while (0)
#define GPROBE_ADD(ts, NB, ph, dt) GPROBE_ADDK((ts) == 8, NB, ph, dt)
#else
#define GPROBE_T(v) (void)0
#define GPROBE_ADDK(kind, NB, ph, dt) (void)0
#define GPROBE_ADD(ts, NB, ph, dt) (void)0
#endif

namespace {

using F4 = float __attribute__((ext_vector_type(4)));
using F2 = float __attribute__((ext_vector_type(2)));
using D4 = double __attribute__((ext_vector_type(4)));
using D2 = double __attribute__((ext_vector_type(2)));

// (GM<T>, the per-type MFMA pieces: msckf_common.h)
__device__ __forceinline__ float gfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double gfma(double a, double b, double c) { return fma(a, b, c); }

__host__ __device__ constexpr int gm_nb(int M) { return (3 * M + 4 + 15) / 16; }
__host__ __device__ constexpr int gm_head(int Mmax) { return (22 * Mmax + 3) & ~3; }   // Ht rows + [r~ | r_n]
// The Y pairs are staged as a dense lower-triangular matrix, row q holding
// columns 0..q plus two padding slots (a diagonal pair block writes its upper
// 3 x 3 corner there): row q starts at gm_rowoff(q).  The assembly then reads
// element (q, 16 CB + col) of every block of a block row at one per-row lane
// address plus a compile-time offset -- no index arithmetic per element.
__host__ __device__ constexpr int gm_rowoff(int q) { return (q * q + 5 * q) / 2; }
// stage elements of observation rows [alo, ahi]
__host__ __device__ constexpr int gm_dense(int alo, int ahi) {
    return ahi < alo ? 0 : gm_rowoff(3 * ahi + 3) - gm_rowoff(3 * alo);
}
// Y staging / panel + the junk panel (written up to 128 NB + 12 RS + 23 by the
// lanes that own no pivot column)
__host__ __device__ constexpr int gm_area(int Mmax, int capf, int RS = 1) {
    return capf > 128 * gm_nb(Mmax) + 16 * RS + 16 ? ((capf + 15) & ~3) : 128 * gm_nb(Mmax) + 16 * RS + 16;
}
// the B rows [H_f~^T ; r~^T] (4 x 16 NB, zero beyond 3M) and a zero row (16 NB)
// the padding rows of the assembly read
__host__ __device__ constexpr int gm_brows(int Mmax) { return 80 * gm_nb(Mmax); }
// elements of T per wave (the two int offset tables take T-sized slots)
__host__ __device__ constexpr int gm_wave_floats(int Mmax, int capf, int RS = 1) {
    return gm_head(Mmax) + gm_area(Mmax, capf, RS) + gm_brows(Mmax) + 2 * ((Mmax + 3) & ~3);
}
// Pair k = a (a + 1) / 2 + b (b <= a) of the Y phase: a | b << 8 | (stage offset
// of element (3a, 3b)) << 16, one table load instead of a square-root decode.
constexpr int GM_MAXM = 84;   // gm_nb(84) = 16: the fp32 large-track class (k_gate_mfma_wt)
struct GmPairTab {
    unsigned v[GM_MAXM * (GM_MAXM + 1) / 2];
    constexpr GmPairTab() : v() {
        int k = 0;
        for (int a = 0; a < GM_MAXM; ++a)
            for (int b = 0; b <= a; ++b) v[k++] = (unsigned)a | ((unsigned)b << 8) | ((unsigned)(gm_rowoff(3 * a) + 3 * b) << 16);
    }
};
static_assert(gm_rowoff(3 * GM_MAXM) < 65536, "pair table offsets are 16-bit");
__device__ constexpr GmPairTab g_gm_pairs{};
__host__ __device__ constexpr int bidx(int rb, int cb) { return rb * (rb + 1) / 2 + cb; }
// The one-wave size classes (GateClasses::LIM) are exactly the 16-row block
// counts: every feature of class c fills nb = c + 1 blocks, so the kernel of a
// class runs with a compile-time block count.
constexpr bool gm_class_exact() {
    for (int c = 0; c < GateClasses::NC - 2; ++c) {
        const int lo = c == 0 ? 1 : GateClasses::LIM[c - 1] + 1;
        if (gm_nb(lo) != c + 1 || gm_nb(GateClasses::LIM[c]) != c + 1) return false;
    }
    return true;
}
static_assert(gm_class_exact(), "gating size classes must match the MFMA block counts");

// Blocked LDL^T of the assembled lower block triangle, 4 pivots per step (see
// the file header).  acc holds blocks (RB, CB), CB <= RB < NB, in the C layout
// of v_mfma_f32_16x16x4_f32; pan is the wave's [16 NB][4] panel, followed by
// a junk copy for the lanes that own no pivot column.  The feature
// fills exactly NB blocks (its size class), so the elimination runs all
// 4 NB - 1 steps up to the B rows: the unit padding pivots beyond 3M have zero
// couplings and leave everything unchanged.  No branches (a non-positive pivot
// only sets the returned flag; its garbage is discarded by gm_finish) and no
// explicit LDS waits (one wave's LDS operations complete in issue order): the
// whole elimination is one basic block, so the scheduler can overlap the next
// step's panel dump / reads / 4x4 factor with this step's MFMA tail.
// Register-lean variants (block rows streamed through the elimination, P rows
// through the multi-pass Y phase): the f64 classes.  (f32 NB = 5 / 6 streamed at
// four waves per SIMD measured no faster -- 2.68 ms -- or slower with NB = 6's
// spill -- 2.92 ms -- than the wide version at three.)
// (round 4 again: fp32 NB = 5 streamed at four waves per SIMD, 123 VGPRs, no
// spill, measured 2.32 ms against 2.19-2.21 -- profiles/r04/ab_gate_st5_*)
__host__ __device__ constexpr bool gm_stream(int NB, int ts) { return ts == 8; }

template <typename T, int NB, bool STREAM = gm_stream(NB, sizeof(T))>
__device__ __forceinline__ bool gm_eliminate(typename GM<T>::V4 (&acc)[NB * (NB + 1) / 2], T* pan, int lane) {
    using V4 = typename GM<T>::V4;
    constexpr int RS = GM<T>::RS, RG = GM<T>::RG;
    const int col_l = lane & 15, rg = lane >> 4;
    const int csel = rg;   // pivot column of this lane's operands
    // this lane's B-operand element of block row RB: panel row 16 RB + col_l, column csel
    const T* bsrc = pan + 4 * col_l + csel;
    const bool owner[4] = {(col_l >> 2) == 0, (col_l >> 2) == 1, (col_l >> 2) == 2, (col_l >> 2) == 3};
    // junk slots of the lanes that own no pivot column: the lane's own bank,
    // except (fp32) that the column 0..3 lanes move 4 sc banks up when another
    // group owns the step -- the owners' banks are theirs (16 rg + c) then, and
    // the dump would be 2-way conflicted
    T* junk[4];
#pragma unroll
    for (int sc = 0; sc < 4; ++sc)
        junk[sc] = pan + 64 * NB + lane + ((RS == 1 && sc > 0 && (col_l >> 2) == 0) ? 4 * sc : 0);
    T dmin = T(1);   // smallest pivot (a NaN pivot poisons the B rows instead: gm_finish)
    T onehot[4];     // e_csel
#pragma unroll
    for (int k = 0; k < 4; ++k) onehot[k] = csel == k ? T(1) : T(0);
#pragma unroll
    for (int KB = 0; KB < NB; ++KB) {
#pragma unroll
        for (int sc = 0; sc < 4; ++sc) {
            if (KB == NB - 1 && sc == 3) break;   // the last four rows are the B rows
            const int p0 = 16 * KB + 4 * sc;
            // 1. owners of columns p0 .. p0 + 3 dump them (rows of blocks KB..NB-1);
            //    the other lanes write to a junk area past the panel (pan + 64 NB,
            //    one dword column per lane: no bank conflicts) -- no divergent
            //    branch in the step
            {
                T* d = owner[sc] ? pan + 4 * (16 * KB + RG * rg) + (col_l & 3) : junk[sc];
#pragma unroll
                for (int RB = KB; RB < NB; ++RB) {
                    const V4 v = acc[bidx(RB, KB)];
                    T* dd = d + 64 * (RB - KB);
                    dd[0] = v[0]; dd[4 * RS] = v[1]; dd[8 * RS] = v[2]; dd[12 * RS] = v[3];
                }
            }
            // 2. every lane factors the diagonal 4x4 A_d = L D L^T (lower entries only)
            const V4 r0 = *reinterpret_cast<const V4*>(pan + 4 * p0);
            const V4 r1 = *reinterpret_cast<const V4*>(pan + 4 * p0 + 4);
            const V4 r2 = *reinterpret_cast<const V4*>(pan + 4 * p0 + 8);
            const V4 r3 = *reinterpret_cast<const V4*>(pan + 4 * p0 + 12);
            V4 xr[NB];   // this lane's panel row of every block row (f32; f64 reads them as it goes)
            T bv[NB];
#pragma unroll
            for (int RB = KB; RB < NB; ++RB) {
                if constexpr (!STREAM) xr[RB] = *reinterpret_cast<const V4*>(pan + 4 * (16 * RB + col_l));
                bv[RB] = bsrc[64 * RB];
            }
            const T d0 = r0.x, e0 = pivot_rcp(d0);
            const T l10 = r1.x * e0, l20 = r2.x * e0, l30 = r3.x * e0;
            const T d1 = r1.y - l10 * r1.x, e1 = pivot_rcp(d1);
            const T m21 = r2.y - l20 * r1.x, m31 = r3.y - l30 * r1.x;
            const T l21 = m21 * e1, l31 = m31 * e1;
            const T d2 = r2.z - l20 * r2.x - l21 * m21, e2 = pivot_rcp(d2);
            const T m32 = r3.z - l30 * r2.x - l31 * m21;
            const T l32 = m32 * e2;
            const T d3 = r3.w - l30 * r3.x - l31 * m31 - l32 * m32;
            dmin = fmin(dmin, fmin(fmin(d0, d1), fmin(d2, d3)));
            const T e3 = pivot_rcp(d3);
            // 3. the rank-4 update is C -= X A_d^-1 X^T, X = the panel columns: the
            //    B operand is X itself (lane: row 16 RB + col_l, pivot csel), the A
            //    operand X m with m = -(column csel of A_d^-1 = L^-T D^-1 L^-1).  Rows
            //    of finished pivots are not masked: exact elimination leaves them
            //    zero, and they only ever feed finished rows / columns.
            //    h = L^-1 e_csel (forward, from the lane's one-hot), u = D^-1 h,
            //    m = L^-T u (backward): 16 FMAs, no per-lane selects
            const T h0 = onehot[0];
            const T h1 = gfma(-l10, h0, onehot[1]);
            const T h2 = gfma(-l21, h1, gfma(-l20, h0, onehot[2]));
            const T h3 = gfma(-l32, h2, gfma(-l31, h1, gfma(-l30, h0, onehot[3])));
            const T u0 = h0 * e0, u1 = h1 * e1, u2 = h2 * e2, u3 = h3 * e3;
            const T m2 = gfma(-l32, u3, u2);
            const T m1 = gfma(-l31, u3, gfma(-l21, m2, u1));
            const T m0 = gfma(-l30, u3, gfma(-l20, m2, gfma(-l10, m1, u0)));
            const T mm3 = -u3, mm2 = -m2, mm1 = -m1, mm0 = -m0;
            if constexpr (STREAM) {
                // one block row at a time -- its panel row, its A operand, its
                // blocks' updates -- so that the accumulators and the step's
                // operands fit two waves per SIMD
#pragma unroll
                for (int RB = KB; RB < NB; ++RB) {
                    const V4 x = *reinterpret_cast<const V4*>(pan + 4 * (16 * RB + col_l));
                    const T a = gfma(x.w, mm3, gfma(x.z, mm2, gfma(x.y, mm1, x.x * mm0)));
#pragma unroll
                    for (int CB = KB; CB <= RB; ++CB)
                        if (CB > KB || sc < 3) acc[bidx(RB, CB)] = GM<T>::mfma(a, bv[CB], acc[bidx(RB, CB)]);
                }
                continue;
            }
            T av[NB];
#pragma unroll
            for (int RB = KB; RB < NB; ++RB) {
                const V4 x = xr[RB];
                av[RB] = gfma(x.w, mm3, gfma(x.z, mm2, gfma(x.y, mm1, x.x * mm0)));
            }
            // 4. trailing rank-4 update of the lower block triangle right of the panel
            //    (after a block's last step its own column is finished: skipped)
            if (sc < 3) {
#pragma unroll
                for (int RB = KB; RB < NB; ++RB)
                    acc[bidx(RB, KB)] = GM<T>::mfma(av[RB], bv[KB], acc[bidx(RB, KB)]);
            }
#pragma unroll
            for (int CB = KB + 1; CB < NB; ++CB)
#pragma unroll
                for (int RB = CB; RB < NB; ++RB)
                    acc[bidx(RB, CB)] = GM<T>::mfma(av[RB], bv[CB], acc[bidx(RB, CB)]);
        }
    }
    return !(dmin > T(0));
}

// gamma from the B rows' 4x4 Schur block (negated [[H_f~^T Y~^-1 H_f~, .],
// [., r~^T Y~^-1 r~]]): rows / cols 12..15 of block (nb-1, nb-1), lanes 60..63.
template <typename T, int NB>
__device__ __forceinline__ void gm_finish(const typename GM<T>::V4 (&acc)[NB * (NB + 1) / 2], T* pan, int nb, int lane,
                                          bool fail, T rn2, T s2, T chi2, const FeatBatch<T>& fb, int f) {
    constexpr int RS = GM<T>::RS, RG = GM<T>::RG;
    const int col_l = lane & 15, rg = lane >> 4;
#pragma unroll
    for (int RB = 0; RB < NB; ++RB)
        if (RB == nb - 1 && col_l >= 12) {
            const typename GM<T>::V4 v = acc[bidx(RB, RB)];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = RG * rg + RS * i;   // rows 12..15 of the block: the B rows
                if (row >= 12) pan[4 * (row - 12) + (col_l - 12)] = v[i];
            }
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) {
        const T* a = pan;
        const T d0 = a[0];
        const T l10 = a[4] / d0, l20 = a[8] / d0, l30 = a[12] / d0;
        const T d1 = a[5] - l10 * l10 * d0;
        const T l21 = (a[9] - l20 * l10 * d0) / d1;
        const T l31 = (a[13] - l30 * l10 * d0) / d1;
        const T d2 = a[10] - l20 * l20 * d0 - l21 * l21 * d1;
        const T l32 = (a[14] - l30 * l20 * d0 - l31 * l21 * d1) / d2;
        const T d3 = a[15] - l30 * l30 * d0 - l31 * l31 * d1 - l32 * l32 * d2;
        T gam = -d3 + rn2 / s2;
        if (fail || !(d0 < T(0)) || !(d1 < T(0)) || !(d2 < T(0)) || !(gam == gam)) gam = T(INFINITY);
        fb.gamma[f] = gam;
        fb.accept[f] = (gam < chi2) ? 1 : 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // pan reads done before it is reused
}

// Matrix assembly into the C-layout blocks of block rows [R0, R1): every
// element written exactly once -- Y entries (lower, s2 on the diagonal) from
// the pass's dense stage (soff0 = gm_rowoff of its first row), the B rows
// [H_f~^T ; r~^T] (H_f~ = -Ht[:, 3:6]) from brow, the padding rows (3M <= q <
// 16 NB - 4: unit pivots) from the zero row, zeros above the diagonal.  Each of
// the lane's four rows of a block row resolves to one LDS address; element
// (q, 16 CB + col) is then that address + 16 CB (an instruction offset), so
// the off-diagonal blocks cost no vector ALU at all.  Rows at or past 3M occur
// only in the last two block rows (the class is exact: 3M >= 16 NB - 19).
template <typename T, int NB>
__device__ __forceinline__ void gm_assemble(typename GM<T>::V4 (&acc)[NB * (NB + 1) / 2], int R0, int R1, int soff0,
                                            int M3, T s2, const T* stage, const T* brow, const T* zrow, int lane) {
    using V4 = typename GM<T>::V4;
    constexpr int RS = GM<T>::RS, RG = GM<T>::RG;
    constexpr int nB = 16 * NB - 4;
    int col_l = lane & 15, rg = lane >> 4;
    // opaque copies: the row offsets are computed in the pass loop, not hoisted
    // out of it into registers live across every pass
    asm volatile("" : "+v"(col_l), "+v"(rg));
    int r[4];
    bool up[4], dg[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        r[i] = RG * rg + RS * i;
        up[i] = r[i] < col_l;
        dg[i] = r[i] == col_l;
    }
#pragma unroll
    for (int RB = 0; RB < NB; ++RB) {
        if (RB < R0 || RB >= R1) continue;   // uniform
        const T* src[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = 16 * RB + r[i];
            const T* ptr = stage + (gm_rowoff(q) - soff0) + col_l;
            if (RB >= NB - 2) {
                ptr = q < M3 ? ptr : zrow + col_l;
                if (RB == NB - 1) ptr = q >= nB ? brow + (q - nB) * (16 * NB) + col_l : ptr;
            }
            src[i] = ptr;
        }
#pragma unroll
        for (int CB = 0; CB <= RB; ++CB) {
            V4 a;
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = src[i][16 * CB];
            if (CB == RB) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int q = 16 * RB + r[i];
                    const T dv = RB < NB - 2 ? s2 : (q < M3 ? s2 : (q < nB ? T(1) : T(0)));
                    a[i] = up[i] ? T(0) : (dg[i] ? a[i] + dv : a[i]);
                }
            }
            acc[bidx(RB, CB)] = a;
            // one block's reads in flight at a time: the reads land in the
            // accumulators themselves, no register peak on top of them (the
            // scheduler otherwise hoists a whole block row of reads -- 152 VGPRs
            // spilled in the fp64 NB = 6 class)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// waves per SIMD the accumulators (4 NB (NB + 1) / 2 registers) leave room for
// (single-pass Y staging keeps two or three pair blocks in flight: one wave less)
// (fp64: 8 NB (NB + 1) / 2 accumulator registers; NB = 7 at one wave per SIMD,
// with the accumulators spread over the AGPRs)
__host__ __device__ constexpr int gm_waves(int NB, bool MP, int ts = 4) {
    return ts == 8 ? (NB <= 3 ? 3 : (NB <= 6 ? 2 : 1))
                   : ((NB <= 2 && MP) ? 5 : (NB <= 4 ? 4 : (NB <= 6 ? 3 : 2)));
}

template <typename T, int NB, bool MP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gm_waves(NB, MP, sizeof(T))))) k_gate_mfma(DevState<T> st, Params<T> prm, FeatBatch<T> fb,
                                                   const int* __restrict__ flist, int nlist, int Mmax, int capf) {
    using V4 = typename GM<T>::V4;
    using V2 = typename GM<T>::V2;
    constexpr int RS = GM<T>::RS;
    constexpr bool GM_STREAM = gm_stream(NB, sizeof(T));
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    // wave-uniform by construction; readfirstlane tells the compiler, so every
    // size test below is a scalar branch instead of an exec-mask region
    const int li = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * wpb + wv);
    if (li >= nlist) return;
    const int f = __builtin_amdgcn_readfirstlane(flist[li]);
    if (!fb.valid[f]) {
        if (lane == 0) { fb.gamma[f] = NAN; fb.accept[f] = 0; }
        return;
    }
    GPROBE_T(t_start);
    // the threshold is loaded with the feature's metadata: the final decision
    // then costs no memory round trip of its own
    const T chi2 = fb.chi2[f];
    const int b = __builtin_amdgcn_readfirstlane(fb.feat_filter[f]);
    const int o0 = __builtin_amdgcn_readfirstlane(fb.obs_off[f]);
    const int M = __builtin_amdgcn_readfirstlane(fb.obs_off[f + 1]) - o0, M3 = 3 * M;
    constexpr int nb = NB;                 // the size class: gm_nb(M) == NB (gm_class_exact)
    T* ht = reinterpret_cast<T*>(smem_raw) + (size_t)wv * gm_wave_floats(Mmax, capf, RS);
    T* rt = ht + 18 * Mmax;                // [Mmax][4]: r~ (3), r_n
    T* area = ht + gm_head(Mmax);
    T* stage = area;                       // [capf] dense lower Y rows of one pass (gm_rowoff)
    T* pan = area;                         // [16 NB][4] panel rows (after the Y phase)
    T* brow = area + gm_area(Mmax, capf, RS);   // [4][16 NB] B rows
    T* zrow = brow + 64 * NB;                    // [16 NB] zeros
    int* slot = reinterpret_cast<int*>(brow + gm_brows(Mmax));
    // The feature's gating records ([M][OBS_HTS] from k_feature: Ht 3 x 6, r~, r_n)
    // as element pairs, and its cam slots: every global load issued before the
    // first wait (one round trip instead of one per loop trip), then scattered
    // into the LDS rows ht [M][6][3] (Ht transposed: Ht[x][u] at 3 u + x, so the
    // Y phase reads the (Ht[0][u], Ht[1][u]) operand pairs as adjacent words) /
    // rt [M][4].
    int* coff = slot + ((Mmax + 3) & ~3);
    {
        constexpr int MCAP = (16 * NB - 4) / 3;   // the class's largest M (gm_class_exact)
        constexpr int NCH = (12 * MCAP + 63) / 64;
        static_assert(OBS_HT == 0 && OBS_RT == 18 && OBS_HTS == 24, "record layout");
        const V2* src = reinterpret_cast<const V2*>(fb.obs_ht + (size_t)o0 * OBS_HTS);
        V2 cv[NCH];
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int k = lane + 64 * j;
            cv[j] = k < 12 * M ? src[k] : V2{0, 0};
        }
        const int sl = lane < M ? fb.obs_cam[o0 + lane] : 0;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int k = lane + 64 * j, o = k / 12, e = 2 * (k - 12 * o);   // elements e, e + 1 of record o
            if (k < 12 * M) {
                if (e < OBS_RT) {   // Ht[x][u], Ht[x][u + 1] (e even: u <= 4)
                    const int x = e / 6, u = e - 6 * x;
                    T* d = ht + 18 * o + 3 * u + x;
                    d[0] = cv[j].x;
                    d[3] = cv[j].y;
                } else if (e < OBS_RT + 4) {
                    *reinterpret_cast<V2*>(rt + 4 * o + (e - OBS_RT)) = cv[j];
                }
            }
        }
        // P offsets of the observations' cam blocks: row part (21 + 6 s) ldp + 21, column part 6 s
        if (lane < M) {
            slot[lane] = (21 + 6 * sl) * st.Dmax + 21;
            coff[lane] = 6 * sl;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // B rows [H_f~^T ; r~^T] over the 16 NB columns (zero past 3M) and the zero row
#pragma unroll
    for (int j = 0; j < (16 * NB + 63) / 64; ++j) {
        const int p = lane + 64 * j;
        if (p < 16 * NB) {
            const bool pv = p < M3;
            const int o = pv ? p / 3 : 0, cp = p - 3 * o;
            const T* h = ht + 18 * o + 9 + cp;   // Ht[cp][3 + j] at h[3 j] (transposed rows)
            brow[p] = pv ? -h[0] : T(0);
            brow[16 * NB + p] = pv ? -h[3] : T(0);
            brow[32 * NB + p] = pv ? -h[6] : T(0);
            brow[48 * NB + p] = pv ? rt[4 * o + cp] : T(0);
            zrow[p] = T(0);
        }
    }
    GPROBE_T(t_fetched);
    GPROBE_ADD(sizeof(T), NB, 0, t_fetched - t_start);
#ifdef MSCKF_GATE_PROBE
    unsigned long long t_y = 0, t_asm = 0;
#endif

    constexpr int NBLK = NB * (NB + 1) / 2;
    V4 acc[NBLK];
    const T s2 = prm.sigma2;
    auto assemble = [&](int R0, int R1, int soff0) {
        gm_assemble<T, NB>(acc, R0, R1, soff0, M3, s2, stage, brow, zrow, lane);
    };

    // ---- Y: observation-pair blocks Ht_a P_ab Ht_b^T (a >= b, 3x3) into the
    // dense lower stage, pairs enumerated in row-major lower order k = a (a + 1)
    // / 2 + b (g_gm_pairs) -- consecutive lanes take consecutive b of one row a,
    // so a load instruction reads consecutive 24-byte row segments of P (cams of
    // a track are usually consecutive slots) instead of 64 scattered blocks.
    // When the whole matrix exceeds capf elements the rows are staged in passes
    // aligned to block rows [R0, R1) (observation rows [16 R0 / 3, (16 R1 - 1) /
    // 3], those straddling a boundary twice), so that every accumulator block is
    // assembled once, never read back.
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ldp = st.Dmax;
    const T* Prow[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) Prow[u] = P + u * ldp;
    // pair blocks per lane in flight: the Y phase's VGPRs are free up to the
    // elimination's peak once the accumulators outgrow them (NB >= 5)
    constexpr int BIF = (MP || sizeof(T) == 8) ? 1 : (NB >= 5 ? 3 : 2);
    auto npairs = [&](int lo, int hi) { return hi < lo ? 0 : (hi + 1) * (hi + 2) / 2 - lo * (lo + 1) / 2; };
    for (int R0 = 0; R0 < nb;) {
        const int alo = (16 * R0) / 3;
        int R1 = R0 + 1, ahi = min(M - 1, (16 * R1 - 1) / 3);
        while (R1 < nb) {
            const int ah2 = min(M - 1, (16 * (R1 + 1) - 1) / 3);
            if (gm_dense(alo, ah2) > capf) break;
            ++R1;
            ahi = ah2;
        }
        const int kbase = alo * (alo + 1) / 2, nbp = npairs(alo, ahi);
        const int soff0 = gm_rowoff(3 * alo);
        // stage rows of pair entry e: 3a, 3a + 1, 3a + 2 (row q + 1 starts q + 3 after row q)
        auto pair_dst = [&](unsigned e, int a, T* (&d)[3]) {
            d[0] = stage + ((int)(e >> 16) - soff0);
            d[1] = d[0] + 3 * a + 3;
            d[2] = d[1] + 3 * a + 4;
        };
        GPROBE_T(t_p0);
        if constexpr (MP && GM_STREAM) {
            // staged in passes (earlier passes' accumulators live): one pair per
            // lane, P streamed a row at a time into Ha P (3 x 6) -- 18 + 6
            // elements in registers instead of the 6 x 6 block's 36
            for (int kk = lane; kk < nbp; kk += 64) {
                const unsigned pe = g_gm_pairs.v[kbase + kk];
                const int a = pe & 0xff, bo = (pe >> 8) & 0xff;
                const unsigned boff = (unsigned)(slot[a] + coff[bo]) * (unsigned)sizeof(T);
                const T* Ha = ht + 18 * a;
                const T* Hb = ht + 18 * bo;
                V2 t[3][3];   // Ha[x] P as three column pairs
#pragma unroll
                for (int x = 0; x < 3; ++x)
#pragma unroll
                    for (int c = 0; c < 3; ++c) t[x][c] = V2{0, 0};
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    T pr[6];
                    __builtin_memcpy(pr, reinterpret_cast<const char*>(Prow[u]) + boff, 6 * sizeof(T));
#pragma unroll
                    for (int x = 0; x < 3; ++x) {
                        const T h = Ha[3 * u + x];
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            t[x][c] = __builtin_elementwise_fma(V2{h, h}, V2{pr[2 * c], pr[2 * c + 1]}, t[x][c]);
                    }
                    __builtin_amdgcn_sched_barrier(0);   // one P row in flight
                }
                T* dst[3];
                pair_dst(pe, a, dst);
#pragma unroll
                for (int x = 0; x < 3; ++x) {
                    const T t1[6] = {t[x][0].x, t[x][0].y, t[x][1].x, t[x][1].y, t[x][2].x, t[x][2].y};
                    V2 y01 = {0, 0};
                    T y2 = 0;
#pragma unroll
                    for (int u = 0; u < 6; ++u) {
                        y01 = __builtin_elementwise_fma(V2{t1[u], t1[u]}, V2{Hb[3 * u], Hb[3 * u + 1]}, y01);
                        y2 = gfma(t1[u], Hb[3 * u + 2], y2);
                    }
                    dst[x][0] = y01.x;
                    dst[x][1] = y01.y;
                    dst[x][2] = y2;
                }
            }
        } else
        {
        // the next trip's pair entries are loaded under this trip's arithmetic
        unsigned pen[BIF];
        auto pload = [&](int k0) {
#pragma unroll
            for (int j = 0; j < BIF; ++j) {
                const int kk = k0 + 64 * j + lane;
                pen[j] = g_gm_pairs.v[kbase + (kk < nbp ? kk : 0)];
            }
        };
        pload(0);
        for (int k0 = 0; k0 < nbp; k0 += 64 * BIF) {
            T Pl[BIF][36];
            int oa[BIF], ob[BIF];
            unsigned pe[BIF];
#pragma unroll
            for (int j = 0; j < BIF; ++j) pe[j] = pen[j];
            if (k0 + 64 * BIF < nbp) pload(k0 + 64 * BIF);
#pragma unroll
            for (int j = 0; j < BIF; ++j) {
                const int kk = k0 + 64 * j + lane;
                oa[j] = pe[j] & 0xff;
                ob[j] = (pe[j] >> 8) & 0xff;
                // row u of the block: the wave-uniform row base P + u ldp (SGPRs)
                // plus the lane's 32-bit element offset -- no 64-bit address
                // arithmetic per row
                const unsigned boff = (unsigned)(slot[oa[j]] + coff[ob[j]]) * (unsigned)sizeof(T);
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    if (kk < nbp) {
                        __builtin_memcpy(Pl[j] + 6 * u, reinterpret_cast<const char*>(Prow[u]) + boff, 6 * sizeof(T));
                    } else {
#pragma unroll
                        for (int c2 = 0; c2 < 6; ++c2) Pl[j][6 * u + c2] = T(0);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < BIF; ++j) {
                const int kk = k0 + 64 * j + lane;
                if (kk >= nbp) continue;
                const T* Ha = ht + 18 * oa[j];
                const T* Hb = ht + 18 * ob[j];
                T* dst[3];
                pair_dst(pe[j], oa[j], dst);
                V2 hb01[6];   // (Hb[0][u], Hb[1][u])
#pragma unroll
                for (int u = 0; u < 6; ++u) hb01[u] = V2{Hb[3 * u], Hb[3 * u + 1]};
#pragma unroll
                for (int x = 0; x < 3; ++x) {
                    V2 t2[3] = {V2{0, 0}, V2{0, 0}, V2{0, 0}};   // Ha[x] P as three column pairs
#pragma unroll
                    for (int u = 0; u < 6; ++u) {
                        const T h = Ha[3 * u + x];
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            t2[c] = __builtin_elementwise_fma(V2{h, h}, V2{Pl[j][6 * u + 2 * c], Pl[j][6 * u + 2 * c + 1]},
                                                              t2[c]);
                    }
                    const T t1[6] = {t2[0].x, t2[0].y, t2[1].x, t2[1].y, t2[2].x, t2[2].y};
                    V2 y01 = {0, 0};
                    T y2 = 0;
#pragma unroll
                    for (int u = 0; u < 6; ++u) {
                        y01 = __builtin_elementwise_fma(V2{t1[u], t1[u]}, hb01[u], y01);
                        y2 = gfma(t1[u], Hb[3 * u + 2], y2);
                    }
                    dst[x][0] = y01.x;
                    dst[x][1] = y01.y;
                    dst[x][2] = y2;
                }
            }
        }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // one wave: its stores are visible to all lanes
        GPROBE_T(t_p1);
        assemble(R0, R1, soff0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next pass / the panel reuse
#ifdef MSCKF_GATE_PROBE
        GPROBE_T(t_p2);
        t_y += t_p1 - t_p0;
        t_asm += t_p2 - t_p1;
#endif
        R0 = R1;
        if (!MP) break;
    }
    GPROBE_ADD(sizeof(T), NB, 1, t_y);
    GPROBE_ADD(sizeof(T), NB, 2, t_asm);
    GPROBE_T(t_e0);

    // ---- blocked LDL^T, 4 pivots per step, MFMA trailing updates ----
    const bool fail = gm_eliminate<T, NB>(acc, pan, lane);
    // |r_n|^2 from the LDS records (rt is outside the stage / panel area): not
    // held in a register across the whole kernel
    T rn2 = lane < M ? rt[4 * lane + 3] * rt[4 * lane + 3] : T(0);
    rn2 = wave_sum(rn2);
    GPROBE_T(t_e1);
    gm_finish<T, NB>(acc, pan, NB, lane, fail, rn2, s2, chi2, fb, f);
    GPROBE_T(t_end);
    GPROBE_ADD(sizeof(T), NB, 3, t_e1 - t_e0);
    GPROBE_ADD(sizeof(T), NB, 4, t_end - t_e1);
    GPROBE_ADD(sizeof(T), NB, 5, t_end - t_start);
    GPROBE_ADD(sizeof(T), NB, 6, 1);
}

// ---------------------------------------------------------------------------
// Large tracks, round 6: k_gate_mfma_wt<NB, W> -- the one-wave kernel's
// elimination spread over a W-wave workgroup per feature of exactly NB blocks
// (the host lists the 40 < M <= 82 class by block count, GateClasses::big_off).
// Wave WV owns block rows RB = WV + W i: every wave runs its own compile-time
// specialised body (gt_body<NB, W, WV>), so its accumulator slots, block
// indices and trailing-update ranges are constants -- no per-block branches,
// no slots for blocks right of the diagonal.  Per 4-pivot step the owners of
// the pivot columns dump them to a double-buffered LDS panel, one barrier,
// then every wave factors the 4x4 diagonal itself (one-hot solves, no
// divisions or selects, as k_gate_mfma), reads the B operands of the block
// rows at or below the panel and updates its own blocks with one
// v_mfma_f32_16x16x4_f32 each.  The Y pairs come from the dense lower stage
// and the pair table of the one-wave kernel, staged by all 64 W threads in
// block-row passes, each followed by the owners' assembly.
// (Replaces round 5's k_gate_mfma_wg: runtime block counts, the B operands of
// all 16 block rows formed every step, a square-root pair decode and per-
// element index arithmetic in the assembly -- 6.0k VALU per wave at 50x400.)
constexpr int GT_NBMAX = 16;   // block counts k_gate_mfma_wt is built for: fp32 9.., fp64 8.. (M <= 84)
__host__ __device__ constexpr int gt_rows(int NB, int W, int WV) { return WV < NB ? (NB - 1 - WV) / W + 1 : 0; }
__host__ __device__ constexpr int gt_off(int W, int WV, int i) { return i * (WV + 1) + W * i * (i - 1) / 2; }
__host__ __device__ constexpr int gt_slots(int NB, int W, int WV) { return gt_off(W, WV, gt_rows(NB, W, WV)); }
__host__ __device__ constexpr int gt_maxslots(int NB, int W) {
    int m = 0;
    for (int v = 0; v < W; ++v) m = gt_slots(NB, W, v) > m ? gt_slots(NB, W, v) : m;
    return m;
}
// waves per SIMD the largest wave's accumulators leave room for
// (ts: bytes of the scalar type = VGPRs per accumulator block / 4 x 4)
__host__ __device__ constexpr int gt_waves(int NB, int W, int ts = 4) {
    return ts * gt_maxslots(NB, W) + (ts == 8 ? 112 : 96) <= 168 ? 3
         : (ts * gt_maxslots(NB, W) + (ts == 8 ? 112 : 96) <= 256 ? 2 : 1);
}
// LDS (elements of T): records | stage / [2][16 NB][4] panel | junk [W][128] | B rows [4][16 NB], zero row [16 NB] |
// slot, coff
__host__ __device__ constexpr int gt_area(int NB, int capf) { return capf + 16 > 128 * NB ? ((capf + 16 + 3) & ~3) : 128 * NB; }
__host__ __device__ constexpr int gt_floats(int Mmax, int NB, int W, int capf) {
    return gm_head(Mmax) + gt_area(NB, capf) + 128 * W + 80 * NB + 2 * ((Mmax + 3) & ~3);
}

template <typename T, int NB, int W, int WV>
__device__ __forceinline__ void gt_body(const DevState<T>& st, const FeatBatch<T>& fb, int f, int b, int M, T s2,
                                        T chi2, T* ht, T* rt, T* area, T* junk, T* brow, T* zrow, const int* slot,
                                        const int* coff, int capf) {
    using V4 = typename GM<T>::V4;
    using V2 = typename GM<T>::V2;
    constexpr int RS = GM<T>::RS, RG = GM<T>::RG;
    constexpr int NT = 64 * W, R = gt_rows(NB, W, WV), NS = gt_slots(NB, W, WV);
    constexpr int nB = 16 * NB - 4;
    const int tid = threadIdx.x, lane = tid & 63, M3 = 3 * M;
    T* stage = area;
    T* pan = area;
    V4 acc[NS > 0 ? NS : 1];

    // ---- Y: pair blocks Ht_a P_ab Ht_b^T into the dense lower stage, in passes of block rows
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ldp = st.Dmax;
    const T* Prow[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) Prow[u] = P + u * ldp;
    auto npairs = [&](int lo, int hi) { return hi < lo ? 0 : (hi + 1) * (hi + 2) / 2 - lo * (lo + 1) / 2; };
    for (int R0 = 0; R0 < NB;) {
        const int alo = (16 * R0) / 3;
        int R1 = R0 + 1, ahi = min(M - 1, (16 * R1 - 1) / 3);
        while (R1 < NB) {
            const int ah2 = min(M - 1, (16 * (R1 + 1) - 1) / 3);
            if (gm_dense(alo, ah2) > capf) break;
            ++R1;
            ahi = ah2;
        }
        const int kbase = alo * (alo + 1) / 2, nbp = npairs(alo, ahi);
        const int soff0 = gm_rowoff(3 * alo);
        unsigned pen = g_gm_pairs.v[kbase + (tid < nbp ? tid : 0)];
        for (int kk = tid; kk < nbp; kk += NT) {
            const unsigned pe = pen;
            if (kk + NT < nbp) pen = g_gm_pairs.v[kbase + kk + NT];
            const int a = pe & 0xff, bo = (pe >> 8) & 0xff;
            const unsigned boff = (unsigned)(slot[a] + coff[bo]) * (unsigned)sizeof(T);
            const T* Ha = ht + 18 * a;
            const T* Hb = ht + 18 * bo;
            T* d0 = stage + ((int)(pe >> 16) - soff0);
            T* dst[3] = {d0, d0 + 3 * a + 3, d0 + 6 * a + 7};
            V2 t[3][3];   // Ha[x] P as three column pairs
#pragma unroll
            for (int x = 0; x < 3; ++x)
#pragma unroll
                for (int c = 0; c < 3; ++c) t[x][c] = V2{0, 0};
            if constexpr (sizeof(T) == 8) {
                // fp64: P streamed a row at a time (as the one-wave kernel's multi-pass Y phase)
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    T pr[6];
                    __builtin_memcpy(pr, reinterpret_cast<const char*>(Prow[u]) + boff, 6 * sizeof(T));
#pragma unroll
                    for (int x = 0; x < 3; ++x) {
                        const T h = Ha[3 * u + x];
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            t[x][c] = __builtin_elementwise_fma(V2{h, h}, V2{pr[2 * c], pr[2 * c + 1]}, t[x][c]);
                    }
                    __builtin_amdgcn_sched_barrier(0);   // one P row in flight
                }
            } else {
                T Pl[36];
#pragma unroll
                for (int u = 0; u < 6; ++u)
                    __builtin_memcpy(Pl + 6 * u, reinterpret_cast<const char*>(Prow[u]) + boff, 6 * sizeof(T));
#pragma unroll
                for (int x = 0; x < 3; ++x)
#pragma unroll
                    for (int u = 0; u < 6; ++u) {
                        const T h = Ha[3 * u + x];
#pragma unroll
                        for (int c = 0; c < 3; ++c)
                            t[x][c] = __builtin_elementwise_fma(V2{h, h}, V2{Pl[6 * u + 2 * c], Pl[6 * u + 2 * c + 1]},
                                                                t[x][c]);
                    }
            }
            V2 hb01[6];
#pragma unroll
            for (int u = 0; u < 6; ++u) hb01[u] = V2{Hb[3 * u], Hb[3 * u + 1]};
#pragma unroll
            for (int x = 0; x < 3; ++x) {
                const T t1[6] = {t[x][0].x, t[x][0].y, t[x][1].x, t[x][1].y, t[x][2].x, t[x][2].y};
                V2 y01 = {0, 0};
                T y2 = 0;
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    y01 = __builtin_elementwise_fma(V2{t1[u], t1[u]}, hb01[u], y01);
                    y2 = gfma(t1[u], Hb[3 * u + 2], y2);
                }
                dst[x][0] = y01.x;
                dst[x][1] = y01.y;
                dst[x][2] = y2;
            }
        }
        __syncthreads();
        // assembly of this wave's block rows in [R0, R1) (as gm_assemble)
        {
            int col_l = lane & 15, rg = lane >> 4;
            asm volatile("" : "+v"(col_l), "+v"(rg));
            int r[4];
            bool up[4], dg[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                r[i] = RG * rg + RS * i;
                up[i] = r[i] < col_l;
                dg[i] = r[i] == col_l;
            }
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int RB = WV + W * i;
                if (RB < R0 || RB >= R1) continue;   // uniform
                const T* src[4];
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) {
                    const int q = 16 * RB + r[ii];
                    const T* ptr = stage + (gm_rowoff(q) - soff0) + col_l;
                    if (RB >= NB - 2) {
                        ptr = q < M3 ? ptr : zrow + col_l;
                        if (RB == NB - 1) ptr = q >= nB ? brow + (q - nB) * (16 * NB) + col_l : ptr;
                    }
                    src[ii] = ptr;
                }
#pragma unroll
                for (int c = 0; c <= RB; ++c) {
                    V4 v;
#pragma unroll
                    for (int ii = 0; ii < 4; ++ii) v[ii] = src[ii][16 * c];
                    if (c == RB) {
#pragma unroll
                        for (int ii = 0; ii < 4; ++ii) {
                            const int q = 16 * RB + r[ii];
                            const T dv = RB < NB - 2 ? s2 : (q < M3 ? s2 : (q < nB ? T(1) : T(0)));
                            v[ii] = up[ii] ? T(0) : (dg[ii] ? v[ii] + dv : v[ii]);
                        }
                    }
                    acc[gt_off(W, WV, i) + c] = v;
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        __syncthreads();   // stage reads done before the next pass / the panel reuse
        R0 = R1;
    }

    // ---- blocked LDL^T, 4 pivots per step, MFMA trailing updates
    const int col_l = lane & 15, rg = lane >> 4, csel = rg;
    const bool owner[4] = {(col_l >> 2) == 0, (col_l >> 2) == 1, (col_l >> 2) == 2, (col_l >> 2) == 3};
    T* jk = junk + lane;
    T dmin = T(1);
    T onehot[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) onehot[k] = csel == k ? T(1) : T(0);
#pragma unroll
    for (int KB = 0; KB < NB; ++KB) {
#pragma unroll
        for (int sc = 0; sc < 4; ++sc) {
            if (KB == NB - 1 && sc == 3) break;   // the last four rows are the B rows
            const int p0 = 16 * KB + 4 * sc;
            T* pb = pan + ((4 * KB + sc) & 1) * (64 * NB);
            // 1. the owners of columns p0 .. p0 + 3 dump this wave's blocks (RB, KB)
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int RB = WV + W * i;
                if (RB < KB) continue;
                const V4 v = acc[gt_off(W, WV, i) + KB];
                T* dd = owner[sc] ? pb + 4 * (16 * RB + RG * rg) + (col_l & 3) : jk;
                dd[0] = v[0]; dd[4 * RS] = v[1]; dd[8 * RS] = v[2]; dd[12 * RS] = v[3];
            }
            LDS_BARRIER();
            // 2. every wave factors A_d = L D L^T
            const V4 r0 = *reinterpret_cast<const V4*>(pb + 4 * p0);
            const V4 r1 = *reinterpret_cast<const V4*>(pb + 4 * p0 + 4);
            const V4 r2 = *reinterpret_cast<const V4*>(pb + 4 * p0 + 8);
            const V4 r3 = *reinterpret_cast<const V4*>(pb + 4 * p0 + 12);
            T bv[NB];
#pragma unroll
            for (int CB = KB; CB < NB; ++CB) bv[CB] = pb[4 * (16 * CB + col_l) + csel];
            const T d0 = r0.x, e0 = pivot_rcp(d0);
            const T l10 = r1.x * e0, l20 = r2.x * e0, l30 = r3.x * e0;
            const T d1 = r1.y - l10 * r1.x, e1 = pivot_rcp(d1);
            const T m21 = r2.y - l20 * r1.x, m31 = r3.y - l30 * r1.x;
            const T l21 = m21 * e1, l31 = m31 * e1;
            const T d2 = r2.z - l20 * r2.x - l21 * m21, e2 = pivot_rcp(d2);
            const T m32 = r3.z - l30 * r2.x - l31 * m21;
            const T l32 = m32 * e2;
            const T d3 = r3.w - l30 * r3.x - l31 * m31 - l32 * m32;
            dmin = fmin(dmin, fmin(fmin(d0, d1), fmin(d2, d3)));
            // formed here: a wave with no block row left would otherwise sink the
            // pivots of every later step to the end, their panel rows live till then
            asm volatile("" : "+v"(dmin));
            const T e3 = pivot_rcp(d3);
            const T h0 = onehot[0];
            const T h1 = gfma(-l10, h0, onehot[1]);
            const T h2 = gfma(-l21, h1, gfma(-l20, h0, onehot[2]));
            const T h3 = gfma(-l32, h2, gfma(-l31, h1, gfma(-l30, h0, onehot[3])));
            const T u0 = h0 * e0, u1 = h1 * e1, u2 = h2 * e2, u3 = h3 * e3;
            const T m2 = gfma(-l32, u3, u2);
            const T m1 = gfma(-l31, u3, gfma(-l21, m2, u1));
            const T m0 = gfma(-l30, u3, gfma(-l20, m2, gfma(-l10, m1, u0)));
            const T mm3 = -u3, mm2 = -m2, mm1 = -m1, mm0 = -m0;
            // 3. this wave's block rows at or below the panel: C -= X A_d^-1 X^T
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int RB = WV + W * i;
                if (RB < KB) continue;
                const V4 x = *reinterpret_cast<const V4*>(pb + 4 * (16 * RB + col_l));
                const T a = gfma(x.w, mm3, gfma(x.z, mm2, gfma(x.y, mm1, x.x * mm0)));
#pragma unroll
                for (int CB = KB; CB <= RB; ++CB)
                    if (CB > KB || sc < 3)   // a block's last step leaves its own column finished
                        acc[gt_off(W, WV, i) + CB] = GM<T>::mfma(a, bv[CB], acc[gt_off(W, WV, i) + CB]);
            }
        }
    }
    // ---- gamma from the B rows' 4x4 Schur block (block (NB - 1, NB - 1), rows / cols 12..15)
    T* fin = brow;   // the B rows are free after the assembly
    if constexpr ((NB - 1) % W == WV) {
        if (col_l >= 12) {
            const V4 v = acc[gt_off(W, WV, R - 1) + NB - 1];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = RG * rg + RS * i;   // rows 12..15 of the block: the B rows
                if (row >= 12) fin[4 * (row - 12) + (col_l - 12)] = v[i];
            }
        }
    }
    T rn2 = T(0);
    if constexpr (WV == 0) {
        for (int o = lane; o < M; o += 64) rn2 += rt[4 * o + 3] * rt[4 * o + 3];
        rn2 = wave_sum(rn2);
    }
    LDS_BARRIER();
    if (tid == 0) {
        const T* a = fin;
        const T d0 = a[0];
        const T l10 = a[4] / d0, l20 = a[8] / d0, l30 = a[12] / d0;
        const T d1 = a[5] - l10 * l10 * d0;
        const T l21 = (a[9] - l20 * l10 * d0) / d1;
        const T l31 = (a[13] - l30 * l10 * d0) / d1;
        const T d2 = a[10] - l20 * l20 * d0 - l21 * l21 * d1;
        const T l32 = (a[14] - l30 * l20 * d0 - l31 * l21 * d1) / d2;
        const T d3 = a[15] - l30 * l30 * d0 - l31 * l31 * d1 - l32 * l32 * d2;
        T gam = -d3 + rn2 / s2;
        if (!(dmin > T(0)) || !(d0 < T(0)) || !(d1 < T(0)) || !(d2 < T(0)) || !(gam == gam)) gam = T(INFINITY);
        fb.gamma[f] = gam;
        fb.accept[f] = (gam < chi2) ? 1 : 0;
    }
}

template <typename T, int NB, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(gt_waves(NB, W, sizeof(T)))))
k_gate_mfma_wt(DevState<T> st, Params<T> prm, FeatBatch<T> fb, const int* __restrict__ flist, int nlist, int Mmax,
               int capf) {
    using V2 = typename GM<T>::V2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    constexpr int NT = 64 * W;
    const int tid = threadIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
    if (li >= nlist) return;
    const int f = __builtin_amdgcn_readfirstlane(flist[li]);
    if (!fb.valid[f]) {
        if (tid == 0) { fb.gamma[f] = NAN; fb.accept[f] = 0; }
        return;
    }
    const T chi2 = fb.chi2[f];
    const int b = __builtin_amdgcn_readfirstlane(fb.feat_filter[f]);
    const int o0 = __builtin_amdgcn_readfirstlane(fb.obs_off[f]);
    const int M = __builtin_amdgcn_readfirstlane(fb.obs_off[f + 1]) - o0, M3 = 3 * M;
    T* ht = reinterpret_cast<T*>(smem_raw);
    T* rt = ht + 18 * Mmax;
    T* area = ht + gm_head(Mmax);
    T* junk = area + gt_area(NB, capf) + 128 * w;
    T* brow = area + gt_area(NB, capf) + 128 * W;   // [4][16 NB] B rows, then the zero row
    T* zrow = brow + 64 * NB;
    int* slot = reinterpret_cast<int*>(zrow + 16 * NB);
    int* coff = slot + ((Mmax + 3) & ~3);
    {   // records (Ht transposed, as k_gate_mfma) and cam slots: every load issued before the first wait
        constexpr int MCAP = (16 * NB - 4) / 3;
        constexpr int NCH = (12 * MCAP + NT - 1) / NT;
        static_assert(MCAP <= NT, "one thread per observation");
        const V2* src = reinterpret_cast<const V2*>(fb.obs_ht + (size_t)o0 * OBS_HTS);
        V2 cv[NCH];
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int k = tid + NT * j;
            cv[j] = k < 12 * M ? src[k] : V2{0, 0};
        }
        const int sl = tid < M ? fb.obs_cam[o0 + tid] : 0;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const int k = tid + NT * j, o = k / 12, e = 2 * (k - 12 * o);
            if (k < 12 * M) {
                if (e < OBS_RT) {
                    const int x = e / 6, u = e - 6 * x;
                    T* d = ht + 18 * o + 3 * u + x;
                    d[0] = cv[j].x;
                    d[3] = cv[j].y;
                } else if (e < OBS_RT + 4) {
                    *reinterpret_cast<V2*>(rt + 4 * o + (e - OBS_RT)) = cv[j];
                }
            }
        }
        if (tid < M) {
            slot[tid] = (21 + 6 * sl) * st.Dmax + 21;
            coff[tid] = 6 * sl;
        }
    }
    __syncthreads();
    for (int p = tid; p < 16 * NB; p += NT) {   // B rows [H_f~^T ; r~^T] (zero past 3M) and the zero row
        const bool pv = p < M3;
        const int o = pv ? p / 3 : 0, cp = p - 3 * o;
        const T* h = ht + 18 * o + 9 + cp;
        brow[p] = pv ? -h[0] : T(0);
        brow[16 * NB + p] = pv ? -h[3] : T(0);
        brow[32 * NB + p] = pv ? -h[6] : T(0);
        brow[48 * NB + p] = pv ? rt[4 * o + cp] : T(0);
        zrow[p] = T(0);
    }
    // (the first Y pass's barrier orders these before the assembly)
    const T s2 = prm.sigma2;
    switch (w) {
        case 0: gt_body<T, NB, W, 0>(st, fb, f, b, M, s2, chi2, ht, rt, area, junk, brow, zrow, slot, coff, capf); break;
        case 1: gt_body<T, NB, W, 1>(st, fb, f, b, M, s2, chi2, ht, rt, area, junk, brow, zrow, slot, coff, capf); break;
#define GT_CASE(V) \
        case V: if constexpr (W > V) gt_body<T, NB, W, V>(st, fb, f, b, M, s2, chi2, ht, rt, area, junk, brow, zrow, slot, coff, capf); break;
        GT_CASE(2) GT_CASE(3) GT_CASE(4) GT_CASE(5) GT_CASE(6) GT_CASE(7)
#undef GT_CASE
        default: break;
    }
    static_assert(W <= 8, "at most eight waves per feature");
}

template <typename T, int NB, int W>
void launch_wt(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb, const int* list,
               int cnt, int Mmax) {
    // LDS: the CU's 160 KB over its workgroups (gt_waves per SIMD); the Y pairs
    // staged in as many block-row passes as that leaves room for
    constexpr int wgs = (4 * gt_waves(NB, W, sizeof(T)) + W - 1) / W;
    const int budget = (160 * 1024 / wgs - 512) / (int)sizeof(T);
    const int full = gm_dense(0, Mmax - 1);
    int cmin = 0;   // one block row per pass at least
    for (int R = 0; R < NB; ++R) {
        const int alo = 16 * R / 3, ahi = (16 * R + 15) / 3 < Mmax - 1 ? (16 * R + 15) / 3 : Mmax - 1;
        cmin = gm_dense(alo, ahi) > cmin ? gm_dense(alo, ahi) : cmin;
    }
    int capf = full;
    while (capf > cmin && gt_floats(Mmax, NB, W, capf) > budget) capf -= 32;
    if (capf < cmin) capf = cmin;
    const size_t lds = (size_t)gt_floats(Mmax, NB, W, capf) * sizeof(T);
    lds_limit((const void*)k_gate_mfma_wt<T, NB, W>, lds);
    hipLaunchKernelGGL((k_gate_mfma_wt<T, NB, W>), dim3(cnt), dim3(64 * W), lds, s, st, prm, fb, list, cnt, Mmax, capf);
}

template <typename T, int NB, bool MP>
void launch_cfg(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                const int* list, int cnt, int Mmax, int capf, int wpb, size_t lds) {
    lds_limit((const void*)k_gate_mfma<T, NB, MP>, lds);
    hipLaunchKernelGGL((k_gate_mfma<T, NB, MP>), dim3((cnt + wpb - 1) / wpb), dim3(64 * wpb), lds, s, st, prm, fb,
                       list, cnt, Mmax, capf);
}

template <typename T, int NB>
void launch_nb(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
               const int* list, int cnt, int Mmax) {
    // Y staging capacity: all M (M + 1) / 2 pair blocks in one pass unless four
    // waves would then need more than single_kb KB; otherwise passes (of
    // whole block rows) sized for half of that.  Multi-pass also drops the Y
    // phase's registers (one pair in flight per lane, 82-88 VGPRs), so the
    // classes with nb >= 4 gain a wave per SIMD.  Measured at 30x200 (gate
    // ms): budget 80: 3.46, 60: 3.28, 50: 3.10, 36: 3.05, 20 / 12: 3.06-3.10.
    // (fp64: twice the bytes per element, and at most two waves per SIMD above NB = 3)
    // (round 3, one-wave workgroups: fp32 budgets of 40 / 44 / 48 KB per four waves
    // measured 2.47 ms against 2.52 ms for 36 -- profiles/r03/ab_gate_kb/; fp64
    // keeps 72, its two waves per SIMD already fill the LDS)
    // (round 4: the staging is the dense lower matrix, capacities in elements)
    constexpr int single_kb = sizeof(T) == 4 ? 44 : 72;
    constexpr int RS = GM<T>::RS;
    const int full = gm_dense(0, Mmax - 1);
    int cmin = 0;   // one block row per pass at least
    for (int R = 0; R < gm_nb(Mmax); ++R) {
        const int alo = 16 * R / 3, ahi = (16 * R + 15) / 3 < Mmax - 1 ? (16 * R + 15) / 3 : Mmax - 1;
        cmin = gm_dense(alo, ahi) > cmin ? gm_dense(alo, ahi) : cmin;
    }
    auto per_wave = [&](int cf) { return (size_t)gm_wave_floats(Mmax, cf, RS) * sizeof(T); };
    // single pass if four waves' LDS fits single_kb, else the largest stage
    // that does (at least one block row)
    int capf = full;
    while (capf > cmin && 4 * per_wave(capf) > (size_t)single_kb * 1024) capf -= 32;
    if (capf < cmin) capf = cmin;
    const size_t pw = per_wave(capf);
    // one wave per workgroup: a wave's LDS and registers are released as soon as
    // its feature is done, not when the slowest of four features sharing a
    // workgroup is (the class's track lengths differ): 2.53 -> 2.49 ms at 30x200,
    // step 9.19 -> 9.15 ms over four alternated runs (profiles/r03/ab_gate_wpb/)
    const int wpb = 1;
    if (capf < full) launch_cfg<T, NB, true>(s, st, prm, fb, list, cnt, Mmax, capf, wpb, wpb * pw);
    else launch_cfg<T, NB, false>(s, st, prm, fb, list, cnt, Mmax, capf, wpb, wpb * pw);
}


}  // namespace

// fp64 up to NB = 7 (M <= 36) at one wave per SIMD, the accumulators in AGPRs
// (round 5: 31 <= M <= 36 off k_gate_wave, 50x400 fp64 gate 60.4 -> 56.0 ms,
// profiles/r05/ab_gate_fp64_nb7/); NB = 8 would spill
bool gate_mfma_fits(int maxM, int ts) { return maxM >= 1 && gm_nb(maxM) <= (ts == 8 ? 7 : 8); }
bool gate_mfma_wt_fits(int maxM) { return maxM >= 1 && gm_nb(maxM) <= GT_NBMAX; }

// (round 5 ran the same elimination on fp64 MFMA for 41 <= M <= 62, three
// block rows per wave: 256 VGPRs + 192 AGPRs, one workgroup per CU, parity
// green but the 50x400 fp64 gate 55.9 -> 61.5 ms against k_gate_big's register
// tiles at two workgroups per CU -- profiles/r05/exp_gate_mfma_wg64/)

// tracks of exactly nb blocks (fp32 9 <= nb <= 16, fp64 8 <= nb <= 16): waves per
// feature by block count (round 6, profiles/r06/wt/: at 80x1000 two waves beat
// four for nb <= 11 -- 1.07 / 1.62 / 1.55 against 1.16 / 2.21 / 1.91 ms -- but
// spill at nb = 12; eight waves keep nb = 16 off scratch, 2.34 ms against 7.93,
// and lose to four below it)
template <typename T>
void launch_gate_mfma_wt(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                         const int* list, int cnt, int nb, int maxM) {
    if (cnt <= 0) return;
    if constexpr (sizeof(T) == 4) {
        switch (nb) {
            case 9: launch_wt<T, 9, 2>(s, st, prm, fb, list, cnt, maxM); break;
            case 10: launch_wt<T, 10, 2>(s, st, prm, fb, list, cnt, maxM); break;
            case 11: launch_wt<T, 11, 2>(s, st, prm, fb, list, cnt, maxM); break;
            case 12: launch_wt<T, 12, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 13: launch_wt<T, 13, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 14: launch_wt<T, 14, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 15: launch_wt<T, 15, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 16: launch_wt<T, 16, 8>(s, st, prm, fb, list, cnt, maxM); break;
            default: break;   // launch_gate sends only 9 <= nb <= GT_NBMAX here
        }
    } else {
        // fp64 (8 VGPRs per accumulator block): four waves up to 10 blocks, eight
        // beyond (50x400 fp64 gate 42.8 ms with eight waves for every count, 32.2
        // with four up to 10 blocks; profiles/r06/wt64/)
        switch (nb) {
            case 8: launch_wt<T, 8, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 9: launch_wt<T, 9, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 10: launch_wt<T, 10, 4>(s, st, prm, fb, list, cnt, maxM); break;
            case 11: launch_wt<T, 11, 8>(s, st, prm, fb, list, cnt, maxM); break;
            case 12: launch_wt<T, 12, 8>(s, st, prm, fb, list, cnt, maxM); break;
            case 13: launch_wt<T, 13, 8>(s, st, prm, fb, list, cnt, maxM); break;
            case 14: launch_wt<T, 14, 8>(s, st, prm, fb, list, cnt, maxM); break;
            case 15: launch_wt<T, 15, 8>(s, st, prm, fb, list, cnt, maxM); break;
            case 16: launch_wt<T, 16, 8>(s, st, prm, fb, list, cnt, maxM); break;
            default: break;   // launch_gate sends only 8 <= nb <= GT_NBMAX here
        }
    }
}
template void launch_gate_mfma_wt<float>(hipStream_t, const DevState<float>&, const Params<float>&,
                                         const FeatBatch<float>&, const int*, int, int, int);
template void launch_gate_mfma_wt<double>(hipStream_t, const DevState<double>&, const Params<double>&,
                                          const FeatBatch<double>&, const int*, int, int, int);

template <typename T>
void launch_gate_mfma(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                      const int* list, int cnt, int maxM) {
    if (cnt <= 0) return;
    switch (gm_nb(maxM)) {
        case 1: launch_nb<T, 1>(s, st, prm, fb, list, cnt, maxM); break;
        case 2: launch_nb<T, 2>(s, st, prm, fb, list, cnt, maxM); break;
        case 3: launch_nb<T, 3>(s, st, prm, fb, list, cnt, maxM); break;
        case 4: launch_nb<T, 4>(s, st, prm, fb, list, cnt, maxM); break;
        case 5: launch_nb<T, 5>(s, st, prm, fb, list, cnt, maxM); break;
        case 6: launch_nb<T, 6>(s, st, prm, fb, list, cnt, maxM); break;
        case 7: launch_nb<T, 7>(s, st, prm, fb, list, cnt, maxM); break;
        default:
            if constexpr (sizeof(T) == 4) launch_nb<T, 8>(s, st, prm, fb, list, cnt, maxM);
            break;
    }
}
#ifdef MSCKF_GATE_PROBE
extern "C" int msckf_gate_probe_read(unsigned long long* out) {   // [2][9][8], then reset
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gate_probe), sizeof(g_gate_probe)) != hipSuccess) return -1;
    static unsigned long long zero[2][9][8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_gate_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

template void launch_gate_mfma<float>(hipStream_t, const DevState<float>&, const Params<float>&,
                                      const FeatBatch<float>&, const int*, int, int);
template void launch_gate_mfma<double>(hipStream_t, const DevState<double>&, const Params<double>&,
                                       const FeatBatch<double>&, const int*, int, int);

}  // namespace msckf
