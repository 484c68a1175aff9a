// msckf_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the MSCKF
// stereo-VIO EKF hot path.  Every kernel is templated on T (float | double)
// and handles a batch of independent filters (one HIP launch per stage for
// all filters), so the single-filter API and the throughput mode share one
// code path.
//
// Stage map (reference file:line -> kernel):
//   process_model / _process_model / _predict_new_state /
//   _propaget_state_Covariance  msckf.py:291-368, jit_utils.py:6-135 -> k_propagate
//   state_augmentation / _state_augmentation msckf.py:385-407,
//                                            jit_utils.py:137-167   -> k_augment
//   Feature.initialize_position feature.py:167-295                  -> k_triangulate
//   measurement_jacobian + feature_jacobian msckf.py:429-541        -> k_feature
//   gating_test msckf.py:606-614                                    -> k_gate_wave /
//                       k_gate_big / k_gate_lds / k_gate (fp32: msckf_gate_mfma.hip)
//   stacking + row cap msckf.py:661-682, 776-798                    -> k_select
//   measurement_update QR msckf.py:549-556 (_fastQR)                -> k_info
//   measurement_update S, K, dx, P msckf.py:559-604 (_fastSolve)    -> msckf_kalman.hip,
//                                                                      k_correct
//   P compaction msckf.py:803-818                                   -> k_prune_*
#include <type_traits>
#include <utility>

#include "msckf_common.h"
#include "msckf_launch.h"
#include "msckf_rchol.h"

namespace msckf {

// ===========================================================================
// IMU propagation (process_model, msckf.py:291-368; jit_utils.py:6-135): ONE
// WAVE per listed filter (64-thread workgroups, ~20 KB of LDS in fp32: eight
// filters resident per CU, the whole 2048-filter batch in one round, no
// workgroup barriers -- the wave's own LDS ordering is the only sync).  Filter
// filters[w] takes samples [smp_off[w], smp_off[w+1]) in order, in chunks of
// PKC samples.  Only the quaternion recursion and the 21x21 covariance
// recursion are serial, so a chunk runs in phases:
//   A   one lane per sample: bias-corrected rates, the RK4 quaternion
//       increments' 4x4 matrices (cos/sin of |w| dt / 2, / 4)
//   B1  lane 0: the quaternion chain q_k -> dq_k -> q_{k+1}
//   B2  one lane per sample: rotations, the RK4 slopes (quirk Q1), R_k
//   B3  lane 0: the velocity / position sums
//   B4  one lane per sample: the Phi edit terms (msckf.py:329-344)
// then per sample, lane (g, c) = (lane / 21, lane % 21) owning rows 3 rb + g of
// column c (or row c):
//   C1..C5  F dt, F^2, Phi = I + F + F^2/2 + F^3/6 with the edits, Phi G Qc and
//       the Q term (Phi G Qc G^T) Phi^T
//   D1, D2  A = Phi P11 and the cumulative Phi, P11' = A Phi^T + Q dt; the
//       symmetrisation P11 = (P11' + P11'^T) / 2 is formed as the next sample's
//       D1 reads P11 (and by the write-back after the last sample)
// Products run over the structurally non-zero 3x3 blocks only (skipped terms
// are exact zeros: same sums, same order); the lane's Phi rows stay in
// registers for C5, D1 and D2.  The IMU x cam cross block is updated once with
// the product Phi_n ... Phi_1 (the per-sample full-P symmetrisation of
// msckf.py:362-363 is a no-op on the cam x cam block and only re-rounds the
// cross block); its columns are prefetched at the start (fp32) and its
// transposed half is staged through LDS so that both halves are written in
// contiguous rows.  Every dot product runs in the reference order (sum over k
// ascending).
// ===========================================================================
// [w]x[r][c] with a run-time (r, c): one read of w[3 - r - c] and a sign,
// no branch ([w]x[r][c] = -w[k] for c = r + 1 mod 3, +w[k] for c = r + 2 mod 3)
template <typename T>
__device__ __forceinline__ T skew_sel(const T* w, int r, int c) {
    const int k = r == c ? 0 : 3 - r - c;
    const T v = w[k];
    const int d = c - r + 3;
    return r == c ? T(0) : ((d == 1 || d == 4) ? -v : v);
}

// LDS row strides of the 21-wide matrices: a lane per
// row (stride RS) hits distinct banks (25 dwords; 42 dwords per fp64 row)
template <typename T> constexpr int prop_rs() { return sizeof(T) == 4 ? 25 : 21; }
template <typename T> constexpr int prop_mat() { return 21 * prop_rs<T>(); }
constexpr int PROP_SC = 104;   // per-sample scalars (PropSample)
enum PropSample { PK_DT = 0, PK_W = 1, PK_A = 4, PK_M1 = 7, PK_M2 = 23, PK_Q = 39, PK_DQ = 43, PK_QN = 47,
                  PK_H = 51, PK_VI = 60, PK_V = 63, PK_P = 66, PK_R = 69, PK_PHI00 = 78, PK_U = 87, PK_S = 90,
                  PK_W1 = 93, PK_W2 = 96 };
// structurally non-zero 3x3 column blocks of each row block (7 bits per row block)
constexpr unsigned long long PM_F = 0x03ull | 0x09ull << 14 | 0x04ull << 28;              // F
constexpr unsigned long long PM_F2 = 0x03ull | 0x03ull << 14 | 0x09ull << 28;             // F^2
constexpr unsigned long long PM_PHI = 0x03ull | 0x02ull << 7 | 0x0Full << 14 | 0x08ull << 21 |
                                      0x1Full << 28 | 0x20ull << 35 | 0x40ull << 42;     // Phi, cumulative Phi

template <typename T>
__host__ __device__ constexpr int prop_lds(int pkc) {   // T per workgroup
    return 7 * prop_mat<T>() + pkc * PROP_SC + IMU_STRIDE;
}
template <typename T> constexpr int prop_pkc() { return sizeof(T) == 4 ? 12 : 10; }

// sum over the blocks of a (compile-time) mask, ascending: x[q] y[q]
template <typename T, int N>
__device__ __forceinline__ T prop_dot(const T* x, const T (&y)[N], unsigned mask) {
    T s = 0;
#pragma unroll
    for (int m = 0; m < 7; ++m)
        if (mask >> m & 1u) {
#pragma unroll
            for (int r = 0; r < 3; ++r) s += x[3 * m + r] * y[3 * m + r];
        }
    return s;
}
template <typename T, int N>
__device__ __forceinline__ T prop_dot(const T (&x)[21], const T (&y)[N], unsigned mask) {
    T s = 0;
#pragma unroll
    for (int m = 0; m < 7; ++m)
        if (mask >> m & 1u) {
#pragma unroll
            for (int r = 0; r < 3; ++r) s += x[3 * m + r] * y[3 * m + r];
        }
    return s;
}
// Phase boundary of the one-wave kernel.  One wave's LDS operations execute in
// issue order, so a lane's read issued after another lane's write sees it: only
// the compiler must not move LDS accesses across the boundary (no hardware wait).
// This holds only for a 64-thread workgroup that is ONE wave: k_propagate is
// launched with blockDim 64 (launch_propagate) and built for wave64 only.
__device__ __forceinline__ void prop_sync() { asm volatile("" ::: "memory"); }
#if defined(__AMDGCN_WAVEFRONT_SIZE) && __AMDGCN_WAVEFRONT_SIZE != 64
#error "k_propagate's phase boundaries (prop_sync) assume a 64-thread workgroup is one wave"
#endif

// Phase timing of k_propagate (probe builds only, `make probe`:
// -DMSCKF_GATE_PROBE; tools/probes/prop_phases.py reads it): per scalar type,
// wave-cycle sums (s_memtime) of the start (P11 load, cross-block prefetch),
// the chunk scalars (A..B4), the per-sample Phi (C1..C3b), the Q term (C4..C5),
// D1, D2, D3, the end (write-back, cross blocks), and the wave count.
#ifdef MSCKF_GATE_PROBE
__device__ unsigned long long g_prop_probe[2][10];
#define PPROBE_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define PPROBE_ADD(ph, dt) \
    do { if (lane == 0) atomicAdd(&g_prop_probe[sizeof(T) == 8][ph], (unsigned long long)(dt)); } while (0)
extern "C" int msckf_prop_probe_read(unsigned long long* out) {   // [2][10], then reset
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prop_probe), sizeof(g_prop_probe)) != hipSuccess) return -1;
    static unsigned long long zero[2][10] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_prop_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#else
#define PPROBE_T(v) (void)0
#define PPROBE_ADD(ph, dt) (void)0
#endif

// Cross-block staging rows (21 values, padded to a 16-byte multiple) and their
// store as rows j0 .. j0 + nj - 1, columns 0..20 of P: 16-byte stores (four
// floats / two doubles per lane, then the last value) instead of one word per
// lane -- 6 (fp32) / 11 (fp64) store instructions per 64 rows instead of 21.
template <typename T> constexpr int prop_xbs() { return sizeof(T) == 4 ? 24 : 22; }
template <typename T>
__device__ __forceinline__ void xb_rows(T* P, int ld, int j0, int nj, const T* xb, int lane) {
    constexpr int NV = 16 / (int)sizeof(T), NF = 21 / NV, NPART = NF + 1, XBS = prop_xbs<T>();
    using V = T __attribute__((ext_vector_type(NV), aligned(sizeof(T))));
    for (int e = lane; e < NPART * nj; e += 64) {
        const int jj = e / NPART, part = e - NPART * jj;
        T* dst = P + (size_t)(j0 + jj) * ld;
        const T* src = xb + jj * XBS;
        if (part < NF) {
            V v;
#pragma unroll
            for (int q = 0; q < NV; ++q) v[q] = src[NV * part + q];
            *reinterpret_cast<V*>(dst + NV * part) = v;
        } else {
            dst[20] = src[20];
        }
    }
}

// One wave per filter: __launch_bounds__(64) with wave64 (see prop_sync) -- the
// phase boundaries are compiler barriers only, which is safe inside one wave.
template <typename T, int PKC>
__global__ void __launch_bounds__(64) k_propagate(DevState<T> st, Params<T> prm, int nfilt,
                                                  const int* __restrict__ filters,
                                                  const int* __restrict__ smp_off,
                                                  const T* __restrict__ samples_all) {
    constexpr int RS = prop_rs<T>(), MAT = prop_mat<T>(), XBS = prop_xbs<T>();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int lane = threadIdx.x;
    const int w = blockIdx.x;
    const int b = filters[w];
    const int n = smp_off[w + 1] - smp_off[w];
    const T* samples = samples_all + 7 * (size_t)smp_off[w];
    if (n <= 0) return;
    PPROBE_T(t_start);
    T* Pa = reinterpret_cast<T*>(smem_raw);  // P11 (ping-pong with Pb)
    T* Pb = Pa + MAT;
    T* cTa = Pb + MAT;                       // (Phi_k ... Phi_1)^T (ping-pong with cTb)
    T* cTb = cTa + MAT;
    T* PH = cTb + MAT;                       // Phi_k
    T* QQ = PH + MAT;                        // F^2, then (Phi G Qc G^T) Phi^T
    T* FP = QQ + MAT;                        // F dt
    T* SK = FP + MAT;                        // [PKC][PROP_SC]
    T* s_imu = SK + PKC * PROP_SC;
    T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax;
    T* imu = st.imu + (size_t)b * IMU_STRIDE;
    const int D = 21 + 6 * st.ncams[b];
    if (lane < IMU_STRIDE) s_imu[lane] = imu[lane];
    for (int e = lane; e < 441; e += 64) {
        const int i = e / 21, j = e - 21 * i;
        Pa[i * RS + j] = P[i * ld + j];
        cTa[i * RS + j] = i == j ? T(1) : T(0);
    }
    // the cross-block columns, prefetched (fp32) once the first chunk's samples
    // are in: vmcnt retires in issue order, so loads issued before the samples'
    // would hold up the first phase instead of hiding behind the chain
    constexpr int NPRE = sizeof(T) == 4 ? 3 : 0;
    T pre[NPRE > 0 ? NPRE : 1][21];
    prop_sync();
    PPROBE_T(t_started);
    PPROBE_ADD(0, t_started - t_start);
#ifdef MSCKF_GATE_PROBE
    unsigned long long t_ph[6] = {0, 0, 0, 0, 0, 0};
#endif
    // matrix phases: lane (g, c), g = lane / 21 the row inside each 3-row block,
    // c = lane % 21 a column
    // lane 63 repeats lane 62's entries (identical values to identical
    // addresses): no lane is masked off, so no phase branches around its loads
    const int le = lane < 63 ? lane : 62;
    const int g = le / 21, c = le - 21 * (le / 21);
    constexpr bool act = true;
    bool symm = false;   // P11 in Pa still needs the last sample's symmetrisation
    for (int k0 = 0; k0 < n; k0 += PKC) {
        const int kc = min(PKC, n - k0);
        PPROBE_T(t_c0);
        // ---- A: one lane per sample ----
        if (lane < kc) {
            T* sk = SK + lane * PROP_SC;
            const T* smp = samples + 7 * (k0 + lane);
            const T dt = smp[0];
            T wg[3], ac[3];
            for (int i = 0; i < 3; ++i) {
                wg[i] = smp[1 + i] - s_imu[I_BG + i];
                ac[i] = smp[4 + i] - s_imu[I_BA + i];
            }
            sk[PK_DT] = dt;
            for (int i = 0; i < 3; ++i) { sk[PK_W + i] = wg[i]; sk[PK_A + i] = ac[i]; }
            const T gn = sqrt(wg[0] * wg[0] + wg[1] * wg[1] + wg[2] * wg[2]);
            const T Om[16] = {0, wg[2], -wg[1], wg[0],
                              -wg[2], 0, wg[0], wg[1],
                              wg[1], -wg[0], 0, wg[2],
                              -wg[0], -wg[1], -wg[2], 0};
            if (gn > T(1e-5)) {
                const T c1 = cos(gn * dt * T(0.5)), s1 = sin(gn * dt * T(0.5)) / gn;
                const T c2 = cos(gn * dt * T(0.25)), s2 = sin(gn * dt * T(0.25)) / gn;
                for (int e = 0; e < 16; ++e) {
                    const T id = (e % 5 == 0) ? T(1) : T(0);
                    sk[PK_M1 + e] = c1 * id + s1 * Om[e];
                    sk[PK_M2 + e] = c2 * id + s2 * Om[e];
                }
            } else {
                const T c1 = cos(gn * dt * T(0.5)), c2 = cos(gn * dt * T(0.25));
                for (int e = 0; e < 16; ++e) {
                    const T id = (e % 5 == 0) ? T(1) : T(0);
                    sk[PK_M1 + e] = c1 * (id + Om[e] * dt * T(0.5));
                    sk[PK_M2 + e] = c2 * (id + Om[e] * dt * T(0.25));
                }
            }
        }
        if (k0 == 0) {
#pragma unroll
            for (int pp = 0; pp < NPRE; ++pp) {
                const int j = 21 + 64 * pp + lane;
#pragma unroll
                for (int m = 0; m < 21; ++m) pre[pp][m] = j < D ? P[m * ld + j] : T(0);
            }
        }
        prop_sync();
        // ---- B1: the quaternion chain (_predict_new_state, jit_utils.py:46-128) ----
        if (lane == 0) {
            T q[4] = {s_imu[I_Q], s_imu[I_Q + 1], s_imu[I_Q + 2], s_imu[I_Q + 3]};
            for (int k = 0; k < kc; ++k) {
                T* sk = SK + k * PROP_SC;
                T dq[4];
                for (int i = 0; i < 4; ++i) {
                    T a1 = 0;
                    for (int j = 0; j < 4; ++j) a1 += sk[PK_M1 + 4 * i + j] * q[j];
                    dq[i] = a1;
                }
                // one division per normalisation on this serial chain (x * (1 / n)
                // instead of x / n: within an ulp of the reference's division)
                const T rq = T(1) / sqrt(dq[0] * dq[0] + dq[1] * dq[1] + dq[2] * dq[2] + dq[3] * dq[3]);
                for (int i = 0; i < 4; ++i) dq[i] *= rq;
                const T rn = T(1) / sqrt(dq[0] * dq[0] + dq[1] * dq[1] + dq[2] * dq[2] + dq[3] * dq[3]);
                for (int i = 0; i < 4; ++i) {
                    sk[PK_Q + i] = q[i];
                    sk[PK_DQ + i] = dq[i];
                    q[i] = dq[i] * rn;
                    sk[PK_QN + i] = q[i];
                }
            }
        }
        prop_sync();
        // ---- B2: rotations and RK4 slopes, one lane per sample ----
        if (lane < kc) {
            T* sk = SK + lane * PROP_SC;
            const T dt = sk[PK_DT];
            const T* gv = s_imu + I_G;
            T q[4], dq[4], dq2[4], acc[3];
            for (int i = 0; i < 4; ++i) { q[i] = sk[PK_Q + i]; dq[i] = sk[PK_DQ + i]; }
            for (int i = 0; i < 3; ++i) acc[i] = sk[PK_A + i];
            for (int i = 0; i < 4; ++i) {
                T a2 = 0;
                for (int j = 0; j < 4; ++j) a2 += sk[PK_M2 + 4 * i + j] * q[j];
                dq2[i] = a2;
            }
            T S1[9];
            skew3(dq, S1);   // reused for dR_dt2 and k1 (Q1)
            T dRT[9], dR2T[9], Rk[9];
            {
                const T ww = dq[3];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)   // transpose stored
                        dRT[3 * j + i] = (i == j ? 2 * ww * ww - 1 : T(0)) - 2 * ww * S1[3 * i + j] + (2 * dq[i]) * dq[j];
            }
            const T nq2 = sqrt(dq2[0] * dq2[0] + dq2[1] * dq2[1] + dq2[2] * dq2[2] + dq2[3] * dq2[3]);
            for (int i = 0; i < 4; ++i) dq2[i] /= nq2;
            {
                const T ww = dq2[3];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        dR2T[3 * j + i] = (i == j ? 2 * ww * ww - 1 : T(0)) - 2 * ww * S1[3 * i + j] + (2 * dq2[i]) * dq2[j];
            }
            const T nq0 = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            const T qn[4] = {q[0] / nq0, q[1] / nq0, q[2] / nq0, q[3] / nq0};
            {
                const T ww = qn[3];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        Rk[3 * i + j] = (i == j ? 2 * ww * ww - 1 : T(0)) - 2 * ww * S1[3 * i + j] + (2 * qn[i]) * qn[j];
            }
            T k1v[3], k2v[3], k3v[3], k4v[3], tmp[3];
            mat3T_vec(Rk, acc, tmp);
            for (int i = 0; i < 3; ++i) k1v[i] = tmp[i] + gv[i];
            mat3_vec(dR2T, acc, tmp);
            for (int i = 0; i < 3; ++i) k2v[i] = tmp[i] + gv[i];
            for (int i = 0; i < 3; ++i) k3v[i] = tmp[i] + gv[i];
            mat3_vec(dRT, acc, tmp);
            for (int i = 0; i < 3; ++i) k4v[i] = tmp[i] + gv[i];
            for (int i = 0; i < 3; ++i) {
                sk[PK_H + i] = k1v[i] * dt / T(2);
                sk[PK_H + 3 + i] = k2v[i] * dt / T(2);
                sk[PK_H + 6 + i] = k3v[i] * dt;
                sk[PK_VI + i] = (k1v[i] + 2 * k2v[i] + 2 * k3v[i] + k4v[i]) * dt / T(6);
            }
            quat_to_rot(q, sk + PK_R);   // R_w_i at the step's start (F, G)
        }
        prop_sync();
        // ---- B3: velocity and position ----
        if (lane == 0) {
            T v[3] = {s_imu[I_V], s_imu[I_V + 1], s_imu[I_V + 2]};
            T p[3] = {s_imu[I_P], s_imu[I_P + 1], s_imu[I_P + 2]};
            for (int k = 0; k < kc; ++k) {
                T* sk = SK + k * PROP_SC;
                const T dt6 = sk[PK_DT] / T(6);   // off the v / p chains
                for (int i = 0; i < 3; ++i) {
                    const T v1 = v[i] + sk[PK_H + i], v2 = v[i] + sk[PK_H + 3 + i], v3 = v[i] + sk[PK_H + 6 + i];
                    const T pn = p[i] + (v[i] + 2 * v1 + 2 * v2 + v3) * dt6;
                    const T vn = v[i] + sk[PK_VI + i];
                    sk[PK_V + i] = vn;
                    sk[PK_P + i] = pn;
                    v[i] = vn;
                    p[i] = pn;
                }
            }
        }
        prop_sync();
        // ---- B4: Phi edit terms (msckf.py:329-344), one lane per sample ----
        if (lane < kc) {
            T* sk = SK + lane * PROP_SC;
            const T* skp = SK + (lane - 1) * PROP_SC;
            const T dt = sk[PK_DT];
            const T* gv = s_imu + I_G;
            T q_null[4], v_null[3], p_null[3];
            if (lane == 0) {   // the record's null state; Q5: entry values once aliased
                const bool alias = s_imu[I_ALIAS] != T(0);
                for (int i = 0; i < 4; ++i) q_null[i] = s_imu[I_QN + i];
                for (int i = 0; i < 3; ++i) {
                    v_null[i] = alias ? s_imu[I_V + i] : s_imu[I_VN + i];
                    p_null[i] = alias ? s_imu[I_P + i] : s_imu[I_PN + i];
                }
            } else {           // the previous sample's result
                for (int i = 0; i < 4; ++i) q_null[i] = skp[PK_QN + i];
                for (int i = 0; i < 3; ++i) { v_null[i] = skp[PK_V + i]; p_null[i] = skp[PK_P + i]; }
            }
            T qk[4], vk[3], pk[3];
            for (int i = 0; i < 4; ++i) qk[i] = sk[PK_QN + i];
            for (int i = 0; i < 3; ++i) { vk[i] = sk[PK_V + i]; pk[i] = sk[PK_P + i]; }
            T Rkk1[9], Rq[9];
            quat_to_rot(q_null, Rkk1);
            quat_to_rot(qk, Rq);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    sk[PK_PHI00 + 3 * i + j] = Rq[3 * i] * Rkk1[3 * j] + Rq[3 * i + 1] * Rkk1[3 * j + 1] + Rq[3 * i + 2] * Rkk1[3 * j + 2];
            T u[3];
            mat3_vec(Rkk1, gv, u);
            const T uu = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
            const T dv[3] = {v_null[0] - vk[0], v_null[1] - vk[1], v_null[2] - vk[2]};
            T Sk[9], w1[3], w2[3];
            skew3(dv, Sk);
            mat3_vec(Sk, gv, w1);
            T dp[3];
            for (int i = 0; i < 3; ++i) dp[i] = dt * v_null[i] + p_null[i] - pk[i];
            skew3(dp, Sk);
            mat3_vec(Sk, gv, w2);
            for (int i = 0; i < 3; ++i) {
                sk[PK_U + i] = u[i];
                sk[PK_S + i] = u[i] / uu;
                sk[PK_W1 + i] = w1[i];
                sk[PK_W2 + i] = w2[i];
            }
        }
        prop_sync();
        if (lane == 0) {   // the record after the chunk
            const T* sk = SK + (kc - 1) * PROP_SC;
            for (int i = 0; i < 4; ++i) { s_imu[I_Q + i] = sk[PK_QN + i]; s_imu[I_QN + i] = sk[PK_QN + i]; }
            for (int i = 0; i < 3; ++i) {
                s_imu[I_V + i] = sk[PK_V + i]; s_imu[I_VN + i] = sk[PK_V + i];
                s_imu[I_P + i] = sk[PK_P + i]; s_imu[I_PN + i] = sk[PK_P + i];
            }
            s_imu[I_ALIAS] = T(1);
        }
        prop_sync();
#ifdef MSCKF_GATE_PROBE
        { PPROBE_T(t_c1); t_ph[0] += t_c1 - t_c0; }
#endif
        for (int k = 0; k < kc; ++k) {
            PPROBE_T(t_s0);
            const T* sk = SK + k * PROP_SC;
            const T dt = sk[PK_DT];
            const T* R = sk + PK_R;
            // ---- C1: F dt (jit_utils.py:25-34), rows 3 rb + g of column c ----
            T fo[7] = {0, 0, 0, 0, 0, 0, 0};
            if (act) {
                const int bj = c / 3, cc = c - 3 * (c / 3);
                const T* wg = sk + PK_W;
                const T* ac = sk + PK_A;
                // every operand loaded, then selected: no branch around an LDS read
                const T f0 = bj == 0 ? -skew_sel(wg, g, cc) : (bj == 1 ? (g == cc ? T(-1) : T(0)) : T(0));
                const T f2a = -R[g] * skew_sel(ac, 0, cc) + -R[3 + g] * skew_sel(ac, 1, cc) + -R[6 + g] * skew_sel(ac, 2, cc);
                const T f2b = -R[3 * cc + g];
                const T f2 = bj == 0 ? f2a : (bj == 3 ? f2b : T(0));
                const T f4 = (bj == 2 && g == cc) ? T(1) : T(0);
                fo[0] = f0 * dt;
                fo[2] = f2 * dt;
                fo[4] = f4 * dt;
#pragma unroll
                for (int rb = 0; rb < 7; ++rb) FP[(3 * rb + g) * RS + c] = fo[rb];
            }
            prop_sync();
            // ---- C2: F^2 ----
            T fcol[12];   // F[q][c], q < 12 (F^2 and F^3 only reach these rows)
#pragma unroll
            for (int q = 0; q < 12; ++q) fcol[q] = act ? FP[q * RS + c] : T(0);
            T f2o[7];
#pragma unroll
            for (int rb = 0; rb < 7; ++rb) {
                const unsigned m = (unsigned)(PM_F >> (7 * rb)) & 0x7fu;
                f2o[rb] = m ? prop_dot(FP + (3 * rb + g) * RS, fcol, m) : T(0);
            }
            prop_sync();   // every lane has read F before FP is reused
            if (act) {
#pragma unroll
                for (int rb = 0; rb < 7; ++rb) QQ[(3 * rb + g) * RS + c] = f2o[rb];
            }
            prop_sync();
            // ---- C3: Phi = I + F + F^2/2 + F^3/6, Phi[0:3, 0:3] edit ----
            if (act) {
#pragma unroll
                for (int rb = 0; rb < 7; ++rb) {
                    const int i = 3 * rb + g;
                    const unsigned m = (unsigned)(PM_F2 >> (7 * rb)) & 0x7fu;
                    const T s3 = m ? prop_dot(QQ + i * RS, fcol, m) : T(0);
                    // F^3 / 6 as a multiply by 1/6 (within an ulp of the division; the
                    // IEEE division sequence sat on every sample's chain)
                    T ph = (i == c ? T(1) : T(0)) + fo[rb] + f2o[rb] / T(2) + s3 * T(1.0 / 6.0);
                    if (rb == 0 && c < 3) ph = sk[PK_PHI00 + 3 * g + c];
                    PH[i * RS + c] = ph;
                }
            }
            prop_sync();
            // ---- C3b: rows 6..8 and 12..14, columns 0..2 (msckf.py:339-344) ----
            if (c < 3 && act) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int i = (e == 0 ? 6 : 12) + g;
                    const T* wvv = sk + (e == 0 ? PK_W1 : PK_W2);
                    const T a1[3] = {PH[i * RS], PH[i * RS + 1], PH[i * RS + 2]};
                    const T au = a1[0] * sk[PK_U] + a1[1] * sk[PK_U + 1] + a1[2] * sk[PK_U + 2];
                    const T cc = au - wvv[g];
                    const T val = a1[c] - cc * sk[PK_S + c];
                    asm volatile("" ::: "memory");   // all lanes read the row before it is edited
                    PH[i * RS + c] = val;
                }
            }
            prop_sync();
#ifdef MSCKF_GATE_PROBE
            PPROBE_T(t_s1);
            t_ph[1] += t_s1 - t_s0;
#endif
            // this lane's rows 3 rb + g of Phi (non-zero blocks only): C5, D1 and D2 use them
            T phr[7][21];
#pragma unroll
            for (int rb = 0; rb < 7; ++rb) {
                const unsigned m = (unsigned)(PM_PHI >> (7 * rb)) & 0x7fu;
#pragma unroll
                for (int q = 0; q < 21; ++q)
                    phr[rb][q] = (m >> (q / 3) & 1u) && act ? PH[(3 * rb + g) * RS + q] : T(0);
            }
            // ---- C4 + C5: Q term row c: (Phi G Qc G^T)[c][q] Phi[j][q], j = 3 jb + g.
            // Every lane forms all of row c of Phi G Qc (G: jit_utils.py:30-34) from
            // row c of Phi itself -- 12 entries, no exchange through LDS ----
            if (act) {
                const T* ph = PH + c * RS;
                T pg[12];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    pg[r] = ph[r] * T(-1) * prm.qc_gyro;
                    pg[3 + r] = ph[3 + r] * T(1) * prm.qc_gbias;
                    pg[6 + r] = (ph[6] * -R[3 * r] + ph[7] * -R[3 * r + 1] + ph[8] * -R[3 * r + 2]) * prm.qc_acc;
                    pg[9 + r] = ph[9 + r] * T(1) * prm.qc_abias;
                }
                T fr[12];
#pragma unroll
                for (int q = 0; q < 12; ++q) {
                    const int r = q - 6;
                    if (q < 3) fr[q] = pg[q] * T(-1);
                    else if (q >= 6 && q < 9) fr[q] = pg[6] * -R[r] + pg[7] * -R[3 + r] + pg[8] * -R[6 + r];
                    else fr[q] = pg[q] * T(1);
                }
#pragma unroll
                for (int jb = 0; jb < 7; ++jb) {
                    const int j = 3 * jb + g;
                    const unsigned m = ((unsigned)(PM_PHI >> (7 * jb)) & 0x7fu) & 0x0Fu;   // G^T rows >= 12 are zero
                    QQ[c * RS + j] = m ? prop_dot(phr[jb], fr, m) : T(0);
                }
            }
            prop_sync();
#ifdef MSCKF_GATE_PROBE
            PPROBE_T(t_s2);
            t_ph[2] += t_s2 - t_s1;
#endif
            // ---- D1: A = Phi P11 (column c), cumulative Phi (row c of its transpose) ----
            if (act) {
                T prow[21], crow[21];
                // P11 = (P11' + P11'^T) / 2 (msckf.py:362-363) of the previous sample,
                // formed as it is read (row c = column c) instead of in a phase of its
                // own; the launch's first sample reads P11 as loaded
                if (symm) {
#pragma unroll
                    for (int q = 0; q < 21; ++q) prow[q] = (Pa[c * RS + q] + Pa[q * RS + c]) / T(2);
                } else {
#pragma unroll
                    for (int q = 0; q < 21; ++q) prow[q] = Pa[c * RS + q];
                }
#pragma unroll
                for (int q = 0; q < 21; ++q) crow[q] = cTa[c * RS + q];
#pragma unroll
                for (int rb = 0; rb < 7; ++rb) {
                    const int i = 3 * rb + g;
                    const unsigned m = (unsigned)(PM_PHI >> (7 * rb)) & 0x7fu;
                    Pb[i * RS + c] = prop_dot(phr[rb], prow, m);
                    cTb[c * RS + i] = prop_dot(phr[rb], crow, m);
                }
            }
            prop_sync();
#ifdef MSCKF_GATE_PROBE
            PPROBE_T(t_s3);
            t_ph[3] += t_s3 - t_s2;
#endif
            // ---- D2: A Phi^T + Q dt (row c) ----
            if (act) {
                T arow[21];
#pragma unroll
                for (int q = 0; q < 21; ++q) arow[q] = Pb[c * RS + q];
#pragma unroll
                for (int jb = 0; jb < 7; ++jb) {
                    const int j = 3 * jb + g;
                    const unsigned m = (unsigned)(PM_PHI >> (7 * jb)) & 0x7fu;
                    Pa[c * RS + j] = prop_dot(phr[jb], arow, m) + QQ[c * RS + j] * dt;
                }
            }
            prop_sync();
#ifdef MSCKF_GATE_PROBE
            PPROBE_T(t_s4);
            t_ph[4] += t_s4 - t_s3;
#endif
#ifdef MSCKF_GATE_PROBE
            PPROBE_T(t_s5);
            t_ph[5] += t_s5 - t_s4;
#endif
            symm = true;
            T* t = cTa; cTa = cTb; cTb = t;   // P11' stays in Pa, A in Pb
        }
    }
    PPROBE_T(t_end0);
#ifdef MSCKF_GATE_PROBE
    for (int q = 0; q < 6; ++q) PPROBE_ADD(1 + q, t_ph[q]);
#endif
    // write back P11 and the IMU record; the cross blocks with the cumulative Phi
    for (int e = lane; e < 441; e += 64) {
        const int i = e / 21, j = e - 21 * i;
        P[i * ld + j] = (Pa[i * RS + j] + Pa[j * RS + i]) / T(2);   // the last sample's symmetrisation
        PH[i * RS + j] = cTa[j * RS + i];   // cumulative Phi, row-major
    }
    if (lane < IMU_STRIDE) imu[lane] = s_imu[lane];
    prop_sync();
    // The IMU x cam cross block P[0:21, 21:D] <- Phi_cum P[0:21, 21:D] (and its
    // transpose), 64 cam columns per chunk, on MFMA tiles (v_mfma_f32_16x16x4f32 /
    // v_mfma_f64_16x16x4f64).  Phi_cum = Phi_n ... Phi_1 differs from I only in row
    // blocks 0, 2, 4 (rows 0-2, 6-8, 12-14), whose non-zeros lie in columns 0..14
    // (PM_PHI): the A operand is those nine rows (padded to 16) over K = 0..15, the
    // B operand the chunk's rows 0..15 staged in LDS as [column][17], four 16-column
    // tiles per chunk; the identity rows are copies.  The results go through the
    // [column][XBS] staging rows (aliasing the B stage: every MFMA operand is read
    // before the first staging write, one wave's LDS operations run in order) to
    // row-major stores of both halves.
    T* xb = reinterpret_cast<T*>(smem_raw);   // [64][XBS] staging rows; the B stage [64][17] first
    static_assert(4 * MAT >= 64 * XBS && 4 * MAT >= 64 * 17, "cross-block staging");
    using XV4 = typename GM<T>::V4;
    constexpr int XRS = GM<T>::RS, XRG = GM<T>::RG;
    const int l15 = lane & 15, lg = lane >> 4;
    const int arow = l15 < 9 ? 6 * (l15 / 3) + l15 % 3 : 0;   // rows 0-2, 6-8, 12-14 of Phi_cum
    T aop[4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const int k = 4 * kk + lg;
        const bool nz = l15 < 9 && k < 15 && ((PM_PHI >> (7 * (arow / 3) + k / 3)) & 1ull);
        aop[kk] = nz ? PH[arow * RS + k] : T(0);
    }
    auto cross_chunk = [&](int j0, const T (&col)[21]) {
        const bool in = j0 + lane < D;
        T* S = xb;
#pragma unroll
        for (int k = 0; k < 16; ++k) S[lane * 17 + k] = (in && k < 15) ? col[k] : T(0);
        prop_sync();
        // one 16-column tile at a time (four accumulator registers: the kernel sits at
        // two waves per SIMD with ~240 VGPRs); the B operands of all four tiles are
        // read before the first staging write
        T bop[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) bop[t][kk] = S[(16 * t + l15) * 17 + 4 * kk + lg];
        prop_sync();
#pragma unroll
        for (int m = 0; m < 21; ++m)
            if ((m / 3) & 1 || m >= 15) xb[lane * XBS + m] = col[m];   // identity rows
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            XV4 acc = XV4{0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) acc = GM<T>::mfma(aop[kk], bop[t][kk], acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = XRG * lg + XRS * i;
                if (r < 9) xb[(16 * t + l15) * XBS + 6 * (r / 3) + r % 3] = acc[i];
            }
        }
        prop_sync();
        if (in) {
#pragma unroll
            for (int i = 0; i < 21; ++i) P[i * ld + j0 + lane] = xb[lane * XBS + i];
        }
        xb_rows(P, ld, j0, min(64, D - j0), xb, lane);
        prop_sync();
    };
#pragma unroll
    for (int pp = 0; pp < NPRE + 1; ++pp) {
        if (pp == NPRE) break;
        if (21 + 64 * pp >= D) break;
        cross_chunk(21 + 64 * pp, pre[pp]);
    }
    for (int j0 = 21 + 64 * NPRE; j0 < D; j0 += 64) {
        const int j = j0 + lane;
        T col[21];
#pragma unroll
        for (int m = 0; m < 21; ++m) col[m] = j < D ? P[m * ld + j] : T(0);
        cross_chunk(j0, col);
    }
    PPROBE_T(t_end1);
    PPROBE_ADD(7, t_end1 - t_end0);
    PPROBE_ADD(8, t_end1 - t_start);
    PPROBE_ADD(9, 1);
}

// ===========================================================================
// State augmentation: one workgroup per listed filter.
// ===========================================================================
template <typename T>
__global__ void __launch_bounds__(256) k_augment(DevState<T> st, const int* __restrict__ filters) {
    __shared__ T J[6 * 21];
    __shared__ T X[36];
    const int tid = threadIdx.x;
    const int b = filters[blockIdx.x];
    T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax;
    const T* imu = st.imu + (size_t)b * IMU_STRIDE;
    const int nc = st.ncams[b];
    const int D = 21 + 6 * nc;
    if (tid == 0) {
        T Rwi[9], Rwc[9], t[3], q[4];
        quat_to_rot(imu + I_Q, Rwi);
        const T* Ric = imu + I_RIC;
        mat3_mul(Ric, Rwi, Rwc);
        mat3T_vec(Rwi, imu + I_TCI, t);          // R_w_i^T t_c_i
        rot_to_quat(Rwc, q);
        T* cam = st.cams + ((size_t)b * st.Nmax + nc) * CAM_STRIDE;
        for (int i = 0; i < 4; ++i) { cam[C_Q + i] = q[i]; cam[C_QN + i] = q[i]; }
        for (int i = 0; i < 3; ++i) cam[C_P + i] = imu[I_P + i] + t[i];
        for (int e = 0; e < 126; ++e) J[e] = 0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) J[21 * i + j] = Ric[3 * i + j];
        for (int i = 0; i < 3; ++i) J[21 * i + 15 + i] = 1;
        T Sk[9];
        skew3(t, Sk);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) J[21 * (3 + i) + j] = Sk[3 * i + j];
        for (int i = 0; i < 3; ++i) { J[21 * (3 + i) + 12 + i] = 1; J[21 * (3 + i) + 18 + i] = 1; }
    }
    __syncthreads();
    for (int j = tid; j < D; j += blockDim.x) {      // J P[0:21, j]
        T col[21];
        for (int m = 0; m < 21; ++m) col[m] = P[m * ld + j];
        for (int r = 0; r < 6; ++r) {
            T s = 0;
            for (int m = 0; m < 21; ++m) s += J[21 * r + m] * col[m];
            P[(size_t)(D + r) * ld + j] = s;
            P[(size_t)j * ld + D + r] = s;
        }
    }
    if (tid < 36) {                                  // J P11 J^T
        int r = tid / 6, c = tid % 6;
        T s = 0;
        for (int m = 0; m < 21; ++m) {
            T jp = 0;
            for (int l = 0; l < 21; ++l) jp += J[21 * r + l] * P[l * ld + m];
            s += jp * J[21 * c + m];
        }
        X[tid] = s;
    }
    __syncthreads();
    if (tid < 36) {
        int r = tid / 6, c = tid % 6;
        P[(size_t)(D + r) * ld + D + c] = (X[tid] + X[c * 6 + r]) / T(2);
    }
    if (tid == 0) st.ncams[b] = nc + 1;
}

// ===========================================================================
// P compaction (msckf.py:803-818), in place: one workgroup per listed filter.
// P'[i][j] = P[keep[i]][keep[j]] with keep ascending, so keep[i] >= i: rows
// are moved in chunks of R through LDS, every read of a chunk before any of
// its writes -- a later chunk only reads rows keep[i'] >= i' that no earlier
// chunk has written.  keep_off / kcam_off delimit each filter's kept indices
// (error-state rows; cam slots) in the concatenated lists.
// ===========================================================================
template <typename T>
__global__ void __launch_bounds__(256) k_prune(DevState<T> st, const int* __restrict__ filters,
                                               const int* __restrict__ keep_off, const int* __restrict__ keep_all,
                                               const int* __restrict__ kcam_off,
                                               const int* __restrict__ keep_cams_all, int R) {
    extern __shared__ unsigned char prune_lds[];
    T* buf = reinterpret_cast<T*>(prune_lds);          // [R][Dn]
    const int b = filters[blockIdx.x];
    const int* keep = keep_all + keep_off[blockIdx.x];
    const int Dn = keep_off[blockIdx.x + 1] - keep_off[blockIdx.x];
    T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax;
    for (int i0 = 0; i0 < Dn; i0 += R) {
        const int nr = min(R, Dn - i0);
        for (int e = threadIdx.x; e < nr * Dn; e += blockDim.x) {
            const int r = e / Dn, j = e - r * Dn;
            buf[e] = P[(size_t)keep[i0 + r] * ld + keep[j]];
        }
        __syncthreads();
        for (int e = threadIdx.x; e < nr * Dn; e += blockDim.x) {
            const int r = e / Dn, j = e - r * Dn;
            P[(size_t)(i0 + r) * ld + j] = buf[e];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int* keep_cams = keep_cams_all + kcam_off[blockIdx.x];
        const int nkeep = kcam_off[blockIdx.x + 1] - kcam_off[blockIdx.x];
        T* cams = st.cams + (size_t)b * st.Nmax * CAM_STRIDE;
        for (int c = 0; c < nkeep; ++c) {   // keep_cams ascending, in-place forward copy
            const int src = keep_cams[c];
            if (src != c)
                for (int e = 0; e < CAM_STRIDE; ++e) cams[c * CAM_STRIDE + e] = cams[src * CAM_STRIDE + e];
        }
        st.ncams[b] = nkeep;
    }
}

// Covariance diagonal entries [i0, i0 + n) of the listed filters (online
// reset, msckf.py:869-871), out[w * n + k].
template <typename T>
__global__ void k_cov_diag(DevState<T> st, const int* __restrict__ filters, int nfilt, int i0, int n,
                           T* __restrict__ out) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nfilt * n) return;
    const int w = e / n, k = i0 + e % n;
    out[e] = st.P[(size_t)filters[w] * st.Dmax * st.Dmax + (size_t)k * st.Dmax + k];
}

// ===========================================================================
// Triangulation: one wavefront per feature, the 2M views spread over the 64
// lanes (<= 4 per lane), LM sums reduced with xor-shuffles so every lane holds
// bit-identical totals and runs the (scalar) LM control flow redundantly.
// ===========================================================================
// Sum over aligned S-lane segments of the wavefront (xor shuffles stay inside
// a segment for offsets < S).
template <int S, typename T>
__device__ __forceinline__ T seg_sum(T x) {
#pragma unroll
    for (int m = S >> 1; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

// views per lane: S lanes per feature (the k_feature segment classes, M <= S
// for S < 128) hold 2M views, VPL = 2 (VPL = 4 in the 64-lane class that
// takes 64 < M <= 128)

template <typename T>
__device__ __forceinline__ void lu3_solve(T A[9], T b[3], T x[3]) {
    // dgesv-style partial pivoting on a 3x3 system.
    int piv[3] = {0, 1, 2};
    for (int k = 0; k < 3; ++k) {
        int p = k;
        T m = fabs(A[3 * k + k]);
        for (int i = k + 1; i < 3; ++i)
            if (fabs(A[3 * i + k]) > m) { m = fabs(A[3 * i + k]); p = i; }
        if (p != k) {
            for (int j = 0; j < 3; ++j) { T t = A[3 * k + j]; A[3 * k + j] = A[3 * p + j]; A[3 * p + j] = t; }
            T t = b[k]; b[k] = b[p]; b[p] = t;
            int ti = piv[k]; piv[k] = piv[p]; piv[p] = ti;
        }
        for (int i = k + 1; i < 3; ++i) {
            T l = A[3 * i + k] / A[3 * k + k];
            A[3 * i + k] = l;
            for (int j = k + 1; j < 3; ++j) A[3 * i + j] -= l * A[3 * k + j];
            b[i] -= l * b[k];
        }
    }
    for (int i = 2; i >= 0; --i) {
        T s = b[i];
        for (int j = i + 1; j < 3; ++j) s -= A[3 * i + j] * x[j];
        x[i] = s / A[3 * i + i];
    }
}

template <typename T, int S, int TRI_VPL>
__global__ void __launch_bounds__(256) k_triangulate(DevState<T> st, Params<T> prm, FeatBatch<T> fb,
                                                     const int* __restrict__ flist, int cnt) {
    // S-lane segment per feature, 64 / S features per wavefront; every lane of
    // a segment runs the (scalar) LM control flow on bit-identical segment sums
    constexpr int PER = 64 / S;
    const int lane = threadIdx.x & 63, sl0 = lane & ~(S - 1);
    const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wid * PER >= cnt) return;
    const int li = wid * PER + lane / S;
    const bool active = li < cnt;
    const int f = flist[active ? li : cnt - 1];
    const int b = fb.feat_filter[f];
    const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
    const int nv = 2 * M;
    const T* cams = st.cams + (size_t)b * st.Nmax * CAM_STRIDE;
    // T_c1_c0 = Iso(R01, t01).inverse()
    T R10[9], t10[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R10[3 * i + j] = prm.R01[3 * j + i];
    {
        T tmp[3];
        mat3_vec(R10, prm.t01, tmp);
        for (int i = 0; i < 3; ++i) t10[i] = -tmp[i];
    }
    // pose of view v (cam -> world): cam0 = (R_wc^T, p); cam1 = cam0 * T_c1_c0
    auto view_pose = [&](int v, T* R, T* t) {
        const T* c = cams + (size_t)fb.obs_cam[o0 + (v >> 1)] * CAM_STRIDE;
        T Rwc[9];
        quat_to_rot(c + C_Q, Rwc);
        T R0[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R0[3 * i + j] = Rwc[3 * j + i];
        if ((v & 1) == 0) {
            for (int e = 0; e < 9; ++e) R[e] = R0[e];
            for (int i = 0; i < 3; ++i) t[i] = c[C_P + i];
        } else {
            mat3_mul(R0, R10, R);
            T tmp[3];
            mat3_vec(R0, t10, tmp);
            for (int i = 0; i < 3; ++i) t[i] = tmp[i] + c[C_P + i];
        }
    };
    T R0w[9], t0w[3];
    view_pose(0, R0w, t0w);   // T_c0_w
    // relative poses T_v = pose_v^-1 * T_c0_w (feature.py:209-213)
    T VR[TRI_VPL][9], Vt[TRI_VPL][3], Vz[TRI_VPL][2];
#pragma unroll
    for (int s = 0; s < TRI_VPL; ++s) {
        int v = (lane & (S - 1)) + S * s;
        if (v < nv) {
            T R[9], t[3];
            view_pose(v, R, t);
            T RT[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) RT[3 * i + j] = R[3 * j + i];
            mat3_mul(RT, R0w, VR[s]);
            T a[3], c[3];
            mat3_vec(RT, t0w, a);
            mat3_vec(RT, t, c);
            for (int i = 0; i < 3; ++i) Vt[s][i] = a[i] + -c[i];
            const T* z = fb.obs_z + (size_t)(o0 + (v >> 1)) * 4 + 2 * (v & 1);
            Vz[s][0] = z[0];
            Vz[s][1] = z[1];
        } else {
            for (int e = 0; e < 9; ++e) VR[s][e] = 0;
            for (int i = 0; i < 3; ++i) Vt[s][i] = 0;
            Vz[s][0] = Vz[s][1] = 0;
        }
    }
    // initial guess from view 0 and the LAST cam0 view (nv-2)  (feature.py:99-122, 216-218)
    T x[3];
    {
        int vl = nv - 2, sl = vl / S, ll = sl0 + (vl & (S - 1));
        T R12[9], t12[3], z2[2], z1[2];
        // broadcast view vl's transform from its lane (static slot index)
        for (int e = 0; e < 9; ++e) {
            T val = VR[0][e];
#pragma unroll
            for (int s = 1; s < TRI_VPL; ++s) val = (sl == s) ? VR[s][e] : val;
            R12[e] = __shfl(val, ll, 64);
        }
        for (int i = 0; i < 3; ++i) {
            T val = Vt[0][i];
#pragma unroll
            for (int s = 1; s < TRI_VPL; ++s) val = (sl == s) ? Vt[s][i] : val;
            t12[i] = __shfl(val, ll, 64);
        }
        for (int i = 0; i < 2; ++i) {
            T val = Vz[0][i];
#pragma unroll
            for (int s = 1; s < TRI_VPL; ++s) val = (sl == s) ? Vz[s][i] : val;
            z2[i] = __shfl(val, ll, 64);
            z1[i] = __shfl(Vz[0][i], sl0, 64);
        }
        T z1h[3] = {z1[0], z1[1], T(1)};
        T m[3];
        mat3_vec(R12, z1h, m);
        T a0 = m[0] - z2[0] * m[2], a1 = m[1] - z2[1] * m[2];
        T b0 = z2[0] * t12[2] - t12[0], b1 = z2[1] * t12[2] - t12[1];
        T depth = (a0 * b0 + a1 * b1) / (a0 * a0 + a1 * a1);
        T p0[3] = {z1[0] * depth, z1[1] * depth, depth};
        x[0] = p0[0] / p0[2];
        x[1] = p0[1] / p0[2];
        x[2] = T(1) / p0[2];
    }
    auto total_cost = [&](const T* xx) {
        T c = 0;
#pragma unroll
        for (int s = 0; s < TRI_VPL; ++s) {
            if ((lane & (S - 1)) + S * s < nv) {
                T h[3];
                for (int i = 0; i < 3; ++i)
                    h[i] = VR[s][3 * i] * xx[0] + VR[s][3 * i + 1] * xx[1] + VR[s][3 * i + 2] + xx[2] * Vt[s][i];
                T e0 = h[0] / h[2] - Vz[s][0], e1 = h[1] / h[2] - Vz[s][1];
                c += e0 * e0 + e1 * e1;
            }
        }
        return seg_sum<S>(c);
    };
    // valid == 2: position given by the host -- never re-triangulated, so the
    // segment skips the LM iterations (segment-uniform: f is the segment's)
    const bool given = fb.valid[f] == 2;
    T lam = prm.damping;
    T cost = total_cost(x);
    bool reduced = false;
    T dnorm = T(INFINITY);
    int outer = 0;
    while (!given && outer < prm.outer_max && dnorm > prm.precision) {
        // Q2: once a step has been accepted the inner loop never runs again and
        // the solution cannot change any more -> done.
        if (reduced) break;
        T A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bb[3] = {0, 0, 0};
#pragma unroll
        for (int s = 0; s < TRI_VPL; ++s) {
            if ((lane & (S - 1)) + S * s < nv) {
                T h[3];
                for (int i = 0; i < 3; ++i)
                    h[i] = VR[s][3 * i] * x[0] + VR[s][3 * i + 1] * x[1] + VR[s][3 * i + 2] + x[2] * Vt[s][i];
                T W[9];
                for (int i = 0; i < 3; ++i) { W[3 * i] = VR[s][3 * i]; W[3 * i + 1] = VR[s][3 * i + 1]; W[3 * i + 2] = Vt[s][i]; }
                T J[6];
                for (int j = 0; j < 3; ++j) {
                    J[j] = W[j] / h[2] - W[6 + j] * h[0] / (h[2] * h[2]);
                    J[3 + j] = W[3 + j] / h[2] - W[6 + j] * h[1] / (h[2] * h[2]);
                }
                T r0 = h[0] / h[2] - Vz[s][0], r1 = h[1] / h[2] - Vz[s][1];
                T e = sqrt(r0 * r0 + r1 * r1);
                T w = e <= prm.huber ? T(1) : prm.huber / (2 * e);
                T w2 = w * w;
                for (int i = 0; i < 3; ++i) {
                    for (int j = 0; j < 3; ++j) A[3 * i + j] += (w2 * J[i]) * J[j] + (w2 * J[3 + i]) * J[3 + j];
                    bb[i] += (w2 * J[i]) * r0 + (w2 * J[3 + i]) * r1;
                }
            }
        }
        for (int e = 0; e < 9; ++e) A[e] = seg_sum<S>(A[e]);
        for (int e = 0; e < 3; ++e) bb[e] = seg_sum<S>(bb[e]);
        int inner = 0;
        while (inner < prm.inner_max && !reduced) {
            T Al[9], bl[3], delta[3];
            for (int e = 0; e < 9; ++e) Al[e] = A[e];
            Al[0] += lam; Al[4] += lam; Al[8] += lam;
            for (int e = 0; e < 3; ++e) bl[e] = bb[e];
            lu3_solve(Al, bl, delta);
            T xn[3] = {x[0] - delta[0], x[1] - delta[1], x[2] - delta[2]};
            dnorm = sqrt(delta[0] * delta[0] + delta[1] * delta[1] + delta[2] * delta[2]);
            T nc = total_cost(xn);
            if (nc < cost) {
                reduced = true;
                x[0] = xn[0]; x[1] = xn[1]; x[2] = xn[2];
                cost = nc;
                lam = fmax(lam / T(10), T(1e-10));
            } else {
                reduced = false;
                lam = fmin(lam * T(10), T(1e12));
            }
            ++inner;
        }
        ++outer;
    }
    T pf[3] = {x[0] / x[2], x[1] / x[2], T(1) / x[2]};
    bool ok = true;
#pragma unroll
    for (int s = 0; s < TRI_VPL; ++s) {
        if ((lane & (S - 1)) + S * s < nv) {
            T z = VR[s][6] * pf[0] + VR[s][7] * pf[1] + VR[s][8] * pf[2] + Vt[s][2];
            if (z <= 0) ok = false;
        }
    }
    {   // every view of the segment in front of the camera
        const unsigned long long bad = __ballot(!ok);
        const unsigned long long segmask = S == 64 ? ~0ull : (((1ull << S) - 1) << sl0);
        ok = (bad & segmask) == 0;
    }
    if ((lane & (S - 1)) == 0 && active && !given) {
        T pw[3];
        mat3_vec(R0w, pf, pw);
        for (int i = 0; i < 3; ++i) fb.p_w[3 * f + i] = pw[i] + t0w[i];
        fb.valid[f] = ok ? 1 : 0;
    }
}

// ===========================================================================
// Feature Jacobian + left-nullspace projection: one S-lane segment of a
// wavefront per feature (64/S features per wavefront, S = 8..64 by size class
// so short tracks do not leave most lanes idle); lane l of the segment owns
// observations l and, for 64 < M <= 128, l + 64 (a feature is seen at most
// once per cam state; the cam capacity is <= 128).  Computes the observability-projected
// 4x6 / 4x3 blocks and residual, Householder-QRs H_f (4M x 3) across the wave
// with xor-shuffle reductions (LAPACK dlarfg sign convention), and stores
//   * in T, for gating: the compact factors of H0 = (Q^T Hx)[3:] =
//     (Hx - V diag(tau) W^T)[3:] plus Q^T r                       (obs_ws, tau)
//   * in fp64, for the information assembly: G_i (the observation's columns
//     of the top 3 rows of Q^T Hx), Hx_i^T Hx_i and Hx_i^T r_i - G_i^T g  (obs_g)
// The whole kernel computes in fp64 (CT) whatever T is: the Gram identity
// H0^T H0 = sum_i Hx_i^T Hx_i - G^T G cancels the feature-position directions,
// and only an fp64 projection keeps the gauge (unobservable) directions of the
// assembled information at rounding level.
// The nullspace basis differs from the reference's SVD basis by an orthogonal
// transform, to which gating and the update are invariant (quirk Q4).
// ===========================================================================

// Store n (even) values as 2-element vectors (8-byte float2 / 16-byte double2
// stores; rows of obs_ws / obs_g keep that alignment).
template <typename T, typename S>
__device__ __forceinline__ void store_pairs(T* dst, const S* src, int n) {
    using V2 = T __attribute__((ext_vector_type(2)));
    V2* d = reinterpret_cast<V2*>(dst);
    for (int e = 0; e < n; e += 2) {
        V2 v;
        v.x = (T)src[e];
        v.y = (T)src[e + 1];
        d[e >> 1] = v;
    }
}

// (one observation per lane: three waves per SIMD -- 168 VGPRs, a 12-byte spill)
// GRAM: also write the per-observation Gram records (obs_g) for the
// record-reading assembly; the fused assembly (k_info_fused) rebuilds them
// from the Jacobians and needs only the per-feature QR record (fqr).
template <typename T, int S, int OPL, bool GRAM>
__global__ void __launch_bounds__(256, OPL == 1 ? 3 : 1) k_feature(DevState<T> st, Params<T> prm, FeatBatch<T> fb,
                                                 const int* __restrict__ flist, int cnt) {
    using CT = double;
    constexpr int PER = 64 / S;   // features per wavefront, one S-lane segment each
    const int lane = threadIdx.x & 63, l = lane & (S - 1), b0 = lane & ~(S - 1);
    const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wid * PER >= cnt) return;
    const int li = wid * PER + lane / S;
    const int f = li < cnt ? flist[li] : 0;
    const bool fvalid = li < cnt && fb.valid[f];
    const int b = fb.feat_filter[f];
    const int o0 = fb.obs_off[f], M = fvalid ? fb.obs_off[f + 1] - o0 : 0;
    const T* cams = st.cams + (size_t)b * st.Nmax * CAM_STRIDE;
    CT g[3], R01[9], t01[3];
    for (int k = 0; k < 3; ++k) {
        g[k] = (CT)st.imu[(size_t)b * IMU_STRIDE + I_G + k];
        t01[k] = (CT)prm.t01[k];
    }
    for (int k = 0; k < 9; ++k) R01[k] = (CT)prm.R01[k];
    const CT pw[3] = {(CT)fb.p_w[3 * f], (CT)fb.p_w[3 * f + 1], (CT)fb.p_w[3 * f + 2]};
    // observation i = l + S s of the feature lives in slot s of segment lane l
    CT Hx[OPL][24], Hf[OPL][12], r[OPL][4], u6[OPL][6];
#pragma unroll
    for (int s = 0; s < OPL; ++s) {
        const int i = l + S * s;
        const bool own = i < M;
        for (int e = 0; e < 24; ++e) Hx[s][e] = 0;
        for (int e = 0; e < 12; ++e) Hf[s][e] = 0;
        for (int e = 0; e < 4; ++e) r[s][e] = 0;
        if (own) {
            const T* c = cams + (size_t)fb.obs_cam[o0 + i] * CAM_STRIDE;
            const T* z = fb.obs_z + (size_t)(o0 + i) * 4;
            CT q0[4], qn[4], cp[3];
            for (int k = 0; k < 4; ++k) { q0[k] = (CT)c[C_Q + k]; qn[k] = (CT)c[C_QN + k]; }
            for (int k = 0; k < 3; ++k) cp[k] = (CT)c[C_P + k];
            CT R0[9], R1[9], t1[3], tmp[3];
            quat_to_rot(q0, R0);
            mat3_mul(R01, R0, R1);
            mat3T_vec(R1, t01, tmp);
            for (int k = 0; k < 3; ++k) t1[k] = cp[k] - tmp[k];
            CT d0[3], d1[3], pc0[3], pc1[3];
            for (int k = 0; k < 3; ++k) { d0[k] = pw[k] - cp[k]; d1[k] = pw[k] - t1[k]; }
            mat3_vec(R0, d0, pc0);
            mat3_vec(R1, d1, pc1);
            // dz/dpc (msckf.py:457-467)
            CT a00 = 1 / pc0[2], a02 = -pc0[0] / (pc0[2] * pc0[2]), a12 = -pc0[1] / (pc0[2] * pc0[2]);
            CT b00 = 1 / pc1[2], b02 = -pc1[0] / (pc1[2] * pc1[2]), b12 = -pc1[1] / (pc1[2] * pc1[2]);
            // dpc/dxc (msckf.py:469-475): [skew(pc0) | -R0], [R01 skew(pc0) | -R1]
            CT Sk[9], RS[9];
            skew3(pc0, Sk);
            mat3_mul(R01, Sk, RS);
            CT D0[18], D1[18];
            for (int k = 0; k < 3; ++k)
                for (int m = 0; m < 3; ++m) {
                    D0[6 * k + m] = Sk[3 * k + m];
                    D0[6 * k + 3 + m] = -R0[3 * k + m];
                    D1[6 * k + m] = RS[3 * k + m];
                    D1[6 * k + 3 + m] = -R1[3 * k + m];
                }
            CT H[24];
            for (int m = 0; m < 6; ++m) {
                H[m] = a00 * D0[m] + a02 * D0[12 + m];
                H[6 + m] = a00 * D0[6 + m] + a12 * D0[12 + m];
                H[12 + m] = b00 * D1[m] + b02 * D1[12 + m];
                H[18 + m] = b00 * D1[6 + m] + b12 * D1[12 + m];
            }
            // observability constraint (msckf.py:484-490)
            CT u[6], Rn[9], dp[3];
            quat_to_rot(qn, Rn);
            mat3_vec(Rn, g, u);
            for (int k = 0; k < 3; ++k) dp[k] = pw[k] - cp[k];
            skew3(dp, Sk);
            mat3_vec(Sk, g, u + 3);
            CT uu = 0;
            for (int k = 0; k < 6; ++k) uu += u[k] * u[k];
            for (int a = 0; a < 4; ++a) {
                CT au = 0;
                for (int k = 0; k < 6; ++k) au += H[6 * a + k] * u[k];
                for (int k = 0; k < 6; ++k) Hx[s][6 * a + k] = H[6 * a + k] - au * u[k] / uu;
                for (int k = 0; k < 3; ++k) Hf[s][3 * a + k] = -Hx[s][6 * a + 3 + k];
            }
            r[s][0] = (CT)z[0] - pc0[0] / pc0[2];
            r[s][1] = (CT)z[1] - pc0[1] / pc0[2];
            r[s][2] = (CT)z[2] - pc1[0] / pc1[2];
            r[s][3] = (CT)z[3] - pc1[1] / pc1[2];
            // rank-3 rows for the register-tile gating: Hx and H_f factor through
            // Jc = dz/dpc0 + dz/dpc1 R01 (4x3); the reflector I - v v^T / (1 + |n_3|)
            // maps Jc's unit left null vector n to -sign(n_3) e_4, so rows 0..2 of
            // the reflected [Hx | r] are the range rows and row 3 carries only the
            // residual r_n (its Hx part vanishes).
            CT J[12] = {a00, 0, a02, 0, a00, a12, 0, 0, 0, 0, 0, 0};
            for (int m = 0; m < 3; ++m) {
                J[6 + m] = b00 * R01[m] + b02 * R01[6 + m];
                J[9 + m] = b00 * R01[3 + m] + b12 * R01[6 + m];
            }
            auto det3 = [](const CT* x, const CT* y, const CT* w) {
                return x[0] * (y[1] * w[2] - y[2] * w[1]) - x[1] * (y[0] * w[2] - y[2] * w[0]) +
                       x[2] * (y[0] * w[1] - y[1] * w[0]);
            };
            CT nv[4] = {det3(J + 3, J + 6, J + 9), -det3(J, J + 6, J + 9), det3(J, J + 3, J + 9),
                        -det3(J, J + 3, J + 6)};
            CT nn = sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2] + nv[3] * nv[3]);
            if (!(nn > 0)) { nv[0] = nv[1] = nv[2] = 0; nv[3] = 1; nn = 1; }
            for (int k = 0; k < 4; ++k) nv[k] /= nn;
            const CT beta = 1 / (1 + fabs(nv[3]));
            nv[3] += nv[3] >= 0 ? CT(1) : CT(-1);
            CT Ht[18], rt4[4];
            for (int c = 0; c < 6; ++c) {
                const CT w = nv[0] * Hx[s][c] + nv[1] * Hx[s][6 + c] + nv[2] * Hx[s][12 + c] + nv[3] * Hx[s][18 + c];
                for (int a = 0; a < 3; ++a) Ht[6 * a + c] = Hx[s][6 * a + c] - beta * nv[a] * w;
            }
            const CT wr = nv[0] * r[s][0] + nv[1] * r[s][1] + nv[2] * r[s][2] + nv[3] * r[s][3];
            for (int a = 0; a < 4; ++a) rt4[a] = r[s][a] - beta * nv[a] * wr;
            T* wsr = fb.obs_ht + (size_t)(o0 + i) * OBS_HTS;
            store_pairs(wsr + OBS_HT, Ht, 18);
            store_pairs(wsr + OBS_RT, rt4, 4);
        }
        for (int c = 0; c < 6; ++c)   // Hx_i^T r_i, before r is reflected
            u6[s][c] = Hx[s][c] * r[s][0] + Hx[s][6 + c] * r[s][1] + Hx[s][12 + c] * r[s][2] + Hx[s][18 + c] * r[s][3];
        if (own && fb.compact) store_pairs(fb.obs_ws + (size_t)(o0 + i) * OBS_WS + OBS_R, r[s], 4);
    }
    // ---- Householder QR of H_f across the segment (rows 4i..4i+3 with observation i) ----
    CT V[OPL][12];
    CT tau[3], rd[3];   // reflector scalars; R's diagonal (beta_j)
#pragma unroll
    for (int s = 0; s < OPL; ++s)
        for (int e = 0; e < 12; ++e) V[s][e] = 0;
    for (int j = 0; j < 3; ++j) {
        CT alpha = __shfl(Hf[0][3 * j + j], b0, 64);   // pivot row j: observation 0, the segment's first lane
        CT xs = 0;
#pragma unroll
        for (int s = 0; s < OPL; ++s)
            for (int a = 0; a < 4; ++a) {
                const int row = 4 * (l + S * s) + a;
                if (row > j && l + S * s < M) xs += Hf[s][3 * a + j] * Hf[s][3 * a + j];
            }
        xs = seg_sum<S>(xs);
        CT tj = 0, scale = 0, beta = alpha;
        if (xs != CT(0)) {
            CT nrm = sqrt(alpha * alpha + xs);
            beta = alpha >= 0 ? -nrm : nrm;
            tj = (beta - alpha) / beta;
            scale = CT(1) / (alpha - beta);
        }
        tau[j] = tj;
        rd[j] = beta;
        // v_j: v[j] = 1, v[row > j] = Hf[row][j] * scale, 0 above
#pragma unroll
        for (int s = 0; s < OPL; ++s)
            for (int a = 0; a < 4; ++a) {
                const int row = 4 * (l + S * s) + a;
                CT v = 0;
                if (l + S * s < M) v = row == j ? CT(1) : (row > j ? Hf[s][3 * a + j] * scale : CT(0));
                V[s][3 * a + j] = v;
            }
        // apply H_j to the remaining H_f columns and to r
        for (int c = j + 1; c <= 3; ++c) {
            CT w = 0;
#pragma unroll
            for (int s = 0; s < OPL; ++s)
                for (int a = 0; a < 4; ++a) w += V[s][3 * a + j] * (c < 3 ? Hf[s][3 * a + c] : r[s][a]);
            w = seg_sum<S>(w);
#pragma unroll
            for (int s = 0; s < OPL; ++s)
                for (int a = 0; a < 4; ++a) {
                    if (c < 3) Hf[s][3 * a + c] -= tj * V[s][3 * a + j] * w;
                    else r[s][a] -= tj * V[s][3 * a + j] * w;
                }
        }
    }
    // ---- per-feature QR record: X = R^-1 and g = (Q^T r)[0:3] (the segment's
    // first lane holds observation 0, i.e. rows 0..2 of the reflected H_f and r).
    // A zero pivot (rank-deficient H_f) drops its direction instead of dividing.
    // Ill-conditioned features (|R| > FQR_RMAX -- a landmark millimetres from
    // the camera -- or cond(R) > FQR_KAPPA) are flagged: k_info_fused's rebuild
    // G_i = X^T H_f,i^T Hx_i loses about eps cond(R)^2 of A's positive
    // semidefiniteness, which the Kalman stage cannot absorb there, so this
    // kernel writes their Householder Gram records (as the record path does)
    // and the fused assembly reads those instead.  (R's diagonal is the same in
    // every lane of the segment: the flag is segment-uniform.)
    const CT rmax = fmax(fabs(rd[0]), fmax(fabs(rd[1]), fabs(rd[2])));
    const CT rmin = fmin(fabs(rd[0]), fmin(fabs(rd[1]), fabs(rd[2])));
    const bool ill = !(rmax <= CT(FQR_RMAX)) || !(rmax <= CT(FQR_KAPPA) * rmin);
    if (l == 0 && M > 0) {
        const CT r01 = Hf[0][1], r02 = Hf[0][2], r12 = Hf[0][5];
        const CT x00 = rd[0] != CT(0) ? 1 / rd[0] : CT(0), x11 = rd[1] != CT(0) ? 1 / rd[1] : CT(0);
        const CT x22 = rd[2] != CT(0) ? 1 / rd[2] : CT(0);
        CT q[FQR_STRIDE];
        q[FQR_X + 0] = x00;
        q[FQR_X + 1] = -r01 * x00 * x11;
        q[FQR_X + 2] = (r01 * r12 * x11 - r02) * x00 * x22;
        q[FQR_X + 3] = x11;
        q[FQR_X + 4] = -r12 * x11 * x22;
        q[FQR_X + 5] = x22;
        for (int t = 0; t < 3; ++t) q[FQR_G + t] = r[0][t];
        q[FQR_FLAG] = ill ? CT(1) : CT(0);
        store_pairs(fb.fqr + (size_t)f * FQR_STRIDE, q, FQR_STRIDE);
    }
    const bool gram = GRAM || ill;
    if (!gram && !fb.compact) return;   // segment-uniform
    // ---- w_j = v_j^T X_{j-1}: 6 columns per observation, local to the lane ----
    CT d10 = 0, d20 = 0, d21 = 0;
#pragma unroll
    for (int s = 0; s < OPL; ++s)
        for (int a = 0; a < 4; ++a) {
            d10 += V[s][3 * a + 1] * V[s][3 * a];
            d20 += V[s][3 * a + 2] * V[s][3 * a];
            d21 += V[s][3 * a + 2] * V[s][3 * a + 1];
        }
    d10 = seg_sum<S>(d10);
    d20 = seg_sum<S>(d20);
    d21 = seg_sum<S>(d21);
    // top 3 rows of V (observation 0: slot 0 of the segment's first lane) and g = (Q^T r)[0:3]
    CT V0[9], gr[3];
    for (int e = 0; e < 9; ++e) V0[e] = __shfl(V[0][e], b0, 64);
    for (int t = 0; t < 3; ++t) gr[t] = __shfl(r[0][t], b0, 64);
#pragma unroll
    for (int s = 0; s < OPL; ++s) {
        const int i = l + S * s;
        if (i >= M) continue;
        CT W[18];
        for (int c = 0; c < 6; ++c) {
            CT w0 = 0, w1 = 0, w2 = 0;
            for (int a = 0; a < 4; ++a) {
                w0 += V[s][3 * a] * Hx[s][6 * a + c];
                w1 += V[s][3 * a + 1] * Hx[s][6 * a + c];
                w2 += V[s][3 * a + 2] * Hx[s][6 * a + c];
            }
            w1 -= tau[0] * d10 * w0;
            w2 -= tau[0] * d20 * w0 + tau[1] * d21 * w1;
            W[c] = w0; W[6 + c] = w1; W[12 + c] = w2;
        }
        T* ws = fb.obs_ws + (size_t)(o0 + i) * OBS_WS;
        if (fb.compact) {   // Hx and the compact factors: only the LDS / global gate and the QR merge read them
            store_pairs(ws + OBS_HX, Hx[s], 24);
            store_pairs(ws + OBS_V, V[s], 12);
            store_pairs(ws + OBS_W, W, 18);
            store_pairs(ws + OBS_QR, r[s], 4);
            if (i == 0)
                for (int j = 0; j < 3; ++j) fb.tau[4 * f + j] = (T)tau[j];
        }
        if (!gram) continue;
        // Gram terms.  (Q^T Hx)[t][i-block] = [i == 0] Hx_0[t] - sum_j tau_j V_0[t][j] W_j(i)
        CT rec[OBG_STRIDE];   // G | DS | UB | pad, stored as 16-byte pairs
        for (int t = 0; t < 3; ++t)
            for (int c = 0; c < 6; ++c) {
                CT v = i == 0 ? Hx[s][6 * t + c] : CT(0);
                for (int j = 0; j < 3; ++j) v -= tau[j] * V0[3 * t + j] * W[6 * j + c];
                rec[OBG_G + 6 * t + c] = v;
            }
        for (int x = 0, e = 0; x < 6; ++x)
            for (int y = 0; y <= x; ++y, ++e)
                rec[OBG_DS + e] = Hx[s][x] * Hx[s][y] + Hx[s][6 + x] * Hx[s][6 + y] + Hx[s][12 + x] * Hx[s][12 + y] +
                                  Hx[s][18 + x] * Hx[s][18 + y];
        for (int c = 0; c < 6; ++c)
            rec[OBG_UB + c] = u6[s][c] - (rec[OBG_G + c] * gr[0] + rec[OBG_G + 6 + c] * gr[1] + rec[OBG_G + 12 + c] * gr[2]);
        for (int e = OBG_UB + 6; e < OBG_STRIDE; ++e) rec[e] = 0;
        rec[OBG_CAM] = (CT)fb.obs_cam[o0 + i];
        store_pairs(fb.obs_g + (size_t)(o0 + i) * OBG_STRIDE, rec, OBG_STRIDE);
    }
}
// ===========================================================================
// Gating (msckf.py:606-614): one workgroup per feature.
// S = H0 P H0^T + sigma^2 I is formed in observation space:
//   Y = Hx P Hx^T (4M x 4M, 4x4 blocks Hx_i P_{s_i s_l} Hx_l^T), then
//   Q^T Y Q by the three reflectors applied two-sided, S = (Q^T Y Q)[3:,3:] + s2 I,
// followed by a Cholesky factorisation and a forward solve: gamma = |L^-1 r0|^2.
// (Same value as the reference's rows-space S; ~10x fewer flops.)
// ===========================================================================
template <typename T>
__global__ void __launch_bounds__(256) k_gate(DevState<T> st, Params<T> prm, FeatBatch<T> fb,
                                              const int* __restrict__ flist) {
    const int f = flist[blockIdx.x];
    const int tid = threadIdx.x;
    if (!fb.valid[f]) {
        if (tid == 0) { fb.gamma[f] = T(NAN); fb.accept[f] = 0; }
        return;
    }
    const int b = fb.feat_filter[f];
    const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
    const int n4 = 4 * M;
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ld = st.Dmax;
    T* Y = fb.ysq + fb.ysq_off[f];
    const T* ws = fb.obs_ws + (size_t)o0 * OBS_WS;
    __shared__ T s_v[3][512], s_p[512], s_w[512], s_r[512];
    __shared__ T s_scalar[2];
    __shared__ int s_fail;
    // 1. Y blocks (i <= l)
    const int npairs = M * (M + 1) / 2;
    for (int pidx = tid; pidx < npairs; pidx += blockDim.x) {
        int i = 0, rem = pidx;
        while (rem >= M - i) { rem -= M - i; ++i; }
        int l = i + rem;
        const T* Hi = ws + (size_t)i * OBS_WS + OBS_HX;
        const T* Hl = ws + (size_t)l * OBS_WS + OBS_HX;
        const int si = fb.obs_cam[o0 + i], sl = fb.obs_cam[o0 + l];
        const T* Pb = P + (size_t)(21 + 6 * si) * ld + 21 + 6 * sl;
        T T1[24];
        for (int a = 0; a < 4; ++a)
            for (int c = 0; c < 6; ++c) {
                T s = 0;
                for (int k = 0; k < 6; ++k) s += Hi[6 * a + k] * Pb[(size_t)k * ld + c];
                T1[6 * a + c] = s;
            }
        for (int a = 0; a < 4; ++a)
            for (int c = 0; c < 4; ++c) {
                T s = 0;
                for (int k = 0; k < 6; ++k) s += T1[6 * a + k] * Hl[6 * c + k];
                Y[(size_t)(4 * i + a) * n4 + 4 * l + c] = s;
                Y[(size_t)(4 * l + c) * n4 + 4 * i + a] = s;
            }
    }
    for (int row = tid; row < n4; row += blockDim.x) {
        const T* w = ws + (size_t)(row >> 2) * OBS_WS;
        for (int j = 0; j < 3; ++j) s_v[j][row] = w[OBS_V + 3 * (row & 3) + j];
        s_r[row] = w[OBS_QR + (row & 3)];
    }
    __syncthreads();
    // 2. two-sided reflectors: Y <- H_j Y H_j
    for (int j = 0; j < 3; ++j) {
        const T tj = fb.tau[4 * f + j];
        if (tj == T(0)) continue;
        for (int a = tid; a < n4; a += blockDim.x) {
            T s = 0;
            for (int c = j; c < n4; ++c) s += Y[(size_t)a * n4 + c] * s_v[j][c];
            s_p[a] = s;
        }
        __syncthreads();
        if (tid < 64) {
            T s = 0;
            for (int a = tid; a < n4; a += 64) s += s_v[j][a] * s_p[a];
            s = wave_sum(s);
            if (tid == 0) s_scalar[0] = s;
        }
        __syncthreads();
        const T K = tj * tj * s_scalar[0] / T(2);
        for (int a = tid; a < n4; a += blockDim.x) s_w[a] = tj * s_p[a] - K * s_v[j][a];
        __syncthreads();
        for (int e = tid; e < n4 * n4; e += blockDim.x) {
            int a = e / n4, c = e % n4;
            Y[e] -= s_v[j][a] * s_w[c] + s_w[a] * s_v[j][c];
        }
        __syncthreads();
    }
    // 3. S = Y[3:,3:] + s2 I ; Cholesky + forward solve fused (gamma = |L^-1 r0|^2)
    const int k = n4 - 3;
    T* S = Y + 3 * (size_t)n4 + 3;
    if (tid == 0) s_fail = 0;
    for (int a = tid; a < k; a += blockDim.x) S[(size_t)a * n4 + a] += prm.sigma2;
    __syncthreads();
    T gam = 0;
    for (int j = 0; j < k; ++j) {
        if (tid == 0) {
            T d = S[(size_t)j * n4 + j];
            if (!(d > 0)) { s_fail = 1; d = T(1); }
            T l = sqrt(d);
            S[(size_t)j * n4 + j] = l;
            T y = s_r[3 + j] / l;
            s_scalar[1] = y;
            gam += y * y;
        }
        __syncthreads();
        const T ljj = S[(size_t)j * n4 + j];
        const T yj = s_scalar[1];
        for (int i = j + 1 + tid; i < k; i += blockDim.x) {
            T lij = S[(size_t)i * n4 + j] / ljj;
            S[(size_t)i * n4 + j] = lij;
            s_r[3 + i] -= lij * yj;
        }
        __syncthreads();
        const int m = k - j - 1;
        for (int e = tid; e < m * m; e += blockDim.x) {
            int i = j + 1 + e / m, l = j + 1 + e % m;
            if (l <= i) S[(size_t)i * n4 + l] -= S[(size_t)i * n4 + j] * S[(size_t)l * n4 + j];
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (s_fail) gam = T(INFINITY);
        fb.gamma[f] = gam;
        fb.accept[f] = (gam < fb.chi2[f]) ? 1 : 0;
    }
}

// Fast path of k_gate with Y / S resident in LDS (ld = 4M+1, odd: conflict-free
// row and column sweeps) and gamma from an LDL^T elimination with the residual
// carried along as an extra column: gamma = sum_j r~_j^2 / d_j.  One barrier
// per pivot; the column being eliminated is read-only during its step.
template <typename T>
__global__ void __launch_bounds__(256) k_gate_lds(DevState<T> st, Params<T> prm, FeatBatch<T> fb,
                                                  const int* __restrict__ flist) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int f = flist[blockIdx.x];
    const int tid = threadIdx.x;
    if (!fb.valid[f]) {
        if (tid == 0) { fb.gamma[f] = T(NAN); fb.accept[f] = 0; }
        return;
    }
    const int b = fb.feat_filter[f];
    const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
    const int n4 = 4 * M, ld = n4 + 1;
    const T* P = st.P + (size_t)b * st.Dmax * st.Dmax;
    const int ldp = st.Dmax;
    const T* ws = fb.obs_ws + (size_t)o0 * OBS_WS;
    T* Y = reinterpret_cast<T*>(smem_raw);                       // [n4][n4+1]
    T* s_hx = Y + (((size_t)n4 * ld + 1) & ~(size_t)1);           // [n4][6]
    T* s_v = s_hx + 6 * n4;                                       // [3][n4]
    T* s_r = s_v + 3 * n4;                                        // [n4]
    T* s_p = s_r + n4;                                            // [n4]
    T* s_w = s_p + n4;                                            // [n4]
    T* s_sc = s_w + n4;                                           // [4]
    int* s_slot = reinterpret_cast<int*>(s_sc + 4);               // [M]
    for (int e = tid; e < n4 * 6; e += blockDim.x) s_hx[e] = ws[(size_t)(e / 24) * OBS_WS + OBS_HX + e % 24];
    for (int row = tid; row < n4; row += blockDim.x) {
        const T* w = ws + (size_t)(row >> 2) * OBS_WS;
        for (int j = 0; j < 3; ++j) s_v[j * n4 + row] = w[OBS_V + 3 * (row & 3) + j];
        s_r[row] = w[OBS_QR + (row & 3)];
    }
    for (int i = tid; i < M; i += blockDim.x) s_slot[i] = fb.obs_cam[o0 + i];
    __syncthreads();
    // 1. Y = Hx P Hx^T, 4x4 blocks
    const int npairs = M * (M + 1) / 2;
    for (int pidx = tid; pidx < npairs; pidx += blockDim.x) {
        int i = 0, rem = pidx;
        while (rem >= M - i) { rem -= M - i; ++i; }
        const int l = i + rem;
        const T* Hi = s_hx + 24 * i;
        const T* Hl = s_hx + 24 * l;
        const T* Pb = P + (size_t)(21 + 6 * s_slot[i]) * ldp + 21 + 6 * s_slot[l];
        T Pl[36];
        for (int k = 0; k < 6; ++k)
            for (int c = 0; c < 6; ++c) Pl[6 * k + c] = Pb[(size_t)k * ldp + c];
        T T1[24];
        for (int a = 0; a < 4; ++a)
            for (int c = 0; c < 6; ++c) {
                T sacc = 0;
                for (int k = 0; k < 6; ++k) sacc += Hi[6 * a + k] * Pl[6 * k + c];
                T1[6 * a + c] = sacc;
            }
        for (int a = 0; a < 4; ++a)
            for (int c = 0; c < 4; ++c) {
                T sacc = 0;
                for (int k = 0; k < 6; ++k) sacc += T1[6 * a + k] * Hl[6 * c + k];
                Y[(4 * i + a) * ld + 4 * l + c] = sacc;
                Y[(4 * l + c) * ld + 4 * i + a] = sacc;
            }
    }
    __syncthreads();
    // 2. Y <- H_j Y H_j for the three reflectors
    for (int j = 0; j < 3; ++j) {
        const T tj = fb.tau[4 * f + j];
        if (tj == T(0)) continue;
        const T* v = s_v + j * n4;
        for (int a = tid; a < n4; a += blockDim.x) {
            T sacc = 0;
            for (int c = j; c < n4; ++c) sacc += Y[a * ld + c] * v[c];
            s_p[a] = sacc;
        }
        __syncthreads();
        if (tid < 64) {
            T sacc = 0;
            for (int a = tid; a < n4; a += 64) sacc += v[a] * s_p[a];
            sacc = wave_sum(sacc);
            if (tid == 0) s_sc[0] = sacc;
        }
        __syncthreads();
        const T K = tj * tj * s_sc[0] / T(2);
        for (int a = tid; a < n4; a += blockDim.x) s_w[a] = tj * s_p[a] - K * v[a];
        __syncthreads();
        for (int a = (tid >> 4); a < n4; a += (int)(blockDim.x >> 4)) {
            const T va = v[a], wa = s_w[a];
            for (int c = (tid & 15); c < n4; c += 16) Y[a * ld + c] -= va * s_w[c] + wa * v[c];
        }
        __syncthreads();
    }
    // 3. S = Y[3:,3:] + s2 I ; LDL^T with the residual as an extra column
    const int k = n4 - 3;
    T* S = Y + 3 * ld + 3;
    T* r = s_r + 3;
    for (int a = tid; a < k; a += blockDim.x) S[a * ld + a] += prm.sigma2;
    __syncthreads();
    T gam = 0;
    bool fail = false;
    for (int j = 0; j < k; ++j) {
        const T d = S[j * ld + j];
        if (!(d > 0)) { fail = true; break; }   // uniform: every thread reads the same d
        const T inv = T(1) / d;
        const T rj = r[j];
        if (tid == 0) gam += rj * rj * inv;
        // (blockDim/16) x 16 thread grid over the trailing lower triangle (no divisions)
        const int rstep = blockDim.x >> 4;
        for (int i = j + 1 + (tid >> 4); i < k; i += rstep) {
            const T ai = S[i * ld + j] * inv;
            for (int l = j + 1 + (tid & 15); l <= i; l += 16) S[i * ld + l] -= ai * S[l * ld + j];
            if ((tid & 15) == 0) r[i] -= ai * rj;
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (fail) gam = T(INFINITY);
        fb.gamma[f] = gam;
        fb.accept[f] = (gam < fb.chi2[f]) ? 1 : 0;
    }
}

// Gating mathematics (M <= 82).  With Y = Hx P Hx^T + s2 I (4M x 4M, PD) and N an orthonormal basis
// of the left nullspace of H_f, the reference's S = N^T Y N (msckf.py:607-609
// on H0 = N^T Hx) satisfies the oblique-projection identity
//   N S^-1 N^T = Y^-1 - Y^-1 H_f (H_f^T Y^-1 H_f)^-1 H_f^T Y^-1,
// so gamma = r0^T S^-1 r0 is what an LDL^T elimination of the saddle-point
// matrix [[Y, H_f, r], [H_f^T, 0, 0], [r^T, 0, 0]] leaves in its last pivot:
// -gamma.  No projection is formed at all.
// Rank-3 reduction: every observation's Hx_i (4x6) and H_f,i (4x3) factor
// through the 4x3 projection Jacobian Jc_i = dz/dp_c0 + dz/dp_c1 R_c0c1
// (msckf.py:457-480: dp_c1/dx = R_c0c1 dp_c0/dx), so k_feature rotates each
// observation's rows by a reflector taking Jc_i's left null vector to e_4:
// three range rows Ht_i = (Q_i^T Hx_i)[0:3], r~_i, and one null row whose
// Hx / H_f entries are exactly zero and whose residual r_n,i decouples (pivot
// s2).  gamma is invariant under these orthogonal row maps (quirk Q4), so
//   gamma = gamma(saddle point of the 3M range rows) + sum_i r_n,i^2 / s2,
// a (3M + 4)-square elimination instead of (4M + 4): ~(3/4)^3 of the flops.
// (The kernels: msckf_gate_mfma.hip -- k_gate_mfma, one wave per feature, and
// k_gate_mfma_wt, a 2- to 8-wave workgroup per feature of 9..16 blocks, both on
// MFMA tiles.  Round 6 removed the fp64 register-tile kernels k_gate_wave and
// k_gate_big they replaced for 37 <= M <= 82: 50x400 fp64 gate 56.2 -> 32.2 ms,
// 80x1000 k_gate_big alone 117 ms -> k_gate_mfma_wt 54 ms, profiles/r06/wt64/.)

// ===========================================================================
// Stacking in feature order with the row cap (msckf.py:671-679): one
// wavefront per filter scans its features; decides the compression (msckf.py:549).
// ===========================================================================
template <typename T>
__global__ void __launch_bounds__(256) k_select(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws, int row_cap) {
    // one wavefront per filter: 64 features at a time, the accepted row counts
    // prefix-summed across the wave.  Feature f is stacked iff it is valid,
    // accepted and the rows stacked before it do not exceed the cap yet (the
    // reference breaks after the count first exceeds it, msckf.py:676-679).
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= st.B) return;
    int carry = 0, count = 0;
    for (int f0 = fb.feat_off[b]; f0 < fb.feat_off[b + 1]; f0 += 64) {
        const int f = f0 + lane;
        const bool in = f < fb.feat_off[b + 1];
        int v = 0;
        if (in && fb.valid[f] && fb.accept[f]) v = 4 * (fb.obs_off[f + 1] - fb.obs_off[f]) - 3;
        int incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        const int excl = carry + incl - v;
        const bool take = v > 0 && (row_cap <= 0 || excl <= row_cap);
        if (in) {
            fb.include[f] = take ? 1 : 0;
            fb.row_off[f] = take ? excl : 0;
        }
        count += wave_sum(take ? v : 0);
        carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) {
        const int C = 6 * st.ncams[b];
        int* info = ws.info + 4 * b;
        info[0] = count;
        info[1] = count > C ? C : count;
        info[2] = count > C ? 1 : 0;
        info[3] = 0;
    }
}

// ===========================================================================
// Information assembly (replaces the QR compression of
// msckf.py:549-556).  The update msckf.py:559-604 depends on the stacked
// (H, r) only through A = H^T H and b = H^T r:
//   K r = P H^T (H P H^T + s2 I)^-1 r = P (A P + s2 I)^-1 b,
//   K H P = P (A P + s2 I)^-1 A P,
// so the Cholesky-form Kalman stage (msckf_kalman.hip) takes [A | b] in place
// of the QR's [R | Q^T r].  Per feature the projected block's Gram matrix is
// assembled from the fp64 terms of k_feature:
//   H0^T H0 = blockdiag_i(Hx_i^T Hx_i) - G^T G,   H0^T r0 = sum_i UB_i,
// which needs O(M^2) work per feature and never materialises the stacked
// rows (the QR merge streamed its C x C factor through memory once per
// 16-row chunk: ~160 GB per 2048-filter launch, profiles/r01/README.md).
//
// One workgroup per filter (several for Nmax > 40).  Each wave owns an 8 x 8
// tile of cam pairs (lane: I = 8 ti + lane / 8, J = 8 tj + lane % 8), the
// thread its 6x6 block of A in registers; features are staged FB at a time in
// LDS, indexed by cam, with a cam bitmask per feature, and each thread
// accumulates the blocks whose two cams the feature observes.
// Output: [A | b] in H_thin (Cmax x (Cmax + 1), KT), info[1] = C.
// ===========================================================================
// features staged per round (one staging wave each): five, capped by what the
// double-buffered slots leave of the LDS (measured at 30x200 four / five / six:
// 2.17 / 2.06 / 2.11 ms; at 50x400 two / three / four: 3.0 / 2.5 / 2.18 ms)
constexpr int INFO_FB_MAX = 5;
// Doubles per staging slot: a feature's M <= Nmax records copied contiguously,
// rounded up to whole 1 KiB global_load_lds wave-instructions.
__host__ __device__ constexpr int info_slot_doubles(int Nmax) { return (Nmax * OBG_STRIDE + 127) / 128 * 128; }

template <typename T, int BPT, int NT>
__global__ void __launch_bounds__(NT) k_info(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws, int fbn, int maxnf,
                                             int maxobs, int rmp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    // grid (parts, B), parts >= 3 (80 cams: 4): a filter's parts get consecutive ids,
    // remapped onto one XCD so that its records come from HBM once into that XCD's
    // L2 (80x1000 compress 15.1 -> 14.1 ms); two parts (50 cams) measured slower
    // that way (8.3 -> 8.9 ms) and keep the plain order, grid (B, parts)
    const Blk3 bk = xcd_blk3();
    const int b = rmp ? bk.y : blockIdx.x, part = rmp ? bk.x : blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nwave = NT >> 6;
    const int nc = st.ncams[b], C = 6 * nc, Cmax = ws.Cmax, Nmax = st.Nmax;
    int* info = ws.info + 4 * b;
    if (info[0] == 0) {   // nothing stacked: empty update
        if (tid == 0) info[1] = 0;
        return;
    }
    const int SLOT = info_slot_doubles(Nmax), INFO_FB = fbn;
    double* rec = reinterpret_cast<double*>(smem_raw);                      // [2][FB][SLOT]
    unsigned long long* mask = reinterpret_cast<unsigned long long*>(rec + (size_t)2 * INFO_FB * SLOT);   // [2][FB][2]
    int* pos = reinterpret_cast<int*>(mask + 4 * INFO_FB);                   // [2][FB][Nmax] cam -> record
    // filter-resident feature metadata (maxobs > 0): every feature's cam mask,
    // first record and record count (0 if not included), and the filter's
    // obs_cam -- read once up front, so that staging a batch involves no
    // dependent global loads (include -> obs_off -> obs_cam was three round
    // trips on the critical path of every batch)
    unsigned long long* fmask = reinterpret_cast<unsigned long long*>(pos + ((2 * INFO_FB * Nmax + 1) & ~1));
    int* fo0 = reinterpret_cast<int*>(fmask + 2 * maxnf);
    int* fM = fo0 + maxnf;
    int* sobs = fM + maxnf;

    double a[BPT][6][6], bv[BPT][6];
    int I[BPT], J[BPT];
    bool act[BPT];
#pragma unroll
    for (int m = 0; m < BPT; ++m) {
        // wave = one 8 x 8 tile of cam pairs (lane: I = 8 ti + lane / 8, J = 8 tj + lane % 8):
        // a feature's contiguous cam range [s, e] activates the pairs s <= J <= I <= e,
        // a triangle that whole tiles cover far better than the row-major block order
        // (whose 64-block strips are mostly inactive for every feature)
        const int tt = part * (NT >> 6) * BPT + (tid >> 6) + (NT >> 6) * m;
        const int TS = (Nmax + 7) >> 3, ntl = TS * (TS + 1) / 2;
        int ti = (int)((sqrtf(8.0f * (float)tt + 1.0f) - 1.0f) * 0.5f);
        while (ti * (ti + 1) / 2 > tt) --ti;
        while ((ti + 1) * (ti + 2) / 2 <= tt) ++ti;
        const int tj = tt - ti * (ti + 1) / 2;
        I[m] = 8 * ti + (lane >> 3);
        J[m] = 8 * tj + (lane & 7);
        act[m] = tt < ntl && I[m] < nc && J[m] <= I[m];
#pragma unroll
        for (int x = 0; x < 6; ++x) {
            bv[m][x] = 0;
#pragma unroll
            for (int y = 0; y < 6; ++y) a[m][x][y] = 0;
        }
    }
    // ---- assembly ----
    // Batches of FB features; wave s < FB stages feature f0 + s of the next
    // batch while all waves accumulate the current one: a contiguous copy of
    // its M records (global_load_lds, 16 B per lane), a cam -> record table
    // and a cam bitmask.
    const int fbeg = fb.feat_off[b], fend = fb.feat_off[b + 1];
    const int obeg = fb.obs_off[fbeg];
    const bool pre = maxobs > 0;   // uniform
    if (pre) {
        const int nobs = fb.obs_off[fend] - obeg;
        for (int e = tid; e < nobs; e += NT) sobs[e] = fb.obs_cam[obeg + e];
        for (int f = fbeg + tid; f < fend; f += NT) {
            const bool in = fb.include[f] != 0;
            fo0[f - fbeg] = fb.obs_off[f];
            fM[f - fbeg] = in ? fb.obs_off[f + 1] - fb.obs_off[f] : 0;
        }
        __syncthreads();
        for (int f = tid; f < fend - fbeg; f += NT) {   // one thread per feature: its cam mask
            unsigned long long m0 = 0, m1 = 0;
            for (int o = 0; o < fM[f]; ++o) {
                const int cam = sobs[fo0[f] - obeg + o];
                if (cam < 64) m0 |= 1ull << cam;
                else m1 |= 1ull << (cam - 64);
            }
            fmask[2 * f] = m0;
            fmask[2 * f + 1] = m1;
        }
        __syncthreads();
    }
    auto stage = [&](int f0, int buf) {
        for (int s = wave; s < INFO_FB; s += nwave) {
            const int f = f0 + s;
            int* ps = pos + (buf * INFO_FB + s) * Nmax;
            unsigned long long mk[2] = {0, 0};
            int o0 = 0, M = 0;
            if (pre) {
                if (f < fend) {
                    o0 = fo0[f - fbeg];
                    M = fM[f - fbeg];
                    for (int o = lane; o < M; o += 64) ps[sobs[o0 - obeg + o]] = o;
                    if (lane < 2) mask[(buf * INFO_FB + s) * 2 + lane] = M ? fmask[2 * (f - fbeg) + lane] : 0ull;
                } else if (lane < 2) {
                    mask[(buf * INFO_FB + s) * 2 + lane] = 0ull;
                }
            } else if (f < fend && fb.include[f]) {
                o0 = fb.obs_off[f];
                M = fb.obs_off[f + 1] - o0;
                for (int o = lane; o < M; o += 64) {
                    const int cam = fb.obs_cam[o0 + o];
                    mk[cam >> 6] |= 1ull << (cam & 63);
                    ps[cam] = o;
                }
            }
#pragma unroll
            for (int h = 0; h < 2 && !pre; ++h) {
                unsigned lo = (unsigned)mk[h], hi = (unsigned)(mk[h] >> 32);
#pragma unroll
                for (int w = 32; w >= 1; w >>= 1) {
                    lo |= (unsigned)__shfl_xor((int)lo, w, 64);
                    hi |= (unsigned)__shfl_xor((int)hi, w, 64);
                }
                if (lane == 0) mask[(buf * INFO_FB + s) * 2 + h] = ((unsigned long long)hi << 32) | lo;
            }
            // after every ordinary global load above: the copy below may stay in flight
            const char* src = reinterpret_cast<const char*>(fb.obs_g + (size_t)o0 * OBG_STRIDE);
            double* dst = rec + (size_t)(buf * INFO_FB + s) * SLOT;
            const int nchunk = M * OBG_STRIDE / 2;   // 16-byte chunks
            for (int c0 = 0; c0 < nchunk; c0 += 64) {
                if (c0 + lane < nchunk)
                    __builtin_amdgcn_global_load_lds((const void*)(src + 16 * (size_t)(c0 + lane)),
                                                     (void*)(dst + 2 * c0), 16, 0, 0);
            }
        }
    };
    if (fbeg < fend) stage(fbeg, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int f0 = fbeg, it = 0; f0 < fend; f0 += INFO_FB, ++it) {
        const int buf = it & 1;
        if (f0 + INFO_FB < fend) stage(f0 + INFO_FB, buf ^ 1);
        for (int s = 0; s < INFO_FB; ++s) {
            const unsigned long long* mk = mask + (buf * INFO_FB + s) * 2;
            const int* ps = pos + (buf * INFO_FB + s) * Nmax;
            const double* rs = rec + (size_t)(buf * INFO_FB + s) * SLOT;
#pragma unroll
            for (int m = 0; m < BPT; ++m) {
                if (!act[m] || !((mk[I[m] >> 6] >> (I[m] & 63)) & (mk[J[m] >> 6] >> (J[m] & 63)) & 1ull)) continue;
                const double* gi = rs + ps[I[m]] * OBG_STRIDE;
                const double* gj = rs + ps[J[m]] * OBG_STRIDE;
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    double u[6], v[6];
#pragma unroll
                    for (int x = 0; x < 6; ++x) { u[x] = gi[OBG_G + 6 * t + x]; v[x] = gj[OBG_G + 6 * t + x]; }
#pragma unroll
                    for (int x = 0; x < 6; ++x)
#pragma unroll
                        for (int y = 0; y < 6; ++y) a[m][x][y] -= u[x] * v[y];
                }
                if (I[m] == J[m]) {
#pragma unroll
                    for (int x = 0, e = 0; x < 6; ++x)
#pragma unroll
                        for (int y = 0; y <= x; ++y, ++e) {
                            const double d = gi[OBG_DS + e];
                            a[m][x][y] += d;
                            if (y < x) a[m][y][x] += d;
                        }
#pragma unroll
                    for (int x = 0; x < 6; ++x) bv[m][x] += gi[OBG_UB + x];
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    KT* F = ws.Hthin + (size_t)b * Cmax * (Cmax + 1);
    const int ldf = Cmax + 1;
#pragma unroll
    for (int m = 0; m < BPT; ++m) {
        if (!act[m]) continue;
#pragma unroll
        for (int x = 0; x < 6; ++x)
#pragma unroll
            for (int y = 0; y < 6; ++y) {
                F[(size_t)(6 * I[m] + x) * ldf + 6 * J[m] + y] = a[m][x][y];
                F[(size_t)(6 * J[m] + y) * ldf + 6 * I[m] + x] = a[m][x][y];
            }
        if (I[m] == J[m])
#pragma unroll
            for (int x = 0; x < 6; ++x) F[(size_t)(6 * I[m] + x) * ldf + Cmax] = bv[m][x];
    }
    if (tid == 0 && part == 0) info[1] = C;
}

// ---------------------------------------------------------------------------
// Information assembly on fp64 MFMA (windows up to 32 cams).  With Gall the
// stacked G blocks of the filter's included features (3 rows per feature, 6
// columns per cam slot),
//     A = blockdiag_i(Hx_i^T Hx_i) - Gall^T Gall,   b = sum_i UB_i,
// and Gall^T Gall is a rank-k update of the lower 16 x 16 tiles of A: the
// included features are staged KF at a time as dense rows of Gall in LDS,
// each wave accumulates five of the (at most 78) tiles with
// v_mfma_f64_16x16x4f64 over 4-row k-steps, and a k-step only updates the
// tiles both of whose column ranges its features touch (per-feature tile
// masks).  The chunk's G blocks are fetched into registers under the previous
// chunk's MFMAs, and its block-diagonal / b terms under its own; two barriers
// per chunk (a feature slot's rows are only touched by one wave).  The block
// diagonal and b are summed per (cam, element) by one thread each, in feature
// order.  Output as k_info: [A | b] in H_thin, info[1] = C.
// ---------------------------------------------------------------------------
typedef double v4d __attribute__((ext_vector_type(4)));
// (round 3: 16 waves x 5 tiles measured 1.43 ms against 1.47 for 14 x 6 -- profiles/r03/ab_info/)
constexpr int IM_NW = 16, IM_PPW = 5, IM_GS = 208;   // waves, tiles per wave, LDS row stride (doubles)
constexpr int IM_KF = 4;                              // features per staged chunk (3 rows each)
// (measured in round 3 at 30x200, fp32 context: 8 features per chunk 1.53 ms, 12
// 1.71 ms, against 1.46 ms for 4 -- profiles/r03/exp_ab_*.json)

__host__ __device__ constexpr size_t info_mfma_lds(int maxnf, int maxobs) {
    return (size_t)3 * IM_KF * IM_GS * sizeof(double) + (3 * IM_KF / 4) * sizeof(unsigned) +
           (size_t)(32 * IM_KF + 4 * maxnf + maxobs + 1) * sizeof(int);
}

template <typename T>
__global__ void __launch_bounds__(64 * IM_NW) k_info_mfma(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws, int maxnf,
                                                          int maxobs) {
    constexpr int NT = 64 * IM_NW, KF = IM_KF, KR = 3 * KF, NKS = KR / 4;
    static_assert(KR % 4 == 0 && 27 * 32 <= NT && 78 <= IM_NW * IM_PPW, "k_info_mfma shape");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* info = ws.info + 4 * b;
    if (info[0] == 0) {   // nothing stacked: empty update
        if (tid == 0) info[1] = 0;
        return;
    }
    const int nc = st.ncams[b], C = 6 * nc, Cmax = ws.Cmax;
    const int TT = (C + 15) >> 4, npair = TT * (TT + 1) / 2;
    double* buf = reinterpret_cast<double*>(smem_raw);              // [KR][IM_GS] dense rows of Gall
    unsigned* kmask = reinterpret_cast<unsigned*>(buf + KR * IM_GS);  // [NKS] tiles touched per k-step
    int* posc = reinterpret_cast<int*>(kmask + NKS);                 // [KF][32] cam -> record (-1)
    int* flist = posc + 32 * KF;                                     // [maxnf] included features, in order
    unsigned* ftm = reinterpret_cast<unsigned*>(flist + maxnf);      // [maxnf] their tile masks
    int* fo0 = reinterpret_cast<int*>(ftm + maxnf);                  // [maxnf] first record
    int* fM = fo0 + maxnf;                                           // [maxnf] records (0: not included)
    int* sobs = fM + maxnf;                                          // [maxobs] obs_cam of the filter
    int* s_n = sobs + maxobs;
    const int fbeg = fb.feat_off[b], fend = fb.feat_off[b + 1], nf = fend - fbeg;
    const int obeg = fb.obs_off[fbeg], nobs = fb.obs_off[fend] - obeg;
    // the filter's obs_cam and feature metadata: four trips' loads issued before
    // their LDS stores (one memory round trip per 4 NT entries, not per NT)
    for (int e0 = 0; e0 < nobs; e0 += 4 * NT) {
        int v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + NT * u + tid;
            v[u] = e < nobs ? fb.obs_cam[obeg + e] : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + NT * u + tid;
            if (e < nobs) sobs[e] = v[u];
        }
    }
    for (int f = tid; f < nf; f += NT) {
        const int a0 = fb.obs_off[fbeg + f], a1 = fb.obs_off[fbeg + f + 1];
        const bool inc = fb.include[fbeg + f];
        fo0[f] = a0;
        fM[f] = inc ? a1 - a0 : 0;
    }
    for (int e = tid; e < KR * IM_GS; e += NT) buf[e] = 0.0;
    for (int e = tid; e < 32 * KF; e += NT) posc[e] = -1;
    __syncthreads();
    if (wv == 0) {   // the included features, in order
        int base = 0;
        for (int f0 = 0; f0 < nf; f0 += 64) {
            const int f = f0 + lane;
            const bool in = f < nf && fM[f] > 0;
            const unsigned long long bal = __ballot(in);
            if (in) flist[base + __popcll(bal & ((1ull << lane) - 1ull))] = f;
            base += __popcll(bal);
        }
        if (lane == 0) *s_n = base;
    }
    __syncthreads();
    const int nl = *s_n;
    for (int i = tid; i < nl; i += NT) {
        const int f = flist[i];
        unsigned m = 0;
        for (int o = 0; o < fM[f]; ++o) {
            const int c = sobs[fo0[f] - obeg + o];
            m |= (1u << ((6 * c) >> 4)) | (1u << ((6 * c + 5) >> 4));
        }
        ftm[i] = m;
    }
    // this wave's tiles (lower, row-major order p -> (ti, tj))
    int pti[IM_PPW], ptj[IM_PPW];
    bool pv[IM_PPW];
    v4d acc[IM_PPW];
#pragma unroll
    for (int q = 0; q < IM_PPW; ++q) {
        const int p = IM_PPW * wv + q;
        int ti = (int)((sqrtf(8.0f * (float)p + 1.0f) - 1.0f) * 0.5f);
        while (ti * (ti + 1) / 2 > p) --ti;
        while ((ti + 1) * (ti + 2) / 2 <= p) ++ti;
        pti[q] = __builtin_amdgcn_readfirstlane(ti);
        ptj[q] = __builtin_amdgcn_readfirstlane(p - ti * (ti + 1) / 2);
        pv[q] = p < npair;
        acc[q] = v4d{0.0, 0.0, 0.0, 0.0};
    }
    // (cam, element) owner of the block diagonal / b: element < 21 packed lower DS, else UB
    const bool dbo = tid < 27 * nc;
    const int dc = tid / 27, de = tid - 27 * (tid / 27);
    const int deoff = de < 21 ? OBG_DS + de : OBG_UB + (de - 21);
    double dsum = 0.0;
    // staging slot: chunk feature ss, its record so (tid < 32 KF)
    const int ss = tid >> 5, so = tid & 31;
    double g[18];
    int gcol = -1;
    auto fetch = [&](int l0) {
        gcol = -1;
        if (tid < 32 * KF && l0 + ss < nl) {
            const int f = flist[l0 + ss];
            if (so < fM[f]) {
                const int o = fo0[f] + so;
                gcol = 6 * sobs[o - obeg];
                const double* r = fb.obs_g + (size_t)o * OBG_STRIDE + OBG_G;
#pragma unroll
                for (int k = 0; k < 18; ++k) g[k] = r[k];
            }
        }
    };
    __syncthreads();   // ftm complete
    fetch(0);
    for (int l0 = 0; l0 < nl; l0 += KF) {
        // ---- stage the chunk (buf is all zero, posc all -1 here) ----
        const int mycol = gcol;
        if (mycol >= 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int u = 0; u < 6; ++u) buf[(3 * ss + r) * IM_GS + mycol + u] = g[6 * r + u];
            posc[32 * ss + mycol / 6] = so;
        }
        for (int k = tid; k < NKS; k += NT) {
            unsigned m = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = l0 + (4 * k + r) / 3;
                if (i < nl) m |= ftm[i];
            }
            kmask[k] = m;
        }
        __syncthreads();
        fetch(l0 + KF);   // the next chunk's G blocks, under this chunk's MFMAs
        double dv[KF];
#pragma unroll
        for (int s = 0; s < KF; ++s) {
            dv[s] = 0.0;
            if (dbo && l0 + s < nl) {
                const int o = posc[32 * s + dc];
                if (o >= 0) dv[s] = fb.obs_g[(size_t)(fo0[flist[l0 + s]] + o) * OBG_STRIDE + deoff];
            }
        }
        // ---- rank-KR update of this wave's tiles ----
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const unsigned km = kmask[ks];
            const double* brow = buf + (4 * ks + lr) * IM_GS + lc;
#pragma unroll
            for (int q = 0; q < IM_PPW; ++q)
                if (pv[q] && ((km >> pti[q]) & (km >> ptj[q]) & 1u))
                    acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(brow[16 * pti[q]], brow[16 * ptj[q]], acc[q], 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < KF; ++s) dsum += dv[s];
        __syncthreads();
        // ---- back to all-zero rows / empty table ----
        if (mycol >= 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int u = 0; u < 6; ++u) buf[(3 * ss + r) * IM_GS + mycol + u] = 0.0;
            posc[32 * ss + mycol / 6] = -1;
        }
        // no barrier before the next scatter: the rows of feature slot ss are written,
        // cleared and re-written only by the 32 lanes (tid >> 5 == ss) of one wave, in
        // program order (in-order LDS), and kmask is rewritten by wave 0 after every wave
        // passed the barrier above
        asm volatile("" ::: "memory");
    }
    KT* F = ws.Hthin + (size_t)b * Cmax * (Cmax + 1);
    const int ldf = Cmax + 1;
#pragma unroll
    for (int q = 0; q < IM_PPW; ++q) {
        if (!pv[q]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * pti[q] + lr + 4 * r, col = 16 * ptj[q] + lc;
            // lower triangle only (stage B reads nothing else; the block-diagonal
            // owners below add their terms to the lower elements)
            if (row < C && col <= row) F[(size_t)row * ldf + col] = -acc[q][r];
        }
    }
    __syncthreads();   // the tiles' stores are visible to the block-diagonal owners
    if (dbo) {
        if (de < 21) {
            int x = (int)((sqrtf(8.0f * (float)de + 1.0f) - 1.0f) * 0.5f);
            while (x * (x + 1) / 2 > de) --x;
            while ((x + 1) * (x + 2) / 2 <= de) ++x;
            const int y = de - x * (x + 1) / 2;
            const size_t i0 = (size_t)(6 * dc + x) * ldf + 6 * dc + y;   // x >= y: lower triangle
            F[i0] += dsum;
        } else {
            F[(size_t)(6 * dc + de - 21) * ldf + Cmax] = dsum;
        }
    }
    if (tid == 0) info[1] = C;
}

// ---------------------------------------------------------------------------
// Record-reading MFMA assembly for windows over 32 cams (round 6): the SYRK of
// k_info_mfma, A = blockdiag_i(Hx_i^T Hx_i) - Gall^T Gall, on fp64 MFMA tiles
// for up to 84 cams.  The lower 16 x 16 tiles of A are dealt over PARTS
// workgroups per filter (IB_NW waves x IB_PPW tiles each, a filter's parts on
// one XCD); every part stages the same chunks of IB_KF included features' G
// rows from k_feature's Gram records (G and the cam of each record in one
// fetch, issued under the previous chunk's MFMAs) and updates only its own
// tiles, staging only the features that touch one of them.  The block-diagonal
// terms are summed by the part that owns their tile, b by the part owning the
// cam's diagonal tile.  A is stored as both triangles: stage B1 of the
// global-memory Kalman path (k_kal_b1) reads whole rows of it.  (Replaces the
// VALU 6 x 6 cam-pair assembly k_info there: 50x400 compress 8.3 ms.)
// ---------------------------------------------------------------------------
constexpr int IB_NW = 16, IB_PPW = 5, IB_KF = 8, IB_TPP = IB_NW * IB_PPW, IB_MAXN = 84;
constexpr int IB_KMS = (3 * IB_KF / 4 + 1) & ~1;   // k-step masks (an even count: posc stays 8-byte aligned)
// LDS row stride (doubles) of the staged Gall rows: >= 16 ceil(C / 16), = 16 mod 32 (as IM_GS)
__host__ __device__ constexpr int ib_gs(int C) { return 32 * ((C + 15) / 32) + 16; }
__host__ __device__ constexpr size_t info_big_lds(int Cmax, int maxnf) {
    return (size_t)3 * IB_KF * ib_gs(Cmax) * sizeof(double) + IB_KMS * sizeof(unsigned) +
           (size_t)(IB_MAXN * IB_KF + 4 * maxnf + 1) * sizeof(int);
}
int info_big_parts(int Cmax) {
    const int TT = (Cmax + 15) / 16;
    return (TT * (TT + 1) / 2 + IB_TPP - 1) / IB_TPP;
}

// NDO: (cam, element) pairs per thread, 27 Nmax <= NDO 64 IB_NW (2: up to 75 cams)
template <typename T, int NDO>
__global__ void __launch_bounds__(64 * IB_NW) k_info_big(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws, int maxnf) {
    constexpr int NT = 64 * IB_NW, KF = IB_KF, KR = 3 * KF, NKS = KR / 4;
    static_assert(KR % 4 == 0 && NKS <= IB_KMS && IB_MAXN * KF <= NT && 27 * IB_MAXN <= 3 * NT, "k_info_big shape");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const Blk3 bk = xcd_blk3();   // grid (parts, B): a filter's parts on one XCD
    const int b = bk.y, part = bk.x;
    const int tid = threadIdx.x, lane = tid & 63, lc = lane & 15, lr = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* info = ws.info + 4 * b;
    if (info[0] == 0) {   // nothing stacked: empty update
        if (tid == 0 && part == 0) info[1] = 0;
        return;
    }
    const int nc = st.ncams[b], C = 6 * nc, Cmax = ws.Cmax, GS = ib_gs(Cmax);
    const int TT = (C + 15) >> 4, npair = TT * (TT + 1) / 2;
    if (part * IB_TPP >= npair) {   // no tile of this window in this part (a smaller window)
        if (tid == 0 && part == 0) info[1] = C;
        return;
    }
    double* buf = reinterpret_cast<double*>(smem_raw);              // [KR][GS] dense rows of Gall
    unsigned* kmask = reinterpret_cast<unsigned*>(buf + KR * GS);   // [NKS] tiles touched per k-step
    int* posc = reinterpret_cast<int*>(kmask + IB_KMS);             // [KF][IB_MAXN] cam -> record (-1)
    int* flist = posc + IB_MAXN * KF;                               // [maxnf] included features, in order
    unsigned* ftm = reinterpret_cast<unsigned*>(flist + maxnf);     // [maxnf] their tile masks
    int* fo0 = reinterpret_cast<int*>(ftm + maxnf);                 // [maxnf] first record
    int* fM = fo0 + maxnf;                                          // [maxnf] records (0: not included)
    int* s_n = fM + maxnf;
    const int fbeg = fb.feat_off[b], fend = fb.feat_off[b + 1], nf = fend - fbeg;
    // tile rows / columns of this part's tiles: a feature none of whose tile pairs
    // falls in the part is not staged here at all
    unsigned prow = 0, pcol = 0;
    for (int p = part * IB_TPP; p < part * IB_TPP + IB_TPP && p < npair; ++p) {
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= p) ++ti;
        prow |= 1u << ti;
        pcol |= 1u << (p - ti * (ti + 1) / 2);
    }
    unsigned* fmk = ftm;   // per feature first (index f), compacted to the list order below
    for (int f = tid; f < nf; f += NT) {
        const int a0 = fb.obs_off[fbeg + f], a1 = fb.obs_off[fbeg + f + 1];
        const int M = fb.include[fbeg + f] ? a1 - a0 : 0;
        unsigned m = 0;
        for (int o = 0; o < M; ++o) {   // tile masks (<= 32 tile rows: C <= 512)
            const int c = fb.obs_cam[a0 + o];
            m |= (1u << ((6 * c) >> 4)) | (1u << ((6 * c + 5) >> 4));
        }
        fo0[f] = a0;
        fM[f] = (m & prow) && (m & pcol) ? M : 0;
        fmk[f] = m;
    }
    for (int e = tid; e < KR * GS; e += NT) buf[e] = 0.0;
    for (int e = tid; e < IB_MAXN * KF; e += NT) posc[e] = -1;
    __syncthreads();
    if (wv == 0) {   // the included features of this part, in order
        int base = 0;
        for (int f0 = 0; f0 < nf; f0 += 64) {
            const int f = f0 + lane;
            const bool in = f < nf && fM[f] > 0;
            const unsigned long long bal = __ballot(in);
            if (in) flist[base + __popcll(bal & ((1ull << lane) - 1ull))] = f;
            base += __popcll(bal);
        }
        if (lane == 0) *s_n = base;
    }
    __syncthreads();
    const int nl = *s_n;
    // ftm[i] (list order) overwrites fmk[f] (feature order) in place: i <= f, so read all first
    unsigned mk[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid + NT * u;
        mk[u] = i < nl ? fmk[flist[i]] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid + NT * u;
        if (i < nl) ftm[i] = mk[u];
    }
    // (maxnf <= 4 NT: launch_compress)
    // this wave's tiles: p = part IB_TPP + IB_PPW wv + q (lower, row-major order)
    int pti[IB_PPW], ptj[IB_PPW];
    bool pv[IB_PPW];
    v4d acc[IB_PPW];
#pragma unroll
    for (int q = 0; q < IB_PPW; ++q) {
        const int p = part * IB_TPP + IB_PPW * wv + q;
        int ti = (int)((sqrtf(8.0f * (float)p + 1.0f) - 1.0f) * 0.5f);
        while (ti * (ti + 1) / 2 > p) --ti;
        while ((ti + 1) * (ti + 2) / 2 <= p) ++ti;
        pti[q] = __builtin_amdgcn_readfirstlane(ti);
        ptj[q] = __builtin_amdgcn_readfirstlane(p - ti * (ti + 1) / 2);
        pv[q] = p < npair;
        acc[q] = v4d{0.0, 0.0, 0.0, 0.0};
    }
    // (cam, element) pairs of the block diagonal (element < 21: packed lower DS) and
    // b (21..26) this part sums: those whose element lies in one of its tiles
    // (b: part 0)
    int dco[NDO], drec[NDO];
    double dsum[NDO];
#pragma unroll
    for (int u = 0; u < NDO; ++u) {
        const int e = tid + NT * u, dc = e / 27, de = e - 27 * dc;
        bool own = false;
        if (e < 27 * nc) {
            if (de < 21) {
                int x = 0;
                while ((x + 1) * (x + 2) / 2 <= de) ++x;
                const int y = de - x * (x + 1) / 2, ti = (6 * dc + x) >> 4, tj = (6 * dc + y) >> 4;
                own = (ti * (ti + 1) / 2 + tj) / IB_TPP == part;
            } else {   // b of cam dc: the part of its diagonal tile (every feature seeing dc is staged there)
                const int t = (6 * dc) >> 4;
                own = (t * (t + 1) / 2 + t) / IB_TPP == part;
            }
        }
        dco[u] = own ? dc : -1;
        drec[u] = de < 21 ? OBG_DS + de : OBG_UB + (de - 21);
        dsum[u] = 0.0;
    }
    // staging slot: chunk feature ss, its record so
    const int ss = tid / IB_MAXN, so = tid - IB_MAXN * (tid / IB_MAXN);
    double g[18];
    int gcol = -1, gcam = 0;
    auto fetch = [&](int l0) {
        gcol = -1;
        if (tid < IB_MAXN * KF && l0 + ss < nl) {
            const int f = flist[l0 + ss];
            if (so < fM[f]) {
                const double* r = fb.obs_g + (size_t)(fo0[f] + so) * OBG_STRIDE;
#pragma unroll
                for (int k = 0; k < 18; ++k) g[k] = r[OBG_G + k];
                gcam = (int)r[OBG_CAM];
                gcol = 6 * gcam;
            }
        }
    };
    __syncthreads();   // ftm complete
    fetch(0);
    for (int l0 = 0; l0 < nl; l0 += KF) {
        // ---- stage the chunk (buf is all zero, posc all -1 here) ----
        const int mycol = gcol, mycam = gcam;
        if (mycol >= 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int u = 0; u < 6; ++u) buf[(3 * ss + r) * GS + mycol + u] = g[6 * r + u];
            posc[IB_MAXN * ss + mycam] = so;
        }
        for (int k = tid; k < NKS; k += NT) {
            unsigned m = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = l0 + (4 * k + r) / 3;
                if (i < nl) m |= ftm[i];
            }
            kmask[k] = m;
        }
        __syncthreads();
        fetch(l0 + KF);   // the next chunk's G blocks, under this chunk's MFMAs
        // ---- rank-KR update of this wave's tiles ----
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const unsigned km = kmask[ks];
            const double* brow = buf + (4 * ks + lr) * GS + lc;
#pragma unroll
            for (int q = 0; q < IB_PPW; ++q)
                if (pv[q] && ((km >> pti[q]) & (km >> ptj[q]) & 1u))
                    acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(brow[16 * pti[q]], brow[16 * ptj[q]], acc[q], 0, 0, 0);
        }
        // block-diagonal / b terms of the chunk (after the MFMAs: no registers held across them)
#pragma unroll
        for (int u = 0; u < NDO; ++u)
#pragma unroll
            for (int s = 0; s < KF; ++s)
                if (dco[u] >= 0 && l0 + s < nl) {
                    const int o = posc[IB_MAXN * s + dco[u]];
                    if (o >= 0) dsum[u] += fb.obs_g[(size_t)(fo0[flist[l0 + s]] + o) * OBG_STRIDE + drec[u]];
                }
        __syncthreads();
        // ---- back to all-zero rows / empty table; a feature slot's 84 records span
        // two waves, so the next chunk's scatter waits for every clear (barrier) ----
        if (mycol >= 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int u = 0; u < 6; ++u) buf[(3 * ss + r) * GS + mycol + u] = 0.0;
            posc[IB_MAXN * ss + mycam] = -1;
        }
        __syncthreads();
    }
    KT* F = ws.Hthin + (size_t)b * Cmax * (Cmax + 1);
    const int ldf = Cmax + 1;
#pragma unroll
    for (int q = 0; q < IB_PPW; ++q) {
        if (!pv[q]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * pti[q] + lr + 4 * r, col = 16 * ptj[q] + lc;
            if (row < C && col < C) {   // both triangles (a diagonal tile holds both already)
                F[(size_t)row * ldf + col] = -acc[q][r];
                if (pti[q] != ptj[q]) F[(size_t)col * ldf + row] = -acc[q][r];
            }
        }
    }
    __syncthreads();   // the tiles' stores are visible to the block-diagonal owners
#pragma unroll
    for (int u = 0; u < NDO; ++u) {
        if (dco[u] < 0) continue;
        const int dc = dco[u], de = drec[u] < OBG_UB ? drec[u] - OBG_DS : 21 + drec[u] - OBG_UB;
        if (de < 21) {
            int x = 0;
            while ((x + 1) * (x + 2) / 2 <= de) ++x;
            const int y = de - x * (x + 1) / 2;
            F[(size_t)(6 * dc + x) * ldf + 6 * dc + y] += dsum[u];
            if (x != y) F[(size_t)(6 * dc + y) * ldf + 6 * dc + x] += dsum[u];
        } else {
            F[(size_t)(6 * dc + de - 21) * ldf + Cmax] = dsum[u];
        }
    }
    if (tid == 0 && part == 0) info[1] = C;
}

// ---------------------------------------------------------------------------
// Fused information assembly (windows up to 32 cams): k_info_mfma's SYRK
// without the per-observation Gram records.  Each staged feature's G_i,
// Hx_i^T Hx_i and UB_i are rebuilt in the workgroup from the inputs -- the
// cam poses (a per-cam geometry table in LDS), p_w, z -- and the feature's QR
// record (fqr: X = R^-1, g = (Q^T r)[0:3], written by k_feature), so k_feature
// stores 80 bytes per feature instead of 368 per observation and nothing is
// read back (msckf.py:429-556: measurement_jacobian, feature_jacobian's
// projection and the QR compression, through the Gram identity of k_info).
//
// Per observation (one producer thread each), with Jc the 4 x 3 derivative of
// z by the cam-0 point (msckf.py:457-475) and B~ = [ [p_c0]x | -R_w_c0 ] with
// the observability projection (msckf.py:484-490) applied, Hx_i = Jc B~ and
// H_f,i = -Hx_i[:, 3:6].  With Jc^T Jc = L L^T (3 x 3 Cholesky):
//     H^ = L^T B~ (3 x 6),  n^ = L^-1 Jc^T r_i
//     Hx_i^T Hx_i = H^^T H^,  Hx_i^T r_i = H^^T n^,
//     H_f,i^T Hx_i = F^T H^ with F = -H^[:, 3:6],  G_i = X^T (F^T H^),
// -- the rank-3 form of the gate's records, in fp64.  The update is invariant
// to the orthogonal row maps involved (quirk Q4).
//
// Pipeline: IF_KF features per chunk; producer thread (s, c) (waves 0..3,
// IF_KF x 32 threads) builds feature s's observation of cam c into the chunk's
// LDS rows of Gall (zeros if the feature does not see cam c) and adds its
// Hx^T Hx / UB terms into the (s, c) slot of an LDS accumulator (summed over
// s at the end).  The producers build chunk i + 1 (its global inputs loaded
// one iteration earlier) while the four tile-owning waves run chunk i's
// MFMAs (double-buffered rows, one barrier per chunk).  Producers and tile
// owners run separate code paths, so neither carries the other's registers:
// the producer's fp64 chain beside 20 accumulator tiles per owner wave.
// ---------------------------------------------------------------------------
constexpr int IF_KF = 8, IF_KR = 3 * IF_KF, IF_NKS = IF_KR / 4, IF_NP = 32 * IF_KF;
constexpr int IF_ACC = 27, IF_CG = 27;   // doubles per accumulator slot / per cam geometry record
constexpr int IF_NPW = IF_NP / 64;       // producer waves
// Phase timing (probe builds, -DMSCKF_GATE_PROBE; tools/probes/info_phases.py):
// s_memtime sums of one producer and one tile-owner wave per filter --
// [0] prologue, [1] producer load issue, [2] producer build, [3] producer
// barrier wait, [4] owner MFMA phase, [5] owner barrier wait, [6] iterations,
// [7] filters.
#ifdef MSCKF_GATE_PROBE
__device__ unsigned long long g_info_probe[8];
extern "C" int msckf_info_probe_read(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_info_probe), sizeof(g_info_probe)) != hipSuccess) return -1;
    static unsigned long long zero[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_info_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#define IPROBE_T(v) const unsigned long long v = __builtin_readcyclecounter()
#else
#define IPROBE_T(v) (void)0
#endif
constexpr int IF_NW = 8;                 // waves per workgroup: 4 producers + 4 tile owners (two per SIMD)

__host__ __device__ constexpr size_t info_fused_lds(int maxnf) {
    return (size_t)(2 * IF_KR * IM_GS + IF_KF * 32 * IF_ACC + 32 * IF_CG) * sizeof(double) + (size_t)maxnf * 48 + 16;
}

// Reciprocal and reciprocal square root of the fused producer: the hardware
// approximations (v_rcp_f64 / v_rsq_f64) and one Newton step each -- within a
// couple of ulps, against ~10 instructions of an IEEE division / sqrt.  (The
// assembled information is invariant to these rounding-level choices well
// inside the 1e-9 fp64 parity bound.)
__device__ __forceinline__ double if_rcp(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    return r * fma(-x, r, 2.0);
}
__device__ __forceinline__ double if_rsq(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    return r * fma(-0.5 * x * r, r, 1.5);
}

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>), in order
template <int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}

// Lower 16 x 16 tile p (row-major lower order) -> row / column tile.
__host__ __device__ constexpr int lt_row(int p) {
    int i = 0;
    while ((i + 1) * (i + 2) / 2 <= p) ++i;
    return i;
}
__host__ __device__ constexpr int lt_col(int p) { return p - lt_row(p) * (lt_row(p) + 1) / 2; }

// Tile-owner wave CW of k_info_fused: tiles p = PPW CW + q.  A tile takes a
// k-step's rank-4 update iff the k-step's features touch both its column
// ranges (km bits ti and tj; tiles past the window's last tile row never
// match, ftm only has bits of real tiles).  Operands of the next batch of
// five tiles are read before the current batch's MFMAs.
template <int CW, int PPW>
__device__ __forceinline__ void info_owner(const double* buf, const unsigned* ftm, int nl, int lane, KT* F, int C,
                                           int ldf) {
    const int lc = lane & 15, lr = lane >> 4;
    v4d tacc[PPW];
#pragma unroll
    for (int q = 0; q < PPW; ++q) tacc[q] = v4d{0.0, 0.0, 0.0, 0.0};
#ifdef MSCKF_GATE_PROBE
    unsigned long long pr4 = 0, pr5 = 0;
#endif
    __syncthreads();   // chunk 0 in buffer 0
    for (int l0 = 0, it = 0; l0 < nl; l0 += IF_KF, ++it) {
        IPROBE_T(u0);
        const double* cb = buf + (size_t)(it & 1) * IF_KR * IM_GS + lr * IM_GS + lc;
        unsigned kmv[IF_NKS];
#pragma unroll
        for (int ks = 0; ks < IF_NKS; ++ks) {
            const int sa = l0 + (4 * ks) / 3, sb = l0 + (4 * ks + 3) / 3;
            kmv[ks] = __builtin_amdgcn_readfirstlane((sa < nl ? ftm[sa] : 0u) | (sb < nl ? ftm[sb] : 0u));
        }
        constexpr int HQ = 5, NHB = (PPW + HQ - 1) / HQ, NBAT = IF_NKS * NHB;
        double oa[2][HQ], ob[2][HQ];
        auto ldb = [&](auto nc) {
            constexpr int n = decltype(nc)::value, ks = n / NHB, h = (n - ks * NHB) * HQ, sl = n & 1;
            static_for<HQ>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (h + q < PPW) {
                    constexpr int p = PPW * CW + h + q;
                    oa[sl][q] = cb[4 * ks * IM_GS + 16 * lt_row(p)];
                    ob[sl][q] = cb[4 * ks * IM_GS + 16 * lt_col(p)];
                }
            });
        };
        auto mfb = [&](auto nc) {
            constexpr int n = decltype(nc)::value, ks = n / NHB, h = (n - ks * NHB) * HQ, sl = n & 1;
            const unsigned km = kmv[ks];
            static_for<HQ>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                if constexpr (h + q < PPW) {
                    constexpr int p = PPW * CW + h + q;
                    constexpr unsigned need = (1u << lt_row(p)) | (1u << lt_col(p));
                    if ((km & need) == need)
                        tacc[h + q] = __builtin_amdgcn_mfma_f64_16x16x4f64(oa[sl][q], ob[sl][q], tacc[h + q], 0, 0, 0);
                }
            });
        };
        ldb(std::integral_constant<int, 0>{});
        static_for<NBAT>([&](auto nc) {
            constexpr int n = decltype(nc)::value;
            if constexpr (n + 1 < NBAT) ldb(std::integral_constant<int, n + 1>{});
            mfb(nc);
        });
#ifdef MSCKF_GATE_PROBE
        for (int q = 0; q < PPW; ++q) asm volatile("" : "+v"(tacc[q]));   // the MFMAs have completed
        IPROBE_T(u1);
#endif
        __syncthreads();
#ifdef MSCKF_GATE_PROBE
        IPROBE_T(u2);
        pr4 += u1 - u0;
        pr5 += u2 - u1;
#endif
    }
#ifdef MSCKF_GATE_PROBE
    if (CW == 0 && lane == 0) {
        atomicAdd(&g_info_probe[4], pr4);
        atomicAdd(&g_info_probe[5], pr5);
    }
#endif
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
        const int p = PPW * CW + q, ti = lt_row(p), tj = lt_col(p);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * ti + lr + 4 * r, col = 16 * tj + lc;
            // the lower triangle only: stage B reads A from it (k_kal_b)
            if (row < C && col <= row) F[(size_t)row * ldf + col] = -tacc[q][r];
        }
    }
}

template <typename T, int NW>
__global__ void __launch_bounds__(64 * NW) k_info_fused(DevState<T> st, Params<T> prm, FeatBatch<T> fb, UpdWs<T> ws,
                                                        int maxnf) {
    // waves 0 .. IF_NPW-1 build the chunks (IF_NP threads), the others own the tiles
    constexpr int NT = 64 * NW, NCW = NW - IF_NPW, PPW = (78 + NCW - 1) / NCW;
    static_assert(IF_NP == 64 * IF_NPW && NCW > 0 && PPW * NCW >= 78 && IF_KR % 4 == 0, "k_info_fused shape");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* info = ws.info + 4 * b;
    if (info[0] == 0) {   // nothing stacked: empty update
        if (tid == 0) info[1] = 0;
        return;
    }
    const int nc = st.ncams[b], C = 6 * nc, Cmax = ws.Cmax;
    double* buf = reinterpret_cast<double*>(smem_raw);          // [2][KR][IM_GS] dense rows of Gall
    double* acc = buf + 2 * IF_KR * IM_GS;                      // [KF][32][IF_ACC] Hx^T Hx (21) | UB (6)
    double* camg = acc + IF_KF * 32 * IF_ACC;                   // [32][IF_CG] R0 | R1 | t1 | p | R(q_null) g
    int* flist = reinterpret_cast<int*>(camg + 32 * IF_CG);     // [maxnf] included features, in order
    unsigned* ftm = reinterpret_cast<unsigned*>(flist + maxnf); // [maxnf] their tile masks
    int* fo0 = reinterpret_cast<int*>(ftm + maxnf);             // [maxnf] first observation
    int* fM = fo0 + maxnf;                                      // [maxnf] observations (0: not included)
    unsigned char* posb = reinterpret_cast<unsigned char*>(fM + maxnf);   // [maxnf][32] cam -> observation (0xff)
    int* s_n = reinterpret_cast<int*>(posb + 32 * (size_t)maxnf);
    const int fbeg = fb.feat_off[b], fend = fb.feat_off[b + 1], nf = fend - fbeg;
    for (int e = tid; e < 2 * IF_KR * IM_GS + IF_KF * 32 * IF_ACC; e += NT) buf[e] = 0.0;   // rows and accumulators
    for (int e = tid; e < 8 * nf; e += NT) reinterpret_cast<int*>(posb)[e] = -1;
    for (int f = tid; f < nf; f += NT) {
        const int a0 = fb.obs_off[fbeg + f], a1 = fb.obs_off[fbeg + f + 1];
        fo0[f] = a0;
        fM[f] = fb.include[fbeg + f] ? a1 - a0 : 0;
    }
    double g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) g[k] = (double)st.imu[(size_t)b * IMU_STRIDE + I_G + k];
    if (tid < nc) {   // per-cam geometry (k_feature's per-observation poses, once per cam)
        const T* cq = st.cams + ((size_t)b * st.Nmax + tid) * CAM_STRIDE;
        double q0[4], qn[4], R0[9], R1[9], Rn[9], R01[9], t01[3], tmp[3];
        for (int k = 0; k < 4; ++k) { q0[k] = (double)cq[C_Q + k]; qn[k] = (double)cq[C_QN + k]; }
        for (int k = 0; k < 9; ++k) R01[k] = (double)prm.R01[k];
        for (int k = 0; k < 3; ++k) t01[k] = (double)prm.t01[k];
        quat_to_rot(q0, R0);
        mat3_mul(R01, R0, R1);
        mat3T_vec(R1, t01, tmp);
        quat_to_rot(qn, Rn);
        double* cg = camg + tid * IF_CG;
        for (int k = 0; k < 9; ++k) { cg[k] = R0[k]; cg[9 + k] = R1[k]; }
        for (int k = 0; k < 3; ++k) {
            const double cp = (double)cq[C_P + k];
            cg[18 + k] = cp - tmp[k];
            cg[21 + k] = cp;
        }
        mat3_vec(Rn, g, cg + 24);
    }
    __syncthreads();
    for (int f = tid >> 5; f < nf; f += NT / 32) {   // cam -> observation, 32 lanes per feature
        const int o = tid & 31;
        if (o < fM[f]) posb[32 * f + fb.obs_cam[fo0[f] + o]] = (unsigned char)o;
    }
    if (wv == 0) {   // the included features, in order
        int base = 0;
        for (int f0 = 0; f0 < nf; f0 += 64) {
            const int f = f0 + lane;
            const bool in = f < nf && fM[f] > 0;
            const unsigned long long bal = __ballot(in);
            if (in) flist[base + __popcll(bal & ((1ull << lane) - 1ull))] = f;
            base += __popcll(bal);
        }
        if (lane == 0) *s_n = base;
    }
    __syncthreads();
    const int nl = *s_n;
    for (int i = tid; i < nl; i += NT) {
        const unsigned char* pb = posb + 32 * flist[i];
        unsigned m = 0;
        for (int c = 0; c < nc; ++c)
            if (pb[c] != 0xff) m |= (1u << ((6 * c) >> 4)) | (1u << ((6 * c + 5) >> 4));
        ftm[i] = m;
    }
    const int ps = (tid % IF_NP) >> 5, pc = tid & 31;
    // Producer thread (ps, pc) of chunk [l0, l0 + KF): feature ps's observation of
    // cam pc.  pload issues its global loads (kept raw in registers: a conversion
    // here would wait for them), pbuild forms the rows one MFMA phase later.
    struct PIn {
        int o, og;   // observation of cam pc in the feature (0xff: none), its global index
        T pw[3], z[4];
        double x[6], gr[3], ill;   // ill != 0: read the feature's Gram records (k_feature, FQR_FLAG)
    };
    auto pload = [&](int l0, PIn& in) {
        const int li = l0 + ps;
        const int f = (li < nl && pc < nc) ? flist[li] : -1;
        in.o = f >= 0 ? (int)posb[32 * f + pc] : 0xff;
        if (in.o == 0xff) return;
        const int fg = fbeg + f, og = fo0[f] + in.o;
        in.og = og;
#pragma unroll
        for (int k = 0; k < 3; ++k) in.pw[k] = fb.p_w[3 * fg + k];
        const T* zp = fb.obs_z + (size_t)og * 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) in.z[k] = zp[k];
        const double* qr = fb.fqr + (size_t)fg * FQR_STRIDE;
#pragma unroll
        for (int k = 0; k < 6; ++k) in.x[k] = qr[FQR_X + k];
#pragma unroll
        for (int k = 0; k < 3; ++k) in.gr[k] = qr[FQR_G + k];
        in.ill = qr[FQR_FLAG];
    };
    auto pbuild = [&](const PIn& in, int bb) {
        if (pc >= nc) return;
        double* dst = buf + (size_t)bb * IF_KR * IM_GS + 3 * ps * IM_GS + 6 * pc;
        if (in.o == 0xff) {
#pragma unroll
            for (int t = 0; t < 3; ++t)
#pragma unroll
                for (int u = 0; u < 6; ++u) dst[t * IM_GS + u] = 0.0;
            return;
        }
        if (in.ill != 0.0) {   // ill-conditioned feature: its Householder Gram record (rare)
            const double* rec = fb.obs_g + (size_t)in.og * OBG_STRIDE;
            double* ac = acc + (ps * 32 + pc) * IF_ACC;
#pragma unroll
            for (int t = 0; t < 3; ++t)
#pragma unroll
                for (int u = 0; u < 6; ++u) dst[t * IM_GS + u] = rec[OBG_G + 6 * t + u];
#pragma unroll
            for (int e = 0; e < 21; ++e) ac[e] += rec[OBG_DS + e];
#pragma unroll
            for (int x = 0; x < 6; ++x) ac[21 + x] += rec[OBG_UB + x];
            return;
        }
        const double pw[3] = {(double)in.pw[0], (double)in.pw[1], (double)in.pw[2]};
        const double z0 = (double)in.z[0], z1 = (double)in.z[1], z2 = (double)in.z[2], z3 = (double)in.z[3];
        const double* cg = camg + pc * IF_CG;
        double d0[3], d1[3], pc0[3], pc1[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) { d0[k] = pw[k] - cg[21 + k]; d1[k] = pw[k] - cg[18 + k]; }
        mat3_vec(cg, d0, pc0);
        mat3_vec(cg + 9, d1, pc1);
        // Jc (msckf.py:457-475): rows [a00 0 a02], [0 a00 a12], b-rows times R01
        const double i0 = if_rcp(pc0[2]), i1 = if_rcp(pc1[2]);
        const double a00 = i0, a02 = -pc0[0] * i0 * i0, a12 = -pc0[1] * i0 * i0;
        const double b00 = i1, b02 = -pc1[0] * i1 * i1, b12 = -pc1[1] * i1 * i1;
        double J2[3], J3[3];
#pragma unroll
        for (int m = 0; m < 3; ++m) {
            J2[m] = b00 * (double)prm.R01[m] + b02 * (double)prm.R01[6 + m];
            J3[m] = b00 * (double)prm.R01[3 + m] + b12 * (double)prm.R01[6 + m];
        }
        const double r0 = z0 - pc0[0] * i0, r1 = z1 - pc0[1] * i0, r2 = z2 - pc1[0] * i1, r3 = z3 - pc1[1] * i1;
        // L L^T = Jc^T Jc, n^ = L^-1 Jc^T r (a direction with no pivot is dropped)
        const double m00 = a00 * a00 + J2[0] * J2[0] + J3[0] * J3[0];
        const double m10 = J2[1] * J2[0] + J3[1] * J3[0];
        const double m20 = a02 * a00 + J2[2] * J2[0] + J3[2] * J3[0];
        const double m11 = a00 * a00 + J2[1] * J2[1] + J3[1] * J3[1];
        const double m21 = a12 * a00 + J2[2] * J2[1] + J3[2] * J3[1];
        const double m22 = a02 * a02 + a12 * a12 + J2[2] * J2[2] + J3[2] * J3[2];
        const double n0 = a00 * r0 + J2[0] * r2 + J3[0] * r3;
        const double n1 = a00 * r1 + J2[1] * r2 + J3[1] * r3;
        const double n2 = a02 * r0 + a12 * r1 + J2[2] * r2 + J3[2] * r3;
        const double il0 = m00 > 0 ? if_rsq(m00) : 0.0, l00 = m00 * il0;
        const double l10 = m10 * il0, l20 = m20 * il0;
        const double e11 = m11 - l10 * l10;
        const double il1 = e11 > 0 ? if_rsq(e11) : 0.0, l11 = e11 * il1;
        const double l21 = (m21 - l20 * l10) * il1;
        const double e22 = m22 - l20 * l20 - l21 * l21;
        const double il2 = e22 > 0 ? if_rsq(e22) : 0.0, l22 = e22 * il2;
        const double h0 = n0 * il0, h1 = (n1 - l10 * h0) * il1, h2 = (n2 - l20 * h0 - l21 * h1) * il2;
        // B~ = [ [p_c0]x | -R_w_c0 ] (I - u u^T / u^T u), u = [R(q_null) g ; (p_w - p) x g]  (msckf.py:484-490)
        double u[6];
#pragma unroll
        for (int k = 0; k < 3; ++k) u[k] = cg[24 + k];
        u[3] = d0[1] * g[2] - d0[2] * g[1];
        u[4] = d0[2] * g[0] - d0[0] * g[2];
        u[5] = d0[0] * g[1] - d0[1] * g[0];
        double uu = 0.0;
#pragma unroll
        for (int k = 0; k < 6; ++k) uu += u[k] * u[k];
        const double iuu = if_rcp(uu);
        double H[3][6];   // B~, then H^ = L^T B~ in place (row a needs rows >= a only)
        {
            const double Sk[9] = {0.0, -pc0[2], pc0[1], pc0[2], 0.0, -pc0[0], -pc0[1], pc0[0], 0.0};
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                double row[6];
#pragma unroll
                for (int m = 0; m < 3; ++m) { row[m] = Sk[3 * a + m]; row[3 + m] = -cg[3 * a + m]; }
                double bu = 0.0;
#pragma unroll
                for (int m = 0; m < 6; ++m) bu += row[m] * u[m];
                bu *= iuu;
#pragma unroll
                for (int m = 0; m < 6; ++m) H[a][m] = row[m] - bu * u[m];
            }
        }
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            H[0][m] = l00 * H[0][m] + l10 * H[1][m] + l20 * H[2][m];
            H[1][m] = l11 * H[1][m] + l21 * H[2][m];
            H[2][m] = l22 * H[2][m];
        }
        // G_i = X^T (F^T H^), F = -H^[:, 3:6]; rows written as soon as formed
        const double x00 = in.x[0], x01 = in.x[1], x02 = in.x[2];
        const double x11 = in.x[3], x12 = in.x[4], x22 = in.x[5];
        double K[3][6];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int m = 0; m < 6; ++m) K[j][m] = -(H[0][3 + j] * H[0][m] + H[1][3 + j] * H[1][m] + H[2][3 + j] * H[2][m]);
#pragma unroll
        for (int m = 0; m < 6; ++m) {
            K[2][m] = x02 * K[0][m] + x12 * K[1][m] + x22 * K[2][m];
            K[1][m] = x01 * K[0][m] + x11 * K[1][m];
            K[0][m] = x00 * K[0][m];
        }
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int m = 0; m < 6; ++m) dst[t * IM_GS + m] = K[t][m];
        // Hx^T Hx (packed lower, as OBG_DS) and UB = Hx^T r - G^T g, into slot (ps, pc)
        const double gr0 = in.gr[0], gr1 = in.gr[1], gr2 = in.gr[2];
        double* ac = acc + (ps * 32 + pc) * IF_ACC;
#pragma unroll
        for (int x = 0, e = 0; x < 6; ++x)
#pragma unroll
            for (int y = 0; y <= x; ++y, ++e) ac[e] += H[0][x] * H[0][y] + H[1][x] * H[1][y] + H[2][x] * H[2][y];
#pragma unroll
        for (int x = 0; x < 6; ++x)
            ac[21 + x] += (H[0][x] * h0 + H[1][x] * h1 + H[2][x] * h2) - (K[0][x] * gr0 + K[1][x] * gr1 + K[2][x] * gr2);
    };
    KT* F = ws.Hthin + (size_t)b * Cmax * (Cmax + 1);
    const int ldf = Cmax + 1;
#ifdef MSCKF_GATE_PROBE
    unsigned long long pr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long t_beg = __builtin_readcyclecounter();
#endif
    if (wv < IF_NPW) {
        // ---- producers: chunk it + 1 is built while the consumers run chunk it;
        // its global loads were issued one iteration earlier ----
        PIn nxt;
        if (nl > 0) {
            PIn c0;
            pload(0, c0);
            pbuild(c0, 0);
        }
        if (IF_KF < nl) pload(IF_KF, nxt);
        __syncthreads();   // chunk 0 in buffer 0
#ifdef MSCKF_GATE_PROBE
        pr[0] += __builtin_readcyclecounter() - t_beg;
#endif
        for (int l0 = 0, it = 0; l0 < nl; l0 += IF_KF, ++it) {
            IPROBE_T(t0);
            PIn far;
            if (l0 + 2 * IF_KF < nl) pload(l0 + 2 * IF_KF, far);
            IPROBE_T(t1);
            if (l0 + IF_KF < nl) pbuild(nxt, (it + 1) & 1);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            IPROBE_T(t2);
            nxt = far;
            __syncthreads();
            IPROBE_T(t3);
#ifdef MSCKF_GATE_PROBE
            pr[1] += t1 - t0; pr[2] += t2 - t1; pr[3] += t3 - t2; pr[6] += 1;
#endif
        }
#ifdef MSCKF_GATE_PROBE
        if (tid == 0) {
            for (int k = 0; k < 4; ++k) atomicAdd(&g_info_probe[k], pr[k]);
            atomicAdd(&g_info_probe[6], pr[6]);
            atomicAdd(&g_info_probe[7], 1ull);
        }
#endif
    } else {
        // ---- tile owners: one code path per owner wave, so that every tile's
        // coordinates, LDS operand offsets and activity test are compile-time
        // constants (a runtime tile list cost ~12 scalar / readlane
        // instructions of bookkeeping per tile and k-step) ----
        const int cw = wv - IF_NPW;
        switch (cw) {
            case 0: info_owner<0, PPW>(buf, ftm, nl, lane, F, C, ldf); break;
            case 1: info_owner<1, PPW>(buf, ftm, nl, lane, F, C, ldf); break;
            case 2: info_owner<2, PPW>(buf, ftm, nl, lane, F, C, ldf); break;
            default: info_owner<3, PPW>(buf, ftm, nl, lane, F, C, ldf); break;
        }
    }
    __syncthreads();   // the tiles' stores are visible to the block-diagonal owners
    for (int e = tid; e < 27 * nc; e += NT) {   // (cam, element) owners: sum the KF slots
        const int dc = e / 27, de = e - 27 * dc;
        double dsum = 0.0;
#pragma unroll
        for (int s2 = 0; s2 < IF_KF; ++s2) dsum += acc[(s2 * 32 + dc) * IF_ACC + de];
        if (de < 21) {
            int x = (int)((sqrtf(8.0f * (float)de + 1.0f) - 1.0f) * 0.5f);
            while (x * (x + 1) / 2 > de) --x;
            while ((x + 1) * (x + 2) / 2 <= de) ++x;
            const int y = de - x * (x + 1) / 2;
            const size_t i0 = (size_t)(6 * dc + x) * ldf + 6 * dc + y;   // x >= y: lower triangle
            F[i0] += dsum;
        } else {
            F[(size_t)(6 * dc + de - 21) * ldf + Cmax] = dsum;
        }
    }
    if (tid == 0) info[1] = C;
}

// State correction (msckf.py:566-595).
template <typename T>
__global__ void __launch_bounds__(64) k_correct(DevState<T> st, UpdWs<T> ws) {
    const int b = blockIdx.x;
    const int n = ws.info[4 * b + 1];
    if (n == 0) return;
    const KT* dxk = ws.dx + (size_t)b * (st.Dmax + ws.Cmax);
    T dxs[21];
    for (int i = 0; i < 21; ++i) dxs[i] = (T)dxk[i];
    const T* dx = dxs;
    T* imu = st.imu + (size_t)b * IMU_STRIDE;
    const int nc = st.ncams[b];
    const int tid = threadIdx.x;
    if (tid == 0) {
        T dq[4], q[4];
        small_angle_quat(dx, dq);
        quat_mul(dq, imu + I_Q, q);
        for (int i = 0; i < 4; ++i) imu[I_Q + i] = q[i];
        for (int i = 0; i < 3; ++i) {
            imu[I_BG + i] += dx[3 + i];
            imu[I_V + i] += dx[6 + i];
            imu[I_BA + i] += dx[9 + i];
            imu[I_P + i] += dx[12 + i];
        }
        T dqe[4], Re[9], Rn[9];
        small_angle_quat(dx + 15, dqe);
        quat_to_rot(dqe, Re);
        mat3_mul(Re, imu + I_RIC, Rn);
        for (int e = 0; e < 9; ++e) imu[I_RIC + e] = Rn[e];
        for (int i = 0; i < 3; ++i) imu[I_TCI + i] += dx[18 + i];
    }
    T* cams = st.cams + (size_t)b * st.Nmax * CAM_STRIDE;
    for (int c = tid; c < nc; c += blockDim.x) {
        T d[6];
        for (int i = 0; i < 6; ++i) d[i] = (T)dxk[21 + 6 * c + i];
        T dq[4], q[4];
        small_angle_quat(d, dq);
        quat_mul(dq, cams + (size_t)c * CAM_STRIDE + C_Q, q);
        for (int i = 0; i < 4; ++i) cams[(size_t)c * CAM_STRIDE + C_Q + i] = q[i];
        for (int i = 0; i < 3; ++i) cams[(size_t)c * CAM_STRIDE + C_P + i] += d[3 + i];
    }
}

// ===========================================================================
// Host launchers
// ===========================================================================
template <typename T>
void launch_propagate(hipStream_t s, const DevState<T>& st, const Params<T>& prm, int nfilt, const int* filters,
                      const int* smp_off, const T* samples) {
    if (nfilt <= 0) return;
    constexpr int PKC = prop_pkc<T>();
    const size_t lds = (size_t)prop_lds<T>(PKC) * sizeof(T);
    lds_limit((const void*)k_propagate<T, PKC>, 160 * 1024);
    hipLaunchKernelGGL((k_propagate<T, PKC>), dim3(nfilt), dim3(64), lds, s, st, prm, nfilt, filters, smp_off,
                       samples);
}
template <typename T>
void launch_augment(hipStream_t s, const DevState<T>& st, int nfilt, const int* filters) {
    if (nfilt <= 0) return;
    hipLaunchKernelGGL(k_augment<T>, dim3(nfilt), dim3(256), 0, s, st, filters);
}
template <typename T>
void launch_prune(hipStream_t s, const DevState<T>& st, int nfilt, const int* filters, const int* keep_off,
                  const int* keep, const int* kcam_off, const int* keep_cams) {
    if (nfilt <= 0) return;
    const int row = st.Dmax * (int)sizeof(T);
    int R = (48 * 1024) / row;
    R = R < 1 ? 1 : (R > 32 ? 32 : R);
    hipLaunchKernelGGL(k_prune<T>, dim3(nfilt), dim3(256), (size_t)R * row, s, st, filters, keep_off, keep,
                       kcam_off, keep_cams, R);
}
template <typename T>
void launch_cov_diag(hipStream_t s, const DevState<T>& st, int nfilt, const int* filters, int i0, int n, T* out) {
    if (nfilt <= 0 || n <= 0) return;
    hipLaunchKernelGGL(k_cov_diag<T>, dim3((nfilt * n + 255) / 256), dim3(256), 0, s, st, filters, nfilt, i0, n,
                       out);
}
template <typename T>
void launch_triangulate(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                        const SegClasses& sc) {
    if (fb.nf == 0) return;
    for (int c = 0; c < SegClasses::NC; ++c) {   // the k_feature classes: S lanes, 2 views per lane
        const int cnt = sc.off[c + 1] - sc.off[c];
        if (cnt == 0) continue;
        const int* list = sc.list + sc.off[c];
        const int lanes = SegClasses::S[c] < 64 ? SegClasses::S[c] : 64;
        const int waves = (cnt * lanes + 63) / 64, blocks = (waves + 3) / 4;
        switch (SegClasses::S[c]) {
            case 8: hipLaunchKernelGGL((k_triangulate<T, 8, 2>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
            case 16: hipLaunchKernelGGL((k_triangulate<T, 16, 2>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
            case 32: hipLaunchKernelGGL((k_triangulate<T, 32, 2>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
            case 64: hipLaunchKernelGGL((k_triangulate<T, 64, 2>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
            default: hipLaunchKernelGGL((k_triangulate<T, 64, 4>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
        }
    }
}
template <typename T>
void launch_feature(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                    const SegClasses& sc) {
    if (fb.nf == 0) return;
    for (int c = 0; c < SegClasses::NC; ++c) {
        const int cnt = sc.off[c + 1] - sc.off[c];
        if (cnt == 0) continue;
        const int* list = sc.list + sc.off[c];
        const int lanes = SegClasses::S[c] < 64 ? SegClasses::S[c] : 64;   // S = 128: 2 observations per lane
        const int waves = (cnt * lanes + 63) / 64, blocks = (waves + 3) / 4;
        if (fb.gram) {
            switch (SegClasses::S[c]) {
                case 8: hipLaunchKernelGGL((k_feature<T, 8, 1, true>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                case 16: hipLaunchKernelGGL((k_feature<T, 16, 1, true>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                case 32: hipLaunchKernelGGL((k_feature<T, 32, 1, true>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                case 64: hipLaunchKernelGGL((k_feature<T, 64, 1, true>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                default: hipLaunchKernelGGL((k_feature<T, 64, 2, true>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
            }
        } else {
            switch (SegClasses::S[c]) {
                case 8: hipLaunchKernelGGL((k_feature<T, 8, 1, false>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                case 16: hipLaunchKernelGGL((k_feature<T, 16, 1, false>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                case 32: hipLaunchKernelGGL((k_feature<T, 32, 1, false>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                case 64: hipLaunchKernelGGL((k_feature<T, 64, 1, false>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
                default: hipLaunchKernelGGL((k_feature<T, 64, 2, false>), dim3(blocks), dim3(256), 0, s, st, prm, fb, list, cnt); break;
            }
        }
    }
}
template <typename T>
size_t gate_lds_bytes(int maxM) {
    const size_t n4 = 4 * maxM;
    return ((n4 * (n4 + 1) + 1) & ~(size_t)1) * sizeof(T) + (6 * n4 + 3 * n4 + 3 * n4 + 4) * sizeof(T) +
           (maxM + 4) * sizeof(int);
}

// Features are launched in size classes (by M, listed on the host at load
// time): the register-tile wave kernel sized for the class, or for the
// largest features the workgroup LDS kernel (global-memory kernel if even
// that does not fit).

// The workgroup gating kernels (M > 82) read the compact factors (V, W,
// Q^T r, tau, Hx, r) that k_feature otherwise skips.
bool feature_needs_compact(int maxM) { return maxM > GateClasses::LIM[GateClasses::NC - 2]; }

template <typename T>
void launch_gate(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                 const GateClasses& gc) {
    if (fb.nf == 0) return;
    lds_limit((const void*)k_gate_lds<T>, 160 * 1024);
    for (int c = 0; c < GateClasses::NC; ++c) {
        const int cnt = gc.off[c + 1] - gc.off[c];
        if (cnt == 0) continue;
        const int maxM = gc.maxM[c];
        const int* list = gc.list + gc.off[c];
        if constexpr (sizeof(T) == 4) {
            // fp32 large tracks (40 < M <= 82): by their block-count sub-lists, 8
            // blocks (M = 41) on the one-wave kernel, 9 .. 16 on k_gate_mfma_wt, a 2- to
            // 8-wave workgroup per feature (round 6; the one-wave classes of 7 and 8
            // blocks on k_gate_mfma_wt<7 / 8, 2> measured slower: 50x400 gate 12.05 ->
            // 12.39 ms, profiles/r06/wt2/)
            constexpr int wt_lo = 9;
            if (c == GateClasses::NC - 2 && gate_mfma_wt_fits(maxM)) {
                for (int j = 0; j + GateClasses::BIG_NB0 <= GateClasses::BIG_NB1; ++j) {
                    const int n = gc.big_off[j + 1] - gc.big_off[j], nb = j + GateClasses::BIG_NB0;
                    if (n == 0) continue;
                    if (nb < wt_lo) launch_gate_mfma<T>(s, st, prm, fb, gc.list + gc.big_off[j], n, gc.big_maxM[j]);
                    else launch_gate_mfma_wt<T>(s, st, prm, fb, gc.list + gc.big_off[j], n, nb, gc.big_maxM[j]);
                }
                continue;
            }
        }
        if constexpr (sizeof(T) == 8) {
            // fp64: 8 blocks and more (37 <= M <= 82) on k_gate_mfma_wt (round 6)
            if (c == GateClasses::NC - 3) {
                launch_gate_mfma_wt<T>(s, st, prm, fb, list, cnt, c + 1, maxM);
                continue;
            }
            if (c == GateClasses::NC - 2 && gate_mfma_wt_fits(maxM)) {
                for (int j = 0; j + GateClasses::BIG_NB0 <= GateClasses::BIG_NB1; ++j) {
                    const int n = gc.big_off[j + 1] - gc.big_off[j], nb = j + GateClasses::BIG_NB0;
                    if (n > 0) launch_gate_mfma_wt<T>(s, st, prm, fb, gc.list + gc.big_off[j], n, nb, gc.big_maxM[j]);
                }
                continue;
            }
        }
        if (c < GateClasses::NC - 2 && gate_mfma_fits(maxM, (int)sizeof(T))) {   // MFMA tiles (msckf_gate_mfma.hip)
            launch_gate_mfma<T>(s, st, prm, fb, list, cnt, maxM);
            continue;
        }
        const size_t lds = gate_lds_bytes<T>(maxM);
        const int threads = maxM <= 12 ? 64 : (maxM <= 20 ? 128 : 256);
        if (lds <= 160 * 1024)
            hipLaunchKernelGGL(k_gate_lds<T>, dim3(cnt), dim3(threads), lds, s, st, prm, fb, list);
        else
            hipLaunchKernelGGL(k_gate<T>, dim3(cnt), dim3(256), 0, s, st, prm, fb, list);
    }
}

template <typename T>
void launch_select(hipStream_t s, const DevState<T>& st, const FeatBatch<T>& fb, const UpdWs<T>& ws,
                   int row_cap) {
    hipLaunchKernelGGL(k_select<T>, dim3((st.B + 3) / 4), dim3(256), 0, s, st, fb, ws, row_cap);
}

template <typename T, int NT>
static void launch_info_cfg(hipStream_t s, const DevState<T>& st, const FeatBatch<T>& fb, const UpdWs<T>& ws,
                            int maxnf, int maxobs) {
    // features staged per batch: INFO_FB_MAX, or as many as the double-buffered slots fit in LDS
    const size_t per = ((size_t)2 * info_slot_doubles(st.Nmax)) * sizeof(double) + 4 * sizeof(unsigned long long) +
                       2 * st.Nmax * sizeof(int);
    int fbn = INFO_FB_MAX;
    while (fbn > 1 && fbn * per + 8 > 160 * 1024) --fbn;
    // filter-resident metadata when it fits beside the staged batches
    const size_t meta = (size_t)maxnf * (2 * sizeof(unsigned long long) + 2 * sizeof(int)) + (size_t)maxobs * sizeof(int);
    const bool pre = maxobs > 0 && fbn * per + 8 + meta <= 160 * 1024;
    const size_t lds = fbn * per + 8 + (pre ? meta : 0);
    const int TS = (st.Nmax + 7) / 8, ntl = TS * (TS + 1) / 2;
    const int parts = (ntl + (NT / 64) - 1) / (NT / 64);
    lds_limit((const void*)k_info<T, 1, NT>, lds);
    const int rmp = parts > 2;
    hipLaunchKernelGGL((k_info<T, 1, NT>), rmp ? dim3(parts, st.B) : dim3(st.B, parts), dim3(NT), lds, s, st, fb, ws, fbn,
                       pre ? maxnf : 0, pre ? maxobs : 0, rmp);
}

bool info_fused_fits(int Nmax, int maxnf) { return Nmax <= 32 && maxnf > 0 && info_fused_lds(maxnf) <= 160 * 1024; }

template <typename T>
void launch_compress(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const FeatBatch<T>& fb,
                     const UpdWs<T>& ws, int maxnf, int maxobs) {
    // windows up to 32 cams, no Gram records: the fused assembly (k_info_fused)
    if (!fb.gram) {
        const size_t lds = info_fused_lds(maxnf);
        lds_limit((const void*)k_info_fused<T, IF_NW>, lds);
        hipLaunchKernelGGL((k_info_fused<T, IF_NW>), dim3(st.B), dim3(64 * IF_NW), lds, s, st, prm, fb, ws, maxnf);
        return;
    }
    // windows up to 32 cams: fp64 MFMA tiles (k_info_mfma)
    const size_t lds_m = info_mfma_lds(maxnf, maxobs);
    if (st.Nmax <= 32 && maxobs > 0 && lds_m <= 160 * 1024) {
        lds_limit((const void*)k_info_mfma<T>, lds_m);
        hipLaunchKernelGGL((k_info_mfma<T>), dim3(st.B), dim3(64 * IM_NW), lds_m, s, st, fb, ws, maxnf, maxobs);
        return;
    }
    // windows of four or more k_info_big parts (over ~58 cams, up to 84): fp64 MFMA
    // tiles over several workgroups per filter.  (80x1000: compress 13.7 -> 12.1 ms;
    // at 50 cams, three parts, it measured 9.0 ms against 8.3 for k_info and is not
    // used there -- profiles/r06/info_big/)
    const size_t lds_b = info_big_lds(ws.Cmax, maxnf);
    if (info_big_parts(ws.Cmax) >= 4 && st.Nmax <= IB_MAXN && maxnf <= 4 * 64 * IB_NW && lds_b <= 160 * 1024) {
        const dim3 grid(info_big_parts(ws.Cmax), st.B);
        if (27 * st.Nmax <= 2 * 64 * IB_NW) {
            lds_limit((const void*)k_info_big<T, 2>, lds_b);
            hipLaunchKernelGGL((k_info_big<T, 2>), grid, dim3(64 * IB_NW), lds_b, s, st, fb, ws, maxnf);
        } else {
            lds_limit((const void*)k_info_big<T, 3>, lds_b);
            hipLaunchKernelGGL((k_info_big<T, 3>), grid, dim3(64 * IB_NW), lds_b, s, st, fb, ws, maxnf);
        }
        return;
    }
    // one wave per 8 x 8 tile of cam pairs
    const int TS = (st.Nmax + 7) / 8, ntl = TS * (TS + 1) / 2;
    if (ntl <= 4) launch_info_cfg<T, 256>(s, st, fb, ws, maxnf, maxobs);
    else if (ntl <= 8) launch_info_cfg<T, 512>(s, st, fb, ws, maxnf, maxobs);
    else if (ntl <= 10) launch_info_cfg<T, 640>(s, st, fb, ws, maxnf, maxobs);
    else launch_info_cfg<T, 1024>(s, st, fb, ws, maxnf, maxobs);   // > 10 tiles: several workgroups per filter
}

template <typename T>
void launch_kalman(hipStream_t s, const DevState<T>& st, const Params<T>& prm, const UpdWs<T>& ws,
                   KernelTimer* kt) {
    launch_kalman_chol<T>(s, st, prm, ws, kt);
    kt->begin(s, "kalman_correct");
    hipLaunchKernelGGL(k_correct<T>, dim3(st.B), dim3(64), 0, s, st, ws);
    kt->end(s);
}

#define INSTANTIATE(T)                                                                                    \
    template void launch_propagate<T>(hipStream_t, const DevState<T>&, const Params<T>&, int, const int*,     \
                                      const int*, const T*);                                               \
    template void launch_augment<T>(hipStream_t, const DevState<T>&, int, const int*);                     \
    template void launch_prune<T>(hipStream_t, const DevState<T>&, int, const int*, const int*, const int*,  \
                                  const int*, const int*);                                                 \
    template void launch_cov_diag<T>(hipStream_t, const DevState<T>&, int, const int*, int, int, T*);      \
    template void launch_triangulate<T>(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&,  \
                                        const SegClasses&);                                                 \
    template void launch_feature<T>(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const SegClasses&); \
    template void launch_gate<T>(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const GateClasses&); \
    template void launch_select<T>(hipStream_t, const DevState<T>&, const FeatBatch<T>&, const UpdWs<T>&, int); \
    template void launch_compress<T>(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const UpdWs<T>&, int, int); \
    template void launch_kalman<T>(hipStream_t, const DevState<T>&, const Params<T>&, const UpdWs<T>&, KernelTimer*);
INSTANTIATE(float)
INSTANTIATE(double)

}  // namespace msckf
