// msckf_common.h -- device layouts, kernel argument structs and SO(3) /
// JPL-quaternion device math shared by the MSCKF kernels (gfx950).
//
// Everything is templated on the arithmetic type T (float or double): one code
// path, two instantiations (fp64 for sequence-level parity, fp32 for the
// throughput configs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msckf {

// ---------------------------------------------------------------- layouts --
// Device IMU record: same field offsets as the ABI record (msckf_hip.h), padded.
constexpr int IMU_STRIDE = 48;
enum ImuField { I_Q = 0, I_P = 4, I_V = 7, I_BG = 10, I_BA = 13, I_QN = 16, I_PN = 20,
                I_VN = 23, I_RIC = 26, I_TCI = 35, I_G = 38, I_ALIAS = 41 };
// Device cam record (msckf_hip.h cam record + pad).
constexpr int CAM_STRIDE = 12;
enum CamField { C_Q = 0, C_P = 4, C_QN = 7 };

// Per-observation workspace written by the feature kernel (units of T):
//   Hx  4x6  measurement Jacobian block, observability-projected (msckf.py:480-490)
//   V   4x3  rows of the 3 Householder vectors of H_f's QR
//   W   3x6  this observation's 6 columns of w_j = v_j^T X_{j-1}
//   Qr  4    rows of Q^T r
//   R   4    the observation's residual r_i (before projection)
// obs_ws record per observation (T): Hx (4x6), V, W, Q^T r, r -- written only
// when a compact-factor consumer runs (large-track gating).
constexpr int OBS_HX = 0, OBS_V = 24, OBS_W = 36, OBS_QR = 54, OBS_R = 58, OBS_WS = 62;
// obs_ht record per observation (T), always written: the rank-3 reduced rows
// of the gating, Ht (3x6) and [r~ (3) | r_n] -- a dense 24-element stride, so
// that k_feature's stores and the gate's loads are contiguous.
constexpr int OBS_HT = 0, OBS_RT = 18, OBS_HTS = 24;

// Per-observation Gram terms written by the feature kernel (always fp64),
// consumed by the information assembly (k_info).  With G = the top 3 rows of
// Q^T Hx (Q = the feature's 3 Householder reflectors) and g = (Q^T r)[0:3]:
//   G   3x6  this observation's columns of G
//   DS  21   Hx_i^T Hx_i, lower triangle packed row-major
//   UB  6    Hx_i^T r_i - G_i^T g
// so that the projected block H0 = (Q^T Hx)[3:] satisfies
//   H0^T H0 = blockdiag_i(Hx_i^T Hx_i) - G^T G,   H0^T r0 = sum_i UB_i.
//   CAM  1   the observation's cam slot (exact in fp64)
// Stride 46 doubles (368 B: 16-byte chunks for global_load_lds; 92 dwords, so
// eight consecutive records start on eight different LDS bank quads -- a
// 48-double stride put them on two and made k_info's record reads 4-way
// bank-conflicted).
constexpr int OBG_G = 0, OBG_DS = 18, OBG_UB = 39, OBG_CAM = 45, OBG_STRIDE = 46;
// Per-feature QR record (fp64, always written by the feature kernel): with
// H_f = Q R the thin Householder QR of the feature's stacked 4M x 3 H_f,
//   X = R^-1 (upper; x00 x01 x02 x11 x12 x22),  g = (Q^T r)[0:3]
// so that the fused information assembly (k_info_fused) rebuilds an
// observation's G_i = (Q^T Hx)[0:3, cam i] = X^T H_f,i^T Hx_i from its own
// Jacobian blocks instead of reading obs_g.
constexpr int FQR_X = 0, FQR_G = 6, FQR_FLAG = 9, FQR_STRIDE = 10;
constexpr double FQR_RMAX = 1e3, FQR_KAPPA = 1e4;   // FQR_FLAG: Gram records written (k_feature)

template <typename T>
struct Params {
    T sigma2;                 // observation noise variance (msckf.py:560)
    T qc_gyro, qc_gbias, qc_acc, qc_abias;   // diag of Qc (msckf.py:132-137)
    T R01[9], t01[3];         // cam0 -> cam1 (msckf.py:148-152)
    T huber, precision, damping;              // feature.py LM
    int outer_max, inner_max;
};

template <typename T>
struct DevState {
    T* P;          // [B][Dmax][Dmax]
    T* imu;        // [B][IMU_STRIDE]
    T* cams;       // [B][Nmax][CAM_STRIDE]
    int* ncams;    // [B]
    int B, Nmax, Dmax;
};

// Feature batch resident in HBM (msckf_batch_load / msckf_update).
template <typename T>
struct FeatBatch {
    int nf;
    const int* feat_filter;   // [nf] filter slot of each feature
    const int* feat_off;      // [B+1] features of slot b: [feat_off[b], feat_off[b+1])
    const int* obs_off;       // [nf+1]
    const int* obs_cam;       // [sum M] cam slot
    const T* obs_z;           // [sum M][4]
    const T* chi2;            // [nf]
    const long long* ysq_off; // [nf+1] offsets of the (4M)^2 gating scratch
    T* p_w;                   // [nf][3]
    uint8_t* valid;           // [nf] triangulation validity (1 if p_w given)
    T* obs_ws;                // [sum M][OBS_WS] (compact-factor consumers only)
    T* obs_ht;                // [sum M][OBS_HTS] gating rows
    double* obs_g;            // [sum M][OBG_STRIDE] Gram terms (fp64), written only if gram
    double* fqr;              // [nf][FQR_STRIDE] R^-1 and (Q^T r)[0:3] of H_f's QR (fp64)
    int gram;                 // write obs_g (record-reading assembly, k_info / k_info_mfma)
    int compact;              // write V / W / Q^T r / tau (LDS gate fallback, QR path)
    T* tau;                   // [nf][4]
    T* ysq;                   // gating scratch
    T* gamma;                 // [nf]
    uint8_t* accept;          // [nf] chi2 test passed
    uint8_t* include;         // [nf] stacked into the update
    int* row_off;             // [nf] first stacked row of the feature
};

// Per-filter update workspace.  The information assembly and the Kalman stage
// always compute in fp64 (KT = double): after compression the rows of H_thin
// carry the information of ~1e4 measurements, so S = H P H^T + s2 I spans ~8
// decades (s2 ~ 1e-3 vs |H P H^T| ~ 1e5) -- beyond fp32 -- while the
// per-feature gating (condition ~1e3) stays in the context's scalar type T.
using KT = double;
template <typename T>
struct UpdWs {
    KT* Hthin;   // [B][Cmax][Cmax+1]   [A | b] = [H^T H | H^T r]; A full (k_info) or its lower triangle (k_info_fused, k_info_mfma)
    KT* dx;      // [B][Dmax + Cmax]
    int* info;   // [B][4]: rows stacked, C (0: no update), compress flag, status
    int Cmax;
    // Cholesky-form Kalman stage (msckf_kalman.hip); Cp = Cmax rounded up to 4
    KT* Lc;      // [B][Cp][Cp]          chol(P_cc), lower
    KT* Vi;      // [B][24][Cp]          P_ic Lc^-T (21 rows used)
    KT* Sii;     // [B][24][24]          P_ii - Vi Vi^T
    KT* G;       // [B][Cmax][Cmax+1]    A Lc
    KT* Tm;      // [B][Cmax][Cmax+1]    (s2 I + Lc^T A Lc | Lc^T b), lower
    KT* W;       // [B][Dmax+1][Cp]      rows [Vi ; Lc ; c^T] L_T^-T
    KT* Wk;      // [B][wk_stride]       global-memory factorisation workspace (large windows only)
    int* afail;  // [B]                  stage A status (1: P_cc not PD), written by every k_kal_a run
    size_t wk_stride;
    int Cp;
    double s2;   // observation noise variance in the context's type, as Params::sigma2: T >= s2 I
};

// ------------------------------------------------------------ device math --
template <typename T> __device__ __forceinline__ T dsqrt(T x) { return sqrt(x); }

template <typename T>
__device__ __forceinline__ void skew3(const T* v, T* S) {
    S[0] = 0;     S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2];  S[4] = 0;     S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0];  S[8] = 0;
}

// utils.py:14-27 -- R = (2w^2-1) I - 2w [v]x + 2 v v^T, q normalised first.
template <typename T>
__device__ __forceinline__ void quat_to_rot(const T* q_in, T* R) {
    T n = sqrt(q_in[0] * q_in[0] + q_in[1] * q_in[1] + q_in[2] * q_in[2] + q_in[3] * q_in[3]);
    T x = q_in[0] / n, y = q_in[1] / n, z = q_in[2] / n, w = q_in[3] / n;
    T v[3] = {x, y, z};
    T S[9];
    skew3(v, S);
    T a = 2 * w * w - 1, tw = 2 * w;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            R[3 * i + j] = (i == j ? a : T(0)) - tw * S[3 * i + j] + (2 * v[i]) * v[j];
}

// utils.py:29-53 (same branch structure -> same sign convention)
template <typename T>
__device__ __forceinline__ void rot_to_quat(const T* R, T* q) {
    T t;
    if (R[8] < 0) {
        if (R[0] > R[4]) {
            t = 1 + R[0] - R[4] - R[8];
            q[0] = t; q[1] = R[1] + R[3]; q[2] = R[6] + R[2]; q[3] = R[5] - R[7];
        } else {
            t = 1 - R[0] + R[4] - R[8];
            q[0] = R[1] + R[3]; q[1] = t; q[2] = R[7] + R[5]; q[3] = R[6] - R[2];
        }
    } else {
        if (R[0] < -R[4]) {
            t = 1 - R[0] - R[4] + R[8];
            q[0] = R[2] + R[6]; q[1] = R[7] + R[5]; q[2] = t; q[3] = R[1] - R[3];
        } else {
            t = 1 + R[0] + R[4] + R[8];
            q[0] = R[5] - R[7]; q[1] = R[6] - R[2]; q[2] = R[1] - R[3]; q[3] = t;
        }
    }
    T n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

// utils.py:67-82: q1 (x) q2 (both normalised first), result normalised.
template <typename T>
__device__ __forceinline__ void quat_mul(const T* a_in, const T* b_in, T* q) {
    T na = sqrt(a_in[0] * a_in[0] + a_in[1] * a_in[1] + a_in[2] * a_in[2] + a_in[3] * a_in[3]);
    T nb = sqrt(b_in[0] * b_in[0] + b_in[1] * b_in[1] + b_in[2] * b_in[2] + b_in[3] * b_in[3]);
    T a[4] = {a_in[0] / na, a_in[1] / na, a_in[2] / na, a_in[3] / na};
    T b[4] = {b_in[0] / nb, b_in[1] / nb, b_in[2] / nb, b_in[3] / nb};
    T r[4];
    r[0] = a[3] * b[0] + a[2] * b[1] - a[1] * b[2] + a[0] * b[3];
    r[1] = -a[2] * b[0] + a[3] * b[1] + a[0] * b[2] + a[1] * b[3];
    r[2] = a[1] * b[0] - a[0] * b[1] + a[3] * b[2] + a[2] * b[3];
    r[3] = -a[0] * b[0] - a[1] * b[1] - a[2] * b[2] + a[3] * b[3];
    T n = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]);
    q[0] = r[0] / n; q[1] = r[1] / n; q[2] = r[2] / n; q[3] = r[3] / n;
}

// utils.py:85-101
template <typename T>
__device__ __forceinline__ void small_angle_quat(const T* dth, T* q) {
    T d0 = dth[0] / 2, d1 = dth[1] / 2, d2 = dth[2] / 2;
    T n2 = d0 * d0 + d1 * d1 + d2 * d2;
    if (n2 <= 1) {
        q[0] = d0; q[1] = d1; q[2] = d2; q[3] = sqrt(1 - n2);
    } else {
        T s = sqrt(1 + n2);
        q[0] = d0 / s; q[1] = d1 / s; q[2] = d2 / s; q[3] = 1 / s;
    }
}

template <typename T>
__device__ __forceinline__ void mat3_vec(const T* A, const T* x, T* y) {
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}
template <typename T>
__device__ __forceinline__ void mat3T_vec(const T* A, const T* x, T* y) {
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = A[i] * x[0] + A[3 + i] * x[1] + A[6 + i] * x[2];
}
template <typename T>
__device__ __forceinline__ void mat3_mul(const T* A, const T* B, T* C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// Workgroup barrier that orders LDS only: outstanding global loads / stores stay
// in flight across it (a __syncthreads() emits s_waitcnt vmcnt(0) first, which
// would drain every prefetch).  Use only where no global data written by
// another thread is read after the barrier.
// XCD-aware block index (MI355X_MICROARCH.md, workgroup dispatch: blocks are
// dealt round-robin over the 8 XCDs, each with its own L2): a bijective remap
// that gives each XCD a contiguous range of logical blocks, so consecutive
// blocks (consecutive features of one filter, sharing its P) share an L2.
// Speed only -- any placement is correct.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}
// Block coordinates of a 2-D / 3-D grid with the linear block id remapped so
// that consecutive ids -- one filter's tiles or chunks (x fastest, then y) --
// run on one XCD and share its L2 (the dispatcher deals linear ids round-robin
// over the 8 XCDs, so a filter's tiles would otherwise re-read its operands from
// HBM on every XCD).
struct Blk3 { int x, y, z; };
__device__ __forceinline__ Blk3 xcd_blk3() {
    const int nx = gridDim.x, ny = gridDim.y, n = nx * ny * gridDim.z;
    const int r = xcd_remap(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), n);
    return {r % nx, (r / nx) % ny, r / (nx * ny)};
}

#define LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Broadcast lane `src` (wave-uniform) of x to the whole wave via v_readlane
// (result lands in an SGPR: no LDS traffic).
__device__ __forceinline__ float lane_bcast(float x, int src) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), src));
}
__device__ __forceinline__ double lane_bcast(double x, int src) {
    long long u = __builtin_bit_cast(long long, x);
    int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffLL), src);
    int hi = __builtin_amdgcn_readlane((int)(u >> 32), src);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// Reciprocal / square root used by the Householder reflectors.  Deliberately
// IEEE (denormal-safe): the hardware v_rcp_f32 / v_sqrt_f32 flush denormal
// inputs, and columns in the near-null (gauge) directions of H carry tiny
// entries with alpha ~ 0 -- the approximations turn those into inf / NaN.
__device__ __forceinline__ float fast_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ double fast_sqrt(double x) { return sqrt(x); }
__device__ __forceinline__ float fast_rcp(float x) { return 1.0f / x; }
__device__ __forceinline__ double fast_rcp(double x) { return 1.0 / x; }
// Pivot reciprocals of the gating LDL^T: v_rcp_f32 (1 ulp) in fp32, IEEE division in fp64.
__device__ __forceinline__ float pivot_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double pivot_rcp(double x) { return 1.0 / x; }

// Column-major enumeration of the lower tiles (ti >= tl) of a grid with nrow
// tile rows: column c holds nrow - c tiles and starts at c nrow - c (c - 1) / 2.
// Returns tl for tile index t (closed form + one-step fix-up).
__device__ __forceinline__ int colmajor_col(int t, int nrow) {
    const float q = 2.0f * nrow + 1.0f;
    int c = (int)((q - sqrtf(fmaxf(q * q - 8.0f * t, 0.0f))) * 0.5f);
    if (c < 0) c = 0;
    while (c > 0 && c * nrow - c * (c - 1) / 2 > t) --c;
    while ((c + 1) * nrow - (c + 1) * c / 2 <= t) ++c;
    return c;
}

// ------------------------------------------------------ wave reductions --
// Per-type MFMA pieces (the gating kernels, the propagation cross block) (fp32 contexts: v_mfma_f32_16x16x4_f32;
// fp64 contexts: v_mfma_f64_16x16x4_f64).  The A / B operand layouts agree (A:
// row l & 15, k = l >> 4; B: k = l >> 4, column l & 15), the result layouts do
// not: lane l holds column l & 15 and rows RG (l >> 4) + RS i, i = 0..3 -- f32:
// 4 (l >> 4) + i, f64: (l >> 4) + 4 i (tools/probes/mfma_f64_layout.hip).
template <typename T> struct GM;
template <> struct GM<float> {
    using V4 = float __attribute__((ext_vector_type(4)));
    using V2 = float __attribute__((ext_vector_type(2)));
    static constexpr int RS = 1, RG = 4;
    __device__ static V4 mfma(float a, float b, V4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
};
template <> struct GM<double> {
    using V4 = double __attribute__((ext_vector_type(4)));
    using V2 = double __attribute__((ext_vector_type(2)));
    static constexpr int RS = 4, RG = 1;
    __device__ static V4 mfma(double a, double b, V4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
};
template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}
template <typename T>
__device__ __forceinline__ T wave_max(T x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x = fmax(x, __shfl_xor(x, m, 64));
    return x;
}

}  // namespace msckf
