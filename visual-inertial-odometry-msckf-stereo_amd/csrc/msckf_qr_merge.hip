// msckf_qr_merge.hip -- QR row-merge compression (round-1 path, kept for A/B).
#include <type_traits>

#include "msckf_common.h"
#include "msckf_launch.h"

namespace msckf {

// ===========================================================================
// Stacked-H assembly / QR compression (msckf.py:549-556): one workgroup per
// filter.  When R > C the included features' rows are merged, chunk by chunk,
// into the running triangular factor [R | Q^T r] with one Householder
// reflector per column (a sequential TSQR; any orthogonal row transform of
// (H, r) leaves the update unchanged -- quirk Q4); when R <= C the stacked rows
// are copied out as H_thin, as the reference does.
// Register-resident merge (the production path of the QR compression).
// Thread t owns columns j = t + 256u (u < COLS) of [R | Q^T r]; the CH rows of
// the current chunk of the feature's projected block live in its registers
// (b[u][0..CH)), generated directly from the compact factors (Hx, V, tau, W)
// without an LDS tile.  Per column c one barrier: every owner of a column
// j > c applies the reflector (v broadcast from LDS), and the owner of column
// c+1 forms the next reflector from its registers (look-ahead).  R lives in
// LDS when it fits, else in global memory with R[c+1][j] prefetched one step
// ahead (row c+1 is not touched by step c).
template <typename T, int CH, int COLS, bool R_LDS>
__global__ void __launch_bounds__(256) k_compress_reg(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int* info = ws.info + 4 * b;
    const int Rn = info[0], n = info[1], compress = info[2];
    if (Rn == 0) return;
    const int C = 6 * st.ncams[b];
    const int ldh = ws.Cmax + 1;
    T* H = ws.Hqr + (size_t)b * ws.Cmax * ldh;
    const int ldr = R_LDS ? (C + 1) : ldh;
    T* s_v = reinterpret_cast<T*>(smem_raw);                  // [2][CH]
    T* s_sc = s_v + 2 * CH;                                   // tau[2] | tau_f[3]
    T* s_V = s_sc + 8;                                        // [CH][4] chunk rows of V, [..][3] = Qr
    int* s_obs = reinterpret_cast<int*>(s_V + 4 * CH);        // [Nmax] obs index of each cam slot
    T* Rm = R_LDS ? reinterpret_cast<T*>(s_obs + ((st.Nmax + 3) & ~3)) : H;   // [C][ldr]
    auto Ridx = [&](int r, int c) -> T& { return Rm[(size_t)r * ldr + (R_LDS ? c : (c == C ? ws.Cmax : c))]; };
    if (compress)
        for (int e = tid; e < C * (C + 1); e += blockDim.x) Ridx(e / (C + 1), e % (C + 1)) = 0;
    else
        for (int e = tid; e < n * ldh; e += blockDim.x) H[e] = 0;
    for (int f = fb.feat_off[b]; f < fb.feat_off[b + 1]; ++f) {
        if (!fb.include[f]) continue;
        const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
        const T* wsf = fb.obs_ws + (size_t)o0 * OBS_WS;
        __syncthreads();
        for (int i = tid; i < st.Nmax; i += blockDim.x) s_obs[i] = -1;
        if (tid < 3) s_sc[2 + tid] = fb.tau[4 * f + tid];
        __syncthreads();
        int smin = 1 << 30;
        for (int i = 0; i < M; ++i) smin = min(smin, fb.obs_cam[o0 + i]);
        for (int i = tid; i < M; i += blockDim.x) s_obs[fb.obs_cam[o0 + i]] = i;
        __syncthreads();
        const T t0 = s_sc[2], t1 = s_sc[3], t2 = s_sc[4];
        // per owned column: its observation (if any), its W entries, its Hx rows
        int oi[COLS];
        T w0[COLS], w1[COLS], w2[COLS], hx[COLS][4];
#pragma unroll
        for (int u = 0; u < COLS; ++u) {
            const int j = tid + 256 * u;
            oi[u] = (j < C) ? s_obs[j / 6] : -1;
            w0[u] = w1[u] = w2[u] = 0;
            hx[u][0] = hx[u][1] = hx[u][2] = hx[u][3] = 0;
            if (oi[u] >= 0) {
                const T* wo = wsf + (size_t)oi[u] * OBS_WS;
                const int c = j % 6;
                w0[u] = t0 * wo[OBS_W + c];
                w1[u] = t1 * wo[OBS_W + 6 + c];
                w2[u] = t2 * wo[OBS_W + 12 + c];
#pragma unroll
                for (int a = 0; a < 4; ++a) hx[u][a] = wo[OBS_HX + 6 * a + c];
            }
        }
        const int c0 = 6 * smin;
        const int n4 = 4 * M;
        for (int a0 = 3; a0 < n4; a0 += CH) {
            const int nr = min(CH, n4 - a0);
            __syncthreads();
            for (int rr = tid; rr < CH; rr += blockDim.x) {
                const int row = a0 + rr;
                if (rr < nr) {
                    const T* wr = wsf + (size_t)(row >> 2) * OBS_WS;
                    s_V[4 * rr + 0] = wr[OBS_V + 3 * (row & 3) + 0];
                    s_V[4 * rr + 1] = wr[OBS_V + 3 * (row & 3) + 1];
                    s_V[4 * rr + 2] = wr[OBS_V + 3 * (row & 3) + 2];
                    s_V[4 * rr + 3] = wr[OBS_QR + (row & 3)];
                } else {
                    s_V[4 * rr + 0] = s_V[4 * rr + 1] = s_V[4 * rr + 2] = s_V[4 * rr + 3] = 0;
                }
            }
            __syncthreads();
            T bv[COLS][CH];
#pragma unroll
            for (int u = 0; u < COLS; ++u) {
                const int j = tid + 256 * u;
#pragma unroll
                for (int rr = 0; rr < CH; ++rr) {
                    const int row = a0 + rr;
                    T x = 0;
                    if (j == C) {
                        x = s_V[4 * rr + 3];
                    } else if (oi[u] >= 0) {
                        const T h = ((row >> 2) == oi[u]) ? hx[u][row & 3] : T(0);
                        x = h - (s_V[4 * rr] * w0[u] + s_V[4 * rr + 1] * w1[u] + s_V[4 * rr + 2] * w2[u]);
                        if (rr >= nr) x = 0;
                    }
                    bv[u][rr] = x;
                }
            }
            if (!compress) {   // R <= C: the stacked rows are H_thin (msckf.py:554-556)
                const int base = fb.row_off[f] + (a0 - 3);
#pragma unroll
                for (int u = 0; u < COLS; ++u) {
                    const int j = tid + 256 * u;
                    if (j > C) continue;
                    const int col = (j == C) ? ws.Cmax : j;
#pragma unroll
                    for (int rr = 0; rr < CH; ++rr)
                        if (rr < nr) H[(size_t)(base + rr) * ldh + col] = bv[u][rr];
                }
                continue;
            }
            // R[j][j] of every owned column: only column j's own reflector touches
            // it, so it is read once per chunk (no global latency per column)
            T rdiag[COLS];
#pragma unroll
            for (int u = 0; u < COLS; ++u) {
                const int j = tid + 256 * u;
                rdiag[u] = (j >= c0 && j < C) ? Ridx(j, j) : T(0);
            }
            // reflector of column c from (R[c][c], bv[u]) by the owner of column c
            auto reflector = [&](int c, int u, int buf) {
                T p0 = 0, p1 = 0, p2 = 0, p3 = 0;
#pragma unroll
                for (int rr = 0; rr < CH; rr += 4) {
                    p0 += bv[u][rr] * bv[u][rr];
                    p1 += bv[u][rr + 1] * bv[u][rr + 1];
                    p2 += bv[u][rr + 2] * bv[u][rr + 2];
                    p3 += bv[u][rr + 3] * bv[u][rr + 3];
                }
                const T xs = (p0 + p1) + (p2 + p3);
                const T alpha = rdiag[u];
                T tj = 0, scale = 0, beta = alpha;
                if (xs != T(0)) {
                    T nrm = sqrt(alpha * alpha + xs);
                    beta = alpha >= 0 ? -nrm : nrm;
                    tj = (beta - alpha) / beta;
                    scale = T(1) / (alpha - beta);
                }
#pragma unroll
                for (int rr = 0; rr < CH; ++rr) s_v[buf * CH + rr] = bv[u][rr] * scale;
                s_sc[buf] = tj;
                rdiag[u] = beta;
                Ridx(c, c) = beta;
            };
#pragma unroll
            for (int u = 0; u < COLS; ++u)
                if (tid + 256 * u == c0) reflector(c0, u, 0);
            T rnext[COLS];
#pragma unroll
            for (int u = 0; u < COLS; ++u) {
                const int j = tid + 256 * u;
                rnext[u] = (j <= C && j > c0) ? Ridx(c0, j) : T(0);
            }
            LDS_BARRIER();
            for (int c = c0; c < C; ++c) {
                const int buf = (c - c0) & 1;
                const T tj = s_sc[buf];
                T v[CH];
#pragma unroll
                for (int rr = 0; rr < CH; ++rr) v[rr] = s_v[buf * CH + rr];
#pragma unroll
                for (int u = 0; u < COLS; ++u) {
                    const int j = tid + 256 * u;
                    const T rcur = rnext[u];
                    if (j > c + 1 && j <= C) rnext[u] = Ridx(c + 1, j);   // prefetch next row
                    if (j > c && j <= C && tj != T(0)) {
                        T q0 = rcur, q1 = 0, q2 = 0, q3 = 0;
#pragma unroll
                        for (int rr = 0; rr < CH; rr += 4) {
                            q0 += v[rr] * bv[u][rr];
                            q1 += v[rr + 1] * bv[u][rr + 1];
                            q2 += v[rr + 2] * bv[u][rr + 2];
                            q3 += v[rr + 3] * bv[u][rr + 3];
                        }
                        const T w = (q0 + q1) + (q2 + q3);
                        const T tw = tj * w;
                        Ridx(c, j) = rcur - tw;
#pragma unroll
                        for (int rr = 0; rr < CH; ++rr) bv[u][rr] -= v[rr] * tw;
                    }
                    if (j == c + 1 && j < C) reflector(j, u, buf ^ 1);
                }
                LDS_BARRIER();   // R prefetches / stores stay in flight
            }
        }
    }
    if (R_LDS && compress) {
        __syncthreads();
        for (int e = tid; e < C * (C + 1); e += blockDim.x) {
            const int r = e / (C + 1), c = e % (C + 1);
            H[(size_t)r * ldh + (c == C ? ws.Cmax : c)] = Rm[e];
        }
    }
}

// Panel-blocked register merge (production path when C+1 <= 256).
// Columns are processed in 16-wide panels aligned to 16.  The wave that owns a
// panel factors it alone (reflector of column q formed by lane q from its
// registers, broadcast to the wave through LDS with a wave-local wait only);
// its lanes apply each reflector to their own columns on the spot.  One
// workgroup barrier per panel publishes the panel's 16 reflectors; every other
// wave then applies them to its columns from registers.  The 16 R rows of a
// panel are prefetched one whole panel ahead (rows of panel P+1 are not
// touched by panel P), so no global latency sits on the per-column path.
template <typename T, int CH>
__global__ void __launch_bounds__(256) k_compress_panel(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws) {
    constexpr int NB = 16;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6;
    const int* info = ws.info + 4 * b;
    const int Rn = info[0], n = info[1], compress = info[2];
    if (Rn == 0) return;
    const int C = 6 * st.ncams[b];
    const int ldh = ws.Cmax + 1;
    T* H = ws.Hqr + (size_t)b * ws.Cmax * ldh;
    T* s_Vp = reinterpret_cast<T*>(smem_raw);       // [2][NB][CH] panel reflectors
    T* s_tp = s_Vp + 2 * NB * CH;                   // [2][NB]
    T* s_sc = s_tp + 2 * NB;                        // tau_f[3] (+pad)
    T* s_V = s_sc + 4;                              // [CH][4] chunk rows of V | Qr
    int* s_obs = reinterpret_cast<int*>(s_V + 4 * CH);
    const int j = tid;                              // the one column this thread owns
    const bool mine = j <= C;
    const int hcol = (j == C) ? ws.Cmax : j;
    if (compress)
        for (int e = tid; e < C * (C + 1); e += blockDim.x) {
            const int r = e / (C + 1), c = e % (C + 1);
            H[(size_t)r * ldh + (c == C ? ws.Cmax : c)] = 0;
        }
    else
        for (int e = tid; e < n * ldh; e += blockDim.x) H[e] = 0;
    for (int f = fb.feat_off[b]; f < fb.feat_off[b + 1]; ++f) {
        if (!fb.include[f]) continue;
        const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
        const T* wsf = fb.obs_ws + (size_t)o0 * OBS_WS;
        __syncthreads();
        for (int i = tid; i < st.Nmax; i += blockDim.x) s_obs[i] = -1;
        if (tid < 3) s_sc[tid] = fb.tau[4 * f + tid];
        __syncthreads();
        int smin = 1 << 30;
        for (int i = 0; i < M; ++i) smin = min(smin, fb.obs_cam[o0 + i]);
        for (int i = tid; i < M; i += blockDim.x) s_obs[fb.obs_cam[o0 + i]] = i;
        __syncthreads();
        const T t0 = s_sc[0], t1 = s_sc[1], t2 = s_sc[2];
        const int oi = (j < C) ? s_obs[j / 6] : -1;
        T w0 = 0, w1 = 0, w2 = 0, hx[4] = {0, 0, 0, 0};
        if (oi >= 0) {
            const T* wo = wsf + (size_t)oi * OBS_WS;
            const int c = j % 6;
            w0 = t0 * wo[OBS_W + c];
            w1 = t1 * wo[OBS_W + 6 + c];
            w2 = t2 * wo[OBS_W + 12 + c];
#pragma unroll
            for (int a = 0; a < 4; ++a) hx[a] = wo[OBS_HX + 6 * a + c];
        }
        const int c0 = 6 * smin;
        const int n4 = 4 * M;
        for (int a0 = 3; a0 < n4; a0 += CH) {
            const int nr = min(CH, n4 - a0);
            __syncthreads();
            for (int rr = tid; rr < CH; rr += blockDim.x) {
                const int row = a0 + rr;
                if (rr < nr) {
                    const T* wr = wsf + (size_t)(row >> 2) * OBS_WS;
                    s_V[4 * rr + 0] = wr[OBS_V + 3 * (row & 3) + 0];
                    s_V[4 * rr + 1] = wr[OBS_V + 3 * (row & 3) + 1];
                    s_V[4 * rr + 2] = wr[OBS_V + 3 * (row & 3) + 2];
                    s_V[4 * rr + 3] = wr[OBS_QR + (row & 3)];
                } else {
                    s_V[4 * rr + 0] = s_V[4 * rr + 1] = s_V[4 * rr + 2] = s_V[4 * rr + 3] = 0;
                }
            }
            __syncthreads();
            T bv[CH];
#pragma unroll
            for (int rr = 0; rr < CH; ++rr) {
                const int row = a0 + rr;
                T x = 0;
                if (j == C) {
                    x = s_V[4 * rr + 3];
                } else if (oi >= 0) {
                    const T h = ((row >> 2) == oi) ? hx[row & 3] : T(0);
                    x = h - (s_V[4 * rr] * w0 + s_V[4 * rr + 1] * w1 + s_V[4 * rr + 2] * w2);
                    if (rr >= nr) x = 0;
                }
                bv[rr] = x;
            }
            if (!compress) {   // R <= C: the stacked rows are H_thin (msckf.py:554-556)
                const int base = fb.row_off[f] + (a0 - 3);
                if (mine)
#pragma unroll
                    for (int rr = 0; rr < CH; ++rr)
                        if (rr < nr) H[(size_t)(base + rr) * ldh + hcol] = bv[rr];
                continue;
            }
            const int P0 = c0 / NB, PL = (C - 1) / NB;
            T rr_[NB], rn[NB];
            {
                const int pb = c0, pe = min(NB * (P0 + 1), C);
#pragma unroll
                for (int t = 0; t < NB; ++t)
                    rn[t] = (mine && pb + t < pe && j >= pb + t) ? H[(size_t)(pb + t) * ldh + hcol] : T(0);
            }
            for (int P = P0; P <= PL; ++P) {
                const int pb = max(NB * P, c0), pe = min(NB * (P + 1), C), nbp = pe - pb;
                const int buf = (P - P0) & 1;
                T* Vb = s_Vp + buf * NB * CH;
                T* tb = s_tp + buf * NB;
#pragma unroll
                for (int t = 0; t < NB; ++t) rr_[t] = rn[t];
                if (P < PL) {   // prefetch the next panel's R rows (untouched by this panel)
                    const int qb = NB * (P + 1), qe = min(NB * (P + 2), C);
#pragma unroll
                    for (int t = 0; t < NB; ++t)
                        rn[t] = (mine && qb + t < qe && j >= qb + t) ? H[(size_t)(qb + t) * ldh + hcol] : T(0);
                }
                const int owner = (NB * P) >> 6;
                if (wave == owner) {
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if (t < nbp) {
                            const int q = pb + t;
                            if (j == q) {   // reflector of column q (LAPACK dlarfg convention)
                                T p0 = 0, p1 = 0, p2 = 0, p3 = 0;
#pragma unroll
                                for (int r = 0; r < CH; r += 4) {
                                    p0 += bv[r] * bv[r];
                                    p1 += bv[r + 1] * bv[r + 1];
                                    p2 += bv[r + 2] * bv[r + 2];
                                    p3 += bv[r + 3] * bv[r + 3];
                                }
                                const T xs = (p0 + p1) + (p2 + p3);
                                const T alpha = rr_[t];
                                T tj = 0, scale = 0, beta = alpha;
                                if (xs != T(0)) {
                                    T nrm = sqrt(alpha * alpha + xs);
                                    beta = alpha >= 0 ? -nrm : nrm;
                                    tj = (beta - alpha) / beta;
                                    scale = T(1) / (alpha - beta);
                                }
#pragma unroll
                                for (int r = 0; r < CH; ++r) Vb[t * CH + r] = bv[r] * scale;
                                tb[t] = tj;
                                rr_[t] = beta;
                            }
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave-local publish
                            const T tj = tb[t];
                            if (j > q && mine && tj != T(0)) {
                                T q0 = rr_[t], q1 = 0, q2 = 0, q3 = 0;
#pragma unroll
                                for (int r = 0; r < CH; r += 4) {
                                    q0 += Vb[t * CH + r] * bv[r];
                                    q1 += Vb[t * CH + r + 1] * bv[r + 1];
                                    q2 += Vb[t * CH + r + 2] * bv[r + 2];
                                    q3 += Vb[t * CH + r + 3] * bv[r + 3];
                                }
                                const T tw = tj * ((q0 + q1) + (q2 + q3));
                                rr_[t] -= tw;
#pragma unroll
                                for (int r = 0; r < CH; ++r) bv[r] -= Vb[t * CH + r] * tw;
                            }
                        }
                    }
                }
                LDS_BARRIER();   // publishes the panel; R prefetches stay in flight
                if (wave != owner && mine && j >= pe) {
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if (t < nbp) {
                            const T tj = tb[t];
                            if (tj != T(0)) {
                                T q0 = rr_[t], q1 = 0, q2 = 0, q3 = 0;
#pragma unroll
                                for (int r = 0; r < CH; r += 4) {
                                    q0 += Vb[t * CH + r] * bv[r];
                                    q1 += Vb[t * CH + r + 1] * bv[r + 1];
                                    q2 += Vb[t * CH + r + 2] * bv[r + 2];
                                    q3 += Vb[t * CH + r + 3] * bv[r + 3];
                                }
                                const T tw = tj * ((q0 + q1) + (q2 + q3));
                                rr_[t] -= tw;
#pragma unroll
                                for (int r = 0; r < CH; ++r) bv[r] -= Vb[t * CH + r] * tw;
                            }
                        }
                    }
                }
#pragma unroll
                for (int t = 0; t < NB; ++t)
                    if (mine && t < nbp && j >= pb + t) H[(size_t)(pb + t) * ldh + hcol] = rr_[t];
            }
        }
    }
}

// One wavefront per filter (the throughput path): no workgroup barriers at
// all.  Lane l owns columns j = l + 64u (u < COLS) of [R | Q^T r] and the CH
// chunk rows of those columns in registers.  Column c's reflector vector is
// read out of the owner lane with v_readlane (SGPR broadcast); every lane
// forms the same scalars (tau, scale) redundantly and updates its own
// columns.  Latency is hidden by running several filters per SIMD.
template <typename T, int CH, int COLS>
__global__ void __launch_bounds__(64) k_compress_wave(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int* info = ws.info + 4 * b;
    const int Rn = info[0], n = info[1], compress = info[2];
    if (Rn == 0) return;
    const int C = 6 * st.ncams[b];
    const int ldh = ws.Cmax + 1;
    T* H = ws.Hqr + (size_t)b * ws.Cmax * ldh;
    T* s_V = reinterpret_cast<T*>(smem_raw);        // [CH][4] chunk rows of V | Qr
    T* s_sc = s_V + 4 * CH;                         // tau_f[3] (+pad)
    int* s_obs = reinterpret_cast<int*>(s_sc + 4);  // [Nmax]
    int hcol[COLS];
#pragma unroll
    for (int u = 0; u < COLS; ++u) {
        const int j = lane + 64 * u;
        hcol[u] = (j == C) ? ws.Cmax : j;
    }
    if (compress) {
        for (int r = 0; r < C; ++r)
#pragma unroll
            for (int u = 0; u < COLS; ++u)
                if (lane + 64 * u <= C) H[(size_t)r * ldh + hcol[u]] = 0;
    } else {
        for (int e = lane; e < n * ldh; e += 64) H[e] = 0;
    }
    for (int f = fb.feat_off[b]; f < fb.feat_off[b + 1]; ++f) {
        if (!fb.include[f]) continue;
        const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
        const T* wsf = fb.obs_ws + (size_t)o0 * OBS_WS;
        for (int i = lane; i < st.Nmax; i += 64) s_obs[i] = -1;
        if (lane < 3) s_sc[lane] = fb.tau[4 * f + lane];
        int smin = 1 << 30;
        for (int i = 0; i < M; ++i) smin = min(smin, fb.obs_cam[o0 + i]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int i = lane; i < M; i += 64) s_obs[fb.obs_cam[o0 + i]] = i;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const T t0 = s_sc[0], t1 = s_sc[1], t2 = s_sc[2];
        int oi[COLS];
        T w0[COLS], w1[COLS], w2[COLS], hx[COLS][4];
#pragma unroll
        for (int u = 0; u < COLS; ++u) {
            const int j = lane + 64 * u;
            oi[u] = (j < C) ? s_obs[j / 6] : -1;
            w0[u] = w1[u] = w2[u] = 0;
            hx[u][0] = hx[u][1] = hx[u][2] = hx[u][3] = 0;
            if (oi[u] >= 0) {
                const T* wo = wsf + (size_t)oi[u] * OBS_WS;
                const int c = j % 6;
                w0[u] = t0 * wo[OBS_W + c];
                w1[u] = t1 * wo[OBS_W + 6 + c];
                w2[u] = t2 * wo[OBS_W + 12 + c];
#pragma unroll
                for (int a = 0; a < 4; ++a) hx[u][a] = wo[OBS_HX + 6 * a + c];
            }
        }
        const int c0 = 6 * smin;
        const int n4 = 4 * M;
        for (int a0 = 3; a0 < n4; a0 += CH) {
            const int nr = min(CH, n4 - a0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int rr = lane; rr < CH; rr += 64) {
                const int row = a0 + rr;
                if (rr < nr) {
                    const T* wr = wsf + (size_t)(row >> 2) * OBS_WS;
                    s_V[4 * rr + 0] = wr[OBS_V + 3 * (row & 3) + 0];
                    s_V[4 * rr + 1] = wr[OBS_V + 3 * (row & 3) + 1];
                    s_V[4 * rr + 2] = wr[OBS_V + 3 * (row & 3) + 2];
                    s_V[4 * rr + 3] = wr[OBS_QR + (row & 3)];
                } else {
                    s_V[4 * rr + 0] = s_V[4 * rr + 1] = s_V[4 * rr + 2] = s_V[4 * rr + 3] = 0;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            T bv[COLS][CH];
#pragma unroll
            for (int u = 0; u < COLS; ++u) {
                const int j = lane + 64 * u;
#pragma unroll
                for (int rr = 0; rr < CH; ++rr) {
                    const int row = a0 + rr;
                    T x = 0;
                    if (j == C) {
                        x = s_V[4 * rr + 3];
                    } else if (oi[u] >= 0) {
                        const T h = ((row >> 2) == oi[u]) ? hx[u][row & 3] : T(0);
                        x = h - (s_V[4 * rr] * w0[u] + s_V[4 * rr + 1] * w1[u] + s_V[4 * rr + 2] * w2[u]);
                        if (rr >= nr) x = 0;
                    }
                    bv[u][rr] = x;
                }
            }
            if (!compress) {   // R <= C: the stacked rows are H_thin (msckf.py:554-556)
                const int base = fb.row_off[f] + (a0 - 3);
#pragma unroll
                for (int u = 0; u < COLS; ++u)
                    if (lane + 64 * u <= C)
#pragma unroll
                        for (int rr = 0; rr < CH; ++rr)
                            if (rr < nr) H[(size_t)(base + rr) * ldh + hcol[u]] = bv[u][rr];
                continue;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // same-address RAW on R rows
            T rcur[COLS];
#pragma unroll
            for (int u = 0; u < COLS; ++u) {
                const int j = lane + 64 * u;
                rcur[u] = (j >= c0 && j <= C) ? H[(size_t)c0 * ldh + hcol[u]] : T(0);
            }
            // the sweep is split by the owner's column slot UC (compile time) so
            // the broadcast reflector stays in SGPRs
#pragma unroll
            for (int UC = 0; UC < COLS; ++UC) {
                const int cb = max(c0, 64 * UC), ce = min(C, 64 * (UC + 1));
                for (int c = cb; c < ce; ++c) {
                    const int lc = c & 63;
                    T rnext[COLS];
#pragma unroll
                    for (int u = 0; u < COLS; ++u) {   // prefetch row c+1 (untouched by column c)
                        const int j = lane + 64 * u;
                        rnext[u] = (j > c && j <= C && c + 1 < C) ? H[(size_t)(c + 1) * ldh + hcol[u]] : T(0);
                    }
                    T v[CH];
#pragma unroll
                    for (int rr = 0; rr < CH; ++rr) v[rr] = lane_bcast(bv[UC][rr], lc);
                    const T alpha = lane_bcast(rcur[UC], lc);
                    T p0 = 0, p1 = 0, p2 = 0, p3 = 0;
#pragma unroll
                    for (int rr = 0; rr < CH; rr += 4) {
                        p0 += v[rr] * v[rr];
                        p1 += v[rr + 1] * v[rr + 1];
                        p2 += v[rr + 2] * v[rr + 2];
                        p3 += v[rr + 3] * v[rr + 3];
                    }
                    const T xs = (p0 + p1) + (p2 + p3);
                    T tj = 0, scale = 0, beta = alpha;
                    if (xs != T(0)) {
                        const T nrm = sqrt(alpha * alpha + xs);
                        beta = alpha >= 0 ? -nrm : nrm;
                        tj = (beta - alpha) / beta;
                        scale = T(1) / (alpha - beta);
                    }
                    const T ts = tj * scale;   // w = R + scale <v_raw, b> ; b -= v_raw (scale tau w)
#pragma unroll
                    for (int u = UC; u < COLS; ++u) {
                        const int j = lane + 64 * u;
                        if (j == c) {
                            H[(size_t)c * ldh + hcol[u]] = beta;
                        } else if (j > c && j <= C && tj != T(0)) {
                            T q0 = 0, q1 = 0, q2 = 0, q3 = 0;
#pragma unroll
                            for (int rr = 0; rr < CH; rr += 4) {
                                q0 += v[rr] * bv[u][rr];
                                q1 += v[rr + 1] * bv[u][rr + 1];
                                q2 += v[rr + 2] * bv[u][rr + 2];
                                q3 += v[rr + 3] * bv[u][rr + 3];
                            }
                            const T w = rcur[u] + scale * ((q0 + q1) + (q2 + q3));
                            H[(size_t)c * ldh + hcol[u]] = rcur[u] - tj * w;
                            const T f2 = ts * w;
#pragma unroll
                            for (int rr = 0; rr < CH; ++rr) bv[u][rr] -= v[rr] * f2;
                        }
                        rcur[u] = rnext[u];
                    }
                }
            }
        }
    }
}

// Lean one-wavefront-per-filter merge (default throughput path, C+1 <= 192).
// Same algorithm as k_compress_wave with less live state: the generation
// temporaries die before the sweep, the column loop is unrolled by two with a
// two-rows-ahead R prefetch ring, and fp32 uses v_sqrt / v_rcp.
template <typename T, int CH>
__global__ void __launch_bounds__(64) k_compress_w(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws) {
    constexpr int COLS = 3;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int* info = ws.info + 4 * b;
    const int Rn = info[0], n = info[1], compress = info[2];
    if (Rn == 0) return;
    const int C = 6 * st.ncams[b];
    const int ldh = ws.Cmax + 1;
    T* H = ws.Hqr + (size_t)b * ws.Cmax * ldh;
    T* s_V = reinterpret_cast<T*>(smem_raw);        // [CH][4] chunk rows of V | Qr
    T* s_sc = s_V + 4 * CH;                         // tau_f[3] (+pad)
    int* s_obs = reinterpret_cast<int*>(s_sc + 4);  // [Nmax]
    int hcol[COLS];
#pragma unroll
    for (int u = 0; u < COLS; ++u) {
        const int j = lane + 64 * u;
        hcol[u] = (j == C) ? ws.Cmax : j;
    }
    if (compress) {
        for (int r = 0; r < C; ++r)
#pragma unroll
            for (int u = 0; u < COLS; ++u)
                if (lane + 64 * u <= C) H[(size_t)r * ldh + hcol[u]] = 0;
    } else {
        for (int e = lane; e < n * ldh; e += 64) H[e] = 0;
    }
    for (int f = fb.feat_off[b]; f < fb.feat_off[b + 1]; ++f) {
        if (!fb.include[f]) continue;
        const int o0 = fb.obs_off[f], M = fb.obs_off[f + 1] - o0;
        const T* wsf = fb.obs_ws + (size_t)o0 * OBS_WS;
        for (int i = lane; i < st.Nmax; i += 64) s_obs[i] = -1;
        if (lane < 3) s_sc[lane] = fb.tau[4 * f + lane];
        int smin = 1 << 30;
        for (int i = 0; i < M; ++i) smin = min(smin, fb.obs_cam[o0 + i]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int i = lane; i < M; i += 64) s_obs[fb.obs_cam[o0 + i]] = i;
        const int c0 = 6 * smin;
        const int n4 = 4 * M;
        for (int a0 = 3; a0 < n4; a0 += CH) {
            const int nr = min(CH, n4 - a0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            for (int rr = lane; rr < CH; rr += 64) {
                const int row = a0 + rr;
                if (rr < nr) {
                    const T* wr = wsf + (size_t)(row >> 2) * OBS_WS;
                    s_V[4 * rr + 0] = wr[OBS_V + 3 * (row & 3) + 0];
                    s_V[4 * rr + 1] = wr[OBS_V + 3 * (row & 3) + 1];
                    s_V[4 * rr + 2] = wr[OBS_V + 3 * (row & 3) + 2];
                    s_V[4 * rr + 3] = wr[OBS_QR + (row & 3)];
                } else {
                    s_V[4 * rr + 0] = s_V[4 * rr + 1] = s_V[4 * rr + 2] = s_V[4 * rr + 3] = 0;
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // chunk rows as 2-wide vectors: rows (2i, 2i+1) pair up for v_pk_fma_f32
            using V2 = T __attribute__((ext_vector_type(2)));
            constexpr int CH2 = CH / 2;
            V2 bv[COLS][CH2];
#pragma unroll
            for (int u = 0; u < COLS; ++u) {
                const int j = lane + 64 * u;
                const int oi = (j < C) ? s_obs[j / 6] : -1;
                T w0 = 0, w1 = 0, w2 = 0, hx0 = 0, hx1 = 0, hx2 = 0, hx3 = 0;
                if (oi >= 0) {
                    const T* wo = wsf + (size_t)oi * OBS_WS;
                    const int c = j % 6;
                    w0 = s_sc[0] * wo[OBS_W + c];
                    w1 = s_sc[1] * wo[OBS_W + 6 + c];
                    w2 = s_sc[2] * wo[OBS_W + 12 + c];
                    hx0 = wo[OBS_HX + c];
                    hx1 = wo[OBS_HX + 6 + c];
                    hx2 = wo[OBS_HX + 12 + c];
                    hx3 = wo[OBS_HX + 18 + c];
                }
#pragma unroll
                for (int rr = 0; rr < CH; ++rr) {
                    const int row = a0 + rr;
                    T x = 0;
                    if (j == C) {
                        x = s_V[4 * rr + 3];
                    } else if (oi >= 0 && rr < nr) {
                        const int ra = row & 3;
                        T h = ra == 0 ? hx0 : (ra == 1 ? hx1 : (ra == 2 ? hx2 : hx3));
                        h = ((row >> 2) == oi) ? h : T(0);
                        x = h - (s_V[4 * rr] * w0 + s_V[4 * rr + 1] * w1 + s_V[4 * rr + 2] * w2);
                    }
                    if (rr & 1) bv[u][rr >> 1].y = x;
                    else bv[u][rr >> 1].x = x;
                }
                __builtin_amdgcn_sched_barrier(0);   // keep the three columns' generation apart
            }
            if (!compress) {   // R <= C: the stacked rows are H_thin (msckf.py:554-556)
                const int base = fb.row_off[f] + (a0 - 3);
#pragma unroll
                for (int u = 0; u < COLS; ++u)
                    if (lane + 64 * u <= C)
#pragma unroll
                        for (int rr = 0; rr < CH; ++rr)
                            if (rr < nr)
                                H[(size_t)(base + rr) * ldh + hcol[u]] = (rr & 1) ? bv[u][rr >> 1].y : bv[u][rr >> 1].x;
                continue;
            }
            auto load_row = [&](int r, int cmin, T* dst) {   // R[r][j] for own columns j >= cmin
#pragma unroll
                for (int u = 0; u < COLS; ++u) {
                    const int j = lane + 64 * u;
                    dst[u] = (r < C && j >= cmin && j <= C) ? H[(size_t)r * ldh + hcol[u]] : T(0);
                }
            };
            // one column step: reflector of column c from the owner lane (slot UC)
            auto step = [&](auto UCc, int c, const T* rrow) {
                constexpr int UC = decltype(UCc)::value;
                const int lc = c & 63;
                V2 v[CH2];
                V2 own2 = {0, 0};
#pragma unroll
                for (int i = 0; i < CH2; ++i) {
                    v[i].x = lane_bcast(bv[UC][i].x, lc);
                    v[i].y = lane_bcast(bv[UC][i].y, lc);
                    own2 += bv[UC][i] * bv[UC][i];
                }
                const T xs = lane_bcast(own2.x + own2.y, lc);
                const T alpha = lane_bcast(rrow[UC], lc);
                T tj = 0, scale = 0, beta = alpha;
                if (xs != T(0)) {
                    const T nrm = fast_sqrt(alpha * alpha + xs);
                    beta = alpha >= 0 ? -nrm : nrm;
                    const T rb = fast_rcp(beta);
                    tj = (beta - alpha) * rb;
                    scale = fast_rcp(alpha - beta);
                }
                const T ts = tj * scale;
#pragma unroll
                for (int u = UC; u < COLS; ++u) {
                    const int j = lane + 64 * u;
                    if (j == c) {
                        H[(size_t)c * ldh + hcol[u]] = beta;
                    } else if (j > c && j <= C && tj != T(0)) {
                        V2 q = {0, 0};
#pragma unroll
                        for (int i = 0; i < CH2; ++i) q += v[i] * bv[u][i];
                        const T w = rrow[u] + scale * (q.x + q.y);
                        H[(size_t)c * ldh + hcol[u]] = rrow[u] - tj * w;
                        const T f2 = ts * w;
                        const V2 f22 = {f2, f2};
#pragma unroll
                        for (int i = 0; i < CH2; ++i) bv[u][i] -= v[i] * f22;
                    }
                }
            };
            // R rows written by this wave's previous chunk (or the zero fill) are
            // re-read below: drain its stores first -- a load may otherwise
            // overtake a same-address store under heavy memory traffic
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            T rA[COLS], rB[COLS], rC[COLS], rD[COLS];
            load_row(c0, c0, rA);
            load_row(c0 + 1, c0 + 1, rB);
            auto segment = [&](auto UCc) {
                constexpr int UC = decltype(UCc)::value;
                const int cb = max(c0, 64 * UC), ce = min(C, 64 * (UC + 1));
                int c = cb;
                for (; c + 1 < ce; c += 2) {
                    load_row(c + 2, c + 2, rC);
                    step(UCc, c, rA);
                    load_row(c + 3, c + 3, rD);
                    step(UCc, c + 1, rB);
#pragma unroll
                    for (int u = 0; u < COLS; ++u) { rA[u] = rC[u]; rB[u] = rD[u]; }
                }
                if (c < ce) {
                    step(UCc, c, rA);
                    load_row(c + 2, c + 2, rC);
#pragma unroll
                    for (int u = 0; u < COLS; ++u) { rA[u] = rB[u]; rB[u] = rC[u]; }
                }
            };
            segment(std::integral_constant<int, 0>{});
            segment(std::integral_constant<int, 1>{});
            segment(std::integral_constant<int, 2>{});
        }
    }
}

static int g_compress_mode = -1;   // -1 auto, 0 global R, 1 LDS R (MSCKF_COMPRESS_R env)

template <typename T, int COLS, int CH>
void launch_compress_reg(hipStream_t s, const DevState<T>& st, const FeatBatch<T>& fb, const UpdWs<T>& ws) {
    const size_t base = (2 * CH + 8 + 4 * CH) * sizeof(T) + ((st.Nmax + 3) & ~3) * sizeof(int);
    const size_t rl = base + (size_t)ws.Cmax * (ws.Cmax + 1) * sizeof(T);
    if (g_compress_mode < 0) {
        const char* e = getenv("MSCKF_COMPRESS_R");
        g_compress_mode = e ? atoi(e) : 0;
    }
    if (g_compress_mode == 1 && rl <= 160 * 1024) {
        (void)hipFuncSetAttribute((const void*)k_compress_reg<T, CH, COLS, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipLaunchKernelGGL((k_compress_reg<T, CH, COLS, true>), dim3(st.B), dim3(256), rl, s, st, fb, ws);
    } else {
        hipLaunchKernelGGL((k_compress_reg<T, CH, COLS, false>), dim3(st.B), dim3(256), base, s, st, fb, ws);
    }
}

static int g_compress_ch = -1;   // rows per register chunk (MSCKF_COMPRESS_CH env: 32 | 64)

template <typename T>
void launch_qr_merge(hipStream_t s, const DevState<T>& st, const FeatBatch<T>& fb, const UpdWs<T>& ws) {
    if (g_compress_ch < 0) {
        const char* e = getenv("MSCKF_COMPRESS_CH");
        g_compress_ch = e ? atoi(e) : 16;
    }
    const bool wide = g_compress_ch >= 64 && sizeof(T) == 4;
    const char* me = getenv("MSCKF_COMPRESS_MODE");   // wave (default) | panel | block
    const int mode = me ? (me[0] == 'p' ? 1 : (me[0] == 'b' ? 2 : 0)) : 0;
    if (mode == 0 && ws.Cmax + 1 <= 192) {
        const char* we = getenv("MSCKF_COMPRESS_W");
        if (!we || atoi(we) != 0) {
            const size_t lds = (4 * 32 + 4) * sizeof(T) + ((st.Nmax + 3) & ~3) * sizeof(int);
            if (g_compress_ch == 32)
                hipLaunchKernelGGL((k_compress_w<T, 32>), dim3(st.B), dim3(64), lds, s, st, fb, ws);
            else
                hipLaunchKernelGGL((k_compress_w<T, 16>), dim3(st.B), dim3(64), lds, s, st, fb, ws);
            return;
        }
        const size_t lds = (4 * 32 + 4) * sizeof(T) + ((st.Nmax + 3) & ~3) * sizeof(int);
        if constexpr (sizeof(T) == 4) {
            if (wide) {
                hipLaunchKernelGGL((k_compress_wave<T, 64, 3>), dim3(st.B), dim3(64), lds + 4 * 32 * sizeof(T), s,
                                   st, fb, ws);
                return;
            }
            if (g_compress_ch == 16) {
                hipLaunchKernelGGL((k_compress_wave<T, 16, 3>), dim3(st.B), dim3(64), lds, s, st, fb, ws);
                return;
            }
        }
        hipLaunchKernelGGL((k_compress_wave<T, 32, 3>), dim3(st.B), dim3(64), lds, s, st, fb, ws);
        return;
    }
    if (mode <= 1 && ws.Cmax + 1 <= 256) {
        constexpr int CHP = 32;
        const size_t lds = (2 * 16 * CHP + 2 * 16 + 4 + 4 * CHP) * sizeof(T) + ((st.Nmax + 3) & ~3) * sizeof(int);
        hipLaunchKernelGGL((k_compress_panel<T, CHP>), dim3(st.B), dim3(256), lds, s, st, fb, ws);
        return;
    }
    if (ws.Cmax + 1 <= 256) {
        if (wide) launch_compress_reg<T, 1, 64>(s, st, fb, ws);
        else launch_compress_reg<T, 1, 32>(s, st, fb, ws);
    } else {
        launch_compress_reg<T, 2, 32>(s, st, fb, ws);
    }
}

// The QR path leaves [R | Q^T r] in the scalar type T; the Kalman stage reads
// H_thin in KT (fp64).
template <typename T>
__global__ void k_widen(DevState<T> st, UpdWs<T> ws) {
    const int b = blockIdx.y;
    const int n = ws.info[4 * b + 1];
    const size_t ld = ws.Cmax + 1, base = (size_t)b * ws.Cmax * ld;
    for (size_t e = blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)n * ld; e += (size_t)gridDim.x * blockDim.x)
        ws.Hthin[base + e] = (KT)ws.Hqr[base + e];
}

template <typename T>
void launch_compress_qr(hipStream_t s, const DevState<T>& st, const FeatBatch<T>& fb, const UpdWs<T>& ws) {
    launch_qr_merge<T>(s, st, fb, ws);
    hipLaunchKernelGGL(k_widen<T>, dim3(32, st.B), dim3(256), 0, s, st, ws);
}

template void launch_compress_qr<float>(hipStream_t, const DevState<float>&, const FeatBatch<float>&,
                                        const UpdWs<float>&);
template void launch_compress_qr<double>(hipStream_t, const DevState<double>&, const FeatBatch<double>&,
                                         const UpdWs<double>&);

}  // namespace msckf
