// msckf_info_mfma.hip -- information assembly [A | b] for the Cholesky-form
// Kalman stage (msckf.py:543-604 through the Gram identity of k_info) on
// fp64 MFMA tiles.
//
// Per stacked feature f (k_feature's fp64 terms, msckf_common.h OBG_*):
//   A = sum_f [ blockdiag_i(Hx_i^T Hx_i) - G_f^T G_f ],   b = sum_f sum_i UB_i,
// with G_f the feature's 3 x C block (rows of Q^T Hx above the nullspace,
// zero outside its cams).  sum_f G_f^T G_f is a sparse SYRK: every 16 x 16
// tile (ti, tj) of A that the feature's cam columns touch takes one
// v_mfma_f64_16x16x4_f64 with the feature's three G rows (plus a zero row)
// as the K = 4 slice -- A operand lane l: G[l >> 4][16 ti + (l & 15)], B operand
// G[l >> 4][16 tj + (l & 15)].  The feature's column range is wave-uniform,
// so untouched tiles are skipped by scalar branches, not idle lanes (the
// thread-per-cam-pair kernel k_info ran ~31 % of its lanes).
//
// One workgroup (8 waves) per filter, or several for large windows (each
// owning a range of tiles, the features restaged per workgroup).  Features are
// staged FB at a time: their records copied contiguously to LDS
// (global_load_lds, double-buffered, one batch ahead), then the G rows
// scattered to dense [4][Cp] images (zeros in the feature's column range
// elsewhere, a zero fourth row) for the MFMA operands, and the per-cam
// Hx_i^T Hx_i | UB_i terms added by the staging wave into its slot's per-cam
// accumulator (slots summed in fixed order at the end: deterministic).  The block diagonal and b accumulate in registers of the threads
// owning (cam, entry) pairs; the tile owners add them when writing A.
#include "msckf_common.h"
#include "msckf_launch.h"

#include <stdlib.h>

namespace msckf {

namespace {

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int IM_NW = 8;                   // waves per workgroup
constexpr int IM_NT = 64 * IM_NW;
constexpr int IM_TPW = 10;                 // 16 x 16 tiles of A per wave
constexpr int IM_TPG = IM_NW * IM_TPW;     // tiles per workgroup
constexpr int IM_META = 4;                 // ints per staged feature: column range [lo, hi), M

__host__ __device__ constexpr int im_fb(int Nmax) { return Nmax <= 32 ? 4 : (Nmax <= 64 ? 2 : 1); }
__host__ __device__ constexpr int im_cp(int Nmax) { return (6 * Nmax + 15) / 16 * 16 + 2; }   // +16 B: row groups on distinct banks
__host__ __device__ constexpr int im_raw(int Nmax) { return (Nmax * OBG_STRIDE + 127) / 128 * 128; }   // doubles, whole 1 KiB copies
__host__ __device__ constexpr int im_ntl(int Nmax) { return (6 * Nmax + 15) / 16; }
__host__ __device__ constexpr size_t im_lds(int Nmax) {
    return ((size_t)2 * im_fb(Nmax) * im_raw(Nmax) + (size_t)im_fb(Nmax) * 4 * im_cp(Nmax)) * sizeof(double) +
           (size_t)im_fb(Nmax) * 27 * Nmax * sizeof(double) + (size_t)im_fb(Nmax) * IM_META * sizeof(int);
}

template <typename T>
__global__ void __launch_bounds__(IM_NT) k_info_mfma(DevState<T> st, FeatBatch<T> fb, UpdWs<T> ws, int phases) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    const int b = blockIdx.x, part = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nc = st.ncams[b], C = 6 * nc, Cmax = ws.Cmax, Nmax = st.Nmax;
    int* info = ws.info + 4 * b;
    if (info[0] == 0) {   // nothing stacked: empty update
        if (tid == 0 && part == 0) info[1] = 0;
        return;
    }
    const int Cp = im_cp(Nmax), RAW = im_raw(Nmax), FB = im_fb(Nmax);
    double* raw = reinterpret_cast<double*>(smem_raw);                     // [2][FB][RAW] the features' records
    double* img = raw + (size_t)2 * FB * RAW;                               // [FB][4][Cp] dense G rows
    double* dslot = img + (size_t)FB * 4 * Cp;                              // [FB][Nmax][27] Hx^T Hx | UB sums
    int* meta = reinterpret_cast<int*>(dslot + (size_t)FB * 27 * Nmax);    // [FB][IM_META]

    // this wave's tiles (wave-uniform): t = part * IM_TPG + wave + IM_NW m
    const int ntl = (C + 15) >> 4, ntiles = ntl * (ntl + 1) / 2;
    int tI[IM_TPW], tJ[IM_TPW];
#pragma unroll
    for (int m = 0; m < IM_TPW; ++m) {
        const int t = part * IM_TPG + wave + IM_NW * m;
        int i = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
        if (i * (i + 1) / 2 > t) --i;
        if ((i + 1) * (i + 2) / 2 <= t) ++i;
        tI[m] = t < ntiles ? i : -1;
        tJ[m] = t - i * (i + 1) / 2;
    }
    v4d acc[IM_TPW];
#pragma unroll
    for (int m = 0; m < IM_TPW; ++m) acc[m] = v4d{0.0, 0.0, 0.0, 0.0};
    // block diagonal | b: one [Nmax][27] accumulator per feature slot, touched
    // only by that slot's staging wave (fixed summation order, no atomics)
    for (int e = tid; e < FB * 27 * Nmax; e += IM_NT) dslot[e] = 0.0;

    // Pipeline, wave s < FB owning feature slot s of every batch:
    //   batch i: issue the contiguous copy of batch i+1's records to LDS
    //   (global_load_lds, 16 B per lane; in flight until the end of batch i),
    //   scalar-load (o0, M) of batch i+2, scatter batch i's G rows (LDS -> LDS,
    //   cam slots from the records), then every wave runs the MFMAs.
    // No ordinary global load sits on the critical path.
    const int fbeg = fb.feat_off[b], fend = fb.feat_off[b + 1];
    const bool stager = wave < FB;
    const int slot = wave % FB;   // waves FB..2FB-1 help with the same slots
    auto feat = [&](int f, int& o0, int& M) {
        o0 = 0;
        M = 0;
        if (wave < 2 * FB && f < fend && fb.include[f]) {
            o0 = fb.obs_off[f];
            M = fb.obs_off[f + 1] - o0;
        }
    };
    auto copy = [&](int o0, int M, int buf) {
        if (!stager) return;
        const char* src = reinterpret_cast<const char*>(fb.obs_g + (size_t)o0 * OBG_STRIDE);
        double* dst = raw + (size_t)(buf * FB + wave) * RAW;
        const int nchunk = M * OBG_STRIDE / 2;   // 16-byte chunks
        for (int c0 = 0; c0 < nchunk; c0 += 64)
            if (c0 + lane < nchunk)
                __builtin_amdgcn_global_load_lds((const void*)(src + 16 * (size_t)(c0 + lane)), (void*)(dst + 2 * c0), 16,
                                                 0, 0);
    };
    for (int e = tid; e < FB * Cp; e += IM_NT) img[(size_t)(e / Cp) * 4 * Cp + 3 * Cp + e % Cp] = 0.0;   // K row 3
    int o0c, Mc, o0n, Mn;   // this batch's M; the next batch's (o0, M)
    feat(fbeg + slot, o0c, Mc);
    copy(o0c, Mc, 0);
    feat(fbeg + FB + slot, o0n, Mn);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int f0 = fbeg, it = 0; f0 < fend; f0 += FB, ++it) {
        const int buf = it & 1;
        if (f0 + FB < fend) copy(o0n, Mn, buf ^ 1);
        int o0f, Mf;   // two batches ahead
        feat(f0 + 2 * FB + slot, o0f, Mf);
        // scatter this batch's G rows to the dense image and its cam -> record table
        // wave s < FB: zero + G rows of slot s and its meta; wave FB + s: its
        // Hx^T Hx | UB terms (4 elements per lane in flight: reads, then writes)
        if (wave < 2 * FB && (phases & 1)) {
            const int s = slot, M = Mc;
            const double* rs = raw + (size_t)(buf * FB + s) * RAW;
            if (wave < FB) {
                int* mt = meta + s * IM_META;
                double* g = img + (size_t)s * 4 * Cp;
                int lo = 1 << 30, hi = 0;
                for (int o = lane; o < M; o += 64) {
                    const int cam = (int)rs[o * OBG_STRIDE + OBG_CAM];
                    lo = min(lo, 6 * cam);
                    hi = max(hi, 6 * cam + 6);
                }
#pragma unroll
                for (int w = 32; w >= 1; w >>= 1) {
                    lo = min(lo, __shfl_xor(lo, w, 64));
                    hi = max(hi, __shfl_xor(hi, w, 64));
                }
                if (lo >= hi) lo = hi = 0;
                // zero the feature's whole 16-column tiles (no per-lane range tests in the MFMA loop)
                const int zlo = lo & ~15, zhi = (hi + 15) & ~15;
                for (int t = 0; t < 3; ++t)
                    for (int c = zlo + lane; c < zhi; c += 64) g[t * Cp + c] = 0.0;
                for (int e0 = lane; e0 < 18 * M; e0 += 256) {
                    double v[4];
                    int d[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int e = e0 + 64 * u, o = e / 18, r = e - 18 * o, t = r / 6;
                        d[u] = -1;
                        if (e < 18 * M) {
                            d[u] = t * Cp + 6 * (int)rs[o * OBG_STRIDE + OBG_CAM] + (r - 6 * t);
                            v[u] = rs[o * OBG_STRIDE + OBG_G + r];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (d[u] >= 0) g[d[u]] = v[u];
                }
                if (lane == 0) {
                    mt[0] = lo;
                    mt[1] = hi;
                }
            } else {
                double* ds = dslot + (size_t)s * 27 * Nmax;
                for (int e0 = lane; e0 < 27 * M; e0 += 256) {
                    double v[4];
                    int d[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int e = e0 + 64 * u, o = e / 27, k = e - 27 * o;
                        d[u] = -1;
                        if (e < 27 * M) {
                            d[u] = 27 * (int)rs[o * OBG_STRIDE + OBG_CAM] + k;
                            v[u] = rs[o * OBG_STRIDE + OBG_DS + k];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (d[u] >= 0) v[u] += ds[d[u]];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (d[u] >= 0) ds[d[u]] = v[u];
                }
            }
        }
        LDS_BARRIER();   // images ready (the next batch's copies stay in flight)
        for (int s = 0; s < FB; ++s) {
            const int* mt = meta + s * IM_META;
            const int lo = __builtin_amdgcn_readfirstlane(mt[0]), hi = __builtin_amdgcn_readfirstlane(mt[1]);
            if (lo >= hi || !(phases & 2)) continue;
            const int tlo = lo >> 4, thi = (hi - 1) >> 4;   // the feature's tile columns
            // G row 3 of the K = 4 slice is zero: lanes 48..63 read the row-3 image (kept zero)
            const double* gl = img + (size_t)s * 4 * Cp + (lane >> 4) * Cp + (lane & 15);
#pragma unroll
            for (int m = 0; m < IM_TPW; ++m) {
                const int ti = tI[m], tj = tJ[m];   // tj <= ti
                if (ti < 0 || tj < tlo || ti > thi) continue;
                acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(gl[16 * ti], gl[16 * tj], acc[m], 0, 0, 0);
            }
        }
        Mc = Mn;
        o0n = o0f;
        Mn = Mf;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // block diagonal | b sums to LDS, then the tile owners write A = D - sum G^T G
    // (both triangles) and workgroup 0 writes b
    double* dsum = raw;   // [Nmax][27]: the slot accumulators summed in slot order
    for (int e = tid; e < 27 * nc; e += IM_NT) {
        double v = 0.0;
        for (int s = 0; s < FB; ++s) v += dslot[(size_t)s * 27 * Nmax + e];
        dsum[e] = v;
    }
    __syncthreads();
    KT* F = ws.Hthin + (size_t)b * Cmax * (Cmax + 1);
    const int ldf = Cmax + 1;
#pragma unroll
    for (int m = 0; m < IM_TPW; ++m) {
        const int ti = tI[m], tj = tJ[m];
        if (ti < 0) continue;
        const int col = 16 * tj + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * ti + (lane >> 4) + 4 * r;   // f64 C/D layout
            if (row >= C || col >= C) continue;
            double v = -acc[m][r];
            const int cr = row / 6, cc = col / 6;
            if (cr == cc) {
                const int x = row - 6 * cr, y = col - 6 * cc;
                const int hi2 = x > y ? x : y, lo2 = x > y ? y : x;
                v += dsum[27 * cr + hi2 * (hi2 + 1) / 2 + lo2];
            }
            F[(size_t)row * ldf + col] = v;
            F[(size_t)col * ldf + row] = v;
        }
    }
    if (part == 0) {
        for (int e = tid; e < C; e += IM_NT) {
            const int cam = e / 6;
            F[(size_t)e * ldf + Cmax] = dsum[27 * cam + 21 + (e - 6 * cam)];
        }
        if (tid == 0) info[1] = C;
    }
}

}  // namespace

bool info_mfma_enabled(int Nmax) {
    static int mode = -1;   // MSCKF_INFO=mfma selects this kernel over k_info (A/B runs)
    if (mode < 0) {
        const char* e = getenv("MSCKF_INFO");
        mode = (e && e[0] == 'm') ? 1 : 0;   // opt-in: HBM-read-bound like k_info, and not faster
    }
    return mode == 1 && im_lds(Nmax) <= 160 * 1024;
}

template <typename T>
void launch_info_mfma(hipStream_t s, const DevState<T>& st, const FeatBatch<T>& fb, const UpdWs<T>& ws) {
    const int ntl = im_ntl(st.Nmax);
    const size_t lds = im_lds(st.Nmax);
    const int parts = (ntl * (ntl + 1) / 2 + IM_TPG - 1) / IM_TPG;
    static size_t attr = 64 * 1024;
    if (lds > attr) {
        (void)hipFuncSetAttribute((const void*)k_info_mfma<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = lds;
    }
    static int phases = -1;   // MSCKF_INFO_PHASES: profiling aid (bit0 staging scatter, bit1 MFMA)
    if (phases < 0) {
        const char* e = getenv("MSCKF_INFO_PHASES");
        phases = e ? atoi(e) : 3;
    }
    hipLaunchKernelGGL(k_info_mfma<T>, dim3(st.B, parts), dim3(IM_NT), lds, s, st, fb, ws, phases);
}

template void launch_info_mfma<float>(hipStream_t, const DevState<float>&, const FeatBatch<float>&,
                                      const UpdWs<float>&);
template void launch_info_mfma<double>(hipStream_t, const DevState<double>&, const FeatBatch<double>&,
                                       const UpdWs<double>&);

}  // namespace msckf
