// msckf_frontend.hip -- the stereo front-end's image operators on gfx950
// (MSCKF/image.py:95-702); C-ABI in
// include/msckf_frontend.h.
//
// The reference does this work through OpenCV (FastFeatureDetector,
// calcOpticalFlowPyrLK, undistortPoints / projectPoints / fisheye).  cv2 is
// absent from this image and from the GPU box, so the kernels restate the
// published OpenCV 4.x algorithms -- the same restatement as
// oracle/frontend_oracle.py (test infrastructure), which the GPU tests check
// them against:
//   k_pyrdown   Gaussian pyramid level (pyrDown, 5x5 [1 4 6 4 1]^2, REFLECT_101)
//   k_scharr    Scharr derivatives of a level (calcScharrDeriv)
//   k_fast      FAST 9/16 segment test + corner score (fast.cpp, fast_score.cpp)
//   k_fast_rows 3x3 non-max suppression + mask, raster-order compaction: one
//               wave per image row, ballot / popcount, two passes around a host
//               prefix sum of the row counts (deterministic order)
//   k_lk        pyramidal Lucas-Kanade (LKTrackerInvoker), one wavefront per
//               point: the 15 x 15 window over the 64 lanes, 14-bit fixed-point
//               bilinear weights, window sums of the integer products reduced
//               exactly (int64) across the wave
//   k_undistort / k_distort   radtan and equidistant camera models, fp64
// Images are 8-bit, small (752 x 480 for EuRoC) and read through the cache:
// these kernels are latency-class work, not HBM-bound.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/msckf_frontend.h"

namespace {

thread_local char g_err[512] = "";
void set_err(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
#define MFE_FAIL(rc, ...)      \
    do {                       \
        set_err(__VA_ARGS__);  \
        return rc;             \
    } while (0)
#define MFE_HIP(x)                                                                          \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) MFE_FAIL(-2, "HIP error %s at %s", hipGetErrorString(e_), #x); \
    } while (0)

constexpr int MAXL = 8;        // pyramid levels (level 0 .. MAXL - 1)
constexpr int W_BITS = 14;     // lkpyramid.cpp interpolation weights
constexpr float FLT_SCALE = 1.0f / (1 << 20);

struct Level {
    int w, h;
    uint8_t* img;
    int16_t* ix;
    int16_t* iy;
};
struct Pyr {
    Level lv[MAXL];
};

__device__ __forceinline__ int refl101(int i, int n) {   // BORDER_REFLECT_101
    if (n == 1) return 0;
    const int p = 2 * n - 2;
    i %= p;
    if (i < 0) i += p;
    return i >= n ? p - i : i;
}

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// ---------------------------------------------------------------- pyramid --
__global__ void __launch_bounds__(256) k_pyrdown(const uint8_t* __restrict__ src, int sw, int sh,
                                                 uint8_t* __restrict__ dst, int dw, int dh) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= dw || y >= dh) return;
    const int k[5] = {1, 4, 6, 4, 1};
    int cols[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) cols[j] = refl101(2 * x - 2 + j, sw);
    int s = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint8_t* row = src + (size_t)refl101(2 * y - 2 + i, sh) * sw;
        int hsum = 0;
#pragma unroll
        for (int j = 0; j < 5; ++j) hsum += k[j] * row[cols[j]];
        s += k[i] * hsum;
    }
    dst[(size_t)y * dw + x] = (uint8_t)((s + 128) >> 8);
}

__global__ void __launch_bounds__(256) k_scharr(const uint8_t* __restrict__ img, int w, int h,
                                                int16_t* __restrict__ ix, int16_t* __restrict__ iy) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= w || y >= h) return;
    const int xm = refl101(x - 1, w), xp = refl101(x + 1, w);
    const uint8_t* rm = img + (size_t)refl101(y - 1, h) * w;
    const uint8_t* r0 = img + (size_t)y * w;
    const uint8_t* rp = img + (size_t)refl101(y + 1, h) * w;
    const int gx = 3 * (rm[xp] + rp[xp]) + 10 * r0[xp] - (3 * (rm[xm] + rp[xm]) + 10 * r0[xm]);
    const int gy = 3 * (rp[xm] + rp[xp]) + 10 * rp[x] - (3 * (rm[xm] + rm[xp]) + 10 * rm[x]);
    ix[(size_t)y * w + x] = (int16_t)gx;
    iy[(size_t)y * w + x] = (int16_t)gy;
}

// ------------------------------------------------------------------- FAST --
// circle of radius 3 (fast.cpp makeOffsets, pattern 16): (dx, dy)
__constant__ int c_fast_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_fast_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

// cornerScore<16> (fast_score.cpp): d[k] = v - circle[k mod 16], k = 0..24
__device__ int fast_corner_score(const int* d, int threshold) {
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = min(min(d[k + 1], d[k + 2]), d[k + 3]);
        if (a <= a0) continue;
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = max(max(d[k + 1], d[k + 2]), d[k + 3]);
        b = max(b, d[k + 4]);
        b = max(b, d[k + 5]);
        if (b >= b0) continue;
        b = max(b, d[k + 6]);
        b = max(b, d[k + 7]);
        b = max(b, d[k + 8]);
        b0 = min(b0, max(b, d[k]));
        b0 = min(b0, max(b, d[k + 9]));
    }
    return -b0 - 1;
}

// true if the 16-bit circle mask holds 9 contiguous set bits (cyclically)
__device__ __forceinline__ bool run9(unsigned m) {
    const unsigned m2 = m | (m << 16);
    unsigned r = m2 & (m2 >> 1);   // 2 in a row
    r &= r >> 2;                   // 4
    r &= r >> 4;                   // 8
    r &= m2 >> 8;                  // 9
    return (r & 0xffffu) != 0;
}

// score map: 0x100 | score for corners, 0 elsewhere (the non-max test reads
// non-corner neighbours as score 0, as fast.cpp's row buffers do)
__global__ void __launch_bounds__(256) k_fast(const uint8_t* __restrict__ img, int w, int h, int threshold,
                                              uint16_t* __restrict__ score) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= w || y >= h) return;
    uint16_t out = 0;
    if (x >= 3 && x < w - 3 && y >= 3 && y < h - 3) {
        const int v = img[(size_t)y * w + x];
        int c[16];
        unsigned bright = 0, dark = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            c[k] = img[(size_t)(y + c_fast_dy[k]) * w + x + c_fast_dx[k]];
            bright |= (unsigned)(c[k] > v + threshold) << k;
            dark |= (unsigned)(c[k] < v - threshold) << k;
        }
        if (run9(bright) || run9(dark)) {
            int d[25];
#pragma unroll
            for (int k = 0; k < 25; ++k) d[k] = v - c[k & 15];
            out = (uint16_t)(0x100 | (fast_corner_score(d, threshold) & 0xff));
        }
    }
    score[(size_t)y * w + x] = out;
}

// one wave per row: corners whose score beats all 8 neighbours (and pass the
// mask); pass 0 counts per row, pass 1 writes at row_off[y] + rank in raster order
__global__ void __launch_bounds__(256) k_fast_rows(const uint16_t* __restrict__ score, const uint8_t* __restrict__ mask,
                                                   int w, int h, int pass, int* __restrict__ row_count,
                                                   const int* __restrict__ row_off, int max_kp,
                                                   float* __restrict__ xy, float* __restrict__ resp) {
    const int lane = threadIdx.x & 63;
    const int y = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (y >= h) return;
    int count = 0;
    for (int x0 = 0; x0 < w; x0 += 64) {
        const int x = x0 + lane;
        bool keep = false;
        int s = 0;
        if (x >= 3 && x < w - 3 && y >= 3 && y < h - 3) {
            const uint16_t c = score[(size_t)y * w + x];
            s = c & 0xff;
            keep = (c >> 8) != 0;
            if (keep) {
                for (int dy = -1; dy <= 1; ++dy)
                    for (int dx = -1; dx <= 1; ++dx)
                        if ((dx || dy) && !(s > (score[(size_t)(y + dy) * w + x + dx] & 0xff))) keep = false;
                if (mask && mask[(size_t)y * w + x] == 0) keep = false;
            }
        }
        const unsigned long long bal = __ballot(keep);
        if (pass == 1 && keep) {
            const int rank = __popcll(bal & ((1ull << lane) - 1ull));
            const int pos = row_off[y] + count + rank;
            if (pos < max_kp) {
                xy[2 * pos] = (float)x;
                xy[2 * pos + 1] = (float)y;
                resp[pos] = (float)s;
            }
        }
        count += __popcll(bal);
    }
    if (pass == 0 && lane == 0) row_count[y] = count;
}

// --------------------------------------------------------------------- LK --
__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const int lo = __shfl_xor((int)(v & 0xffffffffLL), m, 64);
        const int hi = __shfl_xor((int)(v >> 32), m, 64);
        v += ((long long)hi << 32) | (unsigned int)lo;
    }
    return v;
}

template <typename Px>
__device__ __forceinline__ int bilinear(const Px* img, int w, int h, int x, int y, int w00, int w01, int w10,
                                        int w11) {
    const int x0 = refl101(x, w), x1 = refl101(x + 1, w);
    const Px* r0 = img + (size_t)refl101(y, h) * w;
    const Px* r1 = img + (size_t)refl101(y + 1, h) * w;
    return (int)r0[x0] * w00 + (int)r0[x1] * w01 + (int)r1[x0] * w10 + (int)r1[x1] * w11;
}

// The derivatives beyond the image are zero: given raw images,
// calcOpticalFlowPyrLK pads derivI with copyMakeBorder(BORDER_CONSTANT)
// (lkpyramid.cpp); only the pyramid images use BORDER_REFLECT_101.
__device__ __forceinline__ int bilinear_zero(const int16_t* img, int w, int h, int x, int y, int w00, int w01,
                                             int w10, int w11) {
    auto at = [&](int yy, int xx) -> int {
        return (xx >= 0 && xx < w && yy >= 0 && yy < h) ? (int)img[(size_t)yy * w + xx] : 0;
    };
    return at(y, x) * w00 + at(y, x + 1) * w01 + at(y + 1, x) * w10 + at(y + 1, x + 1) * w11;
}

__device__ __forceinline__ void lk_weights(float a, float b, int& w00, int& w01, int& w10, int& w11) {
    w00 = (int)rintf((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
    w01 = (int)rintf(a * (1.f - b) * (float)(1 << W_BITS));
    w10 = (int)rintf((1.f - a) * b * (float)(1 << W_BITS));
    w11 = (1 << W_BITS) - w00 - w01 - w10;
}

constexpr int LK_SLOTS = 4;   // window pixels per lane: win <= 16 (win^2 <= 256)

__global__ void __launch_bounds__(64) k_lk(Pyr P, Pyr N, int n, const float* __restrict__ prev_pts,
                                           float* __restrict__ next_pts, uint8_t* __restrict__ status, int win,
                                           int max_level, int max_iter, double eps) {
#pragma clang fp contract(off)
    const int i = blockIdx.x, lane = threadIdx.x;
    if (i >= n) return;
    const float half = (float)(win - 1) * 0.5f;
    const int npix = win * win;
    const float ppx = prev_pts[2 * i], ppy = prev_pts[2 * i + 1];
    float nx = next_pts[2 * i], ny = next_pts[2 * i + 1];   // nextPts[ptidx]
    bool st = true;
    for (int level = max_level; level >= 0; --level) {
        const Level I = P.lv[level], J = N.lv[level];
        const float sc = (float)(1. / (1 << level));
        const float px = ppx * sc - half, py = ppy * sc - half;
        float gx, gy;
        if (level == max_level) {
            gx = nx * sc;
            gy = ny * sc;
        } else {
            gx = nx * 2.f;
            gy = ny * 2.f;
        }
        nx = gx;
        ny = gy;
        gx -= half;
        gy -= half;
        const int ipx = (int)floorf(px), ipy = (int)floorf(py);
        if (ipx < -win || ipx >= I.w || ipy < -win || ipy >= I.h) {
            if (level == 0) st = false;
            continue;
        }
        int w00, w01, w10, w11;
        lk_weights(px - (float)ipx, py - (float)ipy, w00, w01, w10, w11);
        int ival[LK_SLOTS], ixv[LK_SLOTS], iyv[LK_SLOTS];
        long long s11 = 0, s12 = 0, s22 = 0;
#pragma unroll
        for (int q = 0; q < LK_SLOTS; ++q) {
            const int p = lane + 64 * q;
            ival[q] = ixv[q] = iyv[q] = 0;
            if (p < npix) {
                const int yy = p / win, xx = p - yy * win;
                ival[q] = descale(bilinear(I.img, I.w, I.h, ipx + xx, ipy + yy, w00, w01, w10, w11), W_BITS - 5);
                ixv[q] = descale(bilinear_zero(I.ix, I.w, I.h, ipx + xx, ipy + yy, w00, w01, w10, w11), W_BITS);
                iyv[q] = descale(bilinear_zero(I.iy, I.w, I.h, ipx + xx, ipy + yy, w00, w01, w10, w11), W_BITS);
                s11 += (long long)ixv[q] * ixv[q];
                s12 += (long long)ixv[q] * iyv[q];
                s22 += (long long)iyv[q] * iyv[q];
            }
        }
        s11 = wave_sum64(s11);
        s12 = wave_sum64(s12);
        s22 = wave_sum64(s22);
        const float A11 = (float)s11 * FLT_SCALE, A12 = (float)s12 * FLT_SCALE, A22 = (float)s22 * FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float min_eig =
            (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * win * win);
        if ((double)min_eig < 1e-4 || D < 1.1920928955078125e-7f) {
            if (level == 0) st = false;
            continue;
        }
        D = 1.f / D;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < max_iter; ++j) {
            const int inx = (int)floorf(gx), iny = (int)floorf(gy);
            if (inx < -win || inx >= J.w || iny < -win || iny >= J.h) {
                if (level == 0) st = false;
                break;
            }
            lk_weights(gx - (float)inx, gy - (float)iny, w00, w01, w10, w11);
            long long t1 = 0, t2 = 0;
#pragma unroll
            for (int q = 0; q < LK_SLOTS; ++q) {
                const int p = lane + 64 * q;
                if (p < npix) {
                    const int yy = p / win, xx = p - yy * win;
                    const int diff =
                        descale(bilinear(J.img, J.w, J.h, inx + xx, iny + yy, w00, w01, w10, w11), W_BITS - 5) -
                        ival[q];
                    t1 += (long long)diff * ixv[q];
                    t2 += (long long)diff * iyv[q];
                }
            }
            t1 = wave_sum64(t1);
            t2 = wave_sum64(t2);
            const float b1 = (float)t1 * FLT_SCALE, b2 = (float)t2 * FLT_SCALE;
            const float dx = (A12 * b2 - A22 * b1) * D, dy = (A12 * b1 - A11 * b2) * D;
            gx += dx;
            gy += dy;
            nx = gx + half;
            ny = gy + half;
            if ((double)dx * dx + (double)dy * dy <= eps * eps) break;
            if (j > 0 && fabs((double)(dx + pdx)) < 0.01 && fabs((double)(dy + pdy)) < 0.01) {
                nx -= dx * 0.5f;
                ny -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }
    }
    if (lane == 0) {
        next_pts[2 * i] = nx;
        next_pts[2 * i + 1] = ny;
        status[i] = st ? 1 : 0;
    }
}

// ---------------------------------------------------------- camera models --
struct CamModel {
    double fx, fy, cx, cy, k[4], R[9], nfx, nfy, ncx, ncy;
    int model;
};

__global__ void __launch_bounds__(256) k_undistort(CamModel c, int n, const double* __restrict__ in,
                                                   double* __restrict__ out) {
#pragma clang fp contract(off)
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    double x = (in[2 * t] - c.cx) / c.fx, y = (in[2 * t + 1] - c.cy) / c.fy;
    if (c.model == MFE_EQUIDISTANT) {
        // cv2.fisheye.undistortPoints (4.x) with its default criteria (COUNT +
        // EPS, 10, 1e-8): theta_d clamped to the model's 180-degree field of
        // view, Newton on theta until |step| < 1e-8; a solution that did not
        // converge or flipped sign goes out as (-1e6, -1e6), unrectified
        const double td = fmin(sqrt(x * x + y * y), M_PI / 2);
        double th = td, scale = 0.0;
        bool conv = false;
        if (td > 1e-8) {
            for (int it = 0; it < 10; ++it) {
                const double t2 = th * th, t4 = t2 * t2, t6 = t4 * t2, t8 = t6 * t2;
                const double k0t2 = c.k[0] * t2, k1t4 = c.k[1] * t4, k2t6 = c.k[2] * t6, k3t8 = c.k[3] * t8;
                const double fix = (th * (1 + k0t2 + k1t4 + k2t6 + k3t8) - td) /
                                   (1 + 3 * k0t2 + 5 * k1t4 + 7 * k2t6 + 9 * k3t8);
                th = th - fix;
                if (fabs(fix) < 1e-8) { conv = true; break; }
            }
            scale = tan(th) / td;
        } else {
            conv = true;
        }
        if (!conv || th < 0) {
            out[2 * t] = -1000000.0;
            out[2 * t + 1] = -1000000.0;
            return;
        }
        x = x * scale;
        y = y * scale;
    } else {   // cv2.undistortPoints: 5 fixed-point iterations
        const double x0 = x, y0 = y, k1 = c.k[0], k2 = c.k[1], p1 = c.k[2], p2 = c.k[3], k3 = 0.0;
        for (int it = 0; it < 5; ++it) {
            const double r2 = x * x + y * y;
            const double icdist = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2);
            const double dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x);
            const double dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y;
            x = (x0 - dx) * icdist;
            y = (y0 - dy) * icdist;
        }
    }
    const double X = c.R[0] * x + c.R[1] * y + c.R[2];
    const double Y = c.R[3] * x + c.R[4] * y + c.R[5];
    const double Wz = c.R[6] * x + c.R[7] * y + c.R[8];
    out[2 * t] = c.nfx * X / Wz + c.ncx;
    out[2 * t + 1] = c.nfy * Y / Wz + c.ncy;
}

__global__ void __launch_bounds__(256) k_distort(CamModel c, int n, const double* __restrict__ in,
                                                 double* __restrict__ out) {
#pragma clang fp contract(off)
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= n) return;
    const double x = in[2 * t], y = in[2 * t + 1];
    double xd, yd;
    if (c.model == MFE_EQUIDISTANT) {   // cv2.fisheye.distortPoints
        const double r = sqrt(x * x + y * y);
        const double th = atan(r), t2 = th * th;
        const double td = th * (1 + c.k[0] * t2 + c.k[1] * (t2 * t2) + c.k[2] * (t2 * t2 * t2) + c.k[3] * (t2 * t2 * t2 * t2));
        const double s = r > 1e-8 ? td / r : 1.0;
        xd = x * s;
        yd = y * s;
    } else {   // cv2.projectPoints, zero pose
        const double k1 = c.k[0], k2 = c.k[1], p1 = c.k[2], p2 = c.k[3], k3 = 0.0;
        const double r2 = x * x + y * y;
        const double radial = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2;
        xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x);
        yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y;
    }
    out[2 * t] = c.fx * xd + c.cx;
    out[2 * t + 1] = c.fy * yd + c.cy;
}

}  // namespace

// ================================================================ C-ABI ====
struct mfe_ctx {
    int device = 0, W = 0, H = 0, nslot = 0, max_level = 0, max_points = 0;
    hipStream_t stream = nullptr;
    std::vector<Pyr> slots;
    std::vector<void*> allocs;
    uint16_t* score = nullptr;
    uint8_t* mask = nullptr;
    int* rows = nullptr;   // [2][H]: counts, offsets
    float* kp = nullptr;   // [max_kp][3]
    int kp_cap = 0;
    float* pts = nullptr;  // [2][max_points][2]
    uint8_t* st = nullptr;
    double* dpts = nullptr;   // [2][max_points][2]
};

namespace {

int dev_alloc(mfe_ctx* c, void** p, size_t bytes) {
    MFE_HIP(hipMalloc(p, bytes ? bytes : 16));
    c->allocs.push_back(*p);
    return 0;
}

int check_n(mfe_ctx* c, int n) {
    if (n < 0 || n > c->max_points) MFE_FAIL(-1, "n = %d outside [0, %d]", n, c->max_points);
    return 0;
}

CamModel make_model(const double* intr, int model, const double* coeffs, const double* R, const double* nk) {
    CamModel m{};
    m.fx = intr[0]; m.fy = intr[1]; m.cx = intr[2]; m.cy = intr[3];
    for (int i = 0; i < 4; ++i) m.k[i] = coeffs ? coeffs[i] : 0.0;
    for (int i = 0; i < 9; ++i) m.R[i] = R ? R[i] : (i % 4 == 0 ? 1.0 : 0.0);
    m.nfx = nk ? nk[0] : 1.0; m.nfy = nk ? nk[1] : 1.0; m.ncx = nk ? nk[2] : 0.0; m.ncy = nk ? nk[3] : 0.0;
    m.model = model;
    return m;
}

}  // namespace

extern "C" {

const char* mfe_last_error(void) { return g_err; }

int mfe_create(int hip_device, int width, int height, int nslot, int max_level, int max_points, mfe_ctx_t** out) {
    if (!out) MFE_FAIL(-1, "null out");
    *out = nullptr;
    if (width < 8 || height < 8 || width > 16384 || height > 16384) MFE_FAIL(-1, "bad image size %dx%d", width, height);
    if (nslot < 1 || nslot > 16) MFE_FAIL(-1, "nslot %d outside [1, 16]", nslot);
    if (max_level < 0 || max_level >= MAXL) MFE_FAIL(-1, "max_level %d outside [0, %d]", max_level, MAXL - 1);
    if (max_points < 1) MFE_FAIL(-1, "max_points must be positive");
    MFE_HIP(hipSetDevice(hip_device));
    mfe_ctx* c = new mfe_ctx();
    c->device = hip_device; c->W = width; c->H = height; c->nslot = nslot; c->max_level = max_level;
    c->max_points = max_points;
    auto fail = [&](int rc) { mfe_destroy(c); return rc; };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        set_err("hipStreamCreate failed");
        return fail(-2);
    }
    c->slots.resize(nslot);
    for (int s = 0; s < nslot; ++s) {
        int w = width, h = height;
        for (int l = 0; l < MAXL; ++l) {
            Level& L = c->slots[s].lv[l];
            L.w = w; L.h = h; L.img = nullptr; L.ix = L.iy = nullptr;
            if (l <= max_level) {
                void *a, *b, *d;
                if (dev_alloc(c, &a, (size_t)w * h) || dev_alloc(c, &b, (size_t)w * h * 2) ||
                    dev_alloc(c, &d, (size_t)w * h * 2))
                    return fail(-2);
                L.img = (uint8_t*)a; L.ix = (int16_t*)b; L.iy = (int16_t*)d;
            }
            w = (w + 1) / 2;
            h = (h + 1) / 2;
        }
    }
    void* p;
    if (dev_alloc(c, &p, (size_t)width * height * 2)) return fail(-2);
    c->score = (uint16_t*)p;
    if (dev_alloc(c, &p, (size_t)width * height)) return fail(-2);
    c->mask = (uint8_t*)p;
    if (dev_alloc(c, &p, 2 * (size_t)height * sizeof(int))) return fail(-2);
    c->rows = (int*)p;
    c->kp_cap = 1 << 16;
    if (dev_alloc(c, &p, (size_t)c->kp_cap * 3 * sizeof(float))) return fail(-2);
    c->kp = (float*)p;
    if (dev_alloc(c, &p, 4 * (size_t)max_points * sizeof(float))) return fail(-2);
    c->pts = (float*)p;
    if (dev_alloc(c, &p, (size_t)max_points)) return fail(-2);
    c->st = (uint8_t*)p;
    if (dev_alloc(c, &p, 4 * (size_t)max_points * sizeof(double))) return fail(-2);
    c->dpts = (double*)p;
    *out = c;
    return 0;
}

int mfe_destroy(mfe_ctx_t* c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int mfe_upload(mfe_ctx_t* c, int slot, const uint8_t* image) {
    if (!c || !image) MFE_FAIL(-1, "null argument");
    if (slot < 0 || slot >= c->nslot) MFE_FAIL(-1, "slot %d outside [0, %d)", slot, c->nslot);
    MFE_HIP(hipSetDevice(c->device));
    Pyr& P = c->slots[slot];
    hipStream_t s = c->stream;
    MFE_HIP(hipMemcpyAsync(P.lv[0].img, image, (size_t)c->W * c->H, hipMemcpyHostToDevice, s));
    for (int l = 0; l <= c->max_level; ++l) {
        const Level& L = P.lv[l];
        if (l > 0) {
            const Level& U = P.lv[l - 1];
            hipLaunchKernelGGL(k_pyrdown, dim3((L.w + 15) / 16, (L.h + 15) / 16), dim3(256), 0, s, U.img, U.w, U.h,
                               L.img, L.w, L.h);
        }
        hipLaunchKernelGGL(k_scharr, dim3((L.w + 15) / 16, (L.h + 15) / 16), dim3(256), 0, s, L.img, L.w, L.h, L.ix,
                           L.iy);
    }
    MFE_HIP(hipGetLastError());
    MFE_HIP(hipStreamSynchronize(s));
    return 0;
}

int mfe_fast(mfe_ctx_t* c, int slot, int threshold, const uint8_t* mask, int max_kp, float* xy_out,
             float* response_out, int* n_out) {
    if (!c || !n_out) MFE_FAIL(-1, "null argument");
    if (slot < 0 || slot >= c->nslot) MFE_FAIL(-1, "slot %d outside [0, %d)", slot, c->nslot);
    if (max_kp < 0 || (max_kp > 0 && (!xy_out || !response_out))) MFE_FAIL(-1, "bad keypoint output");
    MFE_HIP(hipSetDevice(c->device));
    threshold = threshold < 0 ? 0 : (threshold > 255 ? 255 : threshold);
    const Level& L = c->slots[slot].lv[0];
    hipStream_t s = c->stream;
    const int W = L.w, H = L.h;
    if (mask) MFE_HIP(hipMemcpyAsync(c->mask, mask, (size_t)W * H, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_fast, dim3((W + 15) / 16, (H + 15) / 16), dim3(256), 0, s, L.img, W, H, threshold, c->score);
    hipLaunchKernelGGL(k_fast_rows, dim3((H + 3) / 4), dim3(256), 0, s, c->score, mask ? c->mask : nullptr, W, H, 0,
                       c->rows, (const int*)nullptr, 0, (float*)nullptr, (float*)nullptr);
    std::vector<int> cnt(H), off(H);
    MFE_HIP(hipMemcpyAsync(cnt.data(), c->rows, H * sizeof(int), hipMemcpyDeviceToHost, s));
    MFE_HIP(hipStreamSynchronize(s));
    int tot = 0;
    for (int y = 0; y < H; ++y) { off[y] = tot; tot += cnt[y]; }
    *n_out = tot;
    const int nw = std::min(std::min(tot, max_kp), c->kp_cap);
    if (nw > 0) {
        MFE_HIP(hipMemcpyAsync(c->rows + H, off.data(), H * sizeof(int), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_fast_rows, dim3((H + 3) / 4), dim3(256), 0, s, c->score, mask ? c->mask : nullptr, W, H, 1,
                           c->rows, (const int*)(c->rows + H), nw, c->kp, c->kp + 2 * (size_t)c->kp_cap);
        MFE_HIP(hipMemcpyAsync(xy_out, c->kp, 2 * (size_t)nw * sizeof(float), hipMemcpyDeviceToHost, s));
        MFE_HIP(hipMemcpyAsync(response_out, c->kp + 2 * (size_t)c->kp_cap, (size_t)nw * sizeof(float),
                               hipMemcpyDeviceToHost, s));
    }
    MFE_HIP(hipGetLastError());
    MFE_HIP(hipStreamSynchronize(s));
    return 0;
}

int mfe_lk(mfe_ctx_t* c, int slot_prev, int slot_next, int n, const float* prev_pts, float* next_pts,
           uint8_t* status, int win, int max_level, int max_iter, double eps) {
    if (!c) MFE_FAIL(-1, "null context");
    if (check_n(c, n)) return -1;
    if (n == 0) return 0;
    if (!prev_pts || !next_pts || !status) MFE_FAIL(-1, "null point array");
    if (slot_prev < 0 || slot_prev >= c->nslot || slot_next < 0 || slot_next >= c->nslot) MFE_FAIL(-1, "bad slot");
    if (win < 3 || win * win > 64 * LK_SLOTS) MFE_FAIL(-1, "window %d outside [3, 16]", win);
    if (max_level < 0 || max_level > c->max_level) MFE_FAIL(-1, "max_level %d outside [0, %d]", max_level, c->max_level);
    if (max_iter < 1) MFE_FAIL(-1, "max_iter must be positive");
    MFE_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    float* dprev = c->pts;
    float* dnext = c->pts + 2 * (size_t)c->max_points;
    MFE_HIP(hipMemcpyAsync(dprev, prev_pts, 2 * (size_t)n * sizeof(float), hipMemcpyHostToDevice, s));
    MFE_HIP(hipMemcpyAsync(dnext, next_pts, 2 * (size_t)n * sizeof(float), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_lk, dim3(n), dim3(64), 0, s, c->slots[slot_prev], c->slots[slot_next], n, dprev, dnext, c->st,
                       win, max_level, max_iter, eps);
    MFE_HIP(hipGetLastError());
    MFE_HIP(hipMemcpyAsync(next_pts, dnext, 2 * (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s));
    MFE_HIP(hipMemcpyAsync(status, c->st, (size_t)n, hipMemcpyDeviceToHost, s));
    MFE_HIP(hipStreamSynchronize(s));
    return 0;
}

static int cam_call(mfe_ctx_t* c, int n, const double* in, double* out, const CamModel& m, bool undist) {
    if (!c) MFE_FAIL(-1, "null context");
    if (check_n(c, n)) return -1;
    if (n == 0) return 0;
    if (!in || !out) MFE_FAIL(-1, "null point array");
    if (m.model != MFE_RADTAN && m.model != MFE_EQUIDISTANT) MFE_FAIL(-1, "unknown distortion model %d", m.model);
    MFE_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    double* din = c->dpts;
    double* dout = c->dpts + 2 * (size_t)c->max_points;
    MFE_HIP(hipMemcpyAsync(din, in, 2 * (size_t)n * sizeof(double), hipMemcpyHostToDevice, s));
    if (undist) hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, s, m, n, din, dout);
    else hipLaunchKernelGGL(k_distort, dim3((n + 255) / 256), dim3(256), 0, s, m, n, din, dout);
    MFE_HIP(hipGetLastError());
    MFE_HIP(hipMemcpyAsync(out, dout, 2 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s));
    MFE_HIP(hipStreamSynchronize(s));
    return 0;
}

int mfe_undistort(mfe_ctx_t* c, int n, const double* pts_in, double* pts_out, const double* intrinsics, int model,
                  const double* coeffs, const double* R, const double* new_intrinsics) {
    if (!intrinsics) MFE_FAIL(-1, "null intrinsics");
    return cam_call(c, n, pts_in, pts_out, make_model(intrinsics, model, coeffs, R, new_intrinsics), true);
}

int mfe_distort(mfe_ctx_t* c, int n, const double* pts_in, double* pts_out, const double* intrinsics, int model,
                const double* coeffs) {
    if (!intrinsics) MFE_FAIL(-1, "null intrinsics");
    return cam_call(c, n, pts_in, pts_out, make_model(intrinsics, model, coeffs, nullptr, nullptr), false);
}

}  // extern "C"
