// msckf_api.hip -- context management and the extern "C" ABI declared in
// include/msckf_hip.h.  Host code only: argument checking, H2D/D2H staging
// (double at the ABI <-> T on the device), launch sequencing on the context's
// HIP stream.  No CPU arithmetic of the filter happens here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/msckf_hip.h"
#include "msckf_common.h"
#include "msckf_launch.h"

using namespace msckf;

static thread_local std::string g_err;

#define FAIL(code, ...)                                  \
    do {                                                 \
        char _b[512];                                    \
        snprintf(_b, sizeof(_b), __VA_ARGS__);           \
        g_err = _b;                                      \
        return (code);                                   \
    } while (0)

#define HIPC(x)                                                                          \
    do {                                                                                 \
        hipError_t _e = (x);                                                             \
        if (_e != hipSuccess) FAIL(-2, "%s failed: %s (%s:%d)", #x, hipGetErrorString(_e), \
                                   __FILE__, __LINE__);                                   \
    } while (0)

// A synchronising call reports the failure of any asynchronous operation
// enqueued before it (kernel faults, copy errors): the message names the last
// asynchronous entry point called on the context, which is where to look first.
#define HIPSYNC(c, x)                                                                           \
    do {                                                                                        \
        hipError_t _e = (x);                                                                    \
        if (_e != hipSuccess)                                                                   \
            FAIL(-2, "%s failed: %s (%s:%d; errors of asynchronous calls surface here -- last " \
                     "asynchronous call: %s)", #x, hipGetErrorString(_e), __FILE__, __LINE__,   \
                 (c)->last_async);                                                              \
    } while (0)

namespace {

template <typename T>
struct DBuf {   // grow-only device buffer
    T* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(n, 64);
        hipError_t e = hipMalloc(&p, c * sizeof(T));
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Pinned host staging for uploads: a ring of page-locked buffers, each
// reused only after the copy out of it has completed (its event), so an
// upload returns as soon as its copy is enqueued -- no stream synchronisation
// (a copy from pageable memory is staged and waited on by the runtime).
struct PinnedRing {
    static constexpr int NS = 8;
    unsigned char* buf[NS] = {};
    size_t cap[NS] = {};
    hipEvent_t ev[NS] = {};
    bool armed[NS] = {};
    int cur = 0;
    hipError_t get(size_t n, unsigned char** out) {
        const int i = cur;
        if (armed[i]) {
            hipError_t e = hipEventSynchronize(ev[i]);
            if (e != hipSuccess) return e;
            armed[i] = false;
        }
        if (!ev[i]) {
            hipError_t e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        if (cap[i] < n) {
            if (buf[i]) (void)hipHostFree(buf[i]);
            buf[i] = nullptr;
            cap[i] = 0;
            const size_t c = std::max<size_t>(n, 1 << 16);
            hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&buf[i]), c, hipHostMallocDefault);
            if (e != hipSuccess) return e;
            cap[i] = c;
        }
        *out = buf[i];
        return hipSuccess;
    }
    hipError_t mark(hipStream_t s) {
        hipError_t e = hipEventRecord(ev[cur], s);
        armed[cur] = e == hipSuccess;
        cur = (cur + 1) % NS;
        return e;
    }
    void release() {
        for (int i = 0; i < NS; ++i) {
            if (armed[i]) (void)hipEventSynchronize(ev[i]);
            if (buf[i]) (void)hipHostFree(buf[i]);
            if (ev[i]) (void)hipEventDestroy(ev[i]);
            buf[i] = nullptr;
            ev[i] = nullptr;
            cap[i] = 0;
            armed[i] = false;
        }
    }
};

// Pinned host buffer for downloads (synchronous calls: the stream is
// synchronised before the buffer is read or reused).
struct PinnedBuf {
    unsigned char* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t c = std::max<size_t>(n, 1 << 16);
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), c, hipHostMallocDefault);
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct msckf_ctx {
    int device = 0, scalar = 8, B = 1, Nmax = 0, Dmax = 0, Cmax = 0;
    hipStream_t stream = nullptr;
    // Kalman stage A reads only P: it runs on `side` under triangulation, the
    // Jacobians and gating (fork / join events on the main stream)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    msckf_config_t cfg{};
    std::vector<int> h_ncams;
    // state
    DBuf<unsigned char> P, imu, cams, P_snap, imu_snap, cams_snap;
    DBuf<int> ncams, ncams_snap;
    DBuf<int> ident;   // [0, B): a contiguous filter list needs no upload (upload_ints)
    // update workspace
    DBuf<unsigned char> Hthin, dx, Lc, Vi, Sii, G, Tm, W, Wk;
    DBuf<int> info, afail;
    // feature batch
    int nf = 0, maxM = 0, max_nf = 0, max_obs = 0;   // per filter, of the loaded batch
    std::vector<int> h_feat_off;
    // One arena per loaded batch (load_features): the host inputs arrive in ONE
    // H2D copy, and the per-feature results [valid | p_w | include | gamma]
    // are one contiguous span for a single D2H copy (read_results).
    DBuf<unsigned char> batch;
    int *feat_filter = nullptr, *feat_off = nullptr, *obs_off = nullptr, *obs_cam = nullptr;
    long long* ysq_off = nullptr;
    int *gate_list = nullptr, *seg_list = nullptr;
    unsigned char *obs_z = nullptr, *chi2 = nullptr, *p_w = nullptr, *gamma = nullptr;
    uint8_t *valid = nullptr, *include = nullptr, *accept = nullptr;
    size_t out_off = 0;   // arena offset of the result span (valid first)
    DBuf<int> row_off;
    GateClasses gc;
    SegClasses sc;
    DBuf<unsigned char> obs_ws, obs_ht, obs_g, fqr, tau, ysq;
    bool gram = true;   // k_feature writes the Gram records (record-reading assembly)
    // misc scratch
    DBuf<unsigned char> scratch;
    DBuf<int> iscratch;
    KernelTimer timer;
    const char* last_async = "none";   // last asynchronous entry point (HIPSYNC's message)
    bool has_snapshot = false;
    PinnedRing up;      // upload staging
    PinnedBuf down;     // download staging
};

namespace {

template <typename T>
Params<T> make_params(const msckf_ctx* c) {
    Params<T> p{};
    const msckf_config_t& k = c->cfg;
    p.sigma2 = (T)k.observation_noise;
    p.qc_gyro = (T)k.gyro_noise;
    p.qc_gbias = (T)k.gyro_bias_noise;
    p.qc_acc = (T)k.acc_noise;
    p.qc_abias = (T)k.acc_bias_noise;
    for (int i = 0; i < 9; ++i) p.R01[i] = (T)k.R_cam0_cam1[i];
    for (int i = 0; i < 3; ++i) p.t01[i] = (T)k.t_cam0_cam1[i];
    p.huber = (T)k.huber_epsilon;
    p.precision = (T)k.estimation_precision;
    p.damping = (T)k.initial_damping;
    p.outer_max = k.outer_loop_max_iteration;
    p.inner_max = k.inner_loop_max_iteration;
    return p;
}

template <typename T>
DevState<T> dev_state(msckf_ctx* c) {
    DevState<T> s;
    s.P = reinterpret_cast<T*>(c->P.p);
    s.imu = reinterpret_cast<T*>(c->imu.p);
    s.cams = reinterpret_cast<T*>(c->cams.p);
    s.ncams = c->ncams.p;
    s.B = c->B;
    s.Nmax = c->Nmax;
    s.Dmax = c->Dmax;
    return s;
}

template <typename T>
UpdWs<T> upd_ws(msckf_ctx* c) {
    UpdWs<T> w;
    w.Hthin = reinterpret_cast<KT*>(c->Hthin.p);
    w.dx = reinterpret_cast<KT*>(c->dx.p);
    w.info = c->info.p;
    w.Cmax = c->Cmax;
    w.Cp = (c->Cmax + 15) & ~15;   // leading dim of Lc / Vi / W (MFMA path pads C to 16)
    w.Lc = reinterpret_cast<KT*>(c->Lc.p);
    w.afail = c->afail.p;
    w.Vi = reinterpret_cast<KT*>(c->Vi.p);
    w.Sii = reinterpret_cast<KT*>(c->Sii.p);
    w.G = reinterpret_cast<KT*>(c->G.p);
    w.Tm = reinterpret_cast<KT*>(c->Tm.p);
    w.W = reinterpret_cast<KT*>(c->W.p);
    w.Wk = reinterpret_cast<KT*>(c->Wk.p);
    w.wk_stride = kalman_global_ws_doubles(c->Cmax);
    w.s2 = (double)(T)c->cfg.observation_noise;
    return w;
}

template <typename T>
FeatBatch<T> feat_batch(msckf_ctx* c) {
    FeatBatch<T> f;
    f.nf = c->nf;
    f.feat_filter = c->feat_filter;
    f.feat_off = c->feat_off;
    f.obs_off = c->obs_off;
    f.obs_cam = c->obs_cam;
    f.obs_z = reinterpret_cast<const T*>(c->obs_z);
    f.chi2 = reinterpret_cast<const T*>(c->chi2);
    f.ysq_off = c->ysq_off;
    f.p_w = reinterpret_cast<T*>(c->p_w);
    f.valid = c->valid;
    f.obs_ws = reinterpret_cast<T*>(c->obs_ws.p);
    f.obs_ht = reinterpret_cast<T*>(c->obs_ht.p);
    f.obs_g = reinterpret_cast<double*>(c->obs_g.p);
    f.fqr = reinterpret_cast<double*>(c->fqr.p);
    f.gram = c->gram ? 1 : 0;
    f.compact = feature_needs_compact(c->maxM) ? 1 : 0;
    f.tau = reinterpret_cast<T*>(c->tau.p);
    f.ysq = reinterpret_cast<T*>(c->ysq.p);
    f.gamma = reinterpret_cast<T*>(c->gamma);
    f.accept = c->accept;
    f.include = c->include;
    f.row_off = c->row_off.p;
    return f;
}

template <typename T>
std::vector<T> to_T(const double* x, size_t n) {
    std::vector<T> v(n);
    for (size_t i = 0; i < n; ++i) v[i] = (T)x[i];
    return v;
}

// Copy a double host array to a device buffer of T: converted into a pinned
// staging buffer and enqueued on the context stream (asynchronous; the
// caller's array may be reused as soon as this returns).
template <typename T>
hipError_t upload(msckf_ctx* c, void* dst, const double* src, size_t n) {
    if (n == 0) return hipSuccess;
    unsigned char* h = nullptr;
    hipError_t e = c->up.get(n * sizeof(T), &h);
    if (e != hipSuccess) return e;
    T* v = reinterpret_cast<T*>(h);
    for (size_t i = 0; i < n; ++i) v[i] = (T)src[i];
    e = hipMemcpyAsync(dst, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    return c->up.mark(c->stream);
}

// Raw bytes, same staging (asynchronous).
hipError_t upload_raw(msckf_ctx* c, void* dst, const void* src, size_t bytes) {
    if (bytes == 0) return hipSuccess;
    unsigned char* h = nullptr;
    hipError_t e = c->up.get(bytes, &h);
    if (e != hipSuccess) return e;
    std::memcpy(h, src, bytes);
    e = hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return e;
    return c->up.mark(c->stream);
}

// Small multi-array downloads (a frame's sync point: IMU records, cams, the
// covariance diagonal, the batch results, the status words) are gathered by
// ONE kernel that writes straight into the pinned buffer -- one launch
// instead of one blit copy per array (each ~4 us of GPU time at B = 1, plus
// its API call).  The kernel's end-of-dispatch release makes the stores
// visible to the host at the stream synchronisation, as for the runtime's own
// blit kernels.  Words where the source is 4-byte aligned, bytes otherwise
// (every destination offset is 16-byte aligned).
struct GatherItems {
    static constexpr int MAX = 8;
    const unsigned char* src[MAX];
    unsigned int bytes[MAX], off[MAX];
    int n;
};
__global__ void __launch_bounds__(256) k_gather_host(GatherItems g, unsigned char* dst) {
    const unsigned t0 = blockIdx.x * 256 + threadIdx.x, step = gridDim.x * 256;
    for (int i = 0; i < g.n; ++i) {
        const unsigned char* s = g.src[i];
        unsigned char* d = dst + g.off[i];
        const unsigned nb = g.bytes[i];
        const unsigned nw = ((reinterpret_cast<uintptr_t>(s) & 3) == 0) ? nb >> 2 : 0;
        for (unsigned w = t0; w < nw; w += step)
            reinterpret_cast<unsigned*>(d)[w] = reinterpret_cast<const unsigned*>(s)[w];
        for (unsigned e = 4 * nw + t0; e < nb; e += step) d[e] = s[e];
    }
}
constexpr size_t GATHER_MAX_BYTES = 1 << 20;   // larger reads keep one runtime copy per array

// Several device arrays into one pinned buffer, ONE stream synchronisation.
struct DownList {
    struct Item { const void* src; size_t bytes, off; };
    std::vector<Item> items;
    size_t total = 0;
    size_t add(const void* src, size_t bytes) {
        const size_t off = total;
        items.push_back({src, bytes, off});
        total += (bytes + 15) & ~(size_t)15;
        return off;
    }
    hipError_t run(msckf_ctx* c) {
        hipError_t e = c->down.ensure(total);
        if (e != hipSuccess) return e;
        if (items.size() > 1 && items.size() <= (size_t)GatherItems::MAX && total <= GATHER_MAX_BYTES) {
            GatherItems g{};
            for (auto& it : items) {
                g.src[g.n] = static_cast<const unsigned char*>(it.src);
                g.bytes[g.n] = (unsigned)it.bytes;
                g.off[g.n] = (unsigned)it.off;
                ++g.n;
            }
            const unsigned grid = (unsigned)std::min<size_t>(64, (total / 4 + 255) / 256 + 1);
            hipLaunchKernelGGL(k_gather_host, dim3(grid), dim3(256), 0, c->stream, g, c->down.p);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        } else {
            for (auto& it : items)
                if (it.bytes) {
                    e = hipMemcpyAsync(c->down.p + it.off, it.src, it.bytes, hipMemcpyDeviceToHost, c->stream);
                    if (e != hipSuccess) return e;
                }
        }
        e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) c->timer.collect();
        return e;
    }
    const unsigned char* at(const msckf_ctx* c, size_t off) const { return c->down.p + off; }
};

template <typename T>
void to_double(double* dst, const unsigned char* src, size_t n) {
    const T* v = reinterpret_cast<const T*>(src);
    for (size_t i = 0; i < n; ++i) dst[i] = (double)v[i];
}

template <typename T>
hipError_t download(msckf_ctx* c, double* dst, const void* src, size_t n) {
    if (n == 0) return hipSuccess;
    DownList d;
    const size_t o = d.add(src, n * sizeof(T));
    hipError_t e = d.run(c);
    if (e == hipSuccess) to_double<T>(dst, d.at(c, o), n);
    return e;
}

int check_ctx(msckf_ctx* c, int filter) {
    if (!c) FAIL(-1, "null context");
    if (filter < 0 || filter >= c->B) FAIL(-1, "filter slot %d out of range [0,%d)", filter, c->B);
    return 0;
}

// Load a feature batch (all filters) into HBM.  feat_off == nullptr means
// all nf features belong to `single_filter`.
template <typename T>
int load_features(msckf_ctx* c, int nf, const int32_t* feat_off, int single_filter, const int32_t* obs_off,
                  const int32_t* obs_cam, const double* obs_z, const double* p_w, const double* chi2) {
    std::vector<int> h_off(c->B + 1, 0);
    if (feat_off) {
        for (int b = 0; b <= c->B; ++b) h_off[b] = feat_off[b];
        nf = h_off[c->B];
    } else {
        for (int b = 0; b <= c->B; ++b) h_off[b] = b <= single_filter ? 0 : nf;
    }
    std::vector<int> h_filt(std::max(nf, 1), 0);
    for (int b = 0; b < c->B; ++b) {
        if (h_off[b + 1] < h_off[b]) FAIL(-1, "feat_off not monotone");
        for (int f = h_off[b]; f < h_off[b + 1]; ++f) h_filt[f] = b;
    }
    if (obs_off[0] != 0) FAIL(-1, "obs_off[0] must be 0");
    const size_t nobs = nf > 0 ? (size_t)obs_off[nf] : 0;
    std::vector<long long> ysq(nf + 1, 0);
    int maxM = 0;
    for (int f = 0; f < nf; ++f) {
        int M = obs_off[f + 1] - obs_off[f];
        maxM = std::max(maxM, M);
        int b = h_filt[f];
        if (M < 1 || M > 128) FAIL(-1, "feature %d has %d observations (1..128 supported)", f, M);
        if (M > c->h_ncams[b]) FAIL(-1, "feature %d has more observations than cam states", f);
        unsigned long long seen[2] = {0, 0};   // cam slots < 128: k_info's cam -> record table needs them distinct
        for (int i = obs_off[f]; i < obs_off[f + 1]; ++i) {
            const int cam = obs_cam[i];
            if (cam < 0 || cam >= c->h_ncams[b])
                FAIL(-1, "feature %d observes cam slot %d (filter %d has %d)", f, cam, b, c->h_ncams[b]);
            if ((seen[cam >> 6] >> (cam & 63)) & 1ull) FAIL(-1, "feature %d observes cam slot %d twice", f, cam);
            seen[cam >> 6] |= 1ull << (cam & 63);
        }
        ysq[f + 1] = ysq[f] + 16LL * M * M;
    }
    const size_t ts = sizeof(T);
    HIPC(c->row_off.ensure(nf + 1));
    HIPC(c->obs_ws.ensure(((feature_needs_compact(maxM) ? nobs : 0) * OBS_WS + OBS_WS) * ts));
    HIPC(c->obs_ht.ensure((nobs * OBS_HTS + OBS_HTS) * ts));
    HIPC(c->fqr.ensure((nf + 1) * FQR_STRIDE * sizeof(double)));
    HIPC(c->tau.ensure((nf * 4 + 4) * ts));
    {   // the (4M)^2 global gating scratch is only needed by features too large
        // for the LDS gating path (M > ~50 in fp32, > ~35 in fp64)
        const size_t n4 = 4 * (size_t)maxM;
        const size_t lds = ((n4 * (n4 + 1) + 1) & ~(size_t)1) * ts + (12 * n4 + 4) * ts + (maxM + 4) * sizeof(int);
        if (lds > 160 * 1024) HIPC(c->ysq.ensure((size_t)(ysq[nf] + 16) * ts));
    }
    // gating size classes, largest first inside the list (long blocks start early)
    std::vector<int> gflat;
    GateClasses gc;
    {
        std::vector<std::vector<int>> cls(GateClasses::NC);
        for (int f = 0; f < nf; ++f) {
            const int M = obs_off[f + 1] - obs_off[f];
            int k = 0;
            while (M > GateClasses::LIM[k]) ++k;
            cls[k].push_back(f);
            gc.maxM[k] = std::max(gc.maxM[k], M);
        }
        for (int k = 0; k < GateClasses::NC; ++k) {
            gc.off[k] = (int)gflat.size();
            if (k == GateClasses::NC - 2) {   // large tracks by block count (the fp32 launches split them)
                constexpr int NS = GateClasses::BIG_NB1 - GateClasses::BIG_NB0 + 1;
                std::vector<int> sub[NS];
                for (int f : cls[k]) {
                    const int M = obs_off[f + 1] - obs_off[f], nb = (3 * M + 4 + 15) / 16 - GateClasses::BIG_NB0;
                    sub[nb].push_back(f);
                    gc.big_maxM[nb] = std::max(gc.big_maxM[nb], M);
                }
                for (int j = 0; j < NS; ++j) {
                    gc.big_off[j] = (int)gflat.size();
                    gflat.insert(gflat.end(), sub[j].begin(), sub[j].end());
                }
                gc.big_off[NS] = (int)gflat.size();
                continue;
            }
            gflat.insert(gflat.end(), cls[k].begin(), cls[k].end());
        }
        gc.off[GateClasses::NC] = (int)gflat.size();
    }
    // segment classes of the per-feature kernels (M <= S)
    std::vector<int> sflat;
    SegClasses sc;
    for (int k = 0; k < SegClasses::NC; ++k) {
        sc.off[k] = (int)sflat.size();
        for (int f = 0; f < nf; ++f) {
            const int M = obs_off[f + 1] - obs_off[f];
            if (M <= SegClasses::S[k] && (k == 0 || M > SegClasses::S[k - 1])) sflat.push_back(f);
        }
    }
    sc.off[SegClasses::NC] = (int)sflat.size();
    // the batch arena: inputs, then the result span [valid | p_w | include | gamma | accept]
    size_t total = 0;
    auto seg = [&](size_t bytes) { const size_t o = total; total += (bytes + 255) & ~(size_t)255; return o; };
    const size_t o_filt = seg(nf * sizeof(int)), o_off = seg((c->B + 1) * sizeof(int));
    const size_t o_obs = seg((nf + 1) * sizeof(int)), o_cam = seg(nobs * sizeof(int));
    const size_t o_ysq = seg((nf + 1) * sizeof(long long));
    const size_t o_gl = seg(gflat.size() * sizeof(int)), o_sl = seg(sflat.size() * sizeof(int));
    const size_t o_z = seg(nobs * 4 * ts), o_chi = seg(nf * ts);
    const size_t o_val = seg(nf), o_pw = seg(nf * 3 * ts);
    const size_t in_bytes = p_w ? total : o_pw;   // p_w uploaded only when given (else triangulation writes it)
    const size_t o_inc = seg(nf), o_gam = seg(nf * ts), o_acc = seg(nf);
    HIPC(c->batch.ensure(total + 256));
    unsigned char* d = c->batch.p;
    c->feat_filter = reinterpret_cast<int*>(d + o_filt);
    c->feat_off = reinterpret_cast<int*>(d + o_off);
    c->obs_off = reinterpret_cast<int*>(d + o_obs);
    c->obs_cam = reinterpret_cast<int*>(d + o_cam);
    c->ysq_off = reinterpret_cast<long long*>(d + o_ysq);
    c->gate_list = reinterpret_cast<int*>(d + o_gl);
    c->seg_list = reinterpret_cast<int*>(d + o_sl);
    c->obs_z = d + o_z;
    c->chi2 = d + o_chi;
    c->valid = d + o_val;
    c->p_w = d + o_pw;
    c->include = d + o_inc;
    c->gamma = d + o_gam;
    c->accept = d + o_acc;
    c->out_off = o_val;
    gc.list = c->gate_list;
    sc.list = c->seg_list;
    c->gc = gc;
    c->sc = sc;
    // every host input staged into one pinned buffer, ONE asynchronous copy
    unsigned char* h = nullptr;
    HIPC(c->up.get(in_bytes, &h));
    auto put = [&](size_t o, const void* src, size_t bytes) { if (bytes) std::memcpy(h + o, src, bytes); };
    auto putT = [&](size_t o, const double* src, size_t n) {
        T* v = reinterpret_cast<T*>(h + o);
        for (size_t i = 0; i < n; ++i) v[i] = (T)src[i];
    };
    put(o_filt, h_filt.data(), nf * sizeof(int));
    put(o_off, h_off.data(), (c->B + 1) * sizeof(int));
    put(o_obs, obs_off, (nf + 1) * sizeof(int));
    put(o_cam, obs_cam, nobs * sizeof(int));
    put(o_ysq, ysq.data(), (nf + 1) * sizeof(long long));
    put(o_gl, gflat.data(), gflat.size() * sizeof(int));
    put(o_sl, sflat.data(), sflat.size() * sizeof(int));
    putT(o_z, obs_z, nobs * 4);
    if (chi2) {
        putT(o_chi, chi2, nf);
    } else {
        T* v = reinterpret_cast<T*>(h + o_chi);
        for (int i = 0; i < nf; ++i) v[i] = (T)1e300;
    }
    // valid: 2 = position given by the host (never re-triangulated), 0 = to be
    // triangulated (p_w NULL, or a NaN row: triangulation fused into the update)
    if (p_w) {
        putT(o_pw, p_w, (size_t)nf * 3);
        for (int f = 0; f < nf; ++f) {
            const double* r = p_w + 3 * (size_t)f;
            h[o_val + f] = (std::isfinite(r[0]) && std::isfinite(r[1]) && std::isfinite(r[2])) ? 2 : 0;
        }
    } else {
        std::memset(h + o_val, 0, nf);
    }
    HIPC(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, c->stream));
    HIPC(c->up.mark(c->stream));
    c->nf = nf;
    c->maxM = maxM;
    c->max_nf = c->max_obs = 0;
    for (int b = 0; b < c->B; ++b) {
        c->max_nf = std::max(c->max_nf, h_off[b + 1] - h_off[b]);
        if (h_off[b + 1] > h_off[b]) c->max_obs = std::max(c->max_obs, obs_off[h_off[b + 1]] - obs_off[h_off[b]]);
    }
    // Gram records only for the record-reading assembly (windows > 32 cams, or
    // per-filter tables too large for the fused kernel's LDS)
    c->gram = !info_fused_fits(c->Nmax, c->max_nf);
    // (allocated in either case: k_feature writes the records of ill-conditioned
    // features for the fused assembly too -- FQR_FLAG)
    HIPC(c->obs_g.ensure(((size_t)nobs + 1) * OBG_STRIDE * sizeof(double)));
    c->h_feat_off = h_off;
    return 0;
}

template <typename T>
int run_update_chain(msckf_ctx* c, int row_cap, bool triangulate) {
    hipStream_t s = c->stream;
    DevState<T> st = dev_state<T>(c);
    Params<T> prm = make_params<T>(c);
    FeatBatch<T> fb = feat_batch<T>(c);
    UpdWs<T> ws = upd_ws<T>(c);
    // stage A (register-tile windows) under the Jacobians and gating
    const bool early_a = kalman_chol_supported(c->Cmax);
    if (triangulate) {
        c->timer.begin(s, "triangulate");
        launch_triangulate<T>(s, st, prm, fb, c->sc);
        c->timer.end(s);
    }
    // Once stage A is on the side stream, every exit path joins it: an early
    // return must not leave k_kal_a reading P while a later call (restore,
    // set_state) on the main stream overwrites it.
    struct SideJoin {
        msckf_ctx* c;
        bool armed = false;
        ~SideJoin() {
            if (armed) (void)hipStreamSynchronize(c->side);
        }
    } join{c};
    if (early_a) {
        HIPC(hipEventRecord(c->ev_fork, s));
        HIPC(hipStreamWaitEvent(c->side, c->ev_fork, 0));
        join.armed = true;
        launch_kalman_a_reg<T>(c->side, st, ws, &c->timer);
        HIPC(hipEventRecord(c->ev_join, c->side));
    }
    c->timer.begin(s, "feature_jacobian");
    launch_feature<T>(s, st, prm, fb, c->sc);
    c->timer.end(s);
    c->timer.begin(s, "gate");
    launch_gate<T>(s, st, prm, fb, c->gc);
    c->timer.end(s);
    c->timer.begin(s, "select");
    launch_select<T>(s, st, fb, ws, row_cap);
    c->timer.end(s);
    c->timer.begin(s, "compress");
    launch_compress<T>(s, st, prm, fb, ws, c->max_nf, c->max_obs);
    c->timer.end(s);
    if (early_a) {
        HIPC(hipStreamWaitEvent(s, c->ev_join, 0));
        join.armed = false;   // the main stream now orders everything after stage A
    }
    launch_kalman<T>(s, st, prm, ws, &c->timer);
    HIPC(hipGetLastError());
    return 0;
}

template <typename T>
int run_kalman_only(msckf_ctx* c) {
    hipStream_t s = c->stream;
    DevState<T> st = dev_state<T>(c);
    Params<T> prm = make_params<T>(c);
    UpdWs<T> ws = upd_ws<T>(c);
    if (kalman_chol_supported(c->Cmax)) launch_kalman_a_reg<T>(s, st, ws, &c->timer);
    launch_kalman<T>(s, st, prm, ws, &c->timer);
    HIPC(hipGetLastError());
    return 0;
}

// The loaded batch's per-feature results: queued on a DownList, unpacked after
// its (single) synchronisation.  The per-feature results are one contiguous span
// of the batch arena ([valid | p_w | include | gamma], load_features).
struct ResultsRead {
    size_t o_span = 0, o_info = 0, span = 0;
};
template <typename T>
ResultsRead add_results(msckf_ctx* c, DownList& d) {
    ResultsRead r;
    const int nf = c->nf;
    r.span = nf ? (size_t)(c->gamma - c->valid) + nf * sizeof(T) : 0;
    r.o_span = r.span ? d.add(c->valid, r.span) : 0;
    r.o_info = d.add(c->info.p, (size_t)4 * c->B * sizeof(int));
    return r;
}
template <typename T>
int unpack_results(msckf_ctx* c, const DownList& d, const ResultsRead& r, uint8_t* accepted_out, double* gamma_out,
                   double* p_w_out, uint8_t* valid_out, int32_t* rows_out) {
    const int nf = c->nf;
    const unsigned char* base = r.span ? d.at(c, r.o_span) : nullptr;
    if (accepted_out && nf) std::memcpy(accepted_out, base + (c->include - c->valid), nf);
    if (valid_out)
        for (int f = 0; f < nf; ++f) valid_out[f] = base[f] != 0;
    if (gamma_out && nf) to_double<T>(gamma_out, base + (c->gamma - c->valid), nf);
    if (p_w_out && nf) to_double<T>(p_w_out, base + (c->p_w - c->valid), (size_t)nf * 3);
    const int* info = reinterpret_cast<const int*>(d.at(c, r.o_info));
    int bad = -1;
    for (int b = 0; b < c->B; ++b) {
        if (rows_out) rows_out[b] = info[4 * b];
        if (info[4 * b + 3] < 0 && bad < 0) bad = b;
    }
    if (bad >= 0) {
        if (info[4 * bad + 3] == -2)   // stage A: the partial Cholesky of P_cc failed, shifted retries included
            FAIL(-3, "state covariance P_cc not positive definite (filter slot %d, %d rows)", bad, info[4 * bad]);
        FAIL(-3, "innovation covariance not positive definite (filter slot %d, %d rows)", bad, info[4 * bad]);
    }
    return 0;
}

template <typename T>
int read_results(msckf_ctx* c, uint8_t* accepted_out, double* gamma_out, double* p_w_out, uint8_t* valid_out,
                 int32_t* rows_out) {
    DownList d;   // every requested array in one pinned D2H batch, one synchronisation
    const ResultsRead r = add_results<T>(c, d);
    HIPSYNC(c, d.run(c));
    return unpack_results<T>(c, d, r, accepted_out, gamma_out, p_w_out, valid_out, rows_out);
}

template <typename T>
int do_create(msckf_ctx* c) {
    const size_t ts = sizeof(T);
    const size_t B = c->B;
    HIPC(c->P.ensure(B * c->Dmax * c->Dmax * ts));
    HIPC(c->imu.ensure(B * IMU_STRIDE * ts));
    HIPC(c->cams.ensure(B * c->Nmax * CAM_STRIDE * ts));
    HIPC(c->ncams.ensure(B));
    {
        std::vector<int> id(B);
        for (size_t b = 0; b < B; ++b) id[b] = (int)b;
        HIPC(c->ident.ensure(B));
        HIPC(hipMemcpy(c->ident.p, id.data(), B * sizeof(int), hipMemcpyHostToDevice));
    }
    HIPC(c->Hthin.ensure(B * c->Cmax * (c->Cmax + 1) * sizeof(KT)));
    HIPC(c->dx.ensure(B * (c->Dmax + c->Cmax) * sizeof(KT)));
    HIPC(c->info.ensure(4 * B));
    HIPC(c->afail.ensure(B));
    HIPC(hipMemset(c->afail.p, 0, B * sizeof(int)));
    {   // Cholesky-form Kalman workspace
        const size_t Cp = (c->Cmax + 15) & ~15, kb = sizeof(KT);
        HIPC(c->Lc.ensure(B * Cp * Cp * kb));
        HIPC(c->Vi.ensure(B * 24 * Cp * kb));
        HIPC(c->Sii.ensure(B * 24 * 24 * kb));
        HIPC(c->G.ensure(B * c->Cmax * (c->Cmax + 1) * kb));
        HIPC(c->Tm.ensure(B * c->Cmax * (c->Cmax + 1) * kb));
        HIPC(c->W.ensure(B * (c->Dmax + 1) * Cp * kb));
        const size_t wk = kalman_global_ws_doubles(c->Cmax);   // large windows only
        if (wk) HIPC(c->Wk.ensure(B * wk * kb));
    }
    HIPC(hipMemset(c->P.p, 0, c->P.cap));
    HIPC(hipMemset(c->cams.p, 0, c->cams.cap));
    HIPC(hipMemset(c->ncams.p, 0, B * sizeof(int)));
    HIPC(hipMemset(c->info.p, 0, 4 * B * sizeof(int)));
    std::vector<T> imu(B * IMU_STRIDE, T(0));
    for (size_t b = 0; b < B; ++b) {
        T* r = &imu[b * IMU_STRIDE];
        r[I_Q + 3] = 1;
        r[I_QN + 3] = 1;
        r[I_RIC + 0] = r[I_RIC + 4] = r[I_RIC + 8] = 1;
        r[I_G + 2] = T(-9.81);
    }
    HIPC(hipMemcpy(c->imu.p, imu.data(), imu.size() * ts, hipMemcpyHostToDevice));
    c->h_ncams.assign(B, 0);
    return 0;
}

template <typename T>
int do_set_state(msckf_ctx* c, int f, const double* imu, int n_cams, const double* cams, const double* P) {
    if (n_cams < 0 || n_cams > c->Nmax) FAIL(-1, "n_cams %d exceeds capacity %d", n_cams, c->Nmax);
    const size_t ts = sizeof(T);
    hipStream_t s = c->stream;
    if (imu) {
        std::vector<double> rec(IMU_STRIDE, 0.0);
        std::memcpy(rec.data(), imu, MSCKF_IMU_LEN * sizeof(double));
        HIPC(upload<T>(c, c->imu.p + (size_t)f * IMU_STRIDE * ts, rec.data(), IMU_STRIDE));
    }
    if (cams && n_cams) {
        std::vector<double> rec((size_t)n_cams * CAM_STRIDE, 0.0);
        for (int i = 0; i < n_cams; ++i)
            std::memcpy(&rec[(size_t)i * CAM_STRIDE], cams + (size_t)i * MSCKF_CAM_LEN, MSCKF_CAM_LEN * sizeof(double));
        HIPC(upload<T>(c, c->cams.p + (size_t)f * c->Nmax * CAM_STRIDE * ts, rec.data(), rec.size()));
    }
    if (P) {
        const int D = 21 + 6 * n_cams;
        std::vector<T> full((size_t)c->Dmax * c->Dmax, T(0));
        for (int i = 0; i < D; ++i)
            for (int j = 0; j < D; ++j) full[(size_t)i * c->Dmax + j] = (T)P[(size_t)i * D + j];
        HIPC(upload_raw(c, c->P.p + (size_t)f * c->Dmax * c->Dmax * ts, full.data(), full.size() * ts));
    }
    HIPC(upload_raw(c, c->ncams.p + f, &n_cams, sizeof(int)));
    c->h_ncams[f] = n_cams;
    (void)s;
    return 0;
}

template <typename T>
int do_get_state(msckf_ctx* c, int f, double* imu, double* cams, double* P, int* n_cams) {
    const size_t ts = sizeof(T);
    const int nc = c->h_ncams[f];
    if (n_cams) *n_cams = nc;
    DownList d;   // one stream synchronisation for all of it
    const size_t o_imu = imu ? d.add(c->imu.p + (size_t)f * IMU_STRIDE * ts, IMU_STRIDE * ts) : 0;
    const size_t o_cam = cams && nc ? d.add(c->cams.p + (size_t)f * c->Nmax * CAM_STRIDE * ts, (size_t)nc * CAM_STRIDE * ts) : 0;
    const size_t o_P = P ? d.add(c->P.p + (size_t)f * c->Dmax * c->Dmax * ts, (size_t)c->Dmax * c->Dmax * ts) : 0;
    HIPSYNC(c, d.run(c));
    if (imu) {
        std::vector<double> rec(IMU_STRIDE);
        to_double<T>(rec.data(), d.at(c, o_imu), IMU_STRIDE);
        std::memcpy(imu, rec.data(), MSCKF_IMU_LEN * sizeof(double));
    }
    if (cams && nc) {
        std::vector<double> rec((size_t)nc * CAM_STRIDE);
        to_double<T>(rec.data(), d.at(c, o_cam), rec.size());
        for (int i = 0; i < nc; ++i)
            std::memcpy(cams + (size_t)i * MSCKF_CAM_LEN, &rec[(size_t)i * CAM_STRIDE], MSCKF_CAM_LEN * sizeof(double));
    }
    if (P) {
        const int D = 21 + 6 * nc;
        const T* full = reinterpret_cast<const T*>(d.at(c, o_P));
        for (int i = 0; i < D; ++i)
            for (int j = 0; j < D; ++j) P[(size_t)i * D + j] = (double)full[(size_t)i * c->Dmax + j];
    }
    return 0;
}

// Per-filter stages over a list of filter slots: one launch for all of them
// (a single-filter call is a list of one).
int check_list(msckf_ctx* c, int nfilt, const int32_t* filters) {
    if (nfilt < 0 || (nfilt > 0 && !filters)) FAIL(-1, "bad filter list");
    std::vector<char> seen(c->B, 0);
    for (int i = 0; i < nfilt; ++i) {
        if (filters[i] < 0 || filters[i] >= c->B) FAIL(-1, "filter slot %d out of range [0,%d)", filters[i], c->B);
        if (seen[filters[i]]) FAIL(-1, "filter slot %d listed twice", filters[i]);
        seen[filters[i]] = 1;
    }
    return 0;
}

// uploads int lists to iscratch back to back; returns device pointers
int upload_ints(msckf_ctx* c, std::initializer_list<const std::vector<int>*> lists, std::vector<const int*>& out) {
    if (lists.size() == 1) {   // a run of consecutive slots (the single-filter path: [0]) is a slice of ident
        const std::vector<int>& l = **lists.begin();
        bool run = !l.empty() && l[0] >= 0 && l.back() < c->B;
        for (size_t i = 1; run && i < l.size(); ++i) run = l[i] == l[i - 1] + 1;
        if (run) {
            out.assign(1, c->ident.p + l[0]);
            return 0;
        }
    }
    size_t tot = 0;
    for (auto* l : lists) tot += l->size();
    HIPC(c->iscratch.ensure(tot + 1));
    std::vector<int> flat;
    flat.reserve(tot);
    out.clear();
    for (auto* l : lists) {
        out.push_back(c->iscratch.p + flat.size());
        flat.insert(flat.end(), l->begin(), l->end());
    }
    if (tot) HIPC(upload_raw(c, c->iscratch.p, flat.data(), tot * sizeof(int)));
    return 0;
}

template <typename T>
int do_propagate_batch(msckf_ctx* c, int nfilt, const int32_t* filters, const int32_t* smp_off, const double* dt,
                       const double* gyro, const double* acc) {
    if (nfilt <= 0) return 1;
    if (smp_off[0] != 0) FAIL(-1, "sample offsets must start at 0");
    for (int i = 0; i < nfilt; ++i)
        if (smp_off[i + 1] < smp_off[i]) FAIL(-1, "sample offsets not monotone");
    const int n = smp_off[nfilt];
    if (n <= 0) return 1;
    std::vector<double> smp((size_t)n * 7);
    for (int k = 0; k < n; ++k) {
        smp[7 * k] = dt[k];
        for (int i = 0; i < 3; ++i) {
            smp[7 * k + 1 + i] = gyro[3 * k + i];
            smp[7 * k + 4 + i] = acc[3 * k + i];
        }
    }
    // filter list, sample offsets and the samples (as T) in ONE staging buffer
    // and one H2D copy into scratch: [filters | offsets | pad to 16 | samples]
    const size_t ib = (size_t)(2 * nfilt + 1) * sizeof(int), ib16 = (ib + 15) & ~(size_t)15;
    const size_t bytes = ib16 + smp.size() * sizeof(T);
    HIPC(c->scratch.ensure(bytes));
    unsigned char* h = nullptr;
    HIPC(c->up.get(bytes, &h));
    std::memcpy(h, filters, (size_t)nfilt * sizeof(int));
    std::memcpy(h + (size_t)nfilt * sizeof(int), smp_off, (size_t)(nfilt + 1) * sizeof(int));
    T* hs = reinterpret_cast<T*>(h + ib16);
    for (size_t i = 0; i < smp.size(); ++i) hs[i] = (T)smp[i];
    HIPC(hipMemcpyAsync(c->scratch.p, h, bytes, hipMemcpyHostToDevice, c->stream));
    HIPC(c->up.mark(c->stream));
    const int* dfl = reinterpret_cast<const int*>(c->scratch.p);
    c->timer.begin(c->stream, "propagate");
    launch_propagate<T>(c->stream, dev_state<T>(c), make_params<T>(c), nfilt, dfl, dfl + nfilt,
                        reinterpret_cast<T*>(c->scratch.p + ib16));
    c->timer.end(c->stream);
    HIPC(hipGetLastError());   // asynchronous: the next synchronising call waits for it
    return 0;
}

template <typename T>
int do_augment_batch(msckf_ctx* c, int nfilt, const int32_t* filters) {
    if (nfilt <= 0) return 1;
    for (int i = 0; i < nfilt; ++i)
        if (c->h_ncams[filters[i]] >= c->Nmax)
            FAIL(-1, "filter %d: cam-state capacity %d exhausted", filters[i], c->Nmax);
    std::vector<int> fl(filters, filters + nfilt);
    std::vector<const int*> d;
    if (int r = upload_ints(c, {&fl}, d)) return r;
    c->timer.begin(c->stream, "augment");
    launch_augment<T>(c->stream, dev_state<T>(c), nfilt, d[0]);
    c->timer.end(c->stream);
    HIPC(hipGetLastError());   // asynchronous
    for (int i = 0; i < nfilt; ++i) c->h_ncams[filters[i]] += 1;
    return 0;
}

template <typename T>
int do_prune_batch(msckf_ctx* c, int nfilt, const int32_t* filters, const int32_t* slot_off, const int32_t* slots) {
    if (nfilt <= 0) return 1;
    if (slot_off[0] != 0) FAIL(-1, "slot offsets must start at 0");
    std::vector<int> fl(filters, filters + nfilt), keep, keep_off{0}, kcam, kcam_off{0};
    std::vector<int> new_n(nfilt);
    for (int w = 0; w < nfilt; ++w) {
        const int f = filters[w], nc = c->h_ncams[f];
        if (slot_off[w + 1] < slot_off[w]) FAIL(-1, "slot offsets not monotone");
        std::vector<char> rm(nc, 0);
        for (int i = slot_off[w]; i < slot_off[w + 1]; ++i) {
            if (slots[i] < 0 || slots[i] >= nc) FAIL(-1, "filter %d: prune slot %d out of range", f, slots[i]);
            rm[slots[i]] = 1;
        }
        for (int i = 0; i < 21; ++i) keep.push_back(i);
        int kept = 0;
        for (int cam = 0; cam < nc; ++cam)
            if (!rm[cam]) {
                kcam.push_back(cam);
                ++kept;
                for (int e = 0; e < 6; ++e) keep.push_back(21 + 6 * cam + e);
            }
        keep_off.push_back((int)keep.size());
        kcam_off.push_back((int)kcam.size());
        new_n[w] = kept;
    }
    std::vector<const int*> d;
    if (int r = upload_ints(c, {&fl, &keep_off, &keep, &kcam_off, &kcam}, d)) return r;
    c->timer.begin(c->stream, "prune");
    launch_prune<T>(c->stream, dev_state<T>(c), nfilt, d[0], d[1], d[2], d[3], d[4]);
    c->timer.end(c->stream);
    HIPC(hipGetLastError());   // asynchronous
    for (int w = 0; w < nfilt; ++w) c->h_ncams[filters[w]] = new_n[w];
    return 0;
}

template <typename T>
int do_cov_diag_batch(msckf_ctx* c, int nfilt, const int32_t* filters, int i0, int n, double* out) {
    if (nfilt <= 0 || n <= 0) return 0;
    for (int w = 0; w < nfilt; ++w)
        if (i0 < 0 || i0 + n > 21 + 6 * c->h_ncams[filters[w]]) FAIL(-1, "diagonal range out of bounds");
    std::vector<int> fl(filters, filters + nfilt);
    std::vector<const int*> d;
    if (int r = upload_ints(c, {&fl}, d)) return r;
    HIPC(c->scratch.ensure((size_t)nfilt * n * sizeof(T)));
    launch_cov_diag<T>(c->stream, dev_state<T>(c), nfilt, d[0], i0, n, reinterpret_cast<T*>(c->scratch.p));
    HIPC(hipGetLastError());
    return download<T>(c, out, c->scratch.p, (size_t)nfilt * n) == hipSuccess ? 0 : -2;
}

// IMU records (and optionally cam records) of the listed filters in one D2H
// copy of the state arrays.
template <typename T>
int do_get_states_batch(msckf_ctx* c, int nfilt, const int32_t* filters, double* imu_out, double* cams_out,
                        int32_t* ncams_out) {
    const size_t ts = sizeof(T);
    DownList d;   // one stream synchronisation
    const size_t o_imu = d.add(c->imu.p, (size_t)c->B * IMU_STRIDE * ts);
    const size_t o_cam = cams_out ? d.add(c->cams.p, (size_t)c->B * c->Nmax * CAM_STRIDE * ts) : 0;
    HIPSYNC(c, d.run(c));
    std::vector<double> imu_all((size_t)c->B * IMU_STRIDE);
    to_double<T>(imu_all.data(), d.at(c, o_imu), imu_all.size());
    std::vector<double> cams_all;
    if (cams_out) {
        cams_all.resize((size_t)c->B * c->Nmax * CAM_STRIDE);
        to_double<T>(cams_all.data(), d.at(c, o_cam), cams_all.size());
    }
    for (int w = 0; w < nfilt; ++w) {
        const int f = filters[w];
        if (imu_out)
            for (int e = 0; e < MSCKF_IMU_LEN; ++e) imu_out[(size_t)w * MSCKF_IMU_LEN + e] = imu_all[(size_t)f * IMU_STRIDE + e];
        if (cams_out)
            for (int k = 0; k < c->Nmax; ++k)
                for (int e = 0; e < MSCKF_CAM_LEN; ++e)
                    cams_out[((size_t)w * c->Nmax + k) * MSCKF_CAM_LEN + e] =
                        k < c->h_ncams[f] ? cams_all[((size_t)f * c->Nmax + k) * CAM_STRIDE + e] : 0.0;
        if (ncams_out) ncams_out[w] = c->h_ncams[f];
    }
    return 0;
}

// One synchronisation for a frame's sync point: the listed filters' IMU (and
// cam) records, their covariance diagonal [i0, i0 + n), and -- when any result
// pointer is given -- the loaded batch's results.
template <typename T>
int do_readback(msckf_ctx* c, int nfilt, const int32_t* filters, double* imu_out, double* cams_out,
                int32_t* ncams_out, int i0, int n, double* cov_out, uint8_t* accepted_out, double* gamma_out,
                double* p_w_out, uint8_t* valid_out, int32_t* rows_out) {
    const size_t ts = sizeof(T);
    const bool cov = nfilt > 0 && n > 0 && cov_out;
    if (cov) {
        for (int w = 0; w < nfilt; ++w)
            if (i0 < 0 || i0 + n > 21 + 6 * c->h_ncams[filters[w]]) FAIL(-1, "diagonal range out of bounds");
        std::vector<int> fl(filters, filters + nfilt);
        std::vector<const int*> dl;
        if (int r = upload_ints(c, {&fl}, dl)) return r;
        HIPC(c->scratch.ensure((size_t)nfilt * n * ts));
        launch_cov_diag<T>(c->stream, dev_state<T>(c), nfilt, dl[0], i0, n, reinterpret_cast<T*>(c->scratch.p));
        HIPC(hipGetLastError());
    }
    const bool res = accepted_out || gamma_out || p_w_out || valid_out || rows_out;
    DownList d;
    const size_t o_imu = d.add(c->imu.p, (size_t)c->B * IMU_STRIDE * ts);
    const size_t o_cam = cams_out ? d.add(c->cams.p, (size_t)c->B * c->Nmax * CAM_STRIDE * ts) : 0;
    const size_t o_cov = cov ? d.add(c->scratch.p, (size_t)nfilt * n * ts) : 0;
    ResultsRead rr;
    if (res) rr = add_results<T>(c, d);
    HIPSYNC(c, d.run(c));
    std::vector<double> imu_all((size_t)c->B * IMU_STRIDE);
    to_double<T>(imu_all.data(), d.at(c, o_imu), imu_all.size());
    std::vector<double> cams_all;
    if (cams_out) {
        cams_all.resize((size_t)c->B * c->Nmax * CAM_STRIDE);
        to_double<T>(cams_all.data(), d.at(c, o_cam), cams_all.size());
    }
    for (int w = 0; w < nfilt; ++w) {
        const int f = filters[w];
        if (imu_out)
            for (int e = 0; e < MSCKF_IMU_LEN; ++e) imu_out[(size_t)w * MSCKF_IMU_LEN + e] = imu_all[(size_t)f * IMU_STRIDE + e];
        if (cams_out)
            for (int k = 0; k < c->Nmax; ++k)
                for (int e = 0; e < MSCKF_CAM_LEN; ++e)
                    cams_out[((size_t)w * c->Nmax + k) * MSCKF_CAM_LEN + e] =
                        k < c->h_ncams[f] ? cams_all[((size_t)f * c->Nmax + k) * CAM_STRIDE + e] : 0.0;
        if (ncams_out) ncams_out[w] = c->h_ncams[f];
    }
    if (cov) to_double<T>(cov_out, d.at(c, o_cov), (size_t)nfilt * n);
    return res ? unpack_results<T>(c, d, rr, accepted_out, gamma_out, p_w_out, valid_out, rows_out) : 0;
}

template <typename T>
int run_triangulate_only(msckf_ctx* c) {
    c->timer.begin(c->stream, "triangulate");
    launch_triangulate<T>(c->stream, dev_state<T>(c), make_params<T>(c), feat_batch<T>(c), c->sc);
    c->timer.end(c->stream);
    HIPC(hipGetLastError());
    return 0;
}

template <typename T>
int do_triangulate(msckf_ctx* c, int f, int nf, const int32_t* obs_off, const int32_t* obs_cam,
                   const double* obs_z, double* p_w_out, uint8_t* valid_out) {
    if (nf <= 0) return 1;
    int r = load_features<T>(c, nf, nullptr, f, obs_off, obs_cam, obs_z, nullptr, nullptr);
    if (r) return r;
    c->timer.begin(c->stream, "triangulate");
    launch_triangulate<T>(c->stream, dev_state<T>(c), make_params<T>(c), feat_batch<T>(c), c->sc);
    c->timer.end(c->stream);
    HIPC(hipGetLastError());
    DownList d;   // one copy of the [valid | p_w] span, one stream synchronisation
    const size_t o = d.add(c->valid, (size_t)(c->p_w - c->valid) + (size_t)nf * 3 * sizeof(T));
    HIPSYNC(c, d.run(c));
    std::memcpy(valid_out, d.at(c, o), nf);
    to_double<T>(p_w_out, d.at(c, o) + (c->p_w - c->valid), (size_t)nf * 3);
    return 0;
}

template <typename T>
int do_update(msckf_ctx* c, int f, int nf, const int32_t* obs_off, const int32_t* obs_cam, const double* obs_z,
              const double* p_w, const double* chi2, int row_cap, uint8_t* accepted_out, double* gamma_out,
              int32_t* rows_out) {
    if (nf <= 0) {
        if (rows_out) *rows_out = 0;
        return 1;
    }
    int r = load_features<T>(c, nf, nullptr, f, obs_off, obs_cam, obs_z, p_w, chi2);
    if (r) return r;
    r = run_update_chain<T>(c, row_cap, false);
    if (r) return r;
    std::vector<int32_t> rows(c->B);
    r = read_results<T>(c, accepted_out, gamma_out, nullptr, nullptr, rows.data());
    if (rows_out) *rows_out = rows[f];
    if (r) return r;
    return rows[f] == 0 ? 1 : 0;
}

#define DISPATCH(c, fn, ...) ((c)->scalar == 4 ? fn<float>(__VA_ARGS__) : fn<double>(__VA_ARGS__))

}  // namespace

extern "C" {

const char* msckf_last_error(void) { return g_err.c_str(); }

int msckf_create(const msckf_config_t* cfg, int hip_device, int scalar_bytes, int n_filters, int n_cam_capacity,
                 msckf_ctx_t** out) {
    if (!cfg || !out) FAIL(-1, "null argument");
    if (scalar_bytes != 4 && scalar_bytes != 8) FAIL(-1, "scalar_bytes must be 4 or 8");
    if (n_filters < 1) FAIL(-1, "n_filters must be >= 1");
    if (n_cam_capacity < 1 || n_cam_capacity > 128) FAIL(-1, "n_cam_capacity must be in [1, 128]");
    int ndev = 0;
    HIPC(hipGetDeviceCount(&ndev));
    if (hip_device < 0 || hip_device >= ndev) FAIL(-1, "HIP device %d not present (%d visible)", hip_device, ndev);
    HIPC(hipSetDevice(hip_device));
    msckf_ctx* c = new msckf_ctx();
    c->device = hip_device;
    c->scalar = scalar_bytes;
    c->B = n_filters;
    c->Nmax = n_cam_capacity;
    c->Dmax = 21 + 6 * n_cam_capacity;
    c->Cmax = 6 * n_cam_capacity;
    c->cfg = *cfg;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    if (e != hipSuccess) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        if (c->side) (void)hipStreamDestroy(c->side);
        if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
        delete c;
        FAIL(-2, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    int r = DISPATCH(c, do_create, c);
    if (r) {
        msckf_destroy(c);
        return r;
    }
    *out = c;
    return 0;
}

int msckf_destroy(msckf_ctx_t* c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);
    for (auto* b : {&c->P, &c->imu, &c->cams, &c->P_snap, &c->imu_snap, &c->cams_snap, &c->Hthin, &c->Lc, &c->Vi, &c->Sii, &c->G, &c->Tm, &c->W, &c->Wk,
                    &c->dx, &c->batch, &c->obs_ws, &c->obs_ht, &c->obs_g, &c->fqr, &c->tau, &c->ysq, &c->scratch})
        b->release();
    for (auto* b : {&c->ncams, &c->ncams_snap, &c->ident, &c->info, &c->afail, &c->row_off, &c->iscratch})
        b->release();
    c->up.release();
    c->down.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    delete c;
    return 0;
}

int msckf_scalar_bytes(const msckf_ctx_t* c) { return c ? c->scalar : 0; }

int msckf_device_info(const msckf_ctx_t* c, int* device_out, char* pci_bus_id, int cap) {
    if (!c) FAIL(-1, "null context");
    HIPC(hipSetDevice(c->device));
    int dev = -1;
    HIPC(hipGetDevice(&dev));
    if (device_out) *device_out = dev;
    if (pci_bus_id && cap > 0) HIPC(hipDeviceGetPCIBusId(pci_bus_id, cap, dev));
    return 0;
}

int msckf_set_state(msckf_ctx_t* c, int filter, const double* imu, int n_cams, const double* cams, const double* P) {
    if (c) c->last_async = "msckf_set_state";
    if (int r = check_ctx(c, filter)) return r;
    return DISPATCH(c, do_set_state, c, filter, imu, n_cams, cams, P);
}

int msckf_get_state(msckf_ctx_t* c, int filter, double* imu, double* cams, double* P, int* n_cams) {
    if (int r = check_ctx(c, filter)) return r;
    return DISPATCH(c, do_get_state, c, filter, imu, cams, P, n_cams);
}

int msckf_get_cov_diag(msckf_ctx_t* c, int filter, int i0, int n, double* out) {
    if (int r = check_ctx(c, filter)) return r;
    if (n > 0 && !out) FAIL(-1, "null output");
    return DISPATCH(c, do_cov_diag_batch, c, 1, &filter, i0, n, out);
}

int msckf_propagate(msckf_ctx_t* c, int filter, int n, const double* dt, const double* gyro, const double* acc) {
    if (c) c->last_async = "msckf_propagate";
    if (int r = check_ctx(c, filter)) return r;
    if (n > 0 && (!dt || !gyro || !acc)) FAIL(-1, "null sample array");
    const int32_t off[2] = {0, n > 0 ? n : 0};
    return DISPATCH(c, do_propagate_batch, c, 1, &filter, off, dt, gyro, acc);
}

int msckf_propagate_batch(msckf_ctx_t* c, int nfilt, const int32_t* filters, const int32_t* sample_off,
                          const double* dt, const double* gyro, const double* acc) {
    if (c) c->last_async = "msckf_propagate_batch";
    if (!c) FAIL(-1, "null context");
    if (int r = check_list(c, nfilt, filters)) return r;
    if (nfilt > 0 && !sample_off) FAIL(-1, "null sample offsets");
    if (nfilt > 0 && sample_off[nfilt] > 0 && (!dt || !gyro || !acc)) FAIL(-1, "null sample array");
    return DISPATCH(c, do_propagate_batch, c, nfilt, filters, sample_off, dt, gyro, acc);
}

int msckf_augment(msckf_ctx_t* c, int filter) {
    if (c) c->last_async = "msckf_augment";
    if (int r = check_ctx(c, filter)) return r;
    return DISPATCH(c, do_augment_batch, c, 1, &filter);
}

int msckf_augment_batch(msckf_ctx_t* c, int nfilt, const int32_t* filters) {
    if (c) c->last_async = "msckf_augment_batch";
    if (!c) FAIL(-1, "null context");
    if (int r = check_list(c, nfilt, filters)) return r;
    return DISPATCH(c, do_augment_batch, c, nfilt, filters);
}

int msckf_triangulate(msckf_ctx_t* c, int filter, int nf, const int32_t* obs_off, const int32_t* obs_cam,
                      const double* obs_z, double* p_w_out, uint8_t* valid_out) {
    if (int r = check_ctx(c, filter)) return r;
    if (nf > 0 && (!obs_off || !obs_cam || !obs_z || !p_w_out || !valid_out)) FAIL(-1, "null argument");
    return DISPATCH(c, do_triangulate, c, filter, nf, obs_off, obs_cam, obs_z, p_w_out, valid_out);
}

int msckf_update(msckf_ctx_t* c, int filter, int nf, const int32_t* obs_off, const int32_t* obs_cam,
                 const double* obs_z, const double* p_w, const double* chi2, int row_cap, uint8_t* accepted_out,
                 double* gamma_out, int32_t* rows_out) {
    if (c) c->last_async = "msckf_update";
    if (int r = check_ctx(c, filter)) return r;
    if (nf > 0 && (!obs_off || !obs_cam || !obs_z || !p_w || !chi2)) FAIL(-1, "null argument");
    return DISPATCH(c, do_update, c, filter, nf, obs_off, obs_cam, obs_z, p_w, chi2, row_cap, accepted_out,
                    gamma_out, rows_out);
}

int msckf_prune(msckf_ctx_t* c, int filter, int n, const int32_t* cam_slots) {
    if (c) c->last_async = "msckf_prune";
    if (int r = check_ctx(c, filter)) return r;
    if (n <= 0) return 1;
    if (!cam_slots) FAIL(-1, "null slot list");
    const int32_t off[2] = {0, n};
    return DISPATCH(c, do_prune_batch, c, 1, &filter, off, cam_slots);
}

int msckf_prune_batch(msckf_ctx_t* c, int nfilt, const int32_t* filters, const int32_t* slot_off,
                      const int32_t* cam_slots) {
    if (c) c->last_async = "msckf_prune_batch";
    if (!c) FAIL(-1, "null context");
    if (int r = check_list(c, nfilt, filters)) return r;
    if (nfilt > 0 && !slot_off) FAIL(-1, "null slot offsets");
    if (nfilt > 0 && slot_off[nfilt] > 0 && !cam_slots) FAIL(-1, "null slot list");
    return DISPATCH(c, do_prune_batch, c, nfilt, filters, slot_off, cam_slots);
}

int msckf_get_states_batch(msckf_ctx_t* c, int nfilt, const int32_t* filters, double* imu_out, double* cams_out,
                           int32_t* ncams_out) {
    if (!c) FAIL(-1, "null context");
    if (int r = check_list(c, nfilt, filters)) return r;
    return DISPATCH(c, do_get_states_batch, c, nfilt, filters, imu_out, cams_out, ncams_out);
}

int msckf_get_cov_diag_batch(msckf_ctx_t* c, int nfilt, const int32_t* filters, int i0, int n, double* out) {
    if (!c) FAIL(-1, "null context");
    if (int r = check_list(c, nfilt, filters)) return r;
    if (nfilt > 0 && n > 0 && !out) FAIL(-1, "null output");
    return DISPATCH(c, do_cov_diag_batch, c, nfilt, filters, i0, n, out);
}

int msckf_readback(msckf_ctx_t* c, int nfilt, const int32_t* filters, double* imu_out, double* cams_out,
                   int32_t* ncams_out, int i0, int n, double* cov_out, uint8_t* accepted_out, double* gamma_out,
                   double* p_w_out, uint8_t* valid_out, int32_t* rows_out) {
    if (!c) FAIL(-1, "null context");
    if (int r = check_list(c, nfilt, filters)) return r;
    return DISPATCH(c, do_readback, c, nfilt, filters, imu_out, cams_out, ncams_out, i0, n, cov_out, accepted_out,
                    gamma_out, p_w_out, valid_out, rows_out);
}

int msckf_batch_triangulate(msckf_ctx_t* c) {
    if (c) c->last_async = "msckf_batch_triangulate";
    if (!c) FAIL(-1, "null context");
    return DISPATCH(c, run_triangulate_only, c);
}

int msckf_batch_load(msckf_ctx_t* c, const int32_t* feat_off, const int32_t* obs_off, const int32_t* obs_cam,
                     const double* obs_z, const double* p_w, const double* chi2) {
    if (c) c->last_async = "msckf_batch_load";
    if (!c || !feat_off || !obs_off || !obs_cam || !obs_z) FAIL(-1, "null argument");
    return DISPATCH(c, load_features, c, 0, feat_off, 0, obs_off, obs_cam, obs_z, p_w, chi2);
}

int msckf_batch_update(msckf_ctx_t* c, int row_cap, int flags) {
    if (c) c->last_async = "msckf_batch_update";
    if (!c) FAIL(-1, "null context");
    return DISPATCH(c, run_update_chain, c, row_cap, (flags & MSCKF_TRIANGULATE) != 0);
}

int msckf_batch_results(msckf_ctx_t* c, uint8_t* accepted_out, double* gamma_out, double* p_w_out,
                        uint8_t* valid_out, int32_t* rows_out) {
    if (!c) FAIL(-1, "null context");
    return DISPATCH(c, read_results, c, accepted_out, gamma_out, p_w_out, valid_out, rows_out);
}

int msckf_snapshot(msckf_ctx_t* c) {
    if (!c) FAIL(-1, "null context");
    HIPC(c->P_snap.ensure(c->P.cap));
    HIPC(c->imu_snap.ensure(c->imu.cap));
    HIPC(c->cams_snap.ensure(c->cams.cap));
    HIPC(c->ncams_snap.ensure(c->B));
    HIPC(hipMemcpyAsync(c->P_snap.p, c->P.p, c->P.cap, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->imu_snap.p, c->imu.p, c->imu.cap, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->cams_snap.p, c->cams.p, c->cams.cap, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->ncams_snap.p, c->ncams.p, c->B * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    c->has_snapshot = true;
    return 0;
}

int msckf_restore(msckf_ctx_t* c) {
    if (c) c->last_async = "msckf_restore";
    if (!c) FAIL(-1, "null context");
    if (!c->has_snapshot) FAIL(-1, "no snapshot");
    c->timer.begin(c->stream, "restore");
    HIPC(hipMemcpyAsync(c->P.p, c->P_snap.p, c->P.cap, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->imu.p, c->imu_snap.p, c->imu.cap, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->cams.p, c->cams_snap.p, c->cams.cap, hipMemcpyDeviceToDevice, c->stream));
    HIPC(hipMemcpyAsync(c->ncams.p, c->ncams_snap.p, c->B * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
    c->timer.end(c->stream);
    return 0;
}

int msckf_sync(msckf_ctx_t* c) {
    if (!c) FAIL(-1, "null context");
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    c->timer.collect();
    return 0;
}

int msckf_set_profiling(msckf_ctx_t* c, int on) {
    if (!c) FAIL(-1, "null context");
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    c->timer.collect();
    c->timer.on = on != 0;
    c->timer.only.clear();
    c->timer.reset();
    return 0;
}

int msckf_set_profiling_stage(msckf_ctx_t* c, const char* stage) {
    if (!c) FAIL(-1, "null context");
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    c->timer.collect();
    c->timer.on = stage != nullptr;
    c->timer.only = stage ? stage : "";
    c->timer.reset();
    return 0;
}

int msckf_kernel_times(msckf_ctx_t* c, int max_k, double* ms_total, int32_t* launches, char* names_out,
                       int names_cap) {
    if (!c) FAIL(-1, "null context");
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    c->timer.collect();
    int k = std::min<int>(max_k, (int)c->timer.names.size());
    std::string all;
    for (int i = 0; i < k; ++i) {
        ms_total[i] = c->timer.total_ms[i];
        launches[i] = c->timer.launches[i];
        all += c->timer.names[i];
        all.push_back('\0');
    }
    if (names_out && names_cap > 0) {
        int n = std::min<int>(names_cap - 1, (int)all.size());
        std::memcpy(names_out, all.data(), n);
        names_out[n] = 0;
    }
    return k;
}

// Debug (not in include/msckf_hip.h): copy the first `count` doubles of a
// Kalman workspace buffer (0 Lc, 1 Vi, 2 Sii, 3 G, 4 Tm, 5 W, 6 H_thin [A | b], 7 afail (ints)) to the host.
int msckf_debug_workspace(msckf_ctx_t* c, int which, double* out, size_t count) {
    if (!c || !out) FAIL(-1, "null argument");
    const void* src = which == 0 ? c->Lc.p : which == 1 ? c->Vi.p : which == 2 ? c->Sii.p
                    : which == 3 ? c->G.p : which == 4 ? c->Tm.p : which == 5 ? c->W.p
                    : which == 6 ? (const void*)c->Hthin.p : which == 7 ? (const void*)c->afail.p : nullptr;
    if (!src) FAIL(-1, "unknown workspace %d", which);
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    HIPC(hipMemcpy(out, src, count * sizeof(double), hipMemcpyDeviceToHost));
    return 0;
}

// Debug (not in include/msckf_hip.h): overwrite the first `count` doubles of a
// Kalman workspace buffer (6: H_thin [A | b], [B][Cmax][Cmax + 1]) from the host.
int msckf_debug_set_workspace(msckf_ctx_t* c, int which, const double* in, size_t count) {
    if (!c || !in) FAIL(-1, "null argument");
    void* dst = which == 6 ? (void*)c->Hthin.p : nullptr;
    if (!dst) FAIL(-1, "unknown workspace %d", which);
    if (count * sizeof(double) > c->Hthin.cap) FAIL(-1, "%zu doubles exceed H_thin", count);
    HIPSYNC(c, hipStreamSynchronize(c->stream));
    HIPC(hipMemcpy(dst, in, count * sizeof(double), hipMemcpyHostToDevice));
    return 0;
}

// Debug: the Kalman stages alone -- stage A (on the main stream), B, C, E and the
// state correction -- on the batch's current H_thin and stacking info, so that a
// test can drive the innovation factorisation with a chosen information matrix.
int msckf_debug_kalman(msckf_ctx_t* c) {
    if (c) c->last_async = "msckf_debug_kalman";
    if (!c) FAIL(-1, "null context");
    return DISPATCH(c, run_kalman_only, c);
}

}  // extern "C"
