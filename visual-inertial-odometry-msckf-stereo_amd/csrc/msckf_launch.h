// msckf_launch.h -- host-side launcher declarations + per-kernel HIP-event timer.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "msckf_common.h"

namespace msckf {

// Raise a kernel's dynamic-LDS limit to at least `bytes` on the current
// device.  hipFuncSetAttribute is per device, so the grant is remembered per
// (kernel, device) -- a process-wide flag would skip a context on a second
// device -- and under a lock (contexts may launch from several threads).
inline void lds_limit(const void* fn, size_t bytes) {
    if (bytes <= 64 * 1024) return;   // the default grant
    struct Grant { const void* fn; int dev; size_t bytes; };
    static std::mutex mu;
    static std::vector<Grant> grants;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    for (auto& e : grants)
        if (e.fn == fn && e.dev == dev) {
            if (e.bytes >= bytes) return;
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
            e.bytes = bytes;
            return;
        }
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    grants.push_back({fn, dev, bytes});
}

// Accumulates device time per kernel name from HIP events recorded on the
// launch stream (so the measurement sees exactly the stream the kernel runs on).
struct KernelTimer {
    bool on = false;
    std::string only;    // non-empty: time this stage only (the others record no events)
    bool open = false;   // the last begin() recorded an event
    struct Pending { std::string name; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<std::string> names;
    std::vector<double> total_ms;
    std::vector<int> launches;
    std::vector<hipEvent_t> pool;

    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e;
        (void)hipEventCreate(&e);
        return e;
    }
    void begin(hipStream_t s, const char* name) {
        open = on && (only.empty() || only == name);
        if (!open) return;
        Pending p{name, get(), get()};
        (void)hipEventRecord(p.a, s);
        pending.push_back(p);
    }
    void end(hipStream_t s) {
        if (!open || pending.empty()) return;
        (void)hipEventRecord(pending.back().b, s);
        open = false;
    }
    // call after the stream is synchronised
    void collect() {
        for (auto& p : pending) {
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, p.a, p.b);
            size_t k = 0;
            while (k < names.size() && names[k] != p.name) ++k;
            if (k == names.size()) { names.push_back(p.name); total_ms.push_back(0); launches.push_back(0); }
            total_ms[k] += ms;
            launches[k] += 1;
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
    void reset() { names.clear(); total_ms.clear(); launches.clear(); }
    ~KernelTimer() {
        for (auto& p : pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

// Per-filter stages batched over a device list of filter slots (one
// workgroup per listed filter).
template <typename T>
void launch_propagate(hipStream_t, const DevState<T>&, const Params<T>&, int nfilt, const int* filters,
                      const int* smp_off, const T* samples);
template <typename T>
void launch_augment(hipStream_t, const DevState<T>&, int nfilt, const int* filters);
template <typename T>
void launch_prune(hipStream_t, const DevState<T>&, int nfilt, const int* filters, const int* keep_off,
                  const int* keep, const int* kcam_off, const int* keep_cams);
template <typename T>
void launch_cov_diag(hipStream_t, const DevState<T>&, int nfilt, const int* filters, int i0, int n, T* out);
// Per-feature kernels packed S lanes per feature: features listed by class
// (M <= S), 64/S features per wavefront.
struct SegClasses {
    static constexpr int NC = 5;
    static constexpr int S[NC] = {8, 16, 32, 64, 128};   // 128: a whole wavefront, 2 observations per lane
    const int* list = nullptr;
    int off[NC + 1] = {};
};
template <typename T>
void launch_triangulate(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const SegClasses&);
template <typename T>
void launch_feature(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const SegClasses&);
// Feature index lists per gating size class (device pointer + host offsets).
// Gating size classes by observation count M.  Class c < NC-2 holds the
// tracks of exactly c + 1 16-row blocks (ceil((3M + 4) / 16)) and runs the
// one-wave MFMA kernel k_gate_mfma (fp64: up to 7 blocks; its 8-block class runs
// k_gate_mfma_wt); class NC-2 (40 < M <= 82) the multi-wave MFMA kernel
// k_gate_mfma_wt by block count (fp32: its 8-block sub-list, M = 41, one-wave);
// the last class the workgroup LDS kernel (or its global-memory variant).
struct GateClasses {
    // block boundaries: ceil((3M + 4) / 16) = 1..8 for M <= 4, 9, 14, 20, 25, 30, 36, 40
    static constexpr int NC = 10;
    static constexpr int LIM[NC] = {4, 9, 14, 20, 25, 30, 36, 40, 82, 1 << 30};
    const int* list = nullptr;
    int off[NC + 1] = {};
    int maxM[NC] = {};
    // class NC - 2 (40 < M <= 82) ordered by the 16-row block count nb =
    // ceil((3M + 4) / 16) = BIG_NB0 .. BIG_NB1: features of block count nb at
    // list[big_off[nb - BIG_NB0] .. big_off[nb - BIG_NB0 + 1])
    static constexpr int BIG_NB0 = 8, BIG_NB1 = 16;
    int big_off[BIG_NB1 - BIG_NB0 + 2] = {};
    int big_maxM[BIG_NB1 - BIG_NB0 + 1] = {};
};
template <typename T>
void launch_gate(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const GateClasses&);
// Gating on MFMA tiles (msckf_gate_mfma.hip), one wavefront per feature, M <= 40
// (fp32: v_mfma_f32_16x16x4_f32, fp64: v_mfma_f64_16x16x4_f64).
bool gate_mfma_fits(int maxM, int scalar_bytes);
template <typename T>
void launch_gate_mfma(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const int* list, int cnt,
                      int maxM);
// fp32 gating of the tracks of exactly nb 16-row blocks (9 <= nb <= 16, 41 < M <= 84)
// on a 2- / 4- / 8-wave workgroup per feature (k_gate_mfma_wt)
bool gate_mfma_wt_fits(int maxM);
template <typename T>
void launch_gate_mfma_wt(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const int* list,
                         int cnt, int nb, int maxM);
template <typename T>
void launch_select(hipStream_t, const DevState<T>&, const FeatBatch<T>&, const UpdWs<T>&, int row_cap);
template <typename T>
void launch_compress(hipStream_t, const DevState<T>&, const Params<T>&, const FeatBatch<T>&, const UpdWs<T>&, int maxnf,
                     int maxobs);
// The fused information assembly (no per-observation Gram records) runs when
// the window has <= 32 cams and its per-filter tables fit the LDS.
bool info_fused_fits(int Nmax, int maxnf);
// The workgroup gating kernels (M > 82) need k_feature's compact QR factors
bool feature_needs_compact(int maxM);
bool kalman_chol_supported(int Cmax);
size_t kalman_global_ws_doubles(int Cmax);
// Stage A of the register-tile windows (kalman_chol_supported) reads only P and
// writes only Lc / Vi / Sii / afail, so it is launched on a side stream at the
// start of the update chain; launch_kalman_chol then skips it.
template <typename T>
void launch_kalman_a_reg(hipStream_t, const DevState<T>&, const UpdWs<T>&, KernelTimer*);
template <typename T>
void launch_kalman_chol(hipStream_t, const DevState<T>&, const Params<T>&, const UpdWs<T>&, KernelTimer*);
template <typename T>
void launch_kalman(hipStream_t, const DevState<T>&, const Params<T>&, const UpdWs<T>&, KernelTimer*);

}  // namespace msckf
