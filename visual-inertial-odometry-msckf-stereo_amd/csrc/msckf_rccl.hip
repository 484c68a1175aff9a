// msckf_rccl.hip -- RCCL transport of the multi-GPU replica launch
// (include/msckf_replicas.h).  Host code only: one communicator per process
// (one process per GPU), control messages only -- the start / stop barriers
// of a timed region, the max over ranks of its elapsed time, the gather of
// each rank's device identity.  The filters on different GPUs share no state
// (SURVEY.md 8(e)); the reference has no collectives at all (its only
// concurrency: MSCKF/vio.py:23-28).
//
// librccl is opened with dlopen, so libmsckf_hip.so loads without it.  The
// communicator is non-blocking (ncclConfig_t.blocking = 0) and every wait is
// a poll with a deadline: a rank that never arrives makes the others return
// an error (after ncclCommAbort) instead of hanging the job.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "msckf_replicas.h"

static thread_local std::string r_err;

#define RFAIL(code, ...)                             \
    do {                                             \
        char _b[512];                                \
        snprintf(_b, sizeof(_b), __VA_ARGS__);       \
        r_err = _b;                                  \
        return (code);                               \
    } while (0)

namespace {

struct RcclApi {
    bool tried = false, ok = false;
    void* h = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
    ncclResult_t (*commGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
    ncclResult_t (*commAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*commFinalize)(ncclComm_t) = nullptr;   // optional (older RCCL lacks it)
    ncclResult_t (*commCount)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*errorString)(ncclResult_t) = nullptr;
    std::string why;
};
RcclApi g_api;

template <typename F>
bool sym(F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(g_api.h, name));
    return f != nullptr;
}

bool load_rccl() {
    if (g_api.tried) return g_api.ok;
    g_api.tried = true;
    for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
        g_api.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
        if (g_api.h) break;
    }
    if (!g_api.h) {
        const char* e = dlerror();
        g_api.why = std::string("dlopen(librccl) failed: ") + (e ? e : "?");
        return false;
    }
    g_api.ok = sym(g_api.getUniqueId, "ncclGetUniqueId") && sym(g_api.commInitRankConfig, "ncclCommInitRankConfig") &&
               sym(g_api.commGetAsyncError, "ncclCommGetAsyncError") && sym(g_api.commAbort, "ncclCommAbort") &&
               sym(g_api.commDestroy, "ncclCommDestroy") && sym(g_api.commCount, "ncclCommCount") &&
               sym(g_api.allReduce, "ncclAllReduce") && sym(g_api.allGather, "ncclAllGather") &&
               sym(g_api.errorString, "ncclGetErrorString");
    if (!g_api.ok) g_api.why = "librccl lacks a required symbol";
    (void)sym(g_api.commFinalize, "ncclCommFinalize");
    return g_api.ok;
}

const char* rstr(ncclResult_t r) { return g_api.errorString ? g_api.errorString(r) : "?"; }

using Clock = std::chrono::steady_clock;

}  // namespace

struct msckf_rccl {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    int rank = 0, nranks = 0, device = 0;
    double timeout_s = 60.0;
    double* dbuf = nullptr;          // device staging for the collectives
    size_t dcap = 0;                 // bytes
};

namespace {

// Wait until the non-blocking communicator has finished enqueuing (ncclInProgress
// -> ncclSuccess); on timeout or error abort it.
int wait_comm(msckf_rccl* c, const char* what) {
    const auto t0 = Clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        ncclResult_t r = g_api.commGetAsyncError(c->comm, &st);
        if (r != ncclSuccess) RFAIL(-4, "%s: ncclCommGetAsyncError: %s", what, rstr(r));
        if (st == ncclSuccess) return 0;
        if (st != ncclInProgress) {
            g_api.commAbort(c->comm);
            c->comm = nullptr;
            RFAIL(-4, "%s: %s", what, rstr(st));
        }
        if (std::chrono::duration<double>(Clock::now() - t0).count() > c->timeout_s) {
            g_api.commAbort(c->comm);
            c->comm = nullptr;
            RFAIL(-4, "%s: timed out after %.0f s", what, c->timeout_s);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// hipStreamSynchronize with a deadline (a peer that never joins the collective
// must not hang this rank forever).
int sync_stream(msckf_rccl* c, const char* what) {
    const auto t0 = Clock::now();
    for (;;) {
        hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) return 0;
        if (e != hipErrorNotReady) RFAIL(-2, "%s: %s", what, hipGetErrorString(e));
        if (std::chrono::duration<double>(Clock::now() - t0).count() > c->timeout_s) {
            g_api.commAbort(c->comm);
            c->comm = nullptr;
            RFAIL(-4, "%s: collective did not complete within %.0f s", what, c->timeout_s);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

int ensure_dbuf(msckf_rccl* c, size_t bytes) {
    if (bytes <= c->dcap) return 0;
    if (c->dbuf) (void)hipFree(c->dbuf);
    c->dbuf = nullptr;
    c->dcap = 0;
    hipError_t e = hipMalloc(&c->dbuf, bytes);
    if (e != hipSuccess) RFAIL(-2, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    c->dcap = bytes;
    return 0;
}

}  // namespace

extern "C" {

const char* msckf_rccl_last_error(void) { return r_err.c_str(); }

int msckf_rccl_unique_id(uint8_t* id_out) {
    if (!id_out) RFAIL(-1, "null id buffer");
    if (!load_rccl()) RFAIL(-5, "%s", g_api.why.c_str());
    static_assert(sizeof(ncclUniqueId) == MSCKF_RCCL_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    ncclResult_t r = g_api.getUniqueId(&id);
    if (r != ncclSuccess) RFAIL(-4, "ncclGetUniqueId: %s", rstr(r));
    std::memcpy(id_out, &id, sizeof(id));
    return 0;
}

int msckf_rccl_init(const uint8_t* id, int nranks, int rank, int hip_device, double timeout_s, msckf_rccl_t** out) {
    if (!id || !out) RFAIL(-1, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) RFAIL(-1, "rank %d of %d", rank, nranks);
    if (!load_rccl()) RFAIL(-5, "%s", g_api.why.c_str());
    hipError_t e = hipSetDevice(hip_device);
    if (e != hipSuccess) RFAIL(-2, "hipSetDevice(%d): %s", hip_device, hipGetErrorString(e));
    auto* c = new msckf_rccl();
    c->rank = rank;
    c->nranks = nranks;
    c->device = hip_device;
    c->timeout_s = timeout_s > 0 ? timeout_s : 60.0;
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        RFAIL(-2, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = g_api.commInitRankConfig(&c->comm, nranks, uid, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        RFAIL(-4, "ncclCommInitRankConfig: %s", rstr(r));
    }
    if (int rc = wait_comm(c, "ncclCommInitRankConfig")) {
        (void)hipStreamDestroy(c->stream);
        delete c;
        return rc;
    }
    *out = c;
    return 0;
}

int msckf_rccl_allreduce(msckf_rccl_t* c, double* v, int n, int op) {
    if (!c || !c->comm) RFAIL(-1, "no communicator");
    if (n <= 0) return 0;
    if (!v) RFAIL(-1, "null buffer");
    if (int rc = ensure_dbuf(c, (size_t)n * sizeof(double))) return rc;
    hipError_t e = hipMemcpyAsync(c->dbuf, v, n * sizeof(double), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) RFAIL(-2, "hipMemcpyAsync: %s", hipGetErrorString(e));
    ncclResult_t r = g_api.allReduce(c->dbuf, c->dbuf, (size_t)n, ncclFloat64, op == 1 ? ncclMax : ncclSum, c->comm,
                                     c->stream);
    if (r != ncclSuccess && r != ncclInProgress) RFAIL(-4, "ncclAllReduce: %s", rstr(r));
    if (int rc = wait_comm(c, "ncclAllReduce")) return rc;
    e = hipMemcpyAsync(v, c->dbuf, n * sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e != hipSuccess) RFAIL(-2, "hipMemcpyAsync: %s", hipGetErrorString(e));
    return sync_stream(c, "ncclAllReduce");
}

int msckf_rccl_allgather(msckf_rccl_t* c, const void* mine, int nbytes, void* all_out) {
    if (!c || !c->comm) RFAIL(-1, "no communicator");
    if (nbytes <= 0) return 0;
    if (!mine || !all_out) RFAIL(-1, "null buffer");
    const size_t per = ((size_t)nbytes + 7) & ~(size_t)7;
    if (int rc = ensure_dbuf(c, per * (c->nranks + 1))) return rc;
    unsigned char* d = reinterpret_cast<unsigned char*>(c->dbuf);
    unsigned char* send = d + per * c->nranks;
    hipError_t e = hipMemcpyAsync(send, mine, nbytes, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) RFAIL(-2, "hipMemcpyAsync: %s", hipGetErrorString(e));
    ncclResult_t r = g_api.allGather(send, d, per, ncclUint8, c->comm, c->stream);
    if (r != ncclSuccess && r != ncclInProgress) RFAIL(-4, "ncclAllGather: %s", rstr(r));
    if (int rc = wait_comm(c, "ncclAllGather")) return rc;
    for (int k = 0; k < c->nranks; ++k) {
        e = hipMemcpyAsync(static_cast<unsigned char*>(all_out) + (size_t)k * nbytes, d + per * k, nbytes,
                           hipMemcpyDeviceToHost, c->stream);
        if (e != hipSuccess) RFAIL(-2, "hipMemcpyAsync: %s", hipGetErrorString(e));
    }
    return sync_stream(c, "ncclAllGather");
}

int msckf_rccl_count(const msckf_rccl_t* c, int* count_out, int* rank_out) {
    if (!c || !c->comm) RFAIL(-1, "no communicator");
    int n = 0;
    ncclResult_t r = g_api.commCount(c->comm, &n);
    if (r != ncclSuccess) RFAIL(-4, "ncclCommCount: %s", rstr(r));
    if (count_out) *count_out = n;
    if (rank_out) *rank_out = c->rank;
    return 0;
}

int msckf_rccl_set_timeout(msckf_rccl_t* c, double timeout_s) {
    if (!c) RFAIL(-1, "no communicator");
    if (!(timeout_s > 0)) RFAIL(-1, "timeout %g s", timeout_s);
    c->timeout_s = timeout_s;
    return 0;
}

int msckf_rccl_destroy(msckf_rccl_t* c) {
    if (!c) return 0;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    int rc = 0;
    if (c->comm) {
        // A non-blocking communicator finishes its teardown asynchronously:
        // finalize it and poll until its outstanding operations are done
        // before destroying it and freeing the buffers they may still touch;
        // a teardown that errors or outlives the deadline is aborted instead.
        bool clean = false;
        if (g_api.commFinalize) {
            ncclResult_t r = g_api.commFinalize(c->comm);
            if (r == ncclSuccess || r == ncclInProgress) {
                const auto t0 = Clock::now();
                for (;;) {
                    ncclResult_t st = ncclSuccess;
                    if (g_api.commGetAsyncError(c->comm, &st) != ncclSuccess) break;
                    if (st == ncclSuccess) { clean = true; break; }
                    if (st != ncclInProgress) break;
                    if (std::chrono::duration<double>(Clock::now() - t0).count() > c->timeout_s) break;
                    std::this_thread::sleep_for(std::chrono::microseconds(50));
                }
            }
        } else {
            ncclResult_t st = ncclSuccess;   // no finalize: destroy only a quiescent communicator
            clean = g_api.commGetAsyncError(c->comm, &st) == ncclSuccess && st == ncclSuccess;
        }
        if (clean) {
            (void)g_api.commDestroy(c->comm);
        } else {
            (void)g_api.commAbort(c->comm);
            r_err = "communicator teardown did not complete: aborted";
            rc = -4;
        }
        c->comm = nullptr;
    }
    if (c->dbuf) (void)hipFree(c->dbuf);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return rc;
}

}  // extern "C"
