// qpb_comm.hip -- the one collective of the path (SURVEY §8b last row, §8e):
// the multi-GPU argmin gather over RCCL (xGMI within a node).
//
// QPs are independent, so each rank solves its shard and reduces it to its own
// winner on the device (qpb_solve_best).  qpb_argmin_allgather then
//   1. builds the rank's payload {fval, global index, x*[n]} on the device,
//   2. ncclAllGather's the 16 + 8n bytes of every rank (112 B for C1),
//   3. reduces the gathered payloads on the device to the global winner,
// all stream-ordered on the caller's stream, no host round trip.  RCCL is loaded
// lazily with dlopen (librccl.so.1: the copy a host process already loaded, e.g.
// torch's, else ROCm's), so the library keeps no link-time dependency on it and
// single-GPU users never touch it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "../../include/qpswift_hip.h"
#include "qpb_runtime.hpp"

namespace {

struct Rccl {
    void *h = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*commCount)(const ncclComm_t, int *) = nullptr;
    ncclResult_t (*allGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char *(*errStr)(ncclResult_t) = nullptr;
    std::string err;
};

const Rccl &rccl() {
    static Rccl r = [] {
        Rccl x;
        for (const char *name : {"librccl.so.1", "librccl.so"}) {
            if ((x.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
        }
        if (!x.h) {
            const char *rp = getenv("ROCM_PATH");
            const std::string p = std::string(rp && *rp ? rp : "/opt/rocm") + "/lib/librccl.so.1";
            x.h = dlopen(p.c_str(), RTLD_NOW | RTLD_GLOBAL);
        }
        if (!x.h) { x.err = std::string("cannot load librccl: ") + dlerror(); return x; }
        auto sym = [&](const char *s) { return dlsym(x.h, s); };
        x.getUniqueId = (decltype(x.getUniqueId))sym("ncclGetUniqueId");
        x.commInitRank = (decltype(x.commInitRank))sym("ncclCommInitRank");
        x.commDestroy = (decltype(x.commDestroy))sym("ncclCommDestroy");
        x.commCount = (decltype(x.commCount))sym("ncclCommCount");
        x.allGather = (decltype(x.allGather))sym("ncclAllGather");
        x.errStr = (decltype(x.errStr))sym("ncclGetErrorString");
        if (!x.getUniqueId || !x.commInitRank || !x.commDestroy || !x.commCount || !x.allGather || !x.errStr)
            x.err = "librccl lacks an expected symbol";
        return x;
    }();
    return r;
}

int rccl_fail(ncclResult_t rc, const char *what) {
    return qpb::set_error(QPB_EHIP, (std::string(what) + ": " + rccl().errStr(rc)).c_str());
}

__device__ __forceinline__ bool better(double va, double ia, double vb, double ib) {
    return ia >= 0 && (ib < 0 || va < vb || (va == vb && ia < ib));
}

// payload of this rank: {fval, base + index, x*[0..n)} from the tiled x (NaN x
// and index -1 when the shard has no optimal QP)
__global__ void __launch_bounds__(64) qpb_payload_k(const double *__restrict__ best, const double *__restrict__ x,
                                                    long n, long B, long base, double *__restrict__ out) {
    const double fv = best[0];
    const long q = (long)best[1];
    const bool ok = q >= 0 && q < B;
    if (threadIdx.x == 0) { out[0] = ok ? fv : INFINITY; out[1] = ok ? (double)(base + q) : -1.0; }
    for (long j = threadIdx.x; j < n; j += 64)
        out[2 + j] = ok ? x[(q >> 6) * n * 64 + j * 64 + (q & 63)] : __builtin_nan("");
}

// global winner over `world` gathered payloads of width 2 + n: lowest fval,
// ties -> lowest global index; the winner's payload is copied to out
__global__ void __launch_bounds__(64) qpb_payload_reduce_k(const double *__restrict__ g, long world, long n,
                                                           double *__restrict__ out) {
    const long w = 2 + n;
    double bv = INFINITY, bi = -1.0;
    long br = -1;
    for (long r = threadIdx.x; r < world; r += 64)
        if (better(g[r * w], g[r * w + 1], bv, bi)) { bv = g[r * w]; bi = g[r * w + 1]; br = r; }
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(bv, off, 64), oi = __shfl_xor(bi, off, 64);
        const long orr = __shfl_xor(br, off, 64);
        if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; br = orr; }
    }
    if (threadIdx.x == 0) { out[0] = bv; out[1] = bi; }
    for (long j = threadIdx.x; j < n; j += 64) out[2 + j] = br >= 0 ? g[br * w + 2 + j] : __builtin_nan("");
}

std::mutex g_mu;
// (comm, stream, n) -> device scratch: send payload | gathered payloads
std::map<std::tuple<void *, void *, long>, std::pair<double *, long>> g_scratch;

}  // namespace

extern "C" {

int qpb_comm_get_unique_id(void *id) {
    if (!id) return qpb::set_error(QPB_EINVAL, "NULL id");
    const Rccl &r = rccl();
    if (!r.err.empty()) return qpb::set_error(QPB_EHIP, r.err.c_str());
    ncclUniqueId u;
    ncclResult_t rc = r.getUniqueId(&u);
    if (rc != ncclSuccess) return rccl_fail(rc, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof u);
    return QPB_OK;
}

int qpb_comm_init(void **comm, int nranks, const void *id, int rank) {
    if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return qpb::set_error(QPB_EINVAL, "bad comm arguments");
    *comm = nullptr;
    const Rccl &r = rccl();
    if (!r.err.empty()) return qpb::set_error(QPB_EHIP, r.err.c_str());
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclComm_t c = nullptr;
    ncclResult_t rc = r.commInitRank(&c, nranks, u, rank);
    if (rc != ncclSuccess) return rccl_fail(rc, "ncclCommInitRank");
    *comm = c;
    return QPB_OK;
}

int qpb_comm_count(void *comm, int *nranks) {
    if (!comm || !nranks) return qpb::set_error(QPB_EINVAL, "NULL comm / nranks");
    const Rccl &r = rccl();
    if (!r.err.empty()) return qpb::set_error(QPB_EHIP, r.err.c_str());
    ncclResult_t rc = r.commCount((ncclComm_t)comm, nranks);
    if (rc != ncclSuccess) return rccl_fail(rc, "ncclCommCount");
    return QPB_OK;
}

void qpb_comm_destroy(void *comm) {
    if (!comm) return;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (auto it = g_scratch.begin(); it != g_scratch.end();) {
            if (std::get<0>(it->first) == comm) {
                (void)hipStreamSynchronize((hipStream_t)std::get<1>(it->first));
                (void)hipFree(it->second.first);
                it = g_scratch.erase(it);
            } else {
                ++it;
            }
        }
    }
    rccl().commDestroy((ncclComm_t)comm);
}

int qpb_argmin_reduce(const double *gathered, long world, long n, double *out, void *stream) {
    if (!gathered || !out || world < 1 || n < 0) return qpb::set_error(QPB_EINVAL, "bad argmin reduce arguments");
    (void)hipGetLastError();   // a stale error of an earlier API call is not this launch's
    hipLaunchKernelGGL(qpb_payload_reduce_k, dim3(1), dim3(64), 0, (hipStream_t)stream, gathered, world, n, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qpb::set_error(QPB_EHIP, hipGetErrorString(e));
    return QPB_OK;
}

int qpb_argmin_allgather(const double *best, const double *x, long n, long B, long base, void *comm, double *out,
                         void *stream) {
    if (!best || !out || !comm || n < 0 || B < 0 || base < 0 || (n > 0 && B > 0 && !x))
        return qpb::set_error(QPB_EINVAL, "bad argmin_allgather arguments");
    const Rccl &r = rccl();
    if (!r.err.empty()) return qpb::set_error(QPB_EHIP, r.err.c_str());
    int world = 0;
    ncclResult_t rc = r.commCount((ncclComm_t)comm, &world);
    if (rc != ncclSuccess) return rccl_fail(rc, "ncclCommCount");
    const long w = 2 + n;
    double *buf = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto &sc = g_scratch[std::make_tuple(comm, stream, n)];
        const long need = w * (1 + (long)world);
        if (sc.second < need) {
            if (sc.first) {
                (void)hipStreamSynchronize((hipStream_t)stream);
                (void)hipFree(sc.first);
            }
            sc = {nullptr, 0};
            if (hipMalloc((void **)&sc.first, sizeof(double) * (size_t)need) != hipSuccess)
                return qpb::set_error(QPB_ENOMEM, "argmin_allgather scratch");
            sc.second = need;
        }
        buf = sc.first;
    }
    double *send = buf, *recv = buf + w;
    (void)hipGetLastError();   // a stale error of an earlier API call is not this launch's
    hipLaunchKernelGGL(qpb_payload_k, dim3(1), dim3(64), 0, (hipStream_t)stream, best, x, n, B, base, send);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return qpb::set_error(QPB_EHIP, hipGetErrorString(e));
    rc = r.allGather(send, recv, (size_t)w, ncclDouble, (ncclComm_t)comm, (hipStream_t)stream);
    if (rc != ncclSuccess) return rccl_fail(rc, "ncclAllGather");
    return qpb_argmin_reduce(recv, world, n, out, stream);
}

}  // extern "C"
