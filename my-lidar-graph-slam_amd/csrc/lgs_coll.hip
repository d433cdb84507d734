// lgs_coll.hip -- the loop batch's one collective.
//
// LoopDetectorRealTimeCorrelative::Detect's candidates are independent
// (C/mapping/loop_detector_real_time_correlative.cpp:38, :66), so with one
// process per GPU each rank matches a contiguous block of them and the only
// exchange is one all-gather of the fixed-size lgs_loop_result records over
// RCCL (xGMI between the GPUs of a node): the C++ counterpart of
// lgs_amd/loopbatch.run_sharded, so a multi-process C++ caller does not
// hand-roll ncclAllGather.
//
// RCCL is resolved at run time from the process (dlopen of librccl.so.1,
// preferring a copy that is already loaded -- e.g. torch's -- so that the
// communicator, the stream and the collective share one RCCL and one HIP
// runtime); the library has no link-time dependency on it.
#include "lgs_internal.hpp"

#include <dlfcn.h>

#include <cstring>
#include <mutex>

namespace {

// the subset of rccl.h used here (ABI-stable NCCL 2.x entry points)
typedef int ncclResult_t;
typedef void* ncclComm_t;
struct ncclUniqueId {
    char internal[128];
};
enum { kNcclUint8 = 1 };   // ncclDataType_t ncclUint8 / ncclChar

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        if (r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_gather) r.h = h;
    });
    if (!r.h) throw lgs::Error(LGS_ERR_INTERNAL, "RCCL (librccl.so.1) not found");
    return r;
}

void check_nccl(ncclResult_t rc, const char* what)
{
    if (rc == 0) return;
    const Rccl& r = rccl();
    std::string m = std::string(what) + ": " + (r.error_string ? r.error_string(rc) : "RCCL error");
    throw lgs::Error(LGS_ERR_INTERNAL, m);
}

}  // namespace

extern "C" int lgs_loop_shard_bounds(int n, int world, int rank, int* lo, int* hi)
{
    if (n < 0 || world < 1 || rank < 0 || rank >= world || !lo || !hi) return LGS_ERR_INVALID_ARG;
    const int base = n / world, rem = n % world;
    *lo = rank * base + (rank < rem ? rank : rem);
    *hi = *lo + base + (rank < rem ? 1 : 0);
    return LGS_OK;
}

extern "C" int lgs_rccl_unique_id(unsigned char* id128)
{
    if (!id128) return LGS_ERR_INVALID_ARG;
    try {
        ncclUniqueId u;
        check_nccl(rccl().get_unique_id(&u), "ncclGetUniqueId");
        std::memcpy(id128, u.internal, sizeof(u.internal));
        return LGS_OK;
    } catch (const lgs::Error& e) {
        return e.code;
    } catch (...) {
        return LGS_ERR_INTERNAL;
    }
}

extern "C" int lgs_rccl_comm_init(lgs_ctx* ctx, const unsigned char* id128, int world, int rank, void** comm)
{
    if (!ctx || !id128 || world < 1 || rank < 0 || rank >= world || !comm) return LGS_ERR_INVALID_ARG;
    using namespace lgs;
    return guarded(ctx, [&] {
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        ncclUniqueId u;
        std::memcpy(u.internal, id128, sizeof(u.internal));
        ncclComm_t c = nullptr;
        check_nccl(rccl().comm_init_rank(&c, world, u, rank), "ncclCommInitRank");
        *comm = c;
    });
}

extern "C" int lgs_rccl_comm_destroy(void* comm)
{
    if (!comm) return LGS_ERR_INVALID_ARG;
    try {
        check_nccl(rccl().comm_destroy((ncclComm_t)comm), "ncclCommDestroy");
        return LGS_OK;
    } catch (const lgs::Error& e) {
        return e.code;
    } catch (...) {
        return LGS_ERR_INTERNAL;
    }
}

extern "C" int lgs_loop_records_allgather(lgs_ctx* ctx, void* comm, int rank, int world, int n,
                                          const lgs_loop_result* local, lgs_loop_result* all)
{
    if (!ctx || !comm || world < 1 || rank < 0 || rank >= world || n < 0 || (n > 0 && !all)) return LGS_ERR_INVALID_ARG;
    using namespace lgs;
    return guarded(ctx, [&] {
        int lo = 0, hi = 0, rows = 0, z = 0;
        lgs_loop_shard_bounds(n, world, rank, &lo, &hi);
        lgs_loop_shard_bounds(n, world, 0, &z, &rows);   // the largest block: rank 0's
        LGS_REQUIRE(hi == lo || local, "local records missing");
        if (n == 0) return;
        LGS_HIP_CHECK(hipSetDevice(ctx->device));
        const size_t rb = sizeof(lgs_loop_result) * (size_t)rows;
        // [send block | world gathered blocks], each padded to the largest block
        char* d = (char*)ctx->ensure(S_COLL, rb * (size_t)(world + 1));
        char* h = (char*)ctx->ensure_pinned(rb * (size_t)world);
        if (hi > lo) std::memcpy(h, local, sizeof(lgs_loop_result) * (size_t)(hi - lo));
        LGS_HIP_CHECK(hipMemcpyAsync(d, h, rb, hipMemcpyHostToDevice, ctx->stream));
        check_nccl(rccl().all_gather(d, d + rb, rb, kNcclUint8, (ncclComm_t)comm, ctx->stream), "ncclAllGather");
        LGS_HIP_CHECK(hipMemcpyAsync(h, d + rb, rb * (size_t)world, hipMemcpyDeviceToHost, ctx->stream));
        ctx->sync();
        // every rank's block, in candidate order (the padding rows dropped)
        for (int r = 0; r < world; ++r) {
            int a = 0, b = 0;
            lgs_loop_shard_bounds(n, world, r, &a, &b);
            if (b > a) std::memcpy(all + a, h + rb * (size_t)r, sizeof(lgs_loop_result) * (size_t)(b - a));
        }
    });
}
