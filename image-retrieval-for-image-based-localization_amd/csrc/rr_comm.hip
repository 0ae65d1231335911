// librr.so — RCCL entry points for a non-Python host of the sharded search.
//
// The Python host shards the database with torch.distributed (ShardedIndex,
// cirtorch/search.py); a C / C++ / Go host of librr.so gets the same exchange
// here: one RCCL communicator per rank (one process per GPU), the per-shard
// top-k lists all-gathered over xGMI, then the on-GPU (score desc, index asc)
// merge, so the result is bit-identical to a 1-GPU search of the whole
// database.  Replaces the reference's missing gather of per-rank descriptors
// / rankings (scripts/train_globalF.py:667-730).
//
// RCCL is opened with dlopen on first use: librr.so links no collective
// library, and in a PyTorch process the RCCL PyTorch already loaded is reused.
#include "rr_internal.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

namespace rr {
namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) return;
        r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
        r.ok = r.get_id && r.init_rank && r.destroy && r.all_gather && r.group_start && r.group_end && r.err;
    });
    return r;
}

int nccl_fail(const char* what, ncclResult_t e) {
    static thread_local char msg[256];
    snprintf(msg, sizeof msg, "%s: %s", what, rccl().err ? rccl().err(e) : "RCCL error");
    return fail(RR_EINVAL, msg);
}

struct Comm {
    ncclComm_t c;
    int nranks, rank;
};

size_t merge_ws(int nranks, int nq, int k) {
    const size_t s = ((size_t)nranks * nq * k * 8 + 255) / 256 * 256;
    return 2 * s;  // gathered scores (f64) + gathered indices (i64)
}

}  // namespace
}  // namespace rr

using namespace rr;

extern "C" {

int rr_comm_unique_id(void* id_out, int id_bytes) {
    if (!id_out || id_bytes < (int)sizeof(ncclUniqueId)) return fail(RR_EINVAL, "rr_comm_unique_id: id buffer < 128 bytes");
    if (!rccl().ok) return fail(RR_EINVAL, "rr_comm_unique_id: RCCL (librccl.so.1) not found");
    ncclUniqueId id;
    const ncclResult_t e = rccl().get_id(&id);
    if (e != ncclSuccess) return nccl_fail("rr_comm_unique_id", e);
    memcpy(id_out, &id, sizeof id);
    return RR_OK;
}

int rr_comm_init(void** comm, int nranks, const void* id, int id_bytes, int rank) {
    if (!comm || !id || id_bytes < (int)sizeof(ncclUniqueId)) return fail(RR_EINVAL, "rr_comm_init: null / short id");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(RR_EINVAL, "rr_comm_init: rank out of range");
    if (!rccl().ok) return fail(RR_EINVAL, "rr_comm_init: RCCL (librccl.so.1) not found");
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    Comm* c = new Comm{nullptr, nranks, rank};
    const ncclResult_t e = rccl().init_rank(&c->c, nranks, uid, rank);  // device = the calling thread's current one
    if (e != ncclSuccess) {
        delete c;
        return nccl_fail("rr_comm_init", e);
    }
    *comm = c;
    return RR_OK;
}

int rr_comm_destroy(void* comm) {
    if (!comm) return RR_OK;
    Comm* c = (Comm*)comm;
    const ncclResult_t e = rccl().destroy(c->c);
    delete c;
    return e == ncclSuccess ? RR_OK : nccl_fail("rr_comm_destroy", e);
}

size_t rr_topk_allgather_workspace_bytes(int nranks, int nq, int k) {
    if (nranks < 1 || nq < 1 || k < 1) return 0;
    return merge_ws(nranks, nq, k);
}

int rr_topk_allgather_merge(void* comm, const double* scores, const long long* idx, int nq, int k,
                            double* out_scores, long long* out_idx, void* workspace, size_t workspace_bytes,
                            void* stream) {
    if (!comm || !scores || !idx || !out_scores || !out_idx || !workspace)
        return fail(RR_EINVAL, "rr_topk_allgather_merge: null pointer");
    if (nq < 1 || k < 1) return fail(RR_EINVAL, "rr_topk_allgather_merge: empty");
    Comm* c = (Comm*)comm;
    if (workspace_bytes < merge_ws(c->nranks, nq, k)) return fail(RR_ENOSPACE, "rr_topk_allgather_merge: workspace");
    const size_t half = merge_ws(c->nranks, nq, k) / 2;
    double* gs = (double*)workspace;
    long long* gi = (long long*)((char*)workspace + half);
    hipStream_t s = as_stream(stream);
    const size_t cnt = (size_t)nq * k;
    ncclResult_t e = rccl().group_start();
    if (e == ncclSuccess) e = rccl().all_gather(scores, gs, cnt, ncclFloat64, c->c, s);
    if (e == ncclSuccess) e = rccl().all_gather(idx, gi, cnt, ncclInt64, c->c, s);
    const ncclResult_t e2 = rccl().group_end();
    if (e != ncclSuccess) return nccl_fail("rr_topk_allgather_merge: all-gather", e);
    if (e2 != ncclSuccess) return nccl_fail("rr_topk_allgather_merge: group", e2);
    return rr_topk_merge(gs, gi, c->nranks, nq, k, k, out_scores, out_idx, stream);
}

}  // extern "C"
