// ic_comm.hip — shard exchange transports (see ic_comm.h).
#include <dlfcn.h>
#include <string.h>

#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ic_comm.h"
#include "ic_internal.h"

namespace icgpu {

// ------------------------------------------------------------ host callbacks

class CallbackComm final : public Comm {
public:
    explicit CallbackComm(const ic_comm_ops &o) : ops(o) {}
    int alloc(void **p, size_t bytes) override { return ops.alloc(ops.ctx, bytes, p); }
    void release(void *p) override
    {
        if (p) (void)ops.release(ops.ctx, p);
    }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t st) override
    {
        return ops.allgather(ops.ctx, send, recv, bytes, (void *)st);
    }
    int alltoallv(const void *send, const size_t *sb, void *recv, const size_t *rb, hipStream_t st) override
    {
        return ops.alltoallv(ops.ctx, send, sb, recv, rb, (void *)st);
    }
    int allreduce_sum_i32(int32_t *buf, size_t n, hipStream_t st) override
    {
        return ops.allreduce_sum_i32(ops.ctx, buf, n, (void *)st);
    }

private:
    ic_comm_ops ops;
};

Comm *make_callback_comm(const ic_comm_ops &ops, int rank, int world)
{
    auto *c = new CallbackComm(ops);
    c->rank = rank;
    c->world = world;
    return c;
}

// ------------------------------------------------------------ in-process group

struct LocalGroup {
    struct Slot {
        const void *send = nullptr;
        const size_t *sb = nullptr;   // nullptr: all-gather (the same `send` for every peer)
        hipEvent_t ready = nullptr;   // send buffer written (recorded on the owner's stream)
        hipEvent_t done = nullptr;    // the owner has read every peer's send buffer
        int device = 0;
        bool taken = false;
    };
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    unsigned long long gen = 0;
    bool aborted = false;
    Slot slot[kMaxShards];

    // all `world` threads meet; -1 if a shard aborted or nobody came for 10 min
    int barrier()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return -1;
        const unsigned long long g0 = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return 0;
        }
        const bool ok = cv.wait_for(lk, std::chrono::minutes(10), [&] { return gen != g0 || aborted; });
        if (gen != g0) return 0;
        if (!ok) aborted = true;
        cv.notify_all();
        return -1;
    }
    void abort()
    {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

LocalGroup *local_group_create(int world)
{
    if (world < 1 || world > kMaxShards) return nullptr;
    auto *g = new LocalGroup();
    g->world = world;
    return g;
}

void local_group_destroy(LocalGroup *g) { delete g; }

int local_group_world(const LocalGroup *g) { return g ? g->world : 0; }

class LocalComm final : public Comm {
public:
    LocalComm(LocalGroup *g_, int r, int dev) : g(g_), device(dev)
    {
        rank = r;
        world = g_->world;
    }
    ~LocalComm() override
    {
        auto &me = g->slot[rank];
        if (me.ready) (void)hipEventDestroy(me.ready);
        if (me.done) (void)hipEventDestroy(me.done);
        if (tmp) (void)hipFree(tmp);
        std::lock_guard<std::mutex> lk(g->mu);
        me = LocalGroup::Slot();
    }
    int init()
    {
        auto &me = g->slot[rank];
        me.device = device;
        if (hipEventCreateWithFlags(&me.ready, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&me.done, hipEventDisableTiming) != hipSuccess) return -1;
        return 0;
    }
    int alloc(void **p, size_t bytes) override { return hipMalloc(p, bytes ? bytes : 8) == hipSuccess ? 0 : -1; }
    void release(void *p) override
    {
        if (p) (void)hipFree(p);
    }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t st) override
    {
        return exchange(send, nullptr, recv, nullptr, bytes, st);
    }
    int alltoallv(const void *send, const size_t *sb, void *recv, const size_t *rb, hipStream_t st) override
    {
        return exchange(send, sb, recv, rb, 0, st);
    }
    int allreduce_sum_i32(int32_t *buf, size_t n, hipStream_t st) override
    {
        if (n * world > tmp_n) {
            if (tmp) (void)hipFree(tmp);
            tmp = nullptr;
            tmp_n = 0;
            if (hipMalloc(&tmp, sizeof(int32_t) * n * world) != hipSuccess) return -1;
            tmp_n = n * world;
        }
        if (int rc = exchange(buf, nullptr, tmp, nullptr, sizeof(int32_t) * n, st)) return rc;
        return launch_sum_i32(st, tmp, world, (int)n, buf) == hipSuccess ? 0 : -1;
    }
    void abort() override { g->abort(); }

private:
    LocalGroup *g;
    int device;
    int32_t *tmp = nullptr;
    size_t tmp_n = 0;
    unsigned long long peer_on = 0;   // devices whose peer access this shard enabled

    int copy(void *dst, const void *src, size_t bytes, int src_dev, hipStream_t st)
    {
        if (!bytes) return 0;
        if (src_dev != device && src_dev < 64 && !((peer_on >> src_dev) & 1ull)) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, device, src_dev) == hipSuccess && can)
                (void)hipDeviceEnablePeerAccess(src_dev, 0);
            (void)hipGetLastError();   // "already enabled" is fine
            peer_on |= 1ull << src_dev;
        }
        const hipError_t e = src_dev == device
                                 ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st)
                                 : hipMemcpyPeerAsync(dst, device, src, src_dev, bytes, st);
        return e == hipSuccess ? 0 : -1;
    }

    // sb == nullptr: all-gather of gbytes; else all-to-all with per-peer sizes.
    // Any failure aborts the group so that no peer waits for this shard.
    int exchange(const void *send, const size_t *sb, void *recv, const size_t *rb, size_t gbytes, hipStream_t st)
    {
        const int rc = exchange_(send, sb, recv, rb, gbytes, st);
        if (rc) g->abort();
        return rc;
    }
    int exchange_(const void *send, const size_t *sb, void *recv, const size_t *rb, size_t gbytes, hipStream_t st)
    {
        auto &me = g->slot[rank];
        me.send = send;
        me.sb = sb;
        if (hipEventRecord(me.ready, st) != hipSuccess) return -1;
        if (g->barrier()) return -2;
        size_t doff = 0;
        for (int p = 0; p < world; ++p) {
            const auto &ps = g->slot[p];
            size_t bytes, soff = 0;
            char *dst;
            if (!sb) {
                bytes = gbytes;
                dst = (char *)recv + (size_t)p * gbytes;
            } else {
                if (!ps.sb) return -3;          // peer is in a different collective
                bytes = ps.sb[rank];
                for (int q = 0; q < rank; ++q) soff += ps.sb[q];
                if (bytes != rb[p]) return -3;  // inconsistent block sizes
                dst = (char *)recv + doff;
                doff += rb[p];
            }
            if (!bytes) continue;
            if (p != rank && hipStreamWaitEvent(st, ps.ready, 0) != hipSuccess) return -1;
            if (copy(dst, (const char *)ps.send + soff, bytes, ps.device, st)) return -1;
        }
        if (hipEventRecord(me.done, st) != hipSuccess) return -1;
        if (g->barrier()) return -2;
        // nobody may overwrite its send buffer before every peer has copied it
        for (int p = 0; p < world; ++p)
            if (p != rank && hipStreamWaitEvent(st, g->slot[p].done, 0) != hipSuccess) return -1;
        return 0;
    }

    friend Comm *make_local_comm(LocalGroup *, int, int, const char **);
};

Comm *make_local_comm(LocalGroup *g, int rank, int device, const char **err)
{
    if (!g || rank < 0 || rank >= g->world) {
        *err = "rank out of range for the group";
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->slot[rank].taken) {
            *err = "rank already has a session in this group";
            return nullptr;
        }
        g->slot[rank].taken = true;
    }
    auto *c = new LocalComm(g, rank, device);
    if (c->init()) {
        delete c;
        *err = "hipEventCreate failed";
        return nullptr;
    }
    return c;
}

// ------------------------------------------------------------ native RCCL

// librccl is opened on first use (dlopen, RTLD_LOCAL): a process that never
// asks for the native transport never loads it, and torch's own bundled RCCL,
// if loaded, stays a separate instance.  The ROCm install's copy by default;
// ic_rccl_set_library() names another file first (a test stub, another RCCL
// build).  Types and the config layout come from ROCm's rccl.h; no symbol is
// linked.
namespace {
struct RcclApi {
    void *h = nullptr;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRankConfig)(ncclComm_t *, int, ncclUniqueId, int, ncclConfig_t *) = nullptr;
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
RcclApi g_api;
bool g_api_tried = false;
std::string g_rccl_path;                 // ic_rccl_set_library ("" = the ROCm install's)
long long g_init_timeout_ms = 600000;    // ic_rccl_set_init_timeout

RcclApi *rccl_api(std::string *err)
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_api_tried) {
        g_api_tried = true;
        std::vector<std::string> paths;
        if (!g_rccl_path.empty())
            paths.push_back(g_rccl_path);
        else
            paths = {"/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"};
        // dlerror() clears its message: read it once per failed dlopen, and
        // report every file tried with its own reason
        std::string why;
        for (const auto &p : paths) {
            if ((g_api.h = dlopen(p.c_str(), RTLD_NOW | RTLD_LOCAL))) break;
            const char *de = dlerror();
            why += (why.empty() ? "" : "; ") + p + ": " + (de ? de : "?");
        }
        if (!g_api.h) {
            g_api.err = "dlopen failed (" + why + ")";
        } else {
#define SYM(F)                                                   \
    if (g_api.err.empty()) {                                     \
        *(void **)(&g_api.F) = dlsym(g_api.h, "nccl" #F);        \
        if (!g_api.F) g_api.err = "librccl lacks nccl" #F;       \
    }
            SYM(GetUniqueId) SYM(CommInitRankConfig) SYM(CommGetAsyncError) SYM(CommDestroy) SYM(CommAbort)
            SYM(AllGather) SYM(AllReduce) SYM(Send) SYM(Recv) SYM(GroupStart) SYM(GroupEnd) SYM(GetErrorString)
#undef SYM
        }
    }
    if (!g_api.err.empty()) {
        *err = "librccl unavailable: " + g_api.err;
        return nullptr;
    }
    return &g_api;
}
}  // namespace

int rccl_set_library(const char *path, const char **err)
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    const std::string p = path ? path : "";
    if (g_api_tried && p != g_rccl_path) {
        *err = "librccl was already loaded by this process (ic_rccl_set_library must come first)";
        return -1;
    }
    g_rccl_path = p;
    return 0;
}

int rccl_set_init_timeout(long long ms, const char **err)
{
    if (ms < 1) {
        *err = "the RCCL init timeout must be >= 1 ms";
        return -1;
    }
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    g_init_timeout_ms = ms;
    return 0;
}

int rccl_unique_id(void *id, std::string *err)
{
    RcclApi *a = rccl_api(err);
    if (!a) return -1;
    ncclUniqueId u;
    const ncclResult_t rc = a->GetUniqueId(&u);
    if (rc != ncclSuccess) {
        *err = a->GetErrorString(rc);
        return -1;
    }
    static_assert(sizeof u == 128, "ncclUniqueId is 128 bytes");
    memcpy(id, &u, sizeof u);
    return 0;
}

// One RCCL communicator per shard session, on the session's device; every
// exchange is issued from here on the session stream (no host callbacks):
// all-gathers and the counter all-reduce as RCCL collectives, the all-to-alls
// as one group of per-peer sends and receives.  The communicator is
// non-blocking (config.blocking = 0): its creation is polled under a timeout,
// so a rank that never joins (it failed before creating its session) makes
// its peers' creation fail instead of blocking them forever, and a call that
// returns ncclInProgress is settled by polling ncclCommGetAsyncError.
class RcclComm final : public Comm {
public:
    ~RcclComm() override
    {
        if (comm) {
            if (aborted)
                (void)api->CommAbort(comm);
            else
                (void)api->CommDestroy(comm);
        }
    }
    int alloc(void **p, size_t bytes) override { return hipMalloc(p, bytes ? bytes : 8) == hipSuccess ? 0 : -1; }
    void release(void *p) override
    {
        if (p) (void)hipFree(p);
    }
    int allgather(const void *send, void *recv, size_t bytes, hipStream_t st) override
    {
        if (!comm) return -1;
        return check(api->AllGather(send, recv, bytes, ncclUint8, comm, st));
    }
    int alltoallv(const void *send, const size_t *sb, void *recv, const size_t *rb, hipStream_t st) override
    {
        if (!comm) return -1;
        if (settle(api->GroupStart()) != ncclSuccess) return check(ncclInternalError);
        // inside a group a non-blocking communicator may report ncclInProgress
        // for a queued call: that is not a failure, and every peer's send and
        // receive must still join the group (a short group would deadlock)
        auto queued = [](ncclResult_t r) { return r == ncclSuccess || r == ncclInProgress; };
        size_t so = 0, ro = 0;
        ncclResult_t rc = ncclSuccess;
        for (int p = 0; p < world && queued(rc); ++p) {
            if (sb[p]) rc = api->Send((const char *)send + so, sb[p], ncclUint8, p, comm, st);
            if (queued(rc) && rb[p]) rc = api->Recv((char *)recv + ro, rb[p], ncclUint8, p, comm, st);
            so += sb[p];
            ro += rb[p];
        }
        const ncclResult_t rc2 = api->GroupEnd();
        return check(rc != ncclSuccess && rc != ncclInProgress ? rc : rc2);
    }
    int allreduce_sum_i32(int32_t *buf, size_t n, hipStream_t st) override
    {
        if (!comm) return -1;
        return check(api->AllReduce(buf, buf, n, ncclInt32, ncclSum, comm, st));
    }
    void abort() override
    {
        if (comm && !aborted) {
            aborted = true;
            (void)api->CommAbort(comm);
            comm = nullptr;
        }
    }
    // a failure RCCL detected asynchronously (a peer's connection lost): the
    // session's host waits poll this between their event queries
    void set_timeout_ms(long long ms) override { timeout_ms = ms; }
    bool remote_error() override
    {
        if (!comm) return aborted;
        ncclResult_t st = ncclSuccess;
        if (api->CommGetAsyncError(comm, &st) != ncclSuccess) return true;
        return st != ncclSuccess && st != ncclInProgress;
    }

private:
    RcclApi *api = nullptr;
    ncclComm_t comm = nullptr;
    bool aborted = false;
    long long timeout_ms = 600000;
    // a non-blocking communicator's call may return ncclInProgress: wait for
    // its state to settle.  Enqueueing takes microseconds, but a grouped
    // send / receive may stay in progress until its peer reaches the same
    // exchange, so the wait is bounded by the session's own host-wait limit
    // (IC_OPT_SYNC_TIMEOUT_MS, set_timeout_ms), not by a fixed figure.
    ncclResult_t settle(ncclResult_t rc)
    {
        if (rc != ncclInProgress) return rc;
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            ncclResult_t st = ncclSuccess;
            if (api->CommGetAsyncError(comm, &st) != ncclSuccess) return ncclInternalError;
            if (st != ncclInProgress) return st;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms))
                return ncclInternalError;
            std::this_thread::yield();
        }
    }
    int check(ncclResult_t rc)
    {
        rc = settle(rc);
        if (rc != ncclSuccess) abort();
        return rc == ncclSuccess ? 0 : -1;
    }
    friend Comm *make_rccl_comm(const void *, int, int, std::string *);
};

Comm *make_rccl_comm(const void *unique_id, int rank, int world, std::string *err)
{
    RcclApi *a = rccl_api(err);
    if (!a) return nullptr;
    long long timeout_ms;
    {
        std::lock_guard<std::mutex> lk(g_rccl_mu);
        timeout_ms = g_init_timeout_ms;
    }
    ncclUniqueId u;
    memcpy(&u, unique_id, sizeof u);
    auto *c = new RcclComm();
    c->api = a;
    c->rank = rank;
    c->world = world;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t rc = a->CommInitRankConfig(&c->comm, world, u, rank, &cfg);   // on the current (session) device
    if (rc != ncclSuccess && rc != ncclInProgress) {
        *err = std::string("ncclCommInitRankConfig: ") + a->GetErrorString(rc);
        if (c->comm) (void)a->CommAbort(c->comm);
        c->comm = nullptr;
        delete c;
        return nullptr;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        rc = a->CommGetAsyncError(c->comm, &st);
        if (rc == ncclSuccess && st == ncclSuccess) break;
        const bool timed_out = std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms);
        if (rc != ncclSuccess || st != ncclInProgress || timed_out) {
            *err = timed_out ? "RCCL communicator init timed out (a rank did not join; ic_rccl_set_init_timeout)"
                             : std::string("RCCL communicator init: ") + a->GetErrorString(rc != ncclSuccess ? rc : st);
            (void)a->CommAbort(c->comm);
            c->comm = nullptr;
            delete c;
            return nullptr;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    return c;
}

}  // namespace icgpu
