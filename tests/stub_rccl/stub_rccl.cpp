// stub_rccl.cpp — TEST INFRASTRUCTURE ONLY: a stand-in librccl for exercising
// libicgpu's native RCCL transport (ic_comm.hip RcclComm) with several ranks
// on ONE GPU, where real RCCL refuses two ranks of a communicator on the same
// device.  Loaded by the tests through ic_rccl_set_library(); never by the
// product.
//
// It exports the nccl* symbols RcclComm binds, with RCCL's types (rccl.h):
// ncclGetUniqueId, ncclCommInitRankConfig (blocking and non-blocking),
// ncclCommGetAsyncError, ncclCommDestroy, ncclCommAbort, ncclAllGather,
// ncclAllReduce (int32 sum), ncclSend / ncclRecv inside ncclGroupStart /
// ncclGroupEnd, ncclGetErrorString.  Every rank is a process; the ranks of a
// communicator meet in a POSIX shared-memory segment named by the unique id.
// A collective is performed when it is called: the caller's stream is
// synchronised, its payload copied device -> shared memory, the peers'
// payloads shared memory -> device (so the data path is host-staged, not
// xGMI; only the semantics are RCCL's).  Each rank owns an outbox of
// outbox bytes (32 MiB, or IC_STUB_RCCL_OUTBOX_MB, the same on every rank); a collective waits until every rank finished reading the
// previous one before it overwrites its outbox.
//
// Failures propagate as they would have to for the library's error paths to
// be testable: ncclCommAbort sets a flag every waiting peer sees
// (ncclRemoteError), and a waiting rank also notices a peer process that has
// died (kill(pid, 0)), or gives up after kWaitSeconds.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

namespace {

constexpr int kMaxRanks = 16;
constexpr size_t kOutboxDefault = 32ull << 20;   // bytes a rank may send per collective
constexpr double kWaitSeconds = 120.0;

struct Header {
    std::atomic<int> joined;
    std::atomic<int> aborted;
    int nranks;
    int pid[kMaxRanks];
    std::atomic<uint64_t> pub[kMaxRanks];    // collective seq whose payload this rank has published
    std::atomic<uint64_t> done[kMaxRanks];   // collective seq this rank has finished reading
    uint64_t off[kMaxRanks][kMaxRanks];      // [src][dst] payload offset in src's outbox (send/recv)
    uint64_t len[kMaxRanks][kMaxRanks];
};

}  // namespace

struct ncclComm {
    Header *h = nullptr;
    char *box = nullptr;   // outboxes, `outbox` bytes per rank
    size_t outbox = kOutboxDefault;
    size_t map_bytes = 0;
    int rank = 0, n = 0;
    uint64_t seq = 0;
    int blocking = 1;
    char name[64] = {0};
};

namespace {

struct Op {
    bool send;
    void *buf;
    size_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};
thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

void shm_name(const ncclUniqueId &id, char *out)
{
    snprintf(out, 64, "/icstub_%.40s", id.internal + 8);
}

// a peer process that is gone, or a zombie its parent has not reaped yet
bool peer_dead(const Header *h, int p)
{
    const int pid = h->pid[p];
    if (pid <= 0) return false;
    if (kill(pid, 0) != 0 && errno == ESRCH) return true;
    char path[64], buf[256];
    snprintf(path, sizeof path, "/proc/%d/stat", pid);
    FILE *f = fopen(path, "r");
    if (!f) return true;
    const size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *rp = strrchr(buf, ')');   // "pid (comm) S ..."
    return rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X');
}

// wait until pred() holds; ncclRemoteError on abort, a dead peer or the time limit
template <typename Pred>
ncclResult_t wait_for(ncclComm_t c, Pred pred)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
        if (c->h->aborted.load(std::memory_order_acquire)) return ncclRemoteError;
        if (pred()) return ncclSuccess;
        if ((it & 1023) == 1023) {
            for (int p = 0; p < c->n; ++p)
                if (p != c->rank && peer_dead(c->h, p)) {
                    c->h->aborted.store(1, std::memory_order_release);
                    return ncclRemoteError;
                }
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (dt > kWaitSeconds) return ncclRemoteError;
        }
        if (it > 4096) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

// one collective: publish this rank's payload(s) for seq, then read the peers'
ncclResult_t begin(ncclComm_t c, hipStream_t st, uint64_t *seq)
{
    if (!c || !c->h) return ncclInvalidArgument;
    if (hipStreamSynchronize(st) != hipSuccess) return ncclUnhandledCudaError;
    *seq = ++c->seq;
    // every rank has read the previous collective's outboxes
    return wait_for(c, [&] {
        for (int p = 0; p < c->n; ++p)
            if (c->h->done[p].load(std::memory_order_acquire) + 1 < *seq) return false;
        return true;
    });
}

ncclResult_t publish(ncclComm_t c, uint64_t seq)
{
    c->h->pub[c->rank].store(seq, std::memory_order_release);
    return ncclSuccess;
}

ncclResult_t await_pub(ncclComm_t c, int p, uint64_t seq)
{
    return wait_for(c, [&] { return c->h->pub[p].load(std::memory_order_acquire) >= seq; });
}

void finish(ncclComm_t c, uint64_t seq) { c->h->done[c->rank].store(seq, std::memory_order_release); }

char *outbox(ncclComm_t c, int p) { return c->box + (size_t)p * c->outbox; }

size_t type_size(ncclDataType_t t)
{
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

ncclResult_t group_end_ops(std::vector<Op> &ops)
{
    if (ops.empty()) return ncclSuccess;
    ncclComm_t c = ops[0].comm;
    for (auto &o : ops)
        if (o.comm != c) return ncclInvalidUsage;   // one communicator per group here
    uint64_t seq;
    if (ncclResult_t r = begin(c, ops[0].stream, &seq)) return r;
    for (auto &o : ops)
        if (o.stream != ops[0].stream && hipStreamSynchronize(o.stream) != hipSuccess) return ncclUnhandledCudaError;
    size_t pos = 0;
    for (int d = 0; d < c->n; ++d) c->h->len[c->rank][d] = 0;
    for (auto &o : ops) {
        if (!o.send) continue;
        if (c->h->len[c->rank][o.peer] != 0) return ncclInvalidUsage;   // one send per peer per group
        if (pos + o.bytes > c->outbox) return ncclInvalidArgument;
        if (o.bytes && hipMemcpy(outbox(c, c->rank) + pos, o.buf, o.bytes, hipMemcpyDeviceToHost) != hipSuccess)
            return ncclUnhandledCudaError;
        c->h->off[c->rank][o.peer] = pos;
        c->h->len[c->rank][o.peer] = o.bytes;
        pos += o.bytes;
    }
    publish(c, seq);
    for (auto &o : ops) {
        if (o.send) continue;
        if (ncclResult_t r = await_pub(c, o.peer, seq)) return r;
        if (c->h->len[o.peer][c->rank] != o.bytes) return ncclInvalidUsage;
        if (o.bytes && hipMemcpy(o.buf, outbox(c, o.peer) + c->h->off[o.peer][c->rank], o.bytes,
                                 hipMemcpyHostToDevice) != hipSuccess)
            return ncclUnhandledCudaError;
    }
    finish(c, seq);
    return ncclSuccess;
}

}  // namespace

extern "C" {

const char *ncclGetErrorString(ncclResult_t r)
{
    switch (r) {
    case ncclSuccess: return "no error (stub)";
    case ncclUnhandledCudaError: return "unhandled HIP error (stub)";
    case ncclInvalidArgument: return "invalid argument (stub)";
    case ncclInvalidUsage: return "invalid usage (stub)";
    case ncclRemoteError: return "remote process exited, aborted or timed out (stub)";
    case ncclInProgress: return "in progress (stub)";
    default: return "stub RCCL error";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id)
{
    memset(id, 0, sizeof *id);
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    snprintf(id->internal, sizeof id->internal, "icstub: %d_%lld_%ld_%u", (int)getpid(), (long long)ts.tv_sec,
             ts.tv_nsec, (unsigned)rand());
    return ncclSuccess;
}

ncclResult_t ncclCommInitRankConfig(ncclComm_t *out, int nranks, ncclUniqueId id, int rank, ncclConfig_t *config)
{
    *out = nullptr;
    if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    if (strncmp(id.internal, "icstub: ", 8) != 0) return ncclInvalidArgument;
    auto *c = new ncclComm();
    c->rank = rank;
    c->n = nranks;
    c->blocking = config && config->blocking == 0 ? 0 : 1;
    shm_name(id, c->name);
    if (const char *mb = getenv("IC_STUB_RCCL_OUTBOX_MB")) {   // test stub only
        const long v = atol(mb);
        if (v > 0 && v <= 4096) c->outbox = (size_t)v << 20;
    }
    c->map_bytes = sizeof(Header) + (size_t)nranks * c->outbox;
    const int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        delete c;
        return ncclSystemError;
    }
    if (ftruncate(fd, (off_t)c->map_bytes) != 0) {
        close(fd);
        delete c;
        return ncclSystemError;
    }
    void *m = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        delete c;
        return ncclSystemError;
    }
    c->h = (Header *)m;
    c->box = (char *)m + sizeof(Header);
    c->h->pid[rank] = (int)getpid();
    c->h->nranks = nranks;
    c->h->joined.fetch_add(1, std::memory_order_acq_rel);
    *out = c;
    if (!c->blocking) return ncclInProgress;
    return wait_for(c, [&] { return c->h->joined.load(std::memory_order_acquire) >= nranks; });
}

ncclResult_t ncclCommInitRank(ncclComm_t *out, int nranks, ncclUniqueId id, int rank)
{
    return ncclCommInitRankConfig(out, nranks, id, rank, nullptr);
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t *state)
{
    if (!c || !c->h) return ncclInvalidArgument;
    if (c->h->aborted.load(std::memory_order_acquire)) {
        *state = ncclRemoteError;
        return ncclSuccess;
    }
    for (int p = 0; p < c->n; ++p)
        if (p != c->rank && peer_dead(c->h, p)) {
            *state = ncclRemoteError;
            return ncclSuccess;
        }
    *state = c->h->joined.load(std::memory_order_acquire) >= c->n ? ncclSuccess : ncclInProgress;
    return ncclSuccess;
}

static void release(ncclComm_t c)
{
    if (!c) return;
    if (c->h) {
        munmap(c->h, c->map_bytes);
        shm_unlink(c->name);   // the segment lives on while a peer still maps it
    }
    delete c;
}

ncclResult_t ncclCommAbort(ncclComm_t c)
{
    if (c && c->h) c->h->aborted.store(1, std::memory_order_release);
    release(c);
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c)
{
    release(c);
    return ncclSuccess;
}

ncclResult_t ncclGroupStart()
{
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd()
{
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    const ncclResult_t r = group_end_ops(ops);
    if (r != ncclSuccess) return r;
    return ops.empty() || ops[0].comm->blocking ? ncclSuccess : ncclInProgress;
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t st)
{
    if (!c || peer < 0 || peer >= c->n || type_size(t) == 0) return ncclInvalidArgument;
    Op o{true, const_cast<void *>(buf), count * type_size(t), peer, c, st};
    if (g_depth == 0) {
        std::vector<Op> one{o};
        return group_end_ops(one);
    }
    g_ops.push_back(o);
    return ncclSuccess;
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t st)
{
    if (!c || peer < 0 || peer >= c->n || type_size(t) == 0) return ncclInvalidArgument;
    Op o{false, buf, count * type_size(t), peer, c, st};
    if (g_depth == 0) {
        std::vector<Op> one{o};
        return group_end_ops(one);
    }
    g_ops.push_back(o);
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t, ncclComm_t c,
                           hipStream_t st)
{
    const size_t bytes = count * type_size(t);
    if (!c || bytes == 0 || bytes > c->outbox) return ncclInvalidArgument;
    uint64_t seq;
    if (ncclResult_t r = begin(c, st, &seq)) return r;
    if (hipMemcpy(outbox(c, c->rank), send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return ncclUnhandledCudaError;
    publish(c, seq);
    for (int p = 0; p < c->n; ++p) {
        if (ncclResult_t r = await_pub(c, p, seq)) return r;
        if (hipMemcpy((char *)recv + (size_t)p * bytes, outbox(c, p), bytes, hipMemcpyHostToDevice) != hipSuccess)
            return ncclUnhandledCudaError;
    }
    finish(c, seq);
    return c->blocking ? ncclSuccess : ncclInProgress;
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t c, hipStream_t st)
{
    if (!c || t != ncclInt32 || op != ncclSum) return ncclInvalidArgument;   // what RcclComm uses
    const size_t bytes = count * sizeof(int32_t);
    if (bytes == 0 || bytes > c->outbox) return ncclInvalidArgument;
    uint64_t seq;
    if (ncclResult_t r = begin(c, st, &seq)) return r;
    if (hipMemcpy(outbox(c, c->rank), send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return ncclUnhandledCudaError;
    publish(c, seq);
    std::vector<int32_t> acc(count, 0);
    for (int p = 0; p < c->n; ++p) {
        if (ncclResult_t r = await_pub(c, p, seq)) return r;
        const int32_t *v = (const int32_t *)outbox(c, p);
        for (size_t i = 0; i < count; ++i) acc[i] += v[i];
    }
    finish(c, seq);
    if (hipMemcpy(recv, acc.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return ncclUnhandledCudaError;
    return c->blocking ? ncclSuccess : ncclInProgress;
}

}  // extern "C"
