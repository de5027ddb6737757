// ic_comm.h — shard exchange transports of libicgpu.so (not part of the C-ABI).
//
// A channel-sharded session (ic_session.hip) exchanges four things per
// cleaning iteration (DESIGN.md "Channel-sharded large archive"): per-subint
// channel-sum roots (all-gather), diagnostics rows to their row owners
// (all-to-all), row medians/MADs (all-gather) and convergence counters
// (all-reduce).  Every exchange is issued in stream order on the session's
// stream; no host synchronisation is implied.
//
// Transports:
//   RcclComm     — native RCCL over xGMI (one process per GPU): a
//                  communicator per shard session, every collective issued
//                  from C++ on the session stream; the host only hands the
//                  unique id of rank 0 to the other ranks once.
//   CallbackComm — the host's ic_comm_ops (one process per GPU; the Python
//                  host binds torch.distributed: gloo in the CPU tests).
//   LocalComm    — shards of one process (threads), device-to-device / peer
//                  copies ordered by HIP events and a host barrier.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/iterative_cleaner.h"

namespace icgpu {

class Comm {
public:
    int rank = 0, world = 1;
    virtual ~Comm() = default;
    // device exchange buffer (host-owned for CallbackComm)
    virtual int alloc(void **p, size_t bytes) = 0;
    virtual void release(void *p) = 0;
    virtual int allgather(const void *send, void *recv, size_t bytes, hipStream_t st) = 0;
    virtual int alltoallv(const void *send, const size_t *send_bytes, void *recv, const size_t *recv_bytes,
                          hipStream_t st) = 0;
    virtual int allreduce_sum_i32(int32_t *buf, size_t n, hipStream_t st) = 0;
    // a failing shard tells its peers (LocalComm: wakes their barriers)
    virtual void abort() {}
    // the transport lost a peer after the fact (RCCL's asynchronous errors)
    virtual bool remote_error() { return false; }
    // longest wait of the transport's own host-side polling (RcclComm: a
    // non-blocking call reported in progress), ms; the session's
    // IC_OPT_SYNC_TIMEOUT_MS
    virtual void set_timeout_ms(long long) {}
};

Comm *make_callback_comm(const ic_comm_ops &ops, int rank, int world);

// RCCL: 128-byte unique id (rank 0's, handed to every rank); the communicator
// is created on the current device.  nullptr + message in *err on failure.
int rccl_unique_id(void *id, std::string *err);
Comm *make_rccl_comm(const void *unique_id, int rank, int world, std::string *err);
// the librccl file to dlopen (nullptr / "": the ROCm install's), before its first use
int rccl_set_library(const char *path, const char **err);
// how long a communicator's creation may wait for every rank to join
int rccl_set_init_timeout(long long ms, const char **err);

struct LocalGroup;
LocalGroup *local_group_create(int world);
void local_group_destroy(LocalGroup *g);
int local_group_world(const LocalGroup *g);
// nullptr + message in *err when the rank is taken / out of range
Comm *make_local_comm(LocalGroup *g, int rank, int device, const char **err);

}  // namespace icgpu
