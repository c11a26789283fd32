// fg_comm.cpp -- the keyBy edge between co-located subtasks as an RCCL exchange (fg_comm_*).
//
// Replaces, for the window aggregation's two-phase plan, the network edge between the local and
// the global operator: KeyGroupStreamPartitioner.selectChannel (SJ/runtime/partitioner/
// KeyGroupStreamPartitioner.java:55-65) picks the owner subtask of every partial row
// (KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup, RT/state/KeyGroupRangeAssignment.java:
// 124-127) and RecordWriter.emit (RT/io/network/api/writer/RecordWriter.java:101-128) ships it
// over Netty. Here every rank (one process per GPU, one subtask each) groups its rows by owner on
// the device, and RCCL moves them over xGMI: one all-to-all of (count, watermark) per peer -- the
// watermark in-band, its minimum over the ranks being StatusWatermarkValve's combined watermark --
// one host read of the counts (the receive sizes), then grouped ncclSend / ncclRecv of each
// column's per-peer runs straight from the partition buffers (no packing copy).
//
// The communicator is bootstrapped the way the JobManager would: one rank makes an
// ncclUniqueId (fg_comm_unique_id), the 128 bytes are distributed with the deployment, every
// rank calls fg_comm_open(device, world, rank, id).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/flinkgpu.h"
#include "fg_kernels.h"

using namespace fg;

namespace {

thread_local std::string g_comm_open_error;

struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    Buf() = default;
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
    ~Buf() {
        if (p) (void)hipFree(p);
    }
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        const size_t nb = std::max(need, bytes + bytes / 2);
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, nb);
        if (e != hipSuccess) return e;
        if (p) (void)hipFree(p);
        p = q;
        bytes = nb;
        return hipSuccess;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

// per peer: {rows for it, this rank's watermark}
__global__ void k_comm_meta(const int64_t* counts, int32_t world, int64_t wm, int64_t* meta) {
    const int i = (int)threadIdx.x;
    if (i < world) {
        meta[2 * i] = counts[i];
        meta[2 * i + 1] = wm;
    }
}

}  // namespace

struct fg_comm {
    int device = 0, world = 1, rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    Buf part[kMaxOwnerCols], recv[kMaxOwnerCols];
    Buf scratch, counts, meta_send, meta_recv;
    int64_t sent_total = 0;      // bytes sent to other ranks, all exchanges
    int64_t* h_meta = nullptr;   // pinned: [world][2] sent, then [world][2] received
    std::string err;
    int fail(int code, const char* fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
};

#define COMM_HIP(c, x)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return (c)->fail(FG_EDEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)
#define COMM_NCCL(c, x)                                                                    \
    do {                                                                                   \
        ncclResult_t r_ = (x);                                                             \
        if (r_ != ncclSuccess) return (c)->fail(FG_EDEVICE, "%s: %s", #x, ncclGetErrorString(r_)); \
    } while (0)

extern "C" {

int fg_comm_unique_id(uint8_t* id) {
    if (!id) return FG_EINVAL;
    static_assert(sizeof(ncclUniqueId) == FG_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) {
        g_comm_open_error = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return FG_EDEVICE;
    }
    std::memcpy(id, &u, FG_COMM_ID_BYTES);
    return FG_OK;
}

int fg_comm_open(int32_t device_id, int32_t world, int32_t rank, const uint8_t* id, fg_comm** out) {
    if (!out) return FG_EINVAL;
    *out = nullptr;
    if (!id || world < 1 || world > 1024 || rank < 0 || rank >= world) {
        g_comm_open_error = "fg_comm_open: world must be in [1, 1024], 0 <= rank < world, id non-NULL";
        return FG_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device_id < 0 || device_id >= ndev) {
        g_comm_open_error = "fg_comm_open: no such HIP device";
        return FG_EDEVICE;
    }
    fg_comm* c = new fg_comm();
    c->device = device_id;
    c->world = world;
    c->rank = rank;
    auto bail = [&](const char* what) {
        g_comm_open_error = std::string("fg_comm_open: ") + what;
        fg_comm_close(c);
        return FG_EDEVICE;
    };
    if (hipSetDevice(device_id) != hipSuccess) return bail("hipSetDevice");
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bail("hipStreamCreate");
    if (hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming) != hipSuccess)
        return bail("hipEventCreate");
    if (hipHostMalloc((void**)&c->h_meta, sizeof(int64_t) * 4 * (size_t)world, hipHostMallocDefault) != hipSuccess)
        return bail("hipHostMalloc");
    ncclUniqueId u;
    std::memcpy(&u, id, FG_COMM_ID_BYTES);
    const ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        return bail(ncclGetErrorString(r));
    }
    *out = c;
    return FG_OK;
}

int64_t fg_comm_bytes_sent(fg_comm* c) { return c ? c->sent_total : 0; }

void* fg_comm_stream(fg_comm* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

const char* fg_comm_last_error(fg_comm* c) { return c ? c->err.c_str() : g_comm_open_error.c_str(); }

void fg_comm_close(fg_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_out) (void)hipEventDestroy(c->ev_out);
    if (c->h_meta) (void)hipHostFree(c->h_meta);
    hipStream_t s = c->stream;
    delete c;
    if (s) (void)hipStreamDestroy(s);
}

int fg_comm_exchange_columns(fg_comm* c, void* stream, int64_t n, int32_t ncols, const int64_t* const* cols,
                             int32_t key_hash, int32_t max_parallelism, int64_t watermark, fg_exchanged* out) {
    if (!c || !out || n < 0 || n > (int64_t)0x7fffffff || ncols < 1 || ncols > kMaxOwnerCols ||
        (n > 0 && !cols) || max_parallelism < c->world)
        return c ? c->fail(FG_EINVAL, "fg_comm_exchange_columns: bad arguments") : FG_EINVAL;
    for (int j = 0; n > 0 && j < ncols; j++)
        if (!cols[j]) return c->fail(FG_EINVAL, "fg_comm_exchange_columns: column %d is NULL", j);
    const int W = c->world;
    COMM_HIP(c, hipSetDevice(c->device));
    // the producer's work (the columns) before ours
    COMM_HIP(c, hipEventRecord(c->ev_in, static_cast<hipStream_t>(stream)));
    COMM_HIP(c, hipStreamWaitEvent(c->stream, c->ev_in, 0));
    COMM_HIP(c, c->counts.ensure(sizeof(int64_t) * W));
    COMM_HIP(c, c->meta_send.ensure(sizeof(int64_t) * 2 * W));
    COMM_HIP(c, c->meta_recv.ensure(sizeof(int64_t) * 2 * W));
    if (n > 0) {
        OwnerCols oc{};
        oc.ncols = ncols;
        for (int j = 0; j < ncols; j++) {
            COMM_HIP(c, c->part[j].ensure(sizeof(int64_t) * (size_t)n));
            oc.in[j] = cols[j];
            oc.out[j] = c->part[j].as<int64_t>();
        }
        const size_t words = partition_scratch_words(n, W);
        COMM_HIP(c, c->scratch.ensure(4 * words));
        COMM_HIP(c, launch_partition_cols_by_owner(oc, n, key_hash, max_parallelism, W, c->counts.as<int64_t>(),
                                                   c->scratch.as<uint32_t>(), words, c->stream));
    } else {
        COMM_HIP(c, hipMemsetAsync(c->counts.p, 0, sizeof(int64_t) * W, c->stream));
    }
    fg_launch(k_comm_meta, dim3(1), dim3(1024), 0, c->stream, (const int64_t*)c->counts.as<int64_t>(), W, watermark,
              c->meta_send.as<int64_t>());
    COMM_HIP(c, hipGetLastError());
    COMM_NCCL(c, ncclAllToAll(c->meta_send.p, c->meta_recv.p, 2, ncclInt64, c->comm, c->stream));
    // the one host read: send and receive sizes, the peers' watermarks
    COMM_HIP(c, hipMemcpyAsync(c->h_meta, c->meta_send.p, sizeof(int64_t) * 2 * W, hipMemcpyDeviceToHost, c->stream));
    COMM_HIP(c, hipMemcpyAsync(c->h_meta + 2 * W, c->meta_recv.p, sizeof(int64_t) * 2 * W, hipMemcpyDeviceToHost,
                               c->stream));
    COMM_HIP(c, hipStreamSynchronize(c->stream));
    const int64_t* ms = c->h_meta;
    const int64_t* mr = c->h_meta + 2 * W;
    std::vector<int64_t> soff(W + 1, 0), roff(W + 1, 0);
    int64_t wmin = INT64_MAX;
    for (int p = 0; p < W; p++) {
        soff[p + 1] = soff[p] + ms[2 * p];
        roff[p + 1] = roff[p] + mr[2 * p];
        wmin = std::min(wmin, mr[2 * p + 1]);
    }
    if (soff[W] != n) return c->fail(FG_EDEVICE, "fg_comm_exchange_columns: partition counted %lld of %lld rows",
                                     (long long)soff[W], (long long)n);
    const int64_t total = roff[W];
    for (int j = 0; j < ncols; j++) COMM_HIP(c, c->recv[j].ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(total, 1)));
    if (total > 0 || n > 0) {
        COMM_NCCL(c, ncclGroupStart());
        for (int p = 0; p < W; p++) {
            for (int j = 0; j < ncols; j++) {
                if (ms[2 * p] > 0)
                    COMM_NCCL(c, ncclSend(c->part[j].as<int64_t>() + soff[p], (size_t)ms[2 * p], ncclInt64, p, c->comm,
                                          c->stream));
                if (mr[2 * p] > 0)
                    COMM_NCCL(c, ncclRecv(c->recv[j].as<int64_t>() + roff[p], (size_t)mr[2 * p], ncclInt64, p, c->comm,
                                          c->stream));
            }
        }
        COMM_NCCL(c, ncclGroupEnd());
    }
    COMM_HIP(c, hipEventRecord(c->ev_out, c->stream));
    std::memset(out, 0, sizeof *out);
    out->n = total;
    out->ncols = ncols;
    for (int j = 0; j < ncols; j++) out->cols[j] = c->recv[j].as<int64_t>();
    out->min_watermark = wmin;
    out->bytes_sent = 8 * (int64_t)ncols * (n - ms[2 * c->rank]);
    c->sent_total += out->bytes_sent;
    return FG_OK;
}

// the local operator's device rows -> owners -> fg_add_partials of this rank's global operator
static int exchange_rows(fg_comm* c, fg_handle* local, const fg_rows* r, int32_t key_hash, int32_t max_parallelism,
                         int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (r->n > 0 && r->location != FG_DEVICE)
        return c->fail(FG_EINVAL, "fg_comm_exchange_partials: the local rows must be FG_DEVICE");
    if (r->num_aggs != 3 && r->num_aggs != 5)
        return c->fail(FG_EINVAL, "fg_comm_exchange_partials: rows of a FG_FLAG_LOCAL_PARTIALS operator expected "
                                  "(3 or 5 accumulator columns, got %d)", r->num_aggs);
    const int64_t* cols[kMaxOwnerCols] = {r->key, r->window_end};
    const int nc = 2 + r->num_aggs;
    for (int a = 0; a < r->num_aggs; a++) cols[2 + a] = r->agg[a];
    fg_exchanged x;
    if (int rc = fg_comm_exchange_columns(c, fg_stream(local), r->n, nc, cols, key_hash, max_parallelism, watermark, &x))
        return rc;
    // the global operator reads the received columns on its own stream, after the collective
    COMM_HIP(c, hipStreamWaitEvent(static_cast<hipStream_t>(fg_stream(global)), c->ev_out, 0));
    fg_partials p{};
    p.n = x.n;
    p.location = FG_DEVICE;
    p.key = x.cols[0];
    p.slice_end = x.cols[1];
    p.cnt_star = x.cols[2];
    p.cnt_val = x.cols[3];
    p.sum = x.cols[4];
    if (nc == 7) {
        p.min = x.cols[5];
        p.max = x.cols[6];
    }
    if (x.n > 0) {
        if (int rc = fg_add_partials(global, &p))
            return c->fail(rc, "fg_add_partials: %s", fg_last_error(global));
    }
    if (min_watermark) *min_watermark = x.min_watermark;
    return FG_OK;
}

int fg_comm_exchange_partials(fg_comm* c, fg_handle* local, const fg_rows* rows, int32_t key_hash,
                              int32_t max_parallelism, int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (!c) return FG_EINVAL;
    if (!local || !rows || !global) return c->fail(FG_EINVAL, "fg_comm_exchange_partials: NULL argument");
    return exchange_rows(c, local, rows, key_hash, max_parallelism, watermark, global, min_watermark);
}

int fg_comm_exchange_fired(fg_comm* c, fg_handle* local, int32_t key_hash, int32_t max_parallelism,
                           int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (!c) return FG_EINVAL;
    if (!local || !global) return c->fail(FG_EINVAL, "fg_comm_exchange_fired: NULL handle");
    fg_rows r;
    if (int rc = fg_collect_fired(local, &r)) return c->fail(rc, "fg_collect_fired: %s", fg_last_error(local));
    return exchange_rows(c, local, &r, key_hash, max_parallelism, watermark, global, min_watermark);
}

int fg_comm_exchange_flushed(fg_comm* c, fg_handle* local, int32_t key_hash, int32_t max_parallelism,
                             int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (!c) return FG_EINVAL;
    if (!local || !global) return c->fail(FG_EINVAL, "fg_comm_exchange_flushed: NULL handle");
    fg_rows r;
    if (int rc = fg_flush_partials(local, FG_DEVICE, &r)) return c->fail(rc, "fg_flush_partials: %s", fg_last_error(local));
    return exchange_rows(c, local, &r, key_hash, max_parallelism, watermark, global, min_watermark);
}

}  // extern "C"
