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

// per peer: {rows for it, this rank's watermark, its epoch, its columns << 1 | its status}. The partition's counts
// must add up to the rows handed in; a rank whose round failed (or whose counts do not) sends zero
// rows and status 1, so every rank learns of it from the one all-to-all and the round ends on all
// of them together instead of leaving the peers blocked in the data collective
__global__ void k_comm_meta(const int64_t* counts, int32_t world, int64_t n, int64_t wm, int64_t epoch,
                            int32_t status, int32_t ncols, int64_t* meta) {
    __shared__ int s_ok;
    const int i = (int)threadIdx.x;
    if (i == 0) {
        int64_t t = 0;
        for (int p = 0; p < world; p++) t += counts ? counts[p] : 0;
        s_ok = status == 0 && t == n;
    }
    __syncthreads();
    if (i < world) {
        meta[4 * i] = s_ok && counts ? counts[i] : 0;
        meta[4 * i + 1] = wm;
        meta[4 * i + 2] = epoch;
        meta[4 * i + 3] = (int64_t)ncols << 1 | (s_ok ? 0 : 1);   // (the columns its rows carry)
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
    int64_t* h_meta = nullptr;   // pinned: [world][4] sent, then [world][4] received
    std::string err;
    // the round prepared by fg_comm_round_begin (or by the one-call exchanges)
    bool pending = false;
    int64_t n = 0;               // rows partitioned
    int32_t ncols = 0;
    int rc_begin = FG_OK;        // this rank's own failure, reported after the collective
    std::string err_begin;
    // the received columns of the last collective, for fg_comm_round_end
    int64_t recv_n = 0;
    int32_t recv_ncols = 0;
    bool recv_ready = false;
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
    if (hipHostMalloc((void**)&c->h_meta, sizeof(int64_t) * 8 * (size_t)world, hipHostMallocDefault) != hipSuccess)
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

// Step 1 of a round: the rows (n, ncols device columns produced on `producer`) grouped by owner
// into the communicator's buffers and the meta words of every peer -- on the communicator's stream,
// the producer's later work ordered after the partition (the columns may then be reused). status != 0
// (this rank failed before the round): zero rows, the failure flag for the peers.
static int round_prepare(fg_comm* c, hipStream_t producer, int64_t n, int32_t ncols, const int64_t* const* cols,
                         int32_t key_hash, int32_t max_parallelism, int64_t watermark, int64_t epoch, int status) {
    const int W = c->world;
    c->pending = true;
    c->recv_ready = false;
    c->n = status ? 0 : n;
    c->ncols = ncols;
    COMM_HIP(c, hipSetDevice(c->device));
    COMM_HIP(c, c->counts.ensure(sizeof(int64_t) * W));
    COMM_HIP(c, c->meta_send.ensure(sizeof(int64_t) * 4 * W));
    COMM_HIP(c, c->meta_recv.ensure(sizeof(int64_t) * 4 * W));
    if (producer) {   // the producer's work (the columns) before ours
        COMM_HIP(c, hipEventRecord(c->ev_in, producer));
        COMM_HIP(c, hipStreamWaitEvent(c->stream, c->ev_in, 0));
    }
    if (c->n > 0) {
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
    fg_launch(k_comm_meta, dim3(1), dim3(1024), 0, c->stream, (const int64_t*)c->counts.as<int64_t>(), W, c->n,
              watermark, epoch, status, ncols, c->meta_send.as<int64_t>());
    COMM_HIP(c, hipGetLastError());
    if (producer && c->n > 0) {   // (the producer may overwrite the columns once the partition has read them)
        COMM_HIP(c, hipEventRecord(c->ev_out, c->stream));
        COMM_HIP(c, hipStreamWaitEvent(producer, c->ev_out, 0));
    }
    return FG_OK;
}

// Step 2: the collectives. One all-to-all of the meta words, one host read; a failed rank (its
// status word) ends the round on every rank with FG_EDEVICE and no data moved; else grouped
// send / receive of each column's per-peer runs.
static int round_collective(fg_comm* c, fg_exchanged* x, fg_round* r) {
    if (!c->pending) return c->fail(FG_ESTATE, "fg_comm_round_exchange: no round begun");
    c->pending = false;
    const int W = c->world;
    COMM_NCCL(c, ncclAllToAll(c->meta_send.p, c->meta_recv.p, 4, ncclInt64, c->comm, c->stream));
    COMM_HIP(c, hipMemcpyAsync(c->h_meta, c->meta_send.p, sizeof(int64_t) * 4 * W, hipMemcpyDeviceToHost, c->stream));
    COMM_HIP(c, hipMemcpyAsync(c->h_meta + 4 * W, c->meta_recv.p, sizeof(int64_t) * 4 * W, hipMemcpyDeviceToHost,
                               c->stream));
    COMM_HIP(c, hipStreamSynchronize(c->stream));
    const int64_t* ms = c->h_meta;
    const int64_t* mr = c->h_meta + 4 * W;
    std::vector<int64_t> soff(W + 1, 0), roff(W + 1, 0);
    int64_t wmin = INT64_MAX, emin = INT64_MAX;
    int failed = -1, rcols = 0;
    bool mixed = false;   // peers sending rows of different column counts (never, for one operator)
    for (int p = 0; p < W; p++) {
        soff[p + 1] = soff[p] + ms[4 * p];
        roff[p + 1] = roff[p] + mr[4 * p];
        wmin = std::min(wmin, mr[4 * p + 1]);
        emin = std::min(emin, mr[4 * p + 2]);
        if ((mr[4 * p + 3] & 1) != 0 && failed < 0) failed = p;
        if (mr[4 * p] > 0) {
            const int pc = (int)(mr[4 * p + 3] >> 1);
            mixed = mixed || (rcols != 0 && pc != rcols) || pc < 1 || pc > kMaxOwnerCols;
            rcols = pc;
        }
    }
    if (mixed && failed < 0) failed = W;   // (every rank sees every peer's count: all decide alike)
    if (r) {
        std::memset(r, 0, sizeof *r);
        r->min_watermark = wmin;
        r->min_epoch = emin;
        r->failed_rank = failed;
    }
    if (failed >= 0) {
        if (c->rc_begin != FG_OK) return c->fail(FG_EDEVICE, "this rank's round failed: %s", c->err_begin.c_str());
        if (failed == W) return c->fail(FG_EDEVICE, "fg_comm round: peers sent rows of different column counts");
        if (failed == c->rank)   // (the counts of the partition did not add up to the rows)
            return c->fail(FG_EDEVICE, "fg_comm round: the owner partition counted %lld of %lld rows",
                           (long long)soff[W], (long long)c->n);
        return c->fail(FG_EDEVICE, "fg_comm round: rank %d failed its round (no rows moved on any rank)", failed);
    }
    const int64_t total = roff[W];
    if (rcols == 0) rcols = c->ncols;
    for (int j = 0; j < rcols; j++)
        COMM_HIP(c, c->recv[j].ensure(sizeof(int64_t) * (size_t)std::max<int64_t>(total, 1)));
    if (total > 0 || c->n > 0) {
        COMM_NCCL(c, ncclGroupStart());
        for (int p = 0; p < W; p++) {
            for (int j = 0; j < c->ncols && ms[4 * p] > 0; j++)
                COMM_NCCL(c, ncclSend(c->part[j].as<int64_t>() + soff[p], (size_t)ms[4 * p], ncclInt64, p, c->comm,
                                      c->stream));
            for (int j = 0; j < rcols && mr[4 * p] > 0; j++)
                COMM_NCCL(c, ncclRecv(c->recv[j].as<int64_t>() + roff[p], (size_t)mr[4 * p], ncclInt64, p, c->comm,
                                      c->stream));
        }
        COMM_NCCL(c, ncclGroupEnd());
    }
    COMM_HIP(c, hipEventRecord(c->ev_out, c->stream));
    const int64_t sent = 8 * (int64_t)c->ncols * (c->n - ms[4 * c->rank]);
    c->sent_total += sent;
    c->recv_n = total;
    c->recv_ncols = rcols;
    c->recv_ready = true;
    if (x) {
        std::memset(x, 0, sizeof *x);
        x->n = total;
        x->ncols = rcols;
        for (int j = 0; j < rcols; j++) x->cols[j] = c->recv[j].as<int64_t>();
        x->min_watermark = wmin;
        x->bytes_sent = sent;
    }
    if (r) {
        r->rows_sent = c->n;
        r->rows_received = total;
        r->bytes_sent = sent;
    }
    return FG_OK;
}

int fg_comm_exchange_columns(fg_comm* c, void* stream, int64_t n, int32_t ncols, const int64_t* const* cols,
                             int32_t key_hash, int32_t max_parallelism, int64_t watermark, fg_exchanged* out) {
    if (!c) return FG_EINVAL;
    int status = 0;
    c->rc_begin = FG_OK;
    if (!out || n < 0 || n > (int64_t)0x7fffffff || ncols < 1 || ncols > kMaxOwnerCols || (n > 0 && !cols) ||
        max_parallelism < c->world) {
        status = 1;
        c->rc_begin = FG_EINVAL;
        c->err_begin = "fg_comm_exchange_columns: bad arguments";
    }
    for (int j = 0; !status && n > 0 && j < ncols; j++)
        if (!cols[j]) {
            status = 1;
            c->rc_begin = FG_EINVAL;
            c->err_begin = "fg_comm_exchange_columns: a column is NULL";
        }
    // (a rank with bad arguments still takes part: its peers learn of the failure from the meta words)
    if (int rc = round_prepare(c, static_cast<hipStream_t>(stream), n, status ? 1 : ncols, cols, key_hash,
                               std::max(max_parallelism, c->world), watermark, 0, status))
        return rc;
    const int rc = round_collective(c, out, nullptr);
    if (status) return c->fail(c->rc_begin, "%s", c->err_begin.c_str());
    return rc;
}

// the received columns of the last collective -> fg_add_partials of `global` (on its stream, after
// the collective)
static int round_merge(fg_comm* c, fg_handle* global) {
    if (!c->recv_ready) return c->fail(FG_ESTATE, "fg_comm_round_end: no round exchanged");
    c->recv_ready = false;
    if (c->recv_n == 0) return FG_OK;
    if (!global) return c->fail(FG_EINVAL, "fg_comm_round_end: NULL global handle");
    if (c->recv_ncols != 5 && c->recv_ncols != 7)
        return c->fail(FG_EINVAL, "fg_comm_round_end: the rows received are not partial accumulator rows (%d columns)",
                       c->recv_ncols);
    COMM_HIP(c, hipStreamWaitEvent(static_cast<hipStream_t>(fg_stream(global)), c->ev_out, 0));
    fg_partials p{};
    p.n = c->recv_n;
    p.location = FG_DEVICE;
    p.key = c->recv[0].as<int64_t>();
    p.slice_end = c->recv[1].as<int64_t>();
    p.cnt_star = c->recv[2].as<int64_t>();
    p.cnt_val = c->recv[3].as<int64_t>();
    p.sum = c->recv[4].as<int64_t>();
    if (c->recv_ncols == 7) {
        p.min = c->recv[5].as<int64_t>();
        p.max = c->recv[6].as<int64_t>();
    }
    if (int rc = fg_add_partials(global, &p)) return c->fail(rc, "fg_add_partials: %s", fg_last_error(global));
    return FG_OK;
}

// step 1 for the local operator's rows (device rows of a FG_FLAG_LOCAL_PARTIALS handle)
static int begin_rows(fg_comm* c, fg_handle* local, const fg_rows* r, int rc_rows, const char* what,
                      int32_t key_hash, int32_t max_parallelism, int64_t watermark, int64_t epoch) {
    c->rc_begin = FG_OK;
    int status = 0;
    auto failed = [&](int code, const std::string& msg) {
        status = 1;
        c->rc_begin = code;
        c->err_begin = msg;
    };
    if (rc_rows) failed(rc_rows, std::string(what) + ": " + (local ? fg_last_error(local) : "NULL handle"));
    else if (r->n > 0 && r->location != FG_DEVICE) failed(FG_EINVAL, "the local rows must be FG_DEVICE");
    else if (r->num_aggs != 3 && r->num_aggs != 5)
        failed(FG_EINVAL, "rows of a FG_FLAG_LOCAL_PARTIALS operator expected (3 or 5 accumulator columns, got " +
                              std::to_string(r->num_aggs) + ")");
    else if (max_parallelism < c->world) failed(FG_EINVAL, "max_parallelism below the world size");
    const int64_t* cols[kMaxOwnerCols] = {};
    int nc = 1;
    if (!status) {
        cols[0] = r->key;
        cols[1] = r->window_end;
        nc = 2 + r->num_aggs;
        for (int a = 0; a < r->num_aggs; a++) cols[2 + a] = r->agg[a];
    }
    return round_prepare(c, local ? static_cast<hipStream_t>(fg_stream(local)) : nullptr, status ? 0 : r->n, nc, cols, key_hash,
                         std::max(max_parallelism, c->world), watermark, epoch, status);
}

// the local operator's device rows -> owners -> fg_add_partials of this rank's global operator
static int exchange_rows(fg_comm* c, fg_handle* local, const fg_rows* r, int rc_rows, const char* what,
                         int32_t key_hash, int32_t max_parallelism, int64_t watermark, fg_handle* global,
                         int64_t* min_watermark) {
    if (int rc = begin_rows(c, local, r, rc_rows, what, key_hash, max_parallelism, watermark, 0)) return rc;
    fg_round rr;
    const int rc = round_collective(c, nullptr, &rr);
    if (c->rc_begin != FG_OK) return c->fail(c->rc_begin, "%s", c->err_begin.c_str());
    if (rc) return rc;
    if (int rc2 = round_merge(c, global)) return rc2;
    if (min_watermark) *min_watermark = rr.min_watermark;
    return FG_OK;
}

int fg_comm_exchange_partials(fg_comm* c, fg_handle* local, const fg_rows* rows, int32_t key_hash,
                              int32_t max_parallelism, int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (!c) return FG_EINVAL;
    fg_rows none{};
    none.num_aggs = 3;
    const bool bad = !local || !rows || !global;
    if (bad) c->err_begin = "fg_comm_exchange_partials: NULL argument";
    return exchange_rows(c, local, bad ? &none : rows, bad ? FG_EINVAL : 0, "fg_comm_exchange_partials", key_hash,
                         max_parallelism, watermark, global, min_watermark);
}

int fg_comm_exchange_fired(fg_comm* c, fg_handle* local, int32_t key_hash, int32_t max_parallelism,
                           int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (!c) return FG_EINVAL;
    fg_rows r{};
    r.num_aggs = 3;
    const int rc = local && global ? fg_collect_fired(local, &r) : FG_EINVAL;
    return exchange_rows(c, local, &r, rc, "fg_collect_fired", key_hash, max_parallelism, watermark, global,
                         min_watermark);
}

int fg_comm_exchange_flushed(fg_comm* c, fg_handle* local, int32_t key_hash, int32_t max_parallelism,
                             int64_t watermark, fg_handle* global, int64_t* min_watermark) {
    if (!c) return FG_EINVAL;
    fg_rows r{};
    r.num_aggs = 3;
    const int rc = local && global ? fg_flush_partials(local, FG_DEVICE, &r) : FG_EINVAL;
    return exchange_rows(c, local, &r, rc, "fg_flush_partials", key_hash, max_parallelism, watermark, global,
                         min_watermark);
}

int fg_comm_round_begin(fg_comm* c, fg_handle* local, int32_t mode, int32_t key_hash, int32_t max_parallelism,
                        int64_t watermark, int64_t epoch) {
    if (!c) return FG_EINVAL;
    if (c->pending) return c->fail(FG_ESTATE, "fg_comm_round_begin: the previous round was not exchanged");
    const int64_t* none[kMaxOwnerCols] = {};
    const int32_t mp = std::max(max_parallelism, c->world);
    if (mode == FG_ROUND_IDLE) {   // (its column count is moot: it sends no rows)
        c->rc_begin = FG_OK;
        return round_prepare(c, nullptr, 0, 5, none, key_hash, mp, watermark, epoch, 0);
    }
    if ((mode != FG_ROUND_FIRED && mode != FG_ROUND_FLUSHED) || !local) {   // (still takes part, failed)
        c->rc_begin = FG_EINVAL;
        c->err_begin = !local ? "fg_comm_round_begin: NULL local handle" : "fg_comm_round_begin: bad mode";
        return round_prepare(c, nullptr, 0, 5, none, key_hash, mp, watermark, epoch, 1);
    }
    fg_rows r{};
    r.num_aggs = 3;
    const int rc = mode == FG_ROUND_FIRED ? fg_collect_fired(local, &r) : fg_flush_partials(local, FG_DEVICE, &r);
    return begin_rows(c, local, &r, rc, mode == FG_ROUND_FIRED ? "fg_collect_fired" : "fg_flush_partials", key_hash,
                      max_parallelism, watermark, epoch);
}

int fg_comm_round_exchange(fg_comm* c, fg_round* out) {
    if (!c) return FG_EINVAL;
    const int rc = round_collective(c, nullptr, out);
    if (rc == FG_OK && c->rc_begin != FG_OK) return c->fail(c->rc_begin, "%s", c->err_begin.c_str());
    return rc;
}

int fg_comm_round_end(fg_comm* c, fg_handle* global) {
    if (!c) return FG_EINVAL;
    return round_merge(c, global);
}

}  // extern "C"
