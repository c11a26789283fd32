#!/usr/bin/env python
"""Benchmark: records/s of the MI355X window-aggregation engine on BASELINE configs[1].

Workload (BASELINE.json configs[1]): SQL TUMBLE 1s
COUNT(*)/SUM/AVG(double) through the SlicingWindowOperator surface, 1B records per GPU,
10M uniform BIGINT keys, 100M records per event-second (10 windows), in order, watermark
= max rowtime - 1 every 1M records; end of input sends Long.MAX_VALUE.

One step = the whole 1B-record job: reset the operator, feed the resident columns in
50M-record micro-batches (each followed by the 1M-cadence watermarks that fall in it),
then the final watermark fires the last window. Inputs (key i64, val f64, rowtime i64;
24 GB) are generated on the GPU and resident in HBM before timing; fired rows stay in
HBM (device output).  N > 1 (torchrun): every rank owns key groups
kg*N/128 and a 1B-record source partition (weak scaling) and runs the two-phase plan of
TwoStageOptimizedWindowAggregateRule: a local operator (LocalAggCombiner) aggregates its
source partition per (key, slice); at each micro-batch's watermark the fired slices'
partial accumulators are routed to their key-group owners by one RCCL all-to-all
(flink_amd.exchange.exchange_partials) and merged by the owner's global operator
(GlobalAggCombiner), which fires the windows. `--exchange raw` ships the records
themselves instead (one all-to-all per micro-batch before a single-phase operator).

Roofline: HBM. Algorithmic bytes: 24 B per input record + 48 B per fired
row. `roofline` is for the dominant kernel, timed with HIP events on the engine's
stream; `job_roofline_frac` is the whole-job B_alg / t / (N * 8 TB/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "records/sec/node, keyed TUMBLE SUM/COUNT/AVG at 1/2/4/8 GPU; % of HBM peak"
HBM_PEAK_GBS = 8000.0
SEED = 0x5EEDF11C
T0 = 1_600_000_000_000
JMAX = (1 << 63) - 1
M64 = (1 << 64) - 1


def s64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def lsr(z: torch.Tensor, s: int) -> torch.Tensor:
    return (z >> s) & ((1 << (64 - s)) - 1)


def splitmix64(x: torch.Tensor) -> torch.Tensor:
    z = x + s64(0x9E3779B97F4A7C15)
    z = (z ^ lsr(z, 30)) * s64(0xBF58476D1CE4E5B9)
    z = (z ^ lsr(z, 27)) * s64(0x94D049BB133111EB)
    return z ^ lsr(z, 31)


# BASELINE configs by workload: window, key space, event-time rate, order
WORKLOADS = {
    # configs[1] (the bench's `value`): SQL TUMBLE 1s COUNT(*)/SUM/AVG(double)
    # (micro-batch = one event-second of records; 50M-record batches: 20.8 vs 20.1 ms per 1B on one box)
    "tumble": dict(window=("tumbling", 1000), keys=10_000_000, rate=100_000_000, jitter=0, delay=0, zipf=0.0,
                   batch=100_000_000, desc="SQL TUMBLE 1s COUNT(*)/SUM/AVG(double) via SlicingWindowOperator, 1B records per GPU, "
                        "10M uniform keys (BASELINE configs[1])"),
    # configs[2]: SQL HOP 5min/1min, rowtime over 30 event-minutes
    "hop": dict(window=("hopping", 300_000, 60_000), keys=10_000_000, rate=1_000_000_000 // 1800, jitter=0, delay=0,
                zipf=0.0, batch=33_333_334, desc="SQL HOP 5min/1min COUNT(*)/SUM/AVG(double), 1B records per GPU over 30 event-minutes, "
                               "10M uniform keys (BASELINE configs[2])"),
    # configs[3]: CUMULATE 1h/1min over 60 event-minutes; 100M keys sharded over 8 GPUs ->
    # the key space is 12.5M per GPU: the per-GPU share at N = 1, the whole 100M space at N = 8
    # (keys_per_gpu: main() multiplies by the world size)
    "cumulate": dict(window=("cumulative", 3_600_000, 60_000), keys=12_500_000, keys_per_gpu=True,
                     rate=1_000_000_000 // 3600,
                     jitter=0, delay=0, zipf=0.0, batch=16_666_667,
                     desc="SQL CUMULATE 1h/1min COUNT(*)/SUM/AVG(double), 1B records per GPU over 60 event-minutes, "
                          "uniform keys: 12.5M x N GPUs (100M at N = 8, each GPU owning a 12.5M key-group share; "
                          "BASELINE configs[3])"),
    # configs[0]: DataStream keyBy().window(TumblingEventTimeWindows 1s).sum on (long key,
    # long val), 10M records, 10k keys, 1M records per event-second, watermark every 10k
    "datastream": dict(window=("tumbling", 1000), keys=10_000, rate=1_000_000, jitter=0, delay=0, zipf=0.0,
                       batch=1_000_000, records=10_000_000, wm_every=10_000, mode="datastream",
                       desc="DataStream keyBy().window(TumblingEventTimeWindows 1s).sum (WindowOperator), "
                            "10M (long, long) records, 10k keys (BASELINE configs[0])"),
    # configs[1] with a STRING grouping key: every record's key is a 32-B BinaryRowData key row
    # ("user" + 8 hex digits) interned by the GPU key dictionary inside the timed region
    "strings": dict(window=("tumbling", 1000), keys=10_000_000, rate=100_000_000, jitter=0, delay=0, zipf=0.0,
                    batch=100_000_000, desc="SQL TUMBLE 1s COUNT(*)/SUM/AVG(double) GROUP BY a STRING key ('user' + 8 hex digits, "
                         "32-B BinaryRowData key rows interned by the GPU key dictionary each micro-batch), "
                         "1B records per GPU, 10M distinct keys (BASELINE configs[1] with a STRING key)"),
    # configs[4]: TUMBLE 1s AVG(double), Zipf s = 1.1 keys, 2 s jitter, bounded out-of-orderness 2 s
    "zipf": dict(window=("tumbling", 1000), keys=10_000_000, rate=100_000_000, jitter=2000, delay=2000, zipf=1.1,
                 desc="SQL TUMBLE 1s AVG(double), 1B records per GPU, 10M Zipf(1.1) keys, rowtime jitter U[0,2s), "
                      "watermark = max rowtime - 2s - 1 (BASELINE configs[4])"),
}


def zipf_distinct_per_slice(keys, s, records):
    """Expected distinct keys among `records` Zipf(s) draws over `keys` ranks:
    sum_k 1 - (1 - p_k)^records -- the operator's sizing hint (fg_config.expected_keys is
    the distinct keys per slice; the key space over-sizes the tables for skewed keys)."""
    p = np.arange(1, keys + 1, dtype=np.float64) ** -s
    p /= p.sum()
    return float(np.sum(-np.expm1(records * np.log1p(-p))))


def zipf_cdf(keys, s, device):
    """CDF of Zipf(s) over ranks 1..keys (float64), summed sequentially on the host so that
    the generated keys are the same in every run (a device cumsum's order is not fixed)."""
    w = np.arange(1, keys + 1, dtype=np.float64) ** -s
    c = np.cumsum(w)
    return torch.from_numpy(c / c[-1]).to(device)


def gen_columns(n, keys, rate_s, base_index, device, chunk=1 << 26, jitter=0, zipf=0.0, t_base=None):
    """key = u % keys (or Zipf(zipf) rank - 1 by inverse CDF), val = uniform [0, 1000) f64,
    rowtime = T0 + (i - t_base) * 1000 // rate_s (+ U[0, jitter) ms) for the records
    i = base_index .. base_index + n - 1 of the stream (t_base: base_index) (tests/streams.py)."""
    if t_base is None:
        t_base = base_index
    key = torch.empty(n, dtype=torch.int64, device=device)
    ts = torch.empty(n, dtype=torch.int64, device=device)
    val = torch.empty(n, dtype=torch.float64, device=device)
    cdf = zipf_cdf(keys, zipf, device) if zipf > 0 else None
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        i = torch.arange(base_index + lo, base_index + hi, dtype=torch.int64, device=device)
        u = splitmix64(i ^ SEED)
        u2 = splitmix64(i ^ (SEED * 3 + 1))
        if cdf is not None:
            q = lsr(u, 11).to(torch.float64) * (1.0 / float(1 << 53))
            key[lo:hi] = torch.searchsorted(cdf, q).clamp_(max=keys - 1)
            del q
        else:
            key[lo:hi] = (lsr(u, 1) % keys * 2 + (u & 1)) % keys        # unsigned u % keys
        val[lo:hi] = lsr(u2, 11).to(torch.float64) * (1000.0 / float(1 << 53))
        ts[lo:hi] = T0 + (i - t_base) * 1000 // rate_s
        if jitter:
            ts[lo:hi] += lsr(u2, 1) % jitter
        del i, u, u2
    return key, ts, val


def string_key_rows(key):
    """32-B BinaryRowData key rows of one STRING field "user%08x" (flink_amd.keys.key_row
    layout: bit set, the slot holding offset 16 << 32 | length 12, the 12 bytes padded to 8),
    as an int64 [n, 4] device tensor."""
    k = key & 0xFFFFFFFF
    hexc = []
    for i in range(8):
        nib = (k >> (28 - 4 * i)) & 15
        hexc.append(torch.where(nib < 10, nib + 48, nib + 87))
    rows = torch.zeros((key.numel(), 4), dtype=torch.int64, device=key.device)
    rows[:, 1] = (16 << 32) | 12
    w2 = ord("u") | ord("s") << 8 | ord("e") << 16 | ord("r") << 24
    rows[:, 2] = w2 | hexc[0] << 32 | hexc[1] << 40 | hexc[2] << 48 | hexc[3] << 56
    rows[:, 3] = hexc[4] | hexc[5] << 8 | hexc[6] << 16 | hexc[7] << 24
    return rows


def watermarks_for(lo, hi, rate_s, every, delay=0, jitter=0):
    """1M-cadence watermarks delivered after records [lo, hi): max rowtime - delay - 1
    (in order: max rowtime = T0 + (j - 1) * 1000 // rate_s; with jitter, a bound of the max)."""
    out = []
    j = (lo // every + 1) * every
    while j <= hi:
        mx = T0 + (j - 1) * 1000 // rate_s + (jitter - 1 if jitter else 0)
        out.append(mx - delay - 1)
        j += every
    return out


class TwoPhase:
    """The N > 1 schedule of one rank (TwoStageOptimizedWindowAggregateRule.java:81-104): the
    local operator (LocalSlicingWindowAggOperator + LocalAggCombiner) -> key-group exchange of its
    partial rows -> the owner's global operator (GlobalAggCombiner). bench.py's timed loop and
    tests/test_gpu_multiproc.py drive this same object, so the tested schedule is the timed one.

    Per micro-batch (`round`): the local operator takes EVERY watermark of the batch
    (LocalSlicingWindowAggOperator.processWatermark, :113-134 -- fg_advance_progress_async_n, its
    flushed partial rows collected once), then one exchange ships the rows with the batch's last
    watermark in-band (StatusWatermarkValve: the min over the ranks), the previous round's global
    fires are collected, the partials merged (late rules per partial row at the global's
    progress) and the global fire at the combined watermark queued asynchronously. Firing only at
    the batch's last combined watermark fires the same windows in the same order as firing at
    each: no partial row reaches the global operator between two watermarks of one batch (the
    batch's records all precede its watermarks), and a window's trigger set is cumulative in the
    watermark.

    `checkpoint()` is prepareSnapshotPreBarrier on both: the local buffer is flushed and its
    partial rows go through the exchange before the barrier (the reference forwards them
    downstream ahead of it, LocalSlicingWindowAggOperator.java:142-144), then the global
    operator's staged state is flushed and imaged (window-aggs)."""

    def __init__(self, op_local, op_global, device, max_parallelism=128, key_hash=None, via_cpu=False,
                 key_rows=None, host_rows=False, comm=None):
        """comm: a flink_amd.comm.Communicator -- the exchange through the C-ABI's RCCL edge
        (fg_comm_exchange_fired / _flushed) instead of torch.distributed (exchange_partials)."""
        from flink_amd import _lib as FL
        if comm is not None and (key_rows is not None or via_cpu):
            raise ValueError("the C-ABI exchange moves BIGINT keys over RCCL (no key rows, no gloo)")
        self.comm = comm
        self.local, self.glob = op_local, op_global
        self.device, self.maxp = device, max_parallelism
        self.key_hash = FL.KEYHASH_BINARYROW_BIGINT if key_hash is None else key_hash
        self.via_cpu, self.key_rows, self.host_rows = via_cpu, key_rows, host_rows
        self.held = False      # the global fire of the last round, not collected yet
        self.wm = -(1 << 63)   # this rank's last watermark

    def _collect(self):
        """the held global fire's rows (numpy with host_rows, else the row count)"""
        if not self.held:
            return None if self.host_rows else 0
        self.held = False
        r = self.glob.collect_fired(host=self.host_rows)
        return r if self.host_rows else r.n

    def _ship(self, r, wm):
        """exchange the local rows `r` (device FgRows) by key-group owner, collect the held global
        fire, merge the received partials; returns (collected, bytes sent, combined watermark)"""
        from flink_amd.exchange import device_columns, exchange_partials
        cols = device_columns(r, aggs=tuple(range(int(r.num_aggs))), device=self.device)
        recv, sent, gwm = exchange_partials(cols, max_parallelism=self.maxp, key_hash=self.key_hash,
                                            via_cpu=self.via_cpu, key_rows=self.key_rows, watermark=wm)
        got = self._collect()   # (rows of the previous fire go out before these partials merge)
        self.glob.process_partials(*recv)
        return got, sent, gwm

    def _ship_capi(self, flushed):
        """the same through the C-ABI (fg_comm_exchange_fired / _flushed: collect or flush the
        local rows, exchange, fg_add_partials of the global operator)"""
        got = self._collect()
        b0 = self.comm.bytes_sent
        f = self.comm.exchange_flushed if flushed else self.comm.exchange_fired
        gwm = f(self.local, self.glob, self.wm, key_hash=self.key_hash, max_parallelism=self.maxp)
        return got, self.comm.bytes_sent - b0, gwm

    def round(self, wms):
        """one micro-batch's watermarks (in order); returns (collected rows, bytes sent)"""
        self.local.process_watermarks(wms)
        self.wm = int(wms[-1])
        if self.comm is not None:
            got, sent, gwm = self._ship_capi(False)
        else:
            got, sent, gwm = self._ship(self.local.collect_fired(), self.wm)
        self.glob.process_watermark(gwm, device_output=True, wait=False)
        self.held = True
        return got, sent

    def checkpoint(self, asynchronous=False):
        """prepareSnapshotPreBarrier + snapshotState; returns (collected rows, bytes sent,
        (global image, timer watermark)) -- asynchronous: the image is None, its copy to the host
        overlaps the next rounds and snapshot_wait returns it"""
        if self.comm is not None:
            got, sent, _ = self._ship_capi(True)
        else:
            got, sent, _ = self._ship(self.local.flush_partials(device_output=True), self.wm)
        self.glob.prepare_snapshot_pre_barrier()
        if asynchronous:
            self.glob.snapshot_state_async()
            return got, sent, None
        # (a copy: the image outlives the operator -- a failover closes it and restores a new one
        # from the image; copy=False would leave views of the closed handle's pinned memory)
        return got, sent, self.glob.snapshot_state(copy=True)

    def snapshot_wait(self):
        """the image of the last asynchronous checkpoint (views of the operator's pinned image)"""
        return self.glob.snapshot_state_wait(copy=False)

    def finish(self):
        """end of input (Long.MAX_VALUE); returns (rows of both last fires, bytes sent)"""
        a, sent = self.round([JMAX])
        b = self._collect()
        if self.host_rows:
            return [x for x in (a, b) if x is not None and len(x)], sent
        return a + b, sent


def measure_copy_peak(dev, nbytes=2 << 30, reps=5):
    """Device-to-device copy bandwidth (read + write bytes / time) on this GPU."""
    try:
        a = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
        b = torch.empty_like(a)
        b.copy_(a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            b.copy_(a)
        e1.record()
        e1.synchronize()
        gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
        del a, b
        return gbs
    except RuntimeError:
        return None


def host_cores():
    """CPUs this process may run on (its affinity mask; os.cpu_count() counts the machine)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs' worth of time the cgroup grants (cpu.max quota / period), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(args, rate):
    """The oracle (C restatement of the reference operator) on the host cores: one instance
    per core (P = nproc, capped at 85 so that maxParallelism stays 128 by
    KeyGroupRangeAssignment.computeDefaultMaxParallelism), records routed by key
    group, on a bounded prefix of the same stream."""
    from oracle import oracle as O
    O.build()
    quota = cpu_quota()
    # P = the CPUs this process may use: its affinity mask, capped by the cgroup's CPU quota (a
    # box grants a 16-CPU share of a larger machine), and by 85 (maxParallelism 128)
    avail = host_cores() if quota is None else max(1, min(host_cores(), int(quota)))
    cores = min(85, avail) if args.cpu_threads is None else args.cpu_threads

    def gen(n):
        i = np.arange(n, dtype=np.uint64)
        with np.errstate(over="ignore"):
            def sm(x):
                z = (x + np.uint64(0x9E3779B97F4A7C15))
                z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
                z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
                return z ^ (z >> np.uint64(31))
            u = sm(i ^ np.uint64(SEED))
            u2 = sm(i ^ np.uint64(SEED * 3 + 1))
        key = (u % np.uint64(args.keys)).astype(np.int64)
        val = (u2 >> np.uint64(11)).astype(np.float64) * (1000.0 / float(1 << 53))
        ts = (T0 + np.arange(n, dtype=np.int64) // rate).astype(np.int64)
        return key, ts, val

    cfg = O.Config(O.MODE_SQL, O.TUMBLE, 1000, 0, 0, 0, O.VAL_F64, 0)

    def run(n):
        key, ts, val = gen(n)
        wm_at = np.arange(args.wm_every, n + 1, args.wm_every, dtype=np.int64)
        wm_val = T0 + (wm_at - 1) // rate - 1
        wm_at = np.append(wm_at, n)
        wm_val = np.append(wm_val, JMAX)
        el, rows, cs, late = O.run_partitioned(cfg, cores, 128, key, ts, val, wm_at, wm_val)
        return el, rows

    el, _ = run(2_000_000)
    rate_est = 2_000_000 / max(el, 1e-6)
    n = int(min(args.cpu_max_records, max(4_000_000, rate_est * args.cpu_seconds)))
    n -= n % args.wm_every
    el, rows = run(n)
    return dict(value=n / el, unit="records/s", cores=cores, kind="port", cpu_quota=quota,
                cores_note="P = min(affinity CPUs, cgroup CPU quota, 85) threads, one operator instance each",
                sample=f"first {n:,} records of the configs[1] stream (10M-key space), watermark every "
                       f"{args.wm_every:,} records + final Long.MAX_VALUE; C restatement of "
                       f"SlicingWindowOperator/RecordsWindowBuffer/AggCombiner, {cores} instances routed by "
                       f"key group (maxParallelism 128); {el:.1f} s, {rows:,} rows fired" +
                       (f"; the cgroup grants {quota:g} CPUs of time" if quota else ""))


def pmc_traffic(kernel_class, workload="tumble"):
    """HBM bytes per launch of `kernel_class` from the newest committed rocprofv3 PMC summary
    (profiles/**/pmc_traffic.json, profiles/pmc_summary.py) -- only if it was counted on THIS
    build's kernels (same sha256 of libflinkgpu.so's device code objects, flink_amd.buildinfo: a
    host-only change keeps the kernels' traffic); otherwise None. Returns (bytes, source)."""
    import glob

    from flink_amd import buildinfo
    try:
        ksha = buildinfo.kernels_sha256()
    except (OSError, ValueError, KeyError):
        return None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_traffic.json"), recursive=True),
                       reverse=True):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("_provenance", {}).get("kernels_sha256") != ksha:
            continue
        if d["_provenance"].get("workload", "tumble") != workload:   # counted on another workload's launches
            continue
        v = d.get(kernel_class.replace("local_", ""), {}).get("hbm_bytes_per_launch")
        if v is not None:
            return v, os.path.relpath(path, ROOT) + f" (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, kernels {ksha[:12]})"
    return None, f"no PMC summary of this build's kernels ({ksha[:12]}) under profiles/"


def h2d_link_peak(dev, nbytes=1 << 30, reps=4):
    """Pinned host -> device copy rate (GB/s) of this box's link."""
    try:
        a = torch.empty(nbytes // 8, dtype=torch.int64).pin_memory()
        b = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
        b.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            b.copy_(a, non_blocking=True)
        torch.cuda.synchronize()
        return nbytes * reps / (time.perf_counter() - t0) / 1e9
    except RuntimeError:
        return None


def h2d_leg(args, wl, window, aggs, expected_keys, dev):
    """SURVEY.md 8(d)'s contract timing: the kernels PLUS the H2D of columnar batches from
    pinned host memory. The whole configs[1] job (`h2d_records`, default all 1B records) as
    pinned host columns handed over as FG_HOST batches: whole-job rate including PCIe, the link
    bytes, and the link's measured pinned H2D rate."""
    import flink_amd as F
    n = args.h2d_records - args.h2d_records % args.batch or args.batch
    hk = torch.empty(n, dtype=torch.int64).pin_memory()
    ht = torch.empty(n, dtype=torch.int64).pin_memory()
    hv = torch.empty(n, dtype=torch.float64).pin_memory()
    chunk = 1 << 27
    for lo in range(0, n, chunk):   # generated on the GPU, copied into the pinned columns
        hi = min(n, lo + chunk)
        k, t, v = gen_columns(hi - lo, args.keys, args.rate, lo, dev, jitter=wl["jitter"], zipf=wl["zipf"], t_base=0)
        hk[lo:hi].copy_(k)
        ht[lo:hi].copy_(t)
        hv[lo:hi].copy_(v)
        del k, t, v
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    op = F.WindowAggOperator(window, aggs=aggs, val_type="f64", expected_keys=expected_keys,
                             buffer_records=max(4 * args.batch, 1 << 26), device=dev.index)
    # the narrow form a shim hands when its keys fit 32 bits (fg_batch.format): int32 keys and
    # rowtime offsets from each micro-batch's first rowtime -- 16 B per record over the link
    nk = nt = bases = None
    if args.keys < (1 << 31):
        nk = torch.empty(n, dtype=torch.int32).pin_memory()
        nt = torch.empty(n, dtype=torch.int32).pin_memory()
        bases = []
        for lo in range(0, n, args.batch):
            hi = min(n, lo + args.batch)
            base = int(ht[lo:hi].min())
            bases.append(base)
            nk[lo:hi].copy_(hk[lo:hi])
            nt[lo:hi].copy_((ht[lo:hi] - base).to(torch.int32))   # (uint32 offsets: < 2^31 here)

    def run(narrow):
        op.reset()
        rows0 = op.stats()["rows_fired"]
        for bi, lo in enumerate(range(0, n, args.batch)):
            hi = min(n, lo + args.batch)
            if narrow:
                op.process_batch(nk[lo:hi], nt[lo:hi].numpy().view("uint32"), hv[lo:hi], rowtime_base=bases[bi])
            else:
                op.process_batch(hk[lo:hi], ht[lo:hi], hv[lo:hi])
            if bi > 0 and not args.wm_sync:   # the previous batch's held watermarks (as in one_step)
                op.collect_fired()
            for wm in watermarks_for(lo, hi, args.rate, args.wm_every, wl["delay"], wl["jitter"]):
                op.process_watermark(wm, device_output=True, wait=args.wm_sync)
        if not args.wm_sync:
            op.collect_fired()
        op.process_watermark(JMAX, device_output=True)
        op.synchronize()
        return op.stats()["rows_fired"] - rows0

    def timed(narrow):
        run(narrow)   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rows = run(narrow)
        return rows, time.perf_counter() - t0
    rows, el = timed(False)
    narrow = None
    if nk is not None:
        nrows, nel = timed(True)
        assert nrows == rows, (nrows, rows)
        narrow = {"value": n / nel, "seconds": nel, "pcie_gbs": 16 * n / nel / 1e9, "bytes_per_record": 16,
                  "note": "the same job as narrow FG_HOST batches (fg_batch.format: int32 keys, rowtime as uint32 "
                          "offsets from the batch's first rowtime, widened on the device)"}
    op.close()
    del hk, ht, hv, nk, nt
    link = h2d_link_peak(dev)
    gbs = 24 * n / el / 1e9
    return {"value": n / el, "unit": "records/s", "records": n, "rows_fired": rows, "seconds": el,
            "pcie_gbs": gbs, "link_peak_gbs": link, "link_frac": gbs / link if link else None,
            "job_roofline_frac": (24 * n + 48 * rows) / el / (HBM_PEAK_GBS * 1e9),
            "narrow": narrow,
            "note": "SURVEY 8(d) contract timing (kernels + H2D of columnar batches from pinned host memory): the "
                    "configs[1] job as FG_HOST batches (double-buffered H2D on the engine's copy stream, "
                    "overlapping the kernels; each call returns once its batch is copied). `value` is the "
                    "kernel pipeline with the inputs resident in HBM"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--records", type=int, default=None, help="records per GPU per step (default: 1B; "
                    "configs[0]: 10M)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="tumble",
                    help="BASELINE config; `tumble` (configs[1]) is the bench's headline value")
    ap.add_argument("--keys", type=int, default=None, help="key space (default: the workload's)")
    ap.add_argument("--rate", type=int, default=None, help="records per event-second (default: the workload's)")
    ap.add_argument("--batch", type=int, default=None,
                    help="micro-batch records (default 50M; hop 25M and cumulate one event-minute (16.7M) so that a "
                         "micro-batch spans at most two 1-minute slices, the staged lanes of a 10M-key operator)")
    ap.add_argument("--wm-every", type=int, default=None, help="records between watermarks (default 1M; "
                    "configs[0]: 10k)")
    ap.add_argument("--checkpoint-every", type=int, default=None,
                    help="micro-batches between checkpoints (prepareSnapshotPreBarrier flush + state image to "
                         "host); default: the zipf workload (configs[4]) checkpoints once per step, others never")
    ap.add_argument("--aggs", default=None, help="comma-separated aggregate list (default: the workload's), "
                    "e.g. count_star,min")
    ap.add_argument("--sync-snapshot", action="store_true",
                    help="checkpoints copy the state image to the host inside snapshotState (A/B; default: "
                         "fg_snapshot_state_async, the copy overlapping the next micro-batches, collected in the step)")
    ap.add_argument("--jitter", type=int, default=None, help="rowtime jitter ms (diagnostic override of the workload's; "
                    "the watermark delay follows it)")
    ap.add_argument("--zipf", type=float, default=None, help="Zipf exponent (diagnostic override; 0 = uniform keys)")
    ap.add_argument("--expected-keys", type=int, default=None,
                    help="operator sizing hint: distinct keys per slice (default: the key space x 1.05)")
    ap.add_argument("--wm-sync", action="store_true",
                    help="deliver watermarks with the synchronous fg_advance_progress (A/B; default: "
                         "fg_advance_progress_async, the host does not wait for a window's fire)")
    ap.add_argument("--intern-at", choices=["batch", "fires"], default="batch",
                    help="STRING keys: launch the next batch's lookup before this batch is handed over "
                         "(beside pass 1) or after its watermarks (beside the fires)")
    ap.add_argument("--intern-serial", action="store_true",
                    help="strings: intern the next micro-batch after the engine's passes instead of beside them (A/B)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-max-records", type=int, default=200_000_000)
    ap.add_argument("--host-input", action="store_true",
                    help="hand the engine pinned host columns (PCIe-inclusive rate; never the headline value)")
    ap.add_argument("--exchange", choices=("partials", "raw"), default="partials",
                    help="N > 1: exchange partial accumulators (two-phase) or raw records")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline instances (default: min(85, CPUs in this process's affinity mask))")
    ap.add_argument("--h2d-records", type=int, default=1_000_000_000,
                    help="records of the pinned-host leg (SURVEY 8(d) contract timing: FG_HOST batches, "
                         "double-buffered H2D overlapping the kernels); 0 skips it. Never the headline value")
    args = ap.parse_args()
    wl = dict(WORKLOADS[args.workload])
    if args.jitter is not None:
        wl["jitter"] = wl["delay"] = args.jitter
    if args.zipf is not None:
        wl["zipf"] = args.zipf
    keys_default = args.keys is None
    if args.keys is None:
        args.keys = wl["keys"]
    if args.rate is None:
        args.rate = wl["rate"]
    if args.batch is None:
        args.batch = wl.get("batch", 50_000_000)
    if args.records is None:
        args.records = wl.get("records", 1_000_000_000)
    if args.wm_every is None:
        args.wm_every = wl.get("wm_every", 1_000_000)
    datastream = wl.get("mode") == "datastream"
    if args.workload != "tumble":
        args.no_cpu_baseline = True   # the CPU baseline is quoted on configs[1]
    if args.checkpoint_every is None:
        # configs[4] checkpoints every 10 s; a step is 1B records = 10 event-seconds at the
        # workload's 100M records per event-second, and its wall time is well under 10 s: one
        # checkpoint per step (at its middle micro-batch: each step restarts at batch 0) is as
        # often as the config asks, or more
        nb = -(-args.records // args.batch)
        args.checkpoint_every = max(1, nb // 2) if args.workload == "zipf" else 0

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if keys_default and wl.get("keys_per_gpu"):   # configs[3]: 12.5M keys per GPU, 100M at N = 8
        args.keys *= world
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = int(os.environ.get("BENCH_DEVICE", local))   # rehearsal: every rank on one device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    # BENCH_DIST_BACKEND=gloo rehearses N > 1 on one device (collectives staged through
    # host memory); the driver's multi-GPU runs use RCCL ("nccl")
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    via_cpu = backend == "gloo"
    if world > 1:
        import torch.distributed as dist
        if via_cpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    import flink_amd as F
    from flink_amd.exchange import exchange, global_watermark

    n = args.records
    key, ts, val = gen_columns(n, args.keys, args.rate, rank * n, dev, jitter=wl["jitter"], zipf=wl["zipf"])
    if datastream:   # Tuple2<Long, Long>: long values in [0, 1000)
        val = val.to(torch.int64)
    strings = args.workload == "strings"
    kdict = None
    if strings:   # key rows instead of BIGINT keys; the dictionary outlives the steps (as in a job)
        rows_u8 = string_key_rows(key).view(torch.uint8).reshape(-1)
        del key
        key = None
        row_off = torch.arange(args.batch, dtype=torch.int64, device=dev) * 32
        row_len = torch.full((args.batch,), 32, dtype=torch.int32, device=dev)
        kdict = F.KeyDictionary(max_parallelism=128, expected_keys=int(args.keys * 1.05), device=local)
        kdict.set_timing(True)   # the dictionary's kernels are timed on its own stream
        if world > 1 and args.exchange == "raw":
            # a rank's dictionary ids are its own: records would have to carry their key rows;
            # the two-phase plan ships each partial row's key row (exchange_partials key_rows)
            raise SystemExit("--workload strings at N > 1 runs the two-phase plan (--exchange partials)")
    from flink_amd import _lib as FL
    key_hash = FL.KEYHASH_DICT_ID if strings else FL.KEYHASH_BINARYROW_BIGINT
    torch.cuda.synchronize()
    if args.host_input:   # FG_HOST columns: the engine copies each micro-batch H2D on its stream
        key, ts, val = (x.cpu().pin_memory() for x in (key, ts, val))

    maxp = 128
    kg_lo, kg_hi = (rank * maxp + world - 1) // world, ((rank + 1) * maxp - 1) // world
    two_phase = world > 1 and args.exchange == "partials" and not datastream
    wname, *wargs = wl["window"]
    window = getattr(F, wname)(*wargs)
    expected_keys = args.expected_keys or int(args.keys / world * 1.05) + 1
    if not args.expected_keys and wl["zipf"] > 0:   # distinct keys in one slice's records, +10 %
        # each rank draws `rate` records per event-second, so an owner's slice holds the keys
        # of world * rate draws, split over the world owners
        expected_keys = int(1.1 * zipf_distinct_per_slice(args.keys, wl["zipf"], args.rate * world) / world) + 1
    aggs = ("avg",) if args.workload == "zipf" else ("sum",) if datastream else ("count_star", "sum", "avg")
    if args.aggs:
        aggs = tuple(args.aggs.split(","))
    op = F.WindowAggOperator(window, aggs=aggs, val_type="i64" if datastream else "f64",
                             mode="datastream" if datastream else "sql",
                             expected_keys=expected_keys,
                             buffer_records=max(4 * args.batch, 1 << 26) if not two_phase else 1 << 24,
                             device=local, key_group_range=(kg_lo, kg_hi), kernel_timing=True)
    # two-phase: the local operator sees every key of its source partition
    op_local = F.WindowAggOperator(window, aggs=aggs, val_type="f64", expected_keys=int(args.keys * 1.05) + 1,
                                   buffer_records=max(4 * args.batch, 1 << 26), device=local,
                                   kernel_timing=True, local_partials=True) if two_phase else None

    # STRING keys over the exchange: the owner's dictionary interns the key rows the partial
    # rows carry (a rank's local ids mean nothing elsewhere)
    kdict_owner = F.KeyDictionary(max_parallelism=128, expected_keys=int(args.keys / world * 1.05) + 1,
                                  device=local) if strings and two_phase else None

    tp = TwoPhase(op_local, op, dev, maxp, key_hash, via_cpu,
                  key_rows=(kdict, kdict_owner) if kdict_owner else None) if two_phase else None

    ckpt = dict(n=0, s=0.0, state_rows=0)

    def checkpoint():
        """CheckpointedFunction path of the window operator: prepareSnapshotPreBarrier flushes
        the staged records into the GPU-resident state, snapshotState copies the window-aggs
        image (key, slice_end, accumulators) to host memory for the keyed state backend.
        Two-phase: the local buffer's partial rows go through the exchange first (TwoPhase.checkpoint).
        Returns (rows collected, bytes sent). (No device-wide synchronization first: the engine
        orders the flush after the work queued before it, and a barrier drains no GPU pipeline;
        avg_ms is the host time of the calls.)"""
        c0 = time.perf_counter()
        if tp is not None:
            snapshot_collect()
            got, sent, image = tp.checkpoint(asynchronous=not args.sync_snapshot)
            if image is None:
                ckpt["pending"] = True
            else:
                ckpt["state_rows"] += len(image[0]["key"])
        else:
            got, sent = 0, 0
            snapshot_collect()
            op.prepare_snapshot_pre_barrier()
            if args.sync_snapshot:
                img, _ = op.snapshot_state(copy=False)   # the pinned image a JNI shim hands to the backend
                ckpt["state_rows"] += len(img["key"])
            else:   # the synchronous part; the image's copy to the host overlaps the next batches
                op.snapshot_state_async()
                ckpt["pending"] = True
        ckpt["n"] += 1
        ckpt["s"] += time.perf_counter() - c0
        return got, sent

    def snapshot_collect():
        """snapshotState's asynchronous part: the host image of the pending snapshot (the state
        backend takes it) -- at the next checkpoint, or after the last step; the timed region
        pays for every copy"""
        if ckpt.pop("pending", False):
            c0 = time.perf_counter()
            img, _ = tp.snapshot_wait() if tp is not None else op.snapshot_state_wait(copy=False)
            ckpt["state_rows"] += len(img["key"])
            ckpt["s"] += time.perf_counter() - c0

    def intern(lo):
        """BinaryRowDataKeySelector.getKey rows -> dictionary ids (on the GPU, the dictionary's
        own stream); the call returns with the ids complete"""
        hi = min(n, lo + args.batch)
        k, _ = kdict.intern(packed=(rows_u8[32 * lo:32 * hi], row_off[:hi - lo], row_len[:hi - lo]),
                            key_groups=False)
        return k

    def intern_async(lo):
        """the same, launched (fg_key_dict_intern_async): the ids are complete after intern_wait"""
        hi = min(n, lo + args.batch)
        k, _ = kdict.intern_async((rows_u8[32 * lo:32 * hi], row_off[:hi - lo], row_len[:hi - lo]))
        return k

    def one_step():
        op.reset()
        rows0 = op.stats()["rows_fired"]
        if op_local:
            op_local.reset()
        rows = 0
        xgmi = 0
        # async watermarks (the default): a batch's watermarks are held until the next batch has
        # been handed over, then their fired rows are collected (fg_collect_fired) -- the fires
        # complete while the next batch's pass 1 is queued, so the host never waits on a merge
        held = False
        # STRING keys: the next micro-batch's key rows are interned while the engine aggregates
        # the current one (the key selector runs as records arrive, ahead of the operator; the
        # dictionary assigns ids in the same first-seen order)
        k_next = intern(0) if strings else None
        for bi, lo in enumerate(range(0, n, args.batch)):
            if args.checkpoint_every and bi > 0 and bi % args.checkpoint_every == 0:
                if held and tp is None:   # the rows go out before the checkpoint barrier
                    rows += op.collect_fired().n
                    held = False
                nr, sent = checkpoint()
                rows += nr
                xgmi += sent
            hi = min(n, lo + args.batch)
            if strings:
                k = k_next
            else:
                k = key[lo:hi]
            t, v = ts[lo:hi], val[lo:hi]
            wms = watermarks_for(lo, hi, args.rate, args.wm_every, wl["delay"], wl["jitter"])
            if strings and hi < n and not two_phase and not args.intern_serial and args.intern_at == "batch":
                # the next micro-batch's lookup runs beside this batch's passes and fires
                k_next = intern_async(hi)
            if two_phase:
                op_local.process_batch(k, t, v)
                if strings and hi < n:
                    k_next = intern(hi)
                if wms:   # every watermark of the micro-batch to the local operator, one exchange
                    nr, sent = tp.round(wms)
                    rows += nr
                    xgmi += sent
                continue
            if world > 1:
                k, t, v2, sent = exchange(k, t, v.view(torch.int64), max_parallelism=maxp, key_hash=key_hash)
                v = v2.view(v.dtype)
                xgmi += sent
                torch.cuda.current_stream().synchronize()
            op.process_batch(k, t, v)
            if held:   # the previous batch's watermarks: their rows, then (a shim) the watermarks go on
                rows += op.collect_fired().n
                held = False
            if world > 1 and wms:
                wms[-1] = global_watermark(wms[-1], device=dev)
            if args.wm_sync:
                for wm in wms:
                    rows += op.process_watermark(wm, device_output=True).n
            elif wms:   # fg_advance_progress_async_n: every watermark's fires queued, the watermarks held
                op.process_watermarks(wms)
                held = True
            # STRING keys: the next micro-batch's lookup (launched above on the dictionary's own
            # stream) ran beside this batch's passes and the fires its watermarks queued; its ids
            # are complete before the next batch is handed over (the key selector runs as the
            # records arrive)
            if strings and hi < n:
                if args.intern_serial:   # A/B: the lookup after them (the dictionary's stream waits
                    # on torch's, which here waits on the engine's)
                    torch.cuda.current_stream().wait_stream(torch.cuda.ExternalStream(op.stream, device=dev))
                    k_next = intern(hi)
                else:
                    if args.intern_at == "fires":
                        k_next = intern_async(hi)
                    kdict.intern_wait()
        if two_phase:
            nr, sent = tp.finish()
            return rows + nr, xgmi + sent
        if held:
            rows += op.collect_fired().n
        r = op.process_watermark(JMAX, device_output=True)
        rows += r.n
        assert args.wm_sync or rows == op.stats()["rows_fired"] - rows0
        return rows, xgmi

    def kstats():
        ks = op.kernel_stats()
        if op_local:   # local-phase kernels under their own names
            for name, d in op_local.kernel_stats().items():
                ks["local_" + name] = d
        if kdict is not None:   # the dictionary's kernels, timed on its stream
            ks.update(kdict.kernel_stats())
        return ks

    pre_last = kstats()
    for i in range(args.warmup):
        if i == args.warmup - 1:
            op.synchronize()
            pre_last = kstats()
        one_step()
    snapshot_collect()
    op.synchronize()
    # every kernel class is timed in the warmup; the timed region brackets only the dominant
    # one with HIP events (two events per launch perturb the stream: timing every class costs
    # 0.4-0.9 ms per step), so `value` and the reported kernel both come from the timed region.
    # The dominant class is the LAST warmup step's (a one-time cost of the first step -- a
    # dictionary filling up, a staging mode given up -- would name a class the steady state
    # never launches); the reported per-step warmup figures stay over all warmup steps
    last = kstats()
    warm = {}
    for k, v in last.items():
        b = pre_last.get(k, dict(launches=0, total_ms=0.0, records=0, rows=0))
        if v["launches"] - b["launches"] > 0:
            warm[k] = {f: v[f] - b[f] for f in ("launches", "total_ms", "records", "rows")}
    dom_class = max(warm.items(), key=lambda kv: kv[1]["total_ms"])[0] if warm else None
    if dom_class and args.warmup > 0:
        is_local = dom_class.startswith("local_")
        is_dict = dom_class.startswith("dict_")   # the dictionary keeps its own (per-chunk) events
        op.set_kernel_timing([] if is_local or is_dict else [dom_class])
        if op_local is not None:
            op_local.set_kernel_timing([dom_class[len("local_"):]] if is_local else [])
    before = kstats()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ckpt.update(n=0, s=0.0, state_rows=0)
    t0 = time.perf_counter()
    tot_rows = 0
    tot_xgmi = 0
    for _ in range(args.steps):
        rows, xg = one_step()
        tot_rows += rows
        tot_xgmi += xg
    # the last checkpoint's image (each earlier one was collected by the next checkpoint: the async
    # part of a snapshot completes while the job runs on, as a heap backend's AsyncSnapshotCallable
    # does); inside the timed region
    snapshot_collect()
    op.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    after = kstats()
    late = op.num_late_records_dropped
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        rr = torch.tensor([tot_rows, late], dtype=torch.int64, device=dev)
        dist.all_reduce(rr)
        tot_rows, late = int(rr[0].item()), int(rr[1].item())

    # per-kernel accounting over the timed region
    ks = {}
    for name, a in after.items():
        b = before.get(name, dict(launches=0, total_ms=0.0, records=0, rows=0))
        d = {k: a[k] - b[k] for k in ("launches", "total_ms", "records", "rows")}
        if d["launches"] > 0:
            ks[name] = d
    if not any(v["total_ms"] > 0 for v in ks.values()):   # kernel timing off (FG_KERNEL_TIMING=0 A/B)
        ks = {"untimed": dict(launches=1, total_ms=float("nan"), records=0, rows=0)}
    dom_name, dom = max(ks.items(), key=lambda kv: kv[1]["total_ms"])
    avg_s = dom["total_ms"] / dom["launches"] / 1e3
    # algorithmic bytes: 24 B per input record + 48 B per fired row; the key
    # dictionary's probe: the 32-B key row read + the 8-B id written per row
    alg_bytes = ((40 if dom_name.startswith("dict_") else 24) * dom["records"] + 48 * dom["rows"]) / dom["launches"]
    achieved = alg_bytes / avg_s / 1e9
    traffic, traffic_src = pmc_traffic(dom_name, args.workload)

    copy_gbs = measure_copy_peak(dev)
    total_records = world * n * args.steps
    value = total_records / el
    b_alg = 24 * total_records + 48 * tot_rows
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64" if datastream else "f64",
        "data": "synthetic (counter-based splitmix64 stream generated on the GPU, " + (
            "handed over as pinned host columns: PCIe-inclusive)" if args.host_input else "resident in HBM)"),
        "config": {
            "workload": wl["desc"],
            "records_per_gpu": n, "keys": args.keys, "records_per_event_second": args.rate,
            "micro_batch": args.batch, "watermark_every": args.wm_every, "expected_keys": expected_keys,
            "jitter_ms": wl["jitter"], "zipf_s": wl["zipf"],
            "parallelism": f"key-group sharded x{world}" + (
                (" + RCCL all-to-all of partial accumulators (two-phase)" if two_phase else
                 " + RCCL all-to-all of records") if world > 1 else ""),
        },
        # the dominant kernel (task contract): algorithmic bytes per launch / its HIP-event duration
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "kernel_frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": dom_name,
                     "avg_launch_ms": avg_s * 1e3,
                     "alg_bytes_per_launch": alg_bytes,
                     # SURVEY.md 8d second denominator: a device-to-device copy measured on this box
                     "copy_peak_gbs": copy_gbs,
                     "frac_of_copy_peak": achieved / copy_gbs if copy_gbs else None,
                     "actual_gbs": traffic / avg_s / 1e9 if traffic else None},
        # the whole job: B_alg = 24 B per record + 48 B per
        # fired row over the wall time of the timed steps, against N x 8 TB/s -- the north-star figure
        "job_roofline": {"achieved": b_alg / el / 1e9, "peak": world * HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": b_alg / el / (world * HBM_PEAK_GBS * 1e9), "b_alg_bytes": b_alg},
        "job_roofline_frac": b_alg / el / (world * HBM_PEAK_GBS * 1e9),
        "rows_fired": tot_rows,
        "late_dropped": late,
        "xgmi_bytes_sent_rank0": tot_xgmi,
        # checkpoints inside the timed region (rank 0): count, mean wall ms, state rows imaged
        "checkpoints": {"count": ckpt["n"], "avg_ms": ckpt["s"] / ckpt["n"] * 1e3 if ckpt["n"] else None,
                        "state_rows": ckpt["state_rows"]},
        "kernels": {k: dict(v, avg_ms=v["total_ms"] / v["launches"]) for k, v in ks.items()},
        # every class, timed in the last warmup step (one step of the steady state)
        "kernels_warmup": {k: dict(v, avg_ms=v["total_ms"] / v["launches"]) for k, v in warm.items()},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.h2d_records > 0 and not args.host_input and args.workload == "tumble":
        # secondary: the same workload handed over as pinned host columns (the FG_HOST
        # boundary a JNI shim uses), H2D double-buffered on the engine's copy stream
        op.close()
        del key, ts, val
        torch.cuda.empty_cache()
        result["h2d"] = h2d_leg(args, wl, window, aggs, expected_keys, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(args, args.rate // 1000)
        except Exception as e:  # reported, not fatal
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    op.close()   # (idempotent)
    if op_local:
        op_local.close()
    if kdict is not None:
        result["key_dictionary"] = {"distinct_keys": len(kdict), "row_bytes": 32}
        kdict.close()
    if kdict_owner is not None:
        kdict_owner.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
