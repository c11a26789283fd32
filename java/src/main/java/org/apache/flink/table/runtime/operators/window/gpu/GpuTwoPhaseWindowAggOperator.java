/*
 * The two-phase window aggregation of one GPU subtask, fused: LocalSlicingWindowAggOperator, the
 * keyBy network edge and GlobalSlicingWindowAggOperator (TwoStageOptimizedWindowAggregateRule.java:
 * 81-104) become ONE operator per subtask, placed where the local operator would run (before the
 * keyBy: its input is not keyed). The edge is an RCCL all-to-all between the subtasks' GPUs over xGMI
 * (fg_comm, include/flinkgpu.h) instead of KeyGroupStreamPartitioner.selectChannel
 * (KeyGroupStreamPartitioner.java:55-65) + Netty.
 *
 * A collective needs every subtask to take part the same number of times, and watermarks do not
 * arrive at the subtasks in step, so the task thread never drives the exchange. An EDGE THREAD per
 * subtask exchanges in rounds until every subtask has reached the end of its input:
 *
 *   commRoundBegin    [under the lock] the local handle's uncollected async fires (ROUND_FIRED), its
 *                     whole buffer before a checkpoint barrier (ROUND_FLUSHED), or nothing
 *                     (ROUND_IDLE), grouped by key-group owner on the GPU, with this subtask's
 *                     watermark and epoch (the last checkpoint id whose pre-barrier rows it sent)
 *   commRoundExchange [no lock: waits for the peers] one all-to-all of (rows, watermark, epoch,
 *                     failure) per peer, then the rows; a round that failed on any subtask fails on all
 *   commRoundEnd      [under the lock] the received partial rows merged into the global handle
 *                     (GlobalAggCombiner.combine); the global advanced to the minimum watermark
 *                     (StatusWatermarkValve) -- its fires queued; a mail to the task thread emits
 *                     their rows and then forwards that watermark downstream
 *
 * Checkpoints are aligned across the edge as the reference aligns barriers on the global operator's
 * input channels: prepareSnapshotPreBarrier asks for the local buffer's flush in the next round
 * (LocalSlicingWindowAggOperator.prepareSnapshotPreBarrier :142-144) and blocks the task thread
 * until a round's minimum epoch reaches the checkpoint id -- every subtask has sent its pre-barrier
 * rows -- then emits the global's rows and takes its image (snapshotStateAsync) before the edge
 * merges another round. A subtask blocked at its barrier processes no post-barrier record, so no
 * post-barrier row reaches an image. The operator is not keyed, so the images are union operator
 * state; on restore every subtask keeps the entries of its own key groups (a rescale works the same).
 *
 * The communicator: subtask 0 makes the id (commUniqueId) and sends it to GpuCommCoordinator, which
 * forwards it to every subtask; the edge thread opens the communicator when the id arrives
 * (commOpen blocks until every subtask joined) while the task thread goes on taking records. The
 * coordinator fails the job when a subtask fails (the collectives join every subtask).
 *
 * BIGINT grouping keys (the C-ABI edge moves the keys themselves: per-subtask dictionary ids of
 * other key types mean nothing on another subtask -- the planner keeps the reference's two operators
 * for those). Python mirror: flink_amd/two_phase.py (TwoPhaseSubtask), tested at world size 2.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.api.common.operators.MailboxExecutor;
import org.apache.flink.api.common.state.ListState;
import org.apache.flink.api.common.state.ListStateDescriptor;
import org.apache.flink.api.common.typeutils.base.array.BytePrimitiveArraySerializer;
import org.apache.flink.runtime.operators.coordination.OperatorEvent;
import org.apache.flink.runtime.operators.coordination.OperatorEventGateway;
import org.apache.flink.runtime.operators.coordination.OperatorEventHandler;
import org.apache.flink.runtime.state.KeyGroupRange;
import org.apache.flink.runtime.state.KeyGroupRangeAssignment;
import org.apache.flink.runtime.state.StateInitializationContext;
import org.apache.flink.runtime.state.StateSnapshotContext;
import org.apache.flink.streaming.api.operators.BoundedOneInput;
import org.apache.flink.streaming.api.operators.OneInputStreamOperator;
import org.apache.flink.streaming.api.operators.TimestampedCollector;
import org.apache.flink.streaming.api.watermark.Watermark;
import org.apache.flink.streaming.runtime.streamrecord.StreamRecord;
import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.data.TimestampData;
import org.apache.flink.table.data.utils.JoinedRowData;
import org.apache.flink.table.runtime.keyselector.RowDataKeySelector;
import org.apache.flink.table.runtime.operators.TableStreamOperator;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.List;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.locks.Condition;
import java.util.concurrent.locks.ReentrantLock;

/** Local phase, RCCL keyBy edge and global phase of one GPU subtask. */
public final class GpuTwoPhaseWindowAggOperator extends TableStreamOperator<RowData>
        implements OneInputStreamOperator<RowData, RowData>, BoundedOneInput, OperatorEventHandler {
    private static final long serialVersionUID = 1L;
    private static final String IMAGE_STATE = "gpu-window-aggs-image";
    private static final int IMAGE_CHUNK_ROWS = 1 << 16;   // rows per union-state chunk (56 B each)
    private static final long IDLE_SLEEP_MS = 1;

    private final GpuWindowAggSpec spec;   // the aggregation: the local handle adds FLAG_LOCAL_PARTIALS
    private final RowDataKeySelector keySelector;
    private transient OperatorEventGateway eventGateway;
    private transient MailboxExecutor mailbox;

    private transient int maxP, parallelism, index;
    private transient long local, global;
    private transient GpuKeyRows keys;
    private transient GpuAccRows accRows;
    private transient ByteBuffer keyCol, timeCol, valCol, nullCol;
    private transient int count;
    private transient TimestampedCollector<RowData> collector;
    private transient ListState<byte[]> imageState;
    private transient List<byte[]> restoredImage;

    // ---- the edge (guarded by lock) ----
    private transient ReentrantLock lock;
    private transient Condition changed;
    private transient Thread edge;
    private transient byte[] commId;
    private transient long comm;
    private transient long wmLocal, globWm, forwarded;
    private transient long flushReq, sentEpoch, aligned, snapDone;
    private transient boolean dirty, closing, pendingFires;
    private transient Throwable edgeError;
    private transient byte[][] snapshotImage;   // chunks of the image taken at the last barrier

    public GpuTwoPhaseWindowAggOperator(GpuWindowAggSpec spec, RowDataKeySelector keySelector) {
        if (!spec.bigintKey) {
            throw new IllegalArgumentException("the RCCL edge moves BIGINT grouping keys only");
        }
        this.spec = spec;
        this.keySelector = keySelector;
    }

    void setOperatorEventGateway(OperatorEventGateway gateway) {
        this.eventGateway = gateway;
    }

    void setMailboxExecutor(MailboxExecutor mailbox) {
        this.mailbox = mailbox;
    }

    // ---- lifecycle -------------------------------------------------------------------------------

    @Override
    public void initializeState(StateInitializationContext context) throws Exception {
        super.initializeState(context);
        imageState =
                context.getOperatorStateStore()
                        .getUnionListState(new ListStateDescriptor<>(IMAGE_STATE, BytePrimitiveArraySerializer.INSTANCE));
        restoredImage = new ArrayList<>();
        if (context.isRestored()) {
            for (byte[] chunk : imageState.get()) {
                restoredImage.add(chunk);
            }
        }
    }

    @Override
    public void open() throws Exception {
        super.open();
        collector = new TimestampedCollector<>(output);
        collector.eraseTimestamp();
        maxP = getRuntimeContext().getMaxNumberOfParallelSubtasks();
        parallelism = getRuntimeContext().getNumberOfParallelSubtasks();
        index = getRuntimeContext().getIndexOfThisSubtask();
        KeyGroupRange range = KeyGroupRangeAssignment.computeKeyGroupRangeForOperatorIndex(maxP, parallelism, index);
        GpuWindowAggSpec ls = spec.copy();
        ls.flags |= FgConfig.FLAG_LOCAL_PARTIALS;
        int nTz = spec.tzTransitionsMs == null ? 0 : spec.tzTransitionsMs.length;
        local = FlinkGpu.open(FgConfig.of(ls, maxP, 0, maxP - 1, nTz), spec.tzTransitionsMs, spec.tzOffsetsMs);
        global =
                FlinkGpu.open(
                        FgConfig.of(spec, maxP, range.getStartKeyGroup(), range.getEndKeyGroup(), nTz),
                        spec.tzTransitionsMs,
                        spec.tzOffsetsMs);
        keys = new GpuKeyRows(spec, maxP);
        accRows = new GpuAccRows(spec.aggs, spec.valType);
        int b = spec.batchRecords;
        keyCol = GpuKeyRows.direct(8L * b);
        timeCol = GpuKeyRows.direct(8L * b);
        valCol = GpuKeyRows.direct(8L * b);
        nullCol = GpuKeyRows.direct(b);
        for (ByteBuffer c : new ByteBuffer[] {keyCol, timeCol, valCol, nullCol}) {
            FlinkGpu.hostRegister(spec.device, c);
        }
        restoreGlobal(range);
        lock = new ReentrantLock();
        changed = lock.newCondition();
        wmLocal = globWm = forwarded = Long.MIN_VALUE;
        flushReq = sentEpoch = aligned = snapDone = 0;
        edge = new Thread(this::runEdge, "gpu-window-edge-" + index);
        edge.setDaemon(true);
        edge.start();
        if (index == 0) {   // subtask 0 makes the communicator id; the coordinator forwards it
            ByteBuffer id = GpuKeyRows.direct(FlinkGpu.COMM_ID_BYTES);
            FlinkGpu.commUniqueId(id);
            byte[] bytes = new byte[FlinkGpu.COMM_ID_BYTES];
            id.get(bytes);
            eventGateway.sendEventToCoordinator(new GpuCommIdEvent(bytes, getRuntimeContext().getAttemptNumber()));
        }
    }

    @Override
    public void handleOperatorEvent(OperatorEvent evt) {
        if (evt instanceof GpuCommIdEvent
                && ((GpuCommIdEvent) evt).attempt() == getRuntimeContext().getAttemptNumber()) {
            lock.lock();
            try {
                commId = ((GpuCommIdEvent) evt).id();
                changed.signalAll();
            } finally {
                lock.unlock();
            }
        }
    }

    // ---- the task thread ---------------------------------------------------------------------------

    private void check() {
        if (edgeError != null) {
            throw new RuntimeException("the GPU window aggregation's RCCL edge failed", edgeError);
        }
    }

    @Override
    public void processElement(StreamRecord<RowData> element) throws Exception {
        RowData row = element.getValue();
        RowData key = keySelector.getKey(row);
        keys.add(key, count, keyCol);
        timeCol.putLong(8 * count, row.getTimestamp(spec.rowtimeIndex, 3).getMillisecond());
        if (spec.valueIndex >= 0) {
            boolean isNull = row.isNullAt(spec.valueIndex);
            nullCol.put(count, (byte) (isNull ? 1 : 0));
            valCol.putLong(
                    8 * count,
                    isNull ? 0L
                            : spec.valType == FgConfig.VAL_F64
                                    ? Double.doubleToRawLongBits(row.getDouble(spec.valueIndex))
                                    : row.getLong(spec.valueIndex));
        }
        if (++count == spec.batchRecords) {
            flushBatch();
        }
    }

    /** the gathered micro-batch to the local handle (which has read it when this returns) */
    private void flushBatch() {
        if (count == 0) {
            return;
        }
        lock.lock();
        try {
            check();
            FlinkGpu.addBatch(
                    local,
                    keyCol,
                    timeCol,
                    spec.valueIndex >= 0 ? valCol : null,
                    spec.valueIndex >= 0 ? nullCol : null,
                    count);
            count = 0;
        } finally {
            lock.unlock();
        }
    }

    /**
     * LocalSlicingWindowAggOperator.processWatermark (:121-134): the local fires are queued; their
     * partial rows leave with the next round. The watermark itself is not forwarded here: downstream
     * sees the global's combined watermark (emitGlobal), as behind the reference's global operator.
     */
    @Override
    public void processWatermark(Watermark mark) throws Exception {
        flushBatch();
        lock.lock();
        try {
            check();
            if (mark.getTimestamp() > wmLocal) {
                FlinkGpu.advanceProgressAsync(local, mark.getTimestamp());
                wmLocal = mark.getTimestamp();
                dirty = true;
                changed.signalAll();
            }
        } finally {
            lock.unlock();
        }
    }

    /** the mail the edge posts after a round advanced the global: its rows, then its watermark */
    private void emitGlobal() throws Exception {
        long wm;
        lock.lock();
        try {
            check();
            if (pendingFires) {
                pendingFires = false;
                ByteBuffer[] cols = new ByteBuffer[5 + spec.aggs.length];
                emit(cols, FlinkGpu.collectFired(global, cols));
            }
            wm = globWm > forwarded ? globWm : Long.MIN_VALUE;
            if (wm != Long.MIN_VALUE) {
                forwarded = wm;
            }
        } finally {
            lock.unlock();
        }
        if (wm != Long.MIN_VALUE) {
            super.processWatermark(new Watermark(wm));
        }
    }

    /** fired rows -> JoinedRowData(key, [aggs..., window_start, window_end]) */
    private void emit(ByteBuffer[] cols, long n) {
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        int nAggs = spec.aggs.length;
        RowData[] keyRows = keys.rows(cols[0], (int) n);
        for (int i = 0; i < n; i++) {
            byte nullMask = cols[3 + nAggs].get(i);
            GenericRowData aggs = new GenericRowData(nAggs + 2);
            for (int a = 0; a < nAggs; a++) {
                if ((nullMask >> a & 1) != 0) {
                    continue;
                }
                long bits = cols[3 + a].getLong(8 * i);
                int agg = spec.aggs[a];
                boolean valueTyped = agg != FgConfig.AGG_COUNT_STAR && agg != FgConfig.AGG_COUNT;
                aggs.setField(
                        a,
                        valueTyped && spec.valType == FgConfig.VAL_F64
                                ? (Object) Double.longBitsToDouble(bits)
                                : (Object) bits);
            }
            aggs.setField(nAggs, TimestampData.fromEpochMillis(cols[1].getLong(8 * i)));
            aggs.setField(nAggs + 1, TimestampData.fromEpochMillis(cols[2].getLong(8 * i)));
            collector.collect(new JoinedRowData(keyRows[i], aggs));
        }
    }

    /**
     * The barrier: the local buffer goes out with the next round (epoch = checkpointId); once every
     * subtask has sent its pre-barrier rows, the global's rows are emitted and its image taken.
     */
    @Override
    public void prepareSnapshotPreBarrier(long checkpointId) throws Exception {
        flushBatch();
        lock.lock();
        try {
            check();
            flushReq = checkpointId;
            changed.signalAll();
            while (aligned < checkpointId && edgeError == null) {
                changed.await(100, TimeUnit.MILLISECONDS);
            }
            check();
        } finally {
            lock.unlock();
        }
        emitGlobal();   // (the rows fired before the barrier precede it)
        lock.lock();
        try {
            FlinkGpu.flush(global);
            snapshotImage = imageChunks();
            snapDone = checkpointId;
            changed.signalAll();   // (the edge merges the next round now)
        } finally {
            lock.unlock();
        }
    }

    @Override
    public void snapshotState(StateSnapshotContext context) throws Exception {
        super.snapshotState(context);
        imageState.clear();
        if (snapshotImage != null) {
            for (byte[] chunk : snapshotImage) {
                imageState.add(chunk);
            }
        }
    }

    /** Long.MAX_VALUE: the edge runs until every subtask has ended; the last rows go out */
    @Override
    public void endInput() throws Exception {
        processWatermark(new Watermark(Long.MAX_VALUE));
        edge.join();
        check();
        emitGlobal();
    }

    @Override
    public void close() throws Exception {
        lock.lock();
        try {
            closing = true;
            changed.signalAll();
        } finally {
            lock.unlock();
        }
        if (edge != null) {
            edge.join(TimeUnit.SECONDS.toMillis(60));
        }
        super.close();
        if (comm != 0) {
            FlinkGpu.commClose(comm);
            comm = 0;
        }
        for (long h : new long[] {local, global}) {
            if (h != 0) {
                FlinkGpu.close(h);
            }
        }
        local = global = 0;
        for (ByteBuffer c : new ByteBuffer[] {keyCol, timeCol, valCol, nullCol}) {
            if (c != null) {
                FlinkGpu.hostUnregister(spec.device, c);
            }
        }
        if (keys != null) {
            keys.close();
        }
    }

    // ---- the edge thread ---------------------------------------------------------------------------

    private void runEdge() {
        long[] r = new long[5];
        try {
            lock.lock();
            try {   // the communicator id (from the coordinator), then every subtask joins
                while (commId == null && !closing) {
                    changed.await(100, TimeUnit.MILLISECONDS);
                }
                if (closing) {
                    return;
                }
            } finally {
                lock.unlock();
            }
            ByteBuffer id = GpuKeyRows.direct(FlinkGpu.COMM_ID_BYTES);
            id.put(commId).flip();
            comm = FlinkGpu.commOpen(spec.device, parallelism, index, id);
            while (true) {
                int mode;
                lock.lock();
                try {
                    long epoch;
                    if (dirty) {   // (fires before a flush: the barrier's flush follows next round)
                        mode = FlinkGpu.ROUND_FIRED;
                        epoch = sentEpoch;
                    } else if (flushReq > sentEpoch) {
                        mode = FlinkGpu.ROUND_FLUSHED;
                        epoch = flushReq;
                    } else {
                        mode = FlinkGpu.ROUND_IDLE;
                        epoch = sentEpoch;
                    }
                    dirty = false;
                    try {
                        FlinkGpu.commRoundBegin(
                                comm,
                                mode == FlinkGpu.ROUND_IDLE ? 0 : local,
                                mode,
                                FlinkGpu.KEYHASH_BINARYROW_BIGINT,
                                maxP,
                                wmLocal,
                                epoch);
                    } catch (RuntimeException beginFailed) {
                        // (still takes part: commRoundExchange reports it on every subtask)
                    }
                    if (mode == FlinkGpu.ROUND_FLUSHED) {
                        sentEpoch = epoch;
                    }
                } finally {
                    lock.unlock();
                }
                FlinkGpu.commRoundExchange(comm, r);   // (no lock: the task thread goes on)
                lock.lock();
                try {
                    FlinkGpu.commRoundEnd(comm, global);
                    if (r[0] > globWm) {
                        FlinkGpu.advanceProgressAsync(global, r[0]);
                        globWm = r[0];
                        pendingFires = true;
                        mailbox.execute(this::emitGlobal, "emit the global window rows");
                    }
                    if (r[1] > aligned) {   // every subtask sent its pre-barrier rows
                        aligned = r[1];
                        changed.signalAll();
                        while (snapDone < aligned && !closing) {   // (its task thread snapshots first)
                            changed.await(100, TimeUnit.MILLISECONDS);
                        }
                    }
                    if (closing) {
                        return;
                    }
                } finally {
                    lock.unlock();
                }
                if (r[0] == Long.MAX_VALUE) {
                    return;   // every subtask has ended (the same round on all of them)
                }
                if (mode == FlinkGpu.ROUND_IDLE && r[3] == 0) {
                    Thread.sleep(IDLE_SLEEP_MS);
                }
            }
        } catch (Throwable t) {
            lock.lock();
            try {
                edgeError = t;
                changed.signalAll();
            } finally {
                lock.unlock();
            }
        }
    }

    // ---- the image as union operator state --------------------------------------------------------

    /** the global's image (snapshotStateAsync + Wait) as chunks: [n, timer wm, n x 7 longs] each */
    private byte[][] imageChunks() {
        FlinkGpu.snapshotStateAsync(global);
        ByteBuffer[] cols = new ByteBuffer[7];
        long[] wm = new long[1];
        int n = (int) FlinkGpu.snapshotStateWait(global, cols, wm);
        for (ByteBuffer c : cols) {
            if (c != null) {
                c.order(ByteOrder.nativeOrder());
            }
        }
        int chunks = Math.max(1, (n + IMAGE_CHUNK_ROWS - 1) / IMAGE_CHUNK_ROWS);
        byte[][] out = new byte[chunks][];
        for (int k = 0; k < chunks; k++) {
            int lo = k * IMAGE_CHUNK_ROWS, hi = Math.min(n, lo + IMAGE_CHUNK_ROWS);
            ByteBuffer b = ByteBuffer.allocate(16 + 56 * (hi - lo)).order(ByteOrder.LITTLE_ENDIAN);
            b.putLong(hi - lo).putLong(wm[0]);
            for (int i = lo; i < hi; i++) {
                for (int c = 0; c < 7; c++) {
                    ByteBuffer col = cols[c] != null ? cols[c] : cols[4];   // (min / max: single-value lists)
                    b.putLong(col.getLong(8 * i));
                }
            }
            out[k] = b.array();
        }
        return out;
    }

    /** initializeState: every subtask's chunks, the entries of this subtask's key groups kept */
    private void restoreGlobal(KeyGroupRange range) {
        if (restoredImage == null || restoredImage.isEmpty()) {
            return;
        }
        long timerWm = Long.MAX_VALUE;
        List<long[]> rows = new ArrayList<>();
        for (byte[] chunk : restoredImage) {
            ByteBuffer b = ByteBuffer.wrap(chunk).order(ByteOrder.LITTLE_ENDIAN);
            long n = b.getLong();
            timerWm = Math.min(timerWm, b.getLong());
            for (long i = 0; i < n; i++) {
                long[] row = new long[7];
                for (int c = 0; c < 7; c++) {
                    row[c] = b.getLong();
                }
                RowData key = keys.rows(GpuKeyRows.direct(8).putLong(0, row[0]), 1)[0];
                if (range.contains(KeyGroupRangeAssignment.assignToKeyGroup(key, maxP))) {
                    rows.add(row);
                }
            }
        }
        int n = rows.size();
        ByteBuffer[] c = new ByteBuffer[7];
        for (int j = 0; j < 7; j++) {
            c[j] = GpuKeyRows.direct(8L * Math.max(n, 1));
            for (int i = 0; i < n; i++) {
                c[j].putLong(8 * i, rows.get(i)[j]);
            }
        }
        boolean mv = accRows.multiValue();
        FlinkGpu.restore(global, n, c[0], c[1], c[2], c[3], c[4], mv ? c[5] : null, mv ? c[6] : null, timerWm);
        restoredImage = null;
    }
}
