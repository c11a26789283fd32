/*
 * The coordinator of the fused two-phase operator (OperatorCoordinator, runs in the JobManager): it
 * distributes subtask 0's fg_comm id to every subtask so that all of them open one RCCL communicator
 * (fg_comm_open blocks until every rank has joined), and it turns the failure of ANY subtask into a
 * failure of the job: the subtasks are joined by the edge's collectives, not by data edges of the job
 * graph, so a region failover that restarted one subtask would leave the others blocked in a round
 * (Context.failJob -> a global failover; every subtask restores from the last checkpoint and
 * subtask 0 makes a new id).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.runtime.jobgraph.OperatorID;
import org.apache.flink.runtime.operators.coordination.OperatorCoordinator;
import org.apache.flink.runtime.operators.coordination.OperatorEvent;

import java.util.HashMap;
import java.util.Map;
import java.util.concurrent.CompletableFuture;

/** Distributes the edge's communicator id; fails the job when a subtask fails. */
public final class GpuCommCoordinator implements OperatorCoordinator {
    private final Context context;
    private final Map<Integer, SubtaskGateway> gateways = new HashMap<>();
    private GpuCommIdEvent current;   // the id of the running attempt (null until subtask 0 sent it)

    GpuCommCoordinator(Context context) {
        this.context = context;
    }

    @Override
    public void start() {}

    @Override
    public void close() {}

    @Override
    public synchronized void handleEventFromOperator(int subtask, OperatorEvent event) {
        if (!(event instanceof GpuCommIdEvent) || subtask != 0) {
            return;
        }
        current = (GpuCommIdEvent) event;
        for (SubtaskGateway g : gateways.values()) {
            g.sendEvent(current);
        }
    }

    @Override
    public synchronized void subtaskReady(int subtask, SubtaskGateway gateway) {
        gateways.put(subtask, gateway);
        if (current != null) {   // (a subtask that deployed after subtask 0 sent its id)
            gateway.sendEvent(current);
        }
    }

    @Override
    public synchronized void subtaskFailed(int subtask, Throwable reason) {
        gateways.remove(subtask);
        current = null;   // (the restarted attempt makes a new id)
        context.failJob(
                new RuntimeException(
                        "a subtask of the GPU two-phase window aggregation failed: every subtask restarts "
                                + "(its RCCL exchange joins them all)",
                        reason));
    }

    @Override
    public synchronized void subtaskReset(int subtask, long checkpointId) {
        gateways.remove(subtask);
        current = null;
    }

    @Override
    public void checkpointCoordinator(long checkpointId, CompletableFuture<byte[]> result) {
        result.complete(new byte[0]);   // (nothing to keep: an id is only valid for its attempt)
    }

    @Override
    public void notifyCheckpointComplete(long checkpointId) {}

    @Override
    public synchronized void resetToCheckpoint(long checkpointId, byte[] checkpointData) {
        current = null;
    }

    /** The provider the operator factory hands to the JobManager. */
    public static final class Provider implements OperatorCoordinator.Provider {
        private static final long serialVersionUID = 1L;
        private final OperatorID operatorId;

        public Provider(OperatorID operatorId) {
            this.operatorId = operatorId;
        }

        @Override
        public OperatorID getOperatorId() {
            return operatorId;
        }

        @Override
        public OperatorCoordinator create(Context context) {
            return new GpuCommCoordinator(context);
        }
    }
}
