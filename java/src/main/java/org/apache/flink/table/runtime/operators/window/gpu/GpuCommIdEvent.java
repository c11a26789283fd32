/*
 * The RCCL communicator id of the fused two-phase operator (GpuTwoPhaseWindowAggOperator): subtask 0
 * makes it (FlinkGpu.commUniqueId -- the id names a bootstrap endpoint in the process that made it,
 * so a subtask makes it, not the JobManager) and sends it to the operator's coordinator, which
 * forwards it to every subtask (GpuCommCoordinator). `attempt` tells ids of different restarts apart.
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.runtime.operators.coordination.OperatorEvent;

/** A 128-byte fg_comm id, from subtask 0 to the coordinator and from the coordinator to every subtask. */
public final class GpuCommIdEvent implements OperatorEvent {
    private static final long serialVersionUID = 1L;

    private final byte[] id;
    private final int attempt;

    public GpuCommIdEvent(byte[] id, int attempt) {
        if (id.length != FlinkGpu.COMM_ID_BYTES) {
            throw new IllegalArgumentException("a communicator id has " + FlinkGpu.COMM_ID_BYTES + " bytes");
        }
        this.id = id.clone();
        this.attempt = attempt;
    }

    public byte[] id() {
        return id.clone();
    }

    public int attempt() {
        return attempt;
    }
}
