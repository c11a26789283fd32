/*
 * The factory the planner puts in place of LocalSlicingWindowAggOperator -> keyBy ->
 * GlobalSlicingWindowAggOperator when the two-phase window aggregation runs on GPUs
 * (INTEGRATION.md section 7): a CoordinatedOperatorFactory, so that the JobManager runs the
 * operator's GpuCommCoordinator (the communicator id, failover of every subtask together), and the
 * operator gets its event gateway and the task's mailbox (the edge thread's rows are emitted there).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.runtime.jobgraph.OperatorID;
import org.apache.flink.runtime.operators.coordination.OperatorCoordinator;
import org.apache.flink.streaming.api.operators.AbstractStreamOperatorFactory;
import org.apache.flink.streaming.api.operators.CoordinatedOperatorFactory;
import org.apache.flink.streaming.api.operators.OneInputStreamOperatorFactory;
import org.apache.flink.streaming.api.operators.StreamOperator;
import org.apache.flink.streaming.api.operators.StreamOperatorParameters;
import org.apache.flink.streaming.runtime.tasks.mailbox.TaskMailbox;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.runtime.keyselector.RowDataKeySelector;

/** Creates GpuTwoPhaseWindowAggOperator and its coordinator. */
public final class GpuTwoPhaseWindowAggOperatorFactory extends AbstractStreamOperatorFactory<RowData>
        implements CoordinatedOperatorFactory<RowData>, OneInputStreamOperatorFactory<RowData, RowData> {
    private static final long serialVersionUID = 1L;

    private final GpuWindowAggSpec spec;
    private final RowDataKeySelector keySelector;

    public GpuTwoPhaseWindowAggOperatorFactory(GpuWindowAggSpec spec, RowDataKeySelector keySelector) {
        this.spec = spec;
        this.keySelector = keySelector;
    }

    @Override
    @SuppressWarnings("unchecked")
    public <T extends StreamOperator<RowData>> T createStreamOperator(StreamOperatorParameters<RowData> parameters) {
        final OperatorID operatorId = parameters.getStreamConfig().getOperatorID();
        GpuTwoPhaseWindowAggOperator op = new GpuTwoPhaseWindowAggOperator(spec.copy(), keySelector);
        op.setOperatorEventGateway(parameters.getOperatorEventDispatcher().getOperatorEventGateway(operatorId));
        op.setMailboxExecutor(parameters.getContainingTask().getMailboxExecutorFactory()
                .createExecutor(TaskMailbox.MIN_PRIORITY));
        op.setup(parameters.getContainingTask(), parameters.getStreamConfig(), parameters.getOutput());
        parameters.getOperatorEventDispatcher().registerEventHandler(operatorId, op);
        return (T) op;
    }

    @Override
    public OperatorCoordinator.Provider getCoordinatorProvider(String operatorName, OperatorID operatorID) {
        return new GpuCommCoordinator.Provider(operatorID);
    }

    @Override
    public Class<? extends StreamOperator> getStreamOperatorClass(ClassLoader classLoader) {
        return GpuTwoPhaseWindowAggOperator.class;
    }
}
