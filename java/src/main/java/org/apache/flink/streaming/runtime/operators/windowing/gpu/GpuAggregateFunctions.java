/*
 * The AggregateFunctions a GPU window operator runs for WindowedStream.aggregate
 * (WindowedStream.java:283-349 -> WindowOperatorBuilder.aggregate :198-224) on Tuple2<Long, V>
 * keyed by f0, V = Long or Double: COUNT, SUM, AVG, MIN, MAX of f1. Each is a plain
 * AggregateFunction -- the CPU WindowOperator runs it unchanged, and its accumulator is what the
 * reference's AggregatingState "window-contents" holds -- and a GpuWindowOperator.Accumulation:
 * the map between its accumulator and the engine's per-(key, window) (value bits, record count).
 *
 *   count()          ACC Long count                      R Long
 *   sum(isDouble)    ACC V sum (0)                        R V
 *   avg(isDouble)    ACC Tuple2<V sum, Long count>        R Double = (double) sum / count
 *   min(isDouble)    ACC V (Long.MAX_VALUE / NaN)         R V   (Long / Double.compareTo order;
 *   max(isDouble)    ACC V (Long.MIN_VALUE / -inf)        R V    a Double result canonical)
 *
 * flink_amd/datastream.py (api="aggregate") is the Python mirror, tested against the oracle in
 * tests/test_gpu_datastream_state.py.
 */
package org.apache.flink.streaming.runtime.operators.windowing.gpu;

import org.apache.flink.api.common.ExecutionConfig;
import org.apache.flink.api.common.functions.AggregateFunction;
import org.apache.flink.api.common.state.AggregatingStateDescriptor;
import org.apache.flink.api.common.state.StateDescriptor;
import org.apache.flink.api.common.typeinfo.TypeInformation;
import org.apache.flink.api.common.typeinfo.Types;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.table.runtime.operators.window.gpu.FgConfig;

/** COUNT / SUM / AVG / MIN / MAX of Tuple2.f1 as AggregateFunctions the GPU operator runs. */
public final class GpuAggregateFunctions {
    private GpuAggregateFunctions() {}

    /** An AggregateFunction of Tuple2<Long, V> whose accumulator the engine keeps. */
    public abstract static class GpuAggregate<V, ACC, R>
            implements AggregateFunction<Tuple2<Long, V>, ACC, R>,
                    GpuWindowOperator.Accumulation<V, ACC, R> {
        private static final long serialVersionUID = 1L;
        final boolean isDouble;

        GpuAggregate(boolean isDouble) {
            this.isDouble = isDouble;
        }

        abstract TypeInformation<ACC> accumulatorType();

        long bits(Object v) {
            return isDouble ? Double.doubleToRawLongBits((Double) v) : (Long) v;
        }

        @SuppressWarnings("unchecked")
        V value(long bits) {
            return (V) (isDouble ? (Object) Double.longBitsToDouble(bits) : (Object) bits);
        }

        @Override
        public StateDescriptor<?, ACC> stateDescriptor(
                String name, TypeInformation<Tuple2<Long, V>> in, ExecutionConfig config) {
            // WindowOperatorBuilder.aggregate: AggregatingStateDescriptor of the accumulator type
            return new AggregatingStateDescriptor<>(name, this, accumulatorType().createSerializer(config));
        }

        @Override
        public long[] merge(long a0, long a1, long b0, long b1) {
            return toBits(merge(fromBits(0L, a0, a1), fromBits(0L, b0, b1)));
        }

        @Override
        public R output(long key, long a0, long a1) {
            return getResult(fromBits(key, a0, a1));
        }
    }

    /** The count of the window's records. */
    public static <V> GpuAggregate<V, Long, Long> count() {
        return new GpuAggregate<V, Long, Long>(false) {
            private static final long serialVersionUID = 1L;

            @Override
            public int valueAgg() {
                return -1;
            }

            @Override
            TypeInformation<Long> accumulatorType() {
                return Types.LONG;
            }

            @Override
            public Long createAccumulator() {
                return 0L;
            }

            @Override
            public Long add(Tuple2<Long, V> v, Long acc) {
                return acc + 1;
            }

            @Override
            public Long getResult(Long acc) {
                return acc;
            }

            @Override
            public Long merge(Long a, Long b) {
                return a + b;
            }

            @Override
            public Long fromBits(long key, long a0, long a1) {
                return a1;
            }

            @Override
            public long[] toBits(Long acc) {
                return new long[] {0L, acc};
            }
        };
    }

    /** The sum of f1 (Java long / double +). */
    public static <V> GpuAggregate<V, V, V> sum(boolean isDouble) {
        return new GpuAggregate<V, V, V>(isDouble) {
            private static final long serialVersionUID = 1L;

            @Override
            public int valueAgg() {
                return FgConfig.AGG_SUM;
            }

            @Override
            @SuppressWarnings("unchecked")
            TypeInformation<V> accumulatorType() {
                return (TypeInformation<V>) (isDouble ? Types.DOUBLE : Types.LONG);
            }

            @Override
            public V createAccumulator() {
                return value(isDouble ? Double.doubleToRawLongBits(0.0) : 0L);
            }

            @Override
            public V add(Tuple2<Long, V> v, V acc) {
                return merge(acc, v.f1);
            }

            @Override
            public V getResult(V acc) {
                return acc;
            }

            @Override
            @SuppressWarnings("unchecked")
            public V merge(V a, V b) {
                return (V) (isDouble ? (Object) ((Double) a + (Double) b) : (Object) ((Long) a + (Long) b));
            }

            @Override
            public V fromBits(long key, long a0, long a1) {
                return value(a0);
            }

            @Override
            public long[] toBits(V acc) {
                return new long[] {bits(acc), 1L};
            }
        };
    }

    /** (double) sum / count of f1; the accumulator is (sum, count). */
    public static <V> GpuAggregate<V, Tuple2<V, Long>, Double> avg(boolean isDouble) {
        return new GpuAggregate<V, Tuple2<V, Long>, Double>(isDouble) {
            private static final long serialVersionUID = 1L;

            @Override
            public int valueAgg() {
                return FgConfig.AGG_SUM;
            }

            @Override
            @SuppressWarnings("unchecked")
            TypeInformation<Tuple2<V, Long>> accumulatorType() {
                return (TypeInformation<Tuple2<V, Long>>)
                        (TypeInformation<?>) Types.TUPLE(isDouble ? Types.DOUBLE : Types.LONG, Types.LONG);
            }

            @Override
            public Tuple2<V, Long> createAccumulator() {
                return Tuple2.of(value(isDouble ? Double.doubleToRawLongBits(0.0) : 0L), 0L);
            }

            @Override
            public Tuple2<V, Long> add(Tuple2<Long, V> v, Tuple2<V, Long> acc) {
                return merge(acc, Tuple2.of(v.f1, 1L));
            }

            @Override
            public Double getResult(Tuple2<V, Long> acc) {
                double s = isDouble ? (Double) acc.f0 : (double) (Long) acc.f0;
                return s / acc.f1;
            }

            @Override
            @SuppressWarnings("unchecked")
            public Tuple2<V, Long> merge(Tuple2<V, Long> a, Tuple2<V, Long> b) {
                Object s = isDouble ? (Object) ((Double) a.f0 + (Double) b.f0) : (Object) ((Long) a.f0 + (Long) b.f0);
                return Tuple2.of((V) s, a.f1 + b.f1);
            }

            @Override
            public Tuple2<V, Long> fromBits(long key, long a0, long a1) {
                return Tuple2.of(value(a0), a1);
            }

            @Override
            public long[] toBits(Tuple2<V, Long> acc) {
                return new long[] {bits(acc.f0), acc.f1};
            }
        };
    }

    /** The minimum of f1 (Long.compareTo / Double.compareTo: -0.0 below +0.0, NaN above all). */
    public static <V> GpuAggregate<V, V, V> min(boolean isDouble) {
        return extreme(isDouble, true);
    }

    /** The maximum of f1 (Long.compareTo / Double.compareTo). */
    public static <V> GpuAggregate<V, V, V> max(boolean isDouble) {
        return extreme(isDouble, false);
    }

    private static <V> GpuAggregate<V, V, V> extreme(boolean isDouble, boolean min) {
        return new GpuAggregate<V, V, V>(isDouble) {
            private static final long serialVersionUID = 1L;

            @Override
            public int valueAgg() {
                return min ? FgConfig.AGG_MIN : FgConfig.AGG_MAX;
            }

            @Override
            @SuppressWarnings("unchecked")
            TypeInformation<V> accumulatorType() {
                return (TypeInformation<V>) (isDouble ? Types.DOUBLE : Types.LONG);
            }

            @Override
            public V createAccumulator() {   // the identity of the order's min / max
                if (isDouble) {
                    return value(Double.doubleToRawLongBits(min ? Double.NaN : Double.NEGATIVE_INFINITY));
                }
                return value(min ? Long.MAX_VALUE : Long.MIN_VALUE);
            }

            @Override
            public V add(Tuple2<Long, V> v, V acc) {
                return merge(acc, v.f1);
            }

            @Override
            public V getResult(V acc) {
                return acc;
            }

            @Override
            @SuppressWarnings("unchecked")
            public V merge(V a, V b) {   // value2 wins unless value1 compares strictly smaller / greater
                int c = ((Comparable<Object>) a).compareTo(b);
                V r = (min ? c < 0 : c > 0) ? a : b;
                return isDouble ? value(Double.doubleToLongBits((Double) r)) : r;
            }

            @Override
            public V fromBits(long key, long a0, long a1) {
                return value(a0);
            }

            @Override
            public long[] toBits(V acc) {
                return new long[] {bits(acc), 1L};
            }
        };
    }
}
