/*
 * The accumulator row of a supported aggregate list, as the planner's generated
 * NamespaceAggsHandleFunction keeps it (AggsHandlerCodeGenerator.scala:578-700): each function's
 * aggBufferAttributes in list order, typed by getAggBufferTypes --
 *
 *   COUNT(*)  Count1AggFunction    [count1 BIGINT NOT NULL]            init 0
 *   COUNT(v)  CountAggFunction     [count BIGINT NOT NULL]             init 0
 *   SUM(v)    SumAggFunction       [sum  T]                            init NULL
 *   AVG(v)    AvgAggFunction       [sum  S NOT NULL, count BIGINT]     init 0, 0
 *   SUM0(v)   Sum0AggFunction      [sum0 T NOT NULL]                   init 0
 *   MIN(v)    MinAggFunction       [min  T]                            init NULL
 *   MAX(v)    MaxAggFunction       [max  T]                            init NULL
 *
 * (T = the value type, BIGINT or DOUBLE; S = AvgAggFunction.getSumType(): BIGINT for integral,
 * DOUBLE for DOUBLE input; TP/functions/aggfunctions/*AggFunction.java, initialValuesExpressions /
 * mergeExpressions.) The engine's partial accumulator of a (key, slice) -- COUNT(*), COUNT(v) and
 * the SUM / MIN / MAX value slots -- maps onto this row one-for-one, so partial rows leave the
 * local phase in LocalAggCombiner's output layout (key, acc..., slice_end), LocalAggCombiner.java:
 * 100-106, and GPU state is written into the reference's "window-aggs" ValueState with the
 * accSerializer's layout (AbstractWindowAggProcessor.java:103-109).
 */
package org.apache.flink.table.runtime.operators.window.gpu;

import org.apache.flink.table.data.GenericRowData;
import org.apache.flink.table.data.RowData;
import org.apache.flink.table.types.logical.BigIntType;
import org.apache.flink.table.types.logical.DoubleType;
import org.apache.flink.table.types.logical.LogicalType;
import org.apache.flink.table.runtime.typeutils.RowDataSerializer;

import java.util.ArrayList;
import java.util.List;

/** Accumulator rows of the planner's window aggregates over one value column. */
public final class GpuAccRows {
    private final int[] aggs;
    private final boolean dbl;   // DOUBLE value column (else BIGINT)
    private final int arity;

    public GpuAccRows(int[] aggs, int valType) {
        this.aggs = aggs.clone();
        this.dbl = valType == FgConfig.VAL_F64;
        int n = 0;
        for (int a : aggs) {
            n += a == FgConfig.AGG_AVG ? 2 : 1;
        }
        this.arity = n;
    }

    public int arity() {
        return arity;
    }

    /**
     * the list mixes the SUM family, MIN and MAX: the engine keeps (and its partial rows carry)
     * three value slots SUM, MIN, MAX; else one (fg_open, include/flinkgpu.h FG_FLAG_LOCAL_PARTIALS)
     */
    public boolean multiValue() {
        boolean sumFamily = false, min = false, max = false;
        for (int a : aggs) {
            sumFamily |= a == FgConfig.AGG_SUM || a == FgConfig.AGG_AVG || a == FgConfig.AGG_SUM0;
            min |= a == FgConfig.AGG_MIN;
            max |= a == FgConfig.AGG_MAX;
        }
        return (sumFamily ? 1 : 0) + (min ? 1 : 0) + (max ? 1 : 0) > 1;
    }

    /** getAggBufferTypes of every function, in list order */
    public LogicalType[] types() {
        List<LogicalType> t = new ArrayList<>();
        for (int a : aggs) {
            switch (a) {
                case FgConfig.AGG_COUNT_STAR:
                case FgConfig.AGG_COUNT:
                    t.add(new BigIntType(false));
                    break;
                case FgConfig.AGG_AVG:
                    t.add(dbl ? new DoubleType(false) : new BigIntType(false));
                    t.add(new BigIntType(false));
                    break;
                case FgConfig.AGG_SUM0:
                    t.add(dbl ? new DoubleType(false) : new BigIntType(false));
                    break;
                default:   // SUM, MIN, MAX: nullable
                    t.add(dbl ? new DoubleType() : new BigIntType());
            }
        }
        return t.toArray(new LogicalType[0]);
    }

    /** the accSerializer of "window-aggs" (AbstractWindowAggProcessor.java:103-109) */
    public RowDataSerializer serializer() {
        return new RowDataSerializer(types());
    }

    private Object value(long bits) {
        return dbl ? (Object) Double.longBitsToDouble(bits) : (Object) bits;
    }

    private long bits(RowData r, int pos) {
        return dbl ? Double.doubleToRawLongBits(r.getDouble(pos)) : r.getLong(pos);
    }

    /** initialValuesExpressions of every function (createAccumulators) */
    public GenericRowData create() {
        GenericRowData r = new GenericRowData(arity);
        int f = 0;
        for (int a : aggs) {
            switch (a) {
                case FgConfig.AGG_COUNT_STAR:
                case FgConfig.AGG_COUNT:
                    r.setField(f++, 0L);
                    break;
                case FgConfig.AGG_AVG:
                    r.setField(f++, value(0L));   // (0 and 0.0 share their bit pattern)
                    r.setField(f++, 0L);
                    break;
                case FgConfig.AGG_SUM0:
                    r.setField(f++, value(0L));
                    break;
                default:
                    r.setField(f++, null);
            }
        }
        return r;
    }

    /**
     * The accumulator of one engine partial row: COUNT(*), COUNT(v), and the SUM / MIN / MAX slot
     * bits (min / max only for a list holding them). A nullable accumulator (SUM, MIN, MAX) is
     * NULL iff no non-null value entered it (COUNT(v) = 0), as its init value says.
     */
    public GenericRowData fromPartial(long cntStar, long cntVal, long sum, long min, long max) {
        GenericRowData r = new GenericRowData(arity);
        int f = 0;
        for (int a : aggs) {
            switch (a) {
                case FgConfig.AGG_COUNT_STAR:
                    r.setField(f++, cntStar);
                    break;
                case FgConfig.AGG_COUNT:
                    r.setField(f++, cntVal);
                    break;
                case FgConfig.AGG_SUM:
                    r.setField(f++, cntVal == 0 ? null : value(sum));
                    break;
                case FgConfig.AGG_AVG:
                    r.setField(f++, value(cntVal == 0 ? 0L : sum));
                    r.setField(f++, cntVal);
                    break;
                case FgConfig.AGG_SUM0:
                    r.setField(f++, value(cntVal == 0 ? 0L : sum));
                    break;
                case FgConfig.AGG_MIN:
                    r.setField(f++, cntVal == 0 ? null : value(min));
                    break;
                default:   // MAX
                    r.setField(f++, cntVal == 0 ? null : value(max));
            }
        }
        return r;
    }

    /**
     * The engine partial of an accumulator row whose fields start at `off` (the inverse of
     * fromPartial: a restore from "window-aggs", a LocalAggCombiner row entering the global
     * phase): {cnt_star, cnt_val, slot0, slot1, slot2} bits in fg_partials / fg_state_rows order --
     * SUM, MIN, MAX for a multi-value list, else slot0 = the list's one value accumulator.
     * COUNT(*) from the row's COUNT(*) (or, without one, from COUNT(v) / AVG's count), COUNT(v)
     * from COUNT / AVG (else = COUNT(*)).
     */
    public long[] toPartial(RowData r, int off) {
        long cs = -1, cv = -1, sum = 0, min = 0, max = 0;
        boolean anyValue = false, hasMin = false, hasMax = false;
        int f = off;
        for (int a : aggs) {
            switch (a) {
                case FgConfig.AGG_COUNT_STAR:
                    cs = r.getLong(f++);
                    break;
                case FgConfig.AGG_COUNT:
                    cv = r.getLong(f++);
                    break;
                case FgConfig.AGG_SUM:
                    if (!r.isNullAt(f)) {
                        sum = bits(r, f);
                        anyValue = true;
                    }
                    f++;
                    break;
                case FgConfig.AGG_AVG:
                    sum = bits(r, f++);
                    cv = r.getLong(f++);
                    break;
                case FgConfig.AGG_SUM0:
                    sum = bits(r, f++);
                    break;
                case FgConfig.AGG_MIN:
                    hasMin = true;
                    if (!r.isNullAt(f)) {
                        min = bits(r, f);
                        anyValue = true;
                    }
                    f++;
                    break;
                default:
                    hasMax = true;
                    if (!r.isNullAt(f)) {
                        max = bits(r, f);
                        anyValue = true;
                    }
                    f++;
            }
        }
        if (cs < 0) {
            cs = cv >= 0 ? cv : (anyValue ? 1 : 0);
        }
        if (cv < 0) {
            cv = cs;
        }
        if (!multiValue()) {
            sum = hasMin ? min : hasMax ? max : sum;
        }
        return new long[] {cs, cv, sum, min, max};
    }

    /**
     * mergeExpressions of every function: acc merged with other (GlobalAggCombiner.combine's
     * globalAggregator.merge). Counts add; SUM adds, NULL-aware; AVG adds sum and count; SUM0 adds;
     * MIN / MAX keep the smaller / larger, NULL-aware, by Java's primitive comparison.
     */
    public GenericRowData merge(RowData acc, RowData other) {
        GenericRowData r = new GenericRowData(arity);
        int f = 0;
        for (int a : aggs) {
            switch (a) {
                case FgConfig.AGG_COUNT_STAR:
                case FgConfig.AGG_COUNT:
                    r.setField(f, acc.getLong(f) + other.getLong(f));
                    f++;
                    break;
                case FgConfig.AGG_AVG:
                    r.setField(f, add(acc, other, f));
                    f++;
                    r.setField(f, acc.getLong(f) + other.getLong(f));
                    f++;
                    break;
                case FgConfig.AGG_SUM0:
                    r.setField(f, add(acc, other, f));
                    f++;
                    break;
                case FgConfig.AGG_SUM:
                    r.setField(f, other.isNullAt(f) ? get(acc, f) : acc.isNullAt(f) ? get(other, f) : add(acc, other, f));
                    f++;
                    break;
                default: {   // MIN / MAX
                    final boolean min = a == FgConfig.AGG_MIN;
                    if (other.isNullAt(f)) {
                        r.setField(f, get(acc, f));
                    } else if (acc.isNullAt(f)) {
                        r.setField(f, get(other, f));
                    } else if (dbl) {
                        final double x = acc.getDouble(f), y = other.getDouble(f);
                        r.setField(f, (min ? y < x : y > x) ? y : x);
                    } else {
                        final long x = acc.getLong(f), y = other.getLong(f);
                        r.setField(f, (min ? y < x : y > x) ? y : x);
                    }
                    f++;
                }
            }
        }
        return r;
    }

    private Object get(RowData r, int f) {
        return r.isNullAt(f) ? null : dbl ? (Object) r.getDouble(f) : (Object) r.getLong(f);
    }

    private Object add(RowData a, RowData b, int f) {
        return dbl ? (Object) (a.getDouble(f) + b.getDouble(f)) : (Object) (a.getLong(f) + b.getLong(f));
    }
}
