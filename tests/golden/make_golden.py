"""Generate the golden fixtures under tests/golden/ from the reference's own tests.

The reference is Java; nothing of it can run here (no JDK). Every vector
below is TRANSCRIBED DATA: the input sequence and the expected output that a
reference test asserts, with the test's file:line.  String keys of the reference tests
are mapped to i64 ids (key identity is the only property the aggregation uses; outputs
are compared sorted, as the reference's assertors do).  Timestamps are epoch millis.

Paths:
  TRT = flink-table/flink-table-runtime-blink/src/test/java/org/apache/flink/table/runtime/
  TPT = flink-table/flink-table-planner-blink/src/test/scala/org/apache/flink/table/planner/
  SJT = flink-streaming-java/src/test/java/org/apache/flink/streaming/

Run:  python tests/golden/make_golden.py   (rewrites the *.json next to this file)
"""
from __future__ import annotations

import datetime as dt
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SHANGHAI = 8 * 3600 * 1000          # Asia/Shanghai: fixed +08:00, useDaylightTime() == false
JMAX = (1 << 63) - 1


def utc_ms(s: str) -> int:
    """LocalDateTime string read as UTC -> epoch millis (the tests' utcMills())."""
    d = dt.datetime.fromisoformat(s).replace(tzinfo=dt.timezone.utc)
    return int(round(d.timestamp() * 1000))


def E(key, val, ts, isnull=0):
    return ["e", key, val, ts, isnull]


def WM(w):
    return ["wm", w]


SNAP = ["snapshot_restore"]


# ----------------------------------------------------------------------------------------
# SlicingWindowAggOperatorTest (TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java)
# SumAndCountAggsFunction (:821-951) computes SUM(f1), COUNT(f1) over an INT column; the
# output row is (key, sum, count, window_start, window_end) with window times in
# localMills() = toUtcTimestampMills(epoch, shiftTimeZone).  key1 -> 1, key2 -> 2.
# Columns checked: key, sum, count(= COUNT(f1)), window_start, window_end.
# ----------------------------------------------------------------------------------------
def slicing_operator_fixtures():
    out = []
    for tzname, tz in (("UTC", 0), ("Asia/Shanghai", SHANGHAI)):
        L = lambda x: x + tz   # localMills(x)
        # testEventTimeHoppingWindows :116-222 (hop 3s/1s, countStarIndex 1)
        ev = [E(2, 1, 3999), E(2, 1, 3000), E(1, 1, 20), E(1, 1, 0), E(1, 1, 999),
              E(2, 1, 1998), E(2, 1, 1999), E(2, 1, 1000)]
        steps = []
        ev.append(WM(999)); steps.append((len(ev) - 1, [[1, 3, 3, L(-2000), L(1000)]]))
        ev.append(WM(1999)); steps.append((len(ev) - 1, [[1, 3, 3, L(-1000), L(2000)], [2, 3, 3, L(-1000), L(2000)]]))
        ev.append(WM(2999)); steps.append((len(ev) - 1, [[1, 3, 3, L(0), L(3000)], [2, 3, 3, L(0), L(3000)]]))
        ev.append(SNAP)
        ev.append(WM(3999)); steps.append((len(ev) - 1, [[2, 5, 5, L(1000), L(4000)]]))
        ev.append(E(2, 1, 3500))   # late for [1K,4K) but accumulated into [2K,5K), [3K,6K)
        ev.append(WM(4999)); steps.append((len(ev) - 1, [[2, 3, 3, L(2000), L(5000)]]))
        ev.append(E(1, 1, 2999))   # late for all assigned windows -> dropped
        ev.append(WM(5999)); steps.append((len(ev) - 1, [[2, 3, 3, L(3000), L(6000)]]))
        ev.append(WM(6999)); steps.append((len(ev) - 1, []))
        ev.append(WM(7999)); steps.append((len(ev) - 1, []))
        out.append(dict(
            name=f"sql_hop_3s_1s_{tzname}", source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:116-222",
            config=dict(mode="sql", kind="hop", size=3000, slide=1000, offset=0, tz_offset_ms=tz,
                        val_type="i64", count_star_index=1),
            columns=["key", "sum", "count", "window_start", "window_end"],
            events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=1))

        # testEventTimeCumulativeWindows :345-452 (cumulate 3s/1s, no count star)
        ev = [E(2, 1, 2999), E(2, 1, 3000), E(1, 1, 20), E(1, 1, 0), E(1, 1, 999),
              E(2, 1, 1998), E(2, 1, 1999), E(2, 1, 1000)]
        steps = []
        ev.append(WM(999)); steps.append((len(ev) - 1, [[1, 3, 3, L(0), L(1000)]]))
        ev.append(WM(1999)); steps.append((len(ev) - 1, [[1, 3, 3, L(0), L(2000)], [2, 3, 3, L(0), L(2000)]]))
        ev.append(WM(2999)); steps.append((len(ev) - 1, [[1, 3, 3, L(0), L(3000)], [2, 4, 4, L(0), L(3000)]]))
        ev.append(SNAP)
        ev.append(WM(3999)); steps.append((len(ev) - 1, [[2, 1, 1, L(3000), L(4000)]]))
        ev.append(E(1, 2, 3500))   # late for [3K,4K) but accumulated into [3K,5K), [3K,6K)
        ev.append(WM(4999)); steps.append((len(ev) - 1, [[2, 1, 1, L(3000), L(5000)], [1, 2, 1, L(3000), L(5000)]]))
        ev.append(E(1, 1, 2999))   # late for all assigned windows -> dropped
        ev.append(WM(5999)); steps.append((len(ev) - 1, [[2, 1, 1, L(3000), L(6000)], [1, 2, 1, L(3000), L(6000)]]))
        ev.append(WM(6999)); steps.append((len(ev) - 1, []))
        ev.append(WM(7999)); steps.append((len(ev) - 1, []))
        out.append(dict(
            name=f"sql_cumulate_3s_1s_{tzname}", source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:345-452",
            config=dict(mode="sql", kind="cumulate", size=3000, slide=1000, offset=0, tz_offset_ms=tz,
                        val_type="i64", count_star_index=-1),
            columns=["key", "sum", "count", "window_start", "window_end"],
            events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=1))

        # testEventTimeTumblingWindows :589-688 (tumble 3s)
        ev = [E(2, 1, 3999), E(2, 1, 3000), E(1, 1, 20), E(1, 1, 0), E(1, 1, 999),
              E(2, 1, 1998), E(2, 1, 1999), E(2, 1, 1000)]
        steps = []
        ev.append(WM(999)); steps.append((len(ev) - 1, []))
        ev.append(WM(1999)); steps.append((len(ev) - 1, []))
        ev.append(SNAP)
        ev.append(WM(2999)); steps.append((len(ev) - 1, [[1, 3, 3, L(0), L(3000)], [2, 3, 3, L(0), L(3000)]]))
        ev.append(WM(3999)); steps.append((len(ev) - 1, []))
        ev.append(E(1, 1, 2500))   # late -> dropped
        ev.append(WM(4999)); steps.append((len(ev) - 1, []))
        ev.append(E(2, 1, 2999))   # late -> dropped
        ev.append(WM(5999)); steps.append((len(ev) - 1, [[2, 2, 2, L(3000), L(6000)]]))
        ev.append(WM(6999)); steps.append((len(ev) - 1, []))
        ev.append(WM(7999)); steps.append((len(ev) - 1, []))
        out.append(dict(
            name=f"sql_tumble_3s_{tzname}", source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:589-688",
            config=dict(mode="sql", kind="tumble", size=3000, slide=0, offset=0, tz_offset_ms=tz,
                        val_type="i64", count_star_index=-1),
            columns=["key", "sum", "count", "window_start", "window_end"],
            events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=2))
    out += proctime_fixtures()
    out += dst_proctime_fixtures()
    return out


# WindowAggregateUseDaylightTimeHarnessTest.scala (TPT/runtime/harness/, :80-197): processing-
# time CUMULATE(1 h step, 3 h max) over `name` in America/Los_Angeles (daylight saving) and
# UTC; setProcessingTime(t) then processElement at t. COUNT(*) is the aggregate transcribed
# (MAX(double) / COUNT(DISTINCT) are outside the engine's aggregate set); all rows are
# compared at the end ("a" -> key 1). Window bounds are local (shifted) times.
def dst_proctime_fixtures():
    out = []
    H = 3600 * 1000
    U = utc_ms
    times = [1615708800000, 1615712400000, 1615716000000, 1615719600000, 1615723200000,
             1636268400000, 1636272000000, 1636275600000, 1636279200000, 1636282800000]
    vals = [1.0, 2.0, 2.0, 5.0, 5.0, 3.0, 3.0, 3.0, 3.0, 3.0]
    ev = []
    for t, v in zip(times, vals):
        ev.append(WM(t))
        ev.append(E(1, v, t))
    ev.append(WM(1636286400000))
    rows = {
        "America/Los_Angeles": [
            (1, "2021-03-14T00:00:00", "2021-03-14T01:00:00"), (2, "2021-03-14T00:00:00", "2021-03-14T02:00:00"),
            (2, "2021-03-14T00:00:00", "2021-03-14T03:00:00"), (1, "2021-03-14T03:00:00", "2021-03-14T04:00:00"),
            (2, "2021-03-14T03:00:00", "2021-03-14T05:00:00"), (3, "2021-03-14T03:00:00", "2021-03-14T06:00:00"),
            (1, "2021-11-07T00:00:00", "2021-11-07T01:00:00"), (3, "2021-11-07T00:00:00", "2021-11-07T02:00:00"),
            (4, "2021-11-07T00:00:00", "2021-11-07T03:00:00"), (1, "2021-11-07T03:00:00", "2021-11-07T04:00:00")],
        "UTC": [
            (1, "2021-03-14T06:00:00", "2021-03-14T09:00:00"), (1, "2021-03-14T09:00:00", "2021-03-14T10:00:00"),
            (2, "2021-03-14T09:00:00", "2021-03-14T11:00:00"), (3, "2021-03-14T09:00:00", "2021-03-14T12:00:00"),
            (1, "2021-03-14T12:00:00", "2021-03-14T13:00:00"), (1, "2021-03-14T12:00:00", "2021-03-14T14:00:00"),
            (1, "2021-03-14T12:00:00", "2021-03-14T15:00:00"),
            (1, "2021-11-07T06:00:00", "2021-11-07T08:00:00"), (2, "2021-11-07T06:00:00", "2021-11-07T09:00:00"),
            (1, "2021-11-07T09:00:00", "2021-11-07T10:00:00"), (2, "2021-11-07T09:00:00", "2021-11-07T11:00:00"),
            (3, "2021-11-07T09:00:00", "2021-11-07T12:00:00")],
    }
    for zone, exp in rows.items():
        cfg = dict(mode="sql", kind="cumulate", size=3 * H, slide=H, offset=0, tz_offset_ms=0, val_type="f64",
                   count_star_index=0, proctime=True)
        if zone != "UTC":
            cfg["zone"] = zone
        out.append(dict(
            name=f"sql_proctime_cumulate_dst_{zone.replace('/', '_')}",
            source="TPT/runtime/harness/WindowAggregateUseDaylightTimeHarnessTest.scala:80-197",
            config=cfg, columns=["key", "cnt_star", "window_start", "window_end"], events=ev,
            expected=[dict(after_event="end", rows=[[1, c, U(s), U(e)] for c, s, e in exp])],
            expected_late_dropped=0))
    return out


# Processing-time variants (:224-343, :454-587, :690-767): a record's time is the harness's
# processing time when it arrives (its rowtime field is ignored); setProcessingTime(t) fires
# the processing-time timers <= t, i.e. advances progress to t. Processing times are
# epochMills(shiftTimeZone, local) = utc_ms(local) - tz; window bounds are local times.
def proctime_fixtures():
    out = []
    H = 3600 * 1000
    for tzname, tz in (("UTC", 0), ("Asia/Shanghai", SHANGHAI)):
        P = lambda s: utc_ms(s) - tz
        U = utc_ms
        # testProcessingTimeHoppingWindows :224-343 (hop 3h/1h, countStarIndex 1)
        ev = []
        steps = []
        t = P("1970-01-01T00:00:00.003")
        ev += [E(2, 1, t)]
        ev.append(WM(P("1970-01-01T01:00:00"))); steps.append((len(ev) - 1, [[2, 1, 1, U("1969-12-31T22:00:00"), U("1970-01-01T01:00:00")]]))
        t = P("1970-01-01T01:00:00")
        ev += [E(2, 1, t), E(2, 1, t)]
        ev.append(WM(P("1970-01-01T02:00:00"))); steps.append((len(ev) - 1, [[2, 3, 3, U("1969-12-31T23:00:00"), U("1970-01-01T02:00:00")]]))
        t = P("1970-01-01T02:00:00")
        ev += [E(1, 1, t), E(1, 1, t)]
        ev.append(WM(P("1970-01-01T03:00:00"))); steps.append((len(ev) - 1, [[2, 3, 3, U("1970-01-01T00:00:00"), U("1970-01-01T03:00:00")],
                                                                             [1, 2, 2, U("1970-01-01T00:00:00"), U("1970-01-01T03:00:00")]]))
        t = P("1970-01-01T03:00:00")
        ev += [E(1, 1, t), E(1, 1, t), E(1, 1, t)]
        ev.append(WM(P("1970-01-01T07:00:00"))); steps.append((len(ev) - 1, [[2, 2, 2, U("1970-01-01T01:00:00"), U("1970-01-01T04:00:00")],
                                                                             [1, 5, 5, U("1970-01-01T01:00:00"), U("1970-01-01T04:00:00")],
                                                                             [1, 5, 5, U("1970-01-01T02:00:00"), U("1970-01-01T05:00:00")],
                                                                             [1, 3, 3, U("1970-01-01T03:00:00"), U("1970-01-01T06:00:00")]]))
        out.append(dict(
            name=f"sql_proctime_hop_3h_1h_{tzname}", source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:224-343",
            config=dict(mode="sql", kind="hop", size=3 * H, slide=H, offset=0, tz_offset_ms=tz,
                        val_type="i64", count_star_index=1, proctime=True),
            columns=["key", "sum", "count", "window_start", "window_end"],
            events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=0))

        # testProcessingTimeCumulativeWindows :454-587 (cumulate 1 day / 8h)
        ev = []
        steps = []
        ev += [E(2, 1, P("1970-01-01T00:00:00.003"))]
        ev.append(WM(P("1970-01-01T08:00:00"))); steps.append((len(ev) - 1, [[2, 1, 1, U("1970-01-01T00:00:00"), U("1970-01-01T08:00:00")]]))
        t = P("1970-01-01T08:00:00")
        ev += [E(2, 1, t), E(2, 1, t)]
        ev.append(WM(P("1970-01-01T16:00:00"))); steps.append((len(ev) - 1, [[2, 3, 3, U("1970-01-01T00:00:00"), U("1970-01-01T16:00:00")]]))
        t = P("1970-01-01T16:00:00")
        ev += [E(1, 1, t), E(1, 1, t)]
        ev.append(WM(P("1970-01-02T00:00:00"))); steps.append((len(ev) - 1, [[2, 3, 3, U("1970-01-01T00:00:00"), U("1970-01-02T00:00:00")],
                                                                             [1, 2, 2, U("1970-01-01T00:00:00"), U("1970-01-02T00:00:00")]]))
        t = P("1970-01-02T00:00:00")
        ev += [E(1, 1, t), E(2, 1, t), E(1, 1, t)]
        ev.append(WM(P("1970-01-03T08:00:00"))); steps.append((len(ev) - 1, [
            [1, 2, 2, U("1970-01-02T00:00:00"), U("1970-01-02T08:00:00")], [2, 1, 1, U("1970-01-02T00:00:00"), U("1970-01-02T08:00:00")],
            [1, 2, 2, U("1970-01-02T00:00:00"), U("1970-01-02T16:00:00")], [2, 1, 1, U("1970-01-02T00:00:00"), U("1970-01-02T16:00:00")],
            [1, 2, 2, U("1970-01-02T00:00:00"), U("1970-01-03T00:00:00")], [2, 1, 1, U("1970-01-02T00:00:00"), U("1970-01-03T00:00:00")]]))
        out.append(dict(
            name=f"sql_proctime_cumulate_1d_8h_{tzname}", source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:454-587",
            config=dict(mode="sql", kind="cumulate", size=24 * H, slide=8 * H, offset=0, tz_offset_ms=tz,
                        val_type="i64", count_star_index=-1, proctime=True),
            columns=["key", "sum", "count", "window_start", "window_end"],
            events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=0))

        # testProcessingTimeTumblingWindows :690-767 (tumble 5h)
        ev = []
        steps = []
        t = P("1970-01-01T00:00:00.003")
        ev += [E(2, 1, t), E(2, 1, t), E(2, 1, t), E(1, 1, t), E(1, 1, t)]
        ev.append(WM(P("1970-01-01T05:00:00"))); steps.append((len(ev) - 1, [[2, 3, 3, U("1970-01-01T00:00:00"), U("1970-01-01T05:00:00")],
                                                                             [1, 2, 2, U("1970-01-01T00:00:00"), U("1970-01-01T05:00:00")]]))
        t = P("1970-01-01T05:00:00")
        ev += [E(1, 1, t), E(1, 1, t), E(1, 1, t)]
        ev.append(WM(P("1970-01-01T10:00:01"))); steps.append((len(ev) - 1, [[1, 3, 3, U("1970-01-01T05:00:00"), U("1970-01-01T10:00:00")]]))
        out.append(dict(
            name=f"sql_proctime_tumble_5h_{tzname}", source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:690-767",
            config=dict(mode="sql", kind="tumble", size=5 * H, slide=0, offset=0, tz_offset_ms=tz,
                        val_type="i64", count_star_index=-1, proctime=True),
            columns=["key", "sum", "count", "window_start", "window_end"],
            events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=0))
    return out


# ----------------------------------------------------------------------------------------
# WindowOperatorTest (SJT/runtime/operators/windowing/WindowOperatorTest.java): SumReducer
# over Tuple2<String,Integer>; output StreamRecord((key, sum), window.maxTimestamp()).
# Columns checked: key, sum, out_ts.
# ----------------------------------------------------------------------------------------
def datastream_fixtures():
    out = []
    base = [E(2, 1, 3999), E(2, 1, 3000), E(1, 1, 20), E(1, 1, 0), E(1, 1, 999),
            E(2, 1, 1998), E(2, 1, 1999), E(2, 1, 1000)]
    # testTumblingEventTimeWindows :293-353 driven by testTumblingEventTimeWindowsReduce :398-433
    ev = list(base)
    steps = []
    ev.append(WM(999)); steps.append((len(ev) - 1, []))
    ev.append(WM(1999)); steps.append((len(ev) - 1, []))
    ev.append(SNAP)
    ev.append(WM(2999)); steps.append((len(ev) - 1, [[1, 3, 2999], [2, 3, 2999]]))
    ev.append(WM(3999)); steps.append((len(ev) - 1, []))
    ev.append(WM(4999)); steps.append((len(ev) - 1, []))
    ev.append(WM(5999)); steps.append((len(ev) - 1, [[2, 2, 5999]]))
    ev.append(WM(6999)); steps.append((len(ev) - 1, []))
    ev.append(WM(7999)); steps.append((len(ev) - 1, []))
    out.append(dict(
        name="ds_tumble_3s_reduce", source="SJT/runtime/operators/windowing/WindowOperatorTest.java:293-353,398-433",
        config=dict(mode="datastream", kind="tumble", size=3000, slide=0, offset=0, tz_offset_ms=0,
                    val_type="i64", count_star_index=-1),
        columns=["key", "sum", "out_ts"],
        events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=0))
    # testSlidingEventTimeWindows :108-211 driven by testSlidingEventTimeWindowsReduce :215-
    ev = list(base)
    steps = []
    ev.append(WM(999)); steps.append((len(ev) - 1, [[1, 3, 999]]))
    ev.append(WM(1999)); steps.append((len(ev) - 1, [[1, 3, 1999], [2, 3, 1999]]))
    ev.append(WM(2999)); steps.append((len(ev) - 1, [[1, 3, 2999], [2, 3, 2999]]))
    ev.append(SNAP)
    ev.append(WM(3999)); steps.append((len(ev) - 1, [[2, 5, 3999]]))
    ev.append(WM(4999)); steps.append((len(ev) - 1, [[2, 2, 4999]]))
    ev.append(WM(5999)); steps.append((len(ev) - 1, [[2, 2, 5999]]))
    ev.append(WM(6999)); steps.append((len(ev) - 1, []))
    ev.append(WM(7999)); steps.append((len(ev) - 1, []))
    out.append(dict(
        name="ds_sliding_3s_1s_reduce", source="SJT/runtime/operators/windowing/WindowOperatorTest.java:108-211,215-250",
        config=dict(mode="datastream", kind="hop", size=3000, slide=1000, offset=0, tz_offset_ms=0,
                    val_type="i64", count_star_index=-1),
        columns=["key", "sum", "out_ts"],
        events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=0))
    # testSideOutputDueToLatenessTumbling :1975-2053 (2 s tumbling, allowedLateness 0,
    # EventTimeTrigger): the element at 1998 arrives after WM 1999 fired its window -> late (the
    # reference side-outputs it; here it is counted in numLateRecordsDropped)
    ev, steps = [], []
    ev.append(E(2, 1, 1000)); ev.append(WM(1985)); steps.append((len(ev) - 1, []))
    ev.append(E(2, 1, 1980)); ev.append(WM(1999)); steps.append((len(ev) - 1, [[2, 2, 1999]]))
    ev.append(E(2, 1, 1998)); ev.append(E(2, 1, 2001))
    ev.append(WM(2999)); steps.append((len(ev) - 1, []))
    ev.append(WM(3999)); steps.append((len(ev) - 1, [[2, 1, 3999]]))
    out.append(dict(
        name="ds_tumble_2s_lateness0_side_output",
        source="SJT/runtime/operators/windowing/WindowOperatorTest.java:1975-2053",
        config=dict(mode="datastream", kind="tumble", size=2000, slide=0, offset=0, tz_offset_ms=0,
                    val_type="i64", count_star_index=-1),
        columns=["key", "sum", "out_ts"],
        events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=1))
    # testSideOutputDueToLatenessSliding :2055-2151 (3 s / 1 s sliding, allowedLateness 0): the
    # elements at 2400 are late for the window ending 2999 only and stay in 3999 / 4999; the last
    # 3001 is late for all three of its windows -> late
    ev, steps = [], []
    ev.append(E(2, 1, 1000)); ev.append(WM(1999)); steps.append((len(ev) - 1, [[2, 1, 1999]]))
    ev.append(E(2, 1, 2000)); ev.append(WM(3000)); steps.append((len(ev) - 1, [[2, 2, 2999]]))
    for e in (E(1, 1, 3001), E(2, 1, 2400), E(2, 1, 2400), E(1, 1, 3001), E(2, 1, 3900)):
        ev.append(e)
    ev.append(WM(6000)); steps.append((len(ev) - 1, [[2, 5, 3999], [1, 2, 3999], [2, 4, 4999], [1, 2, 4999],
                                                     [2, 1, 5999], [1, 2, 5999]]))
    ev.append(E(1, 1, 3001))
    ev.append(WM(25000)); steps.append((len(ev) - 1, []))
    out.append(dict(
        name="ds_sliding_3s_1s_lateness0_side_output",
        source="SJT/runtime/operators/windowing/WindowOperatorTest.java:2055-2151",
        config=dict(mode="datastream", kind="hop", size=3000, slide=1000, offset=0, tz_offset_ms=0,
                    val_type="i64", count_star_index=-1),
        columns=["key", "sum", "out_ts"],
        events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=1))
    # testLateness :1805-1886 (2 s tumbling, allowedLateness 500, PurgingTrigger.of(EventTimeTrigger)):
    # the element at 1997 arrives after WM 2300 fired and purged its window but before its cleanup
    # time 1999 + 500 -> it re-fires the window at once with only itself ("this is 1 and not 3
    # because the trigger fires and purges"); the element at 1998 after WM 6000 is late (the
    # reference side-outputs it; here it is counted in numLateRecordsDropped)
    ev, steps = [], []
    ev.append(E(2, 1, 500)); ev.append(WM(1500)); steps.append((len(ev) - 1, []))
    ev.append(E(2, 1, 1300)); ev.append(WM(2300)); steps.append((len(ev) - 1, [[2, 2, 1999]]))
    ev.append(E(2, 1, 1997)); ev.append(WM(6000)); steps.append((len(ev) - 1, [[2, 1, 1999]]))
    ev.append(E(2, 1, 1998)); ev.append(WM(7000)); steps.append((len(ev) - 1, []))
    out.append(dict(
        name="ds_tumble_2s_lateness500_purging",
        source="SJT/runtime/operators/windowing/WindowOperatorTest.java:1805-1886",
        config=dict(mode="datastream", kind="tumble", size=2000, slide=0, offset=0, tz_offset_ms=0,
                    val_type="i64", count_star_index=-1, allowed_lateness=500, purging=True),
        columns=["key", "sum", "out_ts"],
        events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=1))
    # testCleanupTimeOverflow :1888-1971 (1 s tumbling, allowedLateness 2000, EventTimeTrigger):
    # the window of Long.MAX_VALUE - 1750 has maxTimestamp + lateness past Long.MAX_VALUE -> its
    # cleanup time is Long.MAX_VALUE (no wrapped-around timer cleans it at MAX - 1500); it fires at
    # its maxTimestamp
    jmax = (1 << 63) - 1
    ts = jmax - 1750
    start = jmax - 1807   # getWindowStartWithOffset(ts, 0, 1000): (ts + 1000) wraps, Java % keeps its sign
    max_ts = start + 1000 - 1
    ev, steps = [], []
    ev.append(E(2, 1, ts)); ev.append(WM(jmax - 1500)); steps.append((len(ev) - 1, []))
    ev.append(WM(max_ts)); steps.append((len(ev) - 1, [[2, 1, max_ts]]))
    out.append(dict(
        name="ds_tumble_1s_lateness2000_cleanup_overflow",
        source="SJT/runtime/operators/windowing/WindowOperatorTest.java:1888-1971",
        config=dict(mode="datastream", kind="tumble", size=1000, slide=0, offset=0, tz_offset_ms=0,
                    val_type="i64", count_star_index=-1, allowed_lateness=2000),
        columns=["key", "sum", "out_ts"],
        events=ev, expected=[dict(after_event=i, rows=r) for i, r in steps], expected_late_dropped=0))
    return out


# ----------------------------------------------------------------------------------------
# WindowAggregateITCase (TPT/runtime/stream/sql/WindowAggregateITCase.scala) over
# TestData.windowDataWithTimestamp (TPT/runtime/utils/TestData.scala:601-615):
#   (ts, `double`, name); name a -> 1, b -> 2, null -> 3.
# WATERMARK rowtime - INTERVAL '1' SECOND (:127), emitted after every record here; end of
# input emits Long.MAX_VALUE. Checked: COUNT(*) per (name, window) and whether the
# column `double` had any non-null value (MAX(`double`) is null iff COUNT(`double`) = 0).
# Columns: key, window_start, window_end, cnt_star, val_all_null.
# ----------------------------------------------------------------------------------------
ITCASE_ROWS = [  # (ts, double or None, name)
    ("2020-10-10 00:00:01", 1.0, 1), ("2020-10-10 00:00:02", 2.0, 1), ("2020-10-10 00:00:03", 2.0, 1),
    ("2020-10-10 00:00:04", 5.0, 1), ("2020-10-10 00:00:07", 3.0, 2), ("2020-10-10 00:00:06", 6.0, 2),
    ("2020-10-10 00:00:08", None, 1), ("2020-10-10 00:00:04", 5.0, 1), ("2020-10-10 00:00:16", 4.0, 2),
    ("2020-10-10 00:00:32", 7.0, 3), ("2020-10-10 00:00:34", 3.0, 2),
]


def itcase_fixtures():
    ev = []
    mx = -(1 << 63)
    for ts, d, name in ITCASE_ROWS:
        t = utc_ms(ts.replace(" ", "T"))
        ev.append(E(name, 0.0 if d is None else d, t, 1 if d is None else 0))
        mx = max(mx, t)
        ev.append(WM(mx - 1000))
    ev.append(WM(JMAX))
    T = lambda s: utc_ms("2020-10-10T" + s)
    Tm = lambda s: utc_ms("2020-10-09T" + s)
    tumble = [  # testEventTimeTumbleWindow :176-207
        [1, T("00:00:00"), T("00:00:05"), 4, 0], [1, T("00:00:05"), T("00:00:10"), 1, 1],
        [2, T("00:00:05"), T("00:00:10"), 2, 0], [2, T("00:00:15"), T("00:00:20"), 1, 0],
        [2, T("00:00:30"), T("00:00:35"), 1, 0], [3, T("00:00:30"), T("00:00:35"), 1, 0],
    ]
    hop = [  # testEventTimeHopWindow :394-430 (HOP slide 5s, size 10s)
        [1, Tm("23:59:55"), T("00:00:05"), 4, 0], [1, T("00:00:00"), T("00:00:10"), 6, 0],
        [1, T("00:00:05"), T("00:00:15"), 1, 1], [2, T("00:00:00"), T("00:00:10"), 2, 0],
        [2, T("00:00:05"), T("00:00:15"), 2, 0], [2, T("00:00:10"), T("00:00:20"), 1, 0],
        [2, T("00:00:15"), T("00:00:25"), 1, 0], [2, T("00:00:25"), T("00:00:35"), 1, 0],
        [2, T("00:00:30"), T("00:00:40"), 1, 0], [3, T("00:00:25"), T("00:00:35"), 1, 0],
        [3, T("00:00:30"), T("00:00:40"), 1, 0],
    ]
    cumulate = [  # testEventTimeCumulateWindow :519-562 (CUMULATE step 5s, max 15s)
        [1, T("00:00:00"), T("00:00:05"), 4, 0], [1, T("00:00:00"), T("00:00:10"), 6, 0],
        [1, T("00:00:00"), T("00:00:15"), 6, 0], [2, T("00:00:00"), T("00:00:10"), 2, 0],
        [2, T("00:00:00"), T("00:00:15"), 2, 0], [2, T("00:00:15"), T("00:00:20"), 1, 0],
        [2, T("00:00:15"), T("00:00:25"), 1, 0], [2, T("00:00:15"), T("00:00:30"), 1, 0],
        [2, T("00:00:30"), T("00:00:35"), 1, 0], [2, T("00:00:30"), T("00:00:40"), 1, 0],
        [2, T("00:00:30"), T("00:00:45"), 1, 0], [3, T("00:00:30"), T("00:00:35"), 1, 0],
        [3, T("00:00:30"), T("00:00:40"), 1, 0], [3, T("00:00:30"), T("00:00:45"), 1, 0],
    ]
    base = "TPT/runtime/stream/sql/WindowAggregateITCase.scala"
    cols = ["key", "window_start", "window_end", "cnt_star", "val_all_null"]
    mk = lambda name, src, cfg, rows: dict(
        name=name, source=src + "; data TPT/runtime/utils/TestData.scala:601-615",
        config=cfg, columns=cols, events=ev,
        expected=[dict(after_event="end", rows=rows)], expected_late_dropped=None)
    return [
        mk("itcase_tumble_5s", base + ":176-207",
           dict(mode="sql", kind="tumble", size=5000, slide=0, offset=0, tz_offset_ms=0, val_type="f64",
                count_star_index=0), tumble),
        mk("itcase_hop_10s_5s", base + ":394-430",
           dict(mode="sql", kind="hop", size=10000, slide=5000, offset=0, tz_offset_ms=0, val_type="f64",
                count_star_index=0), hop),
        mk("itcase_cumulate_15s_5s", base + ":519-562",
           dict(mode="sql", kind="cumulate", size=15000, slide=5000, offset=0, tz_offset_ms=0, val_type="f64",
                count_star_index=0), cumulate),
    ]


# ----------------------------------------------------------------------------------------
# The same three ITCase queries assert MAX(`double`) and MIN(`float`) per (name, window)
# (WindowAggregateITCase.scala:176-207 tumble, :394-430 hop, :519-562 cumulate; the data's
# `double` and `float` columns, TestData.scala:601-615, hold different NULLs: the 00:00:08
# row has no `double`, the late 00:00:04 row no `float`). MIN / MAX keep one value column
# per operator here, so each aggregate is a fixture of its own over its column; float
# values are exact in f64. The expected rows are the asserted strings
# "name,window_start,window_end,COUNT(*),SUM(bigdec),MAX(double),MIN(float),..." with
# name a -> 1, b -> 2, null -> 3.
# ----------------------------------------------------------------------------------------
ITCASE_FLOAT = [1.0, 2.0, 2.0, 5.0, 3.0, 6.0, 3.0, None, 4.0, 7.0, 3.0]   # the `float` column, row order

ITCASE_EXPECTED = {   # window -> [(name, start, end, COUNT(*), MAX(double), MIN(float))]
    "tumble": [   # :199-205
        ("a", "00:00", "00:00:05", 4, 5.0, 1.0), ("a", "00:00:05", "00:00:10", 1, None, 3.0),
        ("b", "00:00:05", "00:00:10", 2, 6.0, 3.0), ("b", "00:00:15", "00:00:20", 1, 4.0, 4.0),
        ("b", "00:00:30", "00:00:35", 1, 3.0, 3.0), ("null", "00:00:30", "00:00:35", 1, 7.0, 7.0)],
    "hop": [   # :416-428
        ("a", "-00:00:05", "00:00:05", 4, 5.0, 1.0), ("a", "00:00", "00:00:10", 6, 5.0, 1.0),
        ("a", "00:00:05", "00:00:15", 1, None, 3.0), ("b", "00:00", "00:00:10", 2, 6.0, 3.0),
        ("b", "00:00:05", "00:00:15", 2, 6.0, 3.0), ("b", "00:00:10", "00:00:20", 1, 4.0, 4.0),
        ("b", "00:00:15", "00:00:25", 1, 4.0, 4.0), ("b", "00:00:25", "00:00:35", 1, 3.0, 3.0),
        ("b", "00:00:30", "00:00:40", 1, 3.0, 3.0), ("null", "00:00:25", "00:00:35", 1, 7.0, 7.0),
        ("null", "00:00:30", "00:00:40", 1, 7.0, 7.0)],
    "cumulate": [   # :545-559
        ("a", "00:00", "00:00:05", 4, 5.0, 1.0), ("a", "00:00", "00:00:10", 6, 5.0, 1.0),
        ("a", "00:00", "00:00:15", 6, 5.0, 1.0), ("b", "00:00", "00:00:10", 2, 6.0, 3.0),
        ("b", "00:00", "00:00:15", 2, 6.0, 3.0), ("b", "00:00:15", "00:00:20", 1, 4.0, 4.0),
        ("b", "00:00:15", "00:00:25", 1, 4.0, 4.0), ("b", "00:00:15", "00:00:30", 1, 4.0, 4.0),
        ("b", "00:00:30", "00:00:35", 1, 3.0, 3.0), ("b", "00:00:30", "00:00:40", 1, 3.0, 3.0),
        ("b", "00:00:30", "00:00:45", 1, 3.0, 3.0), ("null", "00:00:30", "00:00:35", 1, 7.0, 7.0),
        ("null", "00:00:30", "00:00:40", 1, 7.0, 7.0), ("null", "00:00:30", "00:00:45", 1, 7.0, 7.0)],
}


def itcase_minmax_fixtures():
    NAME = {"a": 1, "b": 2, "null": 3}
    base = "TPT/runtime/stream/sql/WindowAggregateITCase.scala"
    src = {"tumble": ":176-207", "hop": ":394-430", "cumulate": ":519-562"}
    spec = {"tumble": dict(size=5000, slide=0), "hop": dict(size=10000, slide=5000),
            "cumulate": dict(size=15000, slide=5000)}

    def T(s):   # "00:00:05" on 2020-10-10; "-00:00:05" = 2020-10-09T23:59:55
        if s.startswith("-"):
            return utc_ms("2020-10-10T00:00:00") - (utc_ms("2020-10-10T" + s[1:]) - utc_ms("2020-10-10T00:00:00"))
        return utc_ms("2020-10-10T" + (s if s.count(":") == 2 else s + ":00"))

    out = []
    for agg, col in (("max", "double"), ("min", "float")):
        ev = []
        mx = -(1 << 63)
        for i, (ts, d, name) in enumerate(ITCASE_ROWS):
            v = d if col == "double" else ITCASE_FLOAT[i]
            t = utc_ms(ts.replace(" ", "T"))
            ev.append(E(name, 0.0 if v is None else v, t, 1 if v is None else 0))
            mx = max(mx, t)
            ev.append(WM(mx - 1000))
        ev.append(WM(JMAX))
        for kind in ("tumble", "hop", "cumulate"):
            rows = [[NAME[n], T(a), T(b), c, mxv if agg == "max" else mnv]
                    for n, a, b, c, mxv, mnv in ITCASE_EXPECTED[kind]]
            out.append(dict(
                name=f"itcase_{kind}_{agg}_{col}", source=base + src[kind] + "; data TPT/runtime/utils/TestData.scala:601-615",
                config=dict(mode="sql", kind=kind, offset=0, tz_offset_ms=0, val_type="f64", count_star_index=0,
                            aggs=["count_star", "count", agg], **spec[kind]),
                columns=["key", "window_start", "window_end", "cnt_star", agg], events=ev,
                expected=[dict(after_event="end", rows=rows)], expected_late_dropped=None))
    return out


# ----------------------------------------------------------------------------------------
# Slice assigner known answers (TRT/operators/window/slicing/*SliceAssignerTest.java),
# parameterized there over America/Los_Angeles and Asia/Shanghai; the fixed-offset zone
# Asia/Shanghai (and UTC) are transcribed. Inputs to assignSliceEnd are localMills(str)
# = utc(str) - tz; all other functions take and return utcMills.
# ----------------------------------------------------------------------------------------
def assigner_fixtures():
    H = 3600 * 1000
    U = lambda s: utc_ms(s)
    cases = []
    for tzname, tz in (("UTC", 0), ("Asia/Shanghai", SHANGHAI), ("America/Los_Angeles", -8 * H)):
        A = lambda s: U(s) - tz
        n0 = len(cases)
        cases.append(dict(
            name=f"tumbling_{tzname}", source="TRT/operators/window/slicing/TumblingSliceAssignerTest.java:47-153",
            config=dict(kind="tumble", size=5 * H, slide=0, offset=0, tz_offset_ms=tz),
            assign=[[A("1970-01-01T00:00:00"), U("1970-01-01T05:00:00")],
                    [A("1970-01-01T04:59:59.999"), U("1970-01-01T05:00:00")],
                    [A("1970-01-01T05:00:00"), U("1970-01-01T10:00:00")]],
            window_start=[[U("1970-01-01T00:00:00"), U("1969-12-31T19:00:00")],
                          [U("1970-01-01T05:00:00"), U("1970-01-01T00:00:00")],
                          [U("1970-01-01T10:00:00"), U("1970-01-01T05:00:00")]],
            expired=[[U("1970-01-01T00:00:00"), [U("1970-01-01T00:00:00")]],
                     [U("1970-01-01T05:00:00"), [U("1970-01-01T05:00:00")]],
                     [U("1970-01-01T10:00:00"), [U("1970-01-01T10:00:00")]]]))
        cases.append(dict(
            name=f"tumbling_offset_{tzname}", source="TRT/operators/window/slicing/TumblingSliceAssignerTest.java:62-77",
            config=dict(kind="tumble", size=5 * H, slide=0, offset=100, tz_offset_ms=tz),
            assign=[[A("1970-01-01T00:00:00.100"), U("1970-01-01T05:00:00.100")],
                    [A("1970-01-01T05:00:00.099"), U("1970-01-01T05:00:00.100")],
                    [A("1970-01-01T05:00:00.100"), U("1970-01-01T10:00:00.100")]]))
        cases.append(dict(
            name=f"hopping_{tzname}", source="TRT/operators/window/slicing/HoppingSliceAssignerTest.java:49-251",
            config=dict(kind="hop", size=5 * H, slide=1 * H, offset=0, tz_offset_ms=tz),
            assign=[[A("1970-01-01T00:00:00"), U("1970-01-01T01:00:00")],
                    [A("1970-01-01T04:59:59.999"), U("1970-01-01T05:00:00")],
                    [A("1970-01-01T05:00:00"), U("1970-01-01T06:00:00")]],
            window_start=[[U(f"1970-01-01T{h:02d}:00:00"), U(f"1969-12-31T{19 + h:02d}:00:00")] for h in range(5)]
            + [[U("1970-01-01T05:00:00"), U("1970-01-01T00:00:00")], [U("1970-01-01T06:00:00"), U("1970-01-01T01:00:00")],
               [U("1970-01-01T10:00:00"), U("1970-01-01T05:00:00")]],
            merge=[[U("1970-01-01T00:00:00"), None, [U("1970-01-01T00:00:00"), U("1969-12-31T23:00:00"), U("1969-12-31T22:00:00"),
                                                      U("1969-12-31T21:00:00"), U("1969-12-31T20:00:00")]],
                   [U("1970-01-01T05:00:00"), None, [U(f"1970-01-01T0{h}:00:00") for h in (5, 4, 3, 2, 1)]],
                   [U("1970-01-01T06:00:00"), None, [U(f"1970-01-01T0{h}:00:00") for h in (6, 5, 4, 3, 2)]]],
            next_trigger=[[U(f"1970-01-01T0{h}:00:00"), False, U(f"1970-01-01T0{h + 1}:00:00")] for h in range(7)]
            + [[U(f"1970-01-01T0{h}:00:00"), True, None] for h in range(7)]))
        cases.append(dict(
            name=f"hopping_expired_{tzname}", source="TRT/operators/window/slicing/HoppingSliceAssignerTest.java:150-165",
            config=dict(kind="hop", size=4 * H, slide=1 * H, offset=0, tz_offset_ms=tz),
            expired=[[U("1970-01-01T00:00:00"), [U("1969-12-31T21:00:00")]],
                     [U("1970-01-01T04:00:00"), [U("1970-01-01T01:00:00")]],
                     [U("1970-01-01T08:00:00"), [U("1970-01-01T05:00:00")]]]))
        cases.append(dict(
            name=f"hopping_offset_{tzname}", source="TRT/operators/window/slicing/HoppingSliceAssignerTest.java:65-80",
            config=dict(kind="hop", size=5 * H, slide=1 * H, offset=100, tz_offset_ms=tz),
            assign=[[A("1970-01-01T00:00:00.100"), U("1970-01-01T01:00:00.100")],
                    [A("1970-01-01T05:00:00.099"), U("1970-01-01T05:00:00.100")],
                    [A("1970-01-01T05:00:00.100"), U("1970-01-01T06:00:00.100")]]))
        cases.append(dict(
            name=f"cumulative_day_{tzname}", source="TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:48-63",
            config=dict(kind="cumulate", size=24 * H, slide=1 * H, offset=0, tz_offset_ms=tz),
            assign=[[A("1970-01-01T00:00:00"), U("1970-01-01T01:00:00")],
                    [A("1970-01-02T22:59:59.999"), U("1970-01-02T23:00:00")],
                    [A("1970-01-02T23:00:00"), U("1970-01-03T00:00:00")]]))
        cases.append(dict(
            name=f"cumulative_offset_{tzname}", source="TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:65-80",
            config=dict(kind="cumulate", size=5 * H, slide=1 * H, offset=100, tz_offset_ms=tz),
            assign=[[A("1970-01-01T00:00:00.100"), U("1970-01-01T01:00:00.100")],
                    [A("1970-01-01T05:00:00.099"), U("1970-01-01T05:00:00.100")],
                    [A("1970-01-01T05:00:00.100"), U("1970-01-01T06:00:00.100")]]))
        c5 = lambda s: U("1970-01-01T" + s)
        cases.append(dict(
            name=f"cumulative_5h_1h_{tzname}", source="TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:120-310",
            config=dict(kind="cumulate", size=5 * H, slide=1 * H, offset=0, tz_offset_ms=tz),
            window_start=[[c5("00:00:00"), U("1969-12-31T19:00:00")]]
            + [[c5(f"0{h}:00:00"), c5("00:00:00")] for h in (1, 2, 3, 4, 5)]
            + [[c5("06:00:00"), c5("05:00:00")], [c5("08:00:00"), c5("05:00:00")]],
            expired=[[c5("01:00:00"), []], [c5("02:00:00"), [c5("02:00:00")]], [c5("03:00:00"), [c5("03:00:00")]],
                     [c5("04:00:00"), [c5("04:00:00")]], [c5("05:00:00"), [c5("05:00:00"), c5("01:00:00")]],
                     [c5("06:00:00"), []], [c5("10:00:00"), [c5("10:00:00"), c5("06:00:00")]],
                     [c5("00:00:00"), [c5("00:00:00"), U("1969-12-31T20:00:00")]]],
            merge=[[c5("01:00:00"), c5("01:00:00"), []]]
            + [[c5(f"0{h}:00:00"), c5("01:00:00"), [c5(f"0{h}:00:00")]] for h in (2, 3, 4, 5)]
            + [[c5("06:00:00"), c5("06:00:00"), []], [c5("08:00:00"), c5("06:00:00"), [c5("08:00:00")]],
               [c5("10:00:00"), c5("06:00:00"), [c5("10:00:00")]],
               [c5("00:00:00"), U("1969-12-31T20:00:00"), [c5("00:00:00")]]],
            next_trigger=[[c5("00:00:00"), False, None]]
            + [[c5(f"0{h}:00:00"), False, c5(f"0{h + 1}:00:00")] for h in (1, 2, 3, 4)]
            + [[c5("05:00:00"), False, None], [c5("06:00:00"), False, c5("07:00:00")], [c5("00:00:00"), True, None]]
            + [[c5(f"0{h}:00:00"), True, c5(f"0{h + 1}:00:00")] for h in (1, 2, 3, 4)]
            + [[c5("05:00:00"), True, None], [c5("06:00:00"), True, c5("07:00:00")]]))
        if tzname == "America/Los_Angeles":   # the zone's rules (transitions), not a fixed offset
            for c in cases[n0:]:
                c["config"]["zone"] = tzname
                c["config"]["tz_offset_ms"] = 0
    cases += dst_assigner_fixtures()
    cases += windowed_assigner_fixtures()
    errors = [  # testInvalidParameters of each assigner test
        dict(config=dict(kind="tumble", size=-1000, slide=0, offset=0),
             message="Tumbling Window parameters must satisfy size > 0, but got size -1000ms.",
             source="TRT/operators/window/slicing/TumblingSliceAssignerTest.java:155-160"),
        dict(config=dict(kind="tumble", size=10000, slide=0, offset=20000),
             message="Tumbling Window parameters must satisfy abs(offset) < size, bot got size 10000ms and offset 20000ms.",
             source="TRT/operators/window/slicing/TumblingSliceAssignerTest.java:162-167"),
        dict(config=dict(kind="hop", size=-2000, slide=1000, offset=0),
             message="Hopping Window must satisfy slide > 0 and size > 0, but got slide 1000ms and size -2000ms.",
             source="TRT/operators/window/slicing/HoppingSliceAssignerTest.java:268-272"),
        dict(config=dict(kind="hop", size=2000, slide=-1000, offset=0),
             message="Hopping Window must satisfy slide > 0 and size > 0, but got slide -1000ms and size 2000ms.",
             source="TRT/operators/window/slicing/HoppingSliceAssignerTest.java:274-278"),
        dict(config=dict(kind="hop", size=5000, slide=2000, offset=0),
             message="Slicing Hopping Window requires size must be an integral multiple of slide, but got size 5000ms and slide 2000ms.",
             source="TRT/operators/window/slicing/HoppingSliceAssignerTest.java:280-284"),
        dict(config=dict(kind="cumulate", size=-5000, slide=1000, offset=0),
             message="Cumulative Window parameters must satisfy maxSize > 0 and step > 0, but got maxSize -5000ms and step 1000ms.",
             source="TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:316-321"),
        dict(config=dict(kind="cumulate", size=5000, slide=-1000, offset=0),
             message="Cumulative Window parameters must satisfy maxSize > 0 and step > 0, but got maxSize 5000ms and step -1000ms.",
             source="TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:322-327"),
        dict(config=dict(kind="cumulate", size=5000, slide=2000, offset=0),
             message="Cumulative Window requires maxSize must be an integral multiple of step, but got maxSize 5000ms and step 2000ms.",
             source="TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:328-333"),
        dict(config=dict(kind="hop", size=3000, slide=1000, offset=0, count_star_index=-1),
             message="Hopping window requires a COUNT(*) in the aggregate functions.",
             source="TRT/operators/aggregate/window/SlicingWindowAggOperatorTest.java:769-792"),
    ]
    return cases, errors


# testDstSaving of Tumbling/Hopping/CumulativeSliceAssignerTest (America/Los_Angeles, the
# 2021-03-14 gap and the 2021-11-07 overlap): assertSliceStartEnd(start, end, epoch) checks
# assignSliceEnd(epoch) == end and getWindowStart(end) == start (local times).
DST_EPOCHS = [1615708800000, 1615712400000, 1615716000000, 1615719600000,
              1636268400000, 1636272000000, 1636275600000, 1636279200000, 1636282800000, 1636286400000]


def dst_assigner_fixtures():
    H = 3600 * 1000
    U = lambda s: utc_ms(s + ":00")
    spec = [
        ("tumbling_dst", "TRT/operators/window/slicing/TumblingSliceAssignerTest.java:79-114",
         dict(kind="tumble", size=4 * H, slide=0),
         [("2021-03-14T00:00", "2021-03-14T04:00")] * 3 + [("2021-03-14T04:00", "2021-03-14T08:00")]
         + [("2021-11-07T00:00", "2021-11-07T04:00")] * 5 + [("2021-11-07T04:00", "2021-11-07T08:00")]),
        ("hopping_dst", "TRT/operators/window/slicing/HoppingSliceAssignerTest.java:82-117",
         dict(kind="hop", size=4 * H, slide=H),
         [("2021-03-13T21:00", "2021-03-14T01:00"), ("2021-03-13T22:00", "2021-03-14T02:00"),
          ("2021-03-14T00:00", "2021-03-14T04:00"), ("2021-03-14T01:00", "2021-03-14T05:00"),
          ("2021-11-06T21:00", "2021-11-07T01:00"), ("2021-11-06T22:00", "2021-11-07T02:00"),
          ("2021-11-06T22:00", "2021-11-07T02:00"), ("2021-11-06T23:00", "2021-11-07T03:00"),
          ("2021-11-07T00:00", "2021-11-07T04:00"), ("2021-11-07T01:00", "2021-11-07T05:00")]),
        ("cumulative_dst", "TRT/operators/window/slicing/CumulativeSliceAssignerTest.java:83-119",
         dict(kind="cumulate", size=4 * H, slide=H),
         [("2021-03-14T00:00", "2021-03-14T01:00"), ("2021-03-14T00:00", "2021-03-14T02:00"),
          ("2021-03-14T00:00", "2021-03-14T04:00"), ("2021-03-14T04:00", "2021-03-14T05:00"),
          ("2021-11-07T00:00", "2021-11-07T01:00"), ("2021-11-07T00:00", "2021-11-07T02:00"),
          ("2021-11-07T00:00", "2021-11-07T02:00"), ("2021-11-07T00:00", "2021-11-07T03:00"),
          ("2021-11-07T00:00", "2021-11-07T04:00"), ("2021-11-07T04:00", "2021-11-07T05:00")]),
    ]
    out = []
    for name, src, cfg, exp in spec:
        out.append(dict(
            name=name + "_America/Los_Angeles", source=src,
            config=dict(cfg, offset=0, tz_offset_ms=0, zone="America/Los_Angeles"),
            assign=[[e, U(end)] for e, (start, end) in zip(DST_EPOCHS, exp)],
            window_start=[[U(end), U(start)] for start, end in exp]))
    return out


# WindowedSliceAssignerTest (TRT/operators/window/slicing/WindowedSliceAssignerTest.java:57-170):
# SliceAssigners.windowed(0, inner) over tumbling(4 h), hopping(5 h, 1 h), cumulative(5 h, 1 h);
# parameterized over America/Los_Angeles and Asia/Shanghai, with the same answers (the window
# end attached to the row is taken as is; getWindowStart is the inner assigner's).
def windowed_assigner_fixtures():
    H = 3600 * 1000
    U = utc_ms
    d = lambda s: U("1970-01-01T" + s)
    out = []
    for zname, zcfg in (("America/Los_Angeles", dict(zone="America/Los_Angeles", tz_offset_ms=0)),
                        ("Asia/Shanghai", dict(tz_offset_ms=SHANGHAI))):
        src = "TRT/operators/window/slicing/WindowedSliceAssignerTest.java"
        out.append(dict(
            name=f"windowed_tumble_{zname}", source=src + ":57-84,152-163",
            config=dict(kind="tumble", size=4 * H, slide=0, offset=0, windowed=True, **zcfg),
            assign=[[d("00:00:00"), d("00:00:00")], [d("05:00:00"), d("05:00:00")], [d("10:00:00"), d("10:00:00")]],
            window_start=[[d("00:00:00"), U("1969-12-31T20:00:00")], [d("04:00:00"), d("00:00:00")],
                          [d("08:00:00"), d("04:00:00")]],
            expired=[[d("00:00:00"), [d("00:00:00")]], [d("04:00:00"), [d("04:00:00")]],
                     [d("10:00:00"), [d("10:00:00")]]]))
        out.append(dict(
            name=f"windowed_hop_{zname}", source=src + ":86-118",
            config=dict(kind="hop", size=5 * H, slide=H, offset=0, windowed=True, **zcfg),
            window_start=[[d(f"0{h}:00:00"), U(f"1969-12-31T{19 + h}:00:00")] for h in range(5)]
            + [[d("05:00:00"), d("00:00:00")], [d("06:00:00"), d("01:00:00")], [d("10:00:00"), d("05:00:00")]]))
        out.append(dict(
            name=f"windowed_cumulate_{zname}", source=src + ":120-150",
            config=dict(kind="cumulate", size=5 * H, slide=H, offset=0, windowed=True, **zcfg),
            window_start=[[d("00:00:00"), U("1969-12-31T19:00:00")]]
            + [[d(f"0{h}:00:00"), d("00:00:00")] for h in (1, 2, 3, 4, 5)]
            + [[d("06:00:00"), d("05:00:00")], [d("10:00:00"), d("05:00:00")]]))
    return out


# TimeWindowUtilTest (TRT/util/TimeWindowUtilTest.java:38-128): [zone, function, in, expected]
def timeutil_fixtures():
    U = utc_ms
    SH, LA = "Asia/Shanghai", "America/Los_Angeles"
    v = []
    for s, e in (("1970-01-01T00:00:01", -28799000), ("1970-01-01T07:59:59.999", -1), ("1970-01-01T08:00:01", 1000),
                 ("1970-01-01T08:00:00.001", 1)):
        v += [[SH, "to_epoch_for_timer", U(s), e], [SH, "to_epoch", U(s), e]]
    for s, e in (("2021-03-14T00:00:00", 1615708800000), ("2021-03-14T01:00:00", 1615712400000),
                 ("2021-03-14T02:00:00", 1615716000000), ("2021-03-14T02:30:00", 1615716000000),
                 ("2021-03-14T02:59:59", 1615716000000), ("2021-03-14T03:00:00", 1615716000000),
                 ("2021-03-14T03:30:00", 1615717800000), ("2021-03-14T03:59:59", 1615719599000),
                 ("2021-11-07T00:00:00", 1636268400000), ("2021-11-07T01:00:00", 1636275600000),
                 ("2021-11-07T02:00:00", 1636279200000), ("2021-11-07T00:00:01", 1636268401000),
                 ("2021-11-07T01:59:59", 1636279199000), ("2021-11-07T02:00:01", 1636279201000)):
        v.append([LA, "to_epoch_for_timer", U(s), e])
    for s, e in (("2021-03-14T00:00:00", 1615708800000), ("2021-03-14T01:00:00", 1615712400000),
                 ("2021-03-14T02:00:00", 1615716000000), ("2021-03-14T02:30:00", 1615717800000),
                 ("2021-03-14T02:59:59", 1615719599000), ("2021-03-14T03:30:00", 1615717800000),
                 ("2021-03-14T03:00:00", 1615716000000),
                 ("2021-11-07T00:00:00", 1636268400000), ("2021-11-07T01:00:00", 1636272000000),
                 ("2021-11-07T02:00:00", 1636279200000), ("2021-11-07T00:00:01", 1636268401000),
                 ("2021-11-07T01:59:59", 1636275599000), ("2021-11-07T02:00:01", 1636279201000)):
        v.append([LA, "to_epoch", U(s), e])
    for t, s in ((1636272000000, "2021-11-07T01:00:00"), (1636275600000, "2021-11-07T01:00:00"),
                 (1636272001000, "2021-11-07T01:00:01"), (1636275599000, "2021-11-07T01:59:59")):
        v.append([LA, "to_utc", t, U(s)])
    for f in ("to_utc", "to_epoch_for_timer", "to_epoch"):   # testMaxWatermark
        v.append([SH, f, JMAX, JMAX])
    return v


def main():
    ops = slicing_operator_fixtures() + datastream_fixtures() + itcase_fixtures() + itcase_minmax_fixtures()
    with open(os.path.join(HERE, "operator_cases.json"), "w") as f:
        json.dump(ops, f, indent=1)
    cases, errors = assigner_fixtures()
    with open(os.path.join(HERE, "assigner_cases.json"), "w") as f:
        json.dump(dict(cases=cases, errors=errors, timeutil=timeutil_fixtures()), f, indent=1)
    print(f"wrote {len(ops)} operator cases, {len(cases)} assigner cases, {len(errors)} error cases")


if __name__ == "__main__":
    main()
