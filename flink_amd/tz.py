"""Shift time zones with daylight saving: the zone rules the engine is handed.

The reference converts between epoch millis and "UTC-shifted" local millis with
java.time zone rules (TR/util/TimeWindowUtil.java:53-61 toUtcTimestampMills,
:70-140 toEpochMillsForTimer, :149-157 toEpochMills), and picks the daylight-saving
branch of getNextTriggerWatermark / toEpochMillsForTimer when
TimeZone.getTimeZone(zone).useDaylightTime() (:76, :187-210;
AbstractWindowAggProcessor's useDayLightSaving). The C-ABI takes those rules as data
(fg_config.tz_transition_ms / tz_offset_ms / tz_use_daylight, what ZoneRules.getTransitions()
yields on the Java side): the instants at which the offset changes and the offset in force
between them. Here they come from the IANA database of the `tzdata` package (zoneinfo).
"""
from __future__ import annotations

import datetime as _dt
import functools
import zoneinfo

import numpy as np

_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
_DAY = 86400


def _offset_s(z: zoneinfo.ZoneInfo, t: int) -> int:
    """ZoneRules.getOffset(Instant) in seconds, for an epoch second t."""
    return int((_EPOCH + _dt.timedelta(seconds=t)).astimezone(z).utcoffset().total_seconds())


@functools.lru_cache(maxsize=64)
def zone_rules(name: str, first_year: int = 1900, last_year: int = 2100):
    """(transition instants ms int64[n], offsets ms int64[n + 1], use_daylight) for zone
    `name` over [first_year, last_year): offsets[i] is in force before transition i,
    offsets[n] after the last. Transitions are found by a daily scan of the zone's offset
    and bisected to the second (zone transitions fall on whole seconds)."""
    z = zoneinfo.ZoneInfo(name)
    t0 = int(_dt.datetime(first_year, 1, 1, tzinfo=_dt.timezone.utc).timestamp())
    t1 = int(_dt.datetime(last_year, 1, 1, tzinfo=_dt.timezone.utc).timestamp())
    trans, offs = [], [_offset_s(z, t0)]
    prev_t, prev_o = t0, offs[0]
    for t in range(t0 + _DAY, t1 + 1, _DAY):
        o = _offset_s(z, t)
        if o == prev_o:
            prev_t = t
            continue
        lo, hi = prev_t, t          # offset(lo) == prev_o != offset(hi)
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if _offset_s(z, mid) == prev_o:
                lo = mid
            else:
                hi = mid
        trans.append(hi * 1000)
        offs.append(o)
        prev_t, prev_o = t, o
    # TimeZone.useDaylightTime(): the zone's current rules observe daylight saving
    y = _dt.datetime.now(_dt.timezone.utc).year
    jan = int(_dt.datetime(y, 1, 15, tzinfo=_dt.timezone.utc).timestamp())
    jul = int(_dt.datetime(y, 7, 15, tzinfo=_dt.timezone.utc).timestamp())
    use_dst = _offset_s(z, jan) != _offset_s(z, jul)
    return (np.asarray(trans, dtype=np.int64), np.asarray([o * 1000 for o in offs], dtype=np.int64), use_dst)


def fixed_offset_ms(name: str):
    """The zone's offset in ms when it never changed over the table's range (a fixed-offset
    zone such as UTC or 'GMT+08:00'), else None."""
    trans, offs, _ = zone_rules(name)
    return int(offs[0]) if len(trans) == 0 else None
