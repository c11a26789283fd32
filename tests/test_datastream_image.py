"""CPU checks of the DataStream state-image helpers (flink_amd.datastream): the aggregators'
reduce on value bits (SumAggregator, ComparableAggregator with Double.compareTo's order) and the
per-(key, window) group reduce that turns slice values into "window-contents" values."""
import numpy as np

from flink_amd.datastream import _group_reduce, reduce_bits

NAN = 0x7FF8000000000000


def _f(*x):
    return np.array(x, dtype=np.float64).view(np.int64)


def test_reduce_sum_wraps_like_java_long():
    a = np.array([(1 << 63) - 1, -5], dtype=np.int64)
    b = np.array([1, 7], dtype=np.int64)
    assert reduce_bits("sum", False, a, b).tolist() == [-(1 << 63), 2]


def test_reduce_minmax_double_compareto_order():
    # -0.0 < +0.0; every NaN equal and above +inf, carried canonical (Double.doubleToLongBits)
    assert reduce_bits("min", True, _f(0.0), _f(-0.0)).view(np.float64).tobytes() == _f(-0.0).tobytes()
    assert reduce_bits("max", True, _f(-0.0), _f(0.0)).tolist() == _f(0.0).tolist()
    odd_nan = np.array([0x7FF0000000000001], dtype=np.int64)
    assert reduce_bits("max", True, _f(np.inf), odd_nan).tolist() == [NAN]
    assert reduce_bits("min", True, odd_nan, _f(np.inf)).tolist() == _f(np.inf).tolist()
    assert reduce_bits("min", False, np.array([3]), np.array([-4])).tolist() == [-4]


def test_group_reduce_per_key_window():
    k = np.array([1, 1, 2, 1, 2, 1], dtype=np.int64)
    e = np.array([5, 5, 5, 6, 5, 5], dtype=np.int64)
    v = np.array([3, -7, 4, 2, 9, 10], dtype=np.int64)
    gk, ge, gs = _group_reduce("sum", False, k, e, v)
    assert list(zip(gk.tolist(), ge.tolist(), gs.tolist())) == [(1, 5, 6), (1, 6, 2), (2, 5, 13)]
    assert _group_reduce("min", False, k, e, v)[2].tolist() == [-7, 2, 4]
    assert _group_reduce("max", False, k, e, v)[2].tolist() == [10, 2, 9]
    fs = _group_reduce("sum", True, k, e, _f(0.1, 0.2, 1.0, 2.0, 3.0, 0.3))[2].view(np.float64)
    assert fs.tolist() == [(0.1 + 0.2) + 0.3, 2.0, 4.0]   # (left to right within a group)
