"""flink_amd -- MI355X-native keyed window aggregation for Flink's window operators.

The hot path (slice assignment, keyed hash aggregation in HBM/LDS, slice merge on window
fire, key-group routing) lives in libflinkgpu.so (HIP for gfx950, C-ABI in
include/flinkgpu.h). This package is the host-side mirror of the reference operator
interface used by tests and the benchmark; see DESIGN.md and INTEGRATION.md.
"""
from ._lib import FlinkGpuError, HostRegistration, WindowSpecError  # noqa: F401
from .window_agg import Window, WindowAggOperator, cumulative, hopping, key_groups, tumbling  # noqa: F401
from .composite import CompositeWindowAggOperator, window_agg_operator  # noqa: F401
from .keys import KeyDictionary, decode_key_row, key_row  # noqa: F401

__all__ = ["WindowAggOperator", "CompositeWindowAggOperator", "window_agg_operator", "Window", "tumbling", "hopping", "cumulative", "key_groups",
           "KeyDictionary", "key_row", "decode_key_row", "FlinkGpuError", "WindowSpecError", "HostRegistration"]
