"""CPU-side checks of the drop-in boundary: libflinkgpu.so loads, exports every symbol that
include/flinkgpu.h declares, and validates window specs exactly like the reference (the
validation runs before any device call, so no GPU is needed)."""
import ctypes as C
import os
import re

import pytest

from flink_amd import _lib as L
from tests.fixture_runner import KIND, load_assigner_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "flinkgpu.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|void\*?|const char\*|void)\s+\*?(fg_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    syms = declared_symbols()
    assert set(syms) == set(L.EXPORTS), syms


def test_library_exports_every_declared_symbol():
    lib = L.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert lib.fg_abi_version() == 16


def test_struct_layouts_match_header_sizes(tmp_path):
    """Every ctypes mirror of a C-ABI struct has the header's layout: offsetof/sizeof from the
    C compiler itself (gcc on include/flinkgpu.h) against the ctypes field offsets."""
    import subprocess
    structs = {"fg_config": L.FgConfig, "fg_batch": L.FgBatch, "fg_rows": L.FgRows, "fg_partials": L.FgPartials,
               "fg_state_rows": L.FgStateRows, "fg_row_batch": L.FgRowBatch, "fg_kernel_stat": L.FgKernelStat,
               "fg_stats": L.FgStats, "fg_exchanged": L.FgExchanged, "fg_round": L.FgRound,
               "fg_image_slices": L.FgImageSlices}
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "flinkgpu.h"', "int main(void) {"]
    for cname, py in structs.items():
        src.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            src.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    src.append("return 0; }")
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {(a, b): int(v) for a, b, v in (ln.split() for ln in out if ln)}
    for cname, py in structs.items():
        assert got[(cname, "size")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_binary_row_layout():
    """flink_amd.rows writes BinaryRowData fixed-length parts: the bit-set width of
    calculateBitSetWidthInBytes (BinaryRowData.java:70-72: 8 bytes up to 56 fields, 16 from 57),
    the null bit of field f at bit 8 + f (:155-157), 8 bytes per field after the bit set."""
    import numpy as np

    from flink_amd import rows as R
    assert [R.bit_set_width(a) for a in (1, 3, 56, 57, 120, 121)] == [8, 8, 8, 16, 16, 24]
    assert R.fixed_part_size(3) == 32
    r = R.pack_rows([np.array([5, -1], dtype=np.int64), np.array([100, 200], dtype=np.int64),
                     np.array([1.5, 2.5])], [None, None, np.array([False, True])], stride=40)
    r = r.reshape(2, 40)
    assert r[0, 0] == 0 and r[1, 1] == 1 << 2                       # field 2 NULL in row 1
    assert r[0, 8:16].view(np.int64)[0] == 5 and r[1, 8:16].view(np.int64)[0] == -1
    assert r[0, 24:32].view(np.float64)[0] == 1.5 and r[1, 24:32].view(np.int64)[0] == 0   # NULL: zero bytes


AS = load_assigner_cases()


@pytest.mark.parametrize("case", AS["errors"], ids=[e["message"][:40] for e in AS["errors"]])
def test_window_spec_errors_match_reference(case):
    import flink_amd as F
    c = case["config"]
    aggs = ("count_star", "sum") if c.get("count_star_index", 0) >= 0 else ("sum",)
    w = F.Window(KIND[c["kind"]], c["size"], c["slide"], c["offset"])
    with pytest.raises(F.WindowSpecError) as ei:
        F.WindowAggOperator(w, aggs=aggs, val_type="i64")
    assert str(ei.value) == case["message"]


def test_local_phase_needs_value_column():
    """FG_FLAG_LOCAL_PARTIALS is validated before any device call."""
    import flink_amd as F
    with pytest.raises(F.WindowSpecError):
        F.WindowAggOperator(F.tumbling(1000), val_type="none", local_partials=True)


def test_no_device_is_loud():
    """Without a GPU the product must fail, never fall back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import flink_amd as F
    with pytest.raises(F.FlinkGpuError) as ei:
        F.WindowAggOperator(F.tumbling(1000))
    assert ei.value.code == L.FG_EDEVICE


def test_proctime_only_for_sql():
    """FG_FLAG_PROCTIME is validated before any device call."""
    import flink_amd as F
    with pytest.raises(F.WindowSpecError):
        F.WindowAggOperator(F.tumbling(1000), mode="datastream", val_type="i64", proctime=True)


def test_zone_rules_validated_before_device():
    """Zone rules (daylight saving) are for SQL windows only, checked before any device call."""
    import flink_amd as F
    with pytest.raises(F.WindowSpecError):
        F.WindowAggOperator(F.tumbling(1000), mode="datastream", val_type="i64", zone="America/Los_Angeles")
    import torch
    if not torch.cuda.is_available():   # the local phase takes zone rules: valid, no device
        with pytest.raises(F.FlinkGpuError) as ei:
            F.WindowAggOperator(F.tumbling(1000), local_partials=True, zone="America/Los_Angeles")
        assert ei.value.code == L.FG_EDEVICE


def test_min_max_accumulator_rules():
    """MIN / MAX are SQL aggregates over the value column; they mix with the SUM family in one
    operator (value slots, include/flinkgpu.h fg_agg), the local phase included (its partial rows
    then carry SUM, MIN and MAX); validated before any device call."""
    import torch
    import flink_amd as F
    with pytest.raises(F.WindowSpecError):   # DataStream reduces one aggregation per window
        F.WindowAggOperator(F.tumbling(1000), aggs=("sum", "max"), mode="datastream", val_type="i64")
    with pytest.raises(F.WindowSpecError):
        F.WindowAggOperator(F.tumbling(1000), aggs=("count_star", "min"), val_type="none")
    if torch.cuda.is_available():
        return
    for aggs in (("count_star", "count", "min"), ("max",), ("count_star", "sum", "avg", "min", "max")):
        # valid: fails only for want of a device
        with pytest.raises(F.FlinkGpuError) as ei:
            F.WindowAggOperator(F.tumbling(1000), aggs=aggs, val_type="i64")
        assert ei.value.code == L.FG_EDEVICE
    for vt in ("i64", "f64"):   # WindowedStream.min / max (ComparableAggregator)
        for aggs in (("max",), ("count_star", "min")):
            with pytest.raises(F.FlinkGpuError) as ei:
                F.WindowAggOperator(F.tumbling(1000), aggs=aggs, mode="datastream", val_type=vt)
            assert ei.value.code == L.FG_EDEVICE
    for aggs in (("sum", "min"), ("min", "max"), ("avg", "max")):   # local phase, several accumulators
        with pytest.raises(F.FlinkGpuError) as ei:
            F.WindowAggOperator(F.tumbling(1000), aggs=aggs, val_type="f64", local_partials=True)
        assert ei.value.code == L.FG_EDEVICE


def test_accumulator_groups_split():
    """A query with several value accumulators maps to one handle per kind, each with
    COUNT(*) (flink_amd/composite.py)."""
    from flink_amd import _lib as L
    from flink_amd.composite import accumulator_groups
    codes, groups = accumulator_groups(("count_star", "sum", "avg", "min", "max"))
    assert groups == [(L.AGG_COUNT_STAR, L.AGG_SUM, L.AGG_AVG), (L.AGG_COUNT_STAR, L.AGG_MIN),
                      (L.AGG_COUNT_STAR, L.AGG_MAX)]
    _, groups = accumulator_groups(("count", "max"))
    assert groups == [(L.AGG_COUNT_STAR, L.AGG_COUNT, L.AGG_MAX)]
    _, groups = accumulator_groups(("sum",))
    assert groups == [(L.AGG_COUNT_STAR, L.AGG_SUM)]
