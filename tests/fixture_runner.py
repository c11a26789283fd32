"""Drives a golden fixture (tests/golden/operator_cases.json) through an operator.

The operator is either the oracle (oracle.OracleOperator) or the product engine
(flink_amd.SlicingWindowAggOperator); both expose the reference operator's surface:
process_batch / process_watermark / prepare_snapshot / restore_copy / take_rows /
late_dropped.  Rows are compared SORTED per watermark step, as the reference's
RowDataHarnessAssertor.assertOutputEqualsSorted does.
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

KIND = {"tumble": 0, "hop": 1, "cumulate": 2}
VT = {"none": 0, "i64": 1, "f64": 2}
MODE = {"sql": 0, "datastream": 1}


def load_operator_cases():
    with open(os.path.join(GOLDEN, "operator_cases.json")) as f:
        return json.load(f)


def load_assigner_cases():
    with open(os.path.join(GOLDEN, "assigner_cases.json")) as f:
        return json.load(f)


def project(rows: np.ndarray, columns, val_type: str):
    """Reference-visible columns of fired rows (None = SQL NULL)."""
    out = []
    for r in rows:
        t = []
        for c in columns:
            if c == "key":
                t.append(int(r["key"]))
            elif c == "sum":
                if r["sum_null"]:
                    t.append(None)
                else:
                    t.append(int(r["sum_i"]) if val_type == "i64" else float(r["sum_d"]))
            elif c == "count":
                t.append(int(r["cnt_val"]))
            elif c == "cnt_star":
                t.append(int(r["cnt_star"]))
            elif c == "val_all_null":
                t.append(1 if int(r["cnt_val"]) == 0 else 0)
            elif c in ("min", "max"):   # MIN / MAX accumulator: NULL iff no non-null value
                if int(r["cnt_val"]) == 0:
                    t.append(None)
                else:
                    t.append(int(r[c + "_i"]) if val_type == "i64" else float(r[c + "_d"]))
            else:
                t.append(int(r[c]))
        out.append(tuple(t))
    return sorted(out, key=lambda x: tuple((v is None, v) for v in x))


def _norm(rows):
    return sorted([tuple(x) for x in rows], key=lambda x: tuple((v is None, v) for v in x))


def run_case(case, make_operator):
    """make_operator(cfg_dict) -> operator. Returns list of (step, got, expected)."""
    cfg = case["config"]
    op = make_operator(cfg)
    vt = cfg["val_type"]
    steps = {}
    for st in case["expected"]:
        steps[st["after_event"]] = _norm(st["rows"])
    collected = []
    results = []
    ev = case["events"]
    i = 0
    while i < len(ev):
        e = ev[i]
        if e[0] == "e":
            # group consecutive records into one batch (a micro-batch between watermarks)
            j = i
            while j < len(ev) and ev[j][0] == "e":
                j += 1
            blk = ev[i:j]
            key = np.array([b[1] for b in blk], dtype=np.int64)
            ts = np.array([b[3] for b in blk], dtype=np.int64)
            if vt == "f64":
                val = np.array([float(b[2]) for b in blk], dtype=np.float64)
            else:
                val = np.array([int(b[2]) for b in blk], dtype=np.int64)
            isnull = np.array([b[4] for b in blk], dtype=np.uint8)
            op.process_batch(key, ts, val, isnull if isnull.any() else None)
            i = j
            continue
        if e[0] == "wm":
            op.process_watermark(e[1])
        elif e[0] == "snapshot_restore":
            op.prepare_snapshot()
            new = op.restore_copy()
            op.close()
            op = new
        got = op.take_rows()
        collected.append(got)
        if i in steps:
            results.append((i, project(got, case["columns"], vt), steps[i]))
        i += 1
    if "end" in steps:
        allrows = np.concatenate(collected) if collected else np.zeros(0)
        results.append(("end", project(allrows, case["columns"], vt), steps["end"]))
    late = op.late_dropped
    op.close()
    return results, late
