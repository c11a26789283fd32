"""Teardown of operators that are never closed (Flink's failover path disposes an operator mid-
failure; round 3 saw a pytest process dump core after a test failed with async fires pending).

Each case runs in a fresh child process: it opens operators, stages batches (host and device
columns), queues asynchronous watermarks whose rows are never collected, then raises. The operators
are torn down by the interpreter's finalization (WindowAggOperator.__del__ -> fg_close) while the
exception's traceback still holds them. The child must exit with Python's status for an uncaught
exception (1) -- no signal, no abort, no core."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
sys.path.insert(0, {root!r})
import numpy as np
import flink_amd as F
from tests.streams import make_stream

mode = {mode!r}
n, keys, batch = 600_000, 40_000, 100_000
key, ts, val, _ = make_stream(n, keys, "f64")
ops = []
for kind in (F.tumbling(1000), F.hopping(4000, 1000), F.cumulative(4000, 1000)):
    op = F.WindowAggOperator(kind, aggs=("count_star", "sum", "avg"), val_type="f64", expected_keys=keys,
                             buffer_records=4 * batch)
    ops.append(op)
    if mode == "device":
        import torch
        dk, dt, dv = (torch.from_numpy(a).cuda() for a in (key, ts, val))
    for lo in range(0, n, batch):
        if mode == "device":
            op.process_batch(dk[lo:lo + batch], dt[lo:lo + batch], dv[lo:lo + batch])
        else:
            op.process_batch(key[lo:lo + batch], ts[lo:lo + batch], val[lo:lo + batch])
        op.process_watermark(int(ts[lo:lo + batch].max()) - 1, device_output=True, wait=False)
    if mode == "device":
        del dk, dt, dv   # freed (to torch's cache) while the engine may still read them
print("queued", flush=True)
raise RuntimeError("failure with uncollected async fires and open operators")
'''


@pytest.mark.parametrize("mode", ["host", "device"])
def test_unclosed_operators_with_pending_async_fires_exit_cleanly(mode):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, mode=mode)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert "queued" in p.stdout, p.stderr[-2000:]
    assert "failure with uncollected async fires" in p.stderr
    assert p.returncode == 1, f"child exited with {p.returncode}:\n{p.stderr[-3000:]}"
    assert "core dumped" not in p.stderr and "Segmentation" not in p.stderr
