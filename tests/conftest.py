import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O
    O.build()
    return O


def pytest_sessionfinish(session, exitstatus):
    """DOUBLE SUM / AVG tolerance accounting of the GPU parity tests: per test and column, the
    rows checked and those within the summation-order bound but not within 1e-9 relative
    (mixed-sign and cancelling streams, tests/test_gpu_parity.py assert_rows_equal), written to
    gpurun_out/tolerance_report.json."""
    import json
    mod = sys.modules.get("tests.test_gpu_parity")
    rep = getattr(mod, "TOLERANCE", None) if mod else None
    if not rep:
        return
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    tot = [sum(v[0] for d in rep.values() for v in d.values()), sum(v[1] for d in rep.values() for v in d.values())]
    with open(os.path.join(out, "tolerance_report.json"), "w") as f:
        json.dump({"rows_checked": tot[0], "rows_on_order_bound_only": tot[1],
                   "tests": {k: v for k, v in sorted(rep.items()) if any(x[1] for x in v.values())}}, f, indent=1)
