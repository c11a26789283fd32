# Round 4 GPU check: the new / changed tests first, then the whole GPU suite, then the default bench.
# Usage (GPU box, repo root): bash scripts/gpu_r4.sh TAG [SUITE=1] [BENCH=1]
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_teardown.py tests/test_gpu_async.py "tests/test_gpu_parity.py::test_datastream_lateness_wide_late_keys" \
    > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -40 $O/new_tests.log; exit 1; }
tail -2 $O/new_tests.log
if [ "${2:-1}" = 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
fi
if [ "${3:-1}" = 1 ]; then
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -c 2500 $O/bench.log
fi
