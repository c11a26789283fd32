# Round 5 GPU check: named tests first (TESTS, space-separated pytest ids), then optionally the
# whole GPU suite and the default bench. Every step under its own time limit; stops at the first failure.
# Usage (GPU box, repo root): TESTS="..." bash scripts/gpu_r5.sh TAG [SUITE=0] [BENCH=0] [EXTRA_BENCH_ARGS]
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
if [ -n "$TESTS" ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS \
    > $O/new_tests.log 2>&1 || { echo "new tests failed"; tail -60 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
fi
if [ "${2:-0}" = 1 ]; then
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_suite.log 2>&1 || { echo "suite failed"; tail -60 $O/gpu_suite.log; exit 1; }
tail -3 $O/gpu_suite.log
fi
if [ "${3:-0}" = 1 ]; then
timeout -k 10 400 python bench.py $4 > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
tail -c 1500 $O/bench.log
fi
