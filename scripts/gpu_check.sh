# GPU check: parity tests, then the bench (optionally without the CPU baseline: NOCPU=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
EXTRA=""
[ -n "$NOCPU" ] && EXTRA="--no-cpu-baseline"
timeout -k 10 300 python bench.py $EXTRA > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -c 3000 gpurun_out/bench.log
