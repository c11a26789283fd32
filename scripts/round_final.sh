# Round-end evidence on one GPU box: every GPU test, the driver's default bench command, then the
# profile recipe (kernel trace + PMC passes) of the same build. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 500 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -c 600 gpurun_out/bench_default.log
bash scripts/profile.sh ${1:-r02final} 200000000
