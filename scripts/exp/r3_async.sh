# Round 3: async watermark advance -- its GPU tests, bench A/B (async vs --wm-sync), then the GPU suite
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3a
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py -x -v --timeout 120 --timeout-method thread > $O/async_tests.log 2>&1 || { echo "async tests failed"; tail -30 $O/async_tests.log; exit 1; }
for M in "" "--wm-sync" "" "--wm-sync"; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --h2d-records 0 --steps 10 $M > $O/b${M:-async}.$RANDOM.log 2>&1 || { echo "bench $M failed"; exit 1; }
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_suite.log; exit 1; }
tail -3 $O/gpu_suite.log
echo done
