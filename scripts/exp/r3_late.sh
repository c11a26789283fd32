# Round 3: a pending async fire completes after the next batch's pass 1 is queued -- GPU suite, bench, trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3l
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py -x -q --timeout 120 --timeout-method thread > $O/async_tests.log 2>&1 || { echo "async tests failed"; tail -30 $O/async_tests.log; exit 1; }
tail -1 $O/async_tests.log
for M in "" "--batch 50000000" "" "--batch 50000000"; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --h2d-records 0 --steps 10 $M > $O/b$(echo $M | tr -d ' -').$RANDOM.log 2>&1 || { echo "bench $M failed"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --h2d-records 0 --steps 2 > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
echo done
