# Every GPU test (one pytest process), then smoke(). Usage: bash scripts/gpu_suite.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 450 --timeout-method thread -p no:cacheprovider \
    > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
