# Round 3: CUMULATE restore fix -- async/restore tests, then the whole GPU suite
set -o pipefail
O=gpurun_out/r3fix
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py -x -q --timeout 150 --timeout-method thread > $O/async.log 2>&1 || { tail -30 $O/async.log; exit 1; }
tail -1 $O/async.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
