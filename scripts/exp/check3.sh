# key dictionary + two-phase parity, then the 2-rank one-GPU rehearsal of the exchange path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "keys or two_phase or partials" > gpurun_out/check3_tests.log 2>&1
rc=$?
tail -4 gpurun_out/check3_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit $rc; fi
REC=200000000 BENCH_ARGS="--h2d-records 0" bash scripts/rehearse_2rank.sh
