# two-phase + multi-value parity subset, then the 2-rank one-GPU rehearsal with five aggregates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "two_phase or golden or multi_accumulator or min_max or composite or partials" > gpurun_out/tp_tests.log 2>&1
rc=$?
tail -6 gpurun_out/tp_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit $rc; fi
REC=100000000 BENCH_ARGS="--aggs count_star,sum,avg,min,max --h2d-records 0" bash scripts/rehearse_2rank.sh
