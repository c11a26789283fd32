# merge-path parity subset (incl. Zipf and MIN/MAX), then A/B: default bench and zipf, base vs wp0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "golden or stream_parity or multi_accumulator or min_max or config or two_phase" > gpurun_out/ab_tests.log 2>&1
rc=$?
tail -4 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit $rc; fi
bash scripts/exp/variants.sh base wp0 base wp0 && BENCH_ARGS="--workload zipf" bash scripts/exp/variants.sh base wp0
