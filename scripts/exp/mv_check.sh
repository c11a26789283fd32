# MIN/MAX + multi-value parity subset, then the bench with COUNT(*),SUM,AVG,MIN,MAX and the default list
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "min_max or multi_accumulator or composite or golden" > gpurun_out/mv_tests.log 2>&1
rc=$?
tail -5 gpurun_out/mv_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit $rc; fi
BENCH_ARGS="--aggs count_star,sum,avg,min,max" bash scripts/exp/variants.sh base && mv gpurun_out/variants/base.json gpurun_out/variants/mv5.json
BENCH_ARGS="--aggs count_star,min" bash scripts/exp/variants.sh base && mv gpurun_out/variants/base.json gpurun_out/variants/min.json
bash scripts/exp/variants.sh base
