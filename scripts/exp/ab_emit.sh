# merge-path parity subset, then A/B (base vs variants) on the default bench and hop / cumulate
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "golden or stream_parity or multi_accumulator or restore or regions or config" > gpurun_out/ab_tests.log 2>&1
rc=$?
tail -4 gpurun_out/ab_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit $rc; fi
bash scripts/exp/variants.sh base "$@" base "$@" && bash scripts/exp/wl_variants.sh base "$@"
