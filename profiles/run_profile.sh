#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats of the full bench, then separate PMC passes (one TCC group each).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
TAG=${1:-r01}
REC=${2:-1000000000}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$TAG -o run -- \
    python3 $R/bench.py --records $REC --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_trace_$TAG.log 2>&1
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_LDS"; do
  N=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_${N}_$TAG -o run -- \
      python3 $R/bench.py --records 200000000 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/bench_pmc_${N}_$TAG.log 2>&1
done
echo profile-done
