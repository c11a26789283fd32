#!/bin/bash
# PMC passes (one counter group per run, no trace domains) over a short bench run.
# usage: profiles/run_pmc.sh TAG RECORDS "group1" "group2" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
TAG=$1; REC=$2; shift 2
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_${TAG}_$i -o run -- \
      python3 $R/bench.py --records $REC --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc-done
