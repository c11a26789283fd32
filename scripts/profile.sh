# Profile recipe (GPU box, repo root). Usage: [WL=hop] bash scripts/profile.sh TAG [PMC_RECORDS]
#  1. kernel trace + stats of the default bench command (1B records, 3 steps, no CPU leg)
#  2. PMC passes, one counter group per run (no trace domains), on a shorter bench run:
#     FETCH_SIZE / WRITE_SIZE (HBM traffic) and SQ occupancy / LDS / wait counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
REC=${2:-200000000}
W=${WL:+--workload $WL}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py $W --no-cpu-baseline --h2d-records 0 > $OUT/bench_trace.log 2>&1 || { echo trace failed; exit 1; }
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- \
      python3 $R/bench.py $W --records $REC --steps 1 --warmup 0 --no-cpu-baseline --h2d-records 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo profile-done
