# SQ issue / wait counters of the engine kernels (two PMC passes, no trace domains) on a shorter
# bench run, then the per-kernel summary. Usage: [LIB=path] [WL=hop] bash scripts/pmc_sq.sh TAG [RECORDS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sq}; REC=${2:-200000000}
W=${WL:+--workload $WL}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export FLINKGPU_LIB=$LIB
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- \
      python3 $R/bench.py $W --records $REC --steps 1 --warmup 0 --no-cpu-baseline --h2d-records 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 $R/profiles/pmc_summary.py "$OUT/pmc*/*counter_collection.csv" > $OUT/summary.txt && grep -A20 "k_tile_fire\|k_tile_part1" $OUT/summary.txt | head -50
