# PMC traffic (FETCH_SIZE, WRITE_SIZE passes) of the headline for the current library build ->
# gpurun_out/prof_<tag>/pmc_traffic.json keyed by the library's sha256. Usage: bash scripts/pmc_traffic_only.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o run -- \
      python3 $R/bench.py --records 200000000 --steps 1 --warmup 0 --no-cpu-baseline --h2d-records 0 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd $R
python3 profiles/pmc_summary.py "gpurun_out/prof_$1/pmc*/run_counter_collection.csv" gpurun_out/prof_$1/pmc_traffic.json flink_amd/libflinkgpu.so > gpurun_out/prof_$1/pmc_summary.txt
