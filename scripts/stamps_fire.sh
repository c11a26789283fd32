# Phase cycles of k_tile_fire (FG_STAMPS build, `make -C flink_amd stamps`) for the headline and
# the table / split fires. Usage: bash scripts/stamps_fire.sh TAG
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for W in ${WLS:-tumble hop cumulate zipf}; do
  FG_STAMPS=1 FLINKGPU_LIB=$PWD/flink_amd/libflinkgpu_stamps.so timeout -k 10 200 python bench.py --workload $W \
      --no-cpu-baseline --h2d-records 0 --steps 1 --warmup 0 --records 300000000 > $O/stamps_$W.log 2>&1 \
      || { echo "stamps $W failed"; tail -5 $O/stamps_$W.log; exit 1; }
  echo "== $W"; grep "fg stamps\] tile_fire" $O/stamps_$W.log | sort | uniq -c | sort -rn | head -6
done
