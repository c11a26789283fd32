# Round 3: XCD-aware pass-2 unit order A/B (FG_P2_XCD=1 default vs 0) + part2 FETCH/WRITE PMC of both
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3x
mkdir -p $O
cd $R
for i in 1 2 3; do
for v in default p2x0; do
  L=flink_amd/libflinkgpu.so; [ $v = default ] || L=flink_amd/libflinkgpu_$v.so
  FLINKGPU_LIB=$R/$L timeout -k 10 120 python -u bench.py --no-cpu-baseline --h2d-records 0 --steps 10 > $O/$v.$i.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.$i.log; exit 1; }
done
done
cd /tmp && export TMPDIR=/tmp
for v in default p2x0; do
  L=flink_amd/libflinkgpu.so; [ $v = default ] || L=flink_amd/libflinkgpu_$v.so
  for P in FETCH_SIZE WRITE_SIZE; do
    FLINKGPU_LIB=$R/$L timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/pmc_${v}_$P -o run -- \
      python3 $R/bench.py --records 200000000 --steps 1 --warmup 0 --no-cpu-baseline --h2d-records 0 > $O/pmc_${v}_$P.log 2>&1 || { echo "pmc $v $P failed"; exit 1; }
  done
done
echo done
