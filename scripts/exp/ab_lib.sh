# A/B of two library builds on workloads. Usage: bash scripts/exp/ab_lib.sh TAG LIB_B WL...
O=gpurun_out/$1; LB=$2; shift 2; mkdir -p $O
for W in "$@"; do for r in 1 2; do for v in a b; do
  if [ $v = a ]; then L=$PWD/flink_amd/libflinkgpu.so; else L=$PWD/$LB; fi
  FLINKGPU_LIB=$L timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --h2d-records 0 > $O/${W}_${v}$r.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$O/${W}_${v}$r.log') if l.startswith('{')][-1]); print('$W $v', round(d['ms_per_step'],2))"
done; done; done
echo ab-done
