# configs[4] repeatability: N runs of the zipf bench line. Usage: bash scripts/exp/ab_zipf6.sh TAG N
O=gpurun_out/$1; mkdir -p $O
for i in $(seq 1 $2); do
  timeout -k 10 200 python bench.py --workload zipf --no-cpu-baseline --h2d-records 0 > $O/z$i.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$O/z$i.log') if l.startswith('{')][-1]); print('zipf', round(d['ms_per_step'],2), round(d['job_roofline']['frac'],3), d['checkpoints'])"
done
echo z-done
