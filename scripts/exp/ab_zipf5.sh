# configs[4] micro-batch size; HOP with the narrow policy. Usage: bash scripts/exp/ab_zipf5.sh TAG
O=gpurun_out/$1; mkdir -p $O
run() {   # name, workload, args
  timeout -k 10 200 python bench.py --workload $2 --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 $3 > $O/$1.log 2>&1 || return 1
  python -c "import json; d=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][-1]); print('$1', round(d['ms_per_step'],2), d['checkpoints'], {n:(x['launches'],round(x['avg_ms'],3)) for n,x in d['kernels'].items() if x['launches']})"
}
run zipf50m zipf "" && run zipf100m zipf "--batch 100000000" && run zipf25m zipf "--batch 25000000" && run hop hop "" && echo ab-done
