# configs[4] cost split: Zipf vs jitter vs the checkpoint. Usage: bash scripts/exp/ab_zipf2.sh TAG
O=gpurun_out/$1; mkdir -p $O
run() {   # name, args
  timeout -k 10 200 python bench.py --workload zipf --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 $2 > $O/$1.log 2>&1 || return 1
  python -c "import json; d=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][-1]); print('$1', round(d['ms_per_step'],2), {n:(x['launches'],round(x['avg_ms'],3)) for n,x in d['kernels'].items() if x['launches']})"
}
run default "" && run nockpt "--checkpoint-every 0" && run uniform_jit "--zipf 0" && run zipf_nojit "--jitter 0" && run uniform_nojit "--zipf 0 --jitter 0 --checkpoint-every 0" && echo ab-done
