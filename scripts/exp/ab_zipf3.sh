# the split fire's per-record cost vs skew. Usage: bash scripts/exp/ab_zipf3.sh TAG
O=gpurun_out/$1; mkdir -p $O
run() {   # name, env, args
  env $2 timeout -k 10 200 python bench.py --workload zipf --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 --jitter 0 --checkpoint-every 0 $3 > $O/$1.log 2>&1 || return 1
  python -c "import json; d=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][-1]); print('$1', round(d['ms_per_step'],2), {n:(x['launches'],round(x['avg_ms'],3)) for n,x in d['kernels'].items() if x['launches']})"
}
run z11 "" "" && run z11_nohot "FG_TILE_HOT=0" "" && run z09 "" "--zipf 0.9" && run z07 "" "--zipf 0.7" && run z11_nosplit "FG_TILE_SPLIT=0" "" && echo ab-done
