# configs[4]: async vs sync snapshot, hot pre-combine on/off. Usage: bash scripts/exp/ab_zipf4.sh TAG
O=gpurun_out/$1; mkdir -p $O
run() {   # name, env, args
  env $2 timeout -k 10 200 python bench.py --workload zipf --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 $3 > $O/$1.log 2>&1 || return 1
  python -c "import json; d=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][-1]); print('$1', round(d['ms_per_step'],2), d['checkpoints'], {n:(x['launches'],round(x['avg_ms'],3)) for n,x in d['kernels'].items() if x['launches']})"
}
run async "" "" && run sync "" "--sync-snapshot" && run async_nohot "FG_TILE_HOT=0" "" && run sync_nohot "FG_TILE_HOT=0" "--sync-snapshot" && echo ab-done
