# Zipf (configs[4]) bench A/B: region bits via --expected-keys, split chunk size. Usage: bash scripts/exp/ab_zipf.sh TAG
O=gpurun_out/$1; mkdir -p $O
run() {   # name, env, extra args
  env $2 timeout -k 10 200 python bench.py --workload zipf --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 $3 > $O/$1.log 2>&1 || return 1
  python -c "import json; d=json.loads([l for l in open('$O/$1.log') if l.startswith('{')][-1]); print('$1', round(d['ms_per_step'],2))"
}
run default "" "" && run ek5m "" "--expected-keys 5000000" && run chunk32k "FG_TILE_CHUNK=32768" "" && run chunk16k "FG_TILE_CHUNK=16384" "" && echo ab-done
