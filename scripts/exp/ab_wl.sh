# one bench line per workload (3 steps). Usage: bash scripts/exp/ab_wl.sh TAG WL...
O=gpurun_out/$1; shift; mkdir -p $O
for W in "$@"; do
  timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --h2d-records 0 --steps 3 --warmup 1 > $O/$W.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$O/$W.log') if l.startswith('{')][-1]); print('$W', round(d['ms_per_step'],2), d['roofline']['kernel'], round(d['roofline']['avg_launch_ms'],4), {n:(x['launches'],round(x['avg_ms'],3)) for n,x in d['kernels_warmup'].items() if x['launches']})"
done
echo wl-done
