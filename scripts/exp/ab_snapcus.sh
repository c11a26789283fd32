# configs[4] with the snapshot copy's stream CU-masked to N CUs. Usage: bash scripts/exp/ab_snapcus.sh TAG N...
O=gpurun_out/$1; shift; mkdir -p $O
for c in "$@"; do for i in 1 2; do
  FG_SNAP_CUS=$c timeout -k 10 200 python bench.py --workload zipf --no-cpu-baseline --h2d-records 0 > $O/c${c}_$i.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('$O/c${c}_$i.log') if l.startswith('{')][-1]); print('cus $c', round(d['ms_per_step'],2), round(d['job_roofline']['frac'],3), round(d['checkpoints']['avg_ms'],2))"
done; done
echo cus-done
