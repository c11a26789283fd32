# PMC passes of the tile-merge prototype (experiment). Usage: bash scripts/exp/proto_pmc.sh TAG MODE
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $O/pmc$i -o run -- $R/scripts/exp/tile_proto 100000000 10000000 1 $2 > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd $R
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(o + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} mean {sum(v)/len(v):16.1f}  n={len(v)}")
PY
