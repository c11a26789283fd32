# tile-merge prototype variants x modes (experiment). Usage: bash scripts/exp/proto_run.sh TAG
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for b in scripts/exp/tile_proto_*; do
  for m in 0 1 2 3; do
    echo "== $b mode $m"
    timeout -k 5 60 ./$b 100000000 10000000 5 $m | tail -5 || exit 1
  done
done > $O/run.log 2>&1
cat $O/run.log
