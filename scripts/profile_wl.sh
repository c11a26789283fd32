# Trace + PMC of several workloads in one GPU call. Usage: bash scripts/profile_wl.sh TAG WL [WL...]
set -o pipefail
TAG=$1; shift
for W in "$@"; do
  WL=$W timeout -k 10 500 bash scripts/profile.sh ${TAG}_$W 200000000 || { echo "profile $W failed"; exit 1; }
done
echo all-done
