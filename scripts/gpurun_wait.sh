# Run one gpurun call, waiting for a box: retried only while gpurun reports exit code 3 (no box or
# slot free; nothing ran, nothing charged), at most 6 attempts 3 minutes apart. Any other exit
# code -- the command's own failure included -- ends it. Usage: bash scripts/gpurun_wait.sh TIMEOUT 'COMMAND'
T=$1; shift
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$1"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no box (attempt $i), waiting 180 s"
  sleep 180
done
exit 3
