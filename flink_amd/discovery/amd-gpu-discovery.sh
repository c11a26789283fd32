#!/usr/bin/env bash
# amd-gpu-discovery.sh gpu-amount [--enable-coordination-mode] [--coordination-file path]
#
# Prints a comma-separated list of `gpu-amount` AMD GPU indices for one TaskManager: the
# MI355X counterpart of flink-external-resource-gpu's discovery script, called by its
# GPUDriver (flink-external-resources/flink-external-resource-gpu/.../GPUDriver.java) with the
# same arguments and the same output contract (exit 1 when fewer GPUs than requested).
# Indices come from `rocm-smi --showid --csv` ("cardN" rows; $ROCM_SMI overrides the tool),
# mapped to HIP device ordinals by PCI bus id (`rocm-smi --showbus --csv` against
# hip-pci-bus-ids, i.e. hipDeviceGetPCIBusId).
# Coordination mode: TaskManagers on one host claim disjoint indices through a shared file
# ("index pid" lines, guarded by flock); claims of processes that no longer exist are
# released first.
set -u
if [ $# -lt 1 ]; then
  echo "Usage: ./amd-gpu-discovery.sh gpu-amount [--enable-coordination-mode] [--coordination-file filePath]"
  exit 1
fi
AMOUNT=$1
shift
COORD=0
COORD_FILE=/var/tmp/flink-amd-gpu-coordination
while [ $# -ge 1 ]; do
  case "$1" in
    --enable-coordination-mode) COORD=1 ;;
    --coordination-file) shift; COORD_FILE=${1:-$COORD_FILE} ;;
  esac
  shift
done
[ "$AMOUNT" -eq 0 ] && exit 0

SMI=${ROCM_SMI:-rocm-smi}
out=$("$SMI" --showid --csv 2>/dev/null) || exit 1
indexes=$(printf '%s\n' "$out" | sed -n 's/^card\([0-9][0-9]*\),.*/\1/p' | sort -n | uniq)
[ -z "$indexes" ] && exit 1

# rocm-smi numbers the host's cards; HIP the devices this process sees, in its own order. With
# hip-pci-bus-ids (built next to this script; $HIP_BUS_IDS overrides it) every card is mapped to
# the HIP ordinal of the same PCI bus id, and cards HIP does not see are left out; without it
# the card indices are used as they are.
BUSIDS=${HIP_BUS_IDS:-$(dirname "$0")/hip-pci-bus-ids}
if [ -x "$BUSIDS" ] && hip=$("$BUSIDS" 2>/dev/null) && [ -n "$hip" ] && \
   bus=$("$SMI" --showbus --csv 2>/dev/null); then
  indexes=$(printf '%s\n' "$bus" | sed -n 's/^card\([0-9][0-9]*\),\(.*\)$/\1 \2/p' | sort -n | \
    while read -r card id; do
      id=$(printf '%s' "$id" | tr 'A-F' 'a-f' | tr -d ' ')
      printf '%s\n' "$hip" | awk -v b="$id" '$2 == b { print $1 }'
    done)
  [ -z "$indexes" ] && exit 1
else
  echo "amd-gpu-discovery: no HIP bus-id map ($BUSIDS); card indices taken as HIP ordinals" >&2
fi

pick() {   # first $2 entries of list $1 (newline separated) that are not in list $3
  printf '%s\n' "$1" | while read -r i; do
    [ -z "$i" ] && continue
    printf '%s\n' "$3" | grep -qx "$i" || echo "$i"
  done | head -n "$2"
}

if [ "$COORD" -eq 0 ]; then
  chosen=$(printf '%s\n' "$indexes" | head -n "$AMOUNT")
else
  owner=${FLINK_TM_PID:-$PPID}
  touch "$COORD_FILE" || exit 1
  exec 9<>"$COORD_FILE.lock" || exit 1
  flock 9
  live=""
  while read -r idx pid; do
    [ -z "${idx:-}" ] && continue
    if kill -0 "$pid" 2>/dev/null; then live="$live$idx $pid"$'\n'; fi
  done < "$COORD_FILE"
  taken=$(printf '%s' "$live" | awk '{print $1}')
  chosen=$(pick "$indexes" "$AMOUNT" "$taken")
  n=$(printf '%s\n' "$chosen" | grep -c .)
  if [ "$n" -lt "$AMOUNT" ]; then flock -u 9; exit 1; fi
  { printf '%s' "$live"; printf '%s\n' "$chosen" | sed "s/\$/ $owner/"; } > "$COORD_FILE"
  flock -u 9
fi
n=$(printf '%s\n' "$chosen" | grep -c .)
[ "$n" -lt "$AMOUNT" ] && exit 1
printf '%s\n' "$chosen" | paste -sd, -
