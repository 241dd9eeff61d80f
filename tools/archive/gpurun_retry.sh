#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool has no free slot / box (status "transient":
# nothing ran, nothing was charged).  A call that ran (pass or fail) is never repeated.
# usage: bash tools/archive/gpurun_retry.sh <timeout_s> <max_tries> '<command>'
TO=$1; TRIES=$2; CMD=$3
for i in $(seq 1 "$TRIES"); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[try $i] no slot/box; waiting"
    sleep 150
    continue
  fi
  echo "$out" | tail -60
  exit $rc
done
echo "gave up after $TRIES tries"
exit 3
