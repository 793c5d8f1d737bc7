#!/bin/bash
# Submit one gpurun call, waiting for a box: resubmits only while gpurun reports that the command
# did not start (exit 3 / status=transient: no box, or the box failed before the command ran),
# after the back-off gpurun asks for.  A command that ran -- whatever its result -- is never
# resubmitted.
#   tools/gpurun_wait.sh <out-file> <timeout-s> '<command>'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 60); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient rc=None" "$OUT"; then exit $rc; fi
  w=$(grep -o "retry in [0-9]*s" "$OUT" | tail -1 | grep -o "[0-9]*")
  sleep $(( ${w:-180} + 15 ))
done
exit 3
