#!/bin/bash
# Submit one gpurun call, resubmitting it only while the pool has no box for
# it (status=transient with nothing run or charged: "no free box", "backing
# off", a box lost while being prepared). A call that ran is never repeated.
# Usage: tools/gpurun_wait.sh LOG TIMEOUT 'COMMAND'
LOG=$1; T=$2; CMD=$3
for try in $(seq 1 ${GPURUN_TRIES:-20}); do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && grep -Eq "run (0.0|None)s of limit" "$LOG"; then
    wait_s=$(grep -oE "retry in [0-9]+s" "$LOG" | grep -oE "[0-9]+" | head -1)
    sleep $(( ${wait_s:-120} + 15 ))
    continue
  fi
  exit $rc
done
exit 3
