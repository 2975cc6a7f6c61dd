#!/bin/bash
# Submit one gpurun call; resubmit ONLY while the pool reports no free slot/box (nothing ran,
# nothing charged: exit code 3 or a "busy ... nothing was charged" message).  A call that ran
# (any outcome, including a failed or timed-out GPU step) is never resubmitted.
# usage: tools/gpurun_retry.sh <log> <timeout_s> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  cat "$log" >> "$log.all"
  if [ $rc -eq 3 ] || { { grep -q "nothing was charged" "$log" && grep -q -i "busy\|no box\|no free" "$log"; } || grep -q "status=transient rc=None charged=0.0s\|status=transient rc=None charged=Nones" "$log"; }; then
    # honour the pool's own back-off hint ("retry in Ns") when it gives one
    hint=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    echo "[retry $i] no slot (rc=$rc), waiting ${hint:-90}s" >> "$log.retries"
    sleep $(( ${hint:-85} + 5 ))
    continue
  fi
  exit $rc
done
exit 3
