#!/bin/bash
# Run one command on the GPU box via gpurun; retries ONLY when gpurun reports an
# infrastructure-transient status (nothing ran, nothing charged): no box free, back-off.
# usage: tools/gpu.sh TIMEOUT "command" [max attempts]
T=$1; CMD=$2; MAXA=${3:-30}
for attempt in $(seq 1 $MAXA); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > /root/repo/gpurun_out/call.log 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|no free box\|busy" /root/repo/gpurun_out/call.log; then
    w=$(grep -o "retry in [0-9]*s" /root/repo/gpurun_out/call.log | grep -o "[0-9]*" | head -1); w=${w:-120}
    [ "$w" -lt 60 ] && w=60
    echo "[gpu.sh] transient (attempt $attempt), waiting ${w}s"; sleep $w; continue
  fi
  break
done
tail -2 /root/repo/gpurun_out/call.log
exit $rc
