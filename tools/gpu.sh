#!/bin/bash
# Run one command on the GPU box via gpurun; clears the named output files first,
# retries ONLY when gpurun reports an infrastructure-transient status (nothing ran).
# usage: tools/gpu.sh TIMEOUT "command" [files to clear...]
T=$1; CMD=$2; shift 2
for f in "$@"; do rm -f "/root/repo/gpurun_out/$f"; done
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > /root/repo/gpurun_out/call.log 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|busy" /root/repo/gpurun_out/call.log; then
    echo "[gpu.sh] transient (attempt $attempt), waiting"; sleep 90; continue
  fi
  break
done
tail -2 /root/repo/gpurun_out/call.log
exit $rc
