#!/bin/bash
# usage: tools/gpucall_wait.sh NAME TIMEOUT 'command' — like gpucall.sh, but while the pod has no free
# GPU slot (gpurun exit 3: nothing ran, nothing charged) waits 2 minutes and asks again (at most
# 15 times).  Any other outcome — success, a test failure, a fault, a timeout — ends it at once.
name=$1; t=$2; shift 2
for i in $(seq 1 15); do
  timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "gpurun_out/$name.call" 2>&1
  rc=$?
  echo "rc=$rc attempt=$i" >> "gpurun_out/$name.call"
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
