#!/bin/bash
# usage: tools/gpucall.sh NAME TIMEOUT 'command'  — one gpurun call in the background-friendly form;
# the gpurun verdict goes to gpurun_out/NAME.call
name=$1; t=$2; shift 2
timeout $((t + 900)) /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "gpurun_out/$name.call" 2>&1
echo "rc=$?" >> "gpurun_out/$name.call"
