#!/bin/bash
# Round-3 kernel probes in one gpurun session: kNN scan split (tools/knn_probe.py), attention
# timing + SQ counters (tools/attn_only.py, tools/pmc_attn.sh), block tail variants
# (tools/tail_micro.py).  Every GPU step has its own time limit; a crash/abort/timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 40 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${PROBES:-knn attn tail}; do
  case $s in
    knn)  step knn_probe 300 python tools/knn_probe.py ;;
    attn) step attn_time 120 env REPS=6 python tools/attn_only.py
          step attn_pmc 300 env TAG=${ATAG:-attn} bash tools/pmc_attn.sh ;;
    tail) step tail_micro 300 python tools/tail_micro.py ;;
  esac
done
