#!/bin/bash
# One gpurun session: GPU parity suite, smoke, bench, rocprof stats of the bench.
# Every GPU step has its own time limit; any rc outside {0,1} ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r1}
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 15 "$OUT/$name.log"
  # rc 1 = test failures / a failed check: keep going; anything else (crash, abort, timeout) ends it
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
}
STEPS=${STEPS:-"gpu smoke bench prof"}
for s in $STEPS; do
  case $s in
    gpu)   step pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/$TAG -o bench \
             -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 ;;
  esac
done
echo ALLOK
