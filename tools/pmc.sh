#!/bin/bash
# HBM traffic of the bench kernels from rocprofv3 PMC counters (one counter group per pass,
# no tracing domains besides kernel dispatch; MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --cpu-baseline 0 --train-steps 0"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 bench.py $ARGS \
    > $OUT/$c.log 2>&1 || { echo "pmc $c failed rc=$?"; tail -5 $OUT/$c.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT
