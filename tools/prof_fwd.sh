#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench's forward step only (no f32 leg, no training bench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r2_fwd}
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o bench \
  -- python3 bench.py --steps ${BSTEPS:-5} --warmup 2 --cpu-baseline 0 --f32-leg 0 --train-steps 0 \
  > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -1 gpurun_out/prof_bench_$TAG.log | cut -c1-300
exit $rc
