#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (separate from PMC passes, per the pool rules)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
make -C rag-snvbert_amd -j16 > gpurun_out/make.log 2>&1 || exit 3
TAG=${TAG:-r1}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$TAG -o bench \
  -- python3 bench.py --steps ${BSTEPS:-5} --warmup 2 --cpu-baseline 0 > gpurun_out/prof_bench_$TAG.log 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench_$TAG.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
