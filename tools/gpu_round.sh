#!/bin/bash
# One gpurun session: build, GPU parity tests, smoke, bench.  Each GPU step has its own
# time limit; a crash/abort/timeout (rc not in {0,1}) ends the session immediately.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
make -C rag-snvbert_amd -j16 > $OUT/make.log 2>&1 || { tail $OUT/make.log; exit 3; }
STEPS=${STEPS:-"kernels model smoke bench"}
for s in $STEPS; do
  case $s in
    kernels) step pytest_kernels 900 python -m pytest tests/test_gpu_kernels.py -q -rf --timeout 300 ;;
    model)   step pytest_model 900 python -m pytest tests/test_gpu_model.py -q -rf --timeout 300 ;;
    gpu)     step pytest_gpu 1200 python -u -m pytest tests -m gpu -v -rf --timeout 150 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke)   step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   step bench 900 python bench.py --steps ${BSTEPS:-5} --warmup 2 ${BENCH_ARGS:-} ;;
    benchab) step bench_old 900 env SNVRAG_GEMM_TILE128=1 SNVRAG_UNFUSED_LN=1 python bench.py --steps ${BSTEPS:-5} --warmup 2 --cpu-baseline 0
             step bench_tile128_fusedoff 900 env SNVRAG_UNFUSED_LN=1 python bench.py --steps ${BSTEPS:-5} --warmup 2 --cpu-baseline 0 ;;
    shallow) step bench_shallow 900 env SNVRAG_GEMM_SHALLOW=1 python bench.py --steps ${BSTEPS:-5} --warmup 2 --cpu-baseline 0 ;;
  esac
done
