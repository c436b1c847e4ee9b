#!/bin/bash
# Round-3 validation session: the new kernels' tests first (attention LDS-DMA ring, dW), the
# attention A/B timing, then the whole GPU suite, smoke and the bench.  Each GPU step has its own
# time limit; a crash/abort/timeout (rc not in {0,1}) ends the session.
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
  tail -n ${TAILN:-15} "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v -rf --timeout 150 --timeout-method thread"
for s in ${STEPS:-new ab gpu smoke bench}; do
  case $s in
    new)   step pytest_new 300 $PT tests/test_gpu_kernels.py tests/test_gpu_train.py -k "attention or linear_dw or hip_linear" ;;
    ab)    step attn_dma 120 env REPS=6 python tools/attn_only.py
           step attn_dma_unscaled 120 env REPS=6 PRESCALED=0 python tools/attn_only.py ;;
    gpu)   step pytest_gpu 900 $PT tests -m gpu ${PYTEST_ARGS:-} ;;
    sel)   step pytest_sel 600 $PT tests -m gpu -k "${PYTEST_K}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps ${BSTEPS:-5} --warmup 2 ${BENCH_ARGS:-} ;;
    pmc)   step attn_pmc 300 env TAG=${ATAG:-attn} bash tools/pmc_attn.sh ;;
    knn)   step knn_probe 300 python tools/knn_probe.py ;;
    tail)  step tail_micro 300 python tools/tail_micro.py ;;
    proj)  step proj_micro 300 python tools/proj_micro.py ;;
    tattn) step train_attn_micro 300 python tools/train_attn_micro.py ;;
    exp)   step exp_rate 120 ./tools/micro/exp_rate ;;
    train) step train_only 300 python tools/train_only.py
           step train_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_train -o run -- python3 tools/train_only.py
           rm -f $OUT/prof_train/*/*.db $OUT/prof_train/*.db
           python3 tools/prof_top.py $OUT/prof_train 40 ;;
  esac
done
