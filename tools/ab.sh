#!/bin/bash
# A/B timing of library builds and environment settings on one GPU box (kbench on the bench
# corpus). Every combination of VARIANT x ENV runs twice: whole-call wall time on the default
# two streams, then per-phase HIP-event times on one stream (ACOSS_SPLIT_STREAMS=1), whose
# kernel times add up to the call.
#
#   bash tools/ab.sh [-p PAIRS] [-f FRAMES] [-r REPS] [-c CORPUS] [-x "kbench args"] \
#                    [-e "VAR=val ..."]... [-t] VARIANT...
#
# VARIANT: "base" (acoss-1_amd/acoss/lib/libacoss_hip.so) or a name built by
#          `bash tools/abbuild.sh NAME -DFOO...` (tools/abl/libabl_NAME.so).
# -e:      an environment spec; repeat for several (default: none).
# -t:      run tests/test_gpu_crp.py against each non-base variant first (stops on failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PAIRS=13366; FRAMES=2000; REPS=3; CORPUS=hard; EXTRA=""; TESTS=0
ENVS=()
while getopts "p:f:r:c:x:e:t" o; do
  case $o in
    p) PAIRS=$OPTARG ;; f) FRAMES=$OPTARG ;; r) REPS=$OPTARG ;; c) CORPUS=$OPTARG ;;
    x) EXTRA=$OPTARG ;; e) ENVS+=("$OPTARG") ;; t) TESTS=1 ;; *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ ${#ENVS[@]} -eq 0 ] && ENVS=("ACOSS_AB=1")
mkdir -p gpurun_out
KB="python tools/kbench.py --pairs $PAIRS --frames $FRAMES --reps $REPS --corpus $CORPUS $EXTRA"
last=$((REPS - 1))
for v in "$@"; do
  if [ "$v" = base ]; then L=acoss-1_amd/acoss/lib/libacoss_hip.so; else L=tools/abl/libabl_$v.so; fi
  if [ $TESTS = 1 ] && [ "$v" != base ]; then
    ACOSS_HIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_crp.py -x -q --timeout 120 \
      --timeout-method thread > gpurun_out/ab_tests_$v.log 2>&1 || { echo "tests failed: $v"; tail -30 gpurun_out/ab_tests_$v.log; exit 1; }
    echo "tests $v: $(tail -1 gpurun_out/ab_tests_$v.log)"
  fi
  for e in "${ENVS[@]}"; do
    echo "variant=$v env=[$e]"
    env $e ACOSS_HIP_LIB=$PWD/$L timeout -k 10 180 $KB --noprof > gpurun_out/ab_run.log 2>&1 || { tail -5 gpurun_out/ab_run.log; exit 1; }
    grep -E "rep $last|checksum" gpurun_out/ab_run.log
    env $e ACOSS_SPLIT_STREAMS=1 ACOSS_HIP_LIB=$PWD/$L timeout -k 10 180 $KB > gpurun_out/ab_run.log 2>&1 || { tail -5 gpurun_out/ab_run.log; exit 1; }
    grep -E "rep $last" gpurun_out/ab_run.log
  done
done
