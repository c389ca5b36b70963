#!/bin/bash
# The GPU-box recipes of this repository in one place (run from the repo root,
# e.g. through gpurun; chain several with &&):
#
#   tools/gpu_run.sh tests TAG [pytest args]      the GPU suite            -> gpurun_out/TAG_gpu_tests.log
#   tools/gpu_run.sh smoke TAG                    __graft_entry__.smoke()  -> TAG_smoke.log
#   tools/gpu_run.sh bench TAG [bench args]       bench.py, one line       -> TAG_bench.json / .err
#   tools/gpu_run.sh bench2 TAG [bench args]      bench.py --gpus 2 on this one GPU, no torchrun
#                                                 (gloo collectives)       -> TAG_bench2.json / .err
#   tools/gpu_run.sh ab TAG "LIBS" [ab.py args]   kernel A/B: the product library against
#                                                 kmer-cnt_amd/lib_ab/NAME builds (tools/ab_libs.sh),
#                                                 interleaved, two rounds  -> TAG_ab.log
#   tools/gpu_run.sh abl TAG LIB "VARIANTS" [ab.py args]
#                                                 ablation: time per VAFC_ABLATE variant of one
#                                                 library in one process, then one PMC pass of
#                                                 the same variants        -> TAG_abl_time.log, TAG_abl_pmc/
#   tools/gpu_run.sh prof TAG [CONFIGS]           rocprofv3 kernel trace + stats and the PMC passes
#                                                 of the counting kernel   -> TAG_prof_C/, TAG_pmc_C/
#   tools/gpu_run.sh profbench TAG [bench args]   rocprofv3 --kernel-trace --stats of one whole
#                                                 bench.py command         -> TAG_profbench/
#
# Every GPU step runs under its own time limit; a failing step ends the
# script with a non-zero status (nothing after it runs).
set -o pipefail
STEP=${1:?step}
TAG=${2:?tag}
shift 2
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"
fail() { echo "STEP FAILED ($1): $STEP $TAG"; tail -30 "$2" 2>/dev/null; exit 1; }

case "$STEP" in
tests)
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
    > "$O/${TAG}_gpu_tests.log" 2>&1 || fail $? "$O/${TAG}_gpu_tests.log"
  tail -3 "$O/${TAG}_gpu_tests.log"
  ;;
smoke)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1 ||
    fail $? "$O/${TAG}_smoke.log"
  tail -2 "$O/${TAG}_smoke.log"
  ;;
bench)
  timeout -k 10 900 python bench.py "$@" > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" ||
    fail $? "$O/${TAG}_bench.err"
  cut -c1-600 "$O/${TAG}_bench.json"
  ;;
bench2)
  VAFC_DIST_BACKEND=gloo VAFC_REHEARSAL=1 timeout -k 10 900 python bench.py --gpus 2 "$@" > "$O/${TAG}_bench2.json" \
    2> "$O/${TAG}_bench2.err" || fail $? "$O/${TAG}_bench2.err"
  cut -c1-600 "$O/${TAG}_bench2.json"
  ;;
ab)
  LIBS=${1:?libs}
  shift
  bash tools/r03_ab.sh "$O/${TAG}_ab.log" "$LIBS" "$@" || fail $? "$O/${TAG}_ab.log"
  grep -E "^==|median|identical" "$O/${TAG}_ab.log"
  ;;
abl)
  LIB=${1:?library}
  V=${2:?variants}
  shift 2
  VAFC_LIB=$R/$LIB timeout -k 10 600 python tools/ab.py "$@" $V > "$O/${TAG}_abl_time.log" 2>&1 ||
    fail $? "$O/${TAG}_abl_time.log"
  cat "$O/${TAG}_abl_time.log"
  cd /tmp && export TMPDIR=/tmp
  VAFC_LIB=$R/$LIB timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES -d "$O/${TAG}_abl_pmc" -o p --output-format csv -- \
    python3 "$R/tools/ab.py" --rounds 1 "$@" $V > "$O/${TAG}_abl_pmc.log" 2>&1 || fail $? "$O/${TAG}_abl_pmc.log"
  echo "abl pmc done"
  ;;
prof)
  bash tools/profile_kernels.sh "$TAG" "$@" || fail $? /dev/null
  ;;
profbench)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_profbench" -o p --output-format csv -- \
    python3 "$R/bench.py" "$@" > "$O/${TAG}_profbench.json" 2> "$O/${TAG}_profbench.err" ||
    fail $? "$O/${TAG}_profbench.err"
  cut -c1-400 "$O/${TAG}_profbench.json"
  ;;
*)
  echo "unknown step $STEP"
  exit 2
  ;;
esac
