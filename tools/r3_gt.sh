# Round 3: GPU tests (selection in $SEL, default all) with per-test timeouts
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-900} python -u -m pytest tests -m gpu -x -v --timeout ${TT:-300} --timeout-method thread ${SEL:+-k "$SEL"} > gpurun_out/${OUT:-r3_gt}.log 2>&1
