#!/bin/bash
# GPU-box: a focused pytest selection first (one process), then the full suite.
# Usage: bash tools/gpu_focus.sh <tag> "<pytest -k expr>"
set -o pipefail
TAG=${1:-focus}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread -k "$2" > gpurun_out/gpu_focus_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gpu_focus_$TAG.log | tail -30
exit $rc
