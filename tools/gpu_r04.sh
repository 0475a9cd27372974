#!/bin/bash
# GPU-box iteration: the -m gpu suite (optionally -k), a short bench (headline +
# the STL-mesh Atlas object), stage timing of both Atlas models (debug build).
# Usage: bash tools/gpu_r04.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-it}
K=${2:-}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
if [ "$K" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread "${KA[@]}" > $O/gpu_tests_$TAG.log 2>&1
  rc=$?
  grep -E "passed|failed" $O/gpu_tests_$TAG.log | tail -2
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/gpu_tests_$TAG.log | head -20; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCH FAILED; tail -20 $O/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_$TAG.json'));m=d['atlas_mesh'];print('value',d['value'],'fwd',d['kernels_ms']['forward'],'bwd',d['kernels_ms']['backward'],'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'])"
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/stage_hist_$TAG.json timeout -k 10 120 python tools/stage_timing.py > $O/stage_$TAG.log 2>&1 || { echo STAGE FAILED; tail -20 $O/stage_$TAG.log; exit 1; }
tail -1 $O/stage_$TAG.log
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/stage_hist_mesh_$TAG.json timeout -k 10 200 python tools/stage_timing.py > $O/stage_mesh_$TAG.log 2>&1 || { echo MESH STAGE FAILED; tail -20 $O/stage_mesh_$TAG.log; exit 1; }
tail -1 $O/stage_mesh_$TAG.log
