#!/bin/bash
# r04: the -m gpu suite (optionally -k), the Dantzig micro for
# tools/dantzig_reconcile.py, a short bench (headline + mesh), mesh stage timing.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
TAG=${TAG:-r04b}
mkdir -p $O
KA=()
[ -n "$1" ] && KA=(-k "$1")
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "${KA[@]}" > $O/gpu_tests_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|FAILED" $O/gpu_tests_$TAG.log | tail -6
[ $rc -ne 0 ] && exit $rc
if [ -f tests/cpp/liblcp_bench.so ] && [ -z "$NO_MICRO" ]; then
  timeout -k 10 120 python tools/lcp_bench.py run > $O/lcp_micro_$TAG.log 2>&1 || { echo MICRO FAILED; tail $O/lcp_micro_$TAG.log; exit 1; }
  head -1 $O/lcp_micro_$TAG.log
  grep "n=24" -A1 $O/lcp_micro_$TAG.log
  timeout -k 10 120 python tools/lcp_bench.py run_wide > $O/lcp_wide_$TAG.log 2>&1 || { echo WIDE MICRO FAILED; tail $O/lcp_wide_$TAG.log; exit 1; }
  grep -v amdgpu $O/lcp_wide_$TAG.log | head -3
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo BENCH FAILED; tail -20 $O/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_$TAG.json'));m=d['atlas_mesh'];print('value',d['value'],'fwd',d['kernels_ms']['forward'],'bwd',d['kernels_ms']['backward'],'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'])"
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/stage_hist_mesh_$TAG.json timeout -k 10 200 python tools/stage_timing.py > $O/stage_mesh_$TAG.log 2>&1 || { echo MESH STAGE FAILED; tail -20 $O/stage_mesh_$TAG.log; exit 1; }
tail -1 $O/stage_mesh_$TAG.log
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so BUCKETS_OUT=mesh_buckets_$TAG.json timeout -k 10 200 python tools/mesh_buckets.py > $O/mesh_buckets_$TAG.log 2>&1 || { echo BUCKETS FAILED; tail -20 $O/mesh_buckets_$TAG.log; exit 1; }
grep -v amdgpu.ids $O/mesh_buckets_$TAG.log | sed -n '/step 1/,/step 2/p' | cut -c1-200
