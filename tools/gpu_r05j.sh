# r05j: maskless triangular solves (zeros stored right of the diagonal, the
# packed factor padded per 8-row block) -- the step micro-benchmark, the -m gpu
# suite, the bench of both Atlas workloads, the mesh stage timing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05j}
mkdir -p $O
timeout -k 10 60 tools/micro/tri_bench > $O/${T}_tri_bench.log 2>&1 || { echo TRI FAILED; cat $O/${T}_tri_bench.log; exit 1; }
cat $O/${T}_tri_bench.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];r=d['roofline'];print('value',d['value'],d['kernels_ms'],r['frac'],r.get('frac_with_solvers'),'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'])"
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 300 python tools/stage_timing.py > $O/${T}_stage_timing_atlas_mesh.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing_atlas_mesh.log; exit 1; }
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/${T}_forward_world_latency_hist.json timeout -k 10 120 python tools/stage_timing.py > $O/${T}_stage_timing.log 2>&1 || { echo STAGE2 FAILED; tail -5 $O/${T}_stage_timing.log; exit 1; }
echo R05J DONE
