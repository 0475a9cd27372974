# r05c: full -m gpu suite at the tree (FD bit-exact, packed Dantzig L, MFMA
# pinv), then the mesh Atlas bench with / without the MFMA pinv and the
# stage timing of the mesh world
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05c}
NIMBLE_AMD_VERBOSE=1 timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.')
from nimblephysics_amd import workloads
w = workloads.atlas_mesh_world(True); w.native()" > $O/${T}_layout.log 2>&1
cat $O/${T}_layout.log | grep nimble_amd
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error|assert" $O/${T}_gpu_tests.log | head -20; tail -30 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
for v in 1 0; do
NIMBLE_AMD_PINV_MFMA=$v timeout -k 10 200 python bench.py --workload atlas_mesh --steps 20 --warmup 3 --no-cpu-baseline > $O/${T}_bench_mesh_pinv$v.json 2> $O/${T}_bench_mesh_pinv$v.err || { echo MESH BENCH FAILED; tail -5 $O/${T}_bench_mesh_pinv$v.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_mesh_pinv$v.json'));print('pinv',$v,d['value'],d['kernels_ms'])"
done
STAGE_WORKLOAD=atlas_mesh NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 300 python tools/stage_timing.py > $O/${T}_stage_timing_atlas_mesh.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing_atlas_mesh.log; exit 1; }
echo R05C DONE
