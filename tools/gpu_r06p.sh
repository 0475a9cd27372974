#!/bin/bash
# GPU suite + smoke + bench + stage timing (forward and backward) of HEAD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-mesh > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));r=d['roofline'];print('value',d['value'],d['kernels_ms'],r['frac'])"
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/${T}_forward_world_latency_hist.json timeout -k 10 200 python tools/stage_timing.py > $O/${T}_stage_timing.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing.log; exit 1; }
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 200 python tools/stage_timing_bwd.py > $O/${T}_backward_stage_timing.log 2>&1 || { echo STAGE BWD FAILED; tail -5 $O/${T}_backward_stage_timing.log; exit 1; }
echo R06P DONE
