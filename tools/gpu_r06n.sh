#!/bin/bash
# r06 early-rows pass: -m gpu suite, smoke, bench with the helper's early
# rows on (default) and off (NIMBLE_AMD_EARLY_ROWS=0), same box.
# Usage: TAG=r06n bash tools/gpu_r06n.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06n}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
for v in 1 0 1; do
NIMBLE_AMD_EARLY_ROWS=$v timeout -k 10 400 python bench.py --no-cpu-baseline --no-mesh > $O/${T}_bench_early$v.json 2> $O/${T}_bench_early$v.err || { echo BENCH FAILED; tail -20 $O/${T}_bench_early$v.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_early$v.json'));r=d['roofline'];print('early $v value',d['value'],d['kernels_ms'],r['frac'])"
done
echo R06N DONE
