#!/bin/bash
# two-wave backward: GPU suite, smoke, bench A/B (NIMBLE_AMD_BWD_SPLIT=1/0/1) on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06r}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
for v in 1 0 1; do
NIMBLE_AMD_BWD_SPLIT=$v timeout -k 10 400 python bench.py --no-cpu-baseline > $O/${T}_bench_split$v.json 2> $O/${T}_bench_split$v.err || { echo BENCH FAILED; tail -20 $O/${T}_bench_split$v.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench_split$v.json'));m=d['atlas_mesh'];print('split $v value',d['value'],d['kernels_ms'],'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'])"
done
echo R06R DONE
