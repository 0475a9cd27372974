#!/bin/bash
# r06 GPU pass: -m gpu suite, smoke, the wide Dantzig harness on the 512 wide
# problems (for tools/dantzig_reconcile.py classify_wide), bench.
# Usage: TAG=r06a bash tools/gpu_r06.sh [skip-wide]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_gpu_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAIL|Error" $O/${T}_gpu_tests.log | head -20; tail -40 $O/${T}_gpu_tests.log; exit 1; }
tail -1 $O/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
if [ "$1" != "skip-wide" ] && [ -f dbg/lcp_wide.npz ]; then
timeout -k 10 180 python tools/lcp_bench.py run_wide > $O/${T}_lcp_wide.log 2>&1 || { echo WIDE FAILED; tail $O/${T}_lcp_wide.log; exit 1; }
head -3 $O/${T}_lcp_wide.log
LCP_WIDE_PACKED=1 timeout -k 10 180 python tools/lcp_bench.py run_wide > $O/${T}_lcp_wide_packed.log 2>&1 || { echo WIDE FAILED; tail $O/${T}_lcp_wide_packed.log; exit 1; }
head -3 $O/${T}_lcp_wide_packed.log
fi
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo BENCH FAILED; tail -20 $O/${T}_bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/${T}_bench.json'));m=d['atlas_mesh'];r=d['roofline'];print('value',d['value'],d['kernels_ms'],r['frac'],r.get('frac_with_solvers'),'| mesh',m['value'],m['kernels_ms']['forward'],m['kernels_ms']['backward'])"
echo R06 DONE
