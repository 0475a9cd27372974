#!/bin/bash
# formY micro-benchmark + the r06p pass (tests, smoke, bench, stage timing)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06q}
mkdir -p $O
timeout -k 10 60 tools/micro/formy_bench > $O/${T}_formy_micro.json 2>&1 || { echo MICRO FAILED; cat $O/${T}_formy_micro.json; exit 1; }
cat $O/${T}_formy_micro.json
TAG=$T bash tools/gpu_r06p.sh
