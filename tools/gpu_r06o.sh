#!/bin/bash
# stage timing (forward histogram + per-stage split, backward per-stage split)
# of the current build: dbg/libnimble_dbg.so (-DNIMBLE_STAGE_TIMING)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r06o}
mkdir -p $O
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so STAGE_HIST_OUT=$O/${T}_forward_world_latency_hist.json timeout -k 10 200 python tools/stage_timing.py > $O/${T}_stage_timing.log 2>&1 || { echo STAGE FAILED; tail -5 $O/${T}_stage_timing.log; exit 1; }
NIMBLE_AMD_LIB=dbg/libnimble_dbg.so timeout -k 10 200 python tools/stage_timing_bwd.py > $O/${T}_backward_stage_timing.log 2>&1 || { echo STAGE BWD FAILED; tail -5 $O/${T}_backward_stage_timing.log; exit 1; }
echo STAGE OK
