#!/bin/bash
# GPU-box iteration loop: parity tests, stage timing of the slowest worlds, bench.
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/gpu_tests.log | tail -4
[ $rc -ne 0 ] && exit $rc
NIMBLE_AMD_LIB=$PWD/dbg/libnimble_dbg.so timeout -k 10 200 python tools/stage_timing.py > gpurun_out/st.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/st.log | tail -${ST_TAIL:-24}
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline 2>/dev/null | cut -c1-${BENCH_CUT:-1200}
