#!/bin/bash
# GPU box: baseline harness (dbg/liblcp_bench_base.so) then the current one, solo latencies.
LCP_BENCH_LIB=$PWD/dbg/liblcp_bench_base.so timeout -k 10 120 python tools/lcp_bench.py run > gpurun_out/lb0.log 2>&1 || exit 1
cp gpurun_out/lcp_out.npy dbg/lcp_baseline.npy
timeout -k 10 120 python tools/lcp_bench.py run > gpurun_out/lb1.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/lb1.log | head -${LB_HEAD:-3}; grep "n=24" -A1 gpurun_out/lb1.log
timeout -k 10 120 python tools/lcp_bench.py solo
