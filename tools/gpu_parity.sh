set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_jacobians.py tests/test_gpu_contact_parity.py tests/test_gpu_mesh.py tests/test_gpu_rollout_parity.py -m gpu -v --timeout 300 --timeout-method thread > $O/${T}_parity.log 2>&1; rc=$?
tail -25 $O/${T}_parity.log
exit $rc
