"""configs[4]'s exchange step on the device: the RCCL process group and the
per-step all-gather of the action gradients (north_star's "RCCL all-gather of
gradients over xGMI"), run through bench.init_dist / bench.run on the one GPU
of a test box (world size 1; two ranks cannot share one device under RCCL).

The rank runs in a fresh child interpreter with the torchrun env set before
any HIP call, exactly as `bench.py --gpus N` starts its ranks (bench.py
launch_ranks); every multi-GPU byte path other than this gather is the
single-GPU step the other -m gpu tests already check."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RANK = r"""
import json, os, sys
sys.path.insert(0, {root!r})
import torch
import bench

rec = []
gather0 = bench.gather_grads

def gather(dist, grad, ws):
    out = gather0(dist, grad, ws)
    assert out.device.type == "cuda" and grad.device.type == "cuda"
    assert dist.get_backend() == "nccl", dist.get_backend()
    assert dist.get_world_size() == ws == 1
    rec.append((grad.detach().clone(), out.clone()))
    return out

bench.gather_grads = gather
bench.run(bench.parse_args(["--gpus", "1", "--steps", "2", "--warmup", "1", "--gather-grads", "1",
                            "--batch", "64", "--no-mesh", "--no-cpu-baseline", "--out", {out!r}]))
assert len(rec) == 3, len(rec)  # 1 warmup + 2 timed steps, one gather each
for k, (own, got) in enumerate(rec):
    assert got.shape == own.shape and got.dtype == own.dtype == torch.float64, (k, got.shape, own.shape)
    assert torch.equal(got, own), k
    assert torch.isfinite(own).all() and own.abs().sum() > 0, k
print("RCCL_GATHER_OK", len(rec), rec[0][0].shape[0], flush=True)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_process_group_gathers_action_gradients(tmp_path):
    """bench.init_dist builds a `nccl` (RCCL) process group on cuda:0 with
    `device_id=`, bench.run steps the Atlas-on-ground batch fwd+bwd with
    --gather-grads 1, every all_gather_into_tensor of the per-world action
    gradients returns the rank's own gradients (world size 1), and the JSON
    line reports n_gpus from the process group."""
    out = tmp_path / "bench_rccl.json"
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               NIMBLE_BENCH_LAUNCHER="tests/test_gpu_rccl.py (torchrun env, one rank)")
    p = subprocess.run([sys.executable, "-c", _RANK.format(root=ROOT, out=str(out))], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "RCCL_GATHER_OK 3 64" in p.stdout, p.stdout[-2000:]
    line = json.loads(out.read_text())
    assert line["n_gpus"] == 1 and line["config"]["global_batch"] == 64
    assert "RCCL all-gather" in line["config"]["parallelism"] and line["value"] > 0
