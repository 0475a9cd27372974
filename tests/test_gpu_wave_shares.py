"""The helper wave's early rows (contact.cuh EA_*: rows, J^T, Y and A built
by the helper during wave 0's dynamics) and the two-half Y = L^-1 J^T are
the same operations in the same order as wave 0's own path, so a rollout
with them (the default) and one without (NIMBLE_AMD_EARLY_ROWS=0, read when
the device model is built) must agree bit for bit -- and so must the
post-answer work in two shares (HS_POST) against wave 0 alone
(NIMBLE_AMD_POST_SPLIT=0): next states, warm-start
caches, snapshot headers and the backward's gradients, over three chained
steps of the bench's own batches (box-foot Atlas, 1024 worlds; STL-mesh
Atlas, 256 worlds, whose deferred worlds take the wide kernel)."""
import numpy as np
import pytest
import torch

from nimblephysics_amd import workloads
from test_gpu_contact_parity import SN_STATUS, _device_backward, _device_step

pytestmark = pytest.mark.gpu

_WORLDS = {"box": (lambda: workloads.atlas_world(True), 1024), "mesh": (lambda: workloads.atlas_mesh_world(True), 256)}


def _rollout(make, B, early, monkeypatch, steps=3, var="NIMBLE_AMD_EARLY_ROWS"):
    monkeypatch.setenv(var, "1" if early else "0")
    try:
        world = make()
        world.setStatusPolicy("record")
        st, f = workloads.atlas_states(world, B, 1000)
        g = np.random.default_rng(11).standard_normal(st.shape)
        out = []
        cache = None
        for _ in range(steps):
            nxt, snap, cache, ts, tf = _device_step(world, st, f, cache)
            gs, gf = _device_backward(world, ts, tf, snap, g)
            out.append((nxt.cpu().numpy(), cache.cpu().numpy(), snap[:, :SN_STATUS + 1].cpu().numpy(), gs, gf))
            st = nxt.cpu().numpy()
    finally:
        monkeypatch.delenv(var, raising=False)
    return out


@pytest.mark.parametrize("var", ["NIMBLE_AMD_EARLY_ROWS", "NIMBLE_AMD_POST_SPLIT"])
@pytest.mark.parametrize("kind", sorted(_WORLDS))
def test_early_rows_bit_identical(kind, var, monkeypatch):
    make, B = _WORLDS[kind]
    on = _rollout(make, B, True, monkeypatch, var=var)
    off = _rollout(make, B, False, monkeypatch, var=var)
    names = ("next state", "cache", "snapshot header", "grad state", "grad action")
    for step, (a, b) in enumerate(zip(on, off)):
        for name, x, y in zip(names, a, b):
            assert np.array_equal(x, y, equal_nan=True), (kind, step, name, np.flatnonzero(~np.all(x == y, axis=1))[:8])
    assert (on[0][2][:, 1] > 0).any()  # (worlds with LCP rows took the path)
