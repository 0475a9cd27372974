"""The deadlock guard's failure paths on the device (contact.cuh helperWait /
collideWait and the task board's wait, the GW_* sites), run on purpose: with
NIMBLE_AMD_GUARD_TEST="sites:stride:offset" (capi.cpp, tests only) the wait
at the chosen site expires at once in the worlds env % stride == offset, as
if the world's other wave were late at exactly that point.

Per site, on the bench's own batches (the box-foot Atlas, 1024 worlds, one-row
kernel; the STL-mesh Atlas, 256 worlds, its deferred worlds on the wide kernel
too), against the same batch stepped without the switch:

* the launch drains (the forward and the backward return);
* only targeted worlds carry NIMBLE_STATUS_PROTOCOL -- every targeted world
  where the site is on every world's path (the collision hand-off, the
  helper's task and idle waits, the end-of-world retire), a non-empty subset
  where it is not (the task board's waits);
* a flagged world either abandoned its contact step (snapshot header with no
  contacts and no rows, status ST_PROTOCOL alone, warm start dropped, next
  state = the contact-free step of the same state) or completed it: next
  state, cache and gradients bit-identical to the unforced run;
* every other world is bit-identical to the unforced run.

The deferred worlds' case of ADVICE r5 (a protocol failure of the one-row
kernel's turn must survive the wide kernel's status write) is the
`retire_one_row` case on the mesh Atlas."""
import numpy as np
import pytest

from nimblephysics_amd import _native, workloads
from test_gpu_contact_parity import SN_M, SN_NCON, SN_STATUS, _device_backward, _device_step

pytestmark = pytest.mark.gpu

STRIDE, OFFSET = 3, 1
# site -> (GW_* mask, on every world's path, what a flagged world does)
SITES = {"helper_go": (1, True, "abort"), "collide_done": (2, True, "abort"), "board": (8, False, "abort"),
         "collect": (32, False, "abort"), "helper_task": (64, True, "either"),
         # (the helper's last wait: its failure there can come after wave 0
         # has written the world's status -- a world that then shows no flag
         # is bit-identical to the unforced run, which _check verifies)
         "helper_idle": (256, False, "either"),
         "retire": (512, True, "complete"),
         # the early rows' hand-off (one-row kernel, LCP in the LDS pool): the
         # helper waiting for wave 0's b, wave 0 for the rows and for A
         "early_b": (2048, False, "abort"), "early_dyn": (32768, False, "abort"), "early_rows": (4096, False, "abort"), "early_a": (8192, False, "abort"),
         # wave 0 waiting for the helper's post-answer share (impulse, snapshot rows)
         "post": (16384, False, "abort")}
_base = {}


def _run(make, B, guard, monkeypatch):
    if guard:
        monkeypatch.setenv("NIMBLE_AMD_GUARD_TEST", guard)
    else:
        monkeypatch.delenv("NIMBLE_AMD_GUARD_TEST", raising=False)
    try:
        world = make()
        world.setStatusPolicy("record")
        st, f = workloads.atlas_states(world, B, 1000)
        g = np.random.default_rng(7).standard_normal(st.shape)
        nxt, snap, cache, ts, tf = _device_step(world, st, f)  # (the device model is built here)
        gs, gf = _device_backward(world, ts, tf, snap, g)
    finally:
        monkeypatch.delenv("NIMBLE_AMD_GUARD_TEST", raising=False)
    return {"nxt": nxt.cpu().numpy(), "snap": snap.cpu().numpy(), "cache": cache.cpu().numpy(), "gs": gs, "gf": gf}


def _baseline(kind, monkeypatch):
    if kind not in _base:
        make, B = _WORLDS[kind]
        out = _run(make, B, None, monkeypatch)
        # the contact-free step of the same states (the aborted worlds' next state)
        free = {"box": lambda: workloads.atlas_world(False), "mesh": lambda: workloads.atlas_mesh_world(False)}[kind]
        out["free"] = _run(free, B, None, monkeypatch)["nxt"]
        _base[kind] = out
    return _base[kind]


_WORLDS = {"box": (lambda: workloads.atlas_world(True), 1024), "mesh": (lambda: workloads.atlas_mesh_world(True), 256)}


def _check(kind, site_name, mask, everywhere, expect, monkeypatch):
    base = _baseline(kind, monkeypatch)
    make, B = _WORLDS[kind]
    got = _run(make, B, f"{mask}:{STRIDE}:{OFFSET}", monkeypatch)
    targeted = np.arange(B) % STRIDE == OFFSET
    status = got["snap"][:, SN_STATUS].astype(np.int64)
    flagged = (status & _native.ST_PROTOCOL) != 0
    assert not flagged[~targeted].any(), (site_name, np.flatnonzero(flagged & ~targeted)[:8])
    if everywhere:
        assert flagged[targeted].all(), (site_name, np.flatnonzero(targeted & ~flagged)[:8])
    else:
        assert flagged.any(), site_name
    same = {k: np.array([np.array_equal(got[k][b], base[k][b]) for b in range(B)]) for k in ("nxt", "cache", "gs", "gf")}
    unforced = ~flagged
    for k, eq in same.items():
        assert eq[unforced].all(), (site_name, k, np.flatnonzero(unforced & ~eq)[:8])
    aborted = flagged & (got["snap"][:, SN_NCON] == 0) & (got["snap"][:, SN_M] == 0)
    completed = flagged & ~aborted
    if expect == "abort":
        assert not completed.any(), (site_name, np.flatnonzero(completed)[:8])
    elif expect == "complete":
        assert not aborted[base["snap"][:, SN_M] > 0].any(), site_name
    for k, eq in same.items():
        assert eq[completed].all(), (site_name, k, np.flatnonzero(completed & ~eq)[:8])
    if aborted.any():
        a = np.flatnonzero(aborted)
        assert (status[a] == _native.ST_PROTOCOL).all() and (got["snap"][a, :SN_STATUS] == 0).all()
        assert (got["cache"][a, 0] == -1).all()
        err = np.abs(got["nxt"][a] - base["free"][a]).max() / max(1.0, np.abs(base["free"][a]).max())
        assert err <= 1e-12, (site_name, err)
        assert np.isfinite(got["gs"][a]).all() and np.isfinite(got["gf"][a]).all()
    return flagged, aborted, base


@pytest.mark.parametrize("site", sorted(SITES))
def test_guard_forced_expiry_atlas(site, monkeypatch):
    mask, everywhere, expect = SITES[site]
    flagged, aborted, base = _check("box", site, mask, everywhere, expect, monkeypatch)
    print(site, "flagged", int(flagged.sum()), "aborted", int(aborted.sum()),
          "in contact among aborted", int((base["snap"][aborted, SN_M] > 0).sum()))


@pytest.mark.parametrize("site", ["board", "collect", "collide_done", "retire_one_row"])
def test_guard_forced_expiry_mesh_wide(site, monkeypatch):
    """The STL-mesh Atlas: the one-row kernel's waits and, for the worlds it
    defers (more LCP rows than its pool holds), the wide kernel's own task
    board.  retire_one_row (GW_RETIRE | GW_ONE_ROW_ONLY): the protocol flag of
    the one-row kernel's turn of a deferred world must survive the wide
    kernel, which completes the world's step as without the failure."""
    if site == "retire_one_row":
        mask, everywhere, expect = 512 | 1024, True, "complete"
    else:
        mask, everywhere, expect = SITES[site]
    flagged, aborted, base = _check("mesh", site, mask, everywhere, expect, monkeypatch)
    wide = base["snap"][:, SN_M] > 24  # the worlds the one-row kernel defers
    print(site, "flagged", int(flagged.sum()), "aborted", int(aborted.sum()), "deferred flagged",
          int((flagged & wide).sum()), "of", int(wide.sum()))
    if site in ("board", "collect"):
        assert (flagged & wide).any(), site  # the wide kernel's board waits were reached
    if site == "retire_one_row":
        assert (flagged & wide).sum() == (wide & (np.arange(len(wide)) % STRIDE == OFFSET)).sum() > 0
