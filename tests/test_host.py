"""CPU-only checks of the host side: the C-ABI library exports every symbol
include/nimble_amd.h declares, the world description flattening, the
ctypes struct layout, the product path refusing CPU tensors (no fallback),
and the multi-rank bench harness on gloo (world_size 2)."""
import ctypes as C
import json
import os
import re
import socket

import numpy as np
import pytest
import torch

import models

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "nimble_amd.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|const char\*)\s+(nimble_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    syms = _declared_symbols()
    for s in ("nimble_world_create", "nimble_world_destroy", "nimble_forward", "nimble_backward",
              "nimble_snapshot_doubles", "nimble_lcp_cache_doubles", "nimble_last_error",
              "nimble_num_collision_pairs"):
        assert s in syms


def test_library_exports_declared_symbols():
    from nimblephysics_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libnimble_amd.so not built (run __graft_entry__.build())")
    lib = C.CDLL(_native.LIB_PATH)
    for s in _declared_symbols():
        assert hasattr(lib, s), s


def test_desc_ctypes_layout_matches_header(tmp_path):
    """ctypes mirror == the C compiler's layout of nimble_world_desc."""
    import shutil
    import subprocess
    from nimblephysics_amd import _desc
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    fields = [f for f, _ in _desc.NimbleWorldDesc._fields_]
    src = tmp_path / "layout.c"
    body = "\n".join(f'printf("%zu\\n", offsetof(nimble_world_desc, {f}));' for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "nimble_amd.h"\nint main(void){'
                   f'printf("%zu\\n", sizeof(nimble_world_desc));{body}return 0;}}')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    vals = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert vals[0] == C.sizeof(_desc.NimbleWorldDesc)
    for f, off in zip(fields, vals[1:]):
        assert getattr(_desc.NimbleWorldDesc, f).offset == off, f


def test_world_description_atlas():
    w = models.atlas_world(True)
    d = w.desc_arrays()
    assert int(d["num_dofs"]) == 33
    assert int(d["num_shapes"]) == 3  # two box feet + the ground
    parent = np.asarray(d["parent"])
    assert (parent < np.arange(len(parent))).all()  # topological order
    jt = np.asarray(d["joint_type"])
    assert (jt == 3).sum() == 1 and (jt == 1).sum() == 27


def test_mass_argument_follows_reference_mass_dims():
    """timestep(world, state, action, mass): the reference's mass vector has
    getMassDims() entries, one per World::tuneMass(body, INERTIA_MASS)
    registration in order; setMasses writes the bodies (and re-versions the
    device model only when a value changes); a vector of the wrong size is
    rejected before any device work."""
    import nimblephysics_amd as nimble
    w = models.cartpole_world()
    assert w.getMassDims() == 0 and w.getMasses().shape == (0,)
    w.setMasses(np.zeros(0))
    with pytest.raises(ValueError):
        w.setMasses(np.ones(2))
    st = torch.tensor(w.getState())
    with pytest.raises(ValueError):
        nimble.timestep(w, st, torch.zeros(2, dtype=torch.float64), torch.ones(2, dtype=torch.float64))
    sk = w.skeletons[0]
    pole, cart = sk.bodies[1], sk.bodies[0]
    w.tuneMass(pole, "INERTIA_MASS", np.array([5.0]), np.array([0.1]))
    w.tuneMass(cart, "INERTIA_MASS")
    with pytest.raises(ValueError):
        w.tuneMass(pole, "INERTIA_MASS")
    with pytest.raises(ValueError):
        w.tuneMass(cart, "INERTIA_COLOR")
    assert w.getMassDims() == 2
    assert np.allclose(w.getMasses(), [pole.getMass(), cart.getMass()])
    assert w._mass_body_indices() == [1, 0]
    assert w.getMassUpperBound()[0] == 5.0 and w.getMassLowerBound()[0] == 0.1
    v0 = w._version
    w.setMasses(w.getMasses())
    assert w._version == v0  # unchanged masses keep the device model
    w.setMasses([0.7, 2.5])
    assert pole.getMass() == 0.7 and cart.getMass() == 2.5 and w._version > v0
    assert np.asarray(w.desc_arrays()["mass"])[1] == 0.7


def test_product_rejects_cpu_tensors():
    from nimblephysics_amd import _native
    with pytest.raises(RuntimeError):
        _native._require_device(torch.zeros(3, dtype=torch.float64))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, ws, port, out):
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    dev = torch.device("cpu")
    grad = torch.full((4, 3), float(rank), dtype=torch.float64)
    calls = []

    def step(x):
        calls.append(1)
        g = bench.gather_grads(dist, grad, ws)
        assert g.shape == (ws * 4, 3)
        assert torch.equal(g[4:], torch.full((4, 3), 1.0, dtype=torch.float64))
        return x + 1

    state, elapsed = bench.timed_loop(step, torch.zeros(1), 3, 2, dist, dev)
    out[rank] = (float(state.item()), elapsed, len(calls))
    dist.destroy_process_group()


def test_bench_harness_gloo_two_ranks():
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_rank_main, args=(2, port, out), nprocs=2, join=True)
    assert out[0][0] == 5.0 and out[1][0] == 5.0  # 2 warmup + 3 timed
    assert out[0][2] == 5
    assert abs(out[0][1] - out[1][1]) < 1e-12  # max over ranks agreed


class _OracleTimestep(torch.autograd.Function):
    """CPU stand-in for nimble.timestep in the multi-rank CPU test: the
    oracle's forward / backward (the checker, test-only) behind the same
    autograd signature, so bench's step, sharding and gather run for real."""

    @staticmethod
    def forward(ctx, ow, world, state, action):
        n = world.getNumDofs()
        forces = np.zeros((state.shape[0], n))
        forces[:, world.getActionSpace()] = action.numpy()
        ctx.ow, ctx.world = ow, world
        return torch.from_numpy(ow.forward(state.numpy(), forces))

    @staticmethod
    def backward(ctx, grad):
        gs, gf = ctx.ow.backward(grad.numpy())
        return None, None, torch.from_numpy(gs), torch.from_numpy(gf[:, ctx.world.getActionSpace()])


def _oracle_rollout_grads(world, rank, batch, steps):
    """The action gradients of `steps` bench steps of rank `rank`'s shard,
    computed in this process (no process group)."""
    import bench
    from oracle.oracle import OracleWorld
    ow = OracleWorld(world)
    st, f, g = bench.rank_inputs(world, models._box_sampler, batch, rank)
    action, g = torch.from_numpy(f), torch.from_numpy(g)
    grads = []

    def ts(w, s, a):
        out = _OracleTimestep.apply(ow, w, s, a)
        return out

    state = torch.from_numpy(st)
    for _ in range(steps):
        s = state.detach().requires_grad_(True)
        a = action.detach().requires_grad_(True)
        nxt = ts(world, s, a)
        nxt.backward(g)
        grads.append(a.grad.clone())
        state = nxt.detach()
    return grads


def _rank_bench_main(rank, ws, port, batch, out):
    import torch.distributed as dist
    import bench
    from oracle.oracle import OracleWorld
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    world = models.box_world()
    ow = OracleWorld(world)
    st, f, g = bench.rank_inputs(world, models._box_sampler, batch, rank)
    gathered = []
    step = bench.make_step(lambda w, s, a: _OracleTimestep.apply(ow, w, s, a), world, torch.from_numpy(f),
                           torch.from_numpy(g), True, dist, ws, gathered=gathered)
    state, elapsed = bench.timed_loop(step, torch.from_numpy(st), 2, 1, dist, torch.device("cpu"))
    out[rank] = ([t.numpy() for t in gathered], elapsed)
    dist.destroy_process_group()


def test_bench_sharded_gather_gloo_two_ranks():
    """bench.main's multi-GPU logic on CPU with real gradients: two gloo
    ranks, each stepping its own shard of box-on-ground worlds fwd+bwd
    (rank-seeded inputs, oracle timestep), all-gathering the per-world action
    gradients every step.  The gathered [ws*B, m] tensor of every step equals
    the concatenation of each rank's own gradients, recomputed here rank by
    rank without a process group."""
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, ROOT)
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    B = 6
    mp.spawn(_rank_bench_main, args=(2, port, B, out), nprocs=2, join=True)
    world = models.box_world()
    own = [_oracle_rollout_grads(world, r, B, 3) for r in range(2)]
    for r in range(2):
        gathered, _ = out[r]
        assert len(gathered) == 3  # 1 warmup + 2 timed steps
        for k in range(3):
            want = np.concatenate([own[0][k].numpy(), own[1][k].numpy()])
            assert gathered[k].shape == (2 * B, 6)
            assert np.array_equal(gathered[k], want), (r, k)
    assert not np.array_equal(own[0][0].numpy(), own[1][0].numpy())  # shards differ


_BOX_WL = ("box on ground (launcher test)", models.box_world, models._box_sampler, "launcher test metric", 6)


def _bench_spawned_rank(rank, nranks, port, argv):
    """One rank started by bench.launch_ranks in the launcher test: the host
    timestep (the oracle behind the autograd signature) in place of the GPU
    one, every all-gathered gradient recorded, then bench's own rank body."""
    import sys
    from types import SimpleNamespace
    sys.path.insert(0, ROOT)
    import bench
    from oracle.oracle import OracleWorld
    bench.WORKLOADS["box"] = _BOX_WL
    ows = {}

    def ts(w, s, a):
        return _OracleTimestep.apply(ows.setdefault(id(w), OracleWorld(w)), w, s, a)

    bench.nimble = SimpleNamespace(timestep=ts)
    rec = []
    gather0 = bench.gather_grads

    def gather(dist, grad, ws):
        out = gather0(dist, grad, ws)
        rec.append(out.numpy().copy())
        return out

    bench.gather_grads = gather
    bench._rank_entry(rank, nranks, port, argv)
    outdir = os.path.dirname(argv[argv.index("--out") + 1])
    np.save(os.path.join(outdir, f"gathered_rank{rank}.npy"), np.stack(rec))


def test_bench_main_spawns_ranks_for_gpus_two(tmp_path, monkeypatch):
    """`bench.py --gpus 2` with no launcher env starts its own two rank
    processes (bench.launch_ranks, spawned before any device call), each
    with the env torchrun would set; the ranks form a gloo group, step their
    own shards, all-gather the action gradients every step, and rank 0
    writes the one JSON line with n_gpus = 2.  Every gathered [2B, m] tensor
    equals the concatenation of both ranks' own gradients recomputed here."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setitem(bench.WORKLOADS, "box", _BOX_WL)
    out = tmp_path / "bench.json"
    argv = ["--gpus", "2", "--device", "cpu", "--workload", "box", "--steps", "2", "--warmup", "1",
            "--no-cpu-baseline", "--out", str(out)]
    bench.main(argv, rank_target=_bench_spawned_rank)
    line = json.loads(out.read_text())
    assert line["n_gpus"] == 2 and line["steps"] == 2 and line["config"]["global_batch"] == 12
    assert "all-gather" in line["config"]["parallelism"] and line["value"] > 0
    world = models.box_world()
    own = [_oracle_rollout_grads(world, r, 6, 3) for r in range(2)]
    for r in range(2):
        got = np.load(tmp_path / f"gathered_rank{r}.npy")
        assert got.shape == (3, 12, 6)  # 1 warmup + 2 timed steps
        for k in range(3):
            assert np.array_equal(got[k], np.concatenate([own[0][k].numpy(), own[1][k].numpy()])), (r, k)


def test_bench_main_rejects_world_size_mismatch(monkeypatch):
    """A launcher's WORLD_SIZE that differs from --gpus is an error (the run
    would otherwise time another number of GPUs than it reports)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("WORLD_SIZE", "4")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "2", "--no-cpu-baseline"])
    assert e.value.code not in (0, None)


def test_bench_failed_rank_fails_the_launch(tmp_path, monkeypatch):
    """A rank that exits non-zero makes launch_ranks return non-zero and
    stops the ranks still waiting."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    code = bench.launch_ranks(["--gpus", "2"], 2, target=_bench_failing_rank)
    assert code == 3


def _bench_failing_rank(rank, nranks, port, argv):
    import time
    if rank == 1:
        raise SystemExit(3)
    time.sleep(60)


def test_dynamics_setters_invalidate_device_model():
    """Every model setter bumps the world's version, so the next step
    re-uploads the model (the reference's setters act on the next
    World::step); no GPU needed to check the bookkeeping."""
    w = models.box_world()
    body = w.getSkeleton(0).getBodyNode(0)
    joint = body.getParentJoint()
    calls = [lambda: body.setMass(2.0), lambda: body.setLocalCOM([0.0, 0.1, 0.0]),
             lambda: body.setMomentOfInertia(1, 2, 3), lambda: body.setFrictionCoeff(0.5),
             lambda: body.setRestitutionCoeff(0.2), lambda: joint.setDampingCoefficient(0, 0.1),
             lambda: joint.setSpringStiffness(0, 1.0), lambda: joint.setPositionUpperLimit(0, 1.0),
             lambda: joint.setControlForceLowerLimit(0, -1.0), lambda: w.getSkeleton(1).setMobile(False),
             lambda: body.getShapeNode(0).setRelativeTransform(np.eye(4))]
    for c in calls:
        v = w._version
        c()
        assert w._version > v


def test_tune_inertia_entries_follow_with_respect_to_mass():
    """Every WrtMassBodyNodeEntryType (WithRespectToMass.cpp:35-181): dims,
    get / set order (INERTIA_FULL = mass, COM, Ixx Iyy Izz Ixy Ixz Iyz),
    COM_MU along the body's beta, and the selection from the device's
    [num_bodies, 10] inertia gradients to the mass vector."""
    w = models.cartpole_world()
    sk = w.skeletons[0]
    cart, pole = sk.bodies[0], sk.bodies[1]
    pole.setLocalCOM([0.1, -0.2, 0.3])
    pole.setMomentOfInertia(0.5, 0.6, 0.7, 0.01, 0.02, 0.03)
    pole.setBeta([0.0, 2.0, 1.0])
    w.tuneMass(pole, "INERTIA_COM")
    w.tuneMass(cart, "INERTIA_DIAGONAL")
    w.tuneMass(pole, "INERTIA_OFF_DIAGONAL")
    w.tuneMass(pole, "INERTIA_COM_MU")
    w.tuneMass(cart, "INERTIA_FULL")
    assert w.getMassDims() == 3 + 3 + 3 + 1 + 10
    m = w.getMasses()
    assert np.allclose(m[:3], [0.1, -0.2, 0.3]) and np.allclose(m[6:9], [0.01, 0.02, 0.03])
    assert np.isclose(m[9], -0.2 / 2.0)
    assert np.allclose(m[10:], np.concatenate([[cart.getMass()], cart.com, cart.moment]))
    m2 = m.copy()
    m2[9] = 0.25  # COM_MU: com = beta * mu
    w.setMasses(m2)
    assert np.allclose(pole.com, [0.0, 0.5, 0.25])
    only, S = w._mass_selection()
    assert not only and S.shape == (2 * 10, 20)
    # pole = body 1: COM columns 0..2, off-diagonal 6..8, COM_MU (beta) 9
    assert S[11, 0] == 1 and S[12, 1] == 1 and S[13, 2] == 1
    assert S[17, 6] == 1 and S[19, 8] == 1
    assert np.allclose(S[11:14, 9], [0.0, 2.0, 1.0])
    assert np.array_equal(S[0:10, 10:20], np.eye(10))


def test_set_cached_lcp_solution_host_logic():
    """World::setCachedLCPSolution: one vector for every world or one per
    world, applied to the batch's warm-start rows on the next step (size
    first, then x), empty rows for None; getCachedLCPSolution reads back."""
    from types import SimpleNamespace
    from nimblephysics_amd.timestep import _batch_state
    w = models.box_world()
    dev = SimpleNamespace(cache_doubles=10)
    w.setCachedLCPSolution(np.array([0.5, 0.25, 0.0]))
    assert np.array_equal(w.getCachedLCPSolution(), [0.5, 0.25, 0.0])
    bs = _batch_state(w, 3, dev, torch.device("cpu"))
    c = bs.cache.numpy()
    assert (c[:, 0] == 3).all() and np.array_equal(c[2, 1:4], [0.5, 0.25, 0.0])
    assert w._pending_lcp_cache is None
    w.setCachedLCPSolution([None, np.array([1.0]), np.array([2.0, 3.0])])
    c = _batch_state(w, 3, dev, torch.device("cpu")).cache.numpy()
    assert c[0, 0] == -1 and c[1, 0] == 1 and c[1, 1] == 1.0 and c[2, 0] == 2 and np.array_equal(c[2, 1:3], [2, 3])
    assert np.array_equal(w.getCachedLCPSolution(2), [2.0, 3.0]) and len(w.getCachedLCPSolution(0)) == 0
    w.setCachedLCPSolution([np.ones(2), np.ones(2)])
    with pytest.raises(ValueError):
        _batch_state(w, 3, dev, torch.device("cpu"))
    assert w._pending_lcp_cache is None  # a rejected value is dropped
    before = w._batch_state.cache.clone()
    w.setCachedLCPSolution([np.ones(2), np.ones(20), np.ones(2)])
    with pytest.raises(ValueError):
        _batch_state(w, 3, dev, torch.device("cpu"))
    assert torch.equal(w._batch_state.cache, before)  # validated before any row is written
    w.setCachedLCPSolution(np.ones(12))
    with pytest.raises(ValueError):
        _batch_state(w, 3, dev, torch.device("cpu"))
    # the getter returns a value set since the last step, not the last step's
    w.setCachedLCPSolution(np.array([4.0, 5.0]))
    assert np.array_equal(w.getCachedLCPSolution(1), [4.0, 5.0])


def test_init_dist_world_size_one_has_a_process_group():
    """A launcher's env with WORLD_SIZE=1 (torchrun --nproc-per-node 1, or the
    -m gpu RCCL test) gets a real process group, and the world size bench
    reports is the group's; a plain run (no WORLD_SIZE) has none."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import bench\n"
            "d, r, ws, loc = bench.init_dist('cpu')\n"
            "assert d is not None and d.is_initialized() and d.get_world_size() == ws == 1 and r == 0\n"
            "d.destroy_process_group(); print('PG_OK')\n") % ROOT
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "PG_OK" in p.stdout, p.stderr[-2000:]
    env.pop("WORLD_SIZE")
    p = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import bench; "
                        "assert bench.init_dist('cpu')[0] is None; print('NO_PG')" % ROOT],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "NO_PG" in p.stdout, p.stderr[-2000:]
