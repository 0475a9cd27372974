"""Benchmark: differentiable timesteps/sec (fwd+bwd) on a batch of worlds.

BASELINE.json metric "differentiable timesteps/sec (fwd+bwd), 1024-env Atlas
w/ contact".  One step = nimble.timestep forward over the whole batch +
backward of a synthetic upstream gradient through it (the reference's
TimestepLayer.forward/backward, python/nimblephysics/timestep.py), then the
batch state advances to the new state (a rollout, so contacts evolve and the
LCP warm start is exercised).  Inputs are resident in HBM.

Multi-GPU: one process per GPU, each advancing its own shard of independent
worlds (weak scaling; the per-step RCCL all-gather of the action gradients is
the only exchange); the timed region is bracketed by barriers and the max
over ranks is used.  The ranks come from torchrun (WORLD_SIZE must equal
--gpus) or, without a launcher, `bench.py --gpus N` spawns them itself.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import nimblephysics_amd as nimble  # noqa: E402
from nimblephysics_amd import _native  # noqa: E402
from nimblephysics_amd import workloads as models  # noqa: E402

FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (spec; = FP32 vector 157.3 / 2)
HBM_PEAK_GBS = 8000.0

_atlas_states = models.atlas_states
_cheetah_states = models.cheetah_states


# name -> (description, world factory, synthetic state sampler, metric, default worlds per GPU)
WORKLOADS = {
    "atlas": ("Atlas 33-DoF (atlas_v3_box_colliders) + ground, foot contact", lambda: models.atlas_world(True),
              _atlas_states, "differentiable timesteps/sec (fwd+bwd), 1024-env Atlas w/ contact", 1024),
    "atlas_mesh": ("Atlas 33-DoF (atlas_v3_no_head: 29 STL mesh colliders, the reference atlas_bench's model) "
                   "+ ground, foot contact", lambda: models.atlas_mesh_world(True), _atlas_states,
                   "differentiable timesteps/sec (fwd+bwd), 1024-env Atlas w/ contact, STL mesh colliders", 1024),
    "atlas_air": ("Atlas 33-DoF, no ground (contact-free)", lambda: models.atlas_world(False), _atlas_states,
                  "differentiable timesteps/sec (fwd+bwd), Atlas contact-free", 1024),
    "cartpole": ("cartpole, contact-free", models.cartpole_world, _atlas_states,
                 "differentiable timesteps/sec (fwd+bwd), 1024-env cartpole (configs[1])", 1024),
    "half_cheetah": ("half-cheetah 9-DoF (data/skel/half_cheetah.skel), capsules on the ground box",
                     models.half_cheetah_world, _cheetah_states,
                     "differentiable timesteps/sec (fwd+bwd), 4096-env half-cheetah w/ ground contact (configs[2])",
                     4096),
}


def init_dist(device_type="cuda"):
    """torch.distributed from the env a launcher set (torchrun, or
    launch_ranks below): RCCL ("nccl") on the GPU, gloo for the CPU test
    path.  A launcher's env (WORLD_SIZE set) always gets a process group,
    world size 1 included (torchrun --nproc-per-node 1, and the -m gpu test
    that runs the RCCL gather on the one GPU of a test box); a plain
    `python bench.py` has none.  Returns (dist or None, rank, world size as
    the process group reports it, local rank)."""
    if "WORLD_SIZE" not in os.environ:
        return None, 0, 1, 0
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type == "cuda":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    ws = dist.get_world_size()
    if ws != int(os.environ["WORLD_SIZE"]):
        raise SystemExit(f"bench: process group has {ws} ranks, WORLD_SIZE={os.environ['WORLD_SIZE']}")
    return dist, dist.get_rank(), ws, local


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(rank, nranks, port, argv):
    """Body of one rank started by launch_ranks: the torchrun env for this
    rank, then the ordinary single-rank main."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(nranks), LOCAL_WORLD_SIZE=str(nranks),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      NIMBLE_BENCH_LAUNCHER=f"bench.py --gpus {nranks} (one spawned process per GPU)")
    run(parse_args(argv))


def launch_ranks(argv, nranks, target=None):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes
    (multiprocessing "spawn": new interpreters, one per GPU) before this
    process makes any HIP call, each with the env torchrun would give it, and
    wait for all of them.  Rank 0 prints the JSON line.  Returns the exit code
    (non-zero if any rank failed)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    target = target or _rank_entry
    procs = [ctx.Process(target=target, args=(r, nranks, port, list(argv))) for r in range(nranks)]
    for p in procs:
        p.start()
    from multiprocessing.connection import wait
    code = 0
    live = list(procs)
    while live:
        wait([p.sentinel for p in live])
        for p in [p for p in live if not p.is_alive()]:
            live.remove(p)
            if p.exitcode != 0 and not code:
                code = p.exitcode if p.exitcode and p.exitcode > 0 else 1
                # a failed rank leaves the others waiting in a collective
                for q in live:
                    q.terminate()
    return code


def barrier(dist):
    if dist is not None:
        dist.barrier()


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def timed_loop(step, state, steps, warmup, dist, device):
    """W untimed warmup steps, then EXACTLY `steps` timed steps bracketed by
    barrier + device synchronize on both sides; returns (state, elapsed),
    elapsed = max over ranks."""
    for _ in range(warmup):
        state = step(state)
    _sync(device)
    barrier(dist)
    _sync(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        state = step(state)
    _sync(device)
    barrier(dist)
    _sync(device)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return state, elapsed


def gather_grads(dist, grad, ws):
    """north_star's RCCL all-gather of the per-world action gradients (the
    one exchange step of a multi-GPU training loop); returns [ws*B, m]."""
    out = torch.empty((ws * grad.shape[0],) + tuple(grad.shape[1:]), dtype=grad.dtype, device=grad.device)
    dist.all_gather_into_tensor(out, grad.contiguous())
    return out


def rank_inputs(world, sampler, batch, rank):
    """Rank `rank`'s shard of the synthetic workload: its own `batch`
    independent worlds (states, actions) and the upstream gradient of its
    next states, seeded by the rank so the shards differ and are
    reproducible."""
    st, f = sampler(world, batch, 1000 + rank)
    g = np.random.default_rng(rank).standard_normal(st.shape)
    return st, f, g


def make_step(timestep, world, action, g, gather, dist, ws, status_acc=None, gathered=None):
    """One bench step on this rank's shard: `timestep` forward over the
    batch, backward of the upstream gradient `g`, the per-world action
    gradients all-gathered over the process group when `gather` (appended to
    `gathered` when given), the state advanced to the next state."""

    def one_step(state):
        s = state.detach().requires_grad_(True)
        a = action.detach().requires_grad_(True)
        nxt = timestep(world, s, a)
        if status_acc is not None:
            status_acc.bitwise_or_(world.getLastStatus())
        nxt.backward(g)
        if gather and dist is not None:
            out = gather_grads(dist, a.grad, ws)
            if gathered is not None:
                gathered.append(out)
        return nxt.detach()

    return one_step


class KernelTimer:
    """HIP events around the native launches, on the stream they run on."""

    def __init__(self):
        self.fwd, self.bwd = [], []
        self.enabled = False

    def wrap(self, devworld):
        timer = self
        f0, b0 = devworld.forward, devworld.backward

        def fwd(*a):
            if not timer.enabled:
                return f0(*a)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            f0(*a)
            e.record()
            timer.fwd.append((s, e))

        def bwd(*a):
            if not timer.enabled:
                return b0(*a)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            b0(*a)
            e.record()
            timer.bwd.append((s, e))
        devworld.forward, devworld.backward = fwd, bwd

    @staticmethod
    def mean_ms(pairs):
        return float(np.mean([s.elapsed_time(e) for s, e in pairs])) if pairs else float("nan")


def rollout_stats(world, state, action, warmup, steps):
    """Contacts, LCP rows and clamping rows per world averaged over the timed
    steps: the bench's rollout is deterministic, so it is replayed after the
    timed region from the same initial state and cold LCP cache (forward
    only, through the C-ABI) and the snapshot headers of steps warmup ..
    warmup + steps - 1 are averaged -- the work that was timed."""
    dev = world.native()
    B = state.shape[0]
    cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=state.device)
    cache[:, 0] = -1
    n = world.getNumDofs()
    forces = torch.zeros((B, n), dtype=torch.float64, device=state.device)
    idx = torch.tensor(world.getActionSpace(), dtype=torch.long, device=state.device)
    forces.index_copy_(1, idx, action)
    snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=state.device)
    acc = torch.zeros(7, dtype=torch.float64, device=state.device)
    cur = state.clone()
    stream = torch.cuda.current_stream().cuda_stream
    for k in range(warmup + steps):
        nxt = torch.empty_like(cur)
        dev.forward(cur, forces, cache, nxt, snap, stream)
        if k >= warmup and dev.num_pairs > 0:
            h = snap[:, :3]
            acc[:3] += h.sum(0)
            acc[3] += (h[:, 0] > 0).sum()
            # the LCP solvers' executed work the kernels tally per world
            acc[4:7] += snap[:, _native.SN_PIVOTS:_native.SN_SOLVER_FLOPS + 1].sum(0)
        cur = nxt
    a = (acc / (B * max(steps, 1))).cpu().numpy()
    out = {"contacts": float(a[0]), "rows": float(a[1]), "clamping": float(a[2]), "worlds_in_contact": float(a[3]),
           "source": f"snapshot headers of the {steps} timed steps (deterministic replay after timing)"}
    if dev.num_pairs > 0:
        out["solver_counts"] = {"dantzig_pivots_per_world": float(a[4]), "pgs_sweeps_per_world": float(a[5]),
                                "solver_flops_per_world": float(a[6]),
                                "source": "snapshot elements NIMBLE_SNAPSHOT_PIVOTS / _SWEEPS / _SOLVER_FLOPS: "
                                          "the executed work of every Dantzig / PGS solve of the step (both "
                                          "waves, speculative solves cancelled by the cascade included)"}
    return out


def pmc_traffic(workload, kernels, batch):
    """HBM bytes per step of `kernels` (summed: the mesh model's forward is the
    one-row launch plus the wide launch) from the committed PMC summary
    (profiles/pmc_traffic.json: per-world FETCH_SIZE + WRITE_SIZE of the same
    kernels on the same workload, measured by tools/pmc_traffic.py under
    rocprofv3 --pmc -- counters cannot be read inside this process); None when
    absent.  Returned with the summary's provenance."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        es = [d[workload][k] for k in kernels]
        return (sum(float(e["bytes_per_world"]) for e in es) * batch,
                es[0].get("source", "profiles/pmc_traffic.json") + f" ({' + '.join(kernels)})")
    except Exception:
        return None, None


def pmc_mfma(workload, kernel):
    """fp64 MFMA use of `kernel` per launch from the committed PMC summary
    (profiles/pmc_mfma.json, tools/pmc_mfma.py over the rocprofv3 --pmc pass
    of tools/gpu_measure.sh): rocprofv3's MfmaUtil (SQ_VALU_MFMA_BUSY_CYCLES
    over GRBM_GUI_ACTIVE x SIMDs) and the MFMA FLOP rate; {} when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_mfma.json")
    try:
        e = json.load(open(path))[workload][kernel]
    except Exception:
        return {}
    out = {"mfma_util": e.get("mfma_util"), "mfma_tflops": e.get("mfma_tflops"),
           "mfma_flops_per_launch": e.get("mfma_f64_flops"), "mfma_source": "profiles/pmc_mfma.json"}
    return out


def _cpu_threads():
    """(threads to use, affinity size, why).  The GPU box grants each GPU a
    CPU share that its harness exports as OMP_NUM_THREADS (16 per GPU there;
    os.cpu_count() and the affinity mask show the whole machine): use every
    core of that share, or every affinity core when no share is exported."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        return max(1, min(n, int(share))), n, f"OMP_NUM_THREADS={share}: the host's CPU share for this GPU job"
    return n, n, "every core of the affinity mask"


def _host_cores():
    """(os.cpu_count(), this process's affinity size)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return os.cpu_count(), aff


def cpu_baseline(make, batch, sampler, seconds_target=12.0):
    """The oracle (the CPU restatement of the reference's step, `kind`
    "port") on every usable host core: one thread per core, each stepping its
    own `batch` worlds of the same workload fwd+bwd in a rollout for
    ~seconds_target (ctypes releases the GIL inside the C library)."""
    import threading
    from oracle.oracle import OracleWorld
    threads, usable, why = _cpu_threads()
    host_cpus, affinity = _host_cores()
    counts = [0] * threads
    stop = [False]

    def worker(t):
        world = make()
        o = OracleWorld(world)
        st, f = sampler(world, batch, 11 + t)
        g = np.random.default_rng(5 + t).standard_normal(st.shape)
        while not stop[0]:
            nxt = o.forward(st, f)
            o.backward(g)
            st = nxt
            counts[t] += 1

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(seconds_target)
    stop[0] = True
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    steps = sum(counts)
    return {"value": steps * batch / dt, "unit": "timesteps/s", "cores": threads, "kind": "port",
            "host_cpu_count": host_cpus, "affinity_cpus": affinity,
            "cores_note": f"threads used = {threads} ({why}); affinity mask {usable} cores",
            "sample": f"{steps} fwd+bwd steps x {batch} worlds of the same workload, oracle/liboracle.so "
                      f"(CPU restatement of the reference's step), {threads} threads, {dt:.1f}s"}


def measure(wl, batch, steps, warmup, dist, rank, ws, dev, gather):
    """Time `steps` bench steps (after `warmup`) of workload `wl` on this
    rank's `batch` worlds; returns the measured numbers (value = worlds x
    steps x ranks / max-over-ranks elapsed).  On a CPU device (the launcher's
    gloo test, with a host timestep patched in by the test) only the timing
    and the gather run: the kernel timers, status words, replay statistics and
    roofline need the GPU."""
    wl_name, make, sampler, metric, default_batch = WORKLOADS[wl]
    batch = batch if batch > 0 else default_batch
    gpu = dev.type == "cuda"
    world = make()
    n = world.getNumDofs()
    st, f, g = rank_inputs(world, sampler, batch, rank)
    state = torch.tensor(st, device=dev)
    action = torch.tensor(f, device=dev)
    g = torch.tensor(g, device=dev)
    state0 = state.clone()
    status_acc = None
    timer = KernelTimer()
    if gpu:
        # status words are recorded on the device each step (no per-step host
        # sync) and checked once after the timed region: a world whose step
        # could not be the reference's fails the bench instead of being timed
        world.setStatusPolicy("record")
        timer.wrap(world.native())
        status_acc = torch.zeros(batch, dtype=torch.int32, device=dev)
    one_step = make_step(nimble.timestep, world, action, g, gather, dist, ws, status_acc)
    for _ in range(warmup):
        state = one_step(state)
    timer.enabled = gpu
    state, elapsed = timed_loop(one_step, state, steps, 0, dist, dev)
    timer.enabled = False
    out = {"wl": wl, "wl_name": wl_name, "metric": metric, "make": make, "sampler": sampler, "batch": batch, "n": n,
           "value": batch * ws * steps / elapsed, "ms_per_step": elapsed / steps * 1e3, "cstats": None,
           "flops": None}
    if not gpu:
        return out
    bad = int(((status_acc & _native.ST_DIVERGES) != 0).sum().item())
    if bad:
        raise SystemExit(f"bench ({wl}): {bad} world(s) left the reference's physics "
                         f"({_native.status_message(int(np.bitwise_or.reduce(status_acc.cpu().numpy())))})")
    cstats = rollout_stats(world, state0, action, warmup, steps)
    fwd_ms = timer.mean_ms(timer.fwd)
    bwd_ms = timer.mean_ms(timer.bwd)
    flops = _native.flop_estimate(world, cstats["rows"], cstats["clamping"])
    dom = "backward" if bwd_ms >= fwd_ms else "forward"
    dom_ms = max(bwd_ms, fwd_ms)
    achieved = flops[dom] * batch / (dom_ms * 1e-3) / 1e12
    # (models with mesh colliders run the one-row forward as its mesh instance)
    one_row = "nimble_forward_mesh_kernel" if (dom == "forward" and wl == "atlas_mesh") else f"nimble_{dom}_kernel"
    traffic, traffic_src = pmc_traffic(wl, [one_row] + ([f"nimble_{dom}_wide_kernel"] if wl == "atlas_mesh" else []),
                                       batch)
    out.update(cstats=cstats, fwd_ms=fwd_ms, bwd_ms=bwd_ms, dom=dom, achieved=achieved, flops=flops,
               traffic=traffic, traffic_src=traffic_src)
    sc = cstats.get("solver_counts")
    if sc is not None:
        fs = dict(flops)
        fs["forward"] = flops["forward"] + sc["solver_flops_per_world"]
        out.update(flops_solvers=fs, solver_counts=sc,
                   achieved_solvers=fs[dom] * batch / (dom_ms * 1e-3) / 1e12)
    return out


def roofline(r, wl):
    """The `roofline` object for the dominant kernel of the headline."""
    dom = r["dom"]
    out = {"bound": "fp64-valu", "kernel": f"nimble_{dom}_kernel", "achieved": r["achieved"],
           "peak": FP64_VECTOR_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": r["achieved"] / FP64_VECTOR_PEAK_TFLOPS,
           "traffic": r["traffic"], "traffic_source": r["traffic_src"],
           **pmc_mfma(wl, f"nimble_{dom}_kernel"),
           "flops_per_world": r["flops"][dom]}
    if r.get("achieved_solvers") is not None:
        out["achieved_with_solvers"] = r["achieved_solvers"]
        out["frac_with_solvers"] = r["achieved_solvers"] / FP64_VECTOR_PEAK_TFLOPS
        out["flops_per_world_with_solvers"] = r["flops_solvers"][dom]
        out["solver_counts"] = r["solver_counts"]
    out["note"] = ("peak = MI355X fp64 vector (VALU) rate, which on MI355X equals the fp64 matrix-core rate; "
                   "frac counts the direct work (dynamics, rows, A = Y^T Y on v_mfma_f64_16x16x4f64, COD solves, "
                   "backward precompute); frac_with_solvers adds the iterative solvers' work from the pivot and "
                   "sweep counts the kernels record per world (Dantzig pivots, PGS sweeps); traffic = HBM bytes "
                   "per launch (2 x FETCH_SIZE + WRITE_SIZE, separate rocprofv3 --pmc passes) from the committed "
                   "summary profiles/pmc_traffic.json")
    return out


def mesh_report(args, mesh):
    """The `atlas_mesh` object: the reference atlas_bench's own model."""
    mf = mesh["flops"]
    kern = {"forward": "nimble_forward_mesh_kernel + nimble_forward_wide_kernel",
            "backward": "nimble_backward_kernel + nimble_backward_wide_kernel"}[mesh["dom"]]
    out = {"workload": mesh["wl_name"], "metric": mesh["metric"], "value": mesh["value"], "unit": "timesteps/s",
           "ms_per_step": mesh["ms_per_step"], "steps": min(args.steps, 20),
           "kernels_ms": {"forward": mesh["fwd_ms"], "backward": mesh["bwd_ms"],
                          "note": "forward = nimble_forward_mesh_kernel (the one-row forward's instance for models "
                                  "with mesh colliders) + nimble_forward_wide_kernel (the worlds the "
                                  "one-row kernel defers), backward likewise; per-kernel split in "
                                  "profiles/*kernel_stats_atlas_mesh*"},
           "contacts_per_world": mesh["cstats"]["contacts"], "lcp_rows_per_world": mesh["cstats"]["rows"],
           "clamping_rows_per_world": mesh["cstats"]["clamping"],
           "frac": mesh["achieved"] / FP64_VECTOR_PEAK_TFLOPS, "frac_kernel": kern,
           "flops_per_world": mf[mesh["dom"]], "traffic": mesh["traffic"], "traffic_source": mesh["traffic_src"],
           **pmc_mfma("atlas_mesh", "nimble_forward_wide_kernel")}
    if mesh.get("achieved_solvers") is not None:
        out["frac_with_solvers"] = mesh["achieved_solvers"] / FP64_VECTOR_PEAK_TFLOPS
        out["flops_per_world_with_solvers"] = mesh["flops_solvers"][mesh["dom"]]
        out["solver_counts"] = mesh["solver_counts"]
    return out


def report(args, r, mesh, ws, gather):
    """Rank 0's JSON line."""
    cstats = r["cstats"]
    out = {
        "metric": r["metric"],
        "value": r["value"], "unit": "timesteps/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (perturbed poses near / in ground contact, random torques)",
        "config": {"workload": r["wl_name"], "worlds_per_gpu": r["batch"], "dofs": r["n"],
                   "global_batch": r["batch"] * ws,
                   "parallelism": f"independent worlds x{ws}" + (" + RCCL all-gather of action grads" if gather else ""),
                   "launcher": os.environ.get("NIMBLE_BENCH_LAUNCHER", "torchrun" if ws > 1 else "single process"),
                   **({k: cstats[k] for k in ("contacts", "rows", "clamping", "worlds_in_contact", "source")}
                      if cstats else {})},
    }
    if cstats:
        out["config"] = {**{k: v for k, v in out["config"].items()
                            if k not in ("contacts", "rows", "clamping", "worlds_in_contact", "source")},
                         "contacts_per_world": cstats["contacts"], "lcp_rows_per_world": cstats["rows"],
                         "clamping_rows_per_world": cstats["clamping"],
                         "worlds_in_contact": cstats["worlds_in_contact"], "contact_stats_source": cstats["source"]}
    if r["flops"] is not None:
        out["kernels_ms"] = {"forward": r["fwd_ms"], "backward": r["bwd_ms"]}
        out["roofline"] = roofline(r, args.workload)
    if mesh is not None:
        out["atlas_mesh"] = mesh_report(args, mesh)
    if not args.no_cpu_baseline and args.device == "cuda":
        out["cpu_baseline"] = cpu_baseline(r["make"], 16, r["sampler"])
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="worlds per GPU (default: the workload's)")
    ap.add_argument("--workload", default="atlas", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-mesh", action="store_true",
                    help="skip the second measurement of the reference atlas_bench's STL-mesh Atlas")
    ap.add_argument("--gather-grads", type=int, default=-1,
                    help="all-gather action gradients each step (default: on when N > 1)")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: gloo process group on host tensors (the launcher's CPU test; the product "
                         "timestep itself runs only on the GPU)")
    ap.add_argument("--out", default=None, help="also write rank 0's JSON line to this file")
    return ap.parse_args(argv)


def run(args):
    """One rank: init the process group from the env, measure, rank 0 prints."""
    dist, rank, ws, local = init_dist(args.device)
    if ws != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE {ws} != --gpus {args.gpus}")
    if args.device == "cuda":
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    gather = (ws > 1) if args.gather_grads < 0 else bool(args.gather_grads)
    r = measure(args.workload, args.batch, args.steps, args.warmup, dist, rank, ws, dev, gather)
    # the reference atlas_bench's own model (atlas_v3_no_head.urdf, 29 STL
    # colliders), measured after the headline's timed region on the same
    # ranks: reported beside the headline, never as `value`
    mesh = None
    if args.workload == "atlas" and not args.no_mesh:
        mesh = measure("atlas_mesh", args.batch, min(args.steps, 20), min(args.warmup, 3), dist, rank, ws, dev, gather)
    if rank == 0:
        out = report(args, r, mesh, ws, gather)
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as fh:
                fh.write(line + "\n")
    if dist is not None:
        dist.destroy_process_group()


def main(argv=None, rank_target=None):
    """`python bench.py --gpus N ...`: under a launcher (torchrun: WORLD_SIZE
    set) this process is one rank and WORLD_SIZE must equal N; without one,
    N > 1 starts N rank processes itself (launch_ranks) so the job spans N
    GPUs either way."""
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is not None and int(env_ws) != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={env_ws} from the launcher but --gpus {args.gpus}")
    if args.gpus > 1 and env_ws is None:
        code = launch_ranks(argv, args.gpus, rank_target)
        if code:
            raise SystemExit(code)
        return
    run(args)


if __name__ == "__main__":
    main()
