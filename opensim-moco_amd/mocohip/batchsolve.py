"""configs[4]: a batch of MocoInverse solves (a subject sweep), one solver
per process -- its own HIP context and stream on the GPU, its own host
interior-point solver (mocohip.ipm, the Ipopt restatement) -- all on one
device, started together.  MocoInverse's setup: MocoInverse.cpp:46-120
(configs.gait10dof18musc_inverse); subjects are the generic model scaled by
(length, mass) factors (configs.scale_subject), which keep the generated
back end (structure-only specialization).

Set-up before the common start, per worker: the NLP (HIP context, device
buffers, generated back end) and, where the solve will factor on the
device, the device KKT module with its first kernel launches and graph
captures (mocohip.kkt.DeviceKKT.warm); the timed region holds the solves.

Failures are reported, not raised: a worker whose setup fails still reaches
the start barrier and posts its error, and the parent watches the workers
while it waits, so a worker that dies (a crash, a GPU fault) becomes a
failed entry of the batch instead of a hang."""
from __future__ import annotations

import multiprocessing as mp
import queue
import time
from typing import List, Sequence, Tuple


def sweep(count: int) -> List[Tuple[float, float]]:
    """``count`` subjects: lengths 0.97..1.03 and masses 0.90..1.10."""
    if count == 1:
        return [(1.0, 1.0)]
    return [(0.97 + 0.06 * i / (count - 1), 0.90 + 0.20 * ((i * 5) % count) / (count - 1))
            for i in range(count)]


def _worker(index, subject, num_mesh_intervals, device, start, out, linear_solver):
    nlp = None
    res = {"subject": list(subject), "success": False}
    try:
        from . import configs
        st = configs.gait10dof18musc_inverse(num_mesh_intervals, subject=subject)
        st.solver.device = device
        nlp = st.create_nlp()
        from .ipm import IpmOptions
        if linear_solver == "device" or (linear_solver == "auto" and
                                         nlp.m >= IpmOptions().device_kkt_min_constraints):
            nlp.device_kkt(warm=True)         # the device KKT module (and its first launches) set up before the start
    except Exception as e:   # setup failed: still meet the others at the barrier
        res["error"] = "setup: " + repr(e)[:200]
    try:
        start.wait()                          # every solver built: go
    except Exception:
        pass
    t0 = time.perf_counter()
    try:
        if nlp is not None:
            sol = st.solve(nlp=nlp, linear_solver=linear_solver)
            r = sol.stats
            res = {"subject": list(subject), "success": bool(r.success), "iterations": int(r.iterations),
                   "objective": float(r.objective), "wall_clock_s": round(time.perf_counter() - t0, 3),
                   "seconds_in_evaluations": round((r.timings or {}).get("evaluations_s", 0.0), 3),
                   "seconds_in_kkt": round((r.timings or {}).get("linear_algebra_s", 0.0), 3),
                   "linear_solver": (r.timings or {}).get("linear_solver"),
                   "backend": nlp.backend()[0]}
    except Exception as e:   # reported, not raised: the batch line says which solve failed
        res = {"subject": list(subject), "success": False, "error": repr(e)[:200]}
    finally:
        if nlp is not None:
            nlp.close()
    out.put((index, time.perf_counter(), res))


def solve_batch(subjects: Sequence[Tuple[float, float]], num_mesh_intervals: int = 125,
                device: int = 0, timeout: float = 600.0, linear_solver: str = "auto",
                hw_queues: int | None = 2) -> dict:
    """Solve every subject's MocoInverse at once, one process each; wall
    clock from the common start to the last solution.

    hw_queues: the workers' HIP hardware queues (GPU_MAX_HW_QUEUES, read by
    the HIP runtime at start-up; None keeps the environment's).  The sweep's
    kernels are small and latency-bound, so the solves overlap on the GPU only
    while their queues are mapped to it together: 8 workers with 2 queues
    each finish in 0.58 s, with the default 4 in 0.90 s and with 3 in 1.33 s
    (MI355X, 8 MocoInverse N = 125 solves) -- more queues than the GPU maps at
    once are time-sliced."""
    import os
    ctx = mp.get_context("spawn")
    start = ctx.Barrier(len(subjects) + 1)
    out = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(i, s, num_mesh_intervals, device, start, out, linear_solver),
                         daemon=True)
             for i, s in enumerate(subjects)]
    saved = os.environ.get("GPU_MAX_HW_QUEUES")
    if hw_queues is not None:
        os.environ["GPU_MAX_HW_QUEUES"] = str(int(hw_queues))   # inherited by the spawned workers
    try:
        for p in procs:
            p.start()
    finally:
        if hw_queues is not None:
            if saved is None:
                os.environ.pop("GPU_MAX_HW_QUEUES", None)
            else:
                os.environ["GPU_MAX_HW_QUEUES"] = saved
    try:
        start.wait(timeout=timeout)
    except Exception:      # a worker died before the barrier: the rest still run
        start.abort()
    t0 = time.perf_counter()
    results = {}
    t_last = t0
    deadline = t0 + timeout
    while len(results) < len(procs) and time.perf_counter() < deadline:
        try:
            i, t, r = out.get(timeout=1.0)
            results[i] = r
            t_last = max(t_last, t)
        except queue.Empty:
            # a worker that exited without posting crashed: record it
            for i, p in enumerate(procs):
                if i not in results and not p.is_alive() and p.exitcode not in (0, None):
                    results[i] = {"subject": list(subjects[i]), "success": False,
                                  "error": f"worker exited with code {p.exitcode}"}
    for i in range(len(procs)):
        results.setdefault(i, {"subject": list(subjects[i]), "success": False, "error": "timeout"})
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    wall = t_last - t0
    res = [results[i] for i in range(len(procs))]
    ok = [r for r in res if r.get("success")]
    return {"solves": len(subjects), "processes": len(procs), "succeeded": len(ok),
            "wall_clock_s": round(wall, 3),
            "solves_per_minute": round(60.0 * len(subjects) / wall, 2) if wall > 0 else None,
            "mean_iterations": round(sum(r["iterations"] for r in ok) / len(ok), 1) if ok else None,
            "mean_solve_s": round(sum(r["wall_clock_s"] for r in ok) / len(ok), 3) if ok else None,
            "linear_solver": ok[0].get("linear_solver") if ok else None,
            "results": sorted(res, key=lambda r: r["subject"])}


def rank_share(subjects: Sequence[Tuple[float, float]], rank: int, world: int) -> List[Tuple[float, float]]:
    """The subjects rank ``rank`` of ``world`` solves: every world-th one
    starting at its rank (independent solves: no data-path collective)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return list(subjects[rank::world])


def solve_sweep(count: int, num_mesh_intervals: int = 125, rank: int = 0, world: int = 1, device: int = 0,
                max_concurrent: int = 8, linear_solver: str = "auto", hw_queues: int | None = 2,
                timeout: float = 600.0) -> dict:
    """configs[4] over the ranks of a node: rank r solves rank_share(
    sweep(count), r, world) on its own GPU ``device``, in rounds of at most
    ``max_concurrent`` solver processes started together (solve_batch).
    Returns this rank's record; the caller reduces the ranks' counts and wall
    clocks (bench.py: an all-reduce of [solves, succeeded] and of the max
    wall clock)."""
    mine = rank_share(sweep(count), rank, world)
    rounds, wall, results = [], 0.0, []
    for i in range(0, len(mine), max(1, int(max_concurrent))):
        r = solve_batch(mine[i:i + max_concurrent], num_mesh_intervals, device=device, timeout=timeout,
                        linear_solver=linear_solver, hw_queues=hw_queues)
        rounds.append(r["wall_clock_s"])
        wall += r["wall_clock_s"]
        results += r["results"]
    ok = [r for r in results if r.get("success")]
    return {"rank": rank, "world": world, "solves": len(mine), "succeeded": len(ok),
            "rounds": len(rounds), "round_wall_clock_s": rounds, "wall_clock_s": round(wall, 3),
            "mean_iterations": round(sum(r["iterations"] for r in ok) / len(ok), 1) if ok else None,
            "results": results}
