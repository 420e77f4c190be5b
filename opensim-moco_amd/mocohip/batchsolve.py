"""configs[4]: a batch of MocoInverse solves (a subject sweep), one solver
per process -- its own HIP context and stream on the GPU, its own host
interior-point solver (mocohip.ipm, the Ipopt restatement) -- all on one
device, started together.  MocoInverse's setup: MocoInverse.cpp:46-120
(configs.gait10dof18musc_inverse); subjects are the generic model scaled by
(length, mass) factors (configs.scale_subject), which keep the generated
back end (structure-only specialization)."""
from __future__ import annotations

import multiprocessing as mp
import time
from typing import List, Sequence, Tuple


def sweep(count: int) -> List[Tuple[float, float]]:
    """``count`` subjects: lengths 0.97..1.03 and masses 0.90..1.10."""
    if count == 1:
        return [(1.0, 1.0)]
    return [(0.97 + 0.06 * i / (count - 1), 0.90 + 0.20 * ((i * 5) % count) / (count - 1))
            for i in range(count)]


def _worker(subject, num_mesh_intervals, device, start, out):
    from . import configs
    st = configs.gait10dof18musc_inverse(num_mesh_intervals, subject=subject)
    st.solver.device = device
    nlp = st.create_nlp()
    start.wait()                                  # every solver built: go
    t0 = time.perf_counter()
    try:
        sol = st.solve(nlp=nlp)
        r = sol.stats
        res = {"subject": list(subject), "success": bool(r.success), "iterations": int(r.iterations),
               "objective": float(r.objective), "wall_clock_s": round(time.perf_counter() - t0, 3),
               "backend": nlp.backend()[0]}
    except Exception as e:   # reported, not raised: the batch line says which solve failed
        res = {"subject": list(subject), "success": False, "error": repr(e)[:200]}
    finally:
        nlp.close()
    out.put((time.perf_counter(), res))


def solve_batch(subjects: Sequence[Tuple[float, float]], num_mesh_intervals: int = 125,
                device: int = 0, timeout: float = 600.0) -> dict:
    """Solve every subject's MocoInverse at once, one process each; wall
    clock from the common start to the last solution."""
    ctx = mp.get_context("spawn")
    start = ctx.Barrier(len(subjects) + 1)
    out = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(s, num_mesh_intervals, device, start, out), daemon=True)
             for s in subjects]
    for p in procs:
        p.start()
    start.wait(timeout=timeout)
    t0 = time.perf_counter()
    results = []
    t_last = t0
    for _ in procs:
        t, r = out.get(timeout=timeout)
        t_last = max(t_last, t)
        results.append(r)
    for p in procs:
        p.join(timeout=60)
    wall = t_last - t0
    ok = [r for r in results if r.get("success")]
    return {"solves": len(subjects), "processes": len(procs), "succeeded": len(ok),
            "wall_clock_s": round(wall, 3),
            "solves_per_minute": round(60.0 * len(subjects) / wall, 2) if wall > 0 else None,
            "mean_iterations": round(sum(r["iterations"] for r in ok) / len(ok), 1) if ok else None,
            "mean_solve_s": round(sum(r["wall_clock_s"] for r in ok) / len(ok), 3) if ok else None,
            "results": sorted(results, key=lambda r: r["subject"])}
