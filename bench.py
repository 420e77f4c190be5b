#!/usr/bin/env python
"""Benchmark: NLP eval_g + eval_jac_g calls/sec on MocoTrack gait10dof18musc
(DeGrooteFregly2016 muscles, rigid tendon, 18 excitations + 10 reserves,
GRF external loads, Hermite-Simpson, forward finite differences),
BASELINE.json configs[2] (N=200 mesh intervals).

One step = one eval_g and one eval_jac_g of the full NLP at an iterate
resident in HBM (device-pointer C ABI), results left in HBM
(--mode fused: the one-call form IPOPT's eval_g(new_x) -> eval_jac_g(!new_x)
pair allows; identical results).

Timed region: K steps without per-call instrumentation.  The roofline
numbers come from a second, instrumented pass of the same K steps right
after it (HIP events between the stages on the context stream; they cost
microseconds per call, so they stay out of `value`).

--gpus N > 1 (one process per GPU, torch.distributed.run):
  --multi replicas (default): every rank evaluates its own copy of the NLP
      (the configs[4] batch layout: independent NLPs, one per GPU, no
      collective on the data path) -> "scaling": "weak".
  --multi mesh: the mesh intervals of ONE NLP are sharded over the ranks and
      the g / Jacobian segments all-gathered over RCCL every step (what a
      single host IPOPT needs) -> "scaling": "strong".

Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) dense peak, spec
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md (spec; 6.29 TB/s measured copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--intervals", type=int, default=200)
    ap.add_argument("--fd", default="forward")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["separate", "fused"], default="separate",
                    help="separate: eval_g then eval_jac_g C-ABI calls; fused: one "
                         "mh_eval_g_jac_g call (IPOPT new_x=false pattern)")
    ap.add_argument("--multi", choices=["replicas", "mesh"], default="replicas")
    ap.add_argument("--single-mode", action="store_true",
                    help="measure only --mode (no secondary mode, no batch): for profiler runs, so "
                         "that every launch of a kernel has the same shape")
    ap.add_argument("--inverse-batch", type=int, default=8,
                    help="also measure B MocoInverse NLPs per GPU (configs[4]: prescribed "
                         "kinematics, implicit tendons, random sparsity, mesh_interval 0.02 s), "
                         "0 = skip")
    ap.add_argument("--batch", type=int, default=8,
                    help="also measure B independent NLPs per GPU evaluated concurrently, one "
                         "context (HIP stream) and host thread each (the configs[4] batch layout); "
                         "reported beside the headline, 0 = skip")
    return ap.parse_args()


def latest_pmc():
    """Per-launch HBM bytes of the hot kernels from the committed rocprofv3
    PMC summary of the current code (profiles/pmc_current.json, written by
    tools/pmc_summary.py and copied by tools/collect_profile.sh)."""
    path = os.path.join(ROOT, "profiles", "pmc_current.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as fh:
        d = json.load(fh)
    return d, d.get("source", "profiles/pmc_current.json")


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from mocohip import configs
    from mocohip.distributed import ShardGather, interval_shard
    from mocohip.solver import HipNLP

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    mesh = world > 1 and args.multi == "mesh"

    N = args.intervals
    st = configs.gait10dof18musc(N, fd_scheme=args.fd)
    st.solver.device = local
    rep = st.problem.create_rep()
    ib, ie = interval_shard(N, rank, world) if mesh else (0, N)
    nlp = HipNLP(rep, st.solver.options(ib, ie))
    # iterate: bounds midpoint for the states (where the muscle model is
    # regular), uniform random controls within bounds (seed 0; replicas use
    # seed = rank: independent trials)
    x = nlp.random_iterate(np.random.default_rng(rank if not mesh else 0).uniform(-1, 1, nlp.n))
    xm = nlp.initial_guess_from_bounds()
    x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
    dev = torch.device("cuda", local)
    xd = torch.tensor(x, dtype=torch.float64, device=dev)
    rpi = nlp.m // N
    nzi = nlp.nnz // N
    sg = ShardGather(N, rpi, nzi, world if mesh else 1, dev)
    gseg, vseg = sg.gseg, sg.vseg

    rec = {"g": [], "jac": []}

    def step(record=False):
        if args.mode == "fused":
            nlp.eval_g_jac_g_device(xd.data_ptr(), gseg.data_ptr(), vseg.data_ptr())
            if record:
                rec["jac"].append(nlp.last_timings())
        else:
            nlp.eval_g_device(xd.data_ptr(), gseg.data_ptr())
            if record:
                rec["g"].append(nlp.last_timings())
            nlp.eval_jac_g_device(xd.data_ptr(), vseg.data_ptr())
            if record:
                rec["jac"].append(nlp.last_timings())
        if mesh:
            sg.gather()

    def timed(k, record):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step(record)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    for _ in range(args.warmup):
        step()
    elapsed = timed(args.steps, False)
    # secondary: the same K steps as one fused call each (IPOPT's
    # eval_g(new_x) -> eval_jac_g(!new_x) pair from one DAE pass)
    other = "fused" if args.mode == "separate" else "separate"
    other_elapsed = None
    if not args.single_mode:
        mode0, args.mode = args.mode, other
        for _ in range(args.warmup):
            step()
        other_elapsed = timed(args.steps, False)
        args.mode = mode0
    # instrumented pass (roofline): same K steps with stage events
    nlp.set_timing(True)
    inst_elapsed = timed(args.steps, True)
    nlp.set_timing(False)

    # secondary: the same workload with optim_sparsity_detection "random"
    # (MocoInverse's setting, MocoInverse.cpp:111): detected callback
    # couplings only, same iterate, separate calls
    sparse = None
    if not args.single_mode and not mesh:
        import copy
        s2 = copy.copy(st.solver)
        s2.optim_sparsity_detection = "random"
        nls = HipNLP(rep, s2.options())
        vs = torch.empty(nls.nnz, dtype=torch.float64, device=dev)
        gs = torch.empty(nls.m, dtype=torch.float64, device=dev)

        def sstep():
            nls.eval_g_device(xd.data_ptr(), gs.data_ptr())
            nls.eval_jac_g_device(xd.data_ptr(), vs.data_ptr())
        for _ in range(args.warmup):
            sstep()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            sstep()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        sparse = {"value": round(args.steps * world / el, 3), "unit": "calls/s", "nnz_jac": nls.nnz,
                  "mode": "separate", "note": "optim_sparsity_detection=random (3 iterates)"}
        nls.close()

    ms_per_step = 1e3 * elapsed / args.steps
    value = (args.steps if mesh else args.steps * world) / elapsed
    batch = None
    if args.batch > 1 and not mesh and not args.single_mode:
        batch = batch_throughput(args, rep, st, local, rank, world, dev, torch, dist)
    inverse = None
    if args.inverse_batch > 0 and not mesh and not args.single_mode:
        # MocoTool mesh_interval 0.02 s: ceil((2.499 - 0.001) / 0.02) = 125
        # intervals (MocoTool.cpp:27,68-69)
        ist = configs.gait10dof18musc_inverse(125, fd_scheme="forward", sparsity="random")
        ist.solver.device = local
        irep = ist.problem.create_rep()
        inverse = batch_throughput(args, irep, ist, local, rank, world, dev, torch, dist,
                                   B=args.inverse_batch, make_x=inverse_iterate)
        inverse["workload"] = ("MocoInverse gait10dof18musc (configs[4]): PositionMotion, implicit DGF "
                               "tendons, reserves, N=125, forward FD, random sparsity detection")

    if rank == 0:
        J = np.array(rec["jac"])          # [whole, DAE stage, transcription stage, k_groups] ms
        dae_ms = float(np.median(J[:, 1]))
        tr_ms = float(np.median(J[:, 2]))
        G_local = nlp.G if not mesh else (2 * (ie - ib) + 1)
        ND = nlp.NS + nlp.NC + 2              # FD directions incl. t0, tf
        n_dae = G_local * (ND + 1) if args.fd != "central" else G_local * (2 * ND + 1)
        be_name, f_dae, mhash = nlp.backend()
        work = nlp.work()                     # executed FP64 ops of the (pruned) task kernels
        flops = n_dae * f_dae                 # algorithmic: one full DAE per FD lane
        nnz_local = (ie - ib) * nzi
        alg_bytes_jac = 8 * (nlp.n + nnz_local)   # x in, Jacobian values out
        fused_iv = nlp.uses_interval_kernel()
        tr_kernel = "k_interval" if fused_iv else "k_transcribe"
        pmc, pmc_src = latest_pmc()
        traffic = dae_traffic = None
        if pmc and pmc.get("workload") == f"N={N},fd={args.fd}":
            kb = pmc.get("kernels", {})
            traffic = kb.get(tr_kernel, {}).get("hbm_bytes")
            dae_traffic = kb.get("k_groups", {}).get("hbm_bytes")
        achieved = alg_bytes_jac / (tr_ms * 1e-3) / 1e9
        dae_tf = flops / (dae_ms * 1e-3) / 1e12
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "kernel": (f"{tr_kernel}: finite-difference quotients + Jacobian assembly per mesh interval"
                           + (" (group results combined in LDS)" if fused_iv else "")
                           + "; the longest kernel of eval_jac_g"),
                "kernel_ms": round(tr_ms, 5), "algorithmic_bytes": alg_bytes_jac,
                "traffic_source": pmc_src if traffic is not None else None,
                "dae_stage": {"kernel": "k_groups" if fused_iv else "k_groups + k_combine",
                              "bound": "mfma", "unit": "TFLOP/s",
                              "note": "FP64 VALU; MI355X FP64 vector peak = FP64 matrix peak",
                              "achieved": round(dae_tf, 4), "peak": FP64_PEAK_TFLOPS,
                              "frac": round(dae_tf / FP64_PEAK_TFLOPS, 5), "ms": round(dae_ms, 5),
                              "algorithmic_flops_per_launch": flops, "dae_evals_per_launch": n_dae,
                              "flops_per_dae": f_dae, "executed_flops_per_launch": float(work[0]),
                              "executed_TFLOPs": round(float(work[0]) / (dae_ms * 1e-3) / 1e12, 4),
                              "traffic": dae_traffic},
                "backend": be_name, "model_hash": f"0x{mhash:016x}",
                "instrumented_ms_per_step": round(1e3 * inst_elapsed / args.steps, 4)}
        if rec["g"]:
            Gt = np.array(rec["g"])
            roof["eval_g_stage_ms"] = [round(float(np.median(Gt[:, i])), 5) for i in range(4)]
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(rep, st.solver.options(), x, args.cpu_baseline_seconds)
        line = {
            "metric": "NLP eval_g+eval_jac_g calls/sec (gait10dof18musc)",
            "value": round(value, 3), "unit": "calls/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "strong" if mesh else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "MocoTrack gait10dof18musc DGF rigid tendon (configs[2])",
                       "mesh_intervals": N, "grid_points": nlp.G, "n": nlp.n, "m": nlp.m,
                       "nnz_jac": nlp.nnz, "transcription": "hermite-simpson",
                       "fd": args.fd, "mode": args.mode,
                       "parallelism": (f"mesh-shard{world}+rccl-allgather" if mesh
                                       else f"replicas{world}" if world > 1 else "single"),
                       "iterate": "bounds-midpoint states, uniform random controls"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if other_elapsed:
            line[f"value_{other}"] = round((args.steps if mesh else args.steps * world) / other_elapsed, 3)
        if batch:
            line["batch"] = batch
        if sparse:
            line["sparsity_random"] = sparse
        if inverse:
            line["inverse_batch"] = inverse
        if cpu and cpu.get("value"):
            line["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def track_iterate(nlp, seed):
    """Bounds-midpoint states (where the muscle model is regular), uniform
    random controls within bounds."""
    x = nlp.random_iterate(np.random.default_rng(seed).uniform(-1, 1, nlp.n))
    xm = nlp.initial_guess_from_bounds()
    x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
    return x


def inverse_iterate(nlp, seed):
    """MocoInverse iterate: activations and normalized tendon forces in their
    physiological range, random excitations / reserves and tendon-force
    derivatives (a regular point of the DGF model)."""
    r = np.random.default_rng(seed)
    x = nlp.initial_guess_from_bounds()
    G, NS, NC = nlp.G, nlp.NS, nlp.NC
    S = x[2:2 + NS * G].reshape(G, NS)
    for i, n in enumerate(nlp.rep.state_names):
        S[:, i] = r.uniform(0.2, 0.6, G) if n.endswith("/activation") else r.uniform(0.05, 0.3, G)
    x[2 + NS * G:2 + (NS + NC) * G] = r.uniform(0.05, 0.4, NC * G)
    d0 = 2 + (NS + NC) * G
    x[d0:] = r.uniform(-0.5, 0.5, nlp.n - d0)
    return x


def batch_throughput(args, rep, st, local, rank, world, dev, torch, dist, B=None,
                     make_x=track_iterate):
    """B independent NLPs of the same workload per GPU (different iterates),
    each on its own context / HIP stream and driven by its own host thread
    (ctypes releases the GIL inside the C ABI calls): aggregate eval_g +
    eval_jac_g calls/s over all NLPs and ranks."""
    from concurrent.futures import ThreadPoolExecutor
    from mocohip.solver import HipNLP
    B = B or args.batch
    items = []
    for b in range(B):
        nlp = HipNLP(rep, st.solver.options())
        x = make_x(nlp, 1000 + rank * B + b)
        xd = torch.tensor(x, dtype=torch.float64, device=dev)
        gd = torch.zeros(nlp.m, dtype=torch.float64, device=dev)
        vd = torch.zeros(nlp.nnz, dtype=torch.float64, device=dev)
        items.append((nlp, xd, gd, vd))

    def run(item, k):
        nlp, xd, gd, vd = item
        for _ in range(k):
            if args.mode == "fused":
                nlp.eval_g_jac_g_device(xd.data_ptr(), gd.data_ptr(), vd.data_ptr())
            else:
                nlp.eval_g_device(xd.data_ptr(), gd.data_ptr())
                nlp.eval_jac_g_device(xd.data_ptr(), vd.data_ptr())

    with ThreadPoolExecutor(B) as pool:
        list(pool.map(lambda it: run(it, args.warmup), items))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        list(pool.map(lambda it: run(it, args.steps), items))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    be = items[0][0].backend()[0] if items else None
    for nlp, *_ in items:
        nlp.close()
    return {"nlps_per_gpu": B, "value": round(B * world * args.steps / el, 3), "unit": "calls/s",
            "mode": args.mode, "layout": "one context (HIP stream) + host thread per NLP",
            "backend": be}


def cpu_baseline(rep, opts, x, budget_s):
    """The CPU oracle (C restatement, OpenMP over grid points like CasADi's
    thread map) timed on this host, on a bounded sample of the workload."""
    from mocohip.solver import OracleNLP
    threads = min(16, os.cpu_count() or 1)
    ref = OracleNLP(rep, opts, threads=threads)
    ref.eval_g(x)
    calls = 0
    t0 = time.perf_counter()
    while True:
        ref.eval_g(x)
        ref.eval_jac_g(x)
        calls += 1
        el = time.perf_counter() - t0
        if el > budget_s or calls >= 5000:
            break
    ref.close()
    return {"value": round(calls / el, 4), "unit": "calls/s", "cores": threads, "kind": "port",
            "sample": f"{calls} eval_g+eval_jac_g calls of the same workload (N={opts.num_mesh_intervals}) "
                      f"in {el:.1f}s (oracle/oracle.c, OpenMP over grid points, {threads} threads)"}


if __name__ == "__main__":
    main()
