#!/usr/bin/env python
"""Benchmark: NLP eval_g + eval_jac_g calls/sec on MocoTrack gait10dof18musc
(DeGrooteFregly2016 muscles, rigid tendon, 18 excitations + 10 reserves,
Hermite-Simpson, forward finite differences), BASELINE.json configs[2].

One step = one eval_g and one eval_jac_g of the full NLP at an iterate
resident in HBM (device-pointer C ABI), results left in HBM.  With
--gpus N > 1 the mesh intervals are sharded over the ranks (one process per
GPU) and the g / Jacobian-value segments are all-gathered over RCCL so
every rank holds the whole g and J (what a host IPOPT needs): strong
scaling of the same NLP.

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

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 (vector = matrix) dense peak, spec
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--intervals", type=int, default=200)
    ap.add_argument("--fd", default="forward")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["separate", "fused"], default="separate",
                    help="separate: eval_g then eval_jac_g C-ABI calls; fused: one "
                         "mh_eval_g_jac_g call (IPOPT new_x=false pattern)")
    return ap.parse_args()


def flops_per_dae():
    path = os.path.join(ROOT, "tests", "golden", "flop_counts.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)


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
    if world != args.gpus:
        world = max(world, 1)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    N = args.intervals
    st = configs.gait10dof18musc(N, fd_scheme=args.fd)
    st.solver.device = local
    rep = st.problem.create_rep()
    ib, ie = interval_shard(N, rank, world)
    nlp = HipNLP(rep, st.solver.options(ib, ie))
    x = nlp.random_iterate(np.random.default_rng(0).uniform(-1, 1, nlp.n))
    # an iterate within bounds where the muscle model is regular: bounds
    # midpoint for states, random controls
    xm = nlp.initial_guess_from_bounds()
    x[2:2 + nlp.NS * nlp.G] = xm[2:2 + nlp.NS * nlp.G]
    dev = torch.device("cuda", local)
    xd = torch.tensor(x, dtype=torch.float64, device=dev)
    rpi = nlp.m // N
    nzi = nlp.nnz // N
    sg = ShardGather(N, rpi, nzi, world, dev)
    gseg, vseg = sg.gseg, sg.vseg

    fd_ms = []

    def step(record=False):
        if args.mode == "fused":
            nlp.eval_g_jac_g_device(xd.data_ptr(), gseg.data_ptr(), vseg.data_ptr())
        else:
            nlp.eval_g_device(xd.data_ptr(), gseg.data_ptr())
            nlp.eval_jac_g_device(xd.data_ptr(), vseg.data_ptr())
        if record:
            fd_ms.append(nlp.last_timings())
        if world > 1:
            sg.gather()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(record=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / args.steps
    value = args.steps / elapsed

    if rank == 0:
        T = np.array(fd_ms)            # [whole, dae+fd kernels, assembly] per jac call
        fd_kernel_ms = float(T[:, 1].mean())
        asm_ms = float(T[:, 2].mean())
        G_local = nlp.G if world == 1 else (2 * (ie - ib) + 1)
        ND = nlp.NS + nlp.NC + 2
        n_dae = G_local * (ND + 1) if args.fd != "central" else G_local * (2 * ND + 1)
        # (one lane per FD arm plus the unperturbed base lane per grid point)
        be_name, gen_flops, mhash = nlp.backend()
        fc = flops_per_dae() or {}
        key = "gait10dof18musc_rigid"
        # algorithmic FP64 ops per DAE evaluation of the algorithm the kernel
        # runs: the generator's emitted-op count for a generated back end,
        # the oracle's counted restatement for the generic interpreter.
        f_dae = gen_flops if gen_flops > 0 else fc.get(key, {}).get("flops_per_dae")
        if f_dae:
            flops = n_dae * f_dae
            achieved = flops / (fd_kernel_ms * 1e-3) / 1e12
        else:
            achieved = None
        roof = {"bound": "mfma", "kernel": "k_eval (one lane per DAE evaluation; FP64 VALU; "
                                           "MI355X FP64 vector peak = FP64 matrix peak)",
                "achieved": None if achieved is None else round(achieved, 4),
                "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": None if achieved is None else round(achieved / FP64_PEAK_TFLOPS, 5),
                "traffic": None, "backend": be_name, "model_hash": f"0x{mhash:016x}",
                "dae_evals_per_launch": n_dae, "flops_per_dae": f_dae,
                "oracle_flops_per_dae": fc.get(key, {}).get("flops_per_dae"),
                "kernel_ms": round(fd_kernel_ms, 5),
                "assembly": {"kernel": "k_assemble", "ms": round(asm_ms, 5),
                             "achieved_GBs": round(8 * (nlp.n + (ie - ib) * nzi) / (asm_ms * 1e-3) / 1e9, 2),
                             "peak_GBs": HBM_PEAK_GBS}}
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(rep, st.solver.options(), x, args.cpu_baseline_seconds)
        line = {
            "metric": "NLP eval_g+eval_jac_g calls/sec (gait10dof18musc)",
            "value": round(value, 3), "unit": "calls/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "MocoTrack gait10dof18musc DGF rigid tendon (configs[2])",
                       "mesh_intervals": N, "grid_points": nlp.G, "n": nlp.n, "m": nlp.m,
                       "nnz_jac": nlp.nnz, "transcription": "hermite-simpson",
                       "fd": args.fd, "parallelism": f"mesh-shard{world}", "mode": args.mode,
                       "iterate": "bounds-midpoint states, uniform random controls (seed 0)"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if cpu and cpu.get("value"):
            line["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


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
            "sample": f"{calls} eval_g+eval_jac_g calls of the same workload in {el:.1f}s "
                      f"(oracle/oracle.c, OpenMP over grid points)"}


if __name__ == "__main__":
    main()
