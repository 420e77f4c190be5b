#!/usr/bin/env python
"""Benchmark: NLP eval_g + eval_jac_g calls/sec on MocoTrack gait10dof18musc
(DeGrooteFregly2016 muscles, rigid tendon, 18 excitations + 10 reserves,
GRF external loads, Hermite-Simpson, forward finite differences),
BASELINE.json configs[2] (N=200 mesh intervals).

One step = one eval_g and one eval_jac_g of the full NLP at an iterate
resident in HBM (device-pointer C ABI), results left in HBM.  The calls are
asynchronous (mh_set_async) on torch's current stream: each returns once its
kernels are enqueued and the timed region ends with torch.cuda.synchronize()
(barrier + synchronize on both sides).  Beside the headline:
  value_fused     the IPOPT eval_g(new_x) -> eval_jac_g(!new_x) pair as one
                  mh_eval_g_jac_g_device call (identical results);
  value_blocking  every call synchronizes before returning (what a blocking
                  host caller sees per call, device-resident data);
  n400            the same workload at N=400 (the north-star size);
  host_inclusive  host-pointer calls on page-locked buffers: x host->device,
                  g and the Jacobian device->host every call (what a host
                  IPOPT sees), at N=200 and N=400;
  batch / inverse_batch / sparsity_random  concurrent independent NLPs and
                  the detected-sparsity variants (configs[4] layout);
  roofline        the longest kernel of eval_jac_g, timed with HIP events
                  on the context stream in a second, instrumented pass;
  cpu_baseline    the CPU oracle (kind "port"), 1 thread and all the box's
                  cores, on a bounded sample of the same workload.

--gpus N > 1 (one process per GPU, torch.distributed.run):
  --multi mesh (default): the north star's layout -- ONE NLP (the N = 1
      workload) for one optimizer, its mesh intervals sharded over the
      ranks; value = calls/s of the whole data path per call: x broadcast
      from rank 0 over RCCL, every rank's shard evaluation, the other ranks'
      g / Jacobian slices received into rank 0's HBM over xGMI
      (mocohip.distributed.SliceGather), so g and J are complete in rank 0's
      HBM after every call -- the same quantity as the N = 1 headline (where
      nothing moves); "scaling": "strong", with "one_gpu" (rank 0 alone on
      the whole NLP, the N = 1 quantity) and their ratio "strong_scaling".
      Labelled beside it: "device_resident" (each rank only evaluates its
      shard, no broadcast / gather: an upper bound), "host_inclusive"
      (HostGather: x from and g / J into page-locked host memory over each
      rank's PCIe link), "replicas" (every rank its own NLP, weak scaling),
      "inverse_solve_sweep" (configs[4]: 64 MocoInverse solves distributed
      over the ranks) and "sharded_solve" (configs[2] solved by one
      optimizer over all ranks).  The secondary legs run after the headline
      under try/except and a watchdog (--leg-timeout): a failure lands in
      "errors", never loses the line.
  --multi replicas: every rank evaluates its own NLP (independent trials,
      the configs[4] batch layout), no collective on the data path ->
      "scaling": "weak"; the mesh measurements ride along under "mesh".
--shard-model (one GPU): the per-shard times and gather volumes of
  DESIGN.md's multi-GPU model.

Prints one JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time
import uuid

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))

# One GPU (no torch.distributed launcher): this process and the configs[4]
# sweep's eight solver processes it starts run with 2 HIP hardware queues
# each, read by the HIP runtime at its start (before anything below touches
# the GPU).  The sweep's small, latency-bound kernels overlap on the GPU only
# while every process's queues are mapped together (0.72 -> 0.69 s for the
# sweep with this process at 2 instead of 4; the workers' own setting:
# mocohip.batchsolve); the single-stream lines are unaffected (21.3 k vs
# 21.5 k calls/s).  The multi-GPU runs keep the environment's setting.
if int(os.environ.get("WORLD_SIZE", "1")) == 1:
    os.environ["GPU_MAX_HW_QUEUES"] = "2"

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) dense peak, spec
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md (spec; 6.29 TB/s measured copy)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed wall time of headline calls before the warmup steps (GPU clock ramp)")
    ap.add_argument("--intervals", type=int, default=200)
    ap.add_argument("--fd", default="forward")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=8.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["separate", "fused"], default="separate",
                    help="separate: eval_g then eval_jac_g C-ABI calls; fused: one "
                         "mh_eval_g_jac_g call (IPOPT new_x=false pattern)")
    ap.add_argument("--blocking", action="store_true",
                    help="every C-ABI call synchronizes before returning (default: asynchronous "
                         "device calls, synchronized at the end of the timed region)")
    ap.add_argument("--multi", choices=["replicas", "mesh"], default=None,
                    help="default: mesh when WORLD_SIZE > 1 (strong scaling of one NLP)")
    ap.add_argument("--single-mode", action="store_true",
                    help="measure only the headline (no secondary lines): for profiler runs, so "
                         "that every launch of a kernel has the same shape")
    ap.add_argument("--config3", type=int, default=400,
                    help="mesh intervals of the configs[3] Rajagopal 80-muscle line (0: skip)")
    ap.add_argument("--config", choices=["gait", "rajagopal80"], default="gait",
                    help="--multi mesh workload: configs[2] gait10dof18musc or configs[3] Rajagopal")
    ap.add_argument("--inverse-batch", type=int, default=8)
    ap.add_argument("--solve-batch", type=int, default=8,
                    help="configs[4] MocoInverse solves run together on this GPU (0: skip)")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--sweep", type=int, default=64,
                    help="--multi mesh: configs[4]'s MocoInverse solves distributed over the ranks (0: skip)")
    ap.add_argument("--solve-intervals", type=int, default=200,
                    help="--multi mesh, N > 1: mesh intervals of the configs[2] solve sharded over the ranks "
                         "(0: skip)")
    ap.add_argument("--leg-timeout", type=float, default=300.0,
                    help="--gpus N > 1: seconds the secondary legs (replicas, sweep, sharded solve) may take "
                         "after the headline before the line is printed without them")
    ap.add_argument("--shard-model", action="store_true",
                    help="one GPU: time rank 0's and the last rank's mesh shard of the headline NLP for "
                         "W = 1, 2, 4, 8 (device-resident), the inputs of DESIGN.md's multi-GPU model")
    ap.add_argument("--batch-only", action="store_true",
                    help="print only the batch line (A/B of queue / launch settings)")
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


class Ctx:
    """torch / torch.distributed plumbing of one rank."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        if self.world > 1:
            import datetime
            dist.init_process_group("nccl", device_id=self.dev, timeout=datetime.timedelta(seconds=600))
        # a dedicated (non-null) stream made current: the contexts, torch's
        # tensors and the host copies all order on it (torch's default stream
        # has handle 0, which mh_set_stream reads as "the context's own
        # stream" -- a non-blocking stream that would not order with it)
        self.s = torch.cuda.Stream(device=self.dev)
        torch.cuda.set_stream(self.s)

    def stream(self):
        return self.torch.cuda.current_stream().cuda_stream

    def timed(self, step, k):
        """K steps bracketed by barrier + synchronize; max over ranks."""
        torch, dist = self.torch, self.dist
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el


def make_nlp(cx, st, ib=0, ie=0, blocking=False):
    from mocohip.solver import HipNLP
    st.solver.device = cx.local
    rep = st.problem.create_rep()
    nlp = HipNLP(rep, st.solver.options(ib, ie))
    nlp.set_stream(cx.stream())
    nlp.set_async(not blocking)
    return nlp


def device_steps(cx, nlp, x):
    """(step_separate, step_fused) on device buffers."""
    torch = cx.torch
    xd = torch.tensor(x, dtype=torch.float64, device=cx.dev)
    gd = torch.zeros(max(nlp.row_end - nlp.row_begin, 1), dtype=torch.float64, device=cx.dev)
    vd = torch.zeros(max(nlp.nnz_end - nlp.nnz_begin, 1), dtype=torch.float64, device=cx.dev)
    xp, gp, vp = xd.data_ptr(), gd.data_ptr(), vd.data_ptr()

    def separate():
        nlp.eval_g_device(xp, gp)
        nlp.eval_jac_g_device(xp, vp)

    def fused():
        nlp.eval_g_jac_g_device(xp, gp, vp)
    return separate, fused, (xd, gd, vd)


def settle(cx, step, seconds):
    """Untimed calls of the headline step for a fixed wall time before its
    warmup: the GPU's clocks ramp over the first milliseconds of a burst
    (DESIGN.md section 5), which a short warmup (the driver's 5 steps) does
    not cover.  Reported in the line as "settle_s"; nothing of it is timed."""
    if seconds <= 0:
        return 0.0
    torch = cx.torch
    sync = getattr(cx, "sync", None) or torch.cuda.synchronize
    t0 = time.perf_counter()
    # with several ranks the steps hold collectives: every rank runs the same
    # number of chunks, rank 0's clock deciding (one broadcast per chunk)
    flag = torch.ones(1, dtype=torch.int32, device=cx.dev) if cx.world > 1 else None
    while True:
        for _ in range(50):
            step()
        sync()
        more = time.perf_counter() - t0 < seconds
        if flag is not None:
            flag.fill_(1 if more else 0)
            cx.dist.broadcast(flag, src=0)
            more = bool(flag.item())
        if not more:
            break
    return round(time.perf_counter() - t0, 3)


def measure(cx, step, args, k=None, w=None):
    for _ in range(args.warmup if w is None else w):
        step()
    k = args.steps if k is None else k
    return k, cx.timed(step, k)


def host_inclusive(cx, nlp, x, args):
    """eval_g + eval_jac_g through the host-pointer entries on page-locked
    buffers: x to the device, g and all Jacobian values back, every call."""
    torch = cx.torch
    xh = torch.from_numpy(np.ascontiguousarray(x)).pin_memory()
    gh = torch.empty(nlp.m, dtype=torch.float64).pin_memory()
    vh = torch.empty(nlp.nnz, dtype=torch.float64).pin_memory()
    xn, gn, vn = xh.numpy(), gh.numpy(), vh.numpy()
    from mocohip import abi
    lib, ctx = nlp.lib, nlp.ctx
    xp, gp, vp = abi.dptr(xn), abi.dptr(gn), abi.dptr(vn)

    def step():
        lib.mh_eval_g(ctx, xp, 1, gp)
        lib.mh_eval_jac_g(ctx, xp, 0, vp)
    k = max(20, args.steps // 4)
    k, el = measure(cx, step, args, k=k, w=5)
    return {"value": round(k / el, 3), "unit": "calls/s", "ms_per_step": round(1e3 * el / k, 4),
            "bytes_to_host_per_step": 8 * (nlp.m + nlp.nnz),
            "note": "mh_eval_g + mh_eval_jac_g on page-locked host buffers (x in, g and J out over "
                    "PCIe every call); never the headline"}


def roofline(cx, nlp, steps, args, mode):
    """Instrumented pass: HIP events between the stages on the context
    stream (mh_set_timing) -> per-launch kernel times of eval_jac_g."""
    nlp.set_timing(True)
    rec = {"g": [], "jac": []}

    def step():
        if mode == "fused":
            steps[1]()
            rec["jac"].append(nlp.last_timings())
        else:
            nlp.eval_g_device(*steps[2])
            rec["g"].append(nlp.last_timings())
            nlp.eval_jac_g_device(*steps[3])
            rec["jac"].append(nlp.last_timings())
    _, el = measure(cx, step, args, w=2)
    nlp.set_timing(False)
    J = np.array(rec["jac"])          # [whole, DAE stage, transcription stage, k_groups] ms
    ev_dae_ms, ev_tr_ms = float(np.median(J[:, 1])), float(np.median(J[:, 2]))
    # per-launch kernel durations: the stages of eval_jac_g in call order,
    # a HIP event after each on the context stream (the queue ahead of the
    # GPU; mh_debug_time_stages) -- the figure a rocprofv3 kernel trace of
    # the same launches gives, plus the inter-kernel gap
    dae_ms, tr_ms = nlp.time_stages(steps[3][0], kind=1, reps=max(50, args.steps))
    G, ND = nlp.G, nlp.NS + nlp.NC + 2
    n_dae = G * (ND + 1) if args.fd != "central" else G * (2 * ND + 1)
    be_name, f_dae, mhash = nlp.backend()
    work = nlp.work()                     # executed FP64 ops of the (pruned) task kernels
    alg_flops = n_dae * f_dae             # a full DAE per FD lane (the algorithm's work)
    alg_bytes = 8 * (nlp.n + nlp.nnz)     # x in, Jacobian values out
    fused_iv = nlp.uses_interval_kernel()
    tr_kernel = "k_interval" if fused_iv else "k_transcribe"
    pmc, pmc_src = latest_pmc()
    traffic = dae_traffic = None
    if pmc and pmc.get("workload") == f"N={args.intervals},fd={args.fd}":
        kb = pmc.get("kernels", {})
        traffic = kb.get(tr_kernel, {}).get("hbm_bytes")
        dae_traffic = kb.get("k_groups", {}).get("hbm_bytes")
    gbs = alg_bytes / (tr_ms * 1e-3) / 1e9
    tf_exec = float(work[0]) / (dae_ms * 1e-3) / 1e12
    hbm = {"kernel": f"{tr_kernel}: finite-difference quotients + Jacobian assembly per mesh interval"
                     + (" (group results combined in LDS)" if fused_iv else ""),
           "bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel_ms": round(tr_ms, 5),
           "algorithmic_bytes": alg_bytes,
           "traffic_source": pmc_src if traffic is not None else None}
    fp64 = {"kernel": "k_groups" if fused_iv else "k_groups + k_combine",
            "bound": "mfma", "unit": "TFLOP/s",
            "note": "FP64 VALU (MI355X FP64 vector peak = FP64 matrix peak); achieved = FP64 ops the "
                    "pruned task kernels EXECUTE per launch / kernel time",
            "achieved": round(tf_exec, 4), "peak": FP64_PEAK_TFLOPS,
            "frac": round(tf_exec / FP64_PEAK_TFLOPS, 5), "kernel_ms": round(dae_ms, 5),
            "executed_flops_per_launch": float(work[0]),
            "algorithmic_flops_per_launch": alg_flops,
            "algorithmic_note": f"{n_dae} DAE evaluations x {f_dae:.0f} ops (one full DAE per FD lane)",
            "traffic": dae_traffic}
    # the dominant (longest) kernel of eval_jac_g is the headline roofline
    main, other = (hbm, fp64) if tr_ms >= dae_ms else (fp64, hbm)
    roof = dict(main)
    roof["other_kernel"] = other
    roof.update({"backend": be_name, "model_hash": f"0x{mhash:016x}",
                 "backend_flags": nlp.backend_flags(),
                 "timing": "mh_debug_time_stages: both stages in call order, a HIP event after each",
                 "instrumented_ms_per_step": round(1e3 * el / args.steps, 4),
                 "in_call_stage_ms": [round(ev_dae_ms, 5), round(ev_tr_ms, 5)]})
    if rec["g"]:
        Gt = np.array(rec["g"])
        # [whole call, DAE stage, transcription stage, k_groups] as recorded by
        # events INSIDE each eval_g call (host launch latency included)
        roof["eval_g_stage_ms"] = [round(float(np.median(Gt[:, i])), 5) for i in range(4)]
        # eval_g's two kernels timed the way the roofline's are (in call
        # order, an event after each; the kernel-trace figures)
        gd_ms, gi_ms = nlp.time_stages(steps[2][0], kind=0, reps=max(50, args.steps))
        roof["eval_g_kernels_ms"] = {"k_groups": round(gd_ms, 5), "k_interval_256": round(gi_ms, 5),
                                     "sum": round(gd_ms + gi_ms, 5)}
    return roof


def batched_throughput(cx, st_fn, make_x, args, B):
    """B independent NLPs of the same workload per GPU (different iterates)
    evaluated through one mh_batch: one k_groups and one k_interval launch
    per stage for all B, on one stream, driven by one host thread."""
    from mocohip.solver import HipBatch, HipNLP
    torch = cx.torch
    nlps, xs, gs, vs = [], [], [], []
    for b in range(B):
        st = st_fn()
        st.solver.device = cx.local
        nlp = HipNLP(st.problem.create_rep(), st.solver.options())
        nlp.set_stream(cx.stream())
        nlp.set_async(not args.blocking)
        nlps.append(nlp)
        xs.append(torch.tensor(make_x(nlp, 1000 + cx.rank * B + b), dtype=torch.float64, device=cx.dev))
        gs.append(torch.zeros(nlp.m, dtype=torch.float64, device=cx.dev))
        vs.append(torch.zeros(nlp.nnz, dtype=torch.float64, device=cx.dev))
    bt = HipBatch(nlps)
    xp, gp, vp = [t.data_ptr() for t in xs], [t.data_ptr() for t in gs], [t.data_ptr() for t in vs]

    def step():
        if args.mode == "fused":
            bt.eval_g_jac_g_device(xp, gp, vp)
        else:
            bt.eval_g_device(xp, gp)
            bt.eval_jac_g_device(xp, vp)
    k, el = measure(cx, step, args)
    out = {"nlps_per_gpu": B, "value": round(B * cx.world * k / el, 3), "unit": "calls/s",
           "mode": args.mode, "layout": "mh_batch: one launch per kernel for all B NLPs, one stream",
           "backend": nlps[0].backend()[0], "nnz_jac": nlps[0].nnz, "m": nlps[0].m}
    if args.mode == "separate":
        def fstep():
            bt.eval_g_jac_g_device(xp, gp, vp)
        kf, ef = measure(cx, fstep, args)
        out["value_fused"] = round(B * cx.world * kf / ef, 3)
    bt.close()
    for nlp in nlps:
        nlp.close()
    return out


def batch_throughput(cx, st_fn, make_x, args, B):
    """B independent NLPs of the same workload per GPU (different iterates),
    each on its own HIP stream and driven by its own host thread (ctypes
    releases the GIL inside the C ABI calls): aggregate eval_g + eval_jac_g
    calls/s over all NLPs and ranks.  Asynchronous calls, each thread
    synchronizing its stream after its K steps."""
    from concurrent.futures import ThreadPoolExecutor
    from mocohip.solver import HipNLP
    torch = cx.torch
    items = []
    for b in range(B):
        st = st_fn()
        st.solver.device = cx.local
        nlp = HipNLP(st.problem.create_rep(), st.solver.options())
        s = torch.cuda.Stream(device=cx.dev)
        nlp.set_stream(s.cuda_stream)
        nlp.set_async(not args.blocking)
        x = make_x(nlp, 1000 + cx.rank * B + b)
        xd = torch.tensor(x, dtype=torch.float64, device=cx.dev)
        gd = torch.zeros(nlp.m, dtype=torch.float64, device=cx.dev)
        vd = torch.zeros(nlp.nnz, dtype=torch.float64, device=cx.dev)
        items.append((nlp, s, xd, gd, vd))

    def run(item, k):
        nlp, s, xd, gd, vd = item
        for _ in range(k):
            if args.mode == "fused":
                nlp.eval_g_jac_g_device(xd.data_ptr(), gd.data_ptr(), vd.data_ptr())
            else:
                nlp.eval_g_device(xd.data_ptr(), gd.data_ptr())
                nlp.eval_jac_g_device(xd.data_ptr(), vd.data_ptr())
        nlp.synchronize()

    with ThreadPoolExecutor(B) as pool:
        list(pool.map(lambda it: run(it, args.warmup), items))
        el = cx.timed(lambda: list(pool.map(lambda it: run(it, args.steps), items)), 1)
    be = items[0][0].backend()[0] if items else None
    out = {"nlps_per_gpu": B, "value": round(B * cx.world * args.steps / el, 3), "unit": "calls/s",
           "mode": args.mode, "layout": "one context (HIP stream) + host thread per NLP",
           "backend": be, "nnz_jac": items[0][0].nnz, "m": items[0][0].m}
    for nlp, *_ in items:
        nlp.close()
    return out


def cpu_baseline(rep, opts, x, budget_s, threads):
    """The CPU oracle (C restatement, OpenMP over grid points like CasADi's
    thread map) timed on this host, on a bounded sample of the workload."""
    from mocohip.solver import OracleNLP
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
                      f"in {el:.1f}s (oracle/oracle.c, OpenMP over grid points, {threads} thread"
                      f"{'s' if threads > 1 else ''}; host nproc {os.cpu_count()}, box share "
                      f"{os.environ.get('OMP_NUM_THREADS', '?')} threads)"}


def config3_line(cx, args):
    """configs[3]: the Rajagopal 80-muscle NLP (configs.rajagopal80: 18
    coordinates, 80 DGF muscles, patellofemoral couplers with derivatives and
    velocity-correction slacks, explicit) at N = --config3 on this GPU:
    eval_g + eval_jac_g calls/s on device pointers, the per-launch times of
    its two eval_jac_g stages (the DAE stage of the selected back end, then
    the transcription), and a bounded CPU-oracle sample."""
    from mocohip import configs
    st = configs.rajagopal80(args.config3, fd_scheme=args.fd)
    nlp = make_nlp(cx, st, blocking=args.blocking)
    x = track_iterate(nlp, cx.rank)
    sep, fused, (xd, gd, vd) = device_steps(cx, nlp, x)
    k, el = measure(cx, sep, args, k=max(5, args.steps // 100), w=3)
    dae_ms, tr_ms = nlp.time_stages(xd.data_ptr(), kind=1, reps=5)
    alg_bytes = 8 * (nlp.n + nlp.nnz)
    gbs = alg_bytes / (tr_ms * 1e-3) / 1e9
    # the DAE stage against the FP64 peak: the FP64 ops its (pruned) task
    # kernels execute per eval_jac_g / the stage's time
    work = nlp.work()
    tf_exec = float(work[0]) / (dae_ms * 1e-3) / 1e12 if dae_ms > 0 else 0.0
    out = {"value": round(k * cx.world / el, 3), "unit": "calls/s", "ms_per_step": round(1e3 * el / k, 4),
           "steps": k, "mesh_intervals": args.config3, "n": nlp.n, "m": nlp.m, "nnz_jac": nlp.nnz,
           "backend": nlp.backend()[0],
           "kernels_ms": {f"dae ({nlp.backend()[0]})": round(dae_ms, 4),
                          "transcription": round(tr_ms, 4)},
           "transcription_roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
                                      "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5),
                                      "algorithmic_bytes": alg_bytes},
           "dae_roofline": {"bound": "mfma", "unit": "TFLOP/s", "achieved": round(tf_exec, 4),
                            "peak": FP64_PEAK_TFLOPS, "frac": round(tf_exec / FP64_PEAK_TFLOPS, 5),
                            "executed_flops_per_launch": float(work[0]), "kernel_ms": round(dae_ms, 4),
                            "note": "FP64 VALU (the FP64 vector peak = the FP64 matrix peak): the FP64 ops "
                                    "the task kernels execute per eval_jac_g (k_groups + the combine) / "
                                    "the DAE stage's time"},
           "workload": "configs[3] Rajagopal 80-muscle gait NLP (example3DWalking muscle-driven "
                       "problem, DGF rigid tendons, patellofemoral couplers), HS, forward FD, "
                       "block-dense callback sparsity, 1 GPU"}
    if cx.world == 1 and cx.rank == 0 and not args.no_cpu_baseline:
        box = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(nlp.rep, st.solver.options(), x, args.cpu_baseline_seconds,
                                           max(1, min(box, os.cpu_count() or 1)))
    nlp.close()
    return out


def solve_lines():
    """Wall-clock to a converged solve (the BASELINE metric's second half):
    MocoStudy.solve on the GPU path with the host interior-point solver
    (mocohip.ipm: Ipopt's algorithm with its limited-memory Hessian; Ipopt is
    absent here), at the reference's tolerances, for the reference's golden-
    solution problems and configs[4]'s NLP."""
    from mocohip import configs
    from mocohip.trajectory import MocoTrajectory
    golden = os.path.join(ROOT, "tests", "golden")

    def rms_vs(sol, rep, fname):
        d = np.load(os.path.join(golden, fname))
        labels = [str(l) for l in d["labels"]]
        data = d["data"]
        col = {l: i for i, l in enumerate(labels)}
        sn, cn = list(rep.state_names), list(rep.control_names)
        g = MocoTrajectory(data[:, 0], sn, cn, states=data[:, [col[n] for n in sn]],
                           controls=data[:, [col[n] for n in cn]])
        m = MocoTrajectory(sol.time, sn, cn, states=sol.states, controls=sol.controls)
        return (round(g.compare_continuous_variables_rms(m, states=["none"]), 5),
                round(g.compare_continuous_variables_rms(m, controls=["none"]), 5))
    out = {}
    problems = (
        # BASELINE configs[2] itself: the muscle-driven MocoTrack the headline
        # throughput is quoted on, solved with MocoTrack's settings
        # (MocoTrack.cpp:105-121: tolerances 1e-2, forward FD, bounds guess)
        ("gait10dof18musc_track_N200", lambda: configs.gait10dof18musc_track(200, muscles=True), None,
         "configs[2]: MocoTrack gait10dof18musc, 18 DGF muscles + reserves, N=200 (testMocoTrack.cpp:46-68 "
         "with ModOpReplaceMusclesWithDeGrooteFregly2016)"),
        ("gait10dof18musc_track_N400", lambda: configs.gait10dof18musc_track(400, muscles=True), None,
         "configs[2] at the north-star size N=400"),
        ("moco_inverse_rajagopal18_N11", lambda: configs.rajagopal18_inverse(),
         "std_testMocoInverse_subject_18musc_solution.npz",
         "testMocoInverse.cpp:118-147; reference file: objective 1.087741, 52 Ipopt iterations, 54.5 s"),
        ("moco_track_gait10dof18musc_N65", lambda: configs.gait10dof18musc_track(),
         "std_testMocoTrackGait10dof18musc_solution.npz", "testMocoTrack.cpp:46-68 (tolerance 1e-2)"),
        ("moco_inverse_gait10dof18musc_N125", lambda: configs.gait10dof18musc_inverse(125), None,
         "configs[4]'s NLP (one solve of the batch)"),
        ("sliding_mass_interface", configs.sliding_mass_interface, None,
         "testMocoInterface.cpp:1701-1742"),
    )
    for name, mk, gold, ref in problems:
        st = mk()
        rep = st.problem.create_rep()
        sol = st.solve()
        r = sol.stats
        ev, la = r.timings.get("evaluations_s", 0.0), r.timings.get("linear_algebra_s", 0.0)
        line = {"success": r.success, "wall_clock_s": round(r.duration, 3), "iterations": r.iterations,
                "objective": r.objective, "status": r.status, "evaluations": r.evaluations,
                "seconds_in_evaluations": round(ev, 3), "seconds_in_kkt": round(la, 3),
                "seconds_other_host": round(r.duration - ev - la, 3),
                "evaluation_share": round(ev / r.duration, 4) if r.duration > 0 else None,
                "linear_solver": r.timings.get("linear_solver"),
                "n": int(len(r.x)), "optimizer": r.optimizer, "reference": ref,
                "note": "evaluations are the host-pointer C-ABI calls (x in, f / grad f / g out over PCIe); "
                        "with the device linear solver the Jacobian is evaluated into HBM and never copied"}
        if gold:
            line["rms_controls_states_vs_golden"] = rms_vs(sol, rep, gold)
        out[name] = line
    return out


def _mesh_build(args):
    from mocohip import configs
    N = args.intervals
    return ((lambda: configs.rajagopal80(N, fd_scheme=args.fd)) if args.config == "rajagopal80"
            else (lambda: configs.gait10dof18musc(N, fd_scheme=args.fd)))


def mesh_measure(cx, args):
    """--gpus N > 1, the headline: ONE NLP (the N = 1 headline's workload)
    sharded by mesh interval over the ranks, and per call the north star's
    data path for a single optimizer -- x broadcast from rank 0 over RCCL,
    each rank's shard evaluation, g and the Jacobian values reassembled in
    rank 0's HBM (mocohip.distributed.SliceGather: the other ranks' slices
    received point to point over xGMI into their offsets, rank 0's own
    written in place).  At N = 1 there is nothing to broadcast or gather and
    this is the single-GPU headline (g / J complete in the one GPU's HBM).
    Rank 0 checks the reassembled vectors against one unsharded evaluation
    (bit for bit).  Labelled beside it: "device_resident" (each rank only
    evaluates its shard: no x broadcast, no gather -- an upper bound) and
    "host_inclusive" (x from page-locked host memory over each rank's PCIe
    link, each slice DMA'd into one page-locked host buffer shared by the
    node's ranks, mocohip.distributed.HostGather)."""
    from mocohip.distributed import HostGather, SliceGather, interval_shard
    torch, dist = cx.torch, cx.dist
    N = args.intervals
    ib, ie = interval_shard(N, cx.rank, cx.world)
    build = _mesh_build(args)
    nlp = make_nlp(cx, build(), ib, ie, blocking=False)
    x = track_iterate(nlp, 0)
    xd = torch.tensor(x, dtype=torch.float64, device=cx.dev)
    sg = SliceGather(nlp.m, nlp.nnz, (nlp.row_begin, nlp.row_end, nlp.nnz_begin, nlp.nnz_end), dist, cx.dev)
    xp, gp, vp = xd.data_ptr(), sg.own_g.data_ptr(), sg.own_values.data_ptr()
    fused_mode = args.mode == "fused"

    def evaluate():
        if fused_mode:
            nlp.eval_g_jac_g_device(xp, gp, vp)
            return sg.post("g") + sg.post("values")
        nlp.eval_g_device(xp, gp)
        rg = sg.post("g")                      # g's fan-in overlaps the Jacobian's kernels
        nlp.eval_jac_g_device(xp, vp)
        return rg + sg.post("values")

    def step_reassembled():
        if cx.world > 1:
            dist.broadcast(xd, src=0)          # the iterate from rank 0 to every rank (RCCL)
        sg.wait(evaluate())                    # the current stream waits for the fan-in

    def step_device():                         # x resident in every rank's HBM, results left there
        if fused_mode:
            nlp.eval_g_jac_g_device(xp, gp, vp)
        else:
            nlp.eval_g_device(xp, gp)
            nlp.eval_jac_g_device(xp, vp)
    settled = settle(cx, step_reassembled, args.settle_s)
    k, el = measure(cx, step_reassembled, args)
    ok = None
    if cx.rank == 0:
        # the reassembled vectors against one unsharded evaluation
        torch.cuda.synchronize()
        full = make_nlp(cx, build(), blocking=True)
        ok = bool(np.array_equal(sg.g[:nlp.m].cpu().numpy(), full.eval_g(x))
                  and np.array_equal(sg.values[:nlp.nnz].cpu().numpy(), full.eval_jac_g(x)))
        full.close()
    if cx.world > 1:
        dist.barrier()
    kd, eld = measure(cx, step_device, args)
    # host-inclusive: HostGather over each rank's PCIe link
    tag = os.environ.get("MOCOHIP_BENCH_TAG") or f"mocohip_bench_{os.getppid()}"
    barrier = dist.barrier if cx.world > 1 else (lambda: None)
    hg = HostGather(tag, nlp.m, nlp.nnz, (nlp.row_begin, nlp.row_end), (nlp.nnz_begin, nlp.nnz_end),
                    cx.rank, barrier, pin=True, device=cx.local)
    stream = cx.stream()
    xh = torch.from_numpy(np.ascontiguousarray(x)).pin_memory()   # IPOPT's iterate on the host

    def step_host():
        xd.copy_(xh, non_blocking=True)        # the iterate from host memory over the rank's PCIe link
        step_device()
        hg.copy_from_device_async(gp, vp, stream)
        torch.cuda.current_stream().synchronize()
        if cx.world > 1:
            dist.barrier()                     # every slice has landed on the IPOPT host
    kh, elh = measure(cx, step_host, args, k=max(50, args.steps // 4), w=max(10, args.warmup // 10))
    hok = None
    if cx.rank == 0:
        full = make_nlp(cx, build(), blocking=True)
        hok = bool(np.array_equal(hg.full_g(), full.eval_g(x)) and np.array_equal(hg.full_values(), full.eval_jac_g(x)))
        full.close()
    barrier()
    hg.close(unlink=cx.rank == 0)
    out = {"value": round(k / el, 3), "unit": "calls/s", "steps": k, "settle_s": settled,
           "ms_per_step": round(1e3 * el / k, 5),
           "scaling": "strong", "mesh_intervals": N, "n": nlp.n, "m": nlp.m, "nnz_jac": nlp.nnz,
           "reassembly_bit_exact": ok,
           "bytes_gathered_per_call": sg.bytes_received(),
           "parallelism": f"mesh-shard{cx.world}: rank r evaluates intervals [N r / W, N (r + 1) / W); x broadcast "
                          "from rank 0 (RCCL), every other rank's g / J slice received point to point (RCCL over "
                          "xGMI, one grouped batch per vector) into rank 0's HBM",
           "device_resident": {"value": round(kd / eld, 3), "unit": "calls/s", "steps": kd,
                               "ms_per_step": round(1e3 * eld / kd, 5),
                               "note": "upper bound, not a deliverable rate: x already in every rank's HBM, each "
                                       "rank's g / J slice left in its own HBM (no broadcast, no gather)"},
           "host_inclusive": {"value": round(kh / elh, 3), "unit": "calls/s", "steps": kh,
                              "ms_per_step": round(1e3 * elh / kh, 5), "reassembly_bit_exact": hok,
                              "note": "x from page-locked host memory over each rank's PCIe link, each rank's g / J "
                                      "slice DMA'd into one page-locked host buffer shared by the node's ranks "
                                      "(HostGather), a barrier"}}
    nlp.close()
    return out


def one_gpu_reference(cx, args, build):
    """The strong-scaling denominator inside a multi-rank run: rank 0 alone
    evaluates the WHOLE NLP with x resident and g / J left in its HBM (the
    N = 1 headline's quantity) while the other ranks wait; None elsewhere."""
    out = None
    if cx.rank == 0:
        nlp = make_nlp(cx, build(), blocking=False)
        sep, fused, _ = device_steps(cx, nlp, track_iterate(nlp, 0))
        step = fused if args.mode == "fused" else sep
        for _ in range(args.warmup):
            step()
        cx.torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        cx.torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out = {"value": round(args.steps / el, 3), "unit": "calls/s", "steps": args.steps,
               "ms_per_step": round(1e3 * el / args.steps, 5),
               "note": "rank 0 alone, the whole NLP, x resident and g / J left in its HBM (the N = 1 "
                       "headline's quantity): the denominator of strong_scaling"}
        nlp.close()
    if cx.world > 1:
        cx.dist.barrier()
    return out


def sweep_distributed(cx, args):
    """configs[4] as BASELINE names it: 64 MocoInverse solves over the
    node's ranks -- rank r solves every W-th subject on its own GPU
    (mocohip.batchsolve.solve_sweep, rounds of <= 8 solver processes per
    GPU, at most 16 GPU processes on the node), no collective on the data path; the counts and the wall clock
    (max over ranks) reduced at the end.  A rank whose share fails reports
    zero solves and its error; every rank still reaches the reductions."""
    from mocohip import batchsolve
    torch, dist = cx.torch, cx.dist
    if cx.world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    err = None
    try:
        # at most 16 processes on the node's GPUs at once (the ranks and their
        # solver processes): 7 / 3 / 1 solvers per rank at W = 2 / 4 / 8
        conc = max(1, min(8, 16 // cx.world - 1))
        r = batchsolve.solve_sweep(args.sweep, 125, rank=cx.rank, world=cx.world, device=cx.local,
                                   max_concurrent=conc)
    except Exception as e:   # noqa: BLE001 -- reported in the line, never fatal to it
        r = {"solves": 0, "succeeded": 0, "wall_clock_s": 0.0, "rounds": 0, "mean_iterations": None}
        err = f"rank {cx.rank}: {type(e).__name__}: {e}"
    el = time.perf_counter() - t0
    t = torch.tensor([r["solves"], r["succeeded"], 1.0 if err else 0.0], dtype=torch.float64, device=cx.dev)
    w = torch.tensor([el, r["wall_clock_s"]], dtype=torch.float64, device=cx.dev)
    if cx.world > 1:
        dist.all_reduce(t)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
    solves, ok, failed = int(t[0].item()), int(t[1].item()), int(t[2].item())
    wall = float(w[1].item())
    out = {"solves": solves, "succeeded": ok, "ranks": cx.world, "solves_per_rank": r["solves"],
           "rounds_per_rank": r["rounds"], "wall_clock_s": round(wall, 3),
           "wall_clock_incl_setup_s": round(float(w[0].item()), 3),
           "solves_per_minute": round(60.0 * solves / wall, 2) if wall > 0 else None,
           "mean_iterations_rank0": r["mean_iterations"],
           "workload": "configs[4]: 64 MocoInverse gait10dof18musc N=125 solves (scaled subjects), "
                       "rank r solves subjects r, r+W, ... on its own GPU, <= 8 solver processes at once "
                       "(<= 16 GPU processes on the node: ranks + solvers)"}
    if failed:
        out["ranks_failed"] = failed
    if err:
        out["error"] = err
    return out


def sharded_solve(cx, args):
    """configs[2] solved by ONE optimizer whose NLP spans the ranks
    (mocohip.distributed.ShardedNLP): rank 0 runs the interior-point method
    with its Newton systems on its GPU over the whole Jacobian
    (ShardedDeviceKKT), every rank evaluates its mesh intervals, the other
    ranks' Jacobian slices arrive in rank 0's HBM over RCCL (send / recv,
    xGMI).  Beside it the same solve on rank 0's GPU alone.  Rank 0 releases
    the serving ranks whatever happens to its solve (close() in finally);
    a serving rank whose evaluation fails answers with NaN so that the
    protocol -- and the job -- keeps going, and the failure is reported."""
    from mocohip import configs
    from mocohip.distributed import ShardedNLP, interval_shard
    from mocohip.solver import HipNLP
    N = args.solve_intervals
    st = configs.gait10dof18musc_track(N, muscles=True)
    st.solver.device = cx.local
    rep = st.problem.create_rep()
    ib, ie = interval_shard(N, cx.rank, cx.world)
    snlp = ShardedNLP(HipNLP(rep, st.solver.options(ib, ie)), cx.dist, transport="device", device=cx.local)
    out = None
    if cx.rank == 0:
        try:
            sol = st.solve(nlp=snlp, linear_solver="device")
        finally:
            snlp.close()
        r = sol.stats
        full = HipNLP(rep, st.solver.options())
        ref = st.solve(nlp=full, linear_solver="device").stats
        full.close()
        out = {"success": bool(r.success), "wall_clock_s": round(r.duration, 3), "iterations": r.iterations,
               "objective": r.objective, "ranks": cx.world,
               "seconds_in_kkt": round(r.timings.get("linear_algebra_s", 0.0), 3),
               "one_gpu": {"success": bool(ref.success), "wall_clock_s": round(ref.duration, 3),
                           "iterations": ref.iterations, "objective": ref.objective},
               "workload": f"configs[2] MocoTrack gait10dof18musc, 18 DGF muscles, N={N}, one solve whose "
                           f"mesh intervals are sharded over {cx.world} GPUs (Jacobian slices to rank 0's "
                           "HBM over RCCL, Newton systems on rank 0's GPU)"}
    else:
        snlp.serve()
        if snlp.error:
            out = {"error": snlp.error}
    return out


def shard_model(cx, args):
    """The inputs of DESIGN.md's multi-GPU model, measured on ONE GPU: for
    W = 1, 2, 4, 8 the mesh shards of the headline NLP that rank 0 (the
    endpoint head) and rank W - 1 (the tail) would own, each timed alone,
    device-resident (K separate eval_g + eval_jac_g steps), and the bytes
    rank 0 receives per call when the other W - 1 slices are gathered into its
    HBM.  Predicted per-call time at W GPUs: max over the two shards + the
    x broadcast + the slowest peer's slice over one xGMI link (each peer
    sends over its own link), printed for two link rates (the 153 GB/s per
    link figure of the task statement, and a 50 GB/s achieved P2P rate)."""
    from mocohip.distributed import interval_shard
    N = args.intervals
    build = _mesh_build(args)
    full = make_nlp(cx, build(), blocking=False)
    m, nnz, n = full.m, full.nnz, full.n
    full.close()
    out = {"mesh_intervals": N, "n": n, "m": m, "nnz_jac": nnz, "mode": "separate", "steps": args.steps, "W": {}}
    for W in (1, 2, 4, 8):
        row = {}
        for r in sorted({0, W - 1}):
            ib, ie = interval_shard(N, r, W)
            nlp = make_nlp(cx, build(), ib, ie, blocking=False)
            sep, _, bufs = device_steps(cx, nlp, track_iterate(nlp, 0))
            k, el = measure(cx, sep, args)
            row[f"rank{r}"] = {"intervals": [ib, ie], "ms_per_step": round(1e3 * el / k, 5),
                               "rows": nlp.row_end - nlp.row_begin, "nnz": nlp.nnz_end - nlp.nnz_begin}
            nlp.close()
        r0 = row["rank0"]
        slice_bytes = [8 * ((r["rows"]) + r["nnz"]) for key, r in row.items() if key != "rank0"]
        peer = max(slice_bytes) if slice_bytes else 0
        row["bytes_to_rank0"] = 8 * ((m - r0["rows"]) + (nnz - r0["nnz"])) if W > 1 else 0
        row["largest_peer_slice_bytes"] = peer
        t_eval = max(v["ms_per_step"] for k2, v in row.items() if k2.startswith("rank"))
        xb = 8 * n
        for name, bw in (("link153", 153e9), ("link50", 50e9)):
            t = t_eval + (1e3 * (xb + peer) / bw if W > 1 else 0.0)
            row[f"predicted_ms_{name}"] = round(t, 5)
            row[f"predicted_calls_per_s_{name}"] = round(1e3 / t, 1)
        out["W"][str(W)] = row
    return out


def guarded(cx, name, fn, errors):
    """Run a secondary leg of the multi-GPU line; an exception is reported
    under errors[name] instead of ending the job (the headline is already
    measured).  Every rank then meets at a barrier."""
    res = None
    try:
        res = fn()
    except Exception as e:   # noqa: BLE001
        errors[name] = f"rank {cx.rank}: {type(e).__name__}: {e}"
    if cx.world > 1:
        cx.dist.barrier()
    return res


def mesh_main(cx, args):
    """--multi mesh (the default at N > 1): the headline is one NLP sharded
    over the ranks with g / J reassembled in rank 0's HBM (mesh_measure),
    against rank 0 alone on the whole NLP; the secondary legs follow under a
    watchdog: if they do not finish within --leg-timeout seconds, rank 0
    prints the line with the headline and what finished, and every rank
    exits (a hung collective cannot lose the measured headline)."""
    import threading
    N = args.intervals
    build = _mesh_build(args)
    m = mesh_measure(cx, args)
    one = one_gpu_reference(cx, args, build)
    line = None
    if cx.rank == 0:
        wl = ("Rajagopal 80-muscle gait NLP (configs[3])" if args.config == "rajagopal80"
              else "MocoTrack gait10dof18musc DGF rigid tendon (configs[2])")
        line = {"metric": "NLP eval_g+eval_jac_g calls/sec (gait10dof18musc)" if args.config == "gait"
                          else "NLP eval_g+eval_jac_g calls/sec (Rajagopal 80-muscle)",
                "value": m["value"], "unit": "calls/s", "n_gpus": cx.world, "steps": m["steps"],
                "warmup": args.warmup, "settle_s": m["settle_s"], "ms_per_step": m["ms_per_step"],
                "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
                "config": {"workload": wl + ", one NLP sharded by mesh interval for one optimizer: x broadcast "
                                            "over RCCL, g / J reassembled in rank 0's HBM every call",
                           "mesh_intervals": N, "n": m["n"], "m": m["m"], "nnz_jac": m["nnz_jac"],
                           "fd": args.fd, "mode": args.mode, "parallelism": m["parallelism"]},
                "reassembly_bit_exact": m["reassembly_bit_exact"],
                "bytes_gathered_per_call": m["bytes_gathered_per_call"],
                "device_resident": m["device_resident"], "host_inclusive": m["host_inclusive"]}
        if one is not None:
            line["one_gpu"] = one
            line["strong_scaling"] = round(m["value"] / one["value"], 4)
    if args.single_mode:
        if cx.rank == 0:
            print(json.dumps(line), flush=True)
        return
    errors = {}
    done = threading.Event()

    def fire():   # the watchdog: the measured headline survives a hung secondary leg
        if done.is_set():
            return
        if cx.rank == 0:
            line["errors"] = dict(errors, watchdog=f"secondary legs unfinished after {args.leg_timeout} s")
            print(json.dumps(line), flush=True)
        os._exit(0)
    timer = threading.Timer(args.leg_timeout, fire)
    timer.daemon = True
    timer.start()

    def replicas():
        rnlp = make_nlp(cx, build(), blocking=False)
        rsep, rfused, _ = device_steps(cx, rnlp, track_iterate(rnlp, cx.rank))
        kr, elr = measure(cx, rfused if args.mode == "fused" else rsep, args)
        rnlp.close()
        return {"value": round(kr * cx.world / elr, 3), "unit": "calls/s", "steps": kr, "scaling": "weak",
                "note": "every rank its own whole NLP, no collective"}
    rep_line = guarded(cx, "replicas", replicas, errors)
    sweep = solve = None
    if args.sweep > 0:
        sweep = guarded(cx, "inverse_solve_sweep", lambda: sweep_distributed(cx, args), errors)
    if cx.world > 1 and args.solve_intervals > 0:
        solve = guarded(cx, "sharded_solve", lambda: sharded_solve(cx, args), errors)
    done.set()
    timer.cancel()
    if cx.rank == 0:
        line["replicas"] = rep_line
        if sweep is not None:
            line["inverse_solve_sweep"] = sweep
        if solve is not None:
            line["sharded_solve"] = solve
        if errors:
            line["errors"] = errors
        print(json.dumps(line), flush=True)


def main():
    args = parse()
    cx = Ctx(args)
    if args.multi is None:
        # N > 1: the north star's layout -- ONE NLP sharded by mesh interval
        # for one host optimizer, strong scaling, the host-inclusive rate as
        # the headline (mesh_main); the replicas layout (independent NLPs per
        # GPU, weak scaling) rides along in its line.  N = 1: the single-GPU
        # headline below.
        args.multi = "mesh" if cx.world > 1 else "replicas"
    if args.shard_model:
        res = shard_model(cx, args)
        if cx.rank == 0:
            print(json.dumps(res), flush=True)
        return
    if args.multi == "mesh":
        mesh_main(cx, args)
        if cx.world > 1:
            cx.dist.destroy_process_group()
        return
    from mocohip import configs
    N = args.intervals
    if args.batch_only:
        out = batch_throughput(cx, lambda: configs.gait10dof18musc(N, fd_scheme=args.fd), track_iterate,
                               args, args.batch)
        out["batched"] = batched_throughput(cx, lambda: configs.gait10dof18musc(N, fd_scheme=args.fd),
                                            track_iterate, args, args.batch)
        out["env"] = {k: os.environ[k] for k in ("GPU_MAX_HW_QUEUES", "MOCOHIP_GRAPHS") if k in os.environ}
        if cx.rank == 0:
            print(json.dumps(out), flush=True)
        return
    st = configs.gait10dof18musc(N, fd_scheme=args.fd)
    nlp = make_nlp(cx, st, blocking=args.blocking)
    # iterate: bounds midpoint for the states (where the muscle model is
    # regular), uniform random controls within bounds (replicas: seed =
    # rank, independent trials)
    x = track_iterate(nlp, cx.rank)
    sep, fused, bufs = device_steps(cx, nlp, x)
    xd, gd, vd = bufs
    head = fused if args.mode == "fused" else sep
    settled = settle(cx, head, args.settle_s)
    k, elapsed = measure(cx, head, args)
    value = k * cx.world / elapsed
    extra = {}
    if not args.single_mode:
        other = sep if args.mode == "fused" else fused
        _, el = measure(cx, other, args)
        extra["value_fused" if args.mode == "separate" else "value_separate"] = round(k * cx.world / el, 3)
        nlp.set_async(False)
        _, el = measure(cx, head, args)
        extra["value_blocking"] = round(k * cx.world / el, 3)
        nlp.set_async(not args.blocking)
    roof = roofline(cx, nlp, (sep, fused, (xd.data_ptr(), gd.data_ptr()), (xd.data_ptr(), vd.data_ptr())),
                    args, args.mode)
    if not args.single_mode:
        # the north-star size
        st4 = configs.gait10dof18musc(400, fd_scheme=args.fd)
        n4 = make_nlp(cx, st4, blocking=args.blocking)
        x4 = track_iterate(n4, cx.rank)
        s4, f4, b4 = device_steps(cx, n4, x4)
        k4, e4 = measure(cx, s4, args)
        _, ef4 = measure(cx, f4, args)
        hi4 = host_inclusive(cx, n4, x4, args)
        extra["n400"] = {"value": round(k4 * cx.world / e4, 3), "unit": "calls/s",
                         "ms_per_step": round(1e3 * e4 / k4, 5),
                         "value_fused": round(k4 * cx.world / ef4, 3),
                         "n": n4.n, "m": n4.m, "nnz_jac": n4.nnz, "host_inclusive": hi4,
                         "workload": "configs[2] workload at N=400 (north_star target size)"}
        if cx.world == 1 and not args.no_cpu_baseline:
            # the north star's target ratio is quoted at N=400 (>= 10x the
            # CPU eval_jac_g throughput): the oracle on the same N=400 NLP
            box = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            cb4 = cpu_baseline(n4.rep, st4.solver.options(), x4, max(3.0, args.cpu_baseline_seconds / 2),
                               max(1, min(box, os.cpu_count() or 1)))
            extra["n400"]["cpu_baseline"] = cb4
            extra["n400"]["speedup_vs_cpu_baseline"] = round(extra["n400"]["value"] / cb4["value"], 1)
        n4.close()
        extra["host_inclusive"] = host_inclusive(cx, nlp, x, args)
        # optim_sparsity_detection "random" (MocoInverse's setting,
        # MocoInverse.cpp:111): detected callback couplings only
        from mocohip.solver import HipNLP
        s2 = configs.gait10dof18musc(N, fd_scheme=args.fd)
        s2.solver.optim_sparsity_detection = "random"
        ns = make_nlp(cx, s2, blocking=args.blocking)
        ss, _, _ = device_steps(cx, ns, x)
        ks, es = measure(cx, ss, args)
        extra["sparsity_random"] = {"value": round(ks * cx.world / es, 3), "unit": "calls/s",
                                    "nnz_jac": ns.nnz, "mode": "separate",
                                    "note": "optim_sparsity_detection=random (3 iterates)"}
        ns.close()
        # tropter's Jacobian on the same NLP and GPU (jacobian_mode
        # "global-seeds": central FD of g along the column-coloring seeds,
        # ProblemDecorator_double.cpp:261-291) -- the reference's other
        # algorithm, for comparison with the per-callback lanes
        s3 = configs.gait10dof18musc(N, fd_scheme=args.fd)
        s3.solver.jacobian_mode = "global-seeds"
        n3 = make_nlp(cx, s3, blocking=args.blocking)
        sg, _, _ = device_steps(cx, n3, x)
        kg, eg = measure(cx, sg, args, k=max(3, args.steps // 200), w=2)
        extra["global_seeds"] = {"value": round(kg * cx.world / eg, 3), "unit": "calls/s",
                                 "seeds": n3.jacobian_seeds()[1], "steps": kg, "mode": "separate",
                                 "note": "jacobian_mode=global-seeds (tropter: 2 g evaluations per seed)"}
        n3.close()
        if args.batch > 1:
            extra["batch"] = batch_throughput(
                cx, lambda: configs.gait10dof18musc(N, fd_scheme=args.fd), track_iterate, args, args.batch)
            extra["batched"] = batched_throughput(
                cx, lambda: configs.gait10dof18musc(N, fd_scheme=args.fd), track_iterate, args, args.batch)
        if args.config3 > 0:
            extra["config3"] = config3_line(cx, args)
        if cx.world == 1:
            extra["solve"] = solve_lines()
            if args.solve_batch > 0:
                # configs[4]: the GPU's share of the 64-solve MocoInverse sweep,
                # one solver (process, HIP context + stream, host IPM) each
                from mocohip import batchsolve
                sb = batchsolve.solve_batch(batchsolve.sweep(args.solve_batch), 125, device=cx.local)
                sb["workload"] = ("configs[4]: MocoInverse gait10dof18musc N=125 for scaled subjects "
                                  "(length 0.97-1.03, mass 0.90-1.10), all started together on one GPU")
                extra["inverse_solve_batch"] = sb
        if args.inverse_batch > 0:
            # MocoTool mesh_interval 0.02 s: ceil((2.499 - 0.001) / 0.02) = 125
            # intervals (MocoTool.cpp:27,68-69)
            inv = batch_throughput(cx, lambda: configs.gait10dof18musc_inverse(125), inverse_iterate,
                                   args, args.inverse_batch)
            inv["workload"] = ("MocoInverse gait10dof18musc (configs[4]): PositionMotion, implicit DGF "
                               "tendons, reserves, initial-activation endpoint constraints, no control "
                               "interpolation, N=125, forward FD, random sparsity detection")
            extra["inverse_batch"] = inv
            invb = batched_throughput(cx, lambda: configs.gait10dof18musc_inverse(125), inverse_iterate,
                                      args, args.inverse_batch)
            invb["workload"] = inv["workload"]
            extra["inverse_batched"] = invb
    mesh = None
    if cx.world > 1 and not args.single_mode:
        mesh = mesh_measure(cx, args)
    if cx.rank == 0:
        cpu = cpu1 = None
        if cx.world == 1 and not args.no_cpu_baseline:
            box = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            threads = max(1, min(box, os.cpu_count() or 1))
            cpu = cpu_baseline(nlp.rep, st.solver.options(), x, args.cpu_baseline_seconds, threads)
            if not args.single_mode:
                cpu1 = cpu_baseline(nlp.rep, st.solver.options(), x, args.cpu_baseline_seconds, 1)
        line = {
            "metric": "NLP eval_g+eval_jac_g calls/sec (gait10dof18musc)",
            "value": round(value, 3), "unit": "calls/s", "n_gpus": cx.world,
            "steps": k, "warmup": args.warmup, "settle_s": settled,
            "ms_per_step": round(1e3 * elapsed / k, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "MocoTrack gait10dof18musc DGF rigid tendon (configs[2])",
                       "mesh_intervals": N, "grid_points": nlp.G, "n": nlp.n, "m": nlp.m,
                       "nnz_jac": nlp.nnz, "transcription": "hermite-simpson",
                       "fd": args.fd, "mode": args.mode,
                       "calls": "blocking" if args.blocking else "asynchronous (device pointers, torch stream)",
                       "parallelism": f"replicas{cx.world}" if cx.world > 1 else "single",
                       "iterate": "bounds-midpoint states, uniform random controls"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        line.update(extra)
        if mesh is not None:
            line["mesh"] = mesh
        if cpu1:
            line["cpu_baseline_1thread"] = cpu1
        if cpu and cpu.get("value"):
            line["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 2)
        print(json.dumps(line), flush=True)
    if cx.world > 1:
        cx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
