"""Mesh-interval sharding for one host IPOPT (mocohip.distributed) on the
CPU: world size 2 and 3 over gloo.

Each rank creates a SHARD context of the CPU oracle (mh_options
interval_begin/interval_end: it evaluates only its grid points and returns
its own rows / nonzeros), receives IPOPT's iterate x by broadcast from rank 0
(the one collective on the data path), and copies its slices into its offset
of the node-wide HostGather buffer.  Rank 0 -- the IPOPT rank -- then holds g
and the Jacobian values of the whole NLP; they must equal an unsharded
evaluation bit for bit.  The objective is sharded too: each rank's partial
(mh_eval_f_partial: its own intervals' quadrature, endpoint goals on the last
rank) and gradient partial, all-reduced, give f and grad f of the whole NLP.
The device shard contexts' slices are checked
against the unsharded device evaluation in
tests/test_gpu_parity.py::test_shards_reassemble_bit_exact; bench.py
--multi mesh runs the same HostGather with hipMemcpyAsync over each GPU's
PCIe link and RCCL for the broadcast.
"""
import os
import socket
import uuid

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mocohip import configs
from mocohip.distributed import HostGather, interval_shard, shard_counts, sharded_gradient, sharded_objective
from mocohip.solver import OracleNLP


def test_interval_shard_partition():
    for N in (1, 7, 200, 400):
        for W in (1, 2, 3, 8):
            spans = [interval_shard(N, r, W) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == N
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert sum(shard_counts(N, W)) == N
            assert max(shard_counts(N, W)) - min(shard_counts(N, W)) <= 1
    with pytest.raises(ValueError):
        interval_shard(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CASES = {"pendulum": lambda N: configs.double_pendulum(N),
         "gait": lambda N: configs.gait10dof18musc(N),
         "pendulum_implicit": lambda N: configs.double_pendulum(N, dynamics="implicit"),
         "gait_pathcon": lambda N: configs.gait10dof18musc(N, control_bounds=True),
         "bound_implicit": lambda N: configs.pendulum_control_bound(N, "both", dynamics="implicit"),
         "inverse": lambda N: configs.gait10dof18musc_inverse(N, sparsity="none"),
         "swingup": lambda N: configs.double_pendulum_swingup(N)}


def _worker(rank, world, port, case, N, tag, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hg = None
    try:
        st = CASES[case](N)
        rep = st.problem.create_rep()
        ib, ie = interval_shard(N, rank, world)
        shard = OracleNLP(rep, st.solver.options(ib, ie), threads=1)
        # IPOPT's iterate, on rank 0, broadcast to every rank
        x = torch.zeros(shard.n, dtype=torch.float64)
        if rank == 0:
            x[:] = torch.from_numpy(shard.random_iterate(np.random.default_rng(3).uniform(-1, 1, shard.n)))
        dist.broadcast(x, src=0)
        xn = x.numpy()
        hg = HostGather(tag, shard.m, shard.nnz, (shard.row_begin, shard.row_end),
                        (shard.nnz_begin, shard.nnz_end), rank, dist.barrier)
        g, J = shard.eval_g(xn), shard.eval_jac_g(xn)
        assert len(g) == shard.row_end - shard.row_begin and len(J) == shard.nnz_end - shard.nnz_begin
        hg.copy_from_host(g, J)
        dist.barrier()

        # the sharded objective: each rank's partial, one all-reduce
        def allreduce(a):
            t = torch.from_numpy(np.ascontiguousarray(a, np.float64))
            dist.all_reduce(t)
            return t.numpy()
        f = sharded_objective(shard, xn, allreduce)
        gf = sharded_gradient(shard, xn, allreduce)
        ok = True
        if rank == 0:
            full = OracleNLP(rep, st.solver.options(), threads=1)
            ok = (np.array_equal(hg.full_g(), full.eval_g(xn))
                  and np.array_equal(hg.full_values(), full.eval_jac_g(xn)))
            f0, g0 = full.eval_f(xn), full.eval_grad_f(xn)
            # (the partial sums add the integral's terms in another order)
            ok = ok and abs(f - f0) <= 1e-12 * max(1.0, abs(f0))
            ok = ok and float(np.abs(gf - g0).max()) <= 1e-12 * max(1.0, float(np.abs(g0).max()))
            # an unsharded context's partial is its objective, bit for bit
            ok = ok and full.eval_f_partial(xn) == f0 and np.array_equal(full.eval_grad_f_partial(xn), g0)
        out[rank] = int(ok)
        dist.barrier()
    finally:
        if hg is not None:
            hg.close(unlink=rank == 0)
        dist.destroy_process_group()


@pytest.mark.parametrize("case,N,world", [("pendulum", 7, 2), ("pendulum", 10, 3), ("gait", 5, 2),
                                          ("pendulum_implicit", 7, 3), ("gait_pathcon", 4, 2),
                                          ("bound_implicit", 9, 3), ("inverse", 4, 2), ("inverse", 5, 3),
                                          ("swingup", 6, 2), ("swingup", 7, 3)])
def test_shard_contexts_reassemble_on_the_ipopt_host(case, N, world):
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    tag = f"mocohip_test_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, N, tag, out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1] * world


# ---------------------------------------------------------------------------
# One solve spanning the ranks (mocohip.distributed.ShardedNLP): the
# optimizer on rank 0, the evaluation sharded, g / J reassembled on rank 0.
# ---------------------------------------------------------------------------
SOLVE_CASES = {"pendulum": lambda N: configs.double_pendulum(N),
               "gait_inverse": lambda N: configs.gait10dof18musc_inverse(N, sparsity="none"),
               "gait_track": lambda N: configs.gait10dof18musc_track(N, muscles=True)}


def _ipm_opts(iters):
    from mocohip.ipm import IpmOptions
    o = IpmOptions.from_ipopt({"tol": 1e-8, "constr_viol_tol": 1e-8, "max_iter": iters})
    o.linear_solver = "host"
    return o


def _sharded_worker(rank, world, port, case, N, iters, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mocohip.distributed import ShardedNLP
        from mocohip.ipm import solve_ipm
        st = SOLVE_CASES[case](N)
        rep = st.problem.create_rep()
        ib, ie = interval_shard(N, rank, world)
        snlp = ShardedNLP(OracleNLP(rep, st.solver.options(ib, ie), threads=1), dist)
        if rank > 0:
            snlp.serve()
            out[rank] = 1
            return
        full = OracleNLP(rep, st.solver.options(), threads=1)
        ok = (snlp.n, snlp.m, snlp.nnz) == (full.n, full.m, full.nnz)
        x = full.random_iterate(np.random.default_rng(5).uniform(-1, 1, full.n))
        # g and J reassembled on rank 0: bit for bit the unsharded evaluation
        ok = ok and np.array_equal(snlp.eval_g(x), full.eval_g(x))
        ok = ok and np.array_equal(snlp.eval_jac_g(x), full.eval_jac_g(x))
        f0 = full.eval_f(x)
        ok = ok and abs(snlp.eval_f(x) - f0) <= 1e-12 * max(1.0, abs(f0))
        # the optimizer driven through the shards takes the unsharded run's
        # Newton steps: the same iterates (to the rounding of the objective's
        # partial sums) after `iters` iterations
        x0 = st.solver.starting_point(full, None)
        a = solve_ipm(snlp, x0, _ipm_opts(iters))
        b = solve_ipm(full, x0, _ipm_opts(iters))
        ok = ok and a.iterations == b.iterations
        ok = ok and float(np.abs(a.x - b.x).max()) <= 1e-9 * max(1.0, float(np.abs(b.x).max()))
        out[0] = int(bool(ok))
        snlp.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,N,world,iters", [("pendulum", 8, 2, 1), ("pendulum", 9, 3, 4),
                                                ("gait_inverse", 4, 2, 2), ("gait_track", 4, 2, 1)])
def test_sharded_solve_takes_the_unsharded_steps(case, N, world, iters):
    """ShardedNLP (world 2 / 3 over gloo, oracle shard contexts): rank 0's
    reassembled g and J equal the unsharded evaluation bit for bit, and the
    interior-point method driven through the shards takes the same Newton
    steps as on the unsharded NLP."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, case, N, iters, out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    assert list(out) == [1] * world


def test_sweep_rank_partition():
    """configs[4] over W ranks (mocohip.batchsolve.rank_share): every one
    of the 64 subjects is solved by exactly one rank, the shares differ by at
    most one solve, and W = 1 keeps the sweep's order."""
    from mocohip.batchsolve import rank_share, sweep
    s = sweep(64)
    assert len(set(s)) == 64
    for W in (1, 2, 3, 4, 8):
        parts = [rank_share(s, r, W) for r in range(W)]
        assert sorted(sum(parts, [])) == sorted(s)
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
    assert rank_share(s, 0, 1) == s
    with pytest.raises(ValueError):
        rank_share(s, 8, 8)


# ---------------------------------------------------------------------------
# The multi-GPU headline's reassembly (bench.py --gpus N > 1): every rank's
# g / Jacobian slice into its offset of rank 0's whole-NLP buffers
# (mocohip.distributed.SliceGather; RCCL P2P over xGMI on the GPUs, gloo here).
# ---------------------------------------------------------------------------
def _gather_worker(rank, world, port, case, N, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mocohip.distributed import SliceGather
        st = CASES[case](N)
        rep = st.problem.create_rep()
        ib, ie = interval_shard(N, rank, world)
        shard = OracleNLP(rep, st.solver.options(ib, ie), threads=1)
        sg = SliceGather(shard.m, shard.nnz, (shard.row_begin, shard.row_end, shard.nnz_begin, shard.nnz_end),
                         dist, "cpu")
        ok = True
        for it in range(2):   # two calls through the same buffers
            x = torch.zeros(shard.n, dtype=torch.float64)
            if rank == 0:
                x[:] = torch.from_numpy(shard.random_iterate(np.random.default_rng(11 + it).uniform(-1, 1, shard.n)))
            dist.broadcast(x, src=0)
            xn = x.numpy()
            # the shard's results land in its own slice buffers (rank 0: views
            # of the whole vectors), then the fan-in
            sg.own_g.copy_(torch.from_numpy(shard.eval_g(xn)))
            rg = sg.post("g")
            sg.own_values.copy_(torch.from_numpy(shard.eval_jac_g(xn)))
            rv = sg.post("values")
            sg.wait(rg)
            sg.wait(rv)
            if rank == 0:
                full = OracleNLP(rep, st.solver.options(), threads=1)
                ok = ok and np.array_equal(sg.g.numpy()[:full.m], full.eval_g(xn))
                ok = ok and np.array_equal(sg.values.numpy()[:full.nnz], full.eval_jac_g(xn))
                rb, re, nb, ne = sg.ranges[0]
                ok = ok and sg.bytes_received() == 8 * ((full.m - (re - rb)) + (full.nnz - (ne - nb)))
                full.close()
        # the ranges tile the whole vectors in rank order
        if rank == 0:
            ok = ok and sg.ranges[0][0] == 0 and sg.ranges[-1][1] == shard.m
            ok = ok and sg.ranges[0][2] == 0 and sg.ranges[-1][3] == shard.nnz
        out[rank] = int(bool(ok))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,N,world", [("pendulum", 7, 2), ("gait", 6, 3), ("pendulum_implicit", 16, 8),
                                          ("inverse", 9, 8), ("gait_pathcon", 5, 3)])
def test_slice_gather_reassembles_on_rank0(case, N, world):
    """SliceGather (world 2 / 3 / 8 over gloo, oracle shard contexts): rank
    0's whole-NLP g and Jacobian buffers, filled by its own shard in place and
    by the other ranks' slices at their offsets, equal the unsharded
    evaluation bit for bit, call after call."""
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, case, N, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    assert list(out) == [1] * world


def _settle_worker(rank, world, port, q):
    import os
    import time
    import types
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    calls = [0]
    buf = torch.zeros(4)

    def step():                      # a collective per step, like the mesh step
        calls[0] += 1
        dist.broadcast(buf, src=0)
        if rank == 1:
            time.sleep(0.0005)       # the ranks' clocks disagree
    cx = types.SimpleNamespace(torch=torch, dist=dist, world=world, dev="cpu", sync=lambda: None)
    bench.settle(cx, step, 0.05 if rank == 0 else 0.5)
    dist.barrier()
    q.put((rank, calls[0]))
    dist.destroy_process_group()


def test_bench_settle_runs_the_same_steps_on_every_rank():
    """bench.settle's untimed calls hold collectives at N > 1: every rank
    must run the same number of them whatever its own clock says (rank 0
    decides per chunk), or the next collective deadlocks."""
    import multiprocessing as mp
    import socket
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_settle_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    got = dict(q.get(timeout=5) for _ in range(2))
    assert got[0] == got[1] and got[0] % 50 == 0, got
