"""Mesh-interval sharding with the node-wide HostGather buffer on a real GPU
(mocohip.distributed; the CPU version is tests/test_distributed.py): two
fresh child processes, both on GPU 0, each a device SHARD context of its
contiguous mesh intervals, the iterate broadcast from rank 0 (gloo here;
RCCL in bench.py --multi mesh), each rank's g / Jacobian slices DMA'd with
hipMemcpyAsync from HBM into its offset of one /dev/shm mapping that every
process page-locks with hipHostRegister.  Rank 0 -- the IPOPT rank -- must
then hold g and the Jacobian values of the whole NLP bit for bit equal to
one unsharded device evaluation."""
import os
import socket
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, N, tag, out):
    import torch
    import torch.distributed as dist
    from mocohip import configs
    from mocohip.distributed import HostGather, interval_shard
    from mocohip.solver import HipNLP
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hg = nlp = None
    try:
        torch.cuda.set_device(0)
        st = configs.gait10dof18musc(N)
        rep = st.problem.create_rep()
        ib, ie = interval_shard(N, rank, world)
        nlp = HipNLP(rep, st.solver.options(ib, ie))
        x = torch.zeros(nlp.n, dtype=torch.float64)
        if rank == 0:
            xi = nlp.random_iterate(np.random.default_rng(5).uniform(-1, 1, nlp.n))
            xi[2:2 + nlp.NS * nlp.G] = nlp.initial_guess_from_bounds()[2:2 + nlp.NS * nlp.G]
            x[:] = torch.from_numpy(xi)
        dist.broadcast(x, src=0)
        xd = x.to("cuda:0")
        gd = torch.zeros(max(nlp.row_end - nlp.row_begin, 1), dtype=torch.float64, device="cuda:0")
        vd = torch.zeros(max(nlp.nnz_end - nlp.nnz_begin, 1), dtype=torch.float64, device="cuda:0")
        stream = torch.cuda.current_stream().cuda_stream
        nlp.set_stream(stream)
        hg = HostGather(tag, nlp.m, nlp.nnz, (nlp.row_begin, nlp.row_end), (nlp.nnz_begin, nlp.nnz_end),
                        rank, dist.barrier, pin=True)
        nlp.eval_g_jac_g_device(xd.data_ptr(), gd.data_ptr(), vd.data_ptr())
        nlp.synchronize()
        hg.copy_from_device_async(gd.data_ptr(), vd.data_ptr(), stream)
        torch.cuda.current_stream().synchronize()
        dist.barrier()                      # every slice has landed on the IPOPT host
        ok = True
        if rank == 0:
            full = HipNLP(rep, st.solver.options())
            xn = x.numpy()
            ok = (np.array_equal(hg.full_g(), full.eval_g(xn))
                  and np.array_equal(hg.full_values(), full.eval_jac_g(xn)))
            full.close()
        out[rank] = int(ok)
        dist.barrier()
    finally:
        if hg is not None:
            hg.close(unlink=rank == 0)
        if nlp is not None:
            nlp.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("N", [9, 40])
def test_host_gather_two_processes_on_gpu0(N):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    world = 2
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    tag = f"mocohip_gputest_{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, tag, out)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        for p in procs:
            p.join(150)
            assert p.exitcode == 0, p.exitcode
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
        if os.path.exists(os.path.join("/dev/shm", tag)):
            os.unlink(os.path.join("/dev/shm", tag))
    assert list(out) == [1] * world


def _solve_worker(rank, world, port, N, out, res):
    """One MocoInverse solve spanning two processes on GPU 0: rank 0 the
    optimizer with its Newton systems on the device over the WHOLE Jacobian
    (ShardedDeviceKKT: its own slice by its kernels, rank 1's received into
    the bound buffer), rank 1 serving its shard."""
    import torch
    import torch.distributed as dist
    from mocohip import configs
    from mocohip.distributed import ShardedNLP, interval_shard
    from mocohip.solver import HipNLP
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        st = configs.gait10dof18musc_inverse(N)
        rep = st.problem.create_rep()
        ib, ie = interval_shard(N, rank, world)
        snlp = ShardedNLP(HipNLP(rep, st.solver.options(ib, ie)), dist, transport="host")
        if rank > 0:
            snlp.serve()
            out[rank] = 1
            return
        full = HipNLP(rep, st.solver.options())
        # the whole Jacobian reassembled in rank 0's HBM: bit for bit the
        # unsharded evaluation
        x = full.initial_guess_from_bounds()
        dk = snlp.device_kkt()
        dk.eval_jacobian(x)
        ok = np.array_equal(dk.values(), full.eval_jac_g(x))
        a = st.solve(nlp=snlp, linear_solver="device")
        b = st.solve(nlp=full, linear_solver="device")
        ra, rb = a.stats, b.stats
        ok = ok and ra.success and rb.success and "device" in ra.timings.get("linear_solver", "")
        ok = ok and abs(ra.objective - rb.objective) <= 1e-6 * max(1.0, abs(rb.objective))
        res[0], res[1], res[2], res[3] = ra.objective, rb.objective, ra.iterations, rb.iterations
        out[0] = int(bool(ok))
        snlp.close()
        full.close()
    finally:
        dist.destroy_process_group()


def test_sharded_solve_device_kkt_two_processes_on_gpu0():
    """A solve spanning two processes (ShardedNLP, gloo, both on GPU 0; on a
    node each rank has its own GPU and the slices move over RCCL): rank 0's
    device KKT module factors the whole Jacobian reassembled in its HBM, and
    the solve reaches the unsharded solve's objective."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    world = 2
    out = ctx.Array("i", [0] * world)
    res = ctx.Array("d", [0.0] * 4)
    port = _free_port()
    procs = [ctx.Process(target=_solve_worker, args=(r, world, port, 25, out, res)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        for p in procs:
            p.join(240)
            assert p.exitcode == 0, p.exitcode
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    print("sharded / unsharded objective, iterations:", list(res))
    assert list(out) == [1] * world
