"""Mesh-interval sharding and the all-gather reassembly (mocohip.distributed)
on the CPU: world_size 2 and 3 over gloo.

Each rank takes its shard's g rows and Jacobian values from the CPU oracle's
full evaluation. That is what its shard context writes on the GPU, because
the rows and nonzeros of a shard are a contiguous slice
(tests/test_gpu_parity.py::test_shards_reassemble_bit_exact checks that on
the device). The rank then puts the slice in the padded segment and
all-gathers it. The reassembled vectors must equal the full evaluation
bit for bit. bench.py runs the same ShardGather over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mocohip import configs
from mocohip.distributed import ShardGather, interval_shard, shard_counts
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


def _worker(rank, world, port, case, N, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        st = {"pendulum": lambda: configs.double_pendulum(N),
              "gait": lambda: configs.gait10dof18musc(N),
              "pendulum_implicit": lambda: configs.double_pendulum(N, dynamics="implicit"),
              "gait_pathcon": lambda: configs.gait10dof18musc(N, control_bounds=True),
              "bound_implicit": lambda: configs.pendulum_control_bound(N, "both",
                                                                       dynamics="implicit")}[case]()
        rep = st.problem.create_rep()
        ref = OracleNLP(rep, st.solver.options(), threads=1)
        x = ref.random_iterate(np.random.default_rng(3).uniform(-1, 1, ref.n))
        g, J = ref.eval_g(x), ref.eval_jac_g(x)
        # the final mesh point's path rows and (implicit dynamics) the final
        # point's residual rows follow the last interval (tail), owned by the
        # last rank
        tail_rows = ref.tail_rows
        ir, _ = ref.jac_structure()
        tail_nnz = int((ir >= ref.m - tail_rows).sum())
        rpi, nzi = (ref.m - tail_rows) // N, (ref.nnz - tail_nnz) // N
        sg = ShardGather(N, rpi, nzi, world, "cpu", tail_rows=tail_rows, tail_nnz=tail_nnz)
        ib, ie = interval_shard(N, rank, world)
        rows = (ie - ib) * rpi + (tail_rows if ie == N else 0)
        nz = (ie - ib) * nzi + (tail_nnz if ie == N else 0)
        assert rows == sg.g_sizes[rank] and nz == sg.v_sizes[rank]
        sg.gseg.zero_()
        sg.vseg.zero_()
        sg.gseg[:rows] = torch.from_numpy(g[ib * rpi:ib * rpi + rows])
        sg.vseg[:nz] = torch.from_numpy(J[ib * nzi:ib * nzi + nz])
        sg.gather()
        ok = (np.array_equal(sg.full_g().numpy(), g)
              and np.array_equal(sg.full_values().numpy(), J))
        out[rank] = int(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,N,world", [("pendulum", 7, 2), ("pendulum", 10, 3), ("gait", 5, 2),
                                          ("pendulum_implicit", 7, 3), ("gait_pathcon", 4, 2),
                                          ("bound_implicit", 9, 3)])
def test_shard_gather_reassembles_full_vectors(case, N, world):
    ctx = mp.get_context("spawn")
    out = ctx.Array("i", [0] * world)
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, N, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert list(out) == [1] * world
