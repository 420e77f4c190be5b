"""Mesh-interval sharding over ranks (one process per GPU) for ONE host IPOPT.

The g rows and Jacobian nonzeros of mesh interval i are contiguous, every
interval has the same row and nonzero counts, the endpoint rows (the head)
precede interval 0 and the final mesh point's rows (the tail) follow
interval N-1 (CasOCTranscription.h:219-313).  So rank r owns
the intervals [N*r/W, N*(r+1)/W) (mh_options interval_begin/interval_end),
evaluates only those, and its results are ONE contiguous slice of g and one
of the Jacobian values (mh_nlp_info row_begin/row_end, nnz_begin/nnz_end).
The boundary grid point between two shards is evaluated by both ranks:
recomputing it is cheaper than exchanging it.

Reassembly for a single host IPOPT needs no device
collective on g / J: every rank copies its slice straight into its offset of
one host buffer shared by the node's ranks (``HostGather``: POSIX shared
memory, page-locked with hipHostRegister so the copy is DMA over that GPU's
own PCIe link).  The only collective on the data path is the broadcast of
IPOPT's iterate x to every rank (RCCL over xGMI in bench.py, gloo on the CPU
in tests/test_distributed.py).  The objective is sharded the same way: each
rank's context sums the integral goals over its own mesh intervals
(mh_eval_f_partial; the reference assembles the integral from the
per-interval quadrature, CasOCTranscription.cpp:489-493) and the rank owning
the final grid point adds the endpoint goals, so f is one all-reduce of a
double and grad f one all-reduce of an n-vector (``sharded_objective``,
``sharded_gradient``).
"""
from __future__ import annotations

import ctypes as C
import mmap
import os
from typing import List, Tuple

import numpy as np


def interval_shard(num_intervals: int, rank: int, world: int) -> Tuple[int, int]:
    """[begin, end) mesh intervals owned by ``rank``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return (num_intervals * rank) // world, (num_intervals * (rank + 1)) // world


def shard_counts(num_intervals: int, world: int) -> List[int]:
    return [e - b for b, e in (interval_shard(num_intervals, r, world) for r in range(world))]


_hip = None


def _hip_runtime():
    """The HIP runtime libmocohip and torch share (for hipHostRegister /
    hipMemcpyAsync on the shared buffer)."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
        _hip.hipHostRegister.restype = C.c_int
        _hip.hipHostUnregister.argtypes = [C.c_void_p]
        _hip.hipHostUnregister.restype = C.c_int
        _hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
        _hip.hipMemcpyAsync.restype = C.c_int
    return _hip


HIP_MEMCPY_DEVICE_TO_HOST = 2


def sharded_objective(nlp, x, allreduce) -> float:
    """f(x) of the whole NLP from this rank's shard context: its partial
    (mh_eval_f_partial) summed over the ranks by ``allreduce`` (a callable
    summing a float64 numpy array over the ranks, e.g. torch.distributed
    all_reduce over RCCL or gloo)."""
    return float(allreduce(np.array([nlp.eval_f_partial(x)], dtype=np.float64))[0])


def sharded_gradient(nlp, x, allreduce) -> np.ndarray:
    """grad f(x) of the whole NLP: the shards' gradient partials summed."""
    return allreduce(np.ascontiguousarray(nlp.eval_grad_f_partial(x), dtype=np.float64))


def _device_numa_node(device: int) -> int:
    """The NUMA node of a GPU's PCIe root (-1 when unknown)."""
    hip = _hip_runtime()
    buf = C.create_string_buffer(64)
    try:
        hip.hipDeviceGetPCIBusId.argtypes = [C.c_char_p, C.c_int, C.c_int]
        hip.hipDeviceGetPCIBusId.restype = C.c_int
        if hip.hipDeviceGetPCIBusId(buf, 64, int(device)) != 0:
            return -1
        with open(f"/sys/bus/pci/devices/{buf.value.decode().lower()}/numa_node") as fh:
            return int(fh.read().strip())
    except (OSError, ValueError, AttributeError):
        return -1


def _node_cpus(node: int):
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            spec = fh.read().strip()
    except OSError:
        return None
    cpus = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus or None


_PAGE = mmap.PAGESIZE


class HostGather:
    """One node-wide host buffer [g (m doubles) | Jacobian values (nnz)] that
    every rank fills with its shard's slice; the IPOPT rank reads the full
    vectors from it.

    ``name``: a tag unique to the job (rank 0 creates /dev/shm/<name>, the
    others map it after ``barrier()``).  ``rows`` / ``nnz``: this rank's
    [begin, end) ranges (mh_nlp_info).  ``pin``: page-lock THIS RANK'S
    slices (not the whole buffer) for device-to-host DMA (GPU runs).
    ``device``: the rank's GPU -- its slices' pages are first touched by a
    thread bound to the CPUs of the GPU's NUMA node, so that on a two-socket
    node each rank's DMA lands in memory local to its own PCIe root."""

    def __init__(self, name: str, m: int, nnz: int, rows: Tuple[int, int], nz: Tuple[int, int],
                 rank: int, barrier, pin: bool = False, device: int | None = None):
        self.m, self.nnz = int(m), int(nnz)
        self.rows, self.nz = (int(rows[0]), int(rows[1])), (int(nz[0]), int(nz[1]))
        self.rank = rank
        self.path = os.path.join("/dev/shm", name)
        self.bytes = 8 * (self.m + self.nnz)
        if rank == 0:
            with open(self.path, "wb") as fh:
                fh.truncate(self.bytes)
        barrier()
        fd = os.open(self.path, os.O_RDWR)
        try:
            self._mm = mmap.mmap(fd, self.bytes)
        finally:
            os.close(fd)
        self.buf = np.frombuffer(self._mm, dtype=np.float64)
        self.g = self.buf[:self.m]
        self.values = self.buf[self.m:]
        # this rank's two slices as page ranges (a page two ranks share is
        # registered by both: registration is per process)
        base = self.buf.ctypes.data
        spans = [(8 * self.rows[0], 8 * self.rows[1]), (8 * (self.m + self.nz[0]), 8 * (self.m + self.nz[1]))]
        pages = []
        for a, b in spans:
            if b > a:
                pages.append([(base + a) // _PAGE * _PAGE, -(-(base + b) // _PAGE) * _PAGE])
        merged = []
        for lo, hi in sorted(pages):
            if merged and lo <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], hi)
            else:
                merged.append([lo, hi])
        self._ranges = [(lo, hi - lo) for lo, hi in merged]
        self.numa_node = -1
        if device is not None:
            self._first_touch(device)
        self._pinned = []
        if pin:
            hip = _hip_runtime()
            for lo, n in self._ranges:
                rc = hip.hipHostRegister(lo, n, 0)
                if rc != 0:
                    self.close()
                    raise RuntimeError(f"hipHostRegister failed ({rc})")
                self._pinned.append(lo)

    def _first_touch(self, device: int):
        """Zero this rank's slices from a thread bound to the GPU's NUMA
        node: tmpfs allocates a page on the node of the CPU that first writes
        it."""
        node = _device_numa_node(device)
        cpus = _node_cpus(node) if node >= 0 else None
        if not cpus:
            return
        old = os.sched_getaffinity(0)
        try:
            os.sched_setaffinity(0, cpus & set(range(os.cpu_count() or 1)) or old)
            for a, b in ((self.rows[0], self.rows[1]), (self.m + self.nz[0], self.m + self.nz[1])):
                self.buf[a:b] = 0.0
            self.numa_node = node
        finally:
            os.sched_setaffinity(0, old)

    # -- filling this rank's slice
    def copy_from_host(self, g_slice, v_slice):
        self.g[self.rows[0]:self.rows[1]] = g_slice
        self.values[self.nz[0]:self.nz[1]] = v_slice

    def copy_from_device_async(self, g_dev: int, v_dev: int, stream: int):
        """hipMemcpyAsync of this rank's g / values slices (device pointers)
        into the pinned shared buffer, ordered on ``stream``."""
        hip = _hip_runtime()
        dst_g = self.buf.ctypes.data + 8 * self.rows[0]
        dst_v = self.buf.ctypes.data + 8 * (self.m + self.nz[0])
        for dst, src, n in ((dst_g, g_dev, self.rows[1] - self.rows[0]),
                            (dst_v, v_dev, self.nz[1] - self.nz[0])):
            if n:
                rc = hip.hipMemcpyAsync(dst, src, 8 * n, HIP_MEMCPY_DEVICE_TO_HOST, stream)
                if rc != 0:
                    raise RuntimeError(f"hipMemcpyAsync failed ({rc})")

    # -- the IPOPT rank's view (after every rank's copy completed + barrier)
    def full_g(self):
        return self.g

    def full_values(self):
        return self.values

    def close(self, unlink: bool = False):
        for lo in getattr(self, "_pinned", []):
            _hip_runtime().hipHostUnregister(lo)
        self._pinned = []
        self.g = self.values = self.buf = None
        try:
            self._mm.close()
        except BufferError:
            pass
        if unlink and os.path.exists(self.path):
            os.unlink(self.path)


class SliceGather:
    """g and the Jacobian values of ONE NLP reassembled in rank 0's device
    memory from the ranks' mesh shards (the north star's
    "RCCL all-gather over xGMI to reassemble g and the CSR Jacobian" --
    only rank 0, where the optimizer's Newton systems are factored, needs the
    whole vectors, so it is a fan-in, not an all-gather: every other rank sends
    its contiguous slice (CasOCTranscription.h:219-313) point to point and
    rank 0 receives them straight into their offsets, one grouped
    batch_isend_irecv per vector, so the W - 1 transfers run concurrently, each
    on its own xGMI link).

    Rank 0 allocates the whole-NLP buffers ``g`` (m) and ``values`` (nnz);
    its own context writes its slice in place through the views ``own_g`` /
    ``own_values`` (no copy); the other ranks' ``own_*`` are buffers of their
    slice length.  ``ranges[r]`` = rank r's (row_begin, row_end, nnz_begin,
    nnz_end), all-gathered at construction.  Tensors live on ``device`` (a
    CUDA device: RCCL P2P over xGMI with backend nccl; the CPU: gloo, as in
    tests/test_distributed.py)."""

    def __init__(self, m: int, nnz: int, mine, dist, device):
        import torch
        self.torch, self.dist = torch, dist
        single = not dist.is_initialized()    # one process: nothing to gather
        self.rank, self.world = (0, 1) if single else (dist.get_rank(), dist.get_world_size())
        self.m, self.nnz = int(m), int(nnz)
        self.device = torch.device(device)
        t = torch.tensor([int(v) for v in mine], dtype=torch.int64, device=self.device)
        got = [torch.zeros_like(t) for _ in range(self.world)]
        if single:
            got[0] = t
        else:
            dist.all_gather(got, t)
        self.ranges = [tuple(int(v) for v in a.cpu()) for a in got]
        rb, re, nb, ne = self.ranges[self.rank]
        # the slices must tile [0, m) and [0, nnz) in rank order
        for which, total in ((0, self.m), (2, self.nnz)):
            pos = 0
            for r in range(self.world):
                b, e = self.ranges[r][which], self.ranges[r][which + 1]
                if b != pos or e < b:
                    raise ValueError(f"rank {r}'s slice [{b}, {e}) does not continue at {pos}")
                pos = e
            if pos != total:
                raise ValueError(f"the slices end at {pos}, not {total}")
        f64 = torch.float64
        if self.rank == 0:
            self.g = torch.zeros(max(1, self.m), dtype=f64, device=self.device)
            self.values = torch.zeros(max(1, self.nnz), dtype=f64, device=self.device)
            self.own_g, self.own_values = self.g[rb:re], self.values[nb:ne]
        else:
            self.g = self.values = None
            self.own_g = torch.zeros(max(1, re - rb), dtype=f64, device=self.device)[:re - rb]
            self.own_values = torch.zeros(max(1, ne - nb), dtype=f64, device=self.device)[:ne - nb]

    def post(self, which: str):
        """Start the fan-in of ``which`` ("g" or "values") after the shard's
        evaluation was enqueued on the current stream; returns the requests
        (``wait`` them before reading rank 0's buffer)."""
        dist = self.dist
        k = 0 if which == "g" else 2
        ops = []
        if self.rank == 0:
            whole = self.g if which == "g" else self.values
            for r in range(1, self.world):
                b, e = self.ranges[r][k], self.ranges[r][k + 1]
                if e > b:
                    ops.append(dist.P2POp(dist.irecv, whole[b:e], r))
        else:
            own = self.own_g if which == "g" else self.own_values
            if own.numel():
                ops.append(dist.P2POp(dist.isend, own, 0))
        return dist.batch_isend_irecv(ops) if ops else []

    @staticmethod
    def wait(reqs):
        for q in reqs:
            q.wait()

    def bytes_received(self) -> int:
        """Bytes rank 0 receives per g + Jacobian reassembly."""
        rb, re, nb, ne = self.ranges[0]
        return 8 * ((self.m - (re - rb)) + (self.nnz - (ne - nb)))


# ---------------------------------------------------------------------------
# One solve spanning several GPUs: the optimizer on rank 0, the evaluation
# sharded by mesh interval.
# ---------------------------------------------------------------------------
OP_STOP, OP_F, OP_GRAD, OP_G, OP_JAC, OP_JAC_DEV = range(6)


class ShardedNLP:
    """ONE NLP whose mesh intervals are sharded over the ranks of a
    torch.distributed group, seen from rank 0 as the whole NLP -- the
    interface mocohip.ipm / mocohip.nlpsolve drive (n, m, nnz, bounds,
    jac_structure, eval_f / eval_grad_f / eval_g / eval_jac_g, device_kkt).

    ``shard``: this rank's shard context (HipNLP, or OracleNLP on the CPU),
    created with mh_options interval_begin / interval_end = interval_shard().
    Rank 0 runs the optimizer through this object; every other rank calls
    ``serve()``, which answers rank 0's requests until ``close()``.  Per
    request rank 0 broadcasts an op code and the iterate x (the one
    collective every evaluation needs); then
      f, grad f   each rank's partial (mh_eval_f_partial / _grad_f_partial),
                  summed onto rank 0 by a reduce;
      g, J        each rank's contiguous slice (CasOCTranscription.h:
                  219-313: rows and nonzeros are contiguous per interval)
                  sent to rank 0 point to point;
      J on the device (device_kkt; the optimizer's Newton systems factored
                  on rank 0's GPU, include/mocohip_kkt.h): rank 0's own slice
                  is written by its kernels straight into the KKT module's
                  Jacobian buffer, the other ranks' slices are received into
                  their offsets of that buffer -- over RCCL / xGMI GPU to GPU
                  (``transport="device"``, backend nccl) or staged through
                  host memory (``transport="host"``, backend gloo) -- and the
                  module then gathers its blocks from the whole buffer.
    g and J reach rank 0 bit-identical to an unsharded evaluation; f and
    grad f are sums of partials (another order of the same terms)."""

    def __init__(self, shard, dist, transport: str = "host", device=None):
        if transport not in ("host", "device"):
            raise ValueError("transport must be 'host' or 'device'")
        self.shard, self.dist, self.transport = shard, dist, transport
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.n, self.m, self.nnz = int(shard.n), int(shard.m), int(shard.nnz)
        import torch
        self.torch = torch
        self.device = torch.device("cuda", int(device)) if transport == "device" else torch.device("cpu")
        mine = torch.tensor([shard.row_begin, shard.row_end, shard.nnz_begin, shard.nnz_end],
                            dtype=torch.int64, device=self.device)
        got = [torch.zeros_like(mine) for _ in range(self.world)]
        dist.all_gather(got, mine)
        self.ranges = [tuple(int(v) for v in t.cpu()) for t in got]
        # the whole NLP's view (rank 0 holds every row and nonzero)
        self.row_begin, self.row_end, self.nnz_begin, self.nnz_end = 0, self.m, 0, self.nnz
        self._dkkt = None
        self._vbuf = None      # this rank's device slice buffer (transport "device")
        self.closed = False
        self.error = None      # serving ranks: the first evaluation failure (answered with NaN)

    def __getattr__(self, name):
        # problem attributes (opts, G, NS, NC, rep, NSL, NEP, tail_rows, ...)
        # are the shard context's: the same problem, whole
        if name.startswith("__") or name == "shard":
            raise AttributeError(name)
        return getattr(self.shard, name)

    # -- the protocol ----------------------------------------------------------
    def _tensor(self, a, dtype=None):
        t = self.torch
        return t.as_tensor(np.ascontiguousarray(a), dtype=dtype or t.float64).to(self.device)

    def _request(self, op: int, x):
        """Rank 0: op code and iterate to every rank."""
        t = self.torch
        self.dist.broadcast(t.tensor([op], dtype=t.int64, device=self.device), 0)
        if op != OP_STOP:
            xt = self._tensor(x)
            self.dist.broadcast(xt, 0)
            return xt
        return None

    def _receive(self):
        """Ranks > 0: the next (op, x as a tensor on self.device)."""
        t = self.torch
        hdr = t.zeros(1, dtype=t.int64, device=self.device)
        self.dist.broadcast(hdr, 0)
        op = int(hdr.item())
        if op == OP_STOP:
            return op, None
        xt = t.zeros(self.n, dtype=t.float64, device=self.device)
        self.dist.broadcast(xt, 0)
        return op, xt

    def _sum_to_root(self, a) -> np.ndarray:
        t = self._tensor(a)
        self.dist.reduce(t, 0, op=self.dist.ReduceOp.SUM)
        return t.cpu().numpy()

    def _gather_slices(self, own, which: int, out):
        """Rank 0: its own slice into ``out`` (a float64 tensor of the whole
        vector), the other ranks' slices received into their offsets."""
        b0, e0 = self.ranges[0][which], self.ranges[0][which + 1]
        out[b0:e0] = self._tensor(own) if not isinstance(own, self.torch.Tensor) else own
        # the other ranks' slices as one grouped batch of receives (they run
        # concurrently, each from its own peer)
        ops = []
        for r in range(1, self.world):
            b, e = self.ranges[r][which], self.ranges[r][which + 1]
            if e > b:
                ops.append(self.dist.P2POp(self.dist.irecv, out[b:e], r))
        for q in (self.dist.batch_isend_irecv(ops) if ops else []):
            q.wait()
        return out

    def _send_slice(self, v):
        if len(v):
            self.dist.send(v if isinstance(v, self.torch.Tensor) else self._tensor(v), dst=0)

    # -- rank 0: the NLP the optimizer sees -------------------------------------
    def eval_f(self, x, new_x=True):
        self._request(OP_F, x)
        return float(self._sum_to_root([self.shard.eval_f_partial(x)])[0])

    def eval_grad_f(self, x, new_x=True):
        self._request(OP_GRAD, x)
        return self._sum_to_root(self.shard.eval_grad_f_partial(x))

    def eval_g(self, x, new_x=True):
        self._request(OP_G, x)
        out = self.torch.zeros(self.m, dtype=self.torch.float64, device=self.device)
        return self._gather_slices(self.shard.eval_g(x), 0, out).cpu().numpy()

    def eval_jac_g(self, x, new_x=True):
        self._request(OP_JAC, x)
        out = self.torch.zeros(self.nnz, dtype=self.torch.float64, device=self.device)
        return self._gather_slices(self.shard.eval_jac_g(x), 2, out).cpu().numpy()

    def device_kkt(self, warm: bool = False):
        """The device KKT module on rank 0's GPU over the WHOLE Jacobian
        (mocohip.kkt.ShardedDeviceKKT).  ValueError where the shards are not
        device contexts (the optimizer then takes its host linear algebra)."""
        if not hasattr(self.shard, "eval_jac_g_device"):
            raise ValueError("device_kkt needs HipNLP shards")
        if self._dkkt is None:
            from .kkt import ShardedDeviceKKT
            dk = ShardedDeviceKKT(self)
            if warm:
                dk.warm(self.initial_guess_from_bounds())
            self._dkkt = dk
        return self._dkkt

    def close(self):
        """Rank 0: release the other ranks from serve()."""
        if self.rank == 0 and not self.closed:
            self._request(OP_STOP, None)
        self.closed = True
        if self._dkkt is not None:
            self._dkkt.close()
            self._dkkt = None

    # -- ranks > 0 -----------------------------------------------------------------
    def serve(self) -> int:
        """Answer rank 0's requests until it closes; returns the number of
        requests served."""
        t = self.torch
        served = 0
        while True:
            op, xt = self._receive()
            if op == OP_STOP:
                self.closed = True
                return served
            served += 1
            try:
                self._answer(op, xt)
            except Exception as e:   # noqa: BLE001 -- keep the protocol (and rank 0) going
                if self.error is None:
                    self.error = f"rank {self.rank}, request {op}: {type(e).__name__}: {e}"
                self._answer_nan(op)

    def _answer_nan(self, op):
        """The reply to a request whose evaluation failed: NaN of the reply's
        shape (the optimizer sees a non-finite value and stops)."""
        if op in (OP_F, OP_GRAD):
            self._sum_to_root(np.full(1 if op == OP_F else self.n, np.nan))
        elif op == OP_G:
            self._send_slice(np.full(self.shard.row_end - self.shard.row_begin, np.nan))
        elif op in (OP_JAC, OP_JAC_DEV):
            self._send_slice(np.full(self.shard.nnz_end - self.shard.nnz_begin, np.nan))

    def _answer(self, op, xt):
        t = self.torch
        if op == OP_JAC_DEV and self.transport == "device":
            # the slice stays on the GPU: evaluated into a device buffer
            # on a dedicated stream, sent GPU to GPU from that stream
            if self._vbuf is None:
                self._vbuf = t.zeros(max(1, self.shard.nnz_end - self.shard.nnz_begin),
                                     dtype=t.float64, device=self.device)
                self._stream = t.cuda.Stream(device=self.device)
                self.shard.set_stream(self._stream.cuda_stream)
            self._stream.wait_stream(t.cuda.current_stream(self.device))   # x has arrived
            with t.cuda.stream(self._stream):
                self.shard.eval_jac_g_device(xt.data_ptr(), self._vbuf.data_ptr())
                self._send_slice(self._vbuf[:self.shard.nnz_end - self.shard.nnz_begin])
            return
        x = xt.cpu().numpy()
        if op == OP_F:
            self._sum_to_root([self.shard.eval_f_partial(x)])
        elif op == OP_GRAD:
            self._sum_to_root(self.shard.eval_grad_f_partial(x))
        elif op == OP_G:
            self._send_slice(self.shard.eval_g(x))
        elif op in (OP_JAC, OP_JAC_DEV):
            self._send_slice(self.shard.eval_jac_g(x))
        else:
            raise RuntimeError(f"unknown request {op}")
