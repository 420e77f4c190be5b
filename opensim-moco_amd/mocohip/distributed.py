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
