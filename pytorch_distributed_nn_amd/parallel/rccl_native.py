"""Bucket all-reduces straight through RCCL (SURVEY.md §5.8 comm backend; reference bucket reduction:
pytorch_code/data_parallel_dist/data_parallel_dist.py:238-267).

``ProcessGroupNCCL`` orders every collective after the issuing stream by recording a default HIP event there and
making its own stream wait on it.  A default event's record is a system-scope release (cache write-back +
invalidate when the command processor reaches it): measured ~21 us of the issuing stream per bucket collective
(GPT-2 DDP path kernel trace, gpurun_out/r5_40; 603.0k -> 616.4k tok/s going from 13 to 2 buckets, r5_44).

:class:`NativeComm` issues ``ncclAllReduce`` itself, in place, on a stream it owns, ordered after the issuing
stream by the framework's fence-free events (``kernels.stream_wait``: ``hipEventDisableSystemFence``,
csrc/kernels/streams.hip), and joins back the same way.  The communicator is a second RCCL communicator over the
same ranks (unique id broadcast over the process group), created on the RCCL library torch already loaded.

Opt-in (``DistributedDataParallel(native_comm=True)`` or ``PDNN_DDP_NATIVE_COMM=1``): at world size > 1 it has
not been run on this project's one-GPU boxes; the torch process group still carries the BN-buffer broadcasts and
the straggler counts.  Measured at world 1 (gpurun_out/r5_48, same box): GPT-2 with 13 bucket collectives 608.8k
vs 606.7k tok/s (ProcessGroupNCCL), with 128 MB buckets 612.5k vs 616.9k; ResNet-50, whose collectives are
issued from the weight-gradient side stream, 8,184 vs 11,598 img/s -- not understood yet: the kernel trace
(gpurun_out/r5_49) shows no RCCL kernel at world 1, but the step's own kernels run slower (39.8 vs 34.2 ms of
kernel time over the two streams, span 29.4 vs 22.4 ms), and with the weight gradients on the compute stream
(tuning side_wgrad=0) the native path matches ProcessGroupNCCL (10,031 vs 10,095 img/s, r5_53): the loss comes
from its interplay with the two-stream schedule.  Hence off by default.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

NCCL_SUM, NCCL_AVG = 0, 4
_DT = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6}


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def _lib():
    d = os.path.join(os.path.dirname(torch.__file__), "lib")
    for name in ("librccl.so", "librccl.so.1"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            return ctypes.CDLL(p)
    return ctypes.CDLL("librccl.so")


class _Work:
    """Completion of one native collective: ``wait()`` orders the caller's current stream after it (no host
    block), like ``Work.wait()`` of a ProcessGroupNCCL collective."""

    def __init__(self, comm):
        self._comm = comm

    def wait(self):
        from ..ops import kernels as K
        K.stream_wait(torch.cuda.current_stream(self._comm.device), self._comm.stream)
        return True

    def is_completed(self):
        return self._comm.stream.query()


class NativeComm:
    def __init__(self, pg, device: torch.device):
        self.lib = _lib()
        self.lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        self.lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        self.lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        self.lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        self.device = device
        self.rank = dist.get_rank(pg)
        self.world = dist.get_world_size(pg)
        uid = _UniqueId()
        if self.rank == 0:
            self._check(self.lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        # all 128 bytes (``uid.internal`` as a c_char array would stop at the first NUL of the socket address)
        buf = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(uid), 128)), dtype=torch.uint8).to(device)
        dist.broadcast(buf, 0, group=pg)
        raw = bytes(buf.cpu().tolist())
        ctypes.memmove(ctypes.addressof(uid), raw, 128)
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(device):
            self._check(self.lib.ncclCommInitRank(ctypes.byref(self.comm), self.world, uid, self.rank),
                        "ncclCommInitRank")
        self.stream = torch.cuda.Stream(device=device)

    @staticmethod
    def _check(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: ncclResult {rc}")

    def all_reduce(self, t: torch.Tensor, avg: bool) -> _Work:
        """In-place all-reduce of the contiguous CUDA tensor ``t`` (SUM, or AVG with ``avg``), ordered after
        everything enqueued so far on the current stream."""
        from ..ops import kernels as K
        if t.dtype not in _DT or not t.is_contiguous():
            raise ValueError("NativeComm.all_reduce: contiguous fp32 / bf16 / fp16 tensor")
        K.stream_wait(self.stream, torch.cuda.current_stream(t.device))
        self._check(self.lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                           NCCL_AVG if avg else NCCL_SUM, self.comm, self.stream.cuda_stream),
                    "ncclAllReduce")
        return _Work(self)

    def close(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
