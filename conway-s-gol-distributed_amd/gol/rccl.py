"""Direct RCCL point-to-point for the halo exchange, on the engine's own HIP stream.

``torch.distributed``'s ``batch_isend_irecv`` runs RCCL on ProcessGroupNCCL's internal
stream, so every exchange costs two cross-stream event waits (engine stream -> RCCL
stream -> engine stream).  Measured on MI355X at the 65536^2 / 8-strip shape
(tools/strip_emulate.py --rccl, rocprofv3 kernel trace): 31 us idle before the RCCL
kernel and 16 us after it, around a 14 us transfer kernel.  Here the sends and
receives are enqueued by ``ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd`` straight
onto the stream the stencil launches run on: the exchange is one more kernel in the
stream, ordered by the stream itself.

The library is the RCCL that torch already loaded (``torch/lib/librccl.so``), so there is
one RCCL in the process.  The communicator is our own: rank 0's ``ncclGetUniqueId`` is
broadcast over the existing torch.distributed group (a 128-byte tensor) and every rank
calls ``ncclCommInitRankConfig``.  It replaces the reference's per-turn net/rpc strip transfer
(``Server/gol/distributor.go:185-224``).

The communicator is created non-blocking (``ncclConfig_t.blocking = 0``) and its state polled
against a deadline (``GOL_RCCL_INIT_TIMEOUT_S``, default 60 s): a bootstrap that cannot connect
(a wrong root address, a rank that never arrives) aborts the communicator and raises
``RcclTimeout`` on every rank within the deadline instead of hanging the job -- the reference
Server's dial-or-fatal (``Server/gol/distributor.go:87-97``).  Only this communicator is
non-blocking; torch's own keep their configuration.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time

import torch
import torch.distributed as dist

NCCL_INT8 = 0                       # ncclInt8 (messages are raw packed words, sent as bytes)
NCCL_IN_PROGRESS = 7                # ncclInProgress (a non-blocking communicator's pending state)
_UID_BYTES = 128                    # NCCL_UNIQUE_ID_BYTES
_CONFIG_MAGIC = 0xCAFEBEEF
_UNDEF_INT = -2147483648            # NCCL_CONFIG_UNDEF_INT (INT_MIN)


class RcclTimeout(RuntimeError):
    """The communicator did not come up (or a group did not complete) within the deadline;
    the communicator was aborted.  Not a reason to fall back to another transport: the peer
    ranks are unreachable for that one too."""


class _Config(ctypes.Structure):
    """The leading fields of ncclConfig_t (NCCL 2.17 layout, ``size`` = this struct's size):
    the library copies ``size`` bytes and keeps its defaults for the fields after them."""
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int),
                ("minCTAs", ctypes.c_int), ("maxCTAs", ctypes.c_int),
                ("netName", ctypes.c_char_p), ("splitShare", ctypes.c_int)]


def nonblocking_config(version: int) -> _Config:
    """NCCL_CONFIG_INITIALIZER with blocking = 0 (the library's own version in ``version``)."""
    c = _Config()
    c.size = ctypes.sizeof(_Config)
    c.magic = _CONFIG_MAGIC
    c.version = int(version)
    c.blocking = 0
    c.cgaClusterSize = c.minCTAs = c.maxCTAs = c.splitShare = _UNDEF_INT
    c.netName = None
    return c


def init_timeout_s() -> float:
    v = os.environ.get("GOL_RCCL_INIT_TIMEOUT_S", "")
    try:
        return max(1.0, float(v)) if v else 60.0
    except ValueError:
        return 60.0


class _UniqueId(ctypes.Structure):
    # c_ubyte, not c_char: a c_char array field reads back as a NUL-terminated string, and an
    # RCCL unique id ({uint64 magic; sockaddr root}) holds NULs from byte 2 of the sockaddr on
    # (AF_INET = 02 00), so a c_char field cut every id before the root's port and address
    _fields_ = [("internal", ctypes.c_ubyte * _UID_BYTES)]


def uid_to_bytes(uid: _UniqueId) -> bytes:
    """All NCCL_UNIQUE_ID_BYTES bytes of ``uid``, NULs included."""
    return ctypes.string_at(ctypes.addressof(uid), _UID_BYTES)


def uid_from_bytes(data) -> _UniqueId:
    """A unique id holding exactly ``data`` (NCCL_UNIQUE_ID_BYTES bytes)."""
    data = bytes(data)
    if len(data) != _UID_BYTES:
        raise ValueError(f"unique id must be {_UID_BYTES} bytes, got {len(data)}")
    uid = _UniqueId()
    ctypes.memmove(ctypes.addressof(uid), data, _UID_BYTES)
    return uid


def broadcast_unique_id(uid: _UniqueId, group=None, where="cpu") -> _UniqueId:
    """Rank 0's ``uid`` on every rank of ``group`` (a collective: every rank calls it; the
    other ranks' ``uid`` is ignored).  ``where`` is the device the group's backend moves
    tensors on ("cpu" for gloo, the rank's GPU for nccl).  Byte-exact: the id travels as a
    128-element uint8 tensor, never as a string."""
    t = torch.tensor(list(uid_to_bytes(uid)), dtype=torch.uint8, device=where)
    dist.broadcast(t, src=0, group=group)
    return uid_from_bytes(bytes(t.cpu().tolist()))


_lib = None


def lib() -> ctypes.CDLL:
    """torch's bundled librccl.so (already mapped by torch; CDLL returns that handle)."""
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        L = ctypes.CDLL(path)
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), i32, _UniqueId, i32]
        L.ncclCommInitRankConfig.argtypes = [ctypes.POINTER(vp), i32, _UniqueId, i32,
                                             ctypes.POINTER(_Config)]
        L.ncclCommGetAsyncError.argtypes = [vp, ctypes.POINTER(i32)]
        L.ncclCommAbort.argtypes = [vp]
        L.ncclCommDestroy.argtypes = [vp]
        L.ncclSend.argtypes = [vp, sz, i32, i32, vp, vp]
        L.ncclRecv.argtypes = [vp, sz, i32, i32, vp, vp]
        L.ncclGroupStart.argtypes = []
        L.ncclGroupEnd.argtypes = []
        L.ncclGetErrorString.argtypes = [i32]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        L.ncclGetVersion.argtypes = [ctypes.POINTER(i32)]
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommInitRankConfig",
                  "ncclCommGetAsyncError", "ncclCommAbort", "ncclCommDestroy", "ncclSend",
                  "ncclRecv", "ncclGroupStart", "ncclGroupEnd", "ncclGetVersion"):
            getattr(L, f).restype = i32
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().ncclGetErrorString(rc)
        raise RuntimeError(f"{what}: RCCL error {rc} ({msg.decode() if msg else '?'})")


def version() -> int:
    v = ctypes.c_int()
    _check(lib().ncclGetVersion(ctypes.byref(v)), "ncclGetVersion")
    return int(v.value)


class RcclComm:
    """One RCCL communicator over the ranks of ``group`` (collective constructor: every
    rank must create it, with its HIP device current)."""

    def __init__(self, rank: int, world: int, device: torch.device, group=None,
                 uid_hook=None):
        """``uid_hook`` (tests only): a function applied to this rank's copy of the unique
        id's bytes after the broadcast -- e.g. a wrong root port, to exercise the deadline."""
        self.rank, self.world = int(rank), int(world)
        self.comm = ctypes.c_void_p()
        uid = _UniqueId()
        err = None
        try:
            L = lib()
            if self.rank == 0:
                _check(L.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        except (OSError, AttributeError, RuntimeError) as e:   # no library / symbol / uid
            err = e
        if self.world > 1:
            on_dev = dist.get_backend(group) == "nccl"
            where = device if on_dev else "cpu"
            # every rank learns whether every rank has a library (and rank 0 a unique id)
            # before anyone blocks in the broadcast or in ncclCommInitRank
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=where)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
            if int(ok.item()) == 0:
                raise RuntimeError(f"rank {self.rank}: direct RCCL unavailable on some rank"
                                   + (f" ({err})" if err else ""))
            uid = broadcast_unique_id(uid, group, where)
            if uid_hook is not None:
                uid = uid_from_bytes(uid_hook(uid_to_bytes(uid)))
        elif err is not None:
            raise RuntimeError(f"direct RCCL unavailable ({err})")
        self.timeout_s = init_timeout_s()
        cfg = nonblocking_config(version())
        t0 = time.monotonic()
        with torch.cuda.device(device):
            rc = L.ncclCommInitRankConfig(ctypes.byref(self.comm), self.world, uid, self.rank,
                                          ctypes.byref(cfg))
            if rc not in (0, NCCL_IN_PROGRESS):
                self._abort()
                _check(rc, "ncclCommInitRankConfig")
            self._wait("ncclCommInitRankConfig", t0)
        self.init_s = time.monotonic() - t0

    def _state(self) -> int:
        st = ctypes.c_int(0)
        rc = lib().ncclCommGetAsyncError(self.comm, ctypes.byref(st))
        return rc if rc != 0 else int(st.value)

    def _abort(self):
        """ncclCommAbort on a helper thread, given 10 s: an abort that itself hangs must not
        keep the caller from failing."""
        if not self.comm:
            return
        comm, self.comm = self.comm, ctypes.c_void_p()
        th = threading.Thread(target=lambda: lib().ncclCommAbort(comm), daemon=True)
        th.start()
        th.join(10.0)

    def _wait(self, what: str, t0: float):
        """Poll the communicator until its pending operation is done; abort and raise
        RcclTimeout past the deadline, RuntimeError on an RCCL error."""
        while True:
            st = self._state()
            if st == 0:
                return
            if st != NCCL_IN_PROGRESS:
                self._abort()
                _check(st, what)
            if time.monotonic() - t0 > self.timeout_s:
                self._abort()
                raise RcclTimeout(f"rank {self.rank}: {what} did not complete within "
                                  f"{self.timeout_s:g} s (GOL_RCCL_INIT_TIMEOUT_S); communicator "
                                  f"aborted")
            time.sleep(0.0005)

    def exchange(self, sends, recvs, nbytes: int, stream_ptr: int):
        """One group of point-to-point ops on ``stream_ptr``: ``sends`` / ``recvs`` are
        lists of (device pointer, peer), enqueued in the interleaved order
        send[0], recv[0], send[1], recv[1], ... -- the same on every rank, so FIFO
        matching between a pair of ranks holds even when both neighbours are one rank."""
        L = lib()
        s = ctypes.c_void_p(int(stream_ptr))
        comm, send, recv = self.comm, L.ncclSend, L.ncclRecv
        rc = L.ncclGroupStart()
        if rc != 0:
            _check(rc, "ncclGroupStart")
        try:
            for (sp, speer), (rp, rpeer) in zip(sends, recvs):
                rc = send(sp, nbytes, NCCL_INT8, speer, comm, s)
                if rc != 0:
                    _check(rc, "ncclSend")
                rc = recv(rp, nbytes, NCCL_INT8, rpeer, comm, s)
                if rc != 0:
                    _check(rc, "ncclRecv")
        finally:
            rc = L.ncclGroupEnd()
        if rc not in (0, NCCL_IN_PROGRESS):
            _check(rc, "ncclGroupEnd")
        if rc == NCCL_IN_PROGRESS or self._state() != 0:
            # (non-blocking communicator: the first group also connects the peers; the ops are
            # on the stream once the state is ncclSuccess, so the caller's next launch on the
            # same stream -- and the next RCCL call -- come after them)
            self._wait("ncclGroupEnd", time.monotonic())

    def close(self):
        if self.comm:
            lib().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
