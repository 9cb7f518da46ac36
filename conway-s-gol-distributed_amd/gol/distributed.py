"""Row-strip decomposition of one board over torch.distributed ranks.

The reference splits the board's rows over ``len(SUB)`` SubServers with
base = H/N rows each and the first H%N strips one row more
(``Server/gol/distributor.go:106-116``), and every turn ships each strip plus one
halo row above and below through the Server (``:185-224``).  Here every rank
keeps its strip resident on its own MI355X with ``halo`` = K extra rows above and
below, runs K turns locally (the valid region shrinks by one row per turn), and
then exchanges only the K boundary rows with its ring neighbours
(r-1) mod N and (r+1) mod N — RCCL send/recv over xGMI on GPUs, gloo on CPU for
tests.  On GPUs the messages are the board rows themselves (zero-copy views,
``gol_halo_buffers``) and the sends/receives are enqueued by direct RCCL calls on
the engine's stream (``gol.rccl``); torch's ``batch_isend_irecv`` remains as the
alternative transport.  Results are identical to the single-GPU torus for any N
because the rows owned after every K-turn block are exactly the torus rows.

Message order is the same on every rank — send-up, recv-from-down, send-down,
recv-from-up — so FIFO matching between a pair of ranks is correct even for N=2,
where the up and the down neighbour are the same rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import Engine, strip_split

TAG_UP = 17      # rows travelling to the upper neighbour (they become its bottom halo)
TAG_DOWN = 18    # rows travelling to the lower neighbour (they become its top halo)


class _DeviceRows:
    """``__cuda_array_interface__`` view of ``shape`` int64 words at a device pointer the
    engine owns (torch.as_tensor wraps it without a copy)."""

    def __init__(self, ptr: int, shape):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": "<i8",
                                         "data": (int(ptr), False), "version": 2,
                                         "strides": None}


class EngineStrip:
    """Adapter exposing an Engine strip to the exchange loop with torch tensors.

    The engine and the halo messages share one dedicated torch stream, so the RCCL
    send/recv that torch enqueues are ordered after the engine's turns and before its
    next ones without host synchronisation.

    ``zero_copy`` (default): the messages are views of the engine's own board rows
    (``gol_halo_buffers``) -- RCCL reads the boundary rows and writes the halo rows in
    place, in the engine's stepping layout, so an exchange launches nothing but the
    transport.  Otherwise the rows are copied through separate buffers in the standard
    layout (``gol_export_halo`` / ``gol_import_halo``)."""

    def __init__(self, engine: Engine, device: torch.device, stream=None,
                 zero_copy: bool = True):
        self.engine = engine
        self.device = device
        self.stream = stream if stream is not None else torch.cuda.Stream(device)
        engine.set_stream(self.stream.cuda_stream)
        self.zero_copy = bool(zero_copy)
        self.layout = None
        self._views = None
        K, nw = engine.halo, engine.words_per_row
        self._shape = (K, nw)
        if not self.zero_copy:
            mk = lambda: torch.empty((K, nw), dtype=torch.int64, device=device)  # noqa: E731
            self.top_send, self.bot_send, self.top_recv, self.bot_recv = mk(), mk(), mk(), mk()

    @property
    def halo_valid(self) -> int:
        return self.engine.halo_valid

    def step(self, n: int):
        self._views = None                     # board pointers move with every step
        self.engine.step(n)

    def step_overlap(self, n: int, recv_stream_ptr: int):
        self._views = None
        self.engine.step_overlap(n, recv_stream_ptr)

    def stream_context(self):
        return torch.cuda.stream(self.stream)

    def _board_views(self):
        if self._views is None:
            ptrs, self.layout = self.engine.halo_buffers()
            self._views = tuple(torch.as_tensor(_DeviceRows(p, self._shape), device=self.device)
                                for p in ptrs)
        return self._views

    def export_rows(self):
        if self.zero_copy:
            st, sb, _, _ = self._board_views()
            return st, sb
        s = self.stream.cuda_stream
        self.engine.export_halo(self.top_send.data_ptr(), self.bot_send.data_ptr(), s)
        return self.top_send, self.bot_send

    def recv_buffers(self):
        if self.zero_copy:
            _, _, rt, rb = self._board_views()
            return rt, rb
        return self.top_recv, self.bot_recv

    def import_rows(self, top, bottom):
        if self.zero_copy:
            _, _, rt, rb = self._board_views()
            if top.data_ptr() != rt.data_ptr():
                rt.copy_(top, non_blocking=True)
            if bottom.data_ptr() != rb.data_ptr():
                rb.copy_(bottom, non_blocking=True)
            self.engine.halo_done()
            return
        s = self.stream.cuda_stream
        if top.device != self.device:
            self.top_recv.copy_(top, non_blocking=True)
            self.bot_recv.copy_(bottom, non_blocking=True)
            top, bottom = self.top_recv, self.bot_recv
        self.engine.import_halo(top.data_ptr(), bottom.data_ptr(), s)


class DistStrip:
    """One rank's strip; ``step(turns)`` interleaves local turns and halo exchanges."""

    def __init__(self, strip, rank: int, world: int, group=None, stage_on_host: bool = False,
                 rccl=None, overlap: bool = False):
        """``rccl``: a gol.rccl.RcclComm -- the exchange is enqueued by direct RCCL calls on
        the strip's own stream (no cross-stream waits); None = torch.distributed
        point-to-point (batch_isend_irecv on the nccl backend, isend/irecv on gloo).
        ``overlap`` (direct RCCL, zero-copy strips only): the sends and receives run on a
        stream of their own while the first launch's interior rows compute
        (gol_stream_wait / gol_step_overlap); the rows next to the halos follow the
        receives."""
        self.strip = strip
        self.rccl = rccl
        self.overlap = bool(overlap and rccl is not None and getattr(strip, "zero_copy", False))
        self.comm_stream = torch.cuda.Stream(strip.device) if self.overlap else None
        self.rank, self.world = int(rank), int(world)
        self.up = (self.rank - 1) % self.world
        self.down = (self.rank + 1) % self.world
        self.group = group
        # gloo cannot move device tensors: stage the K-row messages through host memory
        self.stage_on_host = stage_on_host
        self.exchanges = 0
        self._layout_checked = False
        self._stale = False            # start_window(): the next step exchanges first
        self._ev_pool = []             # time_exchanges(): HIP event pairs not yet used
        self._ev_used = []
        self._ptrs = None              # start_window(): the board rows' pointers, until a step

    def start_window(self):
        """Make the next ``step`` begin with an exchange, whatever turns its halos have left:
        a timed region that starts here holds exactly one exchange per ``halo`` turns (the
        run's cadence), not a partial window left over from the warm-up.  (An exchange is
        valid at any turn: the neighbours' owned rows are exact.)  On the direct RCCL path the
        board rows' device pointers are looked up here already (they stay valid until the next
        step), so the exchange that opens the window only enqueues."""
        self._stale = True
        if self.rccl is not None and getattr(self.strip, "zero_copy", False) and not self.overlap:
            self._ptrs = self.strip.engine.halo_buffers()

    def time_exchanges(self, n: int):
        """Bracket each of the next ``n`` exchanges with a HIP event pair on the stream the
        transport runs on (created and recorded once here, so the timed region only records
        them): ``exchange_us()`` then gives each exchange's duration -- the transfer plus
        any wait for the neighbours, as the stream saw it."""
        stream = getattr(self.strip, "stream", None)
        if stream is None:
            return
        self._ev_pool, self._ev_used = [], []
        for _ in range(int(n)):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(stream)
            b.record(stream)
            self._ev_pool.append((a, b))
        stream.synchronize()

    def exchange_us(self):
        """Durations (us) of the exchanges timed since ``time_exchanges`` (synchronises)."""
        if not self._ev_used:
            return []
        self._ev_used[-1][1].synchronize()
        return [a.elapsed_time(b) * 1e3 for a, b in self._ev_used]

    def _ev_begin(self, stream):
        if not self._ev_pool:
            return None
        pair = self._ev_pool.pop()
        pair[0].record(stream)
        return pair

    def _ev_end(self, pair, stream):
        if pair is not None:
            pair[1].record(stream)
            self._ev_used.append(pair)

    def exchange(self):
        self._stale = False
        stream = getattr(self.strip, "stream", None)
        pair = self._ev_begin(stream) if stream is not None else None
        if self.rccl is not None and getattr(self.strip, "zero_copy", False):
            self._exchange_rccl_direct()
        else:
            ctx = getattr(self.strip, "stream_context", None)
            if ctx is None:
                self._exchange()
            else:
                with ctx():
                    self._exchange()
        if stream is not None:
            self._ev_end(pair, stream)

    def _exchange_rccl_direct(self):
        """The bench's exchange (direct RCCL, zero-copy board rows): four device pointers from
        gol_halo_buffers straight into one RCCL group on the engine's stream, then
        gol_halo_done -- no torch tensor views and no stream context, because a timed window
        starts with this call on an idle GPU and every microsecond of host work before the
        first enqueue is in the window (tools/xchg_overhead.py: ~29 us through the tensor path
        at the 8-strip shape)."""
        eng = self.strip.engine
        ptrs, self._ptrs = self._ptrs, None
        (st, sb, rt, rb), lay = ptrs if ptrs is not None else eng.halo_buffers()
        self.strip.layout = lay
        if not self._layout_checked:
            self._check_layout_value(lay, self.strip.device)
        self.rccl.exchange(((st, self.up), (sb, self.down)), ((rb, self.down), (rt, self.up)),
                           self._nbytes(eng), self.strip.stream.cuda_stream)
        eng.halo_done()
        self.exchanges += 1

    def _nbytes(self, eng):
        n = getattr(self, "_msg_bytes", None)
        if n is None:
            n = self._msg_bytes = int(eng.halo) * int(eng.words_per_row) * 8
        return n

    def _check_layout(self, like):
        """Zero-copy messages carry the engines' stepping layout: every rank must agree
        (equal width, halo and flags guarantee it; checked once, before the first
        exchange, with one tiny all-reduce)."""
        self._check_layout_value(getattr(self.strip, "layout", None), like.device)

    def _check_layout_value(self, lay, device):
        self._layout_checked = True
        if lay is None:
            return
        dev = device if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([lay], dtype=torch.int64, device=dev)
        dist.all_reduce(t, group=self.group)
        if int(t.item()) not in (0, self.world):
            raise RuntimeError(f"rank {self.rank}: halo layouts differ across ranks "
                               f"(sum {int(t.item())} of {self.world})")

    def _exchange(self):
        top, bot = self.strip.export_rows()
        top_recv, bot_recv = self.strip.recv_buffers()
        if not self._layout_checked:
            self._check_layout(top)
        if self.rccl is not None:
            nbytes = top.numel() * top.element_size()
            self.rccl.exchange([(top.data_ptr(), self.up), (bot.data_ptr(), self.down)],
                               [(bot_recv.data_ptr(), self.down), (top_recv.data_ptr(), self.up)],
                               nbytes, self.strip.stream.cuda_stream)
            self.strip.import_rows(top_recv, bot_recv)
            self.exchanges += 1
            return
        if self.stage_on_host:
            top, bot = top.cpu(), bot.cpu()
            top_recv, bot_recv = torch.empty_like(top), torch.empty_like(bot)
        if dist.get_backend(self.group) == "nccl":
            ops = [dist.P2POp(dist.isend, top, self.up, self.group),
                   dist.P2POp(dist.irecv, bot_recv, self.down, self.group),
                   dist.P2POp(dist.isend, bot, self.down, self.group),
                   dist.P2POp(dist.irecv, top_recv, self.up, self.group)]
            reqs = dist.batch_isend_irecv(ops)
        else:
            reqs = [dist.isend(top, self.up, self.group, tag=TAG_UP),
                    dist.irecv(bot_recv, self.down, self.group, tag=TAG_UP),
                    dist.isend(bot, self.down, self.group, tag=TAG_DOWN),
                    dist.irecv(top_recv, self.up, self.group, tag=TAG_DOWN)]
        for r in reqs:
            r.wait()
        self.strip.import_rows(top_recv, bot_recv)
        self.exchanges += 1

    def _exchange_overlapped(self, turns: int):
        """Exchange on the comm stream and advance `turns` (<= halo) turns, the first
        launch's interior rows concurrently with the transfer."""
        top, bot = self.strip.export_rows()
        top_recv, bot_recv = self.strip.recv_buffers()
        if not self._layout_checked:
            self._check_layout(top)
        eng = self.strip.engine
        cs = self.comm_stream.cuda_stream
        eng.stream_wait(cs)                     # the send rows are final
        nbytes = top.numel() * top.element_size()
        pair = self._ev_begin(self.comm_stream)
        self.rccl.exchange([(top.data_ptr(), self.up), (bot.data_ptr(), self.down)],
                           [(bot_recv.data_ptr(), self.down), (top_recv.data_ptr(), self.up)],
                           nbytes, cs)
        self._ev_end(pair, self.comm_stream)
        self.strip.step_overlap(turns, cs)
        self._stale = False
        self.exchanges += 1

    def step(self, turns: int):
        turns = int(turns)
        hv = None                               # turns the halos have left (queried once)
        while turns > 0:
            if hv is None:
                hv = self.strip.halo_valid
            if hv == 0 or self._stale:
                if self.overlap:
                    n = min(turns, self.strip.engine.halo)
                    self._ptrs = None
                    self._exchange_overlapped(n)
                    turns -= n
                    hv = None
                    continue
                self.exchange()
                # (fresh halos: an engine strip's depth, without another query)
                eng = getattr(self.strip, "engine", None)
                hv = int(eng.halo) if eng is not None else self.strip.halo_valid
            n = min(turns, hv)
            self._ptrs = None                   # (the board moves: pointers from before are stale)
            self.strip.step(n)
            turns -= n
            hv -= n


def make_engine_strip(width: int, height: int, rank: int, world: int, halo: int,
                      device_index: int, **engine_kw):
    """Engine for rank's strip (Server split) with halo depth min(halo, rows)."""
    off, rows = strip_split(height, world)[rank]
    min_rows = min(r for _, r in strip_split(height, world))
    K = max(1, min(int(halo), min_rows))
    eng = Engine(width, height, device=device_index, row_offset=off, rows=rows, halo=K,
                 **engine_kw)
    return eng
