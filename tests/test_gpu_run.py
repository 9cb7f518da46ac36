"""gol.Run (C++ driver over the HIP engine) against the reference's own tests.

Mirrors Local/gol_test.go (TestGol), Local/pgm_test.go (TestPgm) and
Local/count_test.go (TestAlive), plus the event sequence of
Local/gol/distributor.go:180-226 and the key handling of :107-152.
"""
import os
import time

import numpy as np
import pytest

import golden_data as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gol():
    import gol as g
    return g


@pytest.fixture()
def workdir(tmp_path):
    img = tmp_path / "images"
    img.mkdir()
    for s in (16, 64, 128, 256, 512):
        (img / f"{s}x{s}.pgm").write_bytes(G.input_pgm_bytes(s))
    return tmp_path


def run_collect(gol, p, workdir, keys=None, **kw):
    events = gol.Channel()
    h = gol.Run(p, events, keys, image_dir=str(workdir / "images"),
                out_dir=str(workdir / "out"), **kw)
    evs = list(events)
    h.wait(5)
    assert h.error is None, h.error
    return evs


def read_alive_cells(path, w, h):
    """util.ReadAliveCells (Local/util/cell.go:14-56): cells whose byte != 0."""
    b = G.parse_pgm(open(path, "rb").read())
    assert b.shape == (h, w)
    ys, xs = np.nonzero(b)
    return set(zip(xs.tolist(), ys.tolist()))


@pytest.mark.parametrize("size", (16, 64, 512))
@pytest.mark.parametrize("turns", (0, 1, 100))
@pytest.mark.parametrize("threads", (1, 8, 16))
def test_gol_and_pgm(gol, workdir, size, turns, threads):
    """TestGol (FinalTurnComplete.Alive) and TestPgm (out/WxHxT.pgm) in one run."""
    p = gol.Params(Turns=turns, Threads=threads, ImageWidth=size, ImageHeight=size)
    evs = run_collect(gol, p, workdir)
    final = [e for e in evs if isinstance(e, gol.FinalTurnComplete)]
    assert len(final) == 1
    expected = read_alive_cells_bytes(G.check_pgm_bytes(size, turns))
    assert set((c.X, c.Y) for c in final[0].Alive) == expected
    assert len(final[0].Alive) == len(expected)
    out = workdir / "out" / f"{size}x{size}x{turns}.pgm"
    # byte-identical to the reference writer's output (= the check image)
    assert out.read_bytes() == G.check_pgm_bytes(size, turns)


def read_alive_cells_bytes(data):
    b = G.parse_pgm(data)
    ys, xs = np.nonzero(b)
    return set(zip(xs.tolist(), ys.tolist()))


def test_event_sequence(gol, workdir):
    p = gol.Params(Turns=10, Threads=4, ImageWidth=64, ImageHeight=64)
    evs = run_collect(gol, p, workdir)
    kinds = [type(e).__name__ for e in evs]
    assert kinds[0] == "StateChange" and evs[0].NewState == gol.State.Executing
    assert evs[0].CompletedTurns == 0
    tc = [e.CompletedTurns for e in evs if isinstance(e, gol.TurnComplete)]
    assert tc == list(range(1, 11))
    tail = [e for e in evs if not isinstance(e, (gol.TurnComplete, gol.AliveCellsCount))]
    assert [type(e).__name__ for e in tail] == [
        "StateChange", "FinalTurnComplete", "StateChange", "ImageOutputComplete"]
    assert tail[2].NewState == gol.State.Quitting and tail[2].CompletedTurns == 10
    assert tail[3].Filename == "64x64x10" and tail[3].CompletedTurns == 10
    assert str(tail[3]) == "File 64x64x10 output complete"


def test_alive_counts_ticker(gol, workdir):
    """TestAlive: 512^2, Turns 1e8, Threads 8; the first 5 AliveCellsCount events
    must match check/alive/512x512.csv (or 5565/5567 beyond 10000)."""
    series = G.alive_series(512)
    p = gol.Params(Turns=100000000, Threads=8, ImageWidth=512, ImageHeight=512)
    events, keys = gol.Channel(), gol.Channel(10)
    t0 = time.time()
    h = gol.Run(p, events, keys, image_dir=str(workdir / "images"),
                out_dir=str(workdir / "out"), ticker_ms=300, emit_turn_complete=False)
    seen = []
    for e in events:
        if isinstance(e, gol.AliveCellsCount):
            if not seen:
                assert time.time() - t0 < 5.0, "no AliveCellsCount within 5 s"
            assert e.CellsCount == G.expected_alive(512, e.CompletedTurns, series), e
            seen.append(e)
            if len(seen) == 5:
                keys.send("q")
    h.wait(5)
    assert len(seen) >= 5
    assert seen[-1].CompletedTurns > seen[0].CompletedTurns


def test_keys_save_pause_quit(gol, workdir, oracle):
    p = gol.Params(Turns=100000000, Threads=8, ImageWidth=64, ImageHeight=64)
    events, keys = gol.Channel(), gol.Channel(10)
    h = gol.Run(p, events, keys, image_dir=str(workdir / "images"),
                out_dir=str(workdir / "out"), ticker_ms=100, emit_turn_complete=False)
    keys.send("s")
    saved, states, final = [], [], []
    paused = False
    for e in events:
        if isinstance(e, gol.ImageOutputComplete):
            saved.append(e)
            if len(saved) == 1:
                keys.send("p")
        elif isinstance(e, gol.StateChange):
            states.append(e)
            if e.NewState == gol.State.Paused and not paused:
                paused = True
                time.sleep(0.3)
                keys.send("p")
            elif e.NewState == gol.State.Executing and paused:
                keys.send("q")
        elif isinstance(e, gol.FinalTurnComplete):
            final.append(e)
    h.wait(5)
    assert [s.NewState for s in states] == [gol.State.Executing, gol.State.Paused,
                                           gol.State.Executing, gol.State.Quitting]
    assert states[1].CompletedTurns == states[2].CompletedTurns
    # 's' wrote the board at the reported turn
    t = saved[0].CompletedTurns
    snap = G.parse_pgm((workdir / "out" / f"{saved[0].Filename}.pgm").read_bytes())
    assert np.array_equal(snap, oracle.np_run(G.input_board(64), t))
    # the final image is at the final turn
    T = final[0].CompletedTurns
    assert saved[-1].Filename == f"64x64x{T}"
    fin = G.parse_pgm((workdir / "out" / f"64x64x{T}.pgm").read_bytes())
    assert np.array_equal(fin, oracle.np_run(G.input_board(64), T))


@pytest.mark.parametrize("ngpus", (2, 4, 5))
def test_multi_strip_run(gol, workdir, ngpus):
    """len(SUB) strips (all on device 0 here) give the same board as one engine."""
    p = gol.Params(Turns=100, Threads=2, ImageWidth=512, ImageHeight=512)
    evs = run_collect(gol, p, workdir, ngpus=ngpus, devices=[0] * ngpus, halo=7)
    final = [e for e in evs if isinstance(e, gol.FinalTurnComplete)][0]
    assert set((c.X, c.Y) for c in final.Alive) == read_alive_cells_bytes(
        G.check_pgm_bytes(512, 100))
    assert (workdir / "out" / "512x512x100.pgm").read_bytes() == G.check_pgm_bytes(512, 100)


@pytest.mark.parametrize("ngpus", (1, 4))
def test_run_keys_mid_run_match_oracle(gol, workdir, oracle, ngpus):
    """Keys in the middle of an unbounded run, single engine and 4 strips (the strips'
    chunks are pipelined two deep, with no host sync per chunk): the ticker's counts, the
    's' image at its reported turn, a pause, and 'q' all match the oracle at the turns the
    events report (Local/gol/distributor.go:107-167)."""
    series = G.alive_series(512)
    p = gol.Params(Turns=100000000, Threads=8, ImageWidth=512, ImageHeight=512)
    events, keys = gol.Channel(), gol.Channel(10)
    kw = dict(ngpus=ngpus, devices=[0] * ngpus, halo=7) if ngpus > 1 else {}
    h = gol.Run(p, events, keys, image_dir=str(workdir / "images"),
                out_dir=str(workdir / "out"), ticker_ms=150, emit_turn_complete=False, **kw)
    ticks, saved, states, final = [], [], [], []
    for e in events:
        if isinstance(e, gol.AliveCellsCount):
            assert e.CellsCount == G.expected_alive(512, e.CompletedTurns, series), e
            ticks.append(e.CompletedTurns)
            if len(ticks) == 2:
                keys.send("s")
        elif isinstance(e, gol.ImageOutputComplete):
            saved.append(e)
            if len(saved) == 1:
                keys.send("p")
        elif isinstance(e, gol.StateChange):
            states.append(e)
            if e.NewState == gol.State.Paused:
                time.sleep(0.4)
                keys.send("p")
            elif e.NewState == gol.State.Executing and len(states) > 1:
                keys.send("q")
        elif isinstance(e, gol.FinalTurnComplete):
            final.append(e)
    h.wait(10)
    assert h.error is None, h.error
    assert [s.NewState for s in states] == [gol.State.Executing, gol.State.Paused,
                                           gol.State.Executing, gol.State.Quitting]
    assert states[1].CompletedTurns == states[2].CompletedTurns >= saved[0].CompletedTurns
    start = oracle.pack(G.input_board(512))[0]
    t = saved[0].CompletedTurns
    assert t >= ticks[1] > ticks[0] > 0
    snap = G.parse_pgm((workdir / "out" / f"{saved[0].Filename}.pgm").read_bytes())
    assert np.array_equal(snap, oracle.unpack(oracle.bit_run(start, 512, t, ncores=8), 512))
    T = final[0].CompletedTurns
    assert len(final[0].Alive) == G.expected_alive(512, T, series)
    fin = G.parse_pgm((workdir / "out" / f"512x512x{T}.pgm").read_bytes())
    assert np.array_equal(fin, oracle.unpack(oracle.bit_run(start, 512, T, ncores=8), 512))


def test_cell_flipped(gol, workdir, oracle):
    """CellFlipped for the initial alive cells and every flip, before TurnComplete."""
    p = gol.Params(Turns=3, Threads=1, ImageWidth=16, ImageHeight=16)
    evs = run_collect(gol, p, workdir, emit_cell_flipped=True)
    board = np.zeros((16, 16), dtype=bool)
    turn = 0
    for e in evs:
        if isinstance(e, gol.CellFlipped):
            board[e.Cell.Y, e.Cell.X] ^= True
        elif isinstance(e, gol.TurnComplete):
            turn = e.CompletedTurns
            want = oracle.np_run(G.input_board(16), turn) == 255
            assert np.array_equal(board, want), turn
    assert turn == 3


def test_missing_image_reports_error(gol, workdir):
    p = gol.Params(Turns=1, Threads=1, ImageWidth=32, ImageHeight=32)
    events = gol.Channel()
    h = gol.Run(p, events, None, image_dir=str(workdir / "images"),
                out_dir=str(workdir / "out"))
    # the reference panics (util.Check); here the channel closes with the error and both
    # iteration and wait() raise it
    with pytest.raises(gol.RunError, match="32x32"):
        list(events)
    with pytest.raises(gol.RunError):
        h.wait(5)
    assert h.error and "32x32" in h.error


def test_cont_resume(gol, workdir, oracle):
    """CONT=yes (Local/gol/distributor.go:171-178): a run resumes from the board and turn
    the previous run ended with and runs Turns - TurnCur more turns; 'k' drops that state."""
    p = gol.Params(Turns=40, Threads=4, ImageWidth=64, ImageHeight=64)
    run_collect(gol, p, workdir, resume=False)
    p2 = gol.Params(Turns=100, Threads=4, ImageWidth=64, ImageHeight=64)
    evs = run_collect(gol, p2, workdir, resume=True)
    assert evs[0].CompletedTurns == 40 and evs[0].NewState == gol.State.Executing
    tc = [e.CompletedTurns for e in evs if isinstance(e, gol.TurnComplete)]
    assert tc == list(range(41, 101))
    final = [e for e in evs if isinstance(e, gol.FinalTurnComplete)][0]
    assert final.CompletedTurns == 100
    assert set((c.X, c.Y) for c in final.Alive) == read_alive_cells_bytes(
        G.check_pgm_bytes(64, 100))
    assert (workdir / "out" / "64x64x100.pgm").read_bytes() == G.check_pgm_bytes(64, 100)
    # a killed run leaves nothing to resume
    events, keys = gol.Channel(), gol.Channel(4)
    h = gol.Run(gol.Params(Turns=10 ** 8, Threads=1, ImageWidth=64, ImageHeight=64), events,
                keys, image_dir=str(workdir / "images"), out_dir=str(workdir / "out"),
                resume=False, emit_turn_complete=False)
    keys.send("k")
    list(events)
    h.wait(5)
    events = gol.Channel()
    h = gol.Run(p2, events, None, image_dir=str(workdir / "images"),
                out_dir=str(workdir / "out"), resume=True)
    with pytest.raises(gol.RunError, match="CONT"):
        list(events)
    with pytest.raises(gol.RunError):
        h.wait(5)
    assert h.error and "CONT" in h.error


def _write_random_pgm(workdir, oracle, seed, w, h):
    board = oracle.unpack(oracle.gen_random(seed, w, h), w)
    (workdir / "images" / f"{w}x{h}.pgm").write_bytes(f"P5\n{w} {h}\n255\n".encode() +
                                                     board.tobytes())


def _digest(key):
    import json
    here = os.path.dirname(os.path.abspath(__file__))
    return json.load(open(os.path.join(here, "golden", "large_digests.json")))[key]


@pytest.mark.parametrize("key,ngpus", [("5120x5120_seed1_t1000", 1),
                                       ("16384x16384_seed2_t10000", 2)])
def test_baseline_configs_through_run(gol, workdir, oracle, key, ngpus):
    """BASELINE configs C2 (5120^2 PGM, 1000 turns, 1 GPU) and C3 (16384^2, 10000 turns,
    2 strips) end to end through gol.Run: PGM in (pinned), turns, TurnComplete events,
    FinalTurnComplete, PGM out -- against the oracle-computed digests."""
    import hashlib
    d = _digest(key)
    w, h, turns = d["width"], d["height"], d["turns"]
    _write_random_pgm(workdir, oracle, d["seed"], w, h)
    p = gol.Params(Turns=turns, Threads=8, ImageWidth=w, ImageHeight=h)
    kw = dict(ngpus=ngpus, devices=[0] * ngpus, halo=128) if ngpus > 1 else {}
    # a 2 ms ticker: AliveCellsCount events at many turns of the run (the reference's 2 s
    # ticker would fire at most once in a run this short)
    evs = run_collect(gol, p, workdir, ticker_ms=2, **kw)
    final = [e for e in evs if isinstance(e, gol.FinalTurnComplete)]
    assert len(final) == 1 and final[0].CompletedTurns == turns
    assert len(final[0].Alive) == d["alive"]
    # every AliveCellsCount is the oracle's count at its CompletedTurns (C2 names these
    # events; series from tests/golden/make_alive_series.py)
    series = G.config_alive_series(w, h, d["seed"])
    init = oracle.popcount(oracle.gen_random(d["seed"], w, h), w)
    ticks = [e for e in evs if isinstance(e, gol.AliveCellsCount)]
    assert ticks, "no AliveCellsCount event"
    for e in ticks:
        assert e.CellsCount == (series[e.CompletedTurns] if e.CompletedTurns else init), e
    tc = [e.CompletedTurns for e in evs if isinstance(e, gol.TurnComplete)]
    assert tc == list(range(1, turns + 1))
    out = (workdir / "out" / f"{w}x{h}x{turns}.pgm").read_bytes()
    board = G.parse_pgm(out)
    words, _, nb = oracle.pack(board)
    assert nb == 0 and hashlib.sha256(words.tobytes()).hexdigest() == d["sha256"]


# --------------------------------------- the INTEGRATION.md cgo stub, run as a C program
HARNESS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "conway-s-gol-distributed_amd", "build", "gol_stub_harness")


class Stub:
    """tests/harness/gol_stub_harness.c: the cgo stub's three goroutines (main running the
    whole game in one gol_step, keys through the control word and gol_get_world, a ticker
    calling gol_snapshot concurrently) as pthreads; events come back one per stdout line."""

    def __init__(self, workdir, size, turns, ticker_ms, turn_complete=0):
        import subprocess
        import threading
        assert os.path.exists(HARNESS), "build it: make -C conway-s-gol-distributed_amd/csrc harness"
        (workdir / "out").mkdir(exist_ok=True)
        self.p = subprocess.Popen(
            [HARNESS, str(size), str(size), str(turns), str(workdir / "images"),
             str(workdir / "out"), str(ticker_ms), str(turn_complete)],
            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
        self.lines = []
        self.cv = threading.Condition()
        self.t = threading.Thread(target=self._pump, daemon=True)
        self.t.start()

    def _pump(self):
        for line in self.p.stdout:
            with self.cv:
                self.lines.append(line.split())
                self.cv.notify_all()
        with self.cv:
            self.lines.append(["EOF"])
            self.cv.notify_all()

    def events(self, timeout=60):
        """Yield events (lists of fields) as they arrive, until CLOSED."""
        i, deadline = 0, time.time() + timeout
        while True:
            with self.cv:
                while i >= len(self.lines):
                    left = deadline - time.time()
                    assert left > 0, f"harness: no event within {timeout} s: {self.lines[-5:]}"
                    self.cv.wait(left)
                ev = self.lines[i]
            i += 1
            assert ev[0] not in ("ERROR", "EOF"), self.lines
            if ev[0] == "CLOSED":
                return
            yield ev

    def key(self, k):
        self.p.stdin.write(k + "\n")
        self.p.stdin.flush()

    def wait(self):
        assert self.p.wait(30) == 0


def test_stub_harness_event_sequence(workdir, oracle):
    """The stub's event order for a normal run (Local/gol/distributor.go:180-226), as
    test_event_sequence checks gol.Run's: StateChange Executing at turn 0, TurnComplete 1..T,
    FinalTurnComplete, StateChange Quitting, ImageOutputComplete WxHxT; the final image and
    alive count match the oracle."""
    s = Stub(workdir, 64, 10, 2000, turn_complete=1)
    evs = list(s.events())
    s.wait()
    assert evs[0] == ["StateChange", "0", "Executing"]
    assert [int(e[1]) for e in evs if e[0] == "TurnComplete"] == list(range(1, 11))
    tail = [e for e in evs if e[0] not in ("TurnComplete", "AliveCellsCount")]
    assert [e[0] for e in tail] == ["StateChange", "FinalTurnComplete", "StateChange",
                                    "ImageOutputComplete"]
    assert tail[2] == ["StateChange", "10", "Quitting"]
    assert tail[3] == ["ImageOutputComplete", "10", "64x64x10"]
    want = oracle.np_run(G.input_board(64), 10)
    assert int(tail[1][2]) == int((want == 255).sum())
    fin = G.parse_pgm((workdir / "out" / "64x64x10.pgm").read_bytes())
    assert np.array_equal(fin, want)


def test_stub_harness_keys_and_ticker(workdir, oracle):
    """The stub's keys and ticker, as test_keys_save_pause_quit and TestAlive check gol.Run's:
    's' writes the board at the GetWorld turn, 'p' parks the single gol_step (Paused and
    Executing report the same turn), the ticker's AliveCellsCount keeps firing while paused at
    the paused turn, 'q' ends the run; every count and image matches the oracle."""
    series = G.alive_series(512)
    s = Stub(workdir, 512, 100000000, 100)
    s.key("s")
    saved, states, final, ticks, paused_ticks = [], [], [], [], []
    paused_at = None
    for e in s.events():
        if e[0] == "ImageOutputComplete":
            saved.append(e)
            if len(saved) == 1:
                s.key("p")
        elif e[0] == "StateChange":
            states.append(e)
            if e[2] == "Paused" and paused_at is None:
                paused_at = int(e[1])
                time.sleep(0.5)
                s.key("p")
            elif e[2] == "Executing" and paused_at is not None:
                s.key("q")
        elif e[0] == "AliveCellsCount":
            t, n = int(e[1]), int(e[2])
            assert n == G.expected_alive(512, t, series), e
            ticks.append(t)
            if paused_at is not None and len(states) == 2:
                paused_ticks.append(t)
        elif e[0] == "FinalTurnComplete":
            final.append(e)
    s.wait()
    assert [x[2] for x in states] == ["Executing", "Paused", "Executing", "Quitting"]
    assert states[1][1] == states[2][1]
    # (a tick whose snapshot was served just before the step parked may print after Paused)
    assert paused_ticks.count(paused_at) >= 2 and max(paused_ticks) == paused_at
    t = int(saved[0][1])
    assert saved[0][2] == f"512x512x{t}"
    snap = G.parse_pgm((workdir / "out" / f"512x512x{t}.pgm").read_bytes())
    assert np.array_equal(snap, oracle.np_run(G.input_board(512), t))
    T = int(final[0][1])
    assert T >= paused_at and int(final[0][2]) == G.expected_alive(512, T, series)
    assert saved[-1] == ["ImageOutputComplete", str(T), f"512x512x{T}"]


def test_stub_harness_no_tick_after_quitting(workdir, monkeypatch):
    """The stub's shutdown handshake (round-4 verdict weak #8): main ends the ticker with an
    unbuffered `done <- true` (Local/gol/distributor.go:59,162-163,198), which returns only
    once the ticker is back in its select.  Here every tick sleeps 40 ms between its snapshot
    and its event while ticks come every 5 ms, so the run almost always ends with a tick in
    flight: its AliveCellsCount must still come before FinalTurnComplete, and none after
    StateChange Quitting.  Every count is the oracle's at its turn.  (This order is stricter
    than the reference's own: Local/gol/distributor.go sends FinalTurnComplete and Quitting
    (:194-195) before ticker.Stop and done <- true (:197-198), so a tick in that gap can follow
    Quitting there.  The stub ends the ticker first; its sequences are a subset of the
    reference's.)"""
    monkeypatch.setenv("GOL_HARNESS_TICK_DELAY_MS", "40")
    series = G.alive_series(512)
    ticks_seen = 0
    for _ in range(3):
        s = Stub(workdir, 512, 1000000, 5)          # (~0.15 s of stepping: ~3 ticks)
        evs = list(s.events())
        s.wait()
        names = [e[0] for e in evs]
        i = names.index("FinalTurnComplete")
        assert "AliveCellsCount" not in names[i:], evs[i - 3:]
        assert names[i:] == ["FinalTurnComplete", "StateChange", "ImageOutputComplete"]
        for e in evs:
            if e[0] == "AliveCellsCount":
                ticks_seen += 1
                assert int(e[2]) == G.expected_alive(512, int(e[1]), series), e
    assert ticks_seen >= 1
