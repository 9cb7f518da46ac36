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
