"""Pin the CPU oracle to the reference's golden fixtures before trusting it.

Fixtures (tests/golden/, copied data from the reference):
  Local/check/images/{16,64,512}x{..}x{0,1,100}.pgm, Local/check/alive/*.csv,
  Local/images/*.pgm, digests of Local/out/*.pgm.
"""
import hashlib
import os

import numpy as np
import pytest

import golden_data as G

SIZES = (16, 64, 512)


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("turns", (0, 1, 100))
@pytest.mark.parametrize("nsub,threads", [(1, 1), (1, 16), (2, 8), (4, 6)])
def test_refcpu_check_images(oracle, size, turns, nsub, threads):
    """Literal restatement (Server split x SubServer threads) == check image, for
    every thread count class the reference's TestGol uses (1..16)."""
    got = oracle.ref_run(G.input_board(size), turns, nsub=min(nsub, size), threads=threads)
    assert np.array_equal(got, G.check_board(size, turns))


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("turns", (0, 1, 100))
def test_bitref_and_numpy_check_images(oracle, size, turns):
    b = G.input_board(size)
    w, blk, nb = oracle.pack(b)
    assert nb == 0
    assert np.array_equal(oracle.unpack(oracle.bit_run(w, size, turns), size),
                          G.check_board(size, turns))
    assert np.array_equal(oracle.np_run(b, turns), G.check_board(size, turns))


def test_manifest_counts(oracle):
    man = G.manifest()
    for size in SIZES:
        for t in (0, 1, 100):
            c = G.check_board(size, t)
            entry = man["check"][f"{size}x{size}x{t}.pgm"]
            assert entry["alive"] == int((c == 255).sum())
            assert entry["sha256"] == hashlib.sha256(c.tobytes()).hexdigest()
    # BASELINE.md correctness table
    assert [man["check"][f"512x512x{t}.pgm"]["alive"] for t in (0, 1, 100)] == [6511, 6551, 6645]
    assert [man["check"][f"64x64x{t}.pgm"]["alive"] for t in (0, 1, 100)] == [2819, 281, 219]


@pytest.mark.parametrize("size", SIZES)
def test_bitref_alive_series(oracle, size):
    """Every value of Local/check/alive/{size}x{size}.csv (turns 1..10000)."""
    series = G.alive_series(size)
    w, _, _ = oracle.pack(G.input_board(size))
    _, counts = oracle.bit_run(w, size, 10000, counts=True)
    assert [int(c) for c in counts] == [series[t] for t in range(1, 10001)]


def test_refcpu_alive_series_prefix(oracle):
    series = G.alive_series(64)
    b = G.input_board(64)
    for t in range(1, 40):
        b = oracle.ref_run(b, 1, nsub=4, threads=8)
        assert oracle.ref_alive_count(b) == series[t]


def test_out_dir_secondary(oracle):
    """Local/out/512x512x{T}.pgm files that are correct run outputs."""
    man = G.manifest()["out"]
    labels = [1, 16, 25, 54, 58, 100, 159, 614, 641, 707, 763, 809, 1011, 1055, 1133, 1391,
              1408, 2084, 2236, 2381, 3348, 8964, 10215]
    w, _, _ = oracle.pack(G.input_board(512))
    cur, t = w, 0
    matched = 0
    for T in labels:
        key = f"512x512x{T}.pgm"
        if key not in man:
            continue
        cur = oracle.bit_run(cur, 512, T - t)
        t = T
        board = oracle.unpack(cur, 512)
        assert hashlib.sha256(board.tobytes()).hexdigest() == man[key]["sha256"], key
        matched += 1
    assert matched >= 20


def test_cumulative_turn_mislabels(oracle):
    """Evidence of the reference Server's never-reset `turn` (Server/gol/distributor.go:30,133):
    out/64x64x101.pgm is the turn-0 board and out/64x64x202.pgm the turn-100 board."""
    man = G.manifest()["out"]
    b = G.input_board(64)
    assert man["64x64x101.pgm"]["sha256"] == hashlib.sha256(b.tobytes()).hexdigest()
    assert man["64x64x202.pgm"]["sha256"] == hashlib.sha256(
        oracle.np_run(b, 100).tobytes()).hexdigest()


@pytest.mark.parametrize("w,h", [(2, 2), (3, 5), (17, 9), (64, 1), (65, 4), (130, 33),
                                 (256, 40)])
def test_three_oracles_agree_random(oracle, w, h):
    rng = np.random.default_rng(w * 1000 + h)
    b = np.where(rng.random((h, w)) < 0.4, 255, 0).astype(np.uint8)
    for turns in (1, 3, 8):
        r = oracle.ref_run(b, turns, nsub=min(3, h), threads=min(5, h // min(3, h) + 2))
        n = oracle.np_run(b, turns)
        p = oracle.unpack(oracle.bit_run(oracle.pack(b)[0], w, turns), w)
        assert np.array_equal(r, n) and np.array_equal(r, p)


def test_nonbinary_semantics(oracle):
    """Non-{0,255} bytes are dead neighbours and yield 0 as a centre (SubServer/distributor.go:178-200)."""
    rng = np.random.default_rng(5)
    b = rng.choice(np.array([0, 255, 3, 200], dtype=np.uint8), size=(40, 70))
    r1 = oracle.ref_run(b, 1, nsub=2, threads=3)
    assert np.array_equal(r1, oracle.np_step(b))
    w, blk, nb = oracle.pack(b)
    assert nb == int(((b != 0) & (b != 255)).sum())
    assert np.array_equal(oracle.unpack(oracle.bit_run(w, 70, 1, blocked=blk), 70), r1)
    # a non-binary cell with exactly 3 live neighbours is not born
    z = np.zeros((6, 6), dtype=np.uint8)
    z[1, 1] = z[1, 2] = z[1, 3] = 255
    z[2, 2] = 9
    out = oracle.ref_run(z, 1, nsub=1, threads=1)
    assert out[2, 2] == 0 and out[0, 2] == 255


def test_thread_and_strip_independence(oracle):
    b = G.input_board(64)
    want = G.check_board(64, 100)
    for nsub in (1, 2, 5, 16):
        for threads in (1, 2, 6, 7, 16):
            if threads > 1 and threads > 64 // nsub + 2:
                continue                      # the reference panics there (test below)
            assert np.array_equal(oracle.ref_run(b, 100, nsub=nsub, threads=threads), want)


def test_reference_panics_when_threads_exceed_strip():
    """Quirk: SubServer/distributor.go:111 slices past the strip when Threads > rows_i + 2;
    the Go reference panics (TestGol 16x16 on 4 sub-servers, Threads 7..16)."""
    from oracle.oracle import RefPanic, ref_run
    b = G.input_board(16)
    assert np.array_equal(ref_run(b, 1, nsub=4, threads=6), G.check_board(16, 1))
    with pytest.raises(RefPanic):
        ref_run(b, 1, nsub=4, threads=7)


def test_random_generator_definition(oracle):
    w = oracle.gen_random(42, 130, 3)
    nw = 3
    for y in range(3):
        for j in range(nw):
            v = oracle.lib().bit_splitmix64((42 << 40) + y * nw + j)
            if j == nw - 1:
                v &= (1 << 2) - 1
            assert int(w[y, j]) == v


@pytest.mark.parametrize("key", ["5120x5120_seed1_t1000", "16384x16384_seed2_t10000"])
def test_config_alive_series_consistent(key):
    """The committed C2 / C3 AliveCellsCount series (make_alive_series.py) end at the
    alive count of the committed full-size digest (make_large_digests.py): two runs of the
    pinned bit oracle agree."""
    import json
    import golden_data as G
    d = json.load(open(os.path.join(G.GOLDEN, "large_digests.json")))[key]
    s = G.config_alive_series(d["width"], d["height"], d["seed"])
    assert sorted(s) == list(range(1, d["turns"] + 1))
    assert s[d["turns"]] == d["alive"]


def test_config_alive_series_prefix(oracle):
    """The first turns of the C2 series recomputed here with the bit oracle."""
    import golden_data as G
    s = G.config_alive_series(5120, 5120, 1)
    _, counts = oracle.bit_run(oracle.gen_random(1, 5120, 5120), 5120, 20, counts=True)
    assert [s[t] for t in range(1, 21)] == [int(c) for c in counts]
