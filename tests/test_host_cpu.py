"""Host-side logic that needs no GPU: the reference's strip split, halo row
selection, the Go-channel mirror, the PGM reader rules and the event types."""
import threading

import numpy as np
import pytest

import golden_data as G


def test_strip_split_matches_reference():
    """Server/gol/distributor.go:106-116: base H/N, the first H%N strips +1."""
    from gol import strip_split
    assert strip_split(512, 4) == [(0, 128), (128, 128), (256, 128), (384, 128)]
    assert strip_split(10, 3) == [(0, 4), (4, 3), (7, 3)]
    assert strip_split(65536, 8)[-1] == (57344, 8192)
    for h in (1, 7, 100, 513):
        for n in range(1, min(h, 9) + 1):
            parts = strip_split(h, n)
            assert sum(r for _, r in parts) == h
            assert all(parts[i + 1][0] == parts[i][0] + parts[i][1] for i in range(n - 1))


def test_haloed_rows_wrap():
    from gol import haloed_rows
    b = np.arange(10)[:, None].repeat(3, axis=1).astype(np.uint8)
    s = haloed_rows(b, 0, 3, 2)
    assert s[:, 0].tolist() == [8, 9, 0, 1, 2, 3, 4]
    s = haloed_rows(b, 8, 2, 3)
    assert s[:, 0].tolist() == [5, 6, 7, 8, 9, 0, 1, 2]


def test_channel_semantics():
    from gol import Channel
    c = Channel()
    got = []
    t = threading.Thread(target=lambda: got.extend(list(c)))
    t.start()
    for i in range(100):
        c.send(i)
    c.close()
    t.join(5)
    assert got == list(range(100))
    assert c.recv() == (None, False)
    with pytest.raises(RuntimeError):
        c.send(1)


def test_event_strings_and_turns():
    import gol
    assert str(gol.AliveCellsCount(5, 10)) == "Alive Cells 10"
    assert str(gol.ImageOutputComplete(3, "16x16x3")) == "File 16x16x3 output complete"
    assert str(gol.StateChange(0, gol.State.Executing)) == "Executing"
    assert gol.State.Paused == 0 and gol.State.Quitting == 2
    assert gol.TurnComplete(7).GetCompletedTurns() == 7


def test_pgm_reader_rules():
    data = G.input_pgm_bytes(16)
    assert data.startswith(b"P5\n16 16\n255\n")
    b = G.parse_pgm(data)
    assert b.shape == (16, 16) and set(np.unique(b)) <= {0, 255}
    with pytest.raises(ValueError):
        G.parse_pgm(b"P2\n1 1\n255\n\x00")
    with pytest.raises(ValueError):
        G.parse_pgm(b"P5\n2 2\n255\n\x00")


def test_run_requires_native_library(monkeypatch, tmp_path):
    """No silent fallback: a missing engine library raises."""
    from gol import _native as N
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setattr(N, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(ImportError):
        N.lib()


def _kernel_rule(name):
    """The body of a device rule function in gol_device.h as (dst, op, args) triples."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "conway-s-gol-distributed_amd",
                            "csrc", "gol_device.h")).read()
    body = src[src.index(f"uint32_t {name}("):]
    body = body[body.index("{") + 1:body.index("\n}")]
    ops = []
    for line in body.splitlines():
        m = re.search(r"(?:const uint32_t (\w+) =|return) (xor3|maj|bitop3<(0x[0-9a-f]+)>)\((\w+), (\w+), (\w+)\)",
                      line)
        if m:
            imm = {"xor3": 0x96, "maj": 0xE8}.get(m.group(2)) or int(m.group(3), 16)
            ops.append((m.group(1) or "return", imm, m.group(4, 5, 6)))
    return ops


@pytest.mark.parametrize("name", ["life_rule7", "life_rule8"])
def test_rule_truth_tables(name):
    """The bit-sliced rules in the HIP source (v_bitop3 immediates, index
    (src0 << 2) | (src1 << 1) | src2) reproduce calculateNextState
    (SubServer/distributor.go:178-200) on all 512 3x3 windows."""
    ops = _kernel_rule(name)
    assert ops and ops[-1][0] == "return"
    for m in range(512):
        cell = [(m >> i) & 1 for i in range(9)]
        centre = cell[4]
        n = sum(cell) - centre
        want = int(n == 3 or (centre == 1 and n == 2))
        rs = [sum(cell[3 * r:3 * r + 3]) for r in range(3)]
        env = {"a0": rs[0] & 1, "b0": rs[1] & 1, "c0": rs[2] & 1,
               "a1": rs[0] >> 1, "b1": rs[1] >> 1, "c1": rs[2] >> 1, "C": centre}
        for dst, imm, (x, y, z) in ops:
            env[dst] = (imm >> ((env[x] << 2) | (env[y] << 1) | env[z])) & 1
        assert env["return"] == want, (name, m)
