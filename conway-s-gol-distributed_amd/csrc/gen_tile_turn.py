#!/usr/bin/env python3
"""Generate gol_tile_turn.h: K1t's turn (ORD 8) as one inline-asm block per turn with a
hand-made VGPR assignment.

Why (tools/calib/vgpr_bank_probe, profiles/r05_vgpr_bank_probe.log): on gfx950 a v_bitop3_b32
whose three source VGPRs all have the same register-number parity issues at half rate (4.1-4.3
SIMD cycles per wave64 instruction against 2.2-2.6 when the parities are mixed).  The compiler's
allocation of the ORD 5 turn leaves 68 of its 432 v_bitop3 per SEG-24 turn with same-parity
sources.  Here every v_bitop3 has mixed parities by construction:

* cells: row i's even dword in v(2i), odd dword in v(2i+1) -- every row sum
  xor3 / maj(wl, e, o) and (e, o, er) mixes an even and an odd register;
* row sums: the 3-row window rotates over three 4-register slots X, Y, Z; X and Z hold
  (s0, s1, s2, s3) in (even, odd, even, odd) registers, Y in (odd, even, odd, even), and the
  LDS tuples (own first row F = X, own last row Lr = L, the neighbours' U / D) are
  (even, odd, even, odd) like X: every rule reads one row sum from each of three slots, one of
  which is Y (rows i - 1, i, i + 1 cover all three slots; for SEG % 3 == 0 the slots that the
  LDS tuples replace at the segment ends are never Y's), so each of its majority / parity
  inputs mixes parities;
* rule temporaries: lm, hx even and lx, hm odd; g1 overwrites lm and g2 hm, so
  (lm, lx, C), (hm, C, g1) and (lx, hx, g2) all mix.

The turn is ORD 5's (gol_tile.h): the first and last rows' sums go to LDS, one workgroup
barrier, the interior rows, the edge rows last -- except that row 0's rule runs as soon as
row 1's sums exist (so F and row 1's sums need not be kept) and the own-edge sums are not read
back (Lr stays in L).  LDS layout (ORD 8 only): 64 B per slot, [slot][top / bottom][parity]
16 B each, so the turn parity is a 16-B toggle of the three lane addresses (me, up, dn).

Hazards (the compiler does not see into inline asm): a DPP move reads a cell written in the
previous turn at least 8 VALU earlier (>= 2 wait states); a DPP never overwrites a register
the instruction just before it read (the compiler pads that case with s_nop 0) -- checked
below, s_nop inserted if a schedule ever needs one.

Usage: python3 gen_tile_turn.py > gol_tile_turn.h  (the Makefile does this)
"""
import os
import sys

SEGS = (24, 12, 6)
ALIGN = int(os.environ.get("GOL_TURN_ALIGN", "0"))   # log2 bytes, 0: none (A/B builds only)
VARIANTS = (4, 5)        # the tools build's ORD 8 / 9 (GOL_TURN_VAR = 4); add others for A/B builds


class Gen:
    def __init__(self, seg, var=0, iso=False):
        assert seg % 3 == 0 and seg >= 6 and 0 <= var < 16
        mode = "bperm" if var & 1 else "dpp"
        assert not (iso and var & 7)
        self.seg = seg
        self.var = var
        self.mode = mode
        self.late = bool(var & 2)    # barrier after rows 1 and 2 (ORD 5's compiled placement)
        self.dense = bool(var & 4)   # LDS slots 16 B apart (ORD 5's layout) instead of 64
        self.ahead = bool(var & 8)   # DPP moves issued two rows ahead (double-buffered)
        self.iso = iso          # timing harness: the turn without LDS and barrier (wrong board)
        self.lq = []            # outstanding LDS operations, in issue order (tags)
        self.out = []
        self.prev_reads = set()
        self.written_at = {}
        self.n = 0
        b = 2 * seg
        self.X = [b + 0, b + 1, b + 2, b + 3]          # even-aligned tuple (e, o, e, o)
        self.L = [b + 4, b + 5, b + 6, b + 7]          # own last row's sums (tuple)
        self.U = [b + 8, b + 9, b + 10, b + 11]        # U, then D (tuple)
        self.Z = [b + 12, b + 13, b + 14, b + 15]      # (e, o, e, o)
        self.Y = [b + 17, b + 18, b + 19, b + 20]      # (o, e, o, e)
        self.TA, self.TB = b + 16, b + 21              # row-sum temporaries
        self.LM, self.LX, self.HM, self.HX = b + 22, b + 23, b + 25, b + 24
        self.nregs = b + 26
        # bperm: the lane-shifted words arrive by ds_bpermute_b32 one row ahead, double-buffered
        self.bufs = [(self.TA, self.TB), (b + 26, b + 27)]
        if mode == "bperm" or self.ahead:
            self.nregs = b + 28
        self.free = list(self.bufs)
        self.pending = {}       # row -> buffer its shifted words are (or will be) in
        assert self.LM % 2 == 0 and self.HX % 2 == 0 and self.LX % 2 == 1 and self.HM % 2 == 1
        assert all(r % 2 == 1 for r in self.Y[0::2]) and all(r % 2 == 0 for r in self.Y[1::2])
        for t in (self.X, self.L, self.U, self.Z):
            assert t[0] % 2 == 0

    def emit(self, text, reads=(), writes=(), dpp_src=None):
        # hazard checks for DPP moves (see the module docstring)
        if dpp_src is not None:
            last = self.written_at.get(dpp_src)
            if last is not None and self.n - last <= 2:
                self.out.append("s_nop 1")
            if any(w in self.prev_reads for w in writes):
                self.out.append("s_nop 0")
        self.out.append(text)
        self.prev_reads = set(reads)
        for w in writes:
            self.written_at[w] = self.n
        self.n += 1

    def lds(self, text, tag, reads=(), writes=()):
        if self.iso:
            return
        self.emit(text, reads, writes)
        self.lq.append(tag)

    def wait_for(self, tag):
        """s_waitcnt lgkmcnt(n): LDS operations complete in issue order, so `tag` is done once
        at most the n issued after it are outstanding."""
        if tag not in self.lq:
            return
        k = self.lq.index(tag)
        n = len(self.lq) - k - 1
        assert n <= 15
        self.emit("s_waitcnt lgkmcnt(%d)" % n)
        del self.lq[:k + 1]

    def wait_all(self):
        if not self.iso:
            self.emit("s_waitcnt lgkmcnt(0)")
        self.lq = []

    def issue_shift(self, row):
        """bperm: the west lane's odd dword and the east lane's even dword of `row`; dpp with
        `ahead`: the same by DPP moves, issued early."""
        if self.mode != "bperm" and not self.ahead:
            return
        A, B = self.free.pop(0)
        e, o = 2 * row, 2 * row + 1
        if self.mode == "dpp":
            self.emit("v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, o),
                      (o,), (A,), dpp_src=o)
            self.emit("v_mov_b32_dpp v%d, v%d wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (B, e),
                      (e,), (B,), dpp_src=e)
            self.pending[row] = (A, B)
            return
        self.lds("ds_bpermute_b32 v%d, %%[ba], v%d" % (A, o), ("w", row), (o,), (A,))
        self.lds("ds_bpermute_b32 v%d, %%[ba], v%d offset:8" % (B, e), ("e", row), (e,), (B,))
        self.pending[row] = (A, B)

    def bitop3(self, d, a, b, c, imm):
        pa = {a % 2, b % 2, c % 2}
        assert len(pa) == 2, "same-parity v_bitop3 sources v%d v%d v%d" % (a, b, c)
        self.emit("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x%02x" % (d, a, b, c, imm), (a, b, c), (d,))

    def rsum(self, row, S):
        """3-cell row sums of row `row` into slot S = (s0, s1, s2, s3)."""
        e, o = 2 * row, 2 * row + 1
        # west: wl = (o << 1) | (west lane's o >> 31); east: er = (e >> 1) | (east lane's e << 31)
        if self.mode == "bperm":
            A, B = self.pending.pop(row)
            self.wait_for(("e", row))
        elif self.ahead:
            A, B = self.pending.pop(row)
        else:
            A, B = self.TA, self.TB
            self.emit("v_mov_b32_dpp v%d, v%d wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (A, o),
                      (o,), (A,), dpp_src=o)
            self.emit("v_mov_b32_dpp v%d, v%d wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" % (B, e),
                      (e,), (B,), dpp_src=e)
        self.emit("v_alignbit_b32 v%d, v%d, v%d, 31" % (A, o, A), (o, A), (A,))
        self.emit("v_alignbit_b32 v%d, v%d, v%d, 1" % (B, B, e), (B, e), (B,))
        self.bitop3(S[0], A, e, o, 0x96)
        self.bitop3(S[1], A, e, o, 0xE8)
        self.bitop3(S[2], e, o, B, 0x96)
        self.bitop3(S[3], e, o, B, 0xE8)
        if self.mode == "bperm" or self.ahead:
            self.free.append((A, B))

    def rule(self, row, P, Q, R):
        """life_rule7 on both dwords of row `row` from the sums of rows row-1 (P), row (Q),
        row+1 (R); the result overwrites the cells."""
        for d in range(2):
            a0, b0, c0 = P[2 * d], Q[2 * d], R[2 * d]
            a1, b1, c1 = P[2 * d + 1], Q[2 * d + 1], R[2 * d + 1]
            C = 2 * row + d
            self.bitop3(self.LM, a0, b0, c0, 0xE8)        # L >= 2
            self.bitop3(self.LX, a0, b0, c0, 0x7E)        # L in {1, 2}
            self.bitop3(self.HM, a1, b1, c1, 0xE8)        # H >= 2
            self.bitop3(self.HX, a1, b1, c1, 0x96)        # H odd
            self.bitop3(self.LM, self.LM, self.LX, C, 0x16)     # g1
            self.bitop3(self.HM, self.HM, C, self.LM, 0x86)     # g2
            self.bitop3(C, self.LX, self.HX, self.HM, 0x82)

    def turn(self):
        s = self.seg
        slot = [self.X, self.Y, self.Z]
        X, L, U = self.X, self.L, self.U
        tup = lambda t: "v[%d:%d]" % (t[0], t[3])
        mb = "%[mb]" if self.dense else "%[me]"
        mbo = "" if self.dense else " offset:32"
        # (nothing of the compiler's may still count in lgkmcnt; and it may have written a cell
        # just before the block: 2 wait states before a DPP reads one)
        if not self.iso:
            self.out.append("s_waitcnt lgkmcnt(0)")
        if ALIGN:
            # (A/B: the block's code alignment -- ORD 8's speed changed from build to build)
            self.out.append(".p2align %d" % ALIGN)
        self.out.append("s_nop 1")
        # own edge rows' sums to LDS, one barrier
        self.issue_shift(0)
        self.issue_shift(s - 1)
        self.rsum(0, X)
        self.issue_shift(1)
        self.rsum(s - 1, L)
        self.issue_shift(2)
        self.lds("ds_write_b128 %%[me], %s" % tup(X), "F", tuple(X))
        self.lds("ds_write_b128 %s, %s%s" % (mb, tup(L), mbo), "Lr", tuple(L))
        if not self.late:
            self.wait_all()
            if not self.iso:
                self.emit("s_barrier")
            self.lds("ds_read_b128 %s, %%[up]" % tup(U), "U", (), tuple(U))
        # rows 1, 2 sums; row 1's rule; row 0's rule (U arrived); then D into U's registers
        self.rsum(1, slot[1])
        self.issue_shift(3)
        self.rsum(2, slot[2])
        self.issue_shift(4)
        self.rule(1, slot[0], slot[1], slot[2])
        if self.late:
            self.wait_for("Lr")
            if not self.iso:
                self.emit("s_barrier")
            self.lds("ds_read_b128 %s, %%[up]" % tup(U), "U", (), tuple(U))
        self.wait_for("U")
        self.rule(0, U, slot[0], slot[1])
        self.lds("ds_read_b128 %s, %%[dn]" % tup(U), "D", (), tuple(U))
        for i in range(2, s - 1):
            nxt = L if i + 1 == s - 1 else slot[(i + 1) % 3]
            if i + 1 < s - 1:
                self.rsum(i + 1, nxt)
                if i + 3 <= s - 2:
                    self.issue_shift(i + 3)
            self.rule(i, slot[(i - 1) % 3], slot[i % 3], nxt)
        self.wait_all()
        assert not self.pending
        # row s-1: sums of row s-2 (slot), own (L), below (D)
        assert slot[(s - 2) % 3] is self.Y
        self.rule(s - 1, slot[(s - 2) % 3], L, U)
        # next turn's parity: toggle the addresses' parity bit (ps: 16 B, or the dense layout's
        # half of the slot arrays)
        if not self.iso:
            for a in ("me", "mb", "up", "dn") if self.dense else ("me", "up", "dn"):
                self.emit("v_xor_b32 %%[%s], %%[ps], %%[%s]" % (a, a))

    def header(self):
        self.turn()
        s = self.seg
        ops = ", ".join('"+{v%d}"(v[%d][%d])' % (2 * i + d, i, d) for i in range(s) for d in range(2))
        clob = ", ".join('"v%d"' % r for r in range(2 * s, self.nregs))
        body = "".join('        "%s\\n"\n' % l for l in self.out)
        nv = sum(1 for l in self.out if l.startswith("v_"))
        nbit = sum(1 for l in self.out if l.startswith("v_bitop3"))
        if self.iso:
            return """
// SEG %d, timing harness only (tools/calib/turn_issue.hip): the dpp turn without its LDS
// exchange and barrier (variant %d: 8 = DPP moves two rows ahead)
template <>
__device__ __forceinline__ void tile_turn_iso<%d, %d>(uint32_t (&v)[%d][2])
{
    asm volatile(
%s        : %s
        :
        : %s);
}
""" % (s, self.var, s, self.var, s, body, ops, clob)
        nbp = sum(1 for l in self.out if l.startswith("ds_bpermute"))
        outs = ['[me] "+v"(ad[0])'] + (['[mb] "+v"(ad[1])'] if self.dense else []) + \
               ['[up] "+v"(ad[2])', '[dn] "+v"(ad[3])']
        ins = ['[ps] "s"(ps)'] + (['[ba] "v"(ba)'] if self.mode == "bperm" else [])
        return """
// SEG %d, variant %d (%s lane shifts, barrier %s, LDS slots %s): %d VALU per turn (%d v_bitop3,
// all with mixed-parity sources), %d ds_bpermute, VGPRs v0..v%d
template <>
__device__ __forceinline__ void tile_turn_asm<%d, %d>(uint32_t (&v)[%d][2], uint32_t (&ad)[4],
                                                      uint32_t ps, uint32_t ba)
{
    asm volatile(
%s        : %s,
          %s
        : %s
        : %s, "memory");
}
""" % (s, self.var, "ds_bpermute" if self.mode == "bperm" else "DPP",
       "after rows 1-2" if self.late else "after the edge sums", "16 B apart" if self.dense else "64 B apart",
       nv, nbit, nbp, self.nregs - 1, s, self.var, s, body, ops, ", ".join(outs), ", ".join(ins), clob)


def main():
    parts = ["""// GENERATED by gen_tile_turn.py -- do not edit.  K1t ORD 8: one turn per inline-asm block
// with a hand-made VGPR assignment (every v_bitop3 reads registers of both parities); see the
// generator's docstring.
#pragma once
#include <cstdint>

namespace golk {

// one turn of a SEG-row segment, variant V (bit 0: ds_bpermute lane shifts instead of DPP;
// bit 1: the barrier after rows 1 and 2; bit 2: LDS slots 16 B apart).  ad = the lane's LDS
// addresses (own top slot, own bottom slot, the segment above's bottom slot, the one below's
// top slot), ps = the turn-parity toggle, ba = the lane's ds_bpermute address
template <int SEG, int V>
__device__ __forceinline__ void tile_turn_asm(uint32_t (&v)[SEG][2], uint32_t (&ad)[4], uint32_t ps,
                                              uint32_t ba);
"""]
    for s in SEGS:
        for var in VARIANTS:
            parts.append(Gen(s, var).header())
    parts.append("""
#ifdef GOL_TURN_ISO
template <int SEG, int V> __device__ __forceinline__ void tile_turn_iso(uint32_t (&v)[SEG][2]);
""")
    for s in SEGS:
        for var in (0, 8):
            parts.append(Gen(s, var, iso=True).header())
    parts.append("#endif\n")
    parts.append("\n}  // namespace golk\n")
    sys.stdout.write("".join(parts))


if __name__ == "__main__":
    main()
