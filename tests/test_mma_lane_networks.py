"""Host model of the lane exchanges of the MFMA mat-vec (csrc/mmvq_mma.hip), CPU only.

A wave is 64 lanes in four 16-lane rows g = lane >> 4. The kernel's exchanges use two gfx950
instructions, modelled here on one register per lane:
  v_permlane16_swap(vdst, vsrc): odd rows of vdst <-> even rows of vsrc (row 2k+1 with row 2k)
  v_permlane32_swap(vdst, vsrc): upper 32 lanes of vdst <-> lower 32 lanes of vsrc
and the helpers swap16(even_src, odd_dst) / swap32(lo_src, hi_dst) call them with
(vdst, vsrc) = (odd_dst, even_src) / (hi_dst, lo_src), as mmvq_mma.hip does. Each test loads every
lane's registers with labels of the bytes it holds and checks that the network leaves each lane
the bytes its MFMA fragments need (the layouts are described in the file's header and at each
helper: halves_to_pairs, runs_to_pairs, run_whole, run_half, MmaPair::split).
"""
import numpy as np

LANES = 64
ROW = np.arange(LANES) >> 4        # g


def permlane16_swap(vdst, vsrc):
    vdst, vsrc = vdst.copy(), vsrc.copy()
    for g in (0, 2):
        lo, hi = slice(16 * g, 16 * g + 16), slice(16 * (g + 1), 16 * (g + 2))
        vdst[hi], vsrc[lo] = vsrc[lo].copy(), vdst[hi].copy()
    return vdst, vsrc


def permlane32_swap(vdst, vsrc):
    vdst, vsrc = vdst.copy(), vsrc.copy()
    vdst[32:], vsrc[:32] = vsrc[:32].copy(), vdst[32:].copy()
    return vdst, vsrc


def swap16(even_src, odd_dst):
    odd_dst, even_src = permlane16_swap(odd_dst, even_src)
    return even_src, odd_dst


def swap32(lo_src, hi_dst):
    hi_dst, lo_src = permlane32_swap(hi_dst, lo_src)
    return lo_src, hi_dst


def lab(*parts):
    """one label per lane, e.g. lab('blk', g, 'half', 0) -> ('blk', g, 'half', 0) for each lane's g"""
    out = np.empty(LANES, dtype=object)
    for lane in range(LANES):
        g = ROW[lane]
        out[lane] = tuple(p(g) if callable(p) else p for p in parts)
    return out


def test_halves_to_pairs():
    """Q4_0 / Q8_0 at 8 tokens: lane g loaded block g whole (X = its lower half, Y = its upper);
    pair p needs half g & 1 of block 2p + (g >> 1)"""
    X = lab("blk", lambda g: g, "half", 0)
    Y = lab("blk", lambda g: g, "half", 1)
    Y, X = swap16(Y, X)
    Y, X = swap32(Y, X)
    for lane in range(LANES):
        g = ROW[lane]
        assert X[lane] == ("blk", 0 * 2 + (g >> 1), "half", g & 1)
        assert Y[lane] == ("blk", 1 * 2 + (g >> 1), "half", g & 1)


def test_paired_steps_split():
    """MmaPair::split: lane g loaded blocks 2g (F) and 2g + 1 (S) of a double step; step 2j needs
    block g (blocks 0..3), step 2j + 1 block 4 + g"""
    X = lab("blk", lambda g: 2 * g)
    Y = lab("blk", lambda g: 2 * g + 1)
    Y, X = swap16(Y, X)
    Y, X = swap32(Y, X)
    for lane in range(LANES):
        g = ROW[lane]
        assert X[lane] == ("blk", g)
        assert Y[lane] == ("blk", 4 + g)


def test_runs_to_pairs():
    """K-quants at 8 tokens: lane g holds half g & 1 of run 2h + (g >> 1); pair p needs half g & 1
    of run 2h + p (X: p = 0, Y: p = 1); X = Y = own, then swap32(Y, X)"""
    own = lab("run", lambda g: g >> 1, "half", lambda g: g & 1)
    X, Y = own.copy(), own.copy()
    Y, X = swap32(Y, X)
    for lane in range(LANES):
        g = ROW[lane]
        assert X[lane] == ("run", 0, "half", g & 1)
        assert Y[lane] == ("run", 1, "half", g & 1)


def test_run_whole():
    """K-quants at 4 tokens: lanes g, g ^ 1 loaded bytes 16 (g & 1) .. + 16 of the same run;
    with A = B = own, swap16(A, B) leaves B = bytes 0..15 and A = bytes 16..31 on both"""
    own = lab("bytes", lambda g: 16 * (g & 1))
    A, B = own.copy(), own.copy()
    A, B = swap16(A, B)
    for lane in range(LANES):
        assert B[lane] == ("bytes", 0)
        assert A[lane] == ("bytes", 16)


def test_run_half():
    """K-quants at 8 tokens: lane a = g & 1 loaded bytes 16a .. 16a + 15 (dwords 0, 1 = 16a..,
    dwords 2, 3 = 16a + 8..) and needs bytes 8a .. + 8 then 16 + 8a .. + 8; X = dwords 2, 3,
    Y = dwords 0, 1, swap16(X, Y) -> {Y, X}"""
    X = lab("bytes", lambda g: 16 * (g & 1) + 8)
    Y = lab("bytes", lambda g: 16 * (g & 1))
    X, Y = swap16(X, Y)
    for lane in range(LANES):
        a = ROW[lane] & 1
        assert Y[lane] == ("bytes", 8 * a)
        assert X[lane] == ("bytes", 16 + 8 * a)


def test_chunk_order_pairs_nibbles():
    """mma_elem: chunk m holds elements 8 (m >> 1) + 16 (m & 1) + i, so chunks {2a, 2a + 1} are the
    low / high nibbles of Q4_0 qs bytes 8a .. 8a + 7 (element e < 16 is the low nibble of byte e,
    e >= 16 the high nibble of byte e - 16), and the four chunks cover the block once"""
    def elem(m, i):
        return 8 * (m >> 1) + 16 * (m & 1) + i
    seen = sorted(elem(m, i) for m in range(4) for i in range(8))
    assert seen == list(range(32))
    for a in range(2):
        lo = [elem(2 * a, i) for i in range(8)]
        hi = [elem(2 * a + 1, i) for i in range(8)]
        assert lo == [8 * a + i for i in range(8)]                 # low nibbles of bytes 8a + i
        assert [e - 16 for e in hi] == [8 * a + i for i in range(8)]   # high nibbles, same bytes


def test_block_diagonal_columns():
    """TOK tokens: MFMA column c is token c % TOK of block group c / TOK; a lane's B fragment
    (k-group g) is live only where g / L == c / TOK (L = TOK / 4 k-groups per group), so each
    output (row, c) sums exactly one block's k of one token, and every k-group feeds one group"""
    for TOK in (4, 8):
        G, L = 16 // TOK, TOK // 4
        for c in range(16):
            live = [g for g in range(4) if g // L == c // TOK]
            assert len(live) == L
        for g in range(4):
            cols = [c for c in range(16) if g // L == c // TOK]
            assert len(cols) == TOK
