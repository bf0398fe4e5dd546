"""Host checks of the fused FFT reconstruct, no GPU.

1. The algebra, on the oracle's own transforms: for a residual codeword (zero on every
   received data shard; s = p ^ Enc(d') on the recovery rows R) the reference decode
   (root.zig:268-335: evalPoly, x L, IFFT over W, formal derivative, FFT over W,
   x g^(65535 - e)) equals, block by block, beta_K * FFT_{C, skew KC}(IFFT_{C, skew 0}(L s)).
   Checked against the oracle's full decode for several codes and patterns.
2. The kernel's schedule (rs_fft_decode_selftest): the generated layers, the runtime
   multiply's nibble masks and the decode block, on scalar symbols.
"""
import ctypes as C

import numpy as np
import pytest

from rs_amd import reedsol_amd as R

MOD = 65535


def _deriv(work):
    out = work.copy()
    for i in range(1, out.shape[0]):
        w = i & -i
        out[i - w:i] ^= out[i:i + w]
    return out


def _block_coeffs(O, C, W):
    """(alpha_K, beta_K): block K of the W-point decode of a block-0-only input is
    alpha_K * D_C(a) + beta_K * a (a = IFFT_C of block 0), per the layer schedules of
    Generic.zig:80-147 / 15-78 and root.zig:309-315."""
    EXP, LOG, SKEW = O.table("exp"), O.table("log"), O.table("skew")

    def mul(x, y):
        return 0 if x == 0 or y == 0 else int(EXP[(int(LOG[x]) + int(LOG[y])) % MOD])

    def tw(i):
        return 0 if SKEW[i] == MOD else int(EXP[SKEW[i]])

    nb = W // C
    lam = [1] + [0] * (nb - 1)
    d = C
    while d < W:
        for g in range(0, W, 2 * d):
            t = tw(g + d - 1)
            for i in range(g, g + d, C):
                x, y = i // C, (i + d) // C
                lam[y] ^= lam[x]
                lam[x] ^= mul(t, lam[y])
        d *= 2
    al = list(lam)
    be = [0] * nb
    for K in range(nb):
        b = 1
        while b < nb:
            if not K & b:
                be[K] ^= lam[K | b]
            b <<= 1
    d = W // 2
    while d >= C:
        for g in range(0, W, 2 * d):
            t = tw(g + d - 1)
            for i in range(g, g + d, C):
                x, y = i // C, (i + d) // C
                al[x] ^= mul(t, al[y])
                be[x] ^= mul(t, be[y])
                al[y] ^= al[x]
                be[y] ^= be[x]
        d //= 2
    return al, be, LOG


@pytest.mark.parametrize("k,m,erased", [
    (200, 55, list(range(1, 165, 3))),
    (10, 4, [0, 1, 2, 3]),
    (100, 20, [5, 40, 41, 99]),
    (32, 32, list(range(0, 32, 2))),
    (1000, 64, [0, 63, 64, 500, 999]),
    (33, 17, list(range(16, 33))),
])
def test_block_formula_vs_oracle_decode(oracle, k, m, erased):
    O = oracle
    rng = np.random.default_rng(k + 3 * m)
    sb = 64
    Cn = 1
    while Cn < m:
        Cn *= 2
    W = 1
    while W < Cn + k:
        W *= 2
    data = rng.integers(0, 256, (k, sb), dtype=np.uint8)
    st, par = O.encode(k, m, data)
    assert st == 0
    d2 = data.copy()
    d2[erased] = 0
    st, par2 = O.encode(k, m, d2)
    s = par ^ par2
    er = np.zeros(65536, np.uint16)
    er[m:Cn] = 1
    er[[Cn + e for e in erased]] = 1
    O.eval_poly(er, Cn + k)
    w = np.zeros((Cn, sb), np.uint8)
    for p in range(m):
        w[p] = s[p]
        O.mul_scalar(w[p], int(er[p]))
    a = w.copy()
    O.ifft(a, 0, Cn, Cn, 0)
    al, be, LOG = _block_coeffs(O, Cn, W)
    assert all(x == 0 for x in al[1:])  # the derivative term vanishes on every data block
    orig = [None if i in erased else data[i] for i in range(k)]
    st, ref = O.decode(k, m, orig, list(par), sb)
    assert st == 0
    for K in range(1, W // Cn):
        es = [e for e in erased if (Cn + e) // Cn == K]
        if not es:
            continue
        y = a.copy()
        O.fft(y, 0, Cn, Cn, K * Cn)
        for e in es:
            x = y[(Cn + e) % Cn].copy()
            O.mul_scalar(x, int(LOG[be[K]]))
            O.mul_scalar(x, MOD - int(er[Cn + e]))
            assert np.array_equal(x, data[e]) and np.array_equal(x, ref[e]), (k, m, e)


@pytest.mark.parametrize("k,m,e", [(200, 55, 55), (200, 55, 7), (64, 64, 40), (33, 17, 17), (1000, 64, 64),
                                   (16, 16, 16), (30, 9, 5), (100, 20, 20), (65, 33, 1)])
def test_fdec_schedule_selftest(k, m, e):
    assert R.fft_decode_selftest(k, m, e, 12) == 0


def test_fdec_selftest_rejects():
    L = R.lib()
    bad = C.c_uint64(0)
    assert L.rs_fft_decode_selftest(10, 4, 2, 1, C.byref(bad)) != 0  # chunk 4: no FFT kernel form
    assert L.rs_fft_decode_selftest(200, 55, 56, 1, C.byref(bad)) != 0  # e > m
