"""Model of the on-chip low-rate kernels (rs_lowlds.hip: k_encode_low_lds, k_rec_low_lds; C = 512)
with the field arithmetic of the library's own tables, one symbol per position, against the
oracle-checked scalar encode and the lost data.

Each kernel is restated from its device code: the two register layouts of a workgroup
(P: wave w holds positions 64 w + q; Q: wave w holds positions w + 8 t) and the LDS exchanges
between them, the phase schedule (xform_phases: IFFT 64 @ bits 0-5 then 8 @ bits 6-8, FFT
64 @ bits 3-8 then 8 @ bits 0-2), truncation, the fused IFFT last phase, the syndromes of the
rows used, and the derivative D_C U + gamma U assembled in Q (bits 3-8 in the wave's registers,
bits 0-2 from the other waves' slots). Parity unpinned, as every low-rate path."""
import numpy as np
import pytest

from test_lowblock_model import (EXP, LOG, MOD, block_plan, ceil_pow2, encode_low, fft_sub, fft_tabs, gmul,
                                 ifft_sub, ifft_tabs, mul, xform_phases)

C = 512


def p_to_q(P):  # lds_p_to_q (both rounds): Q[w][t] = position w + 8 t
    return [[P[(w + 8 * t) >> 6][(w + 8 * t) & 63] for t in range(64)] for w in range(8)]


def q_to_p(Q):  # lds_q_to_p: P[w][q] = position 64 w + q
    return [[Q[(64 * w + q) & 7][(64 * w + q) >> 3] for q in range(64)] for w in range(8)]


def qreg(t):  # the Q slot -> register map of the shared array (each round frees what it fills)
    return 32 * ((t >> 2) & 1) + 4 * (t >> 3) + (t & 3)


def phases():
    iph, fph = xform_phases(C, True), xform_phases(C, False)
    assert [(n, d) for n, d, _ in iph] == [(64, 0), (8, 6)] and [(n, d) for n, d, _ in fph] == [(64, 3), (8, 0)]
    return iph[0][2], iph[1][2], fph[0][2], fph[1][2]


def coefficients(vals, k, tabs):  # steps shared by both kernels: P gather, IFFT (bits 0-5), Q (bits 6-8)
    ia, ib, _, _ = phases()
    P = [[vals[64 * w + q] if 64 * w + q < k else 0 for q in range(64)] for w in range(8)]
    for w in range(8):
        if 64 * w < k:
            ifft_sub(P[w], tabs, ia, C, k, 64 * w, 0)
    Q = p_to_q(P)
    for w in range(8):
        for g in range(8):
            gr = [Q[w][g + 8 * t] for t in range(8)]
            ifft_sub(gr, tabs, ib, C, k, 0, 6)
            for t in range(8):
                Q[w][g + 8 * t] = gr[t]
    return Q


def fft_to_p(Q, tf, rmax):  # FFT (Q: bits 3-8), exchange, (P: bits 0-2)
    _, _, fa, fb = phases()
    Q = [list(r) for r in Q]
    for w in range(8):
        fft_sub(Q[w], tf, fa, C, rmax, 0, 3)
    P = q_to_p(Q)
    for w in range(8):
        if 64 * w < rmax:
            for sg in range(8):
                sub = P[w][8 * sg:8 * sg + 8]
                fft_sub(sub, tf, fb, C, rmax, 64 * w + 8 * sg, 0)
                P[w][8 * sg:8 * sg + 8] = sub
    return P


def encode_lds(data, k, m):  # k_encode_low_lds: one workgroup per recovery chunk, coefficients recomputed
    tabs = ifft_tabs(C, 0)
    out = []
    for j in range((m + C - 1) // C):
        rj = min(C, m - j * C)
        P = fft_to_p(coefficients(data, k, tabs), fft_tabs(C, (j + 1) * C), rj)
        out += [P[p >> 6][p & 63] for p in range(rj)]
    return out


def rec_lds(data, par, k, m, present):  # k_rec_low_lds
    ia, ib, _, _ = phases()
    pl = block_plan(k, m, present)
    used = sorted({r // C for r in range(pl["mp"]) if pl["syn_idx"][r] >= 0})
    assert len(used) == 1, used
    j = used[0]
    rj = min(C, pl["mp"] - j * C)
    d = [data[i] if present[i] else 0 for i in range(k)]
    Q = coefficients(d, k, ifft_tabs(C, 0))
    P = fft_to_p(Q, fft_tabs(C, (j + 1) * C), rj)
    for w in range(8):  # syndromes of the rows used (P)
        for q in range(64):
            p, r = 64 * w + q, j * C + 64 * w + q
            if p < rj and pl["syn_idx"][r] >= 0 and pl["syn_log"][r] is not None:
                P[w][q] = mul(P[w][q] ^ par[r], pl["syn_log"][r])
            else:
                P[w][q] = 0
    ti = ifft_tabs(C, (j + 1) * C)
    for w in range(8):
        if 64 * w < rj:
            ifft_sub(P[w], ti, ia, C, rj, 64 * w, 0)
    Q = p_to_q(P)
    for w in range(8):
        for g in range(8):
            gr = [Q[w][g + 8 * t] for t in range(8)]
            ifft_sub(gr, ti, ib, C, rj, 0, 6)
            for t in range(8):
                Q[w][g + 8 * t] = gr[t]
    if pl["u"][j]:  # Z = (1 + gamma) U + the derivative's neighbour terms
        g1 = 1 ^ pl["gamma"][j]
        U = [list(r) for r in Q]
        for w in range(8):
            for t in range(64):
                z = gmul(U[w][t], g1)
                x = 1
                while x < 64:
                    if not (t & x):
                        z ^= U[w][t + x]  # bits 3-8: this wave's registers
                    x <<= 1
                for bb in (1, 2, 4):
                    if not (w & bb):
                        z ^= U[w | bb][t]  # bits 0-2: another wave's slot (LDS)
                Q[w][t] = z
    P = fft_to_p(Q, fft_tabs(C, 0), k)
    out = [None] * sum(1 for i in range(k) if not present[i])
    for p in range(k):
        if pl["pos_dst"][p] >= 0:
            out[pl["pos_dst"][p]] = mul(P[p >> 6][p & 63], pl["post"][p])
    return out


def test_qreg_is_a_permutation_each_round_refills_its_own_registers():
    assert sorted(qreg(t) for t in range(64)) == list(range(64))
    for R in range(2):  # round R frees P registers [32R, 32R + 32) and fills them with Q slots t & 7 in [4R, 4R + 4)
        assert sorted(qreg(t) for t in range(64) if (t & 7) // 4 == R) == list(range(32 * R, 32 * R + 32))


@pytest.mark.parametrize("k,m", [(300, 1000), (512, 600), (260, 600)])
def test_encode_lds_model(k, m):
    rng = np.random.default_rng(k + m)
    data = [int(x) for x in rng.integers(0, 65536, k)]
    assert encode_lds(data, k, m) == encode_low(data, k, m)


@pytest.mark.parametrize("k,m,case", [(300, 1000, "first"), (512, 600, "first"), (260, 600, "all"), (400, 1500, "second")])
def test_rec_lds_model(k, m, case):
    rng = np.random.default_rng(k * 7 + m)
    data = [int(x) for x in rng.integers(0, 65536, k)]
    par = encode_low(data, k, m)
    present = np.ones(k + m, np.uint8)
    if case == "all":
        present[:k] = 0
    else:
        present[rng.choice(k, size=min(k, 97), replace=False)] = 0
        if case == "second":
            present[k:k + 512] = 0
    lost = [data[i] for i in range(k) if not present[i]]
    assert rec_lds(data, par, k, m, [int(x) for x in present]) == lost
