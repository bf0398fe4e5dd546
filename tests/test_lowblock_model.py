"""Model of the low-rate block-form reconstruct's launch sequence (rs_kernels.hip
launch_low_blocks: k_ephase GATHER / FFT / SYN, k_lbfinal, k_dphase LSUM / SCATTER) with the
field arithmetic of the library's own tables (R.table: exp / log / skew / log_walsh), one
symbol per row, against the lost data.

Each kernel is restated from its device code: the phase schedule (xform_phases), the
sub-problem -> positions map, truncation (rows past n_src read as zero, rows past n_dst not
stored, FFT sub-problems past rmax skipped), the fused IFFT last phase (ifft_last_in), the
syndromes, D_C's split (H in k_lbfinal, L in LSUM) and the scatter. Scratch rows never written
are None, so a read of one fails, and a row one sub-problem of a launch writes and another
reads is a race (the GPU runs a launch's sub-problems concurrently). The host plan
(rs_lowrate.cpp build_block_plan: erasure logs, the block scalars alpha / beta, sigma / gamma /
u) is restated too. Parity unpinned, as every low-rate path; the encode it decodes is checked
against the oracle's rso_encode_low."""
import numpy as np
import pytest

from rs_amd import reedsol_amd as R

MOD = 65535
EXP = np.asarray(R.table("exp"), dtype=np.int64)
LOG = np.asarray(R.table("log"), dtype=np.int64)
SKEW = np.asarray(R.table("skew"), dtype=np.int64)
LOG_WALSH = np.asarray(R.table("log_walsh"), dtype=np.int64)


def add_mod(x, y):
    s = x + y
    return (s + (s >> 16)) & 0xFFFF


def mul(x, lm):  # utilities.zig:5-8 (mul16): x * exp(lm)
    return 0 if x == 0 else int(EXP[add_mod(int(LOG[x]), lm)])


def gmul(x, y):
    return 0 if x == 0 or y == 0 else mul(x, int(LOG[y]))


def twiddle(idx):  # make_twiddle: the skew log, MOD = XOR only
    return int(SKEW[idx]) if idx < MOD else MOD


def ifft_bf(s, i, j, lm):
    s[j] ^= s[i]
    if lm != MOD:
        s[i] ^= mul(s[j], lm)


def fft_bf(s, i, j, lm):
    if lm != MOD:
        s[i] ^= mul(s[j], lm)
    s[j] ^= s[i]


# ---------------------------------------------------------------- scalar transforms (rs_gf.cpp)
def scalar_ifft(s, size, trunc, sd):
    d, d4 = 1, 4
    while d4 <= size:
        for r in range(0, trunc, d4):
            b = r + d + sd - 1
            m01, m02, m23 = twiddle(b), twiddle(b + d), twiddle(b + 2 * d)
            for i in range(r, r + d):
                ifft_bf(s, i, i + d, m01)
                ifft_bf(s, i + 2 * d, i + 3 * d, m23)
                ifft_bf(s, i, i + 2 * d, m02)
                ifft_bf(s, i + d, i + 3 * d, m02)
        d, d4 = d4, d4 * 4
    if d < size:
        lm = twiddle(d + sd - 1)
        for i in range(d):
            ifft_bf(s, i, d + i, lm)


def scalar_fft(s, size, trunc, sd):
    d4, d = size, size >> 2
    while d:
        for r in range(0, trunc, d4):
            b = r + d + sd - 1
            m01, m02, m23 = twiddle(b), twiddle(b + d), twiddle(b + 2 * d)
            for i in range(r, r + d):
                fft_bf(s, i, i + 2 * d, m02)
                fft_bf(s, i + d, i + 3 * d, m02)
                fft_bf(s, i, i + d, m01)
                fft_bf(s, i + 2 * d, i + 3 * d, m23)
        d4, d = d, d >> 2
    if d4 == 2:
        for r in range(0, trunc, 2):
            fft_bf(s, r, r + 1, twiddle(r + sd))


def ceil_pow2(x):
    return 1 << (x - 1).bit_length()


def encode_low(data, k, m):  # scalar_encode_low
    C = ceil_pow2(k)
    coef = list(data) + [0] * (C - k)
    scalar_ifft(coef, C, k, 0)
    out = []
    for j in range((m + C - 1) // C):
        b = list(coef)
        t = min(C, m - j * C)
        scalar_fft(b, C, t, (j + 1) * C)
        out += b[:t]
    return out


# ---------------------------------------------------------------- host plan (rs_lowrate.cpp)
def fwht(e, m):  # walsh_hadamard.zig:16-62 over the first m positions (u16 offsets)
    dist, stride = 1, 4
    while stride <= 65536:
        nblk = max(1, -(-m // stride))
        v = e[: nblk * stride].reshape(nblk, 4, dist)
        x0, x1, x2, x3 = v[:, 0].copy(), v[:, 1].copy(), v[:, 2].copy(), v[:, 3].copy()
        sub = lambda x, y: ((x + MOD - y) + ((x + MOD - y) >> 16)) & 0xFFFF
        s0, d0, s1, d1 = add_mod(x0, x1), sub(x0, x1), add_mod(x2, x3), sub(x2, x3)
        v[:, 0], v[:, 1], v[:, 2], v[:, 3] = add_mod(s0, s1), add_mod(d0, d1), sub(s0, s1), sub(d0, d1)
        dist, stride = stride, stride * 4


def erasure_logs_low(received, k, m):
    C = ceil_pow2(k)
    end = C + m
    W = ceil_pow2(end)
    er = np.zeros(65536, np.int64)
    for i in range(k):
        er[i] = 0 if received[i] else 1
    for i in range(C, end):
        er[i] = 0 if received[i] else 1
    er[end:W] = 1
    fwht(er, W)
    p = er * LOG_WALSH
    er = add_mod(p & 0xFFFF, p >> 16)
    fwht(er, 65536)
    return [int(x) for x in er]


def block_coefs(k, m):  # low_block_coefs
    C = ceil_pow2(k)
    W = ceil_pow2(C + m)
    nb = W // C
    lam = [[1 if i == j else 0 for j in range(nb)] for i in range(nb)]

    def tw(idx):
        lm = twiddle(idx)
        return 0 if lm == MOD else int(EXP[lm])

    def axpy(y, t, x):
        for K in range(nb):
            y[K] ^= gmul(t, x[K])

    d = C
    while d < W:
        for g in range(0, W, 2 * d):
            t = tw(g + d - 1)
            for i in range(g, g + d, C):
                x, y = lam[i // C], lam[(i + d) // C]
                for K in range(nb):
                    y[K] ^= x[K]
                axpy(x, t, y)
        d *= 2
    P = [list(r) for r in lam]
    Q = [[0] * nb for _ in range(nb)]
    for J in range(nb):
        b = 1
        while b < nb:
            if not (J & b) and J + b < nb:
                for K in range(nb):
                    Q[J][K] ^= lam[J + b][K]
            b <<= 1
    d = W // 2
    while d >= C and d > 0:
        for g in range(0, W, 2 * d):
            t = tw(g + d - 1)
            for i in range(g, g + d, C):
                x, y = i // C, (i + d) // C
                axpy(P[x], t, P[y])
                axpy(Q[x], t, Q[y])
                for K in range(nb):
                    P[y][K] ^= P[x][K]
                    Q[y][K] ^= Q[x][K]
        d //= 2
    return P[0], Q[0]


def block_plan(k, m, present):  # build_block_plan
    C = ceil_pow2(k)
    W = ceil_pow2(C + m)
    e = sum(1 for i in range(k) if not present[i])
    received = [0] * W
    for i in range(k):
        received[i] = present[i]
    nr = 0
    for r in range(m):
        if nr < e and present[k + r]:
            received[C + r] = 1
            nr += 1
    assert nr == e
    er = erasure_logs_low(received, k, m)
    mp = max(r + 1 for r in range(m) if received[C + r])
    nbk = -(-mp // C)
    alpha, beta = block_coefs(k, m)
    u, sig, gamma = [], [], []
    for j in range(nbk):
        al, be = alpha[j + 1], beta[j + 1]
        if al:
            u.append(1), sig.append(al), gamma.append(gmul(be, int(EXP[(MOD - int(LOG[al])) % MOD])))
        else:
            u.append(0), sig.append(be), gamma.append(1)
    syn_idx = [-1] * (nbk * C)
    syn_log = [None] * (nbk * C)
    for r in range(mp):
        if received[C + r]:
            syn_idx[r] = 1
            syn_log[r] = add_mod(er[C + r], int(LOG[sig[r // C]])) if sig[r // C] else None
    pos_dst, post = [-1] * C, [None] * C
    ne = 0
    for g in range(k):
        if not received[g]:
            pos_dst[g], post[g] = ne, MOD - er[g]
            ne += 1
    return dict(C=C, mp=mp, nbk=nbk, u=u, gamma=gamma, syn_idx=syn_idx, syn_log=syn_log, pos_dst=pos_dst,
                post=post, skip=[not present[i] for i in range(k)])


# ---------------------------------------------------------------- device phases (rs_kernels.hip)
def xform_phases(size, inv):
    lg = size.bit_length() - 1
    n4, layer, r2_done, ti, out = lg // 2, 0, not (lg & 1), 0, []
    while True:
        c = min(3, n4 - layer)
        with_r2 = not r2_done and layer + c == n4 and c < 3
        nn = (1 << (2 * c)) << (1 if with_r2 else 0)
        out.append((nn, 2 * layer if inv else (0 if with_r2 or c == 0 else lg - 2 * (layer + c)), ti))
        for l in range(layer, layer + c):
            ti += 3 * (size >> (2 * l + 2)) if inv else 3 << (2 * l)
        layer += c
        r2_done = r2_done or with_r2 or c == 0
        if not (layer < n4 or not r2_done):
            return out


def ifft_tabs(size, sd):  # push_ifft_tabs
    out, d, d4 = [], 1, 4
    while d4 <= size:
        for r in range(0, size, d4):
            b = r + d + sd - 1
            out += [twiddle(b), twiddle(b + d), twiddle(b + 2 * d)]
        d, d4 = d4, d4 * 4
    if d < size:
        out.append(twiddle(d + sd - 1))
    return out


def fft_tabs(size, sd):  # push_fft_tabs
    out, d4, d = [], size, size >> 2
    while d:
        for r in range(0, size, d4):
            b = r + d + sd - 1
            out += [twiddle(b), twiddle(b + d), twiddle(b + 2 * d)]
        d4, d = d, d >> 2
    if d4 == 2:
        out += [twiddle(r + sd) for r in range(0, size, 2)]
    return out


def ctz(x):
    return (x & -x).bit_length() - 1


def ifft_sub(s, tabs, ti, size, rmax, blk, dlo_log):
    N, jd, jd4 = len(s), 1, 4
    while jd4 <= N:
        lg4 = ctz(jd4) + dlo_log
        for jr in range(0, N, jd4):
            r = blk + (jr << dlo_log)
            if r < rmax:
                g = ti + 3 * (r >> lg4)
                m01, m02, m23 = tabs[g], tabs[g + 1], tabs[g + 2]
                for i in range(jr, jr + jd):
                    ifft_bf(s, i, i + jd, m01)
                    ifft_bf(s, i + 2 * jd, i + 3 * jd, m23)
                    ifft_bf(s, i, i + 2 * jd, m02)
                    ifft_bf(s, i + jd, i + 3 * jd, m02)
        ti += 3 * (size >> lg4)
        jd, jd4 = jd4, jd4 * 4
    if jd < N:
        t = tabs[ti]
        for i in range(jd):
            ifft_bf(s, i, jd + i, t)


def fft_sub(s, tabs, ti, size, rmax, blk, dlo_log):
    N, jd4, jd = len(s), len(s), len(s) >> 2
    while jd:
        lg4 = ctz(jd4) + dlo_log
        for jr in range(0, N, jd4):
            r = blk + (jr << dlo_log)
            if r < rmax:
                g = ti + 3 * (r >> lg4)
                m01, m02, m23 = tabs[g], tabs[g + 1], tabs[g + 2]
                for i in range(jr, jr + jd):
                    fft_bf(s, i, i + 2 * jd, m02)
                    fft_bf(s, i + jd, i + 3 * jd, m02)
                    fft_bf(s, i, i + jd, m01)
                    fft_bf(s, i + 2 * jd, i + 3 * jd, m23)
        ti += 3 * (size >> lg4)
        jd4, jd = jd, jd >> 2
    if jd4 == 2:
        for jr in range(0, N, 2):
            r = blk + jr
            if r < rmax:
                fft_bf(s, jr, jr + 1, tabs[ti + r // 2])


def ifft_last_in(v, NI, tabs_i, ti_i, size, rmax_i, dlo_i):
    if NI:
        G = len(v) // NI
        for g in range(G):
            w = [v[g + t * G] for t in range(NI)]
            ifft_sub(w, tabs_i, ti_i, size, rmax_i, 0, dlo_i)
            for t in range(NI):
                v[g + t * G] = w[t]


class Scratch:
    """One stripe's scratch rows; None = never written. A launch records which sub-problem
    wrote each row: a row read by another sub-problem of the same launch is a race."""

    def __init__(self, rows):
        self.rows = [None] * rows
        self.owner = {}

    def launch(self):
        self.owner = {}

    def read(self, i, sub):
        assert self.rows[i] is not None, f"read of unwritten scratch row {i}"
        assert self.owner.get(i, sub) == sub, f"row {i} written and read by different sub-problems"
        return self.rows[i]

    def write(self, i, v, sub):
        assert self.owner.get(i, sub) == sub, f"row {i} written by two sub-problems"
        self.owner[i] = sub
        self.rows[i] = v


def round_up(x, a):
    return -(-x // a) * a


def model_low_blocks(k, m, data, rec, present):
    """launch_low_blocks on one stripe (data: k symbols, erased ones garbage; rec: m)."""
    P = block_plan(k, m, present)
    C, mp, nbk = P["C"], P["mp"], P["nbk"]
    iph, fph = xform_phases(C, True), xform_phases(C, False)
    assert len(iph) >= 2 and 2 <= len(fph) <= 3 and fph[0][0] == 64 and (64 << fph[0][1]) == C
    assert (64 >> (iph[-1][1] - fph[0][1])) == iph[-1][0]
    ylen = round_up(k, 1 << fph[0][1])
    # two IFFT phases: the derivative whole before the final FFT (k_ephase DLO + k_lbfin1);
    # per stripe X | R1 | W | A' for it, X | R1 | A' | B' for the split (low_block_rows)
    whole = len(iph) == 2 and len(fph) == 2
    X, R1 = 0, C
    Wr, Ap = (2 * C, 3 * C) if whole else (None, 2 * C)
    Bp = None if whole else Ap + ylen
    S = Scratch(3 * C + ylen if whole else 2 * C + 2 * ylen)
    tabsE = ifft_tabs(C, 0)
    TI = len(tabsE)
    for j in range(nbk):
        tabsE += fft_tabs(C, (j + 1) * C)
    TPC = len(fft_tabs(C, 0))
    tabsF = fft_tabs(C, 0)

    def positions(N, sub, dlo_log):
        dlo = 1 << dlo_log
        blk = (sub >> dlo_log) * (N << dlo_log)
        lo = sub & (dlo - 1)
        return blk, [blk + lo + (jj << dlo_log) for jj in range(N)]

    # 1. coefficients: the IFFT's phases but the last (k_ephase GATHER, then plain)
    lim = 0
    for i in range(len(iph) - 1):
        n, dl, ti = iph[i]
        wl = round_up(k, n << dl)
        S.launch()
        for sub in range(wl // n):
            blk, ps = positions(n, sub, dl)
            if i == 0:
                v = [data[p] if p < k and not P["skip"][p] else 0 for p in ps]
            else:
                v = [S.read(X + p, sub) if p < lim else 0 for p in ps]
            ifft_sub(v, tabsE, ti, C, k, blk, dl)
            for p, x in zip(ps, v):
                if p < wl:
                    S.write(X + p, x, sub)
        lim = wl
    ni, dli, tii = iph[-1]
    for j in range(nbk):
        rj = min(C, mp - j * C)
        # 2. FFT_{C, skew (j+1)C}: first phase with the coefficients' IFFT last phase, SYN last
        for i, (n, dl, ti) in enumerate(fph):
            first, last = i == 0, i + 1 == len(fph)
            S.launch()
            for sub in range(C // n):
                blk, ps = positions(n, sub, dl)
                if blk >= rj:
                    continue
                src = X if first else R1
                nsrc = lim if first else C
                v = [S.read(src + p, sub) if p < nsrc else 0 for p in ps]
                if first:
                    ifft_last_in(v, ni, tabsE, tii, C, k, dli)
                fft_sub(v, tabsE[TI + j * TPC:], ti, C, rj, blk, dl)
                if last:  # SYN
                    for jj, p in enumerate(ps):
                        r = j * C + p
                        if p < rj and P["syn_idx"][r] >= 0:
                            lg = P["syn_log"][r]
                            v[jj] = 0 if lg is None else mul(v[jj] ^ rec[r], lg)
                        else:
                            v[jj] = 0
                        if p < rj:
                            S.write(R1 + p, v[jj], sub)
                else:
                    ndst = round_up(rj, 1 << dl)
                    for p, x in zip(ps, v):
                        if p < ndst:
                            S.write(R1 + p, x, sub)
        # IFFT_{C, skew (j+1)C} in region 1 but its last phase
        tabsI = ifft_tabs(C, (j + 1) * C)
        lj = rj
        for i in range(len(iph) - 1):
            n, dl, ti = iph[i]
            wl = round_up(rj, n << dl)
            S.launch()
            for sub in range(wl // n):
                blk, ps = positions(n, sub, dl)
                v = [S.read(R1 + p, sub) if p < lj else 0 for p in ps]
                ifft_sub(v, tabsI, ti, C, rj, blk, dl)
                for p, x in zip(ps, v):
                    if p < wl:
                        S.write(R1 + p, x, sub)
                if whole:  # DLO: W = ((1 + gamma) I + D_lo) U over the phase's 64 positions, ascending
                    g1 = (1 ^ P["gamma"][j]) if P["u"][j] else 0
                    for jj in range(n):
                        t = gmul(v[jj], g1)
                        bb = 1
                        while bb < n:
                            if not (jj & bb):
                                t ^= v[jj + bb]
                            bb <<= 1
                        v[jj] = t
                    for p, x in zip(ps, v):
                        if p < wl:
                            S.write(Wr + p, x, sub)
            lj = wl
        n0, dl0, ti0 = fph[0]
        if whole:  # k_lbfin1
            S.launch()
            G = 64 // ni
            for sub in range(C // 64):
                blk, ps = positions(64, sub, dl0)
                v = [S.read(R1 + p, sub) if p < lj else 0 for p in ps]
                ifft_last_in(v, ni, tabsI, tii, C, rj, dli)
                if P["u"][j]:
                    for jj in range(64):  # D_hi U, ascending
                        t = 0
                        bb = G
                        while bb < 64:
                            if not (jj & bb):
                                t ^= v[jj + bb]
                            bb <<= 1
                        v[jj] = t
                    for gg in range(G):  # + IFFT_last(W)
                        w = [S.read(Wr + ps[gg + t * G], sub) if ps[gg + t * G] < lj else 0 for t in range(ni)]
                        ifft_sub(w, tabsI, tii, C, rj, 0, dli)
                        for t in range(ni):
                            v[gg + t * G] ^= w[t]
                fft_sub(v, tabsF, ti0, C, k, blk, dl0)
                for jj, p in enumerate(ps):
                    if p < ylen:
                        if j > 0:
                            v[jj] ^= S.read(Ap + p, sub)
                        S.write(Ap + p, v[jj], sub)
            continue
        # k_lbfinal
        S.launch()
        for sub in range(C // 64):
            blk, ps = positions(64, sub, dl0)
            for pas in ([0, 1] if P["u"][j] or j == 0 else [1]):
                v = [S.read(R1 + p, sub) if p < lj and (pas == 1 or P["u"][j]) else 0 for p in ps]
                ifft_last_in(v, ni, tabsI, tii, C, rj, dli)
                if pas == 1 and P["u"][j]:
                    for jj in range(64):
                        t = gmul(v[jj], P["gamma"][j])
                        bb = 1
                        while bb < 64:
                            if not (jj & bb):
                                v[jj] ^= v[jj + bb]
                            bb <<= 1
                        v[jj] ^= t
                fft_sub(v, tabsF, ti0, C, k, blk, dl0)
                base = Bp if pas == 0 else Ap
                for jj, p in enumerate(ps):
                    if p < ylen:
                        if j > 0:
                            v[jj] ^= S.read(base + p, sub)
                        S.write(base + p, v[jj], sub)
    # 3. LSUM (+ SCATTER), then SCATTER
    out = {}
    for i in range(1, len(fph)):
        n, dl, ti = fph[i]
        last = i + 1 == len(fph)
        wl = round_up(k, n << dl)
        S.launch()
        for sub in range(wl // n):
            blk, ps = positions(n, sub, dl)
            lo = ps[0] - blk
            if i == 1 and not whole:  # LSUM: A' + L B'
                Bv = [S.read(Bp + p, sub) if p < ylen else 0 for p in ps]
                v = []
                for jj in range(n):
                    t, bb = 0, 1
                    while bb < n:
                        if not (jj & bb):
                            t ^= Bv[jj + bb]
                        bb <<= 1
                    v.append(t)
                for b in range(dl):
                    if (lo >> b) & 1:
                        continue
                    for jj, p in enumerate(ps):
                        if p + (1 << b) < ylen:
                            v[jj] ^= S.read(Bp + p + (1 << b), sub)
                for jj, p in enumerate(ps):
                    if p < ylen:
                        v[jj] ^= S.read(Ap + p, sub)
            else:
                v = [S.read(Ap + p, sub) if p < ylen else 0 for p in ps]
            fft_sub(v, tabsF, ti, C, k, blk, dl)
            for jj, p in enumerate(ps):
                if last:
                    if p < k and P["pos_dst"][p] >= 0:
                        out[p] = mul(v[jj], P["post"][p])
                elif p < ylen:
                    S.write(Ap + p, v[jj], sub)
    return out


CASES = [
    (100, 600, "first"), (100, 600, "spread"), (100, 600, "tail"), (130, 300, "all"), (300, 1000, "first"),
    (300, 1000, "spread"), (200, 1000, "one"), (64 + 1, 200, "spread"),
    (5000, 9000, "spread"),  # C = 8192: three-phase transforms, the A' / B' split and LSUM
]


@pytest.mark.parametrize("k,m,case", CASES)
def test_low_block_model(oracle, k, m, case):
    rng = np.random.default_rng(k * 7 + m + len(case))
    data = [int(x) for x in rng.integers(0, 65536, k)]
    rec = encode_low(data, k, m)
    # pin the model's encode on the oracle (symbol 0 of 64-byte shards)
    sh = np.zeros((k, 64), np.uint8)
    sh[:, 0] = [x & 0xFF for x in data]
    sh[:, 32] = [x >> 8 for x in data]
    st, exp = oracle.encode_low(k, m, sh)
    assert st == 0
    assert [int(exp[r, 0]) | int(exp[r, 32]) << 8 for r in range(m)] == rec
    C = ceil_pow2(k)
    present = [1] * (k + m)
    e = min(k, 97)
    lost = list(rng.choice(k, size=e, replace=False))
    if case == "all":
        lost = list(range(k))
        for r in range(m // 3):
            present[k + r] = 0
    elif case == "one":
        lost = [int(rng.integers(0, k))]
    elif case == "spread":
        for r in range(C - e // 2):
            present[k + r] = 0
    elif case == "tail":
        for r in range(m - e - 3):
            present[k + r] = 0
    for g in lost:
        present[g] = 0
    garbled = [x if present[i] else 0xBEEF for i, x in enumerate(data)]
    got = model_low_blocks(k, m, garbled, rec, present)
    assert sorted(got) == sorted(int(g) for g in lost)
    for g, x in got.items():
        assert x == data[g], (g, x, data[g])
