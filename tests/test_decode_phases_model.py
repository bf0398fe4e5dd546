"""Dataflow model of the generic reconstruct's launch sequence (rs_kernels.hip
launch_decode_generic / k_dphase): the phase schedule (xform_phases), the sub-problem ->
positions map, the IFFT's zero tail (positions past round_up(trunc, span) neither written
nor read), the formal derivative split into in-register bits and partner loads, the FFT's
kept rows (Y) and skipped sub-problems, and the scatter — against the layer-by-layer
decode of root.zig:268-335 (Generic.zig:15-147 transforms, root.zig:306-312 derivative).

Symbols are 64-bit vectors over GF(2) and every twiddle a fixed GF(2)-linear map keyed by
(transform, layer distance, group start), so a schedule that skips, reorders or drops a
butterfly, or reads a position the previous phase did not write, changes the result. CPU
only: it checks index logic, not field arithmetic (the GPU parity tests do that)."""
import random

import pytest

MASK = (1 << 64) - 1


def rotl(x, a):
    a %= 64
    return ((x << a) | (x >> (64 - a))) & MASK if a else x


def tw(key):
    h = hash(key) & 0xFFFFFFFF
    a, b = 1 + h % 61, 1 + (h >> 8) % 59
    return lambda y: rotl(y, a) ^ rotl(y, b) ^ (y >> (h % 7 + 1))


def ifft_bf(x, i, j, f):
    x[j] ^= x[i]
    x[i] ^= f(x[j])


def fft_bf(x, i, j, f):
    x[i] ^= f(x[j])
    x[j] ^= x[i]


def ifft_ref(x, size, trunc):
    d = 1
    while 4 * d <= size:
        for r in range(0, min(trunc, size), 4 * d):
            m01, m23, m02 = tw(("i", d, r, 0)), tw(("i", d, r, 2)), tw(("i", d, r, 1))
            for i in range(r, r + d):
                ifft_bf(x, i, i + d, m01)
                ifft_bf(x, i + 2 * d, i + 3 * d, m23)
                ifft_bf(x, i, i + 2 * d, m02)
                ifft_bf(x, i + d, i + 3 * d, m02)
        d *= 4
    if d < size:  # final odd layer, distance size / 2, no truncation
        t = tw(("i", d, 0, 9))
        for i in range(d):
            ifft_bf(x, i, i + d, t)


def fft_ref(x, size, trunc):
    lg = size.bit_length() - 1
    d = 1 << (lg - 2) if lg >= 2 else 0
    d4 = size
    while d >= 1 and 4 * d == d4:
        for r in range(0, min(trunc, size), 4 * d):
            m01, m23, m02 = tw(("f", d, r, 0)), tw(("f", d, r, 2)), tw(("f", d, r, 1))
            for i in range(r, r + d):
                fft_bf(x, i, i + 2 * d, m02)
                fft_bf(x, i + d, i + 3 * d, m02)
                fft_bf(x, i, i + d, m01)
                fft_bf(x, i + 2 * d, i + 3 * d, m23)
        d4 = d
        d //= 4
    if d4 == 2:  # radix-2 tail, distance 1
        for r in range(0, min(trunc, size), 2):
            fft_bf(x, r, r + 1, tw(("f", 1, r, 9)))


def deriv_ref(x, W):
    for i in range(1, W):  # root.zig:306-312
        w = i & -i
        for j in range(w):
            x[i - w + j] ^= x[i + j]


def decode_ref(src, W, trunc, trunc_fft, dst):
    x = [src.get(p, 0) for p in range(W)]
    ifft_ref(x, W, trunc)
    deriv_ref(x, W)
    fft_ref(x, W, trunc_fft)
    return {p: x[p] for p in dst if p < trunc_fft}


# ---- the launch sequence, as rs_kernels.hip writes it
def xform_phases(size, inv):
    lg = size.bit_length() - 1
    n4, layer, r2_done, out = lg // 2, 0, not (lg & 1), []
    while True:
        c = min(3, n4 - layer)
        with_r2 = (not r2_done) and layer + c == n4 and c < 3
        nn = (1 << (2 * c)) << (1 if with_r2 else 0)
        dlo_log = 2 * layer if inv else (0 if (with_r2 or c == 0) else lg - 2 * (layer + c))
        out.append((nn, dlo_log))
        layer += c
        r2_done = r2_done or with_r2 or c == 0
        if not (layer < n4 or not r2_done):
            return out


def round_up(x, a):
    return (x + a - 1) // a * a


def ifft_sub(v, N, size, rmax, blk, dlo_log):
    jd, jd4 = 1, 4
    while jd4 <= N:
        d = jd << dlo_log
        for jr in range(0, N, jd4):
            r = blk + (jr << dlo_log)
            if r < rmax:
                m01, m23, m02 = tw(("i", d, r, 0)), tw(("i", d, r, 2)), tw(("i", d, r, 1))
                for i in range(jr, jr + jd):
                    ifft_bf(v, i, i + jd, m01)
                    ifft_bf(v, i + 2 * jd, i + 3 * jd, m23)
                    ifft_bf(v, i, i + 2 * jd, m02)
                    ifft_bf(v, i + jd, i + 3 * jd, m02)
        jd, jd4 = jd4, jd4 * 4
    if jd < N:
        t = tw(("i", jd << dlo_log, 0, 9))
        for i in range(jd):
            ifft_bf(v, i, jd + i, t)


def fft_sub(v, N, size, rmax, blk, dlo_log):
    jd4, jd = N, N >> 2
    while jd != 0:
        d = jd << dlo_log
        for jr in range(0, N, jd4):
            r = blk + (jr << dlo_log)
            if r < rmax:
                m01, m23, m02 = tw(("f", d, r, 0)), tw(("f", d, r, 2)), tw(("f", d, r, 1))
                for i in range(jr, jr + jd):
                    fft_bf(v, i, i + 2 * jd, m02)
                    fft_bf(v, i + jd, i + 3 * jd, m02)
                    fft_bf(v, i, i + jd, m01)
                    fft_bf(v, i + 2 * jd, i + 3 * jd, m23)
        jd4, jd = jd, jd >> 2
    if jd4 == 2:
        for jr in range(0, N, 2):
            r = blk + jr
            if r < rmax:
                fft_bf(v, jr, jr + 1, tw(("f", 1, r, 9)))


def decode_phased(src, W, trunc, trunc_fft, dst):
    ri, rf = min(trunc, W), min(trunc_fft, W)
    fph = xform_phases(W, False)
    ylen = min(W, round_up(rf, 1 << fph[0][1])) if len(fph) > 1 else 0
    X = [None] * W  # None: never written (reading it is a schedule bug)
    Y = [None] * max(ylen, 1)  # A: F1((I + H) X), then the later phases in place
    B = [None] * max(ylen, 1)  # F1(X)
    out = {}
    lim = 0
    iph = xform_phases(W, True)
    fuse = len(iph) >= 2  # the last IFFT phase runs inside the first FFT phase's loads
    NI, DI = iph[-1]
    for i, (N, dl) in enumerate(iph[:-1] if fuse else iph):
        span = N << dl
        wl = round_up(ri, span)
        n_src = ri if i == 0 else lim
        for sub in range(wl // N):
            blk, lo = (sub >> dl) * span, sub & ((1 << dl) - 1)
            ps = [blk + lo + (j << dl) for j in range(N)]
            if i == 0:
                v = [src.get(p, 0) if p < n_src else 0 for p in ps]
            else:
                v = [X[p] if p < n_src else 0 for p in ps]
            ifft_sub(v, N, W, ri, blk, dl)
            for j, p in enumerate(ps):
                if p < wl:
                    X[p] = v[j]
        lim = wl
    # the derivative D = I + H + L (H: the bits the first FFT phase holds, L: the bits below
    # its stride). L acts on the low bits only and the first phase F1 on the high bits only,
    # so F1 D = F1 (I + H) + L F1: the first phase writes A = F1((I + H) X) and B = F1(X),
    # the second reads A + L B (L's bits it holds in registers, the rest as loads of B)
    for i, (N, dl) in enumerate(fph):
        span = N << dl
        wl = round_up(rf, span)
        first, last = i == 0, i + 1 == len(fph)
        snap = list(Y)
        for sub in range(wl // N):
            blk, lo = (sub >> dl) * span, sub & ((1 << dl) - 1)
            ps = [blk + lo + (j << dl) for j in range(N)]

            def load_x():
                if not fuse:
                    return [X[p] for p in ps]
                x = [X[p] if p < lim else 0 for p in ps]
                G = N // NI
                assert blk == 0 and (1 << (DI - dl)) == G
                for g in range(G):  # the IFFT's last phase on each of its sub-problems
                    w = [x[g + t * G] for t in range(NI)]
                    ifft_sub(w, NI, W, ri, 0, DI)
                    for t in range(NI):
                        x[g + t * G] = w[t]
                return x
            if first:
                v = load_x()
                for j in range(N):  # in-register derivative bits (ascending)
                    bb = 1
                    while bb < N:
                        if not j & bb:
                            v[j] ^= v[j + bb]
                        bb <<= 1
                if not last:  # B = F1(X): the same sub-problem without the derivative
                    w = load_x()
                    fft_sub(w, N, W, rf, blk, dl)
                    for j, p in enumerate(ps):
                        if p < ylen:
                            B[p] = w[j]
            elif i == 1:
                lsum = fph[0][1]  # L's bits: below the first phase's stride
                v = [B[p] for p in ps]
                for j in range(N):  # L's bits this sub-problem holds (ascending, t excludes v[j])
                    t, bb = 0, 1
                    while bb < N:
                        if not j & bb:
                            t ^= v[j + bb]
                        bb <<= 1
                    v[j] = t
                for b in range(dl):  # L's bits below this phase's stride: loads of B
                    if (lo >> b) & 1:
                        continue
                    for j in range(N):
                        v[j] ^= B[blk + lo + (1 << b) + (j << dl)]
                assert (N << dl) == (1 << lsum) or blk > 0
                for j, p in enumerate(ps):
                    v[j] ^= snap[p]
            else:
                v = [snap[p] for p in ps]
            fft_sub(v, N, W, rf, blk, dl)
            for j, p in enumerate(ps):
                if last:
                    if p < rf and p in dst:
                        out[p] = v[j]
                elif p < ylen:
                    Y[p] = v[j]
    return out


def case(W, trunc, trunc_fft, seed):
    rng = random.Random(seed)
    src = {p: rng.getrandbits(64) for p in range(trunc) if rng.random() < 0.7}
    dst = {p for p in range(trunc_fft) if rng.random() < 0.3}
    return src, dst


@pytest.mark.parametrize("W,trunc,trunc_fft", [
    (64, 40, 40), (128, 100, 70), (256, 200, 77), (512, 300, 300), (1024, 1000, 33),
    (2048, 1512, 300), (2048, 1128, 1128), (4096, 2600, 2600), (8192, 5024, 1000), (128, 128, 128),
])
def test_phased_decode_matches_layer_walk(W, trunc, trunc_fft):
    src, dst = case(W, trunc, trunc_fft, W * 7 + trunc)
    assert decode_phased(src, W, trunc, trunc_fft, dst) == decode_ref(src, W, trunc, trunc_fft, dst)


# ---- the low-rate encode's launch sequence (rs_kernels.hip launch_encode_low_phases)
def encode_ref(data, C, k, m):
    x = [data.get(p, 0) for p in range(C)]
    ifft_ref(x, C, k)
    out = {}
    for j in range((m + C - 1) // C):
        t = min(C, m - j * C)
        y = list(x)
        fft_ref_keyed(y, C, t, j)
        for p in range(t):
            out[j * C + p] = y[p]
    return out


def fft_ref_keyed(x, size, trunc, chunk):
    """fft_ref with twiddles keyed by the chunk too (each chunk has its own skew)."""
    lg = size.bit_length() - 1
    d, d4 = 1 << (lg - 2) if lg >= 2 else 0, size
    while d >= 1 and 4 * d == d4:
        for r in range(0, min(trunc, size), 4 * d):
            m01, m23, m02 = tw(("f", chunk, d, r, 0)), tw(("f", chunk, d, r, 2)), tw(("f", chunk, d, r, 1))
            for i in range(r, r + d):
                fft_bf(x, i, i + 2 * d, m02)
                fft_bf(x, i + d, i + 3 * d, m02)
                fft_bf(x, i, i + d, m01)
                fft_bf(x, i + 2 * d, i + 3 * d, m23)
        d4, d = d, d // 4
    if d4 == 2:
        for r in range(0, min(trunc, size), 2):
            fft_bf(x, r, r + 1, tw(("f", chunk, 1, r, 9)))


def fft_sub_keyed(v, N, rmax, blk, dlo_log, chunk):
    jd4, jd = N, N >> 2
    while jd != 0:
        d = jd << dlo_log
        for jr in range(0, N, jd4):
            r = blk + (jr << dlo_log)
            if r < rmax:
                m01, m23, m02 = tw(("f", chunk, d, r, 0)), tw(("f", chunk, d, r, 2)), tw(("f", chunk, d, r, 1))
                for i in range(jr, jr + jd):
                    fft_bf(v, i, i + 2 * jd, m02)
                    fft_bf(v, i + jd, i + 3 * jd, m02)
                    fft_bf(v, i, i + jd, m01)
                    fft_bf(v, i + 2 * jd, i + 3 * jd, m23)
        jd4, jd = jd, jd >> 2
    if jd4 == 2:
        for jr in range(0, N, 2):
            r = blk + jr
            if r < rmax:
                fft_bf(v, jr, jr + 1, tw(("f", chunk, 1, r, 9)))


def encode_phased(data, C, k, m):
    iph, fph = xform_phases(C, True), xform_phases(C, False)
    fuse = len(iph) >= 2
    NI, DI = iph[-1]
    X = [None] * C
    lim = 0
    for i, (N, dl) in enumerate(iph[:-1] if fuse else iph):
        span = N << dl
        wl = round_up(k, span)
        for sub in range(wl // N):
            blk, lo = (sub >> dl) * span, sub & ((1 << dl) - 1)
            ps = [blk + lo + (j << dl) for j in range(N)]
            v = [data.get(p, 0) if p < k else 0 for p in ps] if i == 0 else [X[p] if p < lim else 0 for p in ps]
            ifft_sub(v, N, C, k, blk, dl)
            for j, p in enumerate(ps):
                if p < wl:
                    X[p] = v[j]
        lim = wl
    out = {}
    for ch in range((m + C - 1) // C):
        t = min(C, m - ch * C)
        Y = [None] * C
        for i, (N, dl) in enumerate(fph):
            span = N << dl
            first, last = i == 0, i + 1 == len(fph)
            snap = list(Y)
            for sub in range(C // N):
                blk, lo = (sub >> dl) * span, sub & ((1 << dl) - 1)
                if blk >= t:
                    continue
                ps = [blk + lo + (j << dl) for j in range(N)]
                if first:
                    v = [X[p] if (not fuse or p < lim) else 0 for p in ps] if fuse else [X[p] for p in ps]
                    if fuse:
                        G = N // NI
                        for g in range(G):
                            w = [v[g + u * G] for u in range(NI)]
                            ifft_sub(w, NI, C, k, 0, DI)
                            for u in range(NI):
                                v[g + u * G] = w[u]
                else:
                    v = [snap[p] for p in ps]
                fft_sub_keyed(v, N, t, blk, dl, ch)
                n_dst = round_up(t, 1 << dl)
                for j, p in enumerate(ps):
                    if last:
                        if p < t:
                            out[ch * C + p] = v[j]
                    elif p < n_dst:
                        Y[p] = v[j]
    return out


@pytest.mark.parametrize("C,k,m", [(64, 40, 100), (128, 100, 300), (512, 300, 1000), (1024, 1000, 4000),
                                   (256, 200, 56), (2048, 1500, 2100)])
def test_phased_low_rate_encode_matches_layer_walk(C, k, m):
    rng = random.Random(C + k + m)
    data = {p: rng.getrandbits(64) for p in range(k)}
    assert encode_phased(data, C, k, m) == encode_ref(data, C, k, m)
