"""Host erasure locators, no GPU (rs_gf.cpp erasure_logs / erasure_logs_low).

A plan's erasure logs (root.zig:277-289: the erasure indicator through evalPoly,
Generic.zig:200-215) are the dyadic convolution er[i] = sum over erased j of log[i ^ j]
mod 65535. The library sums a small erased set point by point instead of running the two
65536-point transforms (~1.1 ms on a first call's critical path); this checks, through the
rs_debug_erasure_logs_check hook, that both agree mod 65535 at every position a plan reads,
for high-rate and low-rate layouts, random and edge patterns (no loss, every recovery row
lost, every original lost, the largest sets still summed directly, sets large enough to
take the transforms).
"""
import numpy as np
import pytest

from rs_amd import reedsol_amd as R


def _ceil_pow2(x):
    return 1 << (x - 1).bit_length()


def _high(k, m, lost_orig, lost_rec):
    C = _ceil_pow2(m)
    rcv = np.zeros(C + k, np.uint8)
    rcv[:m] = 1
    rcv[C:C + k] = 1
    rcv[list(lost_rec)] = 0
    rcv[[C + g for g in lost_orig]] = 0
    return rcv


def _low(k, m, lost_orig, lost_rec):
    C = _ceil_pow2(k)
    rcv = np.zeros(C + m, np.uint8)
    rcv[:C] = 1
    rcv[C:C + m] = 1
    rcv[list(lost_orig)] = 0
    rcv[[C + r for r in lost_rec]] = 0
    return rcv


@pytest.mark.parametrize("k,m", [(1, 1), (2, 2), (3, 2), (10, 4), (16, 16), (32, 8), (40, 12), (64, 64),
                                 (200, 55), (1000, 100), (4096, 512)])
def test_high_rate_direct_logs_match_eval_poly(k, m):
    rng = np.random.default_rng(k * 1000 + m)
    cases = [((), ()), (range(min(k, m)), ()), ((), range(m))]
    for _ in range(6):
        e = int(rng.integers(0, m + 1))
        lost = rng.choice(k + m, size=e, replace=False)
        cases.append(([g for g in lost if g < k], [g - k for g in lost if g >= k]))
    for lo, lr in cases:
        assert R.debug_erasure_logs_check(k, m, _high(k, m, lo, lr)) == 0, (k, m, lo, lr)


@pytest.mark.parametrize("k,m", [(4, 12), (300, 1000), (1000, 4000), (20, 2000)])
def test_low_rate_direct_logs_match_eval_poly(k, m):
    rng = np.random.default_rng(k * 7 + m)
    cases = [((), ())]
    for _ in range(4):
        e = int(rng.integers(0, min(k, m) + 1))
        lost = rng.choice(k + m, size=e, replace=False)
        cases.append(([g for g in lost if g < k], [g - k for g in lost if g >= k]))
    for lo, lr in cases:
        assert R.debug_erasure_logs_check(k, m, _low(k, m, lo, lr), low=True) == 0, (k, m, lo, lr)


def test_invalid_arguments():
    assert R.debug_erasure_logs_check(0, 4, [1] * 8) == -1
    assert R.debug_erasure_logs_check(4, 0, [1] * 8) == -1
