"""CPU: the hybrid lanes' closed-form bisection (wv_lane.h lhy_code, HY == 1) equals the
step loop it replaces (get_word's hybrid branch, WordsUtils.cs:477-492, as the lane runs it
on (lo, n = high - low + 1): a 1 bit keeps the upper n - (n >> 1) values, a 0 bit the
lower n >> 1, while n > error_limit + 1).

The closed form: with B_i the first i step bits (LSB first), n_i = (n + B_i) >> i, the
low end moves by (n + B_i) >> (i + 1) at each 1 bit, and the step count k is the first i
with n_i <= E -- i1 (the first i with n >> i <= E, from the bit lengths) or i1 + 1."""
import random

M32 = 0xFFFFFFFF


def _clz(v):
    return 32 - v.bit_length()


def step_loop(x, low, mc, el):
    e = el + 1
    lo, n, k = low, mc + 1, 0
    act = el != 0 and n > e
    while act:
        h = n >> 1
        if (x >> k) & 1:
            lo += h
            n -= h
        else:
            n = h
        k += 1
        act = n > e
    return lo, n, k


def closed_form(x, low, mc, el):
    e = el + 1
    n0 = mc + 1
    act = el != 0 and n0 > e
    d = _clz(e) - _clz(n0 | 1) if act else 0
    i1 = d + (1 if (n0 >> d) > e else 0)
    t1 = (n0 + (x & ((1 << i1) - 1))) >> i1
    k = i1 + (1 if t1 > e else 0) if act else 0
    xk = x & ((1 << k) - 1)
    acc = 0
    j = 0
    while j < k:  # (the kernel: four steps per test of the wave's longest)
        for u in range(4):
            i = min(j + u, 31)
            term = ((n0 + (xk & ((1 << i) - 1))) >> min(i + 1, 31)) & M32
            if (xk >> i) & 1:
                acc += term
        j += 4
    return low + acc, (n0 + xk) >> k, k


def test_closed_form_matches_step_loop():
    rng = random.Random(20261018)
    checked = 0
    for _ in range(200000):
        mc = rng.choice([rng.randint(0, 64), rng.randint(0, 1 << 16), rng.randint(0, (1 << 31) - 2)])
        el = rng.choice([1, 2, rng.randint(1, 255), rng.randint(1, 1 << 20), rng.randint(1, (1 << 31) - 1)])
        x = rng.getrandbits(32)
        low = rng.randint(0, 1 << 20)
        ref = step_loop(x, low, mc, el)
        assert ref[2] <= 31  # (n < 2^31: at most 31 steps)
        assert closed_form(x, low, mc, el) == ref, (x, low, mc, el)
        checked += 1
    assert checked == 200000


def test_no_steps_when_within_the_limit():
    for mc in range(0, 40):
        for el in range(1, 45):
            for x in (0, M32, 0x55555555):
                assert closed_form(x, 7, mc, el) == step_loop(x, 7, mc, el)
