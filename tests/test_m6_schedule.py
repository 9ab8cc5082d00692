"""Host mirror of the M6 tile schedule (pptk_amd/csrc/rx_kernel.hip
m_schedule / m_rounds): every listed frame gets exactly
one (round, team) slot, no slot lies past the LDS list (M_RMAX rows of 16),
and the padded round count covers the schedule.  The device code itself is
checked by the -m gpu parity tests (tests/test_gpu_parity.py, variant M6)."""
import itertools
import re

import numpy as np

SRC = "pptk_amd/csrc/rx_kernel.hip"


def constants():
    import os
    src = open(os.path.join(os.path.dirname(os.path.dirname(__file__)), SRC)).read()
    m_s = int(re.search(r"constexpr int M_S = (\d+);", src).group(1))
    rmax = int(re.search(r"constexpr int M_RMAX = (\d+);", src).group(1))
    m_d = int(re.search(r"#define PPTK_RX_M_D (\d+)", src).group(1))
    return m_s, rmax, m_d


def schedule(nch, valid, m_d):
    """(slots {lane: (round, team)}, e2, P) as m_schedule / m_rounds build them."""
    cls = np.where(nch <= 24, 0, np.where(nch <= 48, 1, 2))
    n = [int(((cls == c) & valid).sum()) for c in range(3)]
    e0 = (n[0] + 15) >> 4
    e1 = e0 + ((n[1] + 7) >> 3)
    e2 = e1 + ((n[2] + 3) >> 2)
    first_row = [0, e0, e1]
    slots = {}
    rank = [0, 0, 0]
    for lane in range(64):
        if not valid[lane]:
            continue
        c = int(cls[lane])
        rho = rank[c]
        rank[c] += 1
        sh = 4 - c
        slots[lane] = (first_row[c] + (rho >> sh), rho & ((1 << sh) - 1), c)
    g = m_d + 1
    p = 2 * g if e2 <= 2 * g else (e2 + g - 1) // g * g
    return slots, e2, p


def check(nch, valid):
    m_s, rmax, m_d = constants()
    slots, e2, p = schedule(nch, valid, m_d)
    assert len(set((r, t) for r, t, _ in slots.values())) == len(slots)   # one frame per slot
    for lane, (r, t, c) in slots.items():
        assert r < e2 <= p and p < rmax
        assert t < (16 >> c)                       # a team of the round's width
        assert (nch[lane] <= 24) == (c == 0)       # the class's team holds the frame
        assert nch[lane] <= (6 * (4 << c) if c < 2 else 10 ** 9)
    assert p % (m_d + 1) == 0 and p >= 2 * (m_d + 1)


def test_worst_case_class_mixes():
    """Every split of 64 frames into the three classes (and partial tiles)."""
    for n0, n1 in itertools.product(range(65), repeat=2):
        if n0 + n1 > 64:
            continue
        nch = np.array([2] * n0 + [30] * n1 + [90] * (64 - n0 - n1))
        for valid_n in (64, 37, 1):
            check(nch, np.arange(64) < valid_n)


def test_random_tiles():
    rng = np.random.default_rng(7)
    for _ in range(2000):
        lens = rng.integers(0, 1600, 64)
        m = rng.integers(0, 16, 64)
        nch = (m + lens + 15) >> 4
        check(nch, rng.random(64) < 0.97)
