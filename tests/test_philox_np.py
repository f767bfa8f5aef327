"""CPU: the tests' vectorised Philox4x32-10 and DD_ACT_PHILOX action stream
(golden_data) against the C oracle's generator, element by element."""
import numpy as np

import golden_data as gd
from oracle import oracle as ora


def test_philox_np_matches_oracle():
    rng = np.random.default_rng(0)
    c = rng.integers(0, 2**32, (4, 64), dtype=np.uint64).astype(np.uint32)
    k = rng.integers(0, 2**32, (2, 64), dtype=np.uint64).astype(np.uint32)
    v = gd.philox4x32_10_np(*c, *k)
    for i in range(64):
        assert list(ora.philox4x32_10(c[:, i], k[:, i])) == [int(x[i]) for x in v]


def test_philox_actions_np_matches_per_element_draws():
    seed, env0, n, step0, k = 2**40 + 77, 2**33 - 5, 12, 58, 45  # crosses two 32-step blocks
    got = gd.philox_actions_np(seed, env0, n, step0, k)
    key = [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]
    for t in range(k):
        s = step0 + t
        b = s >> 5
        for i in range(n):
            e = env0 + i
            word = ora.philox4x32_10([e & 0xFFFFFFFF, e >> 32, b & 0xFFFFFFFF, (b >> 32) ^ 0xA5A5A5A5], key)
            assert got[t, i] == (int(word[(s >> 3) & 3]) >> (4 * (s & 7))) & 7
    assert len(np.unique(got)) == 8
