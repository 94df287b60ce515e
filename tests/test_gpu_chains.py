"""Deferred statistics chains (P^2 median + immediate variance over a group's best-function
lengths in visit order) through both device chain codes -- one lane per chain (k_chains) and one
wave pair per chain (k_chain_long, ballot cells + scalar walk) -- against the pure-Python
restatement of Boost.Accumulators (tests/pyref.py), raw doubles bit for bit."""
import numpy as np
import pytest

import pyref

pytestmark = pytest.mark.gpu


def ref_chain(xs):
    p2 = pyref.P2()
    cnt, s, var = 0, 0, 0.0
    for x in xs:
        x = int(x)
        cnt += 1
        s = (s + x) & 0xFFFF
        p2.add(x)
        if cnt > 1:
            m = s / cnt
            t = x - m
            var = var * (cnt - 1) / cnt + t * t / (cnt - 1)
    return p2.result(), var


def cases():
    rng = np.random.default_rng(2024)
    out = []
    for n in (1, 2, 3, 4, 5, 6, 7, 63, 64, 65, 69, 70, 133, 1000, 4097):
        out.append((f"uniform-{n}", rng.integers(50, 2000, n)))
    out.append(("narrow-20000", rng.integers(240, 361, 20000)))
    out.append(("ties-6000", rng.choice([100, 200, 300], 6000)))
    out.append(("increasing-3000", np.arange(3000) + 100))
    out.append(("decreasing-3000", 5000 - np.arange(3000)))
    out.append(("constant-500", np.full(500, 333)))
    out.append(("big-lengths-2000", rng.integers(60000, 140000, 2000)))
    out.append(("bimodal-12000", np.where(rng.random(12000) < 0.5, rng.integers(100, 120, 12000),
                                          rng.integers(900, 950, 12000))))
    return out


@pytest.mark.parametrize("name,xs", cases(), ids=[c[0] for c in cases()])
@pytest.mark.parametrize("mode", [1, 2])
def test_chain_matches_reference(skm, gpu, name, xs, mode):
    med, var = skm.debug_chain_eval(xs, mode)
    rmed, rvar = ref_chain(xs)
    assert med == rmed or (np.isnan(med) and np.isnan(rmed)), (name, mode, med, rmed)
    assert var == rvar, (name, mode, var, rvar)
