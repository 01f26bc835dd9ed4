"""GPU: the device Fiat-Shamir draws (DefaultRandomCoin<Blake3_256>::draw::<E>, winter-crypto 0.8.3)
that the prover runs between its commitments, against a Python model of the coin over the oracle's
BLAKE3 (tests/oracle_lib.py; pinned by the published BLAKE3 vectors).

The prover draws the 15 composition and 8 DEEP coefficients with one wave hashing 64 counters at once
(wave_draw_e) and each FRI alpha one at a time (dev_draw_e). A rejected candidate (an element >= p)
has probability 2^-32, so whole-proof parity never exercises the retry bookkeeping; here extra
rejections are forced on chosen counters (xfg_debug_coin_draws), including windows with fewer
accepted candidates than draws, which sends the wave path to its one-at-a-time fallback."""
import random

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu
P = 0xFFFFFFFF00000001


@pytest.fixture(scope="module")
def prover():
    import xfgstark
    pr = xfgstark.XfgBurnMintProver()
    yield pr
    pr.close()


def model_draws(seed, counter, k, ext, forced):
    """Coin::draw_e k times (host_common.hpp Coin, winter-crypto DefaultRandomCoin): candidate
    BLAKE3(seed || counter_le8), first 8 ext bytes as ext LE u64, all < p, and counter not forced"""
    out = []
    for _ in range(k):
        for _ in range(1000):
            counter += 1
            h = O.blake3(bytes(seed) + counter.to_bytes(8, "little"))
            x = int.from_bytes(h[0:8], "little")
            y = int.from_bytes(h[8:16], "little")
            if counter not in forced and x < P and (ext == 1 or y < P):
                out.append((x, y if ext == 2 else 0))
                break
        else:
            return out, counter, False
    return out, counter, True


def mask(forced):
    m = [0, 0, 0, 0]
    for c in forced:
        assert 1 <= c <= 256
        m[(c - 1) >> 6] |= 1 << ((c - 1) & 63)
    return m


CASES = [
    ("none", lambda r: set()),
    ("scattered", lambda r: set(r.sample(range(1, 257), 20))),
    ("first_in_window", lambda r: {1}),
    # more rejections in the 64-candidate window than draws leave room for: one-at-a-time fallback
    ("window_starved", lambda r: set(range(1, 61))),
    ("window_empty", lambda r: set(range(1, 65))),
    ("long_run", lambda r: set(range(3, 200))),
]


@pytest.mark.parametrize("ext", [1, 2])
@pytest.mark.parametrize("k", [1, 8, 15, 64])
@pytest.mark.parametrize("case", [c[0] for c in CASES])
def test_device_draws_match_coin_model(prover, case, k, ext):
    rng = random.Random(f"{case}-{k}-{ext}")
    forced = dict(CASES)[case](rng)
    seed = bytes(rng.randrange(256) for _ in range(32))
    counter = rng.choice([0, 0, 3])  # a fresh reseed starts at 0; a coin mid-transcript does not
    forced = {c for c in forced if c > counter}
    want, want_ctr, want_ok = model_draws(seed, counter, k, ext, forced)
    wave, seq, ctr, ok = prover.debug_coin_draws(seed, counter, k, ext, mask(forced))
    assert ok == (int(want_ok), int(want_ok))
    assert ctr == (want_ctr, want_ctr)
    exp = np.array(want, dtype=np.uint64).reshape(k, 2)
    assert np.array_equal(seq, exp), "one-at-a-time draws differ from the coin model"
    assert np.array_equal(wave, exp), "one-wave draws differ from the coin model"
