"""R default RNG emulator -- TEST INFRASTRUCTURE ONLY (fixture generation).

Emulates R >= 3.6's default generators so the vignette's toy inputs
(`Vignette.rmd:26-48`) can be regenerated offline and pinned against the
values printed in `Vignette.md:136-142,180-186`:

* ``set.seed(s)``: initial scrambling ``seed = 69069*seed + 1`` x50, then
  625 more draws fill ``i_seed``; ``mti = 624`` (R's RNG.c, Mersenne-Twister).
* ``unif_rand``: MT19937 tempering, ``* 2.3283064365386963e-10``, clamped
  into (0, 1) (R's ``fixup``).
* ``norm_rand`` (INVERSION): ``u = unif; u = floor(2^27 u) + unif;
  qnorm(u / 2^27)``.

Nothing here is used by the product path.
"""
from __future__ import annotations

import numpy as np
from scipy.special import ndtri

_N = 624
_M = 397


class RRNG:
    def __init__(self, seed: int):
        self.set_seed(seed)

    def set_seed(self, seed: int) -> None:
        s = seed & 0xFFFFFFFF
        for _ in range(50):
            s = (69069 * s + 1) & 0xFFFFFFFF
        iseed = []
        for _ in range(_N + 1):
            s = (69069 * s + 1) & 0xFFFFFFFF
            iseed.append(s)
        self.mt = iseed[1:]
        self.mti = _N

    def _genrand(self) -> float:
        mt = self.mt
        if self.mti >= _N:
            mag01 = (0, 0x9908B0DF)
            for kk in range(_N - _M):
                y = (mt[kk] & 0x80000000) | (mt[kk + 1] & 0x7FFFFFFF)
                mt[kk] = mt[kk + _M] ^ (y >> 1) ^ mag01[y & 1]
            for kk in range(_N - _M, _N - 1):
                y = (mt[kk] & 0x80000000) | (mt[kk + 1] & 0x7FFFFFFF)
                mt[kk] = mt[kk + (_M - _N)] ^ (y >> 1) ^ mag01[y & 1]
            y = (mt[_N - 1] & 0x80000000) | (mt[0] & 0x7FFFFFFF)
            mt[_N - 1] = mt[_M - 1] ^ (y >> 1) ^ mag01[y & 1]
            self.mti = 0
        y = mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y * 2.3283064365386963e-10

    def unif_rand(self) -> float:
        v = self._genrand()
        i2_32m1 = 2.328306437080797e-10
        if v <= 0.0:
            return 0.5 * i2_32m1
        if 1.0 - v <= 0.0:
            return 1.0 - 0.5 * i2_32m1
        return v

    def runif(self, n: int, a: float = 0.0, b: float = 1.0) -> np.ndarray:
        return np.array([a + (b - a) * self.unif_rand() for _ in range(n)])

    def norm_rand(self) -> float:
        big = 134217728.0
        u = self.unif_rand()
        u = int(big * u) + self.unif_rand()
        return float(ndtri(u / big))

    def rnorm(self, n: int, mean: float = 0.0, sd: float = 1.0) -> np.ndarray:
        return np.array([mean + sd * self.norm_rand() for _ in range(n)])


def vignette_toy():
    """Regenerate the vignette toy example (Vignette.rmd:26-48).

    Returns dict(locs (2000x2), field, X (2000x2), beta, beta_0, noise,
    observed_field).  GpGp::exponential_isotropic(c(1,5,0), locs) is
    exp(-d/5); chol is LAPACK's (numpy) -- same factor as R's chol().
    """
    rng = RRNG(1)
    x = 500.0 * rng.runif(2000)
    locs = np.column_stack([x, np.ones(2000)])
    locs[0, 1] = 1.01
    d = np.sqrt(((locs[:, None, :] - locs[None, :, :]) ** 2).sum(-1))
    C = np.exp(-d / 5.0)
    L = np.linalg.cholesky(C)
    z = rng.rnorm(2000)
    field = np.sqrt(10.0) * (L @ z)
    X = np.column_stack([locs[:, 0], rng.rnorm(2000)])
    beta = np.array([0.01, rng.rnorm(1)[0]])
    beta_0 = rng.rnorm(1)[0]
    noise = np.sqrt(5.0) * rng.rnorm(2000)
    observed_field = field + noise + X @ beta + beta_0
    return dict(locs=locs, field=field, X=X, beta=beta, beta_0=beta_0,
                noise=noise, observed_field=observed_field)
