"""The binade-run summation behind k_xrefine, restated in numpy float32 and checked
on the CPU against the sequential float sum it must reproduce (computeMeanAndCovarianceMatrix's
accu[k] += v, PCL order).  This pins the algorithm, not the kernel: the kernel's own bit-exactness is
tests/test_xrefine_gpu.py.  A lane segment's run is taken only when its estimated partial-sum range
stays inside one binade; its result R u is added only after the exact range test on the chain value
before it; anything else is added element by element.  A failed range test is counted (the kernel
hands such a frame back to the serial chain) and must not change the result here either."""
import numpy as np
import pytest

F32 = np.float32
SEG = 32          # points per lane segment
LANES = 256       # lane segments per iteration (4 waves x 64 lanes)


def _runs_sum(v, margin=2.0 ** -14):
    """v: float32 stream (0 where a point is not an inlier, which adds exactly nothing).  Returns the
    float32 chain value and the number of failed range tests."""
    s = F32(0.0)
    fails = 0
    step = SEG * LANES
    for it0 in range(0, len(v), step):
        blk = v[it0:it0 + step]
        nl = -(-len(blk) // SEG)
        V = np.zeros(nl * SEG, F32)
        V[:len(blk)] = blk
        V = V.reshape(nl, SEG)
        sv = np.add.reduce(V, axis=1, dtype=F32)                 # phase 1: lane sums (estimates)
        sa = np.add.reduce(np.abs(V), axis=1, dtype=F32)
        P = float(s) + np.concatenate([[0.0], np.cumsum(sv.astype(np.float64))[:-1]])
        mg = (abs(float(s)) + float(np.sum(sa, dtype=np.float64))) * margin
        for l in range(nl):
            lo = P[l] + 0.5 * (float(sv[l]) - float(sa[l])) - mg
            hi = P[l] + 0.5 * (float(sv[l]) + float(sa[l])) + mg
            run = None
            if (lo > 0 or hi < 0) and np.isfinite(lo) and np.isfinite(hi):
                up = lo > 0
                a, b = (lo, hi) if up else (-hi, -lo)
                e = int(np.frexp(a)[1]) - 1
                if -100 <= e <= 125 and b < 2.0 ** (e + 1):
                    scale = F32(2.0 ** (23 - e))
                    t = V[l] * scale                                 # exact: a power-of-two scale
                    q = np.rint(t)
                    R = np.add.accumulate(q, dtype=F32)
                    mn, mx = min(0.0, float(R.min())), max(0.0, float(R.max()))
                    if np.max(np.abs(t - q)) < 0.5 and abs(mn) <= 2 ** 25 and abs(mx) <= 2 ** 25:
                        lim = ((2 ** 23 + 1, 2 ** 24 - 1) if up else (-(2 ** 24 - 1), -(2 ** 23 + 1)))
                        run = (F32(np.ldexp(np.float64(R[-1]), e - 23)), e, lim[0] - int(mn), lim[1] - int(mx))
            if run is None:
                for x in V[l]:
                    s = F32(s + x)
                continue
            a_run, e, L, H = run
            ts = float(F32(s * F32(2.0 ** (23 - e))))
            if abs(ts) < 2 ** 26 and L <= int(ts) <= H:
                s = F32(s + a_run)                                   # exact: the result is a float
            else:
                fails += 1
                for x in V[l]:
                    s = F32(s + x)
    return s, fails


def _streams(rng, n):
    i = np.arange(n, dtype=np.float64)
    out = {
        "zero_crossing": ((-1.0) ** i) * (0.25 + 0.5 * rng.random(n)),
        "dyadic": rng.integers(-512, 513, n) / 256.0,
        "dyadic_products": (rng.integers(-512, 513, n) / 64.0) * (rng.integers(-64, 65, n) / 16.0),
        "powers_of_two": 1.0 + (i % 7) * 2.0 ** -20,
        "far": 1000.0 + rng.random(n),
        "far_products": (1000.0 + rng.random(n)) * (-2000.0 + rng.random(n)),
        "small": (rng.random(n) - 0.3) * 1e-15,
        "denormal_products": ((rng.random(n) - 0.3) * 1e-19) ** 2,
        "rows": np.tile(np.linspace(-0.4, 0.45, 640), n // 640 + 1)[:n],
        "sparse_inliers": np.where(rng.random(n) < 0.3, rng.normal(0.5, 0.2, n), 0.0),
    }
    return {k: v.astype(F32) for k, v in out.items()}


@pytest.mark.parametrize("seed", [1, 2])
def test_runs_reproduce_the_sequential_float_sum(seed):
    rng = np.random.default_rng(seed)
    for name, v in _streams(rng, 60000).items():
        ref = np.add.accumulate(v, dtype=F32)[-1]
        got, fails = _runs_sum(v)
        assert got.tobytes() == F32(ref).tobytes(), (name, got, ref)
        assert fails == 0, name


def test_failed_range_test_is_caught():
    """A deliberately wrong estimate (no margin and a shifted start) makes some runs fail their exact
    range test; the result is still the sequential sum, through the element-by-element path."""
    rng = np.random.default_rng(3)
    v = (1.0 + rng.random(40000) * 1e-3).astype(F32)    # the sum crosses 2^12, 2^13, 2^14, 2^15
    ref = np.add.accumulate(v, dtype=F32)[-1]
    got, fails = _runs_sum(v, margin=-2.0 ** -6)         # a negative margin: ranges underestimated
    assert got.tobytes() == F32(ref).tobytes()
    assert fails > 0
