"""Dev tool: fit atan(x) = x + x·z·R(z), z = x², |x| ≤ tan(π/8), as a polynomial R of degree D in
z (least squares on Chebyshev nodes at 60-digit precision), then measure the error of the double
evaluation (Horner) against mpmath. Output: coefficients for geom.hpp's atan2_fast."""
import mpmath as mp
import numpy as np

mp.mp.dps = 60
T8 = mp.tan(mp.pi / 8)
ZMAX = T8 ** 2


def g(z):
    x = mp.sqrt(z)
    return (mp.atan(x) / x - 1) / z if z != 0 else mp.mpf(-1) / 3


def fit(D, npts=400):
    # weighted LS: minimise relative error of the correction term (x·z·R(z))
    nodes = [ZMAX * (1 - mp.cos(mp.pi * (k + 0.5) / npts)) / 2 for k in range(npts)]
    A = mp.matrix(npts, D + 1)
    b = mp.matrix(npts, 1)
    for i, z in enumerate(nodes):
        for j in range(D + 1):
            A[i, j] = z ** j
        b[i] = g(z)
    coef = mp.lu_solve(A.T * A, A.T * b)
    return [coef[j] for j in range(D + 1)]


def atan_d(x, c):
    z = x * x
    r = c[-1]
    for cc in reversed(c[:-1]):
        r = r * z + cc
    return x + x * z * r


for D in (9, 10, 11, 12):
    c = fit(D)
    cd = [float(v) for v in c]
    xs = np.concatenate([np.linspace(0, float(T8), 20001), np.random.default_rng(0).uniform(0, float(T8), 20000)])
    err = 0.0
    for x in xs[::7]:
        y = atan_d(float(x), cd)
        e = abs(mp.mpf(y) - mp.atan(mp.mpf(float(x))))
        ulp = np.spacing(abs(y)) if y != 0 else 5e-324
        err = max(err, float(e) / ulp)
    print(f"D={D}: max error {err:.3f} ulp")
    if D == 11:
        print("coefficients (z^0 .. z^D):")
        for v in cd:
            print(f"  {v!r},")
