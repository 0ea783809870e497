"""Accuracy of the MH update kernel's table-driven log (mh_kernels.hip log_tab, MH_TLOG), restated in numpy.

x = m 2^e, m in [1, 2); row j = floor(64 (m - 1)) holds (1/c_j rounded, -log of it), c_j = 1 + (j + 1/2) / 64;
r = m (1/c_j) - 1 (one fma), log(1 + r) by its degree-8 Taylor polynomial.  The fma steps are emulated in
long double.  Prints the largest absolute error in ulps of max(|log x|, 1) (what a sum of 54 frame terms
sees) and the largest relative error where |log x| > 0.1.

  python scripts/check_log_table.py
"""
import numpy as np

L = np.longdouble


def fma(a, b, c):
    return (L(a) * L(b) + L(c)).astype(np.float64)


def log_tab(x):
    j = np.arange(64)
    inv = 1.0 / (1.0 + (j + 0.5) / 64)
    logc = -np.log(inv)
    m, e = np.frexp(x)
    m, e = m * 2.0, e - 1
    jj = ((m - 1.0) * 64.0).astype(int)
    r = fma(m, inv[jj], -1.0)
    p = np.full_like(r, -0.125)
    for c in (1.4285714285714285e-01, -1.6666666666666666e-01, 0.2, -0.25, 3.3333333333333333e-01, -0.5):
        p = fma(p, r, c)
    l1p = fma(p * r, r, r)
    return fma(e, 6.93147180369123816490e-01, fma(e, 1.90821492927058770002e-10, logc[jj] + l1p))


def main():
    rng = np.random.default_rng(0)
    x = np.concatenate([np.exp(rng.uniform(-30, 30, 200000)), rng.uniform(0.5, 2, 100000),
                        1 + rng.uniform(-1e-6, 1e-6, 10000)])
    got, ref = log_tab(x), np.log(L(x))
    err = np.abs(L(got) - ref).astype(np.float64)
    absu = float((err / np.spacing(np.maximum(np.abs(ref.astype(np.float64)), 1.0))).max())
    big = np.abs(ref) > 0.1
    relu = float((err[big] / np.spacing(np.abs(ref[big].astype(np.float64)))).max())
    print(f'{x.size} points: max abs error {absu:.3f} ulp of max(|log x|, 1); max rel error {relu:.2f} ulp where |log x| > 0.1')
    assert absu < 1.0


if __name__ == '__main__':
    main()
