"""CPU oracle of the SHEncoder direction encoding (reference external/sh_encoder.py:15-193) --
TEST INFRASTRUCTURE: imported by tests/ only, never by the product path.

Restated from the definition of the real spherical harmonics rather than the reference's 64
written-out polynomials: for band l and order m,

    Y_l^0 = K_l^0 Q_l^0(z),   Y_l^{+m} = s_m K_l^m Q_l^m(z) Re (x + i y)^m,
    Y_l^{-m} = s_m K_l^m Q_l^m(z) Im (x + i y)^m,   s_m = sqrt(2) (-1)^m,

with K_l^m = sqrt((2l+1)/(4 pi) (l-m)!/(l+m)!) and Q_l^m = d^m P_l / dz^m (the Legendre polynomial's
m-th derivative: the associated Legendre function without its (1-z^2)^{m/2} factor and phase), in
float64 with numpy.polynomial.  Column l^2 + l + m, as tcnn's spherical_harmonics.h and the
reference order them.  The gradient is analytic: d/dz through Q_l^{m+1}, d/dx and d/dy through
m (x + i y)^{m-1} and i m (x + i y)^{m-1}.

Pinned by tests/golden/sh_encoder.npz (the reference module's outputs and autograd gradients,
tests/golden/make_golden.py gen_sh).
"""
import math

import numpy as np
from numpy.polynomial import legendre as npleg


def _k(l, m):
    return math.sqrt((2 * l + 1) / (4 * math.pi) * math.factorial(l - m) / math.factorial(l + m))


def _q(l, m):
    """Power-series coefficients of d^m P_l / dz^m."""
    c = np.zeros(l + 1)
    c[l] = 1.0
    return npleg.leg2poly(npleg.legder(c, m)) if m <= l else np.zeros(1)


def _terms(coords, degree):
    x, y, z = (np.asarray(coords, dtype=np.float64)[:, i] for i in range(3))
    w = x + 1j * y
    for l in range(degree):
        for m in range(l + 1):
            s = 1.0 if m == 0 else math.sqrt(2.0) * (-1.0) ** m
            yield l, m, s * _k(l, m), x, y, z, w


def sh_encode(coords, degree):
    """(n,3) -> (n, degree^2) float64."""
    n = np.asarray(coords).shape[0]
    out = np.zeros((n, degree * degree))
    for l, m, c, x, y, z, w in _terms(coords, degree):
        q = np.polynomial.polynomial.polyval(z, _q(l, m))
        wm = w ** m
        if m == 0:
            out[:, l * l + l] = c * q
        else:
            out[:, l * l + l + m] = c * q * wm.real
            out[:, l * l + l - m] = c * q * wm.imag
    return out


def sh_encode_grad(coords, degree, d_out):
    """d/d coords of sum(d_out * sh_encode(coords, degree)) -> (n,3) float64."""
    n = np.asarray(coords).shape[0]
    d_out = np.asarray(d_out, dtype=np.float64)
    g = np.zeros((n, 3))
    poly = np.polynomial.polynomial
    for l, m, c, x, y, z, w in _terms(coords, degree):
        q = poly.polyval(z, _q(l, m))
        dq = poly.polyval(z, poly.polyder(_q(l, m))) if l > 0 else np.zeros_like(z)
        wm = w ** m
        dwm = m * w ** (m - 1) if m > 0 else np.zeros_like(w)  # d/dx; d/dy = i * d/dx
        parts = [(l * l + l, 1.0, 0.0)] if m == 0 else [(l * l + l + m, 1.0, 0.0), (l * l + l - m, 0.0, 1.0)]
        for col, re, im in parts:
            pick = (lambda v: v.real) if re else (lambda v: v.imag)
            go = d_out[:, col] * c
            g[:, 0] += go * q * pick(dwm)
            g[:, 1] += go * q * pick(1j * dwm)
            g[:, 2] += go * dq * pick(wm)
    return g
