"""Chebyshev pseudospectral (CGL) discretisation -- host-side constants.

API mirror of ``ChebyshevPseudospectralMethod`` (reference ``nlp/collocation.py:7-121``).
These are one-time host constants; the per-iteration work
runs in ``libmhe.so``.  Semantics kept from the reference:

* ``tau``  ascending CGL nodes (collocation.py:34-40)
* ``D``    the Trefethen matrix built on descending nodes and negated
           (collocation.py:42-64), same scalar operation order -> bit-identical
* ``w``    the reference's quadrature weights *including its bugs*
           (Python-2 floor division at :78/:80, loop-body placement of :82-83) --
           they are inside the objective, so parity needs them verbatim
* ``phi``  Lagrange basis.  The reference multiplies monomial ``poly1d`` factors,
           which loses all accuracy for N >= 30.  The default
           here is the barycentric form of the *same* basis (exact at the nodes);
           ``phi_mode="poly1d"`` reproduces the reference numerics for small N.
"""
import numpy as np


def cgl_nodes(N):
    k = np.arange(N + 1, dtype=np.float64)
    tau = np.cos(k * np.pi / N)
    return tau[::-1].copy()


def cgl_diff_matrix(N, tau):
    x = tau[::-1]
    P = N + 1
    c = np.ones(P)
    c[0] = 2.0
    c[N] = 2.0
    k = np.arange(P)[:, None]
    j = np.arange(P)[None, :]
    sign = np.where((j + k) % 2 == 0, 1.0, -1.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        D = (c[:, None] / c[None, :]) * (sign / (x[:, None] - x[None, :]))
        diag = -x / (2 * (1 - x ** 2))
    D[np.arange(P), np.arange(P)] = diag
    D[0, 0] = (2 * N ** 2 + 1) / 6.0
    D[N, N] = -(2 * N ** 2 + 1) / 6.0
    return -D


def quadrature_weights(N):
    """Bug-compatible weights (see module docstring); scalar loop keeps the op order."""
    w = np.zeros(N + 1)
    if N % 2 == 0:
        w[0] = 1.0 / (N ** 2 - 1)
        a = 0
    else:
        w[0] = 1.0 / N ** 2
        a = 1
    w[N] = w[0]
    half = (N - a) // 2
    for s in range(1, half + 1):
        w[s] = 2.0 / N
        for j in range(1, half):
            w[s] += (4.0 / N) * (1.0 / (1.0 - 4.0 * j ** 2)) * np.cos(2 * np.pi * j * s / N)
            w[s] += (2.0 / N) * (1.0 / (1 - (N - a) ** 2)) * np.cos((N - a) * s * np.pi / N)
            w[N - s] = w[s]
    return w


class ChebyshevPseudospectralMethod:
    def __init__(self, N, t0, tf, phi_mode="bary"):
        if N < 1:
            raise ValueError("N must be >= 1")
        self.N = N
        self.t0 = t0
        self.tf = tf
        self.phi_mode = phi_mode
        self.tau = cgl_nodes(N)
        self.D = cgl_diff_matrix(N, self.tau)
        self.w = quadrature_weights(N)
        c = np.where(np.arange(N + 1) % 2 == 0, 1.0, -1.0)
        c[0] *= 0.5
        c[N] *= 0.5
        self.bary = c
        self._poly = None

    def tau2t(self, tau):
        """collocation.py:26-28"""
        return 0.5 * ((self.tf - self.t0) * tau + (self.tf + self.t0))

    def t2tau(self, t):
        """collocation.py:30-32 (the reference formula; exact for t0 = 0)."""
        return (2.0 * t - (self.tf - self.t0)) / (self.tf - self.t0)

    def _poly1d(self):
        if self._poly is None:
            polys = []
            for j in range(self.N + 1):
                p = np.poly1d([1])
                for k in range(self.N + 1):
                    if k != j:
                        p *= (1 / (self.tau[j] - self.tau[k])) * np.poly1d([1, -self.tau[k]])
                polys.append(p)
            self._poly = polys
        return self._poly

    def lagrange_matrix(self, t_array):
        """Phi (len(t), N+1) with Phi[i, j] = phi_j(t2tau(t_i))."""
        ts = np.asarray(t_array, dtype=np.float64).reshape(-1)
        taus = self.t2tau(ts)
        out = np.zeros((taus.shape[0], self.N + 1))
        if self.phi_mode == "poly1d":
            polys = self._poly1d()
            for i, te in enumerate(taus):
                for j in range(self.N + 1):
                    out[i, j] = polys[j](te)
            return out
        for i, te in enumerate(taus):
            diff = te - self.tau
            hit = np.nonzero(diff == 0.0)[0]
            if hit.size:
                out[i, hit[0]] = 1.0
                continue
            q = self.bary / diff
            out[i] = q / q.sum()
        return out

    def evaluateLagrangePolynomials(self, t):
        """collocation.py:98-107"""
        return self.lagrange_matrix([t])[0]

    def evaluateSolution(self, t, X):
        """collocation.py:113-121: x(t) = sum_j X_j phi_j(t)."""
        phi = self.evaluateLagrangePolynomials(t)
        return np.tensordot(phi, np.asarray(X, dtype=np.float64), axes=(0, 0))
