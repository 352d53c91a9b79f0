"""Oracle: Chebyshev pseudospectral (CGL) constants -- TEST INFRASTRUCTURE ONLY.

Restates ``ChebyshevPseudospectralMethod`` of the reference
(``/root/reference/nlp/collocation.py``) in plain NumPy, operation-for-operation
where bit-exactness is claimed:

* ``nodes``            -> ``buildNodes``              collocation.py:34-40
* ``diff_matrix``      -> ``buildDiffMatrix``         collocation.py:42-64 (negated CGL matrix)
* ``quad_weights``     -> ``buildQuadratureWeights``  collocation.py:66-85, *bug-compatible*:
                          Python-2 integer division at :78/:80 and the two
                          statements of :82-83 repeated inside the inner ``j`` loop.
* ``lagrange_poly1d``  -> ``buildLagrangePolynomials`` + ``evaluateLagrangePolynomials``
                          collocation.py:87-111 (monomial poly1d products; only
                          numerically meaningful for N <= 20)
* ``lagrange_bary``    -> the same Lagrange basis evaluated with the barycentric
                          formula (exact-node shortcut) -- what the product uses.
* ``tau2t`` / ``t2tau`` -> collocation.py:26-32 (t2tau assumes t0 = 0, as the
                          reference does; the estimator always builds with t0=0,
                          nlp/nlp.py:197).
"""
import numpy as np


def nodes(N):
    """CGL nodes on [-1, 1], ascending (collocation.py:34-40)."""
    tau = np.zeros(N + 1)
    for k in range(N + 1):
        tau[k] = np.cos(k * np.pi / N)
    return tau[::-1].copy()


def diff_matrix(N, tau=None):
    """Negated Trefethen CGL differentiation matrix (collocation.py:42-64).

    Same scalar op order as the reference so the result is bit-identical.
    """
    if tau is None:
        tau = nodes(N)
    x = tau[::-1]  # back to [1, -1] ordering (collocation.py:47)
    D = np.zeros((N + 1, N + 1))
    for k in range(N + 1):
        c = np.ones(N + 1)
        c[0] = 2
        c[N] = 2
        for j in range(N + 1):
            if k == 0 and j == 0:
                D[k, j] = (2 * N ** 2 + 1) / 6.0
            elif k == N and j == N:
                D[k, j] = -(2 * N ** 2 + 1) / 6.0
            elif k == j:
                D[k, j] = -x[k] / (2 * (1 - x[k] ** 2))
            else:
                D[k, j] = (c[k] / c[j]) * (np.power(-1, j + k) / (x[k] - x[j]))
    return -D


def quad_weights(N):
    """Bug-compatible 'Clenshaw-Curtis' weights (collocation.py:66-85).

    Python-2 semantics: ``(N-a)/2`` is floor division; the two ``w[s] +=`` /
    ``w[N-s] = w[s]`` statements sit inside the inner loop (collocation.py:82-83),
    so when that loop is empty (N in {2, 3}) ``w[N-s]`` is never assigned.
    """
    w = np.zeros(N + 1)
    if N % 2 == 0:
        w[0] = 1.0 / (N ** 2 - 1)
        w[N] = w[0]
        a = 0
    else:
        w[0] = 1.0 / N ** 2
        w[N] = w[0]
        a = 1
    for s in range(1, (N - a) // 2 + 1):
        w[s] = 2.0 / N
        for j in range(1, (N - a) // 2):
            w[s] += (4.0 / N) * (1.0 / (1.0 - 4.0 * j ** 2)) * np.cos(2 * np.pi * j * s / N)
            w[s] += (2.0 / N) * (1.0 / (1 - (N - a) ** 2)) * np.cos((N - a) * s * np.pi / N)
            w[N - s] = w[s]
    return w


def tau2t(tau, t0, tf):
    """collocation.py:26-28"""
    return 0.5 * ((tf - t0) * tau + (tf + t0))


def t2tau(t, t0, tf):
    """collocation.py:30-32 (reference formula; exact only for t0 = 0)."""
    return (2.0 * t - (tf - t0)) / (tf - t0)


def lagrange_poly1d(N, tau_eval):
    """phi_j(tau) for all j via the reference's poly1d products (collocation.py:87-111)."""
    tau = nodes(N)
    polys = []
    for j in range(N + 1):
        p = np.poly1d([1])
        for k in range(N + 1):
            if k != j:
                p *= (1 / (tau[j] - tau[k])) * np.poly1d([1, -tau[k]])
        polys.append(p)
    tau_eval = np.atleast_1d(np.asarray(tau_eval, dtype=np.float64))
    out = np.zeros((tau_eval.shape[0], N + 1))
    for i, te in enumerate(tau_eval):
        for j in range(N + 1):
            out[i, j] = polys[j](te)
    return out


def bary_weights(N):
    """Barycentric weights of the CGL nodes (ascending order): (-1)^j, halved at the ends."""
    c = np.array([(-1.0) ** j for j in range(N + 1)])
    c[0] *= 0.5
    c[N] *= 0.5
    return c


def lagrange_bary(N, tau_eval):
    """phi_j(tau) via the barycentric formula, exact at the nodes."""
    tau = nodes(N)
    c = bary_weights(N)
    tau_eval = np.atleast_1d(np.asarray(tau_eval, dtype=np.float64))
    out = np.zeros((tau_eval.shape[0], N + 1))
    for i, te in enumerate(tau_eval):
        diff = te - tau
        hit = np.nonzero(diff == 0.0)[0]
        if hit.size:
            out[i, hit[0]] = 1.0
            continue
        q = c / diff
        out[i] = q / q.sum()
    return out


def interp_matrix(N, T, t_eval, mode="bary"):
    """Phi (len(t), N+1): rows phi(t2tau(t)) for a window [0, T] (nlp/nlp.py:264-269)."""
    tau_eval = t2tau(np.asarray(t_eval, dtype=np.float64).reshape(-1), 0.0, T)
    if mode == "poly1d":
        return lagrange_poly1d(N, tau_eval)
    return lagrange_bary(N, tau_eval)
