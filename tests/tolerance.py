"""Parity tolerances derived from the problem.

Two correct fp64 evaluations of the same Gauss-Newton iteration differ for two reasons:

 (1) rounding of the residual y - h(x).  Pseudoranges (|y| ~ 2.2e7 m) carry eps |y|
     ~ 5e-9 m of rounding in ANY evaluation order (h is a sqrt of squares of ~2e7 m
     differences).  Its effect on the result is MEASURED, not assumed: the oracle is
     re-run with every y moved by eps |y| (random sign) and the largest change of
     the result is the floor.
 (2) summation order in the normal equations and the factorisation: relative,
     REL (1 + max|X|) for iterates, SURVEY.md §8(c) (1e-10).

    bound = FLOOR_MULT * floor + REL * (1 + max|X|)

For a pseudorange problem the floor is ~1e-8 m, so the bound is ~1e-6 m and a
1e-4 m error fails (the round-2 bound 1e-9 kappa (1 + max|X|) let ~2 m through).
Every test prints the observed error beside its bound.
"""
import numpy as np

FLOOR_MULT = 32.0
REL = 1e-10
EPS = np.finfo(np.float64).eps


def perturbed(Y, seed=12345):
    """Y with every entry moved by one eps of its own magnitude, random sign."""
    rng = np.random.default_rng(seed)
    return Y * (1.0 + EPS * rng.choice([-1.0, 1.0], size=np.shape(Y)))


def floor(run, Y, seed=12345):
    """max |run(Y') - run(Y)| over the outputs of ``run`` (a tuple of arrays), Y' =
    perturbed(Y): the change any evaluation order may legitimately produce."""
    a, b = run(Y), run(perturbed(Y, seed))
    return [float(np.abs(np.asarray(x) - np.asarray(y)).max()) for x, y in zip(a, b)]


def bound(fl, X, rel=REL):
    return FLOOR_MULT * fl + rel * (1.0 + float(np.abs(X).max()))


def check(name, err, bnd, unit=""):
    print(f"{name}: max err {err:.3e}{unit}  bound {bnd:.3e}{unit}")
    assert err <= bnd, f"{name}: {err:.3e} > bound {bnd:.3e}"
