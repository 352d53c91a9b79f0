"""Estimation-NLP builder and solve facade -- drop-in for kingdwd/nlp-filter nlp/nlp.py.

The reference records a CasADi ``Opti`` problem and hands it to IPOPT
(nlp/nlp.py:61-83).  Here the same calls record a *problem spec*; ``build()``
turns it into device constants (libmhe.so, ``mhe_build_constants``) and
``solve()`` runs the batched Gauss-Newton kernel (``mhe_gn_solve``) on the
GPU.  The process-noise variables ``W`` of ``addDynamics`` are eliminated
through the collocation equality W_k = (2/T) sum_j D_kj X_j - f(X_k, U_k)
(nlp/nlp.py:235) -- the unconstrained least-squares problem has the same
stationary point IPOPT converges to -- and stay extractable by name.

Kept semantics
  * ``addVariables`` / ``addParameter`` return lists of handles; parameters
    (controls, measurements, sat positions, weights) can be set later with
    ``setParameter`` / ``setControl`` / ``setMeasurement`` (nlp/nlp.py:38-56,304-312)
  * ``R`` passed to ``addResidualCost`` is the *information* matrix
    (the reference adds r^T R r, nlp/nlp.py:273)
  * ``solve(warmstart=True)`` starts from the previous solution (nlp/nlp.py:77-79);
    ``self.solver`` holds IPOPT-style stats incl. ``t_wall_total`` (nlp/nlp.py:83)
  * ``extractVariableValue`` / ``extractSolution`` print and return None on a
    missing name or before ``solve()`` (nlp/nlp.py:85-119)

  * ``pseudo_huber_loss`` dynamics cost (cost_functions.py:25-31) -> IRLS on the GPU
  * ``addVarBounds`` on the state trajectory -> projected Newton on the GN model
    (epsilon-active set, reduced step, Armijo search along the projection arc: the
    solution is a KKT point); bounds on other variables are checked after the solve
    (``self.solver["bounds_violated"]``)
  * several measurement plug-ins in one problem (one ``addResidualCost`` call
    each, gnss-multi-receiver.py:70-140), extra decision variables used inside
    measurement params (``{"y": XA}``, multi-receiver.py:73,99) and
    ``addEqConstraint(constraints.equality_constaint, [X[i][a], X[j][b]])``
    (gnss-multi-receiver.py:76-78): encoded as MHE_MEAS_MIXED rows, extra
    variables and constraint pairs (include/mhe.h) and solved with a bordered
    (KKT) Gauss-Newton step on the large-system path -- the constraints hold after
    every step.  Mixed rows carry scalar weights, so a full_state term in a mixed
    problem needs a diagonal R.

Inequality constraints (``addIneqConstraint``) and state bounds together with
constraint rows are held by an active set over Gauss-Newton solves
(``_solve_active_set``).  Not on the Gauss-Newton path (raise
``UnsupportedFeature``): constraint plug-ins other than ``equality_constaint``,
constraints on extra variables, and ``fixedTimeOptimalControlNLP`` (out of
scope: the north star is the estimator).
"""
import time
import warnings

import numpy as np
from scipy.interpolate import interp1d

from . import collocation


class UnsupportedFeature(NotImplementedError):
    pass


class Var:
    """Decision-variable handle (stands in for ``opti.variable(n)``)."""
    __slots__ = ("name", "idx", "size", "value", "init")

    def __init__(self, name, idx, size):
        self.name, self.idx, self.size = name, idx, size
        self.value = None
        self.init = None

    def __getitem__(self, k):
        """Scalar element ``x[k]`` (CasADi MX indexing), e.g. for addEqConstraint."""
        k = int(k)
        if not -self.size <= k < self.size:
            raise IndexError(f"{self!r}[{k}]")
        return Elem(self, k % self.size)

    def __len__(self):
        return self.size

    def __repr__(self):
        return f"Var({self.name}_{self.idx}, n={self.size})"


class Elem:
    """One scalar of a decision variable (``X[i][k]``)."""
    __slots__ = ("var", "k")

    def __init__(self, var, k):
        self.var, self.k = var, k

    def __repr__(self):
        return f"{self.var!r}[{self.k}]"


class ParameterNotSet(ValueError):
    """A parameter (or measurement slot) was read before setParameter()/setMeasurement()."""


class Param:
    """Parameter handle (stands in for ``opti.parameter(n)``)."""
    __slots__ = ("size", "value")

    def __init__(self, size, value=None):
        self.size = size
        self.value = None if value is None else np.asarray(value, dtype=np.float64).reshape(-1)

    def get(self):
        if self.value is None:
            raise ParameterNotSet("parameter used before setParameter()")
        return self.value


def _resolve(v):
    return v.get() if isinstance(v, Param) else v


def _fname(f):
    return getattr(f, "__name__", str(f))


class NLP(object):
    """Variable / parameter bookkeeping and the solve facade (nlp/nlp.py:8-119)."""

    def __init__(self, N):
        self.N = N
        self.var_names = []
        self.var_sizes = []
        self.w = {}
        self.sol = None
        self.solver = None
        self._bounds = []
        self._eq = []
        self._ineq = []
        self._active = []

    def addVariables(self, N_var, n_var, lb=None, ub=None, name='x'):
        X = []
        for i in range(N_var):
            var_name = name + '_' + str(i)
            self.var_names.append(var_name)
            self.var_sizes.append(n_var)
            x = Var(name, i, n_var)
            self.w[var_name] = x
            X.append(x)
        if lb is not None or ub is not None:
            self._bounds.append((X, None, lb, ub))
        return X

    def addParameter(self, N_var, n_var, val=None):
        return [Param(n_var, val) for _ in range(N_var)]

    @staticmethod
    def _constraint_args(h, arguments, kind):
        """The reference's constraint plug-in (nlp/constraints.py: equality_constaint,
        args[0] - args[1]) on scalar elements ``X[i][k]`` of the state trajectory or one
        element and a constant: (a, b) with at least one Elem."""
        if _fname(h) != "equality_constaint":
            raise UnsupportedFeature(f"{kind} constraint plug-in {_fname(h)!r}: supported is equality_constaint "
                                     "(args[0] - args[1])")
        args = list(arguments)
        ok = len(args) == 2 and any(isinstance(a, Elem) for a in args) and all(
            isinstance(a, Elem) or np.ndim(a) == 0 for a in args)
        if not ok:
            raise UnsupportedFeature("equality_constaint needs two scalar elements (or an element and a constant), "
                                     "e.g. [X[i][2], X[i][7]]")
        return tuple(a if isinstance(a, Elem) else float(a) for a in args)

    def addIneqConstraint(self, g, arguments, params=None):
        """nlp/nlp.py:49-50: g(arguments) <= 0 with g = equality_constaint, i.e.
        args[0] <= args[1].  Enforced by an active set over Gauss-Newton solves:
        active rows are held at equality by the bordered KKT step, their multipliers
        decide release (see _solve_active_set).  Row cap: the device's bordered step
        holds at most 48 rows -- equality rows + extra variables + ACTIVE inequality
        rows, where a state bound next to constraint rows counts one row per node.
        More than that raises UnsupportedFeature (before any solve when the start
        already violates too many rows)."""
        self._ineq.append(self._constraint_args(g, arguments, "inequality"))

    def addEqConstraint(self, h, arguments, params=None):
        """nlp/nlp.py:52-53 with the reference's only equality plug-in,
        constraints.equality_constaint (args[0] - args[1] == 0)."""
        self._eq.append(self._constraint_args(h, arguments, "equality"))

    def setParameter(self, p, val):
        if not isinstance(p, Param):
            raise TypeError("setParameter expects a handle returned by addParameter")
        p.value = np.asarray(val, dtype=np.float64).reshape(-1)

    def setObjective(self):
        pass  # the objective is recorded term by term by the add*Cost calls

    def initialGuess(self, x, x0):
        x.init = np.asarray(x0, dtype=np.float64).reshape(-1)

    def extractVariableValue(self, name, idx=0):
        var_name = name + '_' + str(idx)
        if var_name in self.w.keys():
            if self.sol is not None:
                return np.array(self.w[var_name].value, dtype=np.float64).reshape(-1)
            print('Need to run solve() first')
            return None
        print('Could not find ' + name + '_' + str(idx) + '.')
        return None

    def extractSolution(self, name, t_array):
        X = []
        for i in range(self.N + 1):
            value = self.extractVariableValue(name, i)
            if value is None:
                return None
            X.append(value)
        T = len(t_array)
        sol = np.zeros((T, X[0].shape[0]))
        for t in range(T):
            sol[t, :] = self.CPM.evaluateSolution(t_array[t], X)
        return sol


class fixedTimeOptimalControlNLP(NLP):
    def __init__(self, N, T, n, m):
        raise UnsupportedFeature(
            "fixedTimeOptimalControlNLP (nlp/nlp.py:122-186) is out of scope: this framework "
            "accelerates the estimation path (fixedTimeOptimalEstimationNLP)")


class fixedTimeOptimalEstimationNLP(NLP):
    """Moving-horizon / collocation estimation problem (nlp/nlp.py:189-317)."""

    def __init__(self, N, T, n, m, phi_mode="bary", device="cuda"):
        super(fixedTimeOptimalEstimationNLP, self).__init__(N)
        self.T = T
        self.n = n
        self.m = m
        self.CPM = collocation.ChebyshevPseudospectralMethod(self.N, 0, T, phi_mode=phi_mode)
        self.device = device
        self._dyn = None
        self._dyn_cost = None
        self._meas = []
        self._prior = None
        self._X = None
        self._engine = None
        self._engine_key = None
        self.max_iter = 50
        self.tol = 1e-10

    # ------------------------------------------------------------ recording
    def addVariables(self, N_var, n_var, lb=None, ub=None, name='x'):
        X = super().addVariables(N_var, n_var, lb, ub, name)
        if name == 'x' and self._X is None:
            self._X = X
        return X

    def addDynamics(self, func, X, t_array=None, u_array=None, params=None):
        """nlp/nlp.py:202-240 -> (U, W); W is eliminated (see module docstring)."""
        if len(X) != self.N + 1:
            print('X must have N+1 points defined.')
        self._X = X
        U = self.addParameter(self.N + 1, self.m) if self.m != 0 else None
        if self.m == 0:
            print('No control input being used for dynamics.')
        W = super().addVariables(self.N + 1, self.n, name='w')
        self._dyn = (func, params, U, W)
        if u_array is not None:
            self.setControl(U, t_array, u_array)
        return U, W

    def addDynamicsCost(self, cost_function, W, params=None):
        """nlp/nlp.py:242-245: sum_k (T/2) w_k c(W_k)."""
        name = _fname(cost_function)
        self._huber = None
        if name == "weighted_l2_norm":
            Qw = np.asarray(_resolve(params["Q"]), dtype=np.float64).reshape(self.n, self.n)
        elif name == "l2_norm":
            Qw = np.eye(self.n)
        elif name == "pseudo_huber_loss":
            # cost_functions.py:25-31: only diag(Q) enters; solved by IRLS on the GPU
            Qw = np.asarray(_resolve(params["Q"]), dtype=np.float64).reshape(self.n, self.n)
            self._huber = float(_resolve(params["delta"]))
        else:
            raise UnsupportedFeature(f"dynamics cost {name!r}: supported are weighted_l2_norm, l2_norm and "
                                     "pseudo_huber_loss")
        self._dyn_cost = Qw

    def addResidualCost(self, measurement_model, X, t_array, y_array, R, params=None):
        """nlp/nlp.py:247-277: sum_i r_i^T R r_i, r_i = y_i - h(x(t_i), params)."""
        t_array = np.asarray(t_array, dtype=np.float64).reshape(-1)
        M_i = t_array.shape[0]
        p = y_array.shape[0] if y_array is not None else int(params["p"])
        Y = self.addParameter(M_i, p)
        self._meas.append(dict(h=measurement_model, t=t_array, Y=Y, R=R, params=params or {}, p=p))
        if y_array is not None:
            self.setMeasurement(Y, t_array, y_array)
        return Y

    def addInitialCost(self, cost_function, X0, params=None, x0=None):
        """nlp/nlp.py:279-286: c(X_0 - x0_guess)."""
        name = _fname(cost_function)
        if name == "weighted_l2_norm":
            Pw = params["Q"]
        elif name == "l2_norm":
            Pw = np.eye(self.n)
        else:
            raise UnsupportedFeature(f"initial cost {name!r} is not least-squares")
        x0_guess = self.addParameter(1, self.n)[0]
        self._prior = (Pw, x0_guess)
        if x0 is not None:
            self.setParameter(x0_guess, x0)
        return x0_guess

    def initializeEstimate(self, X, t_array, xhat_array):
        """nlp/nlp.py:288-302: interp1d of xhat (n, T) at the node times."""
        t_nodes = self.CPM.tau2t(self.CPM.tau)
        xhat_nodes = interp1d(t_array, xhat_array, fill_value="extrapolate")(t_nodes)
        for (i, x) in enumerate(X):
            self.initialGuess(x, xhat_nodes[:, i])

    def setControl(self, U, t_array, u_array):
        """nlp/nlp.py:304-308: linear interp1d with extrapolation at tau2t(tau_k)."""
        u_t = interp1d(t_array, u_array, fill_value="extrapolate")
        for k in range(self.N + 1):
            self.setParameter(U[k], u_t(self.CPM.tau2t(self.CPM.tau[k])))

    def setMeasurement(self, Y, t_array, y_array):
        """nlp/nlp.py:310-312 (Y may be one parameter handle, as CasADi's Y[i] indexing
        of a single MX parameter allows, gnss-multi-receiver.py:197)"""
        if isinstance(Y, Param):
            Y = [Y]
        for (i, t) in enumerate(t_array):
            self.setParameter(Y[i], np.asarray(y_array)[:, i])

    def addVarBounds(self, X, idx, lb, ub):
        """nlp/nlp.py:314-317.  Bounds on a component of the state trajectory are
        enforced by the projected Newton method (KKT point of the bounded problem);
        bounds on other variables are recorded and checked after solve()."""
        self._bounds.append((X, idx, lb, ub))

    def _enforced_bounds(self):
        """(component, lb, ub) for bounds on the state variables, intersected per component."""
        box = {}
        for X, idx, lb, ub in self._bounds:
            if self._X is None or (X is not self._X and list(X) != list(self._X)):
                continue  # not the state trajectory: recorded and checked only
            comps = list(range(self.n)) if idx is None else [int(idx)]
            lbv = np.broadcast_to(np.asarray(-np.inf if lb is None else lb, dtype=np.float64).reshape(-1), (len(comps),))
            ubv = np.broadcast_to(np.asarray(np.inf if ub is None else ub, dtype=np.float64).reshape(-1), (len(comps),))
            for c, lo, hi in zip(comps, lbv, ubv):
                plo, phi = box.get(c, (-np.inf, np.inf))
                box[c] = (max(plo, float(lo)), min(phi, float(hi)))
        return [(c, lo, hi) for c, (lo, hi) in sorted(box.items()) if np.isfinite(lo) or np.isfinite(hi)]

    # ------------------------------------------------------------ assembly
    _SIMPLE = ("full_state", "pseudorange", "vehicle_pseudorange", "multi_receiver_range_3d")

    def _extra_vars(self):
        """Decision variables other than the state trajectory that measurement params
        reference (``{"y": XA}``) -- the z of the bordered solve -- in declaration
        order: ([(Var, z offset)], total size).  Variables no cost term references
        keep their initial value, as they would under IPOPT (zero gradient)."""
        used = {id(v) for g in self._meas for v in g["params"].values() if isinstance(v, Var)}
        out, off = [], 0
        for vn in self.var_names:
            v = self.w[vn]
            if id(v) in used and not any(v is x for x in self._X):
                out.append((v, off))
                off += v.size
        return out, off

    def _is_general(self):
        names = {_fname(g["h"]) for g in self._meas}
        if len(names) != 1 or names.pop() not in self._SIMPLE:
            return True
        for g in self._meas:
            par = g["params"]
            if "idxA" in par or any(isinstance(v, Var) for v in par.values()):
                return True
        return False

    def _state_index(self, e):
        for j, x in enumerate(self._X):
            if e.var is x:
                return j * self.n + e.k
        raise UnsupportedFeature(f"constraint on {e!r}: only elements of the state trajectory are supported")

    def _row(self, a, b):
        """A constraint a - b (elements or constants) as (ia, ib, r, s): s (v[ia] - v[ib] - r)."""
        if isinstance(a, Elem) and isinstance(b, Elem):
            return self._state_index(a), self._state_index(b), 0.0, 1.0
        if isinstance(a, Elem):
            return self._state_index(a), -1, b, 1.0
        return self._state_index(b), -1, a, -1.0

    def _ineq_rows(self):
        """Every inequality row s (v[ia] - v[ib] - r) <= 0: addIneqConstraint rows and, when
        the problem also has constraint rows, the state bounds at every node (the device's
        projected Newton handles bounds alone, not bounds together with a bordered step)."""
        rows = [self._row(a, b) for a, b in self._ineq]
        if rows or self._eq:
            for c, lo, hi in self._enforced_bounds():
                for j in range(self.N + 1):
                    if np.isfinite(lo):
                        rows.append((j * self.n + c, -1, lo, -1.0))
                    if np.isfinite(hi):
                        rows.append((j * self.n + c, -1, hi, 1.0))
        return rows

    def _eq_pairs(self):
        """Equality rows for the device: the addEqConstraint rows, then the active set's."""
        rows = [self._row(a, b)[:3] for a, b in self._eq]
        ineq = self._ineq_rows() if self._active else []
        rows += [ineq[i][:3] for i in self._active]
        if not rows:
            return None, None
        return (np.array([(ia, ib) for ia, ib, _ in rows], dtype=np.int32),
                np.array([r for _, _, r in rows], dtype=np.float64))

    def _mixed_rows(self, zoff):
        """MHE_MEAS_MIXED encoding (include/mhe.h) of every addResidualCost term:
        (t (M,), rows (M,14), Rw (M,), Y (M,)), sorted by time (stable) so that
        rows at one time form one epoch on the device."""
        n = self.n

        def vec(v, k):
            return np.asarray(_resolve(v), dtype=np.float64).reshape(k)

        def var_or_const(par, key, k):
            y = par[key]
            if isinstance(y, Var):
                return [n + zoff[id(y)] + c for c in range(k)], np.zeros(k)
            return [-1] * k, vec(y, k)

        t_all, rows, Rw, Yv = [], [], [], []
        for g in self._meas:
            name, par, p = _fname(g["h"]), g["params"], g["p"]
            R = np.asarray(_resolve(g["R"]), dtype=np.float64).reshape(p, p)
            if name == "full_state":
                if np.any(R != np.diag(np.diag(R))):
                    raise UnsupportedFeature("full_state term in a mixed problem needs a diagonal R")
                proto = [([6, a] + [-1] * 6, np.zeros(6), R[a, a]) for a in range(p)]
            else:
                if p != 1:
                    raise UnsupportedFeature(f"{name}: scalar measurement expected, got p={p}")
                v = np.zeros(6)
                if name in ("pseudorange", "vehicle_pseudorange"):
                    idx = list(par.get("idx", [0, 1, 2, 3])) if name == "pseudorange" else [0, 1, 8, 6]
                    ids = [1] + idx + [-1] * 3
                    v[:3] = vec(par["sat_pos"], 3)
                elif name == "pseudorange_rate":
                    ids = [2, 0, 1, 2, 4, 5, 6, 7]
                    v[:3], v[3:6] = vec(par["sat_pos"], 3), vec(par["sat_vel"], 3)
                elif name in ("multi_receiver_range_2d", "multi_receiver_range_3d"):
                    K = 2 if name.endswith("2d") else 3
                    code = 3 if K == 2 else 4
                    if "y" in par:
                        ia = list(par.get("idx", list(range(K))))[:K]
                        ib, yv = var_or_const(par, "y", K)
                        v[:K] = yv
                    else:
                        ia, ib = list(par["idxA"])[:K], list(par["idxB"])[:K]
                    ids = [code] + ia + ib + [-1] * (7 - 2 * K)
                elif name == "multi_receiver_heading_2d":
                    if "y" in par:   # r_x = y0 - x[idx0], r_y = y1 - x[idx1]
                        idx = list(par.get("idx", [0, 1]))
                        yi, yv = var_or_const(par, "y", 2)
                        ids = [5, yi[0], idx[0], yi[1], idx[1], -1, -1, -1]
                        v[:2] = yv
                    else:            # r_x = x[b0] - x[a0] + 1e-5, r_y = x[b1] - x[a1]
                        a_, b_ = list(par["idxA"]), list(par["idxB"])
                        ids = [5, b_[0], a_[0], b_[1], a_[1], -1, -1, -1]
                        v[0] = .00001
                else:
                    raise UnsupportedFeature(f"measurement plug-in {name!r} has no mixed-row encoding")
                proto = [(ids, v, R[0, 0])]
            for i, t in enumerate(g["t"]):
                yi = g["Y"][i].get()
                for r, (ids, v, w) in enumerate(proto):
                    t_all.append(t)
                    rows.append(np.concatenate([np.asarray(ids, dtype=np.float64), v]))
                    Rw.append(w)
                    Yv.append(yi[r] if len(proto) > 1 else yi[0])
        t_all = np.asarray(t_all)
        order = np.argsort(t_all, kind="stable")
        return t_all[order], np.stack(rows)[order], np.asarray(Rw)[order], np.asarray(Yv)[order]

    def _spec(self):
        if self._dyn is None:
            raise ValueError("addDynamics() must be called before build()")
        if self._dyn_cost is None:
            raise ValueError("addDynamicsCost() must be called before build()")
        if not self._meas:
            raise ValueError("at least one addResidualCost() term is required")
        names = {_fname(g["h"]) for g in self._meas}
        mname = next(iter(names))
        t_meas, Rw, PAR, idx = [], [], [], None
        for g in self._meas:
            R = np.asarray(_resolve(g["R"]), dtype=np.float64).reshape(g["p"], g["p"])
            par = g["params"]
            row_par = None
            if mname in ("pseudorange", "vehicle_pseudorange"):
                row_par = np.asarray(_resolve(par["sat_pos"]), dtype=np.float64).reshape(3)
                if "idx" in par:
                    idx = list(par["idx"])
            elif mname == "multi_receiver_range_3d":
                row_par = np.asarray(_resolve(par["y"]), dtype=np.float64).reshape(3)
                idx = list(par.get("idx", [0, 1, 2]))
            for t in g["t"]:
                t_meas.append(t)
                Rw.append(R)
                if row_par is not None:
                    PAR.append(row_par)
        return mname, np.asarray(t_meas), np.stack(Rw), (np.stack(PAR) if PAR else None), idx

    def build(self, verbose=True):
        """Build the device constants (nlp/nlp.py:61-69).  As with the reference, build()
        may come before setParameter()/setMeasurement() (gnss-multi-receiver.py:142 vs
        :200-230): constants that depend on unset parameters are then built by solve()."""
        if self._dyn is None or self._dyn_cost is None or not self._meas:
            self._spec()  # raises the precise structural error
        try:
            self._build()
        except ParameterNotSet:
            self._engine_key = None

    def _verify_plugins(self):
        """Each user plug-in is checked once against the registered plug-in of its
        name (mhe.registry.verify_dyn / verify_meas): same values at seeded points,
        or UnsupportedPlugin -- a name alone does not select a device functor."""
        from mhe import registry
        done = self.__dict__.setdefault("_verified", set())
        rng = np.random.default_rng(7)

        def num(params):
            out = {}
            for k, v in (params or {}).items():
                if isinstance(v, Param):
                    out[k] = v.get()
                elif isinstance(v, Var):
                    out[k] = rng.normal(size=v.size) * 10.0   # an extra decision variable: any value
                else:
                    out[k] = v
            return out

        func, dparams = self._dyn[0], self._dyn[1]
        if id(func) not in done:
            registry.verify_dyn(func, num(dparams))
            done.add(id(func))
        for g in self._meas:
            h = g["h"]
            if id(h) in done:
                continue
            registry.verify_meas(h, num(g["params"]), self.n)
            done.add(id(h))

    def _build(self):
        from mhe import registry
        from mhe import solver as _solver
        if self._dyn is None or self._dyn_cost is None or not self._meas:
            self._spec()  # raises the precise error
        self._verify_plugins()
        func = self._dyn[0]
        dname = _fname(func)
        dyn_par = registry.dyn_params(dname, self._dyn[1]) if dname in registry.DYN else None
        Pw = None if self._prior is None else np.asarray(_resolve(self._prior[0]), dtype=np.float64)
        bounds = self._enforced_bounds()
        if self._ineq or self._eq:
            bounds = []   # held by the active set as constraint rows (_ineq_rows)
        huber = getattr(self, "_huber", None)
        extra, nz = self._extra_vars()
        eq, eq_rhs = self._eq_pairs()
        general = self._is_general() or nz > 0
        if general:
            if nz > 4:
                raise UnsupportedFeature(f"{nz} extra decision variables (at most 4 on the GPU path)")
            zoff = {id(v): off for v, off in extra}
            t_meas, rows, Rw, Yv = self._mixed_rows(zoff)
            mname, idx, PAR = "mixed", None, rows
            self._Ymixed = Yv
        else:
            mname, t_meas, Rw, PAR, idx = self._spec()
            self._Ymixed = None
        Phi = self.CPM.lagrange_matrix(t_meas)
        # R enters the device constants only for a linear h (folded into J^T W J); a
        # nonlinear model takes it per solve (mhe_solve_args.Rw), so re-setting R every
        # window -- the R = 0 slot masks of autonomous-car.py:250-263 -- reuses the engine
        linear = registry.MEAS[mname][3]
        key = (mname, t_meas.tobytes(), Rw.tobytes() if linear else Rw.shape, None if Pw is None else Pw.tobytes(),
               self._dyn_cost.tobytes(), huber, tuple(bounds), nz, None if eq is None else eq.tobytes(),
               None if eq_rhs is None else eq_rhs.tobytes(), None if dyn_par is None else dyn_par.tobytes())
        if self._engine is None or self._engine_key != key:
            self._engine = _solver.BatchSolver(self.N, self.T, func, mname, self.CPM.D, (self.T / 2.0) * self.CPM.w,
                                               Phi, self._dyn_cost, Rw, Pw=Pw, meas_idx=idx, device=self.device,
                                               dyn_cost="huber" if huber is not None else "l2", huber_delta=huber,
                                               bounds=bounds, n_extra=nz, eq=eq, eq_rhs=eq_rhs, dyn_par=dyn_par)
            self._engine_key = key
            self.engine_builds = getattr(self, "engine_builds", 0) + 1
        self._Rw_solve = None if linear else Rw
        self._PAR = PAR
        self._extra = extra

    def batch_solver(self):
        """The BatchSolver of this problem structure (many trajectories at once)."""
        if self._engine is None:
            self._build()
        return self._engine

    # ------------------------------------------------------------ solve
    MAX_ACTIVE_SET_STEPS = 60

    def solve(self, warmstart=False):
        """Gauss-Newton on the GPU (replaces opti.solve(), nlp/nlp.py:76-83)."""
        if warmstart and self.sol is not None:
            print('Warmstarting with previous solution')
        if self._ineq or (self._eq and self._enforced_bounds()):
            return self._solve_active_set(warmstart)
        return self._solve_once(warmstart)

    def _solve_active_set(self, warmstart):
        """Inequality rows s (v[a] - v[b] - r) <= 0 by a primal active set over GN solves
        (the KKT conditions IPOPT's interior point also reaches: feasibility, mu >= 0,
        mu_i = 0 off the active set).  Each step solves the problem with the active rows
        held at equality (bordered KKT step, multipliers lambda from the device:
        L = J + lambda^T (C v - r), so mu = s lambda); then every violated inactive row
        is added, or else the active row with the most negative mu is released.  The
        start is the first solve's: rows violated at the initial iterate are active."""
        rows = self._ineq_rows()
        n_fixed = len(self._eq) + self._extra_vars()[1]
        if n_fixed > 48:
            raise UnsupportedFeature("more than 48 equality rows and extra variables")

        def gvals():
            v = np.concatenate([x.value if x.value is not None else (x.init if x.init is not None else
                                np.zeros(self.n)) for x in self._X]).astype(np.float64)
            return np.array([s_ * (v[ia] - (v[ib] if ib >= 0 else 0.0) - r) for ia, ib, r, s_ in rows])

        if warmstart and self.sol is not None:
            g0 = gvals()
        else:
            saved = [x.value for x in self._X]
            for x in self._X:
                x.value = None
            g0 = gvals()
            for x, v in zip(self._X, saved):
                x.value = v
        # the device's bordered step holds at most 48 rows (equality rows + extra variables
        # + active inequality rows): start with the most-violated rows up to that cap --
        # holding them may pull the rest feasible; rows still violated once no room is
        # left end the loop below with UnsupportedFeature
        start_active = [i for i in np.argsort(-g0) if g0[i] > 0][:48 - n_fixed]
        self._active = start_active
        history = []
        for step in range(self.MAX_ACTIVE_SET_STEPS):
            lam_t = self._solve_once(warmstart or step > 0, _quiet=True)
            if not self.solver["success"]:
                # an inner Gauss-Newton failure is the result: keep its status
                warnings.warn(f"active set step {step}: Gauss-Newton solve ended with "
                              f"{self.solver['return_status']}")
                self.solver["active_set_steps"] = step + 1
                return
            g = gvals()
            scale = 1.0 + max(np.abs(x.value).max() for x in self._X)
            lam = lam_t.cpu().numpy()[0] if lam_t is not None else np.zeros(0)
            mu = np.array([rows[i][3] * lam[len(self._eq) + k] for k, i in enumerate(self._active)])
            viol = [i for i in np.argsort(-g) if g[i] > 1e-9 * scale and i not in self._active]
            history.append(len(self._active))
            mu_tol = 1e-9 * (1.0 + (np.abs(lam).max() if lam.size else 0.0))
            if viol:
                room = 48 - n_fixed - len(self._active)
                if room <= 0:
                    raise UnsupportedFeature("active set needs more than 48 constraint rows")
                self._active = self._active + viol[:room]
            elif mu.size and mu.min() < -mu_tol:
                self._active = [i for k, i in enumerate(self._active) if k != int(np.argmin(mu))]
            else:
                self.solver["active_set"] = [rows[i] for i in self._active]
                self.solver["multipliers"] = mu
                self.solver["active_set_steps"] = step + 1
                return
        warnings.warn("active set did not settle: returning the last Gauss-Newton solve")
        self.solver["success"] = False
        self.solver["active_set_steps"] = len(history)

    def _solve_once(self, warmstart=False, _quiet=False):
        self._build()  # cheap when nothing changed; picks up re-set R / prior weights / params
        eng = self._engine
        P, n = self.N + 1, self.n

        def start(x):
            if warmstart and self.sol is not None and x.value is not None:
                return x.value
            return x.init if x.init is not None else 0.0  # CasADi's default initial value

        X0 = np.zeros((1, P, n))
        for k, x in enumerate(self._X):
            X0[0, k] = start(x)
        Z0 = None
        if eng.n_extra:
            Z0 = np.concatenate([np.broadcast_to(np.asarray(start(v), dtype=np.float64).reshape(-1), (v.size,))
                                 for v, _ in self._extra])[None]
        U = None
        if self.m > 0:
            U = np.stack([u.get() for u in self._dyn[2]])[None]
        if self._Ymixed is not None:
            Y = self._Ymixed.reshape(1, -1, 1)
        else:
            Y = np.concatenate([np.stack([y.get() for y in g["Y"]]) for g in self._meas])[None]
        PAR = None if self._PAR is None else self._PAR[None]
        x0 = None if self._prior is None else self._prior[1].get()[None]
        import torch
        t0 = time.perf_counter()
        Rw = None if self._Rw_solve is None else self._Rw_solve[None]
        lam_t = None
        if eng.n_eq:
            lam_t = torch.empty((1, eng.n_eq), dtype=torch.float64, device=eng.device)
        out = eng.solve(X0, U, Y, PAR, x0, max_iter=self.max_iter, tol=self.tol, Z0=Z0, Rw=Rw, lam_out=lam_t)
        X, cost, iters, status = out[:4]
        torch.cuda.synchronize()
        t_wall = time.perf_counter() - t0
        X = X.cpu().numpy()[0]
        st = int(status.cpu().numpy()[0])
        for k, x in enumerate(self._X):
            x.value = X[k].copy()
        if eng.n_extra:
            Z = out[4].cpu().numpy()[0]
            for v, off in self._extra:
                v.value = Z[off:off + v.size].copy()
        # W eliminated: W_k = (2/T) sum_j D_kj X_j - f(X_k, U_k)  (nlp/nlp.py:235)
        func, dparams, Uh, W = self._dyn
        for k, wv in enumerate(W):
            f = func(X[k], Uh[k].get(), dparams) if self.m > 0 else func(X[k], dparams)
            wv.value = (2.0 / self.T) * (self.CPM.D[k] @ X) - np.asarray(f, dtype=np.float64).reshape(-1)
        self.sol = {v: self.w[v].value for v in self.var_names}
        statuses = {0: "Solve_Succeeded", 1: "Maximum_Iterations_Exceeded", 2: "Not_Positive_Definite",
                    3: "Invalid_Number_Detected"}
        self.solver = {"t_wall_total": t_wall, "iter_count": int(iters.cpu().numpy()[0]),
                       "return_status": statuses[st], "success": st == 0,
                       "objective": float(cost.cpu().numpy()[0]), "bounds_violated": self._check_bounds()}
        if st != 0 and not _quiet:
            warnings.warn(f"Gauss-Newton solve ended with {statuses[st]}")
        return lam_t

    def _check_bounds(self):
        viol = False
        for X, idx, lb, ub in self._bounds:
            for x in X:
                if x.value is None:
                    continue
                v = x.value if idx is None else x.value[idx]
                if lb is not None and np.any(v < np.asarray(lb) - 1e-9):
                    viol = True
                if ub is not None and np.any(v > np.asarray(ub) + 1e-9):
                    viol = True
        if viol:
            warnings.warn("solution violates a recorded variable bound (only state-trajectory bounds are enforced)")
        return viol
