"""A lazy-expression stand-in for the part of CasADi the reference's nlp/nlp.py uses
(build container only; test infrastructure, never imported by the product or on the
GPU box).

CasADi is not installed here, so the reference's own problem builder
(``fixedTimeOptimalEstimationNLP``, /root/reference/nlp/nlp.py:189-317) cannot run
against it.  This module provides just enough of its surface for that builder and the
reference plug-ins to run UNMODIFIED and record what they build:

  * ``Opti``: ``variable`` / ``parameter`` return symbols; ``set_value`` /
    ``set_initial`` record values; ``subject_to`` records the constraint expressions
    (``==``, ``<=``, ``>=``); ``minimize`` records the objective; ``solver`` is
    recorded; ``solve`` refuses (there is no IPOPT -- this is for evaluation only);
  * ``MX.sym``, ``Function`` (a call node that evaluates its body with the actual
    arguments bound -- free symbols inside the body, e.g. opti parameters captured in
    a measurement's params dict, resolve from the outer bindings as in CasADi);
  * the operators the plug-ins import: vertcat, sin, cos, tan, sqrt, atan2, dot,
    norm_2, mtimes, plus numpy ufuncs on expressions (kinematic_bycicle_and_bias
    calls np.cos on a symbol).

Every expression is a node of a DAG; ``evaluate(expr, bindings)`` computes its value
(float64 column vectors / matrices, CasADi's shapes: a vector is n x 1, x[i] is 1 x 1,
x.T a row) iteratively, so a long ``J += ...`` chain needs no recursion.
"""
import numpy as np

_NEXT = [0]


def _shape_of(v):
    return tuple(np.shape(v))


def _const_value(c):
    a = np.asarray(c, dtype=np.float64)
    if a.ndim == 0:
        return a.reshape(1, 1)
    if a.ndim == 1:
        return a.reshape(-1, 1)  # a 1-D array is a column (DM semantics)
    return a


class Expr:
    """One node: op in {sym, const, add, sub, mul, div, pow, neg, mtimes, T, index,
    vcat, fn1, fn2, call}."""
    __array_priority__ = 1000

    def __init__(self, op, args, shape, name=None):
        self.op, self.args, self.shape, self.name = op, args, shape, name
        _NEXT[0] += 1
        self.uid = _NEXT[0]

    __hash__ = object.__hash__

    # ---------------------------------------------------------------- building
    @staticmethod
    def sym(name, n=1, m=1):
        return Expr("sym", (), (int(n), int(m)), name)

    @staticmethod
    def wrap(x):
        if isinstance(x, Expr):
            return x
        v = _const_value(x)
        return Expr("const", (v,), v.shape)

    @staticmethod
    def _ew(op, a, b):
        a, b = Expr.wrap(a), Expr.wrap(b)
        if a.shape == b.shape or b.shape == (1, 1):
            sh = a.shape
        elif a.shape == (1, 1):
            sh = b.shape
        else:
            raise ValueError(f"dimension mismatch {a.shape} {op} {b.shape}")
        return Expr(op, (a, b), sh)

    def __add__(self, o): return Expr._ew("add", self, o)
    def __radd__(self, o): return Expr._ew("add", o, self)
    def __sub__(self, o): return Expr._ew("sub", self, o)
    def __rsub__(self, o): return Expr._ew("sub", o, self)
    def __mul__(self, o): return Expr._ew("mul", self, o)
    def __rmul__(self, o): return Expr._ew("mul", o, self)
    def __truediv__(self, o): return Expr._ew("div", self, o)
    def __rtruediv__(self, o): return Expr._ew("div", o, self)
    def __pow__(self, o): return Expr._ew("pow", self, o)
    def __rpow__(self, o): return Expr._ew("pow", o, self)
    def __neg__(self): return Expr("neg", (self,), self.shape)
    def __pos__(self): return self

    @property
    def T(self):
        return Expr("T", (self,), (self.shape[1], self.shape[0]))

    def __getitem__(self, key):
        probe = np.zeros(self.shape)[self._key(key)]
        sh = (1, 1) if np.ndim(probe) == 0 else (np.reshape(probe, (np.shape(probe)[0], -1)).shape)
        return Expr("index", (self, key), sh)

    def _key(self, key):
        # CasADi indexes a column vector by its rows: x[i], x[a:b], x[[i, j]]
        if self.shape[1] == 1 and not isinstance(key, tuple):
            return (key, 0) if isinstance(key, (int, np.integer)) else (key, slice(None))
        return key

    def __len__(self):
        return self.shape[0]

    # comparisons record constraints (nlp.py:33-35, :50, :53, :235, :316-317)
    def __eq__(self, o): return Constraint("==", self, Expr.wrap(o))
    def __le__(self, o): return Constraint("<=", self, Expr.wrap(o))
    def __ge__(self, o): return Constraint(">=", self, Expr.wrap(o))

    # numpy ufuncs on expressions (np.cos(x[2]), np.float64 * x, ...)
    _UFUNC = {"add": "add", "subtract": "sub", "multiply": "mul", "true_divide": "div", "divide": "div",
              "power": "pow"}
    _UNARY = {"sin", "cos", "tan", "sqrt", "negative", "arctan", "exp", "log", "absolute"}

    def __array_ufunc__(self, ufunc, method, *inputs, **kw):
        if method != "__call__" or kw:
            return NotImplemented
        name = ufunc.__name__
        if name in Expr._UFUNC:
            return Expr._ew(Expr._UFUNC[name], inputs[0], inputs[1])
        if name == "negative":
            return -Expr.wrap(inputs[0])
        if name in Expr._UNARY:
            return fn1(name, inputs[0])
        if name == "arctan2":
            return fn2("arctan2", inputs[0], inputs[1])
        if name in ("equal", "less_equal", "greater_equal"):
            op = {"equal": "==", "less_equal": "<=", "greater_equal": ">="}[name]
            return Constraint(op, Expr.wrap(inputs[0]), Expr.wrap(inputs[1]))
        return NotImplemented

    # methods numpy calls for ufuncs on 0-d object arrays
    def sin(self): return fn1("sin", self)
    def cos(self): return fn1("cos", self)
    def tan(self): return fn1("tan", self)
    def sqrt(self): return fn1("sqrt", self)


class Constraint:
    def __init__(self, kind, lhs, rhs):
        self.kind, self.lhs, self.rhs = kind, lhs, rhs

    def residual(self):
        """lhs - rhs (== 0, <= 0 or >= 0 as `kind` says)."""
        return self.lhs - self.rhs


def fn1(name, x):
    if not isinstance(x, Expr):
        return getattr(np, {"sqrt": "sqrt"}.get(name, name))(x)
    return Expr("fn1", (name, x), x.shape)


def fn2(name, a, b):
    if not isinstance(a, Expr) and not isinstance(b, Expr):
        return getattr(np, name)(a, b)
    return Expr._ew("fn2:" + name, a, b)


def _is_sym(x):
    return isinstance(x, Expr)


# ---------------------------------------------------------------- casadi surface
def vertcat(*args):
    if not any(_is_sym(a) for a in args):
        return np.concatenate([np.atleast_1d(np.asarray(a, dtype=np.float64)).ravel() for a in args])
    parts = [Expr.wrap(a) for a in args]
    return Expr("vcat", tuple(parts), (sum(p.shape[0] for p in parts), 1))


def sin(x): return fn1("sin", x)
def cos(x): return fn1("cos", x)
def tan(x): return fn1("tan", x)
def sqrt(x): return fn1("sqrt", x)
def atan2(y, x): return fn2("arctan2", y, x)


def mtimes(a, b):
    if not _is_sym(a) and not _is_sym(b):
        a, b = np.asarray(a), np.asarray(b)
        return a * b if a.ndim == 0 or b.ndim == 0 else a @ b
    a, b = Expr.wrap(a), Expr.wrap(b)
    if a.shape == (1, 1) or b.shape == (1, 1):
        return Expr._ew("mul", a, b)
    if a.shape[1] != b.shape[0]:
        raise ValueError(f"mtimes {a.shape} x {b.shape}")
    return Expr("mtimes", (a, b), (a.shape[0], b.shape[1]))


def dot(a, b):
    if not _is_sym(a) and not _is_sym(b):
        return float(np.sum(np.asarray(a) * np.asarray(b)))
    a, b = Expr.wrap(a), Expr.wrap(b)
    return mtimes(a.T, b)


def norm_2(a):
    if not _is_sym(a):
        return float(np.sqrt(np.sum(np.asarray(a) ** 2)))
    return sqrt(dot(a, a))


class MX:
    @staticmethod
    def sym(name, n=1, m=1):
        return Expr.sym(name, n, m)


class Function:
    """casadi.Function(name, inputs, outputs): calling it on expressions makes a call
    node; its body is evaluated with the formal inputs bound to the actual values
    (free symbols in the body resolve from the outer bindings)."""

    def __init__(self, name, inputs, outputs, *opts):
        self.name, self.inputs = name, list(inputs)
        outs = [Expr.wrap(o) for o in outputs]
        self.outputs = outs

    def __call__(self, *args):
        if len(args) != len(self.inputs):
            raise TypeError(f"{self.name}: {len(self.inputs)} inputs, got {len(args)}")
        args = tuple(Expr.wrap(a) for a in args)
        for a, f in zip(args, self.inputs):
            if a.shape != f.shape:
                raise ValueError(f"{self.name}: argument shape {a.shape} for input {f.shape}")
        return Expr("call", (self, args), self.outputs[0].shape)


class Opti:
    def __init__(self):
        self.variables, self.parameters, self.constraints = [], [], []
        self.values, self.initial = {}, {}
        self.objective, self.solver_args = None, None

    def variable(self, n=1, m=1):
        s = Expr.sym(f"opti_x_{len(self.variables)}", n, m)
        self.variables.append(s)
        return s

    def parameter(self, n=1, m=1):
        s = Expr.sym(f"opti_p_{len(self.parameters)}", n, m)
        self.parameters.append(s)
        return s

    @staticmethod
    def _as(sym, val):
        v = np.asarray(val, dtype=np.float64)
        if v.size == 1:
            return np.full(sym.shape, float(v.ravel()[0]))
        return v.reshape(sym.shape)

    def set_value(self, p, val):
        if p.op == "index" and p.args[0].op == "sym":
            # a slice of a parameter (setMeasurement passes Y[i] of a single parameter:
            # nlp.py:310-312 indexes it): write into that parameter's value
            base = p.args[0]
            cur = self.values.get(base)
            if cur is None:
                cur = np.full(base.shape, np.nan)
            cur = cur.copy()
            cur[base._key(p.args[1])] = self._as(p, val).reshape(np.shape(cur[base._key(p.args[1])]))
            self.values[base] = cur
            return
        if p.op != "sym":
            raise TypeError("set_value expects a parameter")
        self.values[p] = self._as(p, val)

    def set_initial(self, x, val):
        self.initial[x] = self._as(x, val)

    def subject_to(self, c):
        if not isinstance(c, Constraint):
            raise TypeError("subject_to expects a constraint expression")
        self.constraints.append(c)

    def minimize(self, J):
        self.objective = Expr.wrap(J)

    def solver(self, *args):
        self.solver_args = args

    def solve(self):
        raise NotImplementedError("casadi_lazy has no IPOPT: it records and evaluates the problem only")


# ---------------------------------------------------------------- evaluation
def _apply(node, vals):
    op, a = node.op, node.args
    if op == "const":
        return a[0]
    if op == "add":
        return vals[0] + vals[1]
    if op == "sub":
        return vals[0] - vals[1]
    if op == "mul":
        return vals[0] * vals[1]
    if op == "div":
        return vals[0] / vals[1]
    if op == "pow":
        return vals[0] ** vals[1]
    if op == "neg":
        return -vals[0]
    if op == "mtimes":
        return vals[0] @ vals[1]
    if op == "T":
        return vals[0].T
    if op == "index":
        v = vals[0][node.args[0]._key(a[1])]
        return np.asarray(v, dtype=np.float64).reshape(node.shape)
    if op == "vcat":
        return np.concatenate([v.reshape(-1, 1) for v in vals], axis=0)
    if op == "fn1":
        return getattr(np, a[0])(vals[0])
    if op.startswith("fn2:"):
        return getattr(np, op[4:])(vals[0], vals[1])
    raise KeyError(op)


def _children(node):
    op, a = node.op, node.args
    if op in ("sym", "const"):
        return ()
    if op in ("neg", "T"):
        return (a[0],)
    if op == "index":
        return (a[0],)
    if op == "fn1":
        return (a[1],)
    if op == "call":
        return a[1]
    return tuple(a)


def evaluate(expr, bindings):
    """Value of `expr` with symbol -> value `bindings` (dict keyed by the symbol
    objects).  A call node evaluates its Function's body with the formal inputs bound
    to the evaluated arguments on top of `bindings`."""
    if not isinstance(expr, Expr):
        return _const_value(expr)
    memo = {}
    stack = [(expr, False)]
    while stack:
        node, ready = stack.pop()
        if node.uid in memo:
            continue
        kids = _children(node)
        if not ready:
            stack.append((node, True))
            stack.extend((k, False) for k in kids if k.uid not in memo)
            continue
        if node.op == "sym":
            if node not in bindings:
                raise KeyError(f"unbound symbol {node.name} {node.shape}")
            memo[node.uid] = np.asarray(bindings[node], dtype=np.float64).reshape(node.shape)
        elif node.op == "call":
            fn, args = node.args
            inner = dict(bindings)
            for f, v in zip(fn.inputs, (memo[k.uid] for k in args)):
                inner[f] = v
            memo[node.uid] = evaluate(fn.outputs[0], inner)
        else:
            v = _apply(node, [memo[k.uid] for k in kids])
            memo[node.uid] = np.asarray(v, dtype=np.float64).reshape(node.shape)
    return memo[expr.uid]
