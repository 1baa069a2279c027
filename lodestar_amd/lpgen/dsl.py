"""Graph of Fp / flag nodes with lazy linear forms.

Fp values are linear forms sum_k c_k * node_k over materialized nodes (small
integer coefficients).  Additions, subtractions and small multiples are free:
they only merge forms.  A product, select, inversion or predicate creates a
node whose operands are forms -- the device unit evaluates each form limb-wise
(bls_coop.h), so e.g. a Karatsuba operand (a0 + a1) costs no round of its own.

Arithmetic domain: 13-limb Montgomery form, R = 2^416 (bls_coop.h).  Every
materialized node has an exclusive upper bound on its (non-canonical) value; a
product of operands x, y is < x y / 2^416 + p, so products of forms up to
~2^399 stay below 2^383 with no reduction, and a form's worst case
sum_pos c B + K p (K p covering the negative terms) decides whether its unit
reduces it first (rare).  Inputs arrive canonical in the one-lane code's
Montgomery form (R = 2^384) and are converted by one product each.
"""
from __future__ import annotations

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 416              # Montgomery radix of the latency path (13 x 32-bit limbs)
R384 = 1 << 384           # the one-lane code's radix (inputs)
RINV = pow(R, -1, P)
B383 = 1 << 383
LIMIT = 1 << 404          # a form's worst case must stay below this (reduce's quotient estimate)
RED_BOUND = 11 * P // 10  # bound after reduce (< 1.1 p)
MUL_LIMIT = R * (B383 - P - 1)  # operand bounds' product for a product < 2^383
LIN_REDUCE = 1 << 390     # a materialized form above this is reduced first
MAX_TERMS = 16            # larger operand forms are materialized before a unit uses them
MAX_LIN_TERMS = 64        # a materializing (LIN) unit takes up to this many terms
IN_CONV = R * R * pow(R384, -1, P) % P  # mont384(v) * IN_CONV / R = mont416(v)


def mont(v: int) -> int:
    return v % P * R % P


# node kinds with an Fp value (others produce flags)
FP_KINDS = ("in", "const", "mul", "lin", "sel", "inv", "canon")
FLAG_KINDS = ("inflag", "iszero", "bit0", "gthalf", "fop")


class Graph:
    def __init__(self, name: str):
        self.name = name
        self.kind: list = []
        self.args: list = []
        self.bound: list = []
        self.consts: dict = {}      # stored value -> node
        self.n_in = 0
        self.n_inflag = 0
        self.outs: list = []        # (name, node): Fp outputs
        self.outflags: list = []    # (name, node): flag outputs
        self.in_names: list = []
        self.inflag_names: list = []
        self._lin_cache: dict = {}
        self._fop_cache: dict = {}

    # ---- node creation -------------------------------------------------
    def _new(self, kind, args, bound=None) -> int:
        self.kind.append(kind)
        self.args.append(args)
        self.bound.append(bound)
        return len(self.kind) - 1

    def input(self, name: str) -> "Fp":
        """An input given canonical in Montgomery form with R = 2^384 (the one-lane
        code's form), loaded before round 0 and converted by one product."""
        n = self._new("in", (self.n_in,), P)
        self.in_names.append(name)
        self.n_in += 1
        return self.mul(Fp(self, {n: 1}), self._const_stored(IN_CONV))

    def input_raw(self, name: str) -> "Fp":
        """An input already in this domain (R = 2^416), e.g. a Miller value passed
        between programs."""
        n = self._new("in", (self.n_in,), B383)
        self.in_names.append(name)
        self.n_in += 1
        return Fp(self, {n: 1})

    def input_flag(self, name: str) -> "Flag":
        n = self._new("inflag", (self.n_inflag,))
        self.inflag_names.append(name)
        self.n_inflag += 1
        return Flag(self, n)

    def const(self, v: int) -> "Fp":
        """The field element v (stored in Montgomery form)."""
        v %= P
        if v == 0:
            return Fp(self, {})
        return self._const_stored(mont(v))

    def const_raw(self, stored: int) -> "Fp":
        """A register holding `stored` verbatim (e.g. raw 1: x * raw1 = from_mont(x))."""
        return self._const_stored(stored)

    def _const_stored(self, stored: int) -> "Fp":
        n = self.consts.get(stored)
        if n is None:
            n = self._new("const", (stored,), P if stored < P else B383)
            self.consts[stored] = n
        return Fp(self, {n: 1})

    def zero(self) -> "Fp":
        return Fp(self, {})

    def one(self) -> "Fp":
        return self.const(1)

    # ---- forms -----------------------------------------------------------
    def form_stats(self, t: dict):
        """(worst-case value, K) of sum c x + K p for form t."""
        pos = sum(c * self.bound[n] for n, c in t.items() if c > 0)
        neg = sum(-c * self.bound[n] for n, c in t.items() if c < 0)
        K = -(-neg // P)
        return pos + K * P, K

    def operand(self, f: "Fp") -> tuple:
        """A unit operand: the form as a sorted tuple of (node, coef), materializing
        it first when it is too large for one unit."""
        t = f.t
        if not t:
            return ()
        worst, _ = self.form_stats(t)
        if len(t) > MAX_TERMS or worst >= LIMIT:
            return ((self.materialize(f), 1),)
        return tuple(sorted(t.items()))

    def materialize(self, f: "Fp") -> int:
        """Node holding the value of form f (< 2^383)."""
        t = f.t
        if len(t) == 1:
            (n, c), = t.items()
            if c == 1:
                return n
        key = tuple(sorted(t.items()))
        n = self._lin_cache.get(key)
        if n is not None:
            return n
        if len(t) > MAX_LIN_TERMS or self.form_stats(t)[0] >= LIMIT:
            assert len(t) > 1, "a single term out of range: materialize the chain earlier"
            # split into materialized halves
            items = list(key)
            half = len(items) // 2
            a = Fp(self, dict(items[:half]))
            b = Fp(self, dict(items[half:]))
            op = ((self.materialize(a), 1), (self.materialize(b), 1))
        else:
            op = key
        worst, _ = self.form_stats(dict(op))
        n = self._new("lin", (op,), RED_BOUND if worst > LIN_REDUCE else worst)
        self._lin_cache[key] = n
        return n

    # ---- units -------------------------------------------------------------
    def mul(self, a: "Fp", b: "Fp") -> "Fp":
        if not a.t or not b.t:
            return Fp(self, {})
        x = self.operand(a)
        y = self.operand(b)
        bx = self.form_stats(dict(x))[0]
        by = self.form_stats(dict(y))[0]
        rx = ry = 0
        # reduce the larger operand(s) until the product stays below 2^383
        while bx * by >= MUL_LIMIT:
            if bx >= by and not rx:
                rx, bx = 1, RED_BOUND
            elif not ry:
                ry, by = 1, RED_BOUND
            else:
                rx, bx = 1, RED_BOUND
        n = self._new("mul", (x, y, rx, ry), bx * by // R + P + 1)
        assert self.bound[n] <= B383
        return Fp(self, {n: 1})

    def _op_bound(self, op) -> int:
        worst, _ = self.form_stats(dict(op))
        return RED_BOUND if worst > LIN_REDUCE else worst

    def select(self, flag: "Flag", a: "Fp", b: "Fp") -> "Fp":
        """flag ? a : b"""
        return self.select_n([(flag, a)], b)

    def select_n(self, cases, default: "Fp") -> "Fp":
        """The value of the first case whose flag is set, else default: ONE unit
        (the flags are row-uniform; the unit evaluates only the chosen form)."""
        live = []
        for fl, v in cases:
            if fl.const is None:
                live.append((fl, v))
            elif fl.const:
                default = v
                break
        if all(v.t == default.t for _, v in live):
            return default
        ops = tuple(self.operand(v) for _, v in live) + (self.operand(default),)
        flags = tuple(fl.n for fl, _ in live)
        n = self._new("sel", (flags, ops), max([self._op_bound(o) for o in ops] + [1]))
        return Fp(self, {n: 1})

    def inv(self, a: "Fp") -> "Fp":
        """a^-1 (0 -> 0)."""
        if not a.t:
            return Fp(self, {})
        n = self._new("inv", (self.operand(a),), P)
        return Fp(self, {n: 1})

    def canon(self, a: "Fp") -> "Fp":
        n = self._new("canon", (self.operand(a),), P)
        return Fp(self, {n: 1})

    def _pred(self, kind, a: "Fp") -> "Flag":
        return Flag(self, self._new(kind, (self.operand(a),)))

    def is_zero(self, a: "Fp") -> "Flag":
        if not a.t:
            return Flag(self, None, True)
        return self._pred("iszero", a)

    def bit0(self, a: "Fp") -> "Flag":
        """lowest bit of the canonical value of a (a raw, non-Montgomery value)"""
        if not a.t:
            return Flag(self, None, False)
        return self._pred("bit0", a)

    def gt_half(self, a: "Fp") -> "Flag":
        """canonical value of a > (p - 1)/2 (a raw)"""
        if not a.t:
            return Flag(self, None, False)
        return self._pred("gthalf", a)

    def fop(self, op: str, a: "Flag", b: "Flag") -> "Flag":
        key = (op, a.n, b.n) if op != "not" else (op, a.n, None)
        n = self._fop_cache.get(key)
        if n is None:
            n = self._new("fop", (op, a.n, b.n if b is not None else None))
            self._fop_cache[key] = n
        return Flag(self, n)

    # ---- outputs -----------------------------------------------------------
    def output(self, name: str, f: "Fp", canonical: bool = False):
        if not f.t:
            f = self._const_stored(0)
        n = self.canon(f).node() if canonical else self.materialize(f)
        self.outs.append((name, n))

    def output_flag(self, name: str, fl: "Flag"):
        if fl.const is not None:
            # a constant flag still needs a node: fold it into an op on an input-free node
            fl = Flag(self, self._new("fop", ("const", int(fl.const), None)))
        self.outflags.append((name, fl.n))


class Fp:
    """Lazy linear form over materialized nodes."""
    __slots__ = ("g", "t")

    def __init__(self, g: Graph, t: dict):
        self.g = g
        self.t = {k: v for k, v in t.items() if v}

    def _lift(self, o):
        if isinstance(o, Fp):
            return o
        if isinstance(o, int):
            return self.g.const(o)
        raise TypeError(o)

    def __add__(self, o):
        o = self._lift(o)
        t = dict(self.t)
        for k, v in o.t.items():
            t[k] = t.get(k, 0) + v
        return Fp(self.g, t)

    __radd__ = __add__

    def __neg__(self):
        return Fp(self.g, {k: -v for k, v in self.t.items()})

    def __sub__(self, o):
        return self + (-self._lift(o))

    def __rsub__(self, o):
        return self._lift(o) - self

    def scale(self, k: int) -> "Fp":
        return Fp(self.g, {n: c * k for n, c in self.t.items()})

    def __mul__(self, o):
        if isinstance(o, int):
            return self.scale(o)
        return self.g.mul(self, o)

    def __rmul__(self, o):
        if isinstance(o, int):
            return self.scale(o)
        return NotImplemented

    def sqr(self) -> "Fp":
        return self.g.mul(self, self)

    def mat(self) -> "Fp":
        """Materialize (one LIN unit) unless already a single node."""
        if not self.t:
            return self
        return Fp(self.g, {self.g.materialize(self): 1})

    def node(self) -> int:
        (n, c), = self.t.items()
        assert c == 1
        return n

    def is_zero_form(self) -> bool:
        return not self.t


class Flag:
    __slots__ = ("g", "n", "const")

    def __init__(self, g: Graph, n, const=None):
        self.g, self.n, self.const = g, n, const

    def __and__(self, o: "Flag") -> "Flag":
        if self.const is not None:
            return o if self.const else self
        if o.const is not None:
            return self if o.const else o
        if self.n == o.n:
            return self
        return self.g.fop("and", self, o)

    def __or__(self, o: "Flag") -> "Flag":
        if self.const is not None:
            return self if self.const else o
        if o.const is not None:
            return o if o.const else self
        if self.n == o.n:
            return self
        return self.g.fop("or", self, o)

    def __xor__(self, o: "Flag") -> "Flag":
        if self.const is not None and o.const is not None:
            return Flag(self.g, None, self.const != o.const)
        if self.const is not None:
            return ~o if self.const else o
        if o.const is not None:
            return ~self if o.const else self
        return self.g.fop("xor", self, o)

    def __invert__(self) -> "Flag":
        if self.const is not None:
            return Flag(self.g, None, not self.const)
        return self.g.fop("not", self, None)


def _parts(x):
    if isinstance(x, tuple):
        return list(x)
    return [getattr(x, s) for s in type(x).__slots__]


def _rebuild(x, parts):
    if isinstance(x, tuple):
        return tuple(parts)
    return type(x)(*parts)


def select_n(cases, default):
    """First case (flag, value) whose flag is set, else default, on Fp or
    structure-wise on tuples / tower elements / points (classes whose
    __slots__ are their constructor arguments)."""
    if isinstance(default, Fp):
        return default.g.select_n(list(cases), default)
    dp = _parts(default)
    cps = [(f, _parts(v)) for f, v in cases]
    return _rebuild(default, [select_n([(f, vp[i]) for f, vp in cps], dp[i]) for i in range(len(dp))])


def select(flag: Flag, a, b):
    """flag ? a : b (structure-wise)"""
    return select_n([(flag, a)], b)
