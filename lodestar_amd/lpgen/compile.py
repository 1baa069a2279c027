"""Round programs: scheduling, register allocation, encoding, CPU execution.

``compile_graph(g, rows)`` turns a ``dsl.Graph`` into an ``Program``:
  * dead nodes (not reaching an output) are dropped;
  * units are list-scheduled into rounds of at most ``rows`` units (one per
    16-lane row of the workgroup), longest remaining path first;
  * Fp values get LDS registers (a register is reused only by a value defined
    in a LATER round than the old value's last read: within a round every unit
    reads the state left by the previous round);
  * the program is encoded as 32-bit words for the device interpreter
    (csrc/k_lp.hip, record format below).

``Program.run(inputs, flags)`` executes the encoded words with Python
integers exactly as the device does (the same reduction quotient, the same
Montgomery products), checking every value bound on the way: the CPU tests run
every program against the oracle through this executor, and the GPU tests
compare the device's outputs with it bit for bit.

Encoding (u32 words), one program:
  header: MAGIC, n_rounds, n_regs, n_flags, n_const, n_in, n_inflag, n_out, n_outflag, stream_words
  consts: n_const x (reg, 12 limbs)        in: n_in x reg        inflag: n_inflag x flag
  out: n_out x reg                          outflag: n_outflag x flag
  stream: the rounds' blocks back to back, each a multiple of 4 words:
          block r = [block words, n_units, 0, 0] + n_units fixed records of 20 words
          + extended records; the device streams it through an LDS ring far ahead
          of the round it executes and loads round r+1's records into registers
          during round r
fixed record (20 words):
  w0 = op | nx << 4 | ny << 9 | negx << 14 | negy << 15 | redx << 16 | redy << 17 | ext << 18 | dst << 19
  w1 = Kx | Ky << 16
  w2 = SEL: the flag (x if set, else y); FOP: fop | f1 << 3 | f2 << 16; ext: offset of the
       extended record from the block start
  w3..w10: up to 8 x terms, w11..w18: up to 8 y terms (reg | coef << 16, coef int16); w19 = 0
  (op, nx, terms) of MUL x*y, LIN x, INV / CANON / predicates on x
extended record (forms over 8 terms, selects of more than two cases):
  e0 = op | nops << 4 | nflags << 7 | dst << 16, [nflags flags],
  per operand: nterms | red << 8 | neg << 9 | K << 16, then the terms
"""
from __future__ import annotations

import heapq
from typing import Dict, List

from .dsl import B383, FLAG_KINDS, LIMIT, LIN_REDUCE, P, R, Graph

MAGIC = 0x4C500004
HDR_WORDS = 10
INLINE_TERMS = 16
REC_WORDS = 4 + 2 * INLINE_TERMS  # w0, K, aux, x terms, y terms, pad
OP_MUL, OP_LIN, OP_SEL, OP_INV, OP_CANON, OP_ISZERO, OP_BIT0, OP_GTHALF, OP_FOP, OP_LIN2 = range(10)
# OP_LIN2: a linear unit whose form fills both term lists of the fixed record (x: the first
# INLINE_TERMS terms, y: the rest; value = their sum), so forms of up to 2 INLINE_TERMS terms stay inline
FOPS = {"and": 0, "or": 1, "xor": 2, "not": 3, "const": 4}
KIND_OP = {"mul": OP_MUL, "lin": OP_LIN, "sel": OP_SEL, "inv": OP_INV, "canon": OP_CANON, "iszero": OP_ISZERO,
           "bit0": OP_BIT0, "gthalf": OP_GTHALF, "fop": OP_FOP}
FREE = ("in", "const", "inflag")
_KIND_RANK = {"mul": 0, "lin": 1, "sel": 2, "canon": 3, "iszero": 4, "bit0": 4, "gthalf": 4, "inv": 5, "fop": 6}
INV_WEIGHT = 80        # an inversion unit (one-lane binary GCD) costs ~ this many rounds
BLOCK_CAP = 1536       # words of one round's block (bls_lp.h LB_LP_BLOCK_CAP)
NINV_D = (1.0 / 436277739.0) * (1.0 - 2.0 ** -40)   # bls_coop.h reduce()
PINV = (-pow(P, -1, R)) % R
LIMB_MASK = (1 << 32) - 1


def _operands(kind, args):
    if kind in ("mul",):
        return [args[0], args[1]]
    if kind in ("lin", "inv", "canon", "iszero", "bit0", "gthalf"):
        return [args[0]]
    if kind == "sel":
        return list(args[1])
    return []


def _preds(g: Graph, n: int):
    k = g.kind[n]
    a = g.args[n]
    ps = set()
    for op in _operands(k, a):
        for m, _ in op:
            ps.add(m)
    if k == "sel":
        ps.update(a[0])
    elif k == "fop":
        if a[0] != "const":
            ps.add(a[1])
            if a[2] is not None:
                ps.add(a[2])
    return ps


class Program:
    def __init__(self, name, words, n_rounds, n_units, in_names, inflag_names, out_names, outflag_names, stats):
        self.name = name
        self.words = words
        self.n_rounds = n_rounds
        self.n_units = n_units
        self.in_names = in_names
        self.inflag_names = inflag_names
        self.out_names = out_names
        self.outflag_names = outflag_names
        self.stats = stats

    # ------------------------------------------------------------------
    def run(self, inputs: List[int], flags: List[int], trace=None):
        """Execute the encoded program; inputs as the program declares them
        (canonical Montgomery R = 2^384, or this domain for input_raw)."""
        w = self.words
        assert w[0] == MAGIC
        n_rounds, n_regs, n_flags, n_const, n_in, n_inflag, n_out, n_outflag, sw = w[1:HDR_WORDS]
        pos = HDR_WORDS
        reg = [None] * n_regs
        flg = [None] * n_flags
        for _ in range(n_const):
            r = w[pos]
            v = 0
            for j in range(13):
                v |= w[pos + 1 + j] << (32 * j)
            reg[r] = v
            pos += 14
        assert len(inputs) == n_in and len(flags) == n_inflag
        for i in range(n_in):
            assert 0 <= inputs[i] < B383
            reg[w[pos + i]] = inputs[i]
        pos += n_in
        for i in range(n_inflag):
            flg[w[pos + i]] = 1 if flags[i] else 0
        pos += n_inflag
        outs = w[pos:pos + n_out]
        pos += n_out
        outfl = w[pos:pos + n_outflag]
        pos += n_outflag
        pos = (pos + 3) & ~3
        assert pos + sw == len(w)
        boff = pos
        for r in range(n_rounds):
            bwords, nu = w[boff], w[boff + 1]
            writes = [self._unit(w, boff, boff + 4 + REC_WORDS * u, reg, flg) for u in range(nu)]
            boff += bwords
            for kind, idx, val in writes:
                if kind == 0:
                    reg[idx] = val
                else:
                    flg[idx] = val
            if trace is not None:
                trace.append(writes)
        assert boff == len(w)
        return [reg[r] for r in outs], [flg[f] for f in outfl]

    @staticmethod
    def _sum(terms, K, red, reg):
        T = K * P
        for x in terms:
            c = x >> 16
            if c >= 1 << 15:
                c -= 1 << 16
            v = reg[x & 0xFFFF]
            assert v is not None, "read of an undefined register"
            T += c * v
        assert 0 <= T < LIMIT, "form out of range"
        if red:
            q = int(float(T >> 352) * NINV_D)
            T -= q * P
            assert 0 <= T < 11 * P // 10
        return T

    def _unit(self, w, boff, o, reg, flg):
        w0 = w[o]
        op = w0 & 15
        dst = w0 >> 19
        if op == OP_FOP:
            x = w[o + 2]
            fop, f1, f2 = x & 7, (x >> 3) & 0x1FFF, x >> 16
            a = flg[f1] if fop != 4 else None
            v = (a & flg[f2] if fop == 0 else a | flg[f2] if fop == 1 else a ^ flg[f2] if fop == 2
                 else 1 - a if fop == 3 else f1 & 1)
            return (1, dst, v)
        if (w0 >> 18) & 1:
            return self._ext_unit(w, boff + w[o + 2], reg, flg)
        nx, ny = (w0 >> 4) & 31, (w0 >> 9) & 31
        redx, redy = (w0 >> 16) & 1, (w0 >> 17) & 1
        Kx, Ky = w[o + 1] & 0xFFFF, w[o + 1] >> 16
        xt = w[o + 3:o + 3 + nx]
        yt = w[o + 3 + INLINE_TERMS:o + 3 + INLINE_TERMS + ny]
        if op == OP_LIN2:
            return self._single(OP_LIN, dst, self._sum(xt + yt, Kx, redx, reg))
        if op == OP_SEL:
            if flg[w[o + 2]]:
                return (0, dst, self._sum(xt, Kx, redx, reg))
            return (0, dst, self._sum(yt, Ky, redy, reg))
        x = self._sum(xt, Kx, redx, reg)
        if op == OP_MUL:
            return (0, dst, _mont(x, self._sum(yt, Ky, redy, reg)))
        return self._single(op, dst, x)

    def _ext_unit(self, w, o, reg, flg):
        w0 = w[o]
        op, nops, nfl, dst = w0 & 15, (w0 >> 4) & 7, (w0 >> 7) & 7, w0 >> 16
        o += 1
        fls = [w[o + i] for i in range(nfl)]
        o += nfl
        forms = []
        for _ in range(nops):
            h = w[o]
            nt = h & 255
            forms.append((w[o + 1:o + 1 + nt], h >> 16, (h >> 8) & 1))
            o += 1 + nt
        if op == OP_SEL:
            choice = nops - 1
            for i, f in enumerate(fls):
                if flg[f]:
                    choice = i
                    break
            t, K, red = forms[choice]
            return (0, dst, self._sum(t, K, red, reg))
        vals = [self._sum(t, K, red, reg) for t, K, red in forms]
        if op == OP_MUL:
            return (0, dst, _mont(vals[0], vals[1]))
        return self._single(op, dst, vals[0])

    @staticmethod
    def _single(op, dst, x):
        if op == OP_LIN:
            assert x < (1 << 400)
            return (0, dst, x)
        c = x % P
        if op == OP_CANON:
            return (0, dst, c)
        if op == OP_INV:
            return (0, dst, (pow(c, P - 2, P) * R * R) % P if c else 0)
        if op == OP_ISZERO:
            return (1, dst, int(c == 0))
        if op == OP_BIT0:
            return (1, dst, c & 1)
        if op == OP_GTHALF:
            return (1, dst, int(c > (P - 1) // 2))
        raise ValueError(op)


def _mont(x, y):
    """13-step CIOS over a row: (x y + m p) / 2^416, m = -x y p^-1 mod 2^416"""
    t = x * y
    m = (t * PINV) % R
    v = (t + m * P) >> 416
    assert v < B383, "product >= 2^383"
    return v


# ---------------------------------------------------------------------------
def compile_graph(g: Graph, rows: int = 64) -> Program:
    N = len(g.kind)
    roots = [n for _, n in g.outs] + [n for _, n in g.outflags]
    live = [False] * N
    stack = list(roots)
    while stack:
        n = stack.pop()
        if live[n]:
            continue
        live[n] = True
        stack.extend(_preds(g, n))
    succ: Dict[int, list] = {n: [] for n in range(N) if live[n]}
    npred = {}
    for n in range(N):
        if not live[n]:
            continue
        ps = [m for m in _preds(g, n) if g.kind[m] not in FREE]
        npred[n] = len(ps)
        for m in ps:
            succ[m].append(n)
    # longest remaining path (rounds), inversions weighted
    height = [0] * N
    for n in range(N - 1, -1, -1):
        if not live[n] or g.kind[n] in FREE:
            continue
        h = 0
        for s in succ[n]:
            h = max(h, height[s])
        height[n] = h + (INV_WEIGHT if g.kind[n] == "inv" else 1)
    units = [n for n in range(N) if live[n] and g.kind[n] not in FREE]
    heap = [(-height[n], n) for n in units if npred[n] == 0]
    heapq.heapify(heap)
    rounds: List[list] = []
    rnd = [-1] * N
    pending = {n: npred[n] for n in units}
    def est_words(n):
        """the unit's words in its round block (fixed record + extended record)"""
        k = g.kind[n]
        ops = _operands(k, g.args[n])
        nfl = len(g.args[n][0]) if k == "sel" else 0
        if len(ops) <= 2 and nfl <= 1 and all(len(op) <= INLINE_TERMS for op in ops) and \
                (k != "sel" or len(ops) == 2):
            return REC_WORDS
        if k == "lin" and len(ops) == 1 and len(ops[0]) <= 2 * INLINE_TERMS:
            return REC_WORDS
        return REC_WORDS + 1 + nfl + sum(1 + len(op) for op in ops)

    while heap:
        cur = []
        deferred = []
        used = 4
        while heap and len(cur) < rows:
            item = heapq.heappop(heap)
            w = est_words(item[1])
            if used + w + 3 > BLOCK_CAP:  # (+3: the block's alignment)
                deferred.append(item)
                if len(deferred) > 4 * rows:
                    break
                continue
            used += w
            cur.append(item[1])
        assert cur, "a unit larger than a round block"
        # rows in kind order: a wave holds 4 consecutive rows, so a round's MUL units share
        # their waves and the rarer kinds (LIN, SEL, predicates, extended records) theirs,
        # instead of every wave running several code paths one after the other
        cur.sort(key=lambda m: (_KIND_RANK.get(g.kind[m], 9), est_words(m) > REC_WORDS))
        r = len(rounds)
        for n in cur:
            rnd[n] = r
        rounds.append(cur)
        nxt = []
        for n in cur:
            for s in succ[n]:
                pending[s] -= 1
                if pending[s] == 0:
                    nxt.append(s)
        for s in nxt:
            heapq.heappush(heap, (-height[s], s))
        for d in deferred:
            heapq.heappush(heap, d)
    assert all(rnd[n] >= 0 for n in units), "unscheduled units (cycle?)"
    n_rounds = len(rounds)
    # last read round of every value
    last = [-1] * N
    for n in units:
        for m in _preds(g, n):
            last[m] = max(last[m], rnd[n])
    for n in roots:
        last[n] = n_rounds
    # registers: constants and inputs fixed, the rest by linear scan
    is_flag = [g.kind[n] in FLAG_KINDS for n in range(N)]
    reg = [-1] * N
    const_nodes = [n for n in range(N) if live[n] and g.kind[n] == "const"]
    in_nodes = sorted((g.args[n][0], n) for n in range(N) if g.kind[n] == "in")
    inflag_nodes = sorted((g.args[n][0], n) for n in range(N) if g.kind[n] == "inflag")
    nreg = 0
    for n in const_nodes:
        reg[n] = nreg
        nreg += 1
    for _, n in in_nodes:
        reg[n] = nreg
        nreg += 1
    nflag = 0
    for _, n in inflag_nodes:
        reg[n] = nflag
        nflag += 1
    free_r: list = []
    free_f: list = []
    expire: Dict[int, list] = {}
    hw_r, hw_f = nreg, nflag
    for r, cur in enumerate(rounds):
        for n in expire.pop(r, []):
            (free_f if is_flag[n] else free_r).append(n)
        for n in cur:
            if is_flag[n]:
                if free_f:
                    reg[n] = reg[free_f.pop()]
                else:
                    reg[n] = hw_f
                    hw_f += 1
            else:
                if free_r:
                    reg[n] = reg[free_r.pop()]
                else:
                    reg[n] = hw_r
                    hw_r += 1
            # free for definitions from round last + 1 on
            expire.setdefault(max(last[n], r) + 1, []).append(n)
    assert hw_r < 65536 and hw_f < 4096
    # encode
    words = [MAGIC, n_rounds, hw_r, hw_f, len(const_nodes), len(in_nodes), len(inflag_nodes), len(g.outs),
             len(g.outflags), 0]
    for n in const_nodes:
        v = g.args[n][0]
        words += [reg[n]] + [(v >> (32 * j)) & LIMB_MASK for j in range(13)]
    words += [reg[n] for _, n in in_nodes]
    words += [reg[n] for _, n in inflag_nodes]
    words += [reg[n] for _, n in g.outs]
    words += [reg[n] for _, n in g.outflags]
    words += [0] * (-len(words) % 4)  # the stream starts 16-byte aligned (the device loads it 16 B at a time)
    stream0 = len(words)
    max_terms = 0
    max_block = 0
    for r, cur in enumerate(rounds):
        recs = []
        for n in cur:
            rec = _encode_unit(g, n, reg)
            max_terms = max(max_terms, max([0] + [len(op) for op in _operands(g.kind[n], g.args[n])]))
            recs.append(rec)
        boff = len(words)
        fixed = []
        ext = []
        o = 4 + REC_WORDS * len(cur)
        for rec in recs:
            if isinstance(rec, tuple):  # (fixed record with an ext placeholder, ext record)
                fx, ex = rec
                fx = list(fx)
                fx[2] = o
                fixed += fx
                ext += ex
                o += len(ex)
            else:
                fixed += rec
        o = (o + 3) & ~3
        words += [o, len(cur), 0, 0] + fixed + ext
        words += [0] * (boff + o - len(words))
        assert len(words) - boff == o <= BLOCK_CAP, "round block too large"
        max_block = max(max_block, o)
    words[9] = len(words) - stream0
    kinds = {}
    for n in units:
        kinds[g.kind[n]] = kinds.get(g.kind[n], 0) + 1
    stats = {"rounds": n_rounds, "units": len(units), "regs": hw_r, "flags": hw_f, "words": len(words),
             "kinds": kinds, "max_terms": max_terms, "max_block": max_block,
             "inv_rounds": sum(1 for cur in rounds if any(g.kind[n] == "inv" for n in cur)),
             "mul_rounds": sum(1 for cur in rounds if any(g.kind[n] == "mul" for n in cur))}
    prog = Program(g.name, words, n_rounds, len(units), list(g.in_names), list(g.inflag_names),
                   [nm for nm, _ in g.outs], [nm for nm, _ in g.outflags], stats)
    prog.node_round = rnd  # round of every node (-1: free or dead), for schedule analysis
    return prog


def _form_info(g: Graph, op, red_unit=None):
    """(terms, K, red, neg) of an operand form; red_unit: the unit's explicit
    decision (products), else reduce above LIN_REDUCE"""
    t = dict(op)
    if not t:
        return [], 0, 0, 0
    worst, K = g.form_stats(t)
    assert worst < LIMIT and K < 65536
    red = red_unit if red_unit is not None else (1 if worst > LIN_REDUCE else 0)
    terms = []
    for m, c in op:
        assert -32768 <= c < 32768 and g.kind[m] not in FLAG_KINDS
        terms.append((m, c))
    return terms, K, red, 1 if K else 0


def _term_words(terms, reg):
    return [reg[m] | (c & 0xFFFF) << 16 for m, c in terms]


def _encode_unit(g: Graph, n: int, reg):
    k = g.kind[n]
    a = g.args[n]
    op = KIND_OP[k]
    dst = reg[n]
    assert dst < 8192
    if k == "fop":
        fop, f1, f2 = a
        if fop == "const":
            x = FOPS["const"] | (f1 & 1) << 3
        else:
            x = FOPS[fop] | reg[f1] << 3 | (reg[f2] if f2 is not None else 0) << 16
        return [op | dst << 19, 0, x] + [0] * (REC_WORDS - 3)
    if k == "mul":
        forms = [_form_info(g, a[0], a[2]), _form_info(g, a[1], a[3])]
        flags = []
    elif k == "sel":
        forms = [_form_info(g, o) for o in a[1]]
        flags = list(a[0])
    else:
        forms = [_form_info(g, a[0], 0 if k in ("inv", "canon", "iszero", "bit0", "gthalf") else None)]
        flags = []
    if k == "lin" and INLINE_TERMS < len(forms[0][0]) <= 2 * INLINE_TERMS:
        terms, K, red, neg = forms[0]
        xt = _term_words(terms[:INLINE_TERMS], reg)
        yt = _term_words(terms[INLINE_TERMS:], reg)
        w0 = OP_LIN2 | len(xt) << 4 | len(yt) << 9 | neg << 14 | red << 16 | dst << 19
        return [w0, K, 0] + xt + yt + [0] * (INLINE_TERMS - len(yt)) + [0]
    inline = len(forms) <= 2 and len(flags) <= 1 and all(len(f[0]) <= INLINE_TERMS for f in forms) and \
        (k != "sel" or len(forms) == 2)
    if inline:
        fx = forms[0]
        fy = forms[1] if len(forms) > 1 else ([], 0, 0, 0)
        w0 = op | len(fx[0]) << 4 | len(fy[0]) << 9 | fx[3] << 14 | fy[3] << 15 | fx[2] << 16 | fy[2] << 17 | dst << 19
        xt = _term_words(fx[0], reg)
        yt = _term_words(fy[0], reg)
        aux = reg[flags[0]] if flags else 0
        return [w0, fx[1] | fy[1] << 16, aux] + xt + [0] * (INLINE_TERMS - len(xt)) + yt + \
            [0] * (INLINE_TERMS - len(yt)) + [0]
    # extended record
    assert len(forms) < 8 and len(flags) < 8
    ex = [op | len(forms) << 4 | len(flags) << 7 | dst << 16] + [reg[f] for f in flags]
    for terms, K, red, neg in forms:
        assert len(terms) < 256
        ex += [len(terms) | red << 8 | neg << 9 | K << 16] + _term_words(terms, reg)
    fixed = [op | 1 << 18 | dst << 19, 0, 0] + [0] * (REC_WORDS - 3)
    return (fixed, ex)
