#!/usr/bin/env python3
"""Generate bls_fp_ps.h: straight-line product-scanning (FIPS) Montgomery
multiplication and squaring for the BLS12-381 base field on gfx950.

Why: the compiler's lowering of the CIOS loop in C spends ~640 v_mov_b32 and
~250 v_lshl_add_u64 around the 288 v_mad_u64_u32 of one product, because
v_mad_u64_u32's 64-bit destination may not overlap its 64-bit addend (so the
accumulator is copied around every multiply-add).  Here every column of the
product is a 96-bit accumulator (H:A) fed by v_mad_u64_u32 whose carry-out
goes to an SGPR pair and is folded into H by v_addc_co_u32; two products per
asm statement ping-pong the accumulator between two VGPR pairs, so there are
no copies, and the second product fills the one wait state the carry read
needs (VALU SGPR write -> VALU carry read).

Algorithm (Koc, Acar, Kaliski 1996, "FIPS" = finely integrated product
scanning), radix 2^32, n = 12 limbs, R = 2^384, p < 2^381 so a, b < p gives
r < 2p and one conditional subtraction.

Usage: python gen_fp_asm.py OUT.h
"""
import sys

N = 12


def mad_pair(x1, y1, t1, x2, y2, t2):
    """Two products x1*y1, x2*y2 added into (H:A).  t = 'v' or 's' operand kind for y."""
    return (f"  LB_PS_MAD2_{t1.upper()}{t2.upper()}(A, H, {x1}, {y1}, {x2}, {y2});\n")


def mad_one(x, y, t):
    return f"  LB_PS_MAD1_{t.upper()}(A, H, {x}, {y});\n"


def emit_column(prods, acc="A", hi="H"):
    """ONE asm statement for all products of a column: n v_mad_u64_u32 into the
    96-bit accumulator (hi:acc), each carry-out folded into hi by a
    v_addc_co_u32 issued one instruction later (the VALU-SGPR-write ->
    carry-read wait state is filled by the next product or carry), the 64-bit
    accumulator ping-ponging between acc and a temporary.  One statement per
    column instead of one per two products: the compiler's hazard recognizer
    pads every inline-asm boundary with an s_nop, ~140 of them per product."""
    n = len(prods)
    if n == 0:
        return ""
    ins, lines = [], []
    for i, (x, y, t) in enumerate(prods):
        ins.append(f'[x{i}] "v"({x})')
        ins.append(f'[y{i}] "{t}"({y})')
    for i in range(n):
        dst, add = ("t", "a") if i % 2 == 0 else ("a", "t")
        lines.append(f"v_mad_u64_u32 %[{dst}], %[c{i % 2}], %[x{i}], %[y{i}], %[{add}]")
        if i >= 1:
            lines.append(f"v_addc_co_u32_e64 %[h], %[c{(i - 1) % 2}], 0, %[h], %[c{(i - 1) % 2}]")
    if n == 1:
        lines.append("s_nop 0")
    lines.append(f"v_addc_co_u32_e64 %[h], %[c{(n - 1) % 2}], 0, %[h], %[c{(n - 1) % 2}]")
    body = "\\n\\t".join(lines)
    out = "  {\n    uint64_t T_, c0_, c1_;\n"
    out += f'    asm("{body}"\n'
    out += f'        : [a] "+v"({acc}), [h] "+v"({hi}), [t] "=&v"(T_), [c0] "=&s"(c0_), [c1] "=&s"(c1_)\n'
    out += f'        : {", ".join(ins)});\n'
    if n % 2 == 1:
        out += f"    {acc} = T_;\n"
    out += "  }\n"
    return out


def emit_products(prods):
    out = ""
    i = 0
    while i + 1 < len(prods):
        (x1, y1, t1), (x2, y2, t2) = prods[i], prods[i + 1]
        # keep the VV / VS / SS macro set small: order each pair as (v, s)
        if t1 == "s" and t2 == "v":
            (x1, y1, t1), (x2, y2, t2) = (x2, y2, t2), (x1, y1, t1)
        out += mad_pair(x1, y1, t1, x2, y2, t2)
        i += 2
    if i < len(prods):
        x, y, t = prods[i]
        out += mad_one(x, y, t)
    return out


def gen_mul():
    s = "// r = a b R^-1 mod p (a, b < p): FIPS product scanning, 288 v_mad_u64_u32\n"
    s += "LB_DEV void fp_mul_ps_body(fp& r, const fp& a, const fp& b) {\n"
    s += "  uint64_t A = 0;\n  uint32_t H = 0;\n"
    s += "  uint32_t " + ", ".join(f"m{j}" for j in range(N)) + ";\n"
    s += "  uint32_t t[12];\n"
    for k in range(2 * N - 1):
        lo, hi = max(0, k - N + 1), min(k, N - 1)
        prods = [(f"a.l[{j}]", f"b.l[{k - j}]", "v") for j in range(lo, hi + 1)]
        if k < N:
            prods += [(f"m{j}", f"LB_PS_P{k - j}", "s") for j in range(lo, k)]
            s += emit_column(prods)
            s += f"  m{k} = (uint32_t)A * (uint32_t)LB_P_INV32;\n"
            s += emit_column([(f"m{k}", "LB_PS_P0", "s")])
        else:
            prods += [(f"m{j}", f"LB_PS_P{k - j}", "s") for j in range(lo, hi + 1)]
            s += emit_column(prods)
            s += f"  t[{k - N}] = (uint32_t)A;\n"
        s += "  A = (A >> 32) | ((uint64_t)H << 32);\n  H = 0;\n"
    s += "  t[11] = (uint32_t)A;\n"
    s += "  fp_csub_p(r, t);\n}\n\n"
    return s


def gen_sqr():
    """Squaring: per column the cross products a_i a_j (i < j) go to a second
    accumulator (G:C) which is added twice; squares and m p products go to (H:A)."""
    s = "// r = a^2 R^-1 mod p (a < p): 66 cross + 12 square + 144 reduction v_mad_u64_u32\n"
    s += "LB_DEV void fp_sqr_ps_body(fp& r, const fp& a) {\n"
    s += "  uint64_t A = 0, C;\n  uint32_t H = 0, G;\n"
    s += "  uint32_t " + ", ".join(f"m{j}" for j in range(N)) + ";\n"
    s += "  uint32_t t[12];\n"
    for k in range(2 * N - 1):
        lo, hi = max(0, k - N + 1), min(k, N - 1)
        cross = [(f"a.l[{i}]", f"a.l[{k - i}]", "v") for i in range(lo, hi + 1) if i < k - i]
        prods = []
        if k % 2 == 0:
            prods.append((f"a.l[{k // 2}]", f"a.l[{k // 2}]", "v"))
        if k < N:
            prods += [(f"m{j}", f"LB_PS_P{k - j}", "s") for j in range(lo, k)]
        else:
            prods += [(f"m{j}", f"LB_PS_P{k - j}", "s") for j in range(lo, hi + 1)]
        if len(cross) == 1:
            # a lone cross product: add it twice to the main accumulator
            prods = cross + cross + prods
        elif cross:
            s += "  C = 0;\n  G = 0;\n"
            s += emit_column(cross, acc="C", hi="G")
            s += "  LB_PS_ADD96(A, H, C, G);\n  LB_PS_ADD96(A, H, C, G);\n"
        s += emit_column(prods)
        if k < N:
            s += f"  m{k} = (uint32_t)A * (uint32_t)LB_P_INV32;\n"
            s += emit_column([(f"m{k}", "LB_PS_P0", "s")])
        else:
            s += f"  t[{k - N}] = (uint32_t)A;\n"
        s += "  A = (A >> 32) | ((uint64_t)H << 32);\n  H = 0;\n"
    s += "  t[11] = (uint32_t)A;\n"
    s += "  fp_csub_p(r, t);\n}\n\n"
    return s


# ---- modular additions: interleaved carry chains ---------------------------
# A VALU carry (SGPR lane mask) written by one v_add/v_sub *_co instruction
# needs two wait states before the next carry-chain instruction reads it; the
# compiler's lowering of a 12-limb chain therefore pads every step with
# s_nop 1 (~3,600 s_nop per Fp12 squaring).  Here the four chains of an Fp2
# addition or subtraction -- (c0, c1) x (sum, reduction) -- are interleaved so
# that every carry is read four instructions after it is written: no s_nop.
#   add: t = a + b; s = t - p (borrow = t < p); r = borrow ? t : s
#   sub: t = a - b (borrow = a < b); u = t + p; r = borrow ? u : t
# (a + b < 2p < 2^382: no carry out of the top limb.)

ADD_I = ("v_add_co_u32_e64", "v_addc_co_u32_e64")
SUB_I = ("v_sub_co_u32_e64", "v_subb_co_u32_e64")


def gen_addsub(name, op, nc):
    """r = a op b mod p over nc = 1 (fp) or 2 (fp2) coefficients; op is 'add',
    'sub', or a tuple of one of them per coefficient (e.g. multiply by xi)."""
    ops = (op,) * nc if isinstance(op, str) else tuple(op)
    L = []

    def chain1(c, j):  # r_c[j] = r_c[j] op b_c[j]   (carry k1_c)
        first, nxt = ADD_I if ops[c] == "add" else SUB_I
        if j == 0:
            return f"{first} %[r{c}_{j}], %[k1{c}], %[r{c}_{j}], %[b{c}_{j}]"
        return f"{nxt} %[r{c}_{j}], %[k1{c}], %[r{c}_{j}], %[b{c}_{j}], %[k1{c}]"

    def chain2(c, j):  # x_c[j] = r_c[j] -/+ p[j]   (carry k2_c)
        first, nxt = SUB_I if ops[c] == "add" else ADD_I
        if j == 0:
            return f"{first} %[x{c}_{j}], %[k2{c}], %[r{c}_{j}], %[p{j}]"
        return f"{nxt} %[x{c}_{j}], %[k2{c}], %[r{c}_{j}], %[p{j}], %[k2{c}]"
    for j in range(13):
        if j < 12:
            L += [chain1(c, j) for c in range(nc)]
        if j == 12:
            L.append("s_nop 0")  # the last step has no chain-1 instructions
        if j >= 1:
            L += [chain2(c, j - 1) for c in range(nc)]
        # pad to the two wait states where fewer than two instructions separate
        # a carry from its reader: the first step, and every step of a lone Fp
        if j == 0:
            L.append("s_nop 1" if nc == 1 else "s_nop 0")
        elif nc == 1 and j < 12:
            L.append("s_nop 0")
    L.append("s_nop 1")
    for c in range(nc):
        for j in range(12):
            if ops[c] == "add":  # keep t when t - p borrowed
                L.append(f"v_cndmask_b32_e64 %[r{c}_{j}], %[x{c}_{j}], %[r{c}_{j}], %[k2{c}]")
            else:            # take t + p when a - b borrowed
                L.append(f"v_cndmask_b32_e64 %[r{c}_{j}], %[r{c}_{j}], %[x{c}_{j}], %[k1{c}]")
    body = "\\n\\t".join(L)
    T = "fp2" if nc == 2 else "fp"
    acc = (lambda c: f"t.c{c}") if nc == 2 else (lambda c: "t")
    bcc = (lambda c: f"b.c{c}") if nc == 2 else (lambda c: "b")
    outs = [f'[r{c}_{j}] "+&v"({acc(c)}.l[{j}])' for c in range(nc) for j in range(12)]
    outs += [f'[x{c}_{j}] "=&v"(x{c}[{j}])' for c in range(nc) for j in range(12)]
    outs += [f'[k1{c}] "=&s"(k1{c})' for c in range(nc)] + [f'[k2{c}] "=&s"(k2{c})' for c in range(nc)]
    ins = [f'[b{c}_{j}] "v"({bcc(c)}.l[{j}])' for c in range(nc) for j in range(12)]
    ins += [f'[p{j}] "v"(LB_PS_P{j})' for j in range(12)]
    sym = "".join("+" if o == "add" else "-" for o in ops)
    out = f"// {T} r = a ({sym}) b mod p per coefficient: {2 * nc} interleaved carry chains\n"
    out += f"LB_DEV void {name}({T}& r, const {T}& a, const {T}& b) {{\n"
    out += "  uint32_t " + ", ".join(f"x{c}[12]" for c in range(nc)) + ";\n"
    out += "  uint64_t " + ", ".join(f"k1{c}, k2{c}" for c in range(nc)) + ";\n"
    out += f"  {T} t = a;\n"
    out += f'  asm("{body}"\n      : {", ".join(outs)}\n      : {", ".join(ins)});\n'
    out += "  r = t;\n}\n\n"
    return out


# ---- lazy reduction: double-width products and one Montgomery reduction ----
# An Fp2 product by Karatsuba needs three 12x12-limb products but only TWO
# reductions when the products are kept double width (Aranha et al., "Faster
# explicit formulas for computing pairings over ordinary curves", EUROCRYPT
# 2011): T0 = a0 b0, T1 = a1 b1, T2 = (a0 + a1)(b0 + b1) (plain sums < 2p),
#   W0 = T0 - T1 mod pR  (add p to the upper 12 limbs when it borrows)
#   W1 = T2 - T0 - T1 = a0 b1 + a1 b0 < 2p^2
# and c = REDC(W) < 2p for any W < pR (pR ~ 9.8 p^2), one conditional
# subtraction.  720 v_mad_u64_u32 per Fp2 product instead of 864.

def gen_mulw():
    s = "// w = a b (24 limbs, no reduction; a, b < 2^384): 144 v_mad_u64_u32\n"
    s += "LB_DEV void fp_mulw_ps_body(uint32_t* w, const fp& a, const fp& b) {\n"
    s += "  uint64_t A = 0;\n  uint32_t H = 0;\n"
    for k in range(2 * N - 1):
        lo, hi = max(0, k - N + 1), min(k, N - 1)
        s += emit_column([(f"a.l[{j}]", f"b.l[{k - j}]", "v") for j in range(lo, hi + 1)])
        s += f"  w[{k}] = (uint32_t)A;\n"
        s += "  A = (A >> 32) | ((uint64_t)H << 32);\n  H = 0;\n"
    s += f"  w[{2 * N - 1}] = (uint32_t)A;\n}}\n\n"
    return s


def gen_redc():
    s = "// r = w R^-1 mod p for w < p R (24 limbs): 144 v_mad_u64_u32, one conditional subtraction\n"
    s += "LB_DEV void fp_redc_ps_body(fp& r, const uint32_t* w) {\n"
    s += "  uint64_t A = w[0];\n  uint32_t H = 0;\n"
    s += "  uint32_t " + ", ".join(f"m{j}" for j in range(N)) + ";\n"
    s += "  uint32_t t[12];\n"
    for k in range(2 * N - 1):
        if k < N:
            s += emit_column([(f"m{j}", f"LB_PS_P{k - j}", "s") for j in range(0, k)])
            s += f"  m{k} = (uint32_t)A * (uint32_t)LB_P_INV32;\n"
            s += emit_column([(f"m{k}", "LB_PS_P0", "s")])
        else:
            s += emit_column([(f"m{j}", f"LB_PS_P{k - j}", "s") for j in range(k - N + 1, N)])
            s += f"  t[{k - N}] = (uint32_t)A;\n"
        # the shifted accumulator is < 2^38: adding the next input limb cannot carry out
        s += f"  A = ((A >> 32) | ((uint64_t)H << 32)) + w[{k + 1}];\n  H = 0;\n"
    s += "  t[11] = (uint32_t)A;\n"
    s += "  fp_csub_p(r, t);\n}\n\n"
    return s


class ChainSched:
    """Interleave independent carry chains into one asm body.  A VALU-written
    carry (SGPR lane mask) may be read by a VALU instruction only two
    instructions later: before each reader the scheduler inserts the s_nop the
    gap still needs.  Instructions are (text, reads_carry, writes_carry)."""

    def __init__(self):
        self.lines = []
        self.pos = 0
        self.written = {}

    def emit(self, text, reads=None, writes=None):
        if reads is not None and reads in self.written:
            gap = self.pos - self.written[reads] - 1
            if gap < 2:
                self.lines.append(f"s_nop {1 - gap}")
        self.lines.append(text)
        if writes is not None:
            self.written[writes] = self.pos
        self.pos += 1


def chain_op(op, j, d, c, a, b):
    """Step j of a carry chain: d = a op b (+/- carry c)."""
    first, nxt = ADD_I if op == "add" else SUB_I
    if j == 0:
        return (f"{first} {d}, {c}, {a}, {b}", None, c)
    return (f"{nxt} {d}, {c}, {a}, {b}, {c}", c, c)


def kcombine_program():
    """Karatsuba combine in place: (T0, T1, T2) -> W0 in T0, W1 in T2.
      B: T0[j] = T0[j] - T1[j]             (borrow kb)
      C: T2[j] = T2[j] - T0_old[j]          (kc; runs before B in each round)
      D: T2[j] = T2[j] - T1[j]              (kd; one round behind C)
      E: T1[12+j] = T0[12+j] + p[j]         (ke; after D has read T1[12+j])
      W0[12+j] = kb ? T1[12+j] : T0[12+j]   (add p R when T0 - T1 borrowed)
    Returns the list of asm lines (operands %[t0_j], %[t1_j], %[t2_j], %[p_j],
    SGPR pairs %[kb], %[kc], %[kd], %[ke])."""
    S = ChainSched()
    n = 2 * N
    for r in range(n + 2):
        step = []
        if r < n:
            step.append(chain_op("sub", r, f"%[t2_{r}]", "%[kc]", f"%[t2_{r}]", f"%[t0_{r}]"))
            step.append(chain_op("sub", r, f"%[t0_{r}]", "%[kb]", f"%[t0_{r}]", f"%[t1_{r}]"))
        if 1 <= r <= n:
            j = r - 1
            step.append(chain_op("sub", j, f"%[t2_{j}]", "%[kd]", f"%[t2_{j}]", f"%[t1_{j}]"))
        if r >= N + 2 and r - N - 2 < N:
            j = r - N - 2  # T1[12+j] was last read by D at round 13+j
            step.append(chain_op("add", j, f"%[t1_{N + j}]", "%[ke]", f"%[t0_{N + j}]", f"%[p_{j}]"))
        for text, rd, wr in step:
            S.emit(text, rd, wr)
    for j in range(N):
        S.emit(f"v_cndmask_b32_e64 %[t0_{N + j}], %[t0_{N + j}], %[t1_{N + j}], %[kb]", "%[kb]")
    return S.lines


def gen_kcombine():
    L = kcombine_program()
    body = "\\n\\t".join(L)
    outs = [f'[t{i}_{j}] "+&v"(t{i}[{j}])' for i in range(3) for j in range(2 * N)]
    outs += [f'[k{c}] "=&s"(k{c})' for c in "bcde"]
    ins = [f'[p_{j}] "v"(LB_PS_P{j})' for j in range(N)]
    s = "// Karatsuba combine of three double-width products, in place (see kcombine_program):\n"
    s += "// t0 <- t0 - t1 mod pR, t2 <- t2 - t0 - t1.  t1's upper half is clobbered.\n"
    s += "LB_DEV void fpw_kcombine_ps(uint32_t* t0, uint32_t* t1, uint32_t* t2) {\n"
    s += "  uint64_t kb, kc, kd, ke;\n"
    s += f'  asm("{body}"\n      : {", ".join(outs)}\n      : {", ".join(ins)});\n}}\n\n'
    return s


def plain_add2_program():
    """(s, t) = (a0 + a1, b0 + b1) without reduction (inputs < p, sums < 2^382)."""
    S = ChainSched()
    for j in range(N):
        for x, c in (("s", "%[ks]"), ("t", "%[kt]")):
            text, rd, wr = chain_op("add", j, f"%[{x}{j}]", c, f"%[{x}{j}]", f"%[{x}b{j}]")
            S.emit(text, rd, wr)
    return S.lines


def gen_plain_add2():
    body = "\\n\\t".join(plain_add2_program())
    outs = [f'[{x}{j}] "+&v"({x}.l[{j}])' for x in "st" for j in range(N)]
    outs += ['[ks] "=&s"(ks)', '[kt] "=&s"(kt)']
    ins = [f'[{x}b{j}] "v"({y}.l[{j}])' for x, y in (("s", "a1"), ("t", "b1")) for j in range(N)]
    s = "// (s, t) = (a0 + a1, b0 + b1), no reduction (Karatsuba operands, < 2p)\n"
    s += "LB_DEV void fp_add2_plain_ps(fp& s, fp& t, const fp& a0, const fp& a1, const fp& b0, const fp& b1) {\n"
    s += "  uint64_t ks, kt;\n  s = a0;\n  t = b0;\n"
    s += f'  asm("{body}"\n      : {", ".join(outs)}\n      : {", ".join(ins)});\n}}\n\n'
    return s


HEADER = r'''// GENERATED by gen_fp_asm.py -- do not edit.
//
// Product-scanning Montgomery multiplication / squaring for gfx950: every
// multiply-add is one v_mad_u64_u32 into a 96-bit column accumulator (H:A);
// carries leave through an SGPR pair into H (v_addc_co_u32).  Two products
// per asm statement: the accumulator ping-pongs between two VGPR pairs
// (v_mad_u64_u32's destination must not overlap its addend) and the second
// multiply-add is the wait state before the first carry is read.
#pragma once

#define LB_PS_MAD2_VV(AC_, HI_, X1_, Y1_, X2_, Y2_)                                                        \
  do {                                                                                             \
    uint64_t t_, c1_, c2_;                                                                         \
    asm("v_mad_u64_u32 %[t], %[c1], %[x1], %[y1], %[a]\n\t"                                        \
        "v_mad_u64_u32 %[a], %[c2], %[x2], %[y2], %[t]\n\t"                                        \
        "v_addc_co_u32_e64 %[h], %[c1], 0, %[h], %[c1]\n\t"                                        \
        "v_addc_co_u32_e64 %[h], %[c2], 0, %[h], %[c2]"                                            \
        : [a] "+v"(AC_), [h] "+v"(HI_), [t] "=&v"(t_), [c1] "=&s"(c1_), [c2] "=&s"(c2_)                \
        : [x1] "v"(X1_), [y1] "v"(Y1_), [x2] "v"(X2_), [y2] "v"(Y2_));                                 \
  } while (0)
#define LB_PS_MAD2_VS(AC_, HI_, X1_, Y1_, X2_, Y2_)                                                        \
  do {                                                                                             \
    uint64_t t_, c1_, c2_;                                                                         \
    asm("v_mad_u64_u32 %[t], %[c1], %[x1], %[y1], %[a]\n\t"                                        \
        "v_mad_u64_u32 %[a], %[c2], %[x2], %[y2], %[t]\n\t"                                        \
        "v_addc_co_u32_e64 %[h], %[c1], 0, %[h], %[c1]\n\t"                                        \
        "v_addc_co_u32_e64 %[h], %[c2], 0, %[h], %[c2]"                                            \
        : [a] "+v"(AC_), [h] "+v"(HI_), [t] "=&v"(t_), [c1] "=&s"(c1_), [c2] "=&s"(c2_)                \
        : [x1] "v"(X1_), [y1] "v"(Y1_), [x2] "v"(X2_), [y2] "s"(Y2_));                                 \
  } while (0)
#define LB_PS_MAD2_SS(AC_, HI_, X1_, Y1_, X2_, Y2_)                                                        \
  do {                                                                                             \
    uint64_t t_, c1_, c2_;                                                                         \
    asm("v_mad_u64_u32 %[t], %[c1], %[x1], %[y1], %[a]\n\t"                                        \
        "v_mad_u64_u32 %[a], %[c2], %[x2], %[y2], %[t]\n\t"                                        \
        "v_addc_co_u32_e64 %[h], %[c1], 0, %[h], %[c1]\n\t"                                        \
        "v_addc_co_u32_e64 %[h], %[c2], 0, %[h], %[c2]"                                            \
        : [a] "+v"(AC_), [h] "+v"(HI_), [t] "=&v"(t_), [c1] "=&s"(c1_), [c2] "=&s"(c2_)                \
        : [x1] "v"(X1_), [y1] "s"(Y1_), [x2] "v"(X2_), [y2] "s"(Y2_));                                 \
  } while (0)
#define LB_PS_MAD1_V(AC_, HI_, X_, Y_)                                                                   \
  do {                                                                                             \
    uint64_t t_, c_;                                                                               \
    asm("v_mad_u64_u32 %[t], %[c], %[x], %[y], %[a]\n\t"                                           \
        "s_nop 0\n\t"                                                                              \
        "v_addc_co_u32_e64 %[h], %[c], 0, %[h], %[c]"                                              \
        : [t] "=&v"(t_), [h] "+v"(HI_), [c] "=&s"(c_)                                                \
        : [a] "v"(AC_), [x] "v"(X_), [y] "v"(Y_));                                                     \
    AC_ = t_;                                                                                        \
  } while (0)
#define LB_PS_MAD1_S(AC_, HI_, X_, Y_)                                                                   \
  do {                                                                                             \
    uint64_t t_, c_;                                                                               \
    asm("v_mad_u64_u32 %[t], %[c], %[x], %[y], %[a]\n\t"                                           \
        "s_nop 0\n\t"                                                                              \
        "v_addc_co_u32_e64 %[h], %[c], 0, %[h], %[c]"                                              \
        : [t] "=&v"(t_), [h] "+v"(HI_), [c] "=&s"(c_)                                                \
        : [a] "v"(AC_), [x] "v"(X_), [y] "s"(Y_));                                                     \
    AC_ = t_;                                                                                        \
  } while (0)
// (H:A) += (G:C), 96-bit: 64-bit add, carry = (sum < addend)
#define LB_PS_ADD96(AC_, HI_, C_, G_)                                                                    \
  do {                                                                                             \
    uint64_t t_, c_;                                                                               \
    asm("v_lshl_add_u64 %[t], %[x], 0, %[a]\n\t"                                                  \
        "v_cmp_lt_u64_e64 %[c], %[t], %[x]\n\t"                                                    \
        "s_nop 0\n\t"                                                                              \
        "v_addc_co_u32_e64 %[h], %[c], %[h], %[g], %[c]"                                           \
        : [t] "=&v"(t_), [h] "+v"(HI_), [c] "=&s"(c_)                                                \
        : [a] "v"(AC_), [x] "v"(C_), [g] "v"(G_));                                                     \
    AC_ = t_;                                                                                        \
  } while (0)

'''


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "bls_fp_ps.h"
    consts = "".join(f"#define LB_PS_P{j} ((uint32_t)P_[{j}])\n" for j in range(N))
    with open(out, "w") as f:
        f.write(HEADER + consts + "\n" + gen_mul() + gen_sqr() + gen_addsub("fp_add_ps", "add", 1)
                + gen_addsub("fp_sub_ps", "sub", 1) + gen_addsub("fp2_add_ps", "add", 2)
                + gen_addsub("fp2_sub_ps", "sub", 2)
                + gen_addsub("fp2_subadd_ps", ("sub", "add"), 2)
                + gen_mulw() + gen_redc() + gen_kcombine() + gen_plain_add2())


if __name__ == "__main__":
    main()
