// Row-cooperative Fp arithmetic for the latency path (gfx950).
//
// One Fp element per 16-lane DPP row: lane j of the row holds 32-bit limb j
// (j < 12; lane 12 takes the carry of an unreduced sum, lanes 13-15 stay 0), so
// a wave holds four independent elements and one Montgomery product is 12 CIOS
// steps of two v_mad_u64_u32 per lane instead of 288 serial multiply-adds on
// one lane.  The latency of a product -- not the work -- is what a lone
// verification waits for: a one-lane product is a ~4k-cycle
// dependent chain, this one ~0.7k.
//
// Broadcasts inside a row use DPP row_newbcast, limb shifts row_shl / row_shr.
// Carries across limbs are resolved with carry-lookahead on the wave's ballot
// masks (generate / propagate bits of all four rows at once in one 64-bit
// scalar add), so no step ever walks the 12 limbs serially.
//
// Value invariant of the latency path: every stored element is < 2^383 (about
// 4.9 p), normalized to 32-bit limbs.  A Montgomery product of two such values
// is again < 2^383 (xy/R + p < 2^382 + 2^381), and a linear combination is
// brought back under 2^383 by one quotient estimate from its top 64 bits
// (reduce); predicates canonicalise to [0, p) first (canon).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bls_constants.h"

namespace lb {
namespace co {

#define LB_CO __device__ __forceinline__

static constexpr uint64_t ROW_LANE0 = 0x0001000100010001ull;
static constexpr uint64_t ROW_LANE15 = 0x8000800080008000ull;
static constexpr uint32_t N0 = LB_P_INV32;  // -p^-1 mod 2^32
// DPP controls (gfx9 encoding): row_shl:1 -> lane j reads lane j+1; row_shr:1 -> lane j reads lane j-1
static constexpr int DPP_ROW_SHL1 = 0x101;
static constexpr int DPP_ROW_SHR1 = 0x111;
static constexpr int DPP_ROW_BCAST0 = 0x150;  // row_newbcast:n = 0x150 + n

LB_CO uint32_t lane64() { return __lane_id(); }
LB_CO uint32_t lane16() { return __lane_id() & 15u; }

template <int CTRL>
LB_CO uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int I>
LB_CO uint32_t bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_ROW_BCAST0 + I, 0xF, 0xF, false);
}
LB_CO uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
// bit (lane) of a wave-uniform mask, as 0 / 1
LB_CO uint32_t lanebit(uint64_t m) { return (uint32_t)(m >> lane64()) & 1u; }
// carry INTO each lane from generate / propagate masks (g, p disjoint):
// the carries of the binary sum (g|p) + g; lane 15 of a row never carries out
LB_CO uint64_t lookahead(uint64_t g, uint64_t p) {
  g &= ~ROW_LANE15;
  p &= ~ROW_LANE15;
  const uint64_t a = g | p;
  return (a + g) ^ a ^ g;
}

static constexpr uint32_t P_LIMB[12] = LB_P_LIMBS;
static constexpr uint32_t HALF_P_LIMB[12] = LB_HALF_P_RAW_LIMBS;
// limb j of a 12-limb constant for this lane (0 for lanes >= 12); a chain of
// selects keeps the constant in registers, not in memory
LB_CO uint32_t const_limb(const uint32_t (&c)[12]) {
  const uint32_t j = lane16();
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) r = (j == (uint32_t)k) ? c[k] : r;
  return r;
}
LB_CO uint32_t p_limb() { return const_limb(P_LIMB); }
LB_CO uint32_t halfp_limb() { return const_limb(HALF_P_LIMB); }

// Signed per-limb partials -> 32-bit limbs.  t: this lane's partial (lanes 13-15
// of the row 0); the row's value sum_j t_j 2^(32 j) must be >= 0 and < 2^416.
// NEG: some partials may be negative (a linear form with negative terms, or
// after subtracting q p).  One DPP shift moves each partial's high word (|h| <
// 2^31) up a limb, leaving per-limb carries c in {-1, 0, 1}; a second shift adds
// them.  A carry ripples further only where it meets a limb 0xffffffff (+1) or 0
// (-1): one ballot detects that (probability ~2^-32 per limb on data) and only
// then the carries resolve by lookahead (one pass adds the +1 carries, one
// subtracts the -1 carries) -- the common case has no scalar round trip but the
// one branch.
template <bool NEG>
LB_CO uint32_t norm(int64_t t) {
  const uint32_t lo = (uint32_t)t;
  const int32_t h = (int32_t)(t >> 32);
  const int32_t hs = (int32_t)dpp<DPP_ROW_SHR1>((uint32_t)h);
  const int64_t u = (int64_t)(uint64_t)lo + (int64_t)hs;
  const uint32_t v = (uint32_t)u;
  const int32_t c = (int32_t)(u >> 32);
  const int32_t ci = (int32_t)dpp<DPP_ROW_SHR1>((uint32_t)c);  // carry into this limb (lane 0 of a row: 0)
  const bool ripple = (ci == 1 && v == 0xffffffffu) || (NEG && ci == -1 && v == 0u);
  if (__builtin_expect(ballot(ripple) == 0, 1)) return v + (uint32_t)ci;
  uint32_t r = v;
  {
    const uint32_t x = ci == 1 ? 1u : 0u;
    const uint64_t g = ballot(x && r == 0xffffffffu);
    const uint64_t p = ballot(x ? r == 0xfffffffeu : r == 0xffffffffu);
    r = r + x + lanebit(lookahead(g, p));
  }
  if (NEG) {
    const uint32_t y = ci == -1 ? 1u : 0u;
    const uint64_t g = ballot(y && r == 0u);
    const uint64_t p = ballot(y ? r == 1u : r == 0u);
    r = r - y - lanebit(lookahead(g, p));
  }
  return r;
}

// two normalisations (signed partials) sharing the ripple test
LB_CO void norm2(int64_t tx, int64_t ty, uint32_t& x, uint32_t& y) {
  const int32_t hx = (int32_t)dpp<DPP_ROW_SHR1>((uint32_t)(int32_t)(tx >> 32));
  const int32_t hy = (int32_t)dpp<DPP_ROW_SHR1>((uint32_t)(int32_t)(ty >> 32));
  const int64_t ux = (int64_t)(uint64_t)(uint32_t)tx + (int64_t)hx;
  const int64_t uy = (int64_t)(uint64_t)(uint32_t)ty + (int64_t)hy;
  const uint32_t vx = (uint32_t)ux, vy = (uint32_t)uy;
  const int32_t cx = (int32_t)dpp<DPP_ROW_SHR1>((uint32_t)(int32_t)(ux >> 32));
  const int32_t cy = (int32_t)dpp<DPP_ROW_SHR1>((uint32_t)(int32_t)(uy >> 32));
  const bool ripple = (cx == 1 && vx == 0xffffffffu) || (cx == -1 && vx == 0u) || (cy == 1 && vy == 0xffffffffu) ||
                      (cy == -1 && vy == 0u);
  if (__builtin_expect(ballot(ripple) == 0, 1)) {
    x = vx + (uint32_t)cx;
    y = vy + (uint32_t)cy;
    return;
  }
  x = norm<true>(tx);
  y = norm<true>(ty);
}

template <int I, int N>
struct MontStep {
  LB_CO static void run(uint64_t& acc, uint32_t x, uint32_t y, uint32_t pj) {
    const uint32_t xi = bcast<I>(x);
    const uint64_t P = (uint64_t)xi * y + acc;
    const uint32_t m = bcast<0>((uint32_t)P) * N0;
    const uint64_t Q = (uint64_t)m * pj + (uint32_t)P;
    const uint32_t qs = dpp<DPP_ROW_SHL1>((uint32_t)Q);
    acc = (uint64_t)qs + (Q >> 32) + (P >> 32);
    MontStep<I + 1, N>::run(acc, x, y, pj);
  }
};
template <int N>
struct MontStep<N, N> {
  LB_CO static void run(uint64_t&, uint32_t, uint32_t, uint32_t) {}
};

// x y R^-1 (mod p), R = 2^(32 N), normalized limbs in and out.  CIOS over the
// row: step i broadcasts x_i, every lane j adds x_i y_j, lane 0's low word gives
// m, every lane adds m p_j, and the row shifts down one limb.  A lane's
// accumulator stays < 3 * 2^32 (64-bit), so the carries wait for one lookahead
// at the end.  N = 12 (R = 2^384): x, y < 2^383 -> result < 2^383.  N = 13
// (R = 2^416, the latency path's domain): x, y < 2^415 with x y < 2^416 (2^383 - p)
// -> result < 2^383, so sums of many reduced values multiply unreduced.
template <int N = 12>
LB_CO uint32_t mont_mul(uint32_t x, uint32_t y, uint32_t pj) {
  uint64_t acc = 0;
  MontStep<0, N>::run(acc, x, y, pj);
  return norm<false>((int64_t)acc);
}

// 13-limb constant (R = 2^416 values may use limb 12)
LB_CO uint32_t const_limb13(const uint32_t (&c)[13]) {
  const uint32_t j = lane16();
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 13; k++) r = (j == (uint32_t)k) ? c[k] : r;
  return r;
}

// T (normalized limbs 0..12, T < 2^404) -> T - q p < 2^383 with q = a slight
// underestimate of floor(T / p) from T's top 64 bits (limbs 11, 12): the
// quotient of t = floor(T / 2^352) by p_11 + 1 never overshoots floor(T / p)
// (p < 2^352 (p_11 + 1), and the factor below 1/(p_11+1) absorbs the f64
// rounding) and undershoots T / p by less than 1 + 2^-16, so the result is
// < 1.03 p + 2^376 < 1.1 p: one conditional subtraction makes it canonical.
LB_CO uint32_t reduce(uint32_t v, uint32_t pj) {
  const uint32_t l11 = bcast<11>(v), l12 = bcast<12>(v);
  const double th = (double)l12 * 4294967296.0 + (double)l11;
  // 1 / (p_11 + 1), scaled by (1 - 2^-40) so the product never rounds up
  constexpr double inv_d = (1.0 / 436277739.0) * (1.0 - 0x1p-40);
  const uint32_t q = (uint32_t)(th * inv_d);
  return norm<true>((int64_t)(uint64_t)v - (int64_t)((uint64_t)q * pj));
}

// borrow-lookahead subtraction d = v - m (v, m normalized, lanes 13.. zero);
// returns d and sets `ge` (row-uniform) when v >= m
LB_CO uint32_t sub_cmp(uint32_t v, uint32_t m, bool& ge) {
  const uint64_t b = lookahead(ballot(v < m), ballot(v == m));
  ge = ((b >> ((lane64() & ~15u) + 13u)) & 1u) == 0;  // no borrow into lane 13: v >= m
  return v - m - lanebit(b);
}

// v < 2^383 -> v mod p (canonical)
LB_CO uint32_t canon(uint32_t v, uint32_t pj) {
  v = reduce(v, pj);  // < 1.1 p
  bool ge;
  const uint32_t d = sub_cmp(v, pj, ge);
  return ge ? d : v;
}

// row-uniform predicates on normalized limbs
LB_CO bool row_is_zero(uint32_t v) {
  const uint64_t nz = ballot(v != 0u);
  return ((nz >> (lane64() & ~15u)) & 0xffffull) == 0;
}
// canonical raw value c > (p-1)/2  (the ZCash "lexicographically largest" flag)
LB_CO bool row_gt_half(uint32_t c) {
  bool ge;
  (void)sub_cmp(halfp_limb(), c, ge);  // (p-1)/2 >= c ?
  return !ge;
}
// lowest bit of the row's value
LB_CO uint32_t row_bit0(uint32_t v) { return bcast<0>(v) & 1u; }

// ---- inversion (the latency path's INV unit) --------------------------------
// y^-1 mod p for a raw y in [0, p) held by ONE row of the wave (its lanes 0-11; 0 -> 0),
// by the binary GCD of bls_inv.h (Pornin, ePrint 2020/972, Alg. 2 with k = 31): 25
// rounds of 31 divsteps on 64-bit approximations of (a, b), then the step matrix
// applied to the full a, b, u, v.  Here the divsteps run on scalar registers (the
// approximations are read out of the row: uniform values) and the matrix products
// run across the row (one limb per lane, norm for the carries) -- a one-lane
// inversion's 381-bit limb loops were ~90% of its ~150 us.  base: the row's first
// lane (wave-uniform); lanes of other rows compute on zeros and keep their values.
LB_CO uint32_t row_readlane(uint32_t v, uint32_t lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane); }
// a < b for wave-uniform 64-bit values, on the scalar unit (the borrow of a - b)
LB_CO bool s_lt64(uint64_t a, uint64_t b) {
  uint32_t r, t;
  asm("s_cmp_lt_u32 %2, %4\n\ts_subb_u32 %1, %3, %5\n\ts_cselect_b32 %0, 1, 0"
      : "=s"(r), "=&s"(t)
      : "s"((uint32_t)a), "s"((uint32_t)(a >> 32)), "s"((uint32_t)b), "s"((uint32_t)(b >> 32))
      : "scc");
  return r != 0;
}

// The two new (a, b) = (|x f0 + y g0|, |x f1 + y g1|) / 2^31 for x, y >= 0 (< 2^381)
// and |f| + |g| <= 2^31, with their signs; both at once (shared normalisations).
// t + 2^413 >= 0: the bias (on lane 12, where x, y are 0) keeps the normalised value
// non-negative (|t| < 2^412); a negative t comes back as 2^413 - (t + 2^413).
LB_CO void row_lin_shift2(uint32_t x, uint32_t y, int64_t f0, int64_t g0, int64_t f1, int64_t g1, bool mine,
                          uint32_t base, uint32_t& ra, uint32_t& rb, bool& na, bool& nb) {
  const uint32_t j = lane16();
  const int64_t bias = j == 12 ? (1ll << 29) : 0;
  const int64_t ta = mine ? (int64_t)(uint64_t)x * f0 + (int64_t)(uint64_t)y * g0 + bias : 0;
  const int64_t tb = mine ? (int64_t)(uint64_t)x * f1 + (int64_t)(uint64_t)y * g1 + bias : 0;
  uint32_t va, vb;
  norm2(ta, tb, va, vb);
  na = row_readlane(va, base + 12) < (1u << 29);
  nb = row_readlane(vb, base + 12) < (1u << 29);
  if (na || nb) {
    const int64_t da = mine ? (na ? bias - (int64_t)(uint64_t)va : (int64_t)(uint64_t)va - bias) : 0;
    const int64_t db = mine ? (nb ? bias - (int64_t)(uint64_t)vb : (int64_t)(uint64_t)vb - bias) : 0;
    norm2(da, db, va, vb);
  } else if (j == 12) {
    va -= 1u << 29;
    vb -= 1u << 29;
  }
  const uint32_t ua = dpp<DPP_ROW_SHL1>(va), ub = dpp<DPP_ROW_SHL1>(vb);  // limb j + 1 (lane 15: 0)
  ra = (va >> 31) | (ua << 1);
  rb = (vb >> 31) | (ub << 1);
}

// The two new (u, v) = (u f0 + v g0, u f1 + v g1) / 2^31 mod p for u, v in [0, p),
// |f| + |g| <= 2^31 (canonical results), both at once.  |t| < 2^31 p: t + 2^414
// normalises (the bias on lane 12, where u, v are 0, so no lane's partial leaves
// int64), then the bias becomes 2^32 p (t + 2^32 p > 0, = t mod p after / 2^31), then
// + k p with k = -t p^-1 mod 2^31 makes the sum divisible by 2^31:
// (t + (2^32 + k) p) / 2^31 in (p, 4 p).
LB_CO void row_lin_mod2(uint32_t u, uint32_t v, int64_t f0, int64_t g0, int64_t f1, int64_t g1, bool mine,
                        uint32_t base, uint32_t pj, uint32_t& ru, uint32_t& rv) {
  const uint32_t j = lane16();
  const int64_t bias = j == 12 ? (1ll << 30) : 0;
  const int64_t ta = mine ? (int64_t)(uint64_t)u * f0 + (int64_t)(uint64_t)v * g0 + bias : 0;
  const int64_t tb = mine ? (int64_t)(uint64_t)u * f1 + (int64_t)(uint64_t)v * g1 + bias : 0;
  uint32_t na, nb;
  norm2(ta, tb, na, nb);
  const int64_t pb = (int64_t)(uint64_t)dpp<DPP_ROW_SHR1>(pj) - bias;  // p_{j-1}: the limbs of 2^32 p
  norm2(mine ? (int64_t)(uint64_t)na + pb : 0, mine ? (int64_t)(uint64_t)nb + pb : 0, na, nb);
  const uint32_t ka = (row_readlane(na, base) * N0) & 0x7fffffffu;
  const uint32_t kb = (row_readlane(nb, base) * N0) & 0x7fffffffu;
  norm2(mine ? (int64_t)((uint64_t)na + (uint64_t)ka * pj) : 0, mine ? (int64_t)((uint64_t)nb + (uint64_t)kb * pj) : 0,
        na, nb);
  const uint32_t ua = dpp<DPP_ROW_SHL1>(na), ub = dpp<DPP_ROW_SHL1>(nb);
  ru = canon((na >> 31) | (ua << 1), pj);
  rv = canon((nb >> 31) | (ub << 1), pj);
}

LB_CO uint32_t row_inv_raw(uint32_t y, bool mine, uint32_t base, uint32_t pj) {
  const uint32_t j = lane16();
  uint32_t a = mine ? y : 0u, b = mine ? pj : 0u, u = mine && j == 0 ? 1u : 0u, v = 0u;
#pragma unroll 1
  for (int round = 0; round < 25; round++) {
    // n = bit length of max(a, b) (at least 64); the approximations' words, read out
    const uint64_t nz = ballot((a | b) != 0u) >> base;
    const uint32_t top = (nz & 0xfffull) ? 63u - (uint32_t)__builtin_clzll(nz & 0xfffull) : 0u;
    const uint32_t wt = row_readlane(a | b, base + top);
    int n = wt ? (int)(32 * top + 32 - __builtin_clz(wt)) : 0;
    if (n < 64) n = 64;
    const int s = n - 33, li = s >> 5, sh = s & 31;
    auto approx = [&](uint32_t x) {
      const uint32_t w0 = row_readlane(x, base + li), w1 = row_readlane(x, base + li + 1);
      const uint32_t w2 = li + 2 < 12 ? row_readlane(x, base + li + 2) : 0u;
      const uint64_t lo64 = (uint64_t)w0 | ((uint64_t)w1 << 32);
      uint64_t tp = sh ? ((lo64 >> sh) | ((uint64_t)w2 << (64 - sh))) : lo64;
      tp &= (1ull << 33) - 1;
      return (uint64_t)(row_readlane(x, base) & 0x7fffffffu) | (tp << 31);
    };
    uint64_t xa = approx(a), xb = approx(b);
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 1
    for (int i = 0; i < 31; i++) {
      const bool odd = (xa & 1u) != 0;
      // xa < xb from 32-bit halves: scalar compares (a 64-bit compare is a VALU
      // instruction, and its round trip to the scalar unit cost ~300 cycles per divstep)
      const bool sw = odd && s_lt64(xa, xb);
      const uint64_t ta = sw ? xb : xa, tb = sw ? xa : xb;
      const int64_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      xa = odd ? (ta - tb) >> 1 : ta >> 1;
      xb = tb;
      f0 = odd ? tf0 - tf1 : tf0;
      g0 = odd ? tg0 - tg1 : tg0;
      f1 = tf1 * 2;
      g1 = tg1 * 2;
    }
    bool an, bn;
    uint32_t na, nb;
    row_lin_shift2(a, b, f0, g0, f1, g1, mine, base, na, nb, an, bn);
    if (an) {
      f0 = -f0;
      g0 = -g0;
    }
    if (bn) {
      f1 = -f1;
      g1 = -g1;
    }
    uint32_t nu, nv;
    row_lin_mod2(u, v, f0, g0, f1, g1, mine, base, pj, nu, nv);
    if (mine) {
      a = na;
      b = nb;
      u = nu;
      v = nv;
    }
  }
  return v;  // b = gcd(y, p) = 1 for y != 0, and then v = y^-1
}

}  // namespace co
}  // namespace lb
