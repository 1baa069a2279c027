// Latency path: the round-program interpreter (one workgroup per program
// instance, one unit per 16-lane row per round; bls_coop.h arithmetic in the
// 13-limb Montgomery domain, R = 2^416).
//
// A program (lodestar_amd/lpgen, encoding in lpgen/compile.py) is a sequence
// of rounds; round r's units are independent, each reads LDS registers written
// by earlier rounds and writes one register or flag.  The workgroup runs a
// round between two barriers.  What a lone verification waits for is then the
// DAG depth of its products (~1.8k rounds for hash_to_G2 + decode + Miller
// loop) instead of the ~12k-product serial chains of the one-lane kernels
// (DESIGN.md §7), so the fixed cost of a round is what the design minimises:
//   * the program stream (the rounds' blocks back to back) is read from global
//     memory (L2: every workgroup running a program reads the same blocks), the
//     next round's header and records issued at the start of a round and waited
//     for only where the next round uses them (LB_LP_RING: through an LDS ring
//     ~50 rounds ahead instead, which costs a ring store and an LDS read a round);
//   * a unit is a fixed 36-word record loaded into registers during the
//     PREVIOUS round (three words per lane of its row), so a round starts with
//     every register read of its forms already addressable: one LDS round trip,
//     then arithmetic;
//   * forms multiply unreduced (13-limb Montgomery: operands up to ~2^399).
#include "bls_coop.h"
// The program stream: read straight from global memory one round ahead (default; lone set
// 3.14 -> 2.94 ms, 128-set request 3.48 -> 3.28 ms, profiles/r05/lp_direct/), or through
// an LDS ring filled ~50 rounds ahead (-DLB_LP_RING, rounds 4-5)
#ifndef LB_LP_RING
#define LB_LP_DIRECT 1
#endif
#include "bls_kernels.h"
#include "bls_lp.h"
#ifdef LB_LP_PROGS_HEADER  // (a variant's programs, tools/lp_rows_variant.py)
#include LB_LP_PROGS_HEADER
#else
#include "bls_lp_progs.h"
#endif

static_assert(LB_LP_MTAIL_ROWS == LB_LP_MTAIL_ROWS_GEN, "k_lp_mtail's rows == the merged-check programs' (gen_lp.py)");

namespace lb {

using namespace co;

namespace {

template <int NREGS>
struct LpSharedT {
  uint32_t reg[NREGS * 16];
  uint32_t flag[LB_LP_MAX_FLAGS];
#ifndef LB_LP_DIRECT
  uint32_t ring[LB_LP_RING];
#endif
};
using LpShared = LpSharedT<LB_LP_MAX_REGS>;
using LpSharedMtail = LpSharedT<LB_LP_MTAIL_REGS>;  // (k_lp_mtail: the level products as inputs)
using LpSharedRtail = LpSharedT<LB_LP_RTAIL_REGS>;  // (k_lp_rtail: a small program, two workgroups per CU)
constexpr uint32_t RMASK = LB_LP_RING - 1;
#ifndef LB_LP_DIRECT
static_assert((LB_LP_RING & (LB_LP_RING - 1)) == 0, "ring size: power of two");
static_assert(LB_LP_CHUNK % LB_LP_TPB == 0 && LB_LP_RING >= LB_LP_CHUNK + 2 * LB_LP_BLOCK_CAP, "ring sizing");
constexpr int PFW = LB_LP_CHUNK / LB_LP_TPB;  // stream words per thread per chunk (one 16-byte load)
static_assert(PFW == 4, "one uint4 of the stream per thread and chunk");
#endif
constexpr int NT = 16;                        // inline terms per operand
constexpr int RECW = 4 + 2 * NT;              // fixed unit record (lpgen/compile.py)
constexpr int YT = 3 + NT;                    // first y term word
static constexpr uint32_t INV_FIX_RAW[13] = LB_LP_INV_FIX_RAW_LIMBS;
__device__ __constant__ const uint32_t LB_LP_R416_RAW[12] = LB_LP_R416_RAW_LIMBS;

// A row's unit record, spread over the row: lane j holds words j, 16 + j and 32 + j;
// a word reaches the whole row by a DPP broadcast (row_newbcast).  Every lane loading
// all 36 words instead would move 9 KB per wave and round through the LDS.
struct Desc {
  uint32_t v[3];
  // word k of the record (k a constant after unrolling: the switch folds to one DPP)
  LB_CO uint32_t w(int k) const {
    const uint32_t x = v[k >> 4];
    switch (k & 15) {
      case 0: return bcast<0>(x);
      case 1: return bcast<1>(x);
      case 2: return bcast<2>(x);
      case 3: return bcast<3>(x);
      case 4: return bcast<4>(x);
      case 5: return bcast<5>(x);
      case 6: return bcast<6>(x);
      case 7: return bcast<7>(x);
      case 8: return bcast<8>(x);
      case 9: return bcast<9>(x);
      case 10: return bcast<10>(x);
      case 11: return bcast<11>(x);
      case 12: return bcast<12>(x);
      case 13: return bcast<13>(x);
      case 14: return bcast<14>(x);
      default: return bcast<15>(x);
    }
  }
};
static_assert(RECW <= 48, "a record spans three words per lane");

LB_CO void load_desc(Desc& d, const uint32_t* ring, uint32_t base, uint32_t lane) {
#pragma unroll
  for (int k = 0; k < 3; k++)
    d.v[k] = 16u * k + lane < (uint32_t)RECW ? ring[(base + 16u * k + lane) & RMASK] : 0u;
}

// Both operand forms of an inline record at once (one loop over the wave's longest
// form, the two normalisations sharing their ripple test): x = sum_t c_t vx_t + Kx p,
// y likewise; a form's unused terms have coefficient 0.  A wave whose rows all read
// plain registers (one term, coefficient 1, K = 0) skips the arithmetic.  LIN2 rows:
// x = the form over both term lists.
LB_CO void forms2(uint32_t K, const uint32_t (&tx)[NT], const uint32_t (&ty)[NT], const uint32_t (&vx)[NT],
                  const uint32_t (&vy)[NT], uint32_t n, bool lin2, bool redx, bool redy, uint32_t pj, uint32_t& x,
                  uint32_t& y) {
  const bool plain = n <= 1 && K == 0 && (tx[0] >> 16) <= 1u && (ty[0] >> 16) <= 1u;
  if (!ballot(!plain)) {  // (coefficient 0: an absent form, value 0 -- not read)
    x = vx[0];
    y = vy[0];
    return;
  }
  uint64_t Ux = (uint64_t)(K & 0xffffu) * pj, Vx = 0, Uy = (uint64_t)(K >> 16) * pj, Vy = 0;
#pragma unroll
  for (int t = 0; t < NT; t++) {
    if (!ballot((uint32_t)t < n)) break;
    const int32_t cx = (int32_t)tx[t] >> 16, cy = (int32_t)ty[t] >> 16;
    Ux += (uint64_t)(uint32_t)cx * vx[t];
    Vx += cx < 0 ? (uint64_t)vx[t] : 0ull;
    Uy += (uint64_t)(uint32_t)cy * vy[t];
    Vy += cy < 0 ? (uint64_t)vy[t] : 0ull;
  }
  int64_t Sx = (int64_t)(Ux - (Vx << 32)), Sy = (int64_t)(Uy - (Vy << 32));
  if (lin2) Sx += Sy;
  norm2(Sx, Sy, x, y);
  if (ballot(redx || redy)) {
    if (redx) x = reduce(x, pj);
    if (redy) y = reduce(y, pj);
  }
}

// ---- extended records (forms over 8 terms, multi-way selects), read from the ring
struct Rec {
  const uint32_t* ring;
  uint32_t base;
  LB_CO uint32_t operator[](uint32_t i) const { return ring[(base + i) & RMASK]; }
};
// LB_LP_DIRECT: the record straight from the program stream in global memory (L2)
struct RecG {
  const uint32_t* __restrict__ sp;
  uint32_t base;
  LB_CO uint32_t operator[](uint32_t i) const { return sp[base + i]; }
};

template <class R>
LB_CO uint32_t ext_form(const R& rec, int& o, const uint32_t* __restrict__ reg, uint32_t lane, uint32_t pj) {
  const uint32_t hdr = rec[o];
  const int nt = (int)(hdr & 255u);
  const bool red = (hdr >> 8) & 1u, neg = (hdr >> 9) & 1u;
  const uint32_t K = hdr >> 16;
  const int t0 = o + 1;
  o += 1 + nt;
  // 16 terms per LDS round trip (term words, then their registers), one product per term
  uint64_t U = (uint64_t)K * pj, V = 0;
  for (int t = 0; t < nt; t += 16) {
    uint32_t x[16], v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = t + k < nt ? rec[t0 + t + k] : 0u;
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = reg[(x[k] & 0xffffu) * 16u + lane];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const int32_t c = (int32_t)x[k] >> 16;  // (0 for the padding: no contribution)
      U += (uint64_t)(uint32_t)c * v[k];
      V += c < 0 ? (uint64_t)v[k] : 0ull;
    }
  }
  const int64_t S = (int64_t)(U - (V << 32));
  uint32_t r = neg ? norm<true>(S) : norm<false>(S);
  if (red) r = reduce(r, pj);
  return r;
}

template <class R>
LB_CO void skip_form(const R& rec, int& o) { o += 1 + (int)(rec[o] & 255u); }

// the one-operand units on a normalized value x; returns true when it wrote a flag
template <class SH>
LB_CO bool single_op(uint32_t op, uint32_t dst, uint32_t x, SH& S, uint32_t lane, uint32_t pj, uint32_t& v) {
  if (op == LB_LP_OP_LIN) {
    v = x;
    return false;
  }
  const uint32_t c = canon(x, pj);
  if (op == LB_LP_OP_CANON) {
    v = c;
    return false;
  }
  if (op == LB_LP_OP_INV) {
    // the row-cooperative binary GCD (bls_coop.h row_inv_raw), one INV row of the wave
    // after the other (its divsteps run on scalar registers: one row at a time)
    uint32_t r = 0;
    for (uint64_t m = ballot(lane == 0); m; m &= m - 1) {
      const uint32_t base = (uint32_t)__builtin_ctzll(m);
      const bool mine = (lane64() & ~15u) == base;
      const uint32_t ri = row_inv_raw(c, mine, base, pj);
      if (mine) r = ri;
    }
    v = canon(mont_mul<13>(r, const_limb13(INV_FIX_RAW), pj), pj);  // canonical, as the executor's
    return false;
  }
  bool f;
  if (op == LB_LP_OP_ISZERO)
    f = row_is_zero(c);
  else if (op == LB_LP_OP_BIT0)
    f = row_bit0(c) != 0;
  else
    f = row_gt_half(c);
  if (lane == 0) S.flag[dst] = f ? 1u : 0u;
  return true;
}

template <class R, class SH>
LB_CO void ext_unit(const R& rec, SH& S, uint32_t lane, uint32_t pj) {
  const uint32_t w0 = rec[0];
  const uint32_t op = w0 & 15u, nops = (w0 >> 4) & 7u, nfl = (w0 >> 7) & 7u, dst = w0 >> 16;
  int o = 1 + (int)nfl;
  uint32_t v;
  if (op == LB_LP_OP_SEL) {
    uint32_t choice = nops - 1;
    for (uint32_t i = 0; i < nfl; i++)
      if (S.flag[rec[1 + i]] && choice == nops - 1) choice = i;
    for (uint32_t i = 0; i < choice; i++) skip_form(rec, o);
    v = ext_form(rec, o, S.reg, lane, pj);
  } else {
    const uint32_t x = ext_form(rec, o, S.reg, lane, pj);
    if (op == LB_LP_OP_MUL) {
      const uint32_t y = ext_form(rec, o, S.reg, lane, pj);
      v = mont_mul<13>(x, y, pj);
    } else if (single_op(op, dst, x, S, lane, pj, v)) {
      return;
    }
  }
  S.reg[dst * 16u + lane] = v;
}

// one unit from its prefetched record; every lane of the row calls it
template <class SH>
LB_CO void run_unit(const Desc& d, SH& S, uint32_t cons, uint32_t lane, uint32_t pj,
                    const uint32_t* __restrict__ gsp, unsigned long long* ustamp = nullptr) {
  // ustamp (diagnostic): s_memtime after the register reads / x form / y form / product
#define LB_LP_USTAMP(k)                                                       \
  do {                                                                        \
    if (ustamp && (threadIdx.x & 63u) == 0) ustamp[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  const uint32_t w0 = d.w(0);
  const uint32_t op = w0 & 15u, dst = w0 >> 19;
  const uint32_t aux = d.w(2);  // (a DPP broadcast: read with the whole row active)
  if (op == LB_LP_OP_FOP) {
    if (lane == 0) {
      const uint32_t x = aux, fop = x & 7u, f1 = (x >> 3) & 0x1fffu, f2 = x >> 16;
      uint32_t v;
      if (fop == 0)
        v = S.flag[f1] & S.flag[f2];
      else if (fop == 1)
        v = S.flag[f1] | S.flag[f2];
      else if (fop == 2)
        v = S.flag[f1] ^ S.flag[f2];
      else if (fop == 3)
        v = S.flag[f1] ^ 1u;
      else
        v = f1 & 1u;
      S.flag[dst] = v;
    }
    return;
  }
  if ((w0 >> 18) & 1u) {
#ifdef LB_LP_DIRECT
    ext_unit(RecG{gsp, cons + aux}, S, lane, pj);
#else
    (void)gsp;
    ext_unit(Rec{S.ring, cons + aux}, S, lane, pj);
#endif
    return;
  }
  const uint32_t nx = (w0 >> 4) & 31u, ny = (w0 >> 9) & 31u;
  const bool redx = (w0 >> 16) & 1u, redy = (w0 >> 17) & 1u;
  // every register read of both forms in one LDS round trip, unconditionally: a record's
  // unused term words are 0 (register 0, coefficient 0), so no lane masks or branches
  // (in tiers of 4 terms, each tier behind a wave-uniform test of the wave's longest form)
  const uint32_t n = nx > ny ? nx : ny;
  uint32_t tx[NT], ty[NT], vx[NT], vy[NT];
#pragma unroll
  for (int t = 0; t < NT; t++) tx[t] = ty[t] = vx[t] = vy[t] = 0u;
#pragma unroll
  for (int tier = 0; tier < NT / 4; tier++) {
    if (tier > 0 && !ballot(n > 4u * tier)) break;
#pragma unroll
    for (int t = 4 * tier; t < 4 * tier + 4; t++) {
      tx[t] = d.w(3 + t);
      ty[t] = d.w(YT + t);
      vx[t] = S.reg[(tx[t] & 0xffffu) * 16u + lane];
      vy[t] = S.reg[(ty[t] & 0xffffu) * 16u + lane];
    }
  }
  if (ustamp) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    LB_LP_USTAMP(0);
  }
  uint32_t x, y;
  const bool lin2 = op == LB_LP_OP_LIN2;
  forms2(d.w(1), tx, ty, vx, vy, lin2 ? NT : n, lin2, redx, redy, pj, x, y);
  LB_LP_USTAMP(1);
  LB_LP_USTAMP(2);
  uint32_t v;
  if (op == LB_LP_OP_MUL) {
    v = mont_mul<13>(x, y, pj);
    LB_LP_USTAMP(3);
  } else if (op == LB_LP_OP_SEL) {
    v = S.flag[aux] ? x : y;
  } else if (single_op(lin2 ? LB_LP_OP_LIN : op, dst, x, S, lane, pj, v)) {
    return;
  }
  S.reg[dst * 16u + lane] = v;
#undef LB_LP_USTAMP
}

struct Stream {
  const uint32_t* sp;  // first stream word
  uint32_t sw;         // stream words
  uint32_t cons;       // stream position of the round executing
  uint32_t done;       // words stored in the ring (valid: [cons, done))
  uint32_t issued;     // words requested (in registers: [done, issued))
};

// one round.  d / bw / nu: this round's record (row) and block header, prefetched;
// the next round's are loaded into them.  pf: the chunk issued last round (stored
// into the ring first), then the chunk this round issues -- ONE register set: with a
// double buffer swapped at the end of the round the compiler copies the fresh loads
// right after issuing them, which waits out a global-memory round trip every round.
#ifdef LB_LP_DIRECT
// LB_LP_DIRECT: no LDS ring.  The next round's header and this row's record come straight
// from the program stream (global memory; every workgroup running the program reads the
// same blocks, so L2), issued one round ahead like the ring's prefetch and waited for only
// where the next round uses them; extended records are read from the stream in place.
template <class SH>
LB_CO void lp_round(SH& S, Stream& st, Desc& d, uint32_t& bw, uint32_t& nu, uint4& pf,
                    uint32_t tid, uint32_t lane, uint32_t row, uint32_t pj,
                    unsigned long long* stamps, uint32_t r) {
  (void)pf;
  // stamps (diagnostic, tools/lp_probe.py; only in a -DLB_LP_STAMPS_ON build, which keeps them
  // out of the product's register allocation): the ring build's points 0-5 (1, 2: no ring store)
#ifndef LB_LP_STAMPS_ON
  stamps = nullptr;
#endif
#define LB_LP_STAMP(k)                                                                     \
  do {                                                                                     \
    if (stamps && tid == 0) stamps[r * LB_LP_STAMPS + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  LB_LP_STAMP(0);
  LB_LP_STAMP(1);
  LB_LP_STAMP(2);
  const uint32_t cons_n = st.cons + bw;
  Desc dn;
  uint32_t bwn = 0, nun = 0;
  if (cons_n < st.sw) {
    // (kept in vector registers: a readfirstlane into scalar ones waits for the load in this
    // round, exposing its latency -- lone set 2.93-2.96 -> 3.18 ms, profiles/r05/lp_direct/r05r)
    const uint4 h = *reinterpret_cast<const uint4*>(st.sp + cons_n);
    bwn = h.x;
    nun = h.y;
#pragma unroll
    for (int k = 0; k < 3; k++)
      dn.v[k] = 16u * k + lane < (uint32_t)RECW ? st.sp[cons_n + 4 + RECW * row + 16u * k + lane] : 0u;
  }
  LB_LP_STAMP(3);
  if (stamps && (tid & 63u) == 0) stamps[r * LB_LP_STAMPS + 6 + (tid >> 6)] = __builtin_amdgcn_s_memtime();
  if (row < nu)
    run_unit(d, S, st.cons, lane, pj, st.sp,
             stamps ? stamps + r * LB_LP_STAMPS + 6 + 2 * LB_LP_TPB / 64 + 4 * (tid >> 6) : nullptr);
  if (stamps && (tid & 63u) == 0) stamps[r * LB_LP_STAMPS + 6 + LB_LP_TPB / 64 + (tid >> 6)] = __builtin_amdgcn_s_memtime();
  LB_LP_STAMP(4);
  st.cons = cons_n;
  d = dn;
  bw = bwn;
  nu = nun;
  __syncthreads();
  LB_LP_STAMP(5);
#undef LB_LP_STAMP
}
#else
template <class SH>
LB_CO void lp_round(SH& S, Stream& st, Desc& d, uint32_t& bw, uint32_t& nu, uint4& pf,
                    uint32_t tid, uint32_t lane, uint32_t row, uint32_t pj,
                    unsigned long long* stamps, uint32_t r) {
  // stamps (diagnostic): LB_LP_STAMPS s_memtime points per round, lane 0 of the workgroup
#define LB_LP_STAMP(k)                                                              \
  do {                                                                             \
    if (stamps && tid == 0) stamps[r * LB_LP_STAMPS + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
  LB_LP_STAMP(0);
  const uint32_t cons_n = st.cons + bw;
  // the ring must hold the next round's block: catch up synchronously when the
  // prefetch ran dry (rare: it runs far ahead)
  const uint32_t need = min(st.sw, cons_n + LB_LP_BLOCK_CAP);
  while (st.done < need) {
    const uint32_t n = min((uint32_t)LB_LP_CHUNK, st.issued - st.done);
    if (n) {
      if (4u * tid < n) *reinterpret_cast<uint4*>(&S.ring[(st.done + 4u * tid) & RMASK]) = pf;
      st.done += n;
    } else {
      const uint32_t m = min((uint32_t)LB_LP_CHUNK, st.sw - st.done);
      if (4u * tid < m)
        *reinterpret_cast<uint4*>(&S.ring[(st.done + 4u * tid) & RMASK]) =
            *reinterpret_cast<const uint4*>(st.sp + st.done + 4u * tid);
      st.done += m;
      st.issued = st.done;
    }
    __syncthreads();
  }
  // the chunk loaded last round (in pf) into the ring first: its loads had a whole round
  // to arrive, and this round's loads, issued after, are not waited for (a wait placed
  // after them would expose a global-memory round trip in every round).  Stream words
  // move 4 per thread: one 16-byte global load and one ds_write_b128 (the stream starts
  // 16-byte aligned and every block is a multiple of 4 words: lpgen/compile.py)
  LB_LP_STAMP(1);
  const uint32_t pending = st.issued - st.done;  // words in pf
  if (4u * tid < pending) *reinterpret_cast<uint4*>(&S.ring[(st.done + 4u * tid) & RMASK]) = pf;
  st.done += pending;
  asm volatile("" ::: "memory");
  LB_LP_STAMP(2);
  uint32_t n_new = 0;
  if (st.issued < st.sw && st.issued + LB_LP_CHUNK <= cons_n + LB_LP_RING) {
    n_new = min((uint32_t)LB_LP_CHUNK, st.sw - st.issued);
    if (4u * tid < n_new) pf = *reinterpret_cast<const uint4*>(st.sp + st.issued + 4u * tid);
  }
  // the next round's header and this row's record (consumed after the barrier)
  Desc dn;
  uint32_t bwn = 0, nun = 0;
  if (cons_n < st.sw) {
    const uint4 h = *reinterpret_cast<const uint4*>(S.ring + (cons_n & RMASK));
    bwn = h.x;
    nun = h.y;
    load_desc(dn, S.ring, cons_n + 4 + RECW * row, lane);
  }
  LB_LP_STAMP(3);
  if (stamps && (tid & 63u) == 0) stamps[r * LB_LP_STAMPS + 6 + (tid >> 6)] = __builtin_amdgcn_s_memtime();
  if (row < nu)
    run_unit(d, S, st.cons, lane, pj, st.sp,
             stamps ? stamps + r * LB_LP_STAMPS + 6 + 2 * LB_LP_TPB / 64 + 4 * (tid >> 6) : nullptr);
  if (stamps && (tid & 63u) == 0) stamps[r * LB_LP_STAMPS + 6 + LB_LP_TPB / 64 + (tid >> 6)] = __builtin_amdgcn_s_memtime();
  LB_LP_STAMP(4);
  st.issued += n_new;
  st.cons = cons_n;
  d = dn;
  bw = bwn;
  nu = nun;
  __syncthreads();
  LB_LP_STAMP(5);
#undef LB_LP_STAMP
}

#endif

}  // namespace

// Run program `prog` for one instance on this workgroup.  Inputs i < split come
// from in_a[16 i ...], the rest from in_b[16 (i - split) ...] (16-word records of
// canonical limbs: R = 2^384 Montgomery for the set programs, this domain for
// Miller values); in_flags: n_inflag words; out: n_out 16-word records;
// out_flags: n_outflag words.  stamps (diagnostic, usually nullptr): s_memtime
// after every round's barrier.
template <class SH>
LB_DEV void lp_run(SH& S, const uint32_t* __restrict__ prog, const uint32_t* __restrict__ in_a, uint32_t split,
                   const uint32_t* __restrict__ in_b, const uint32_t* __restrict__ in_flags,
                   uint32_t* __restrict__ out, uint32_t* __restrict__ out_flags,
                   unsigned long long* __restrict__ stamps = nullptr) {
  // (rows = the workgroup's: 32 for the verification programs, LB_LP_MTAIL_ROWS for k_lp_mtail's;
  // a program never schedules more units in a round than the rows it was compiled for)
  const uint32_t tid = threadIdx.x, lane = tid & 15u, row = tid >> 4, tpb = blockDim.x, rows = tpb >> 4;
  const uint32_t pj = p_limb();
  const uint32_t n_rounds = prog[1], n_const = prog[4], n_in = prog[5], n_inflag = prog[6], n_out = prog[7],
                 n_outflag = prog[8];
  Stream st;
  st.sw = prog[9];
  uint32_t pos = LB_LP_HDR;
  for (uint32_t i = row; i < n_const; i += rows) {
    const uint32_t* c = prog + pos + 14 * i;
    S.reg[c[0] * 16u + lane] = lane < 13 ? c[1 + lane] : 0u;
  }
  pos += 14 * n_const;
  for (uint32_t i = row; i < n_in; i += rows) {
    const uint32_t* src = i < split ? in_a + 16 * i : in_b + 16 * (i - split);
    S.reg[prog[pos + i] * 16u + lane] = lane < 13 ? src[lane] : 0u;
  }
  pos += n_in;
  for (uint32_t i = tid; i < n_inflag; i += tpb) S.flag[prog[pos + i]] = in_flags[i] ? 1u : 0u;
  pos += n_inflag;
  const uint32_t* outs = prog + pos;
  pos += n_out;
  const uint32_t* outfl = prog + pos;
  pos += n_outflag;
  pos = (pos + 3u) & ~3u;  // (the stream starts 16-byte aligned)
  st.sp = prog + pos;
  st.cons = 0;
  Desc d;
  uint32_t bw = 0, nu = 0;
#ifdef LB_LP_DIRECT
  st.done = st.issued = 0;
  __syncthreads();
  if (st.sw) {
    const uint4 h = *reinterpret_cast<const uint4*>(st.sp);
    bw = h.x;
    nu = h.y;
#pragma unroll
    for (int k = 0; k < 3; k++)
      d.v[k] = 16u * k + lane < (uint32_t)RECW ? st.sp[4 + RECW * row + 16u * k + lane] : 0u;
  }
#else
  st.done = st.issued = min(st.sw, (uint32_t)(LB_LP_RING - LB_LP_CHUNK));
  for (uint32_t i = tid; i < st.done; i += tpb) S.ring[i] = st.sp[i];
  __syncthreads();
  if (st.sw) {
    const uint4 h = *reinterpret_cast<const uint4*>(S.ring);
    bw = h.x;
    nu = h.y;
    load_desc(d, S.ring, 4 + RECW * row, lane);
  }
#endif
  uint4 pf = make_uint4(0u, 0u, 0u, 0u);
  // one copy of the round in the loop (the round's code is most of the kernel's, and the
  // instruction cache is 64 KB)
#pragma unroll 1
  for (uint32_t r = 0; r < n_rounds; r++) lp_round(S, st, d, bw, nu, pf, tid, lane, row, pj, stamps, r);
  for (uint32_t i = row; i < n_out; i += rows) out[16 * i + lane] = lane < 13 ? S.reg[outs[i] * 16u + lane] : 0u;
  for (uint32_t i = tid; i < n_outflag; i += tpb) out_flags[i] = S.flag[outfl[i]];
}

// ---------------------------------------------------------------------------
// The small-call pipeline (lb_verify_requests on calls of at most lp_max_sets sets):
//   k_lp_prep     one lane per set: hash_to_field of the signing root, the
//                 signature's byte-level decode (Signature.fromBytes up to the
//                 curve arithmetic), the pubkey (from k_pubkeys_*), the batch
//                 scalar's GLV halves as flags -> the set program's inputs
//   k_lp_verify   one workgroup per set: the set program (1-set requests: core
//                 verify; >= 2 sets: the batch equation's factor of this set),
//                 then the request's product tree across its sets' workgroups
//                 (the second workgroup to reach a node multiplies), and at the
//                 root the final exponentiation and the request's verdict.
// Verdict rules: verifySignatureSetsMaybeBatch (BN/chain/bls/maybeBatch.ts:16-46),
// exactly as the throughput pipeline applies them (bls_host.hip).
// ---------------------------------------------------------------------------
static constexpr uint32_t LP_NIN = LB_LP_NIN, LP_NFL = LB_LP_NFL;

__global__ void __launch_bounds__(TPB) k_lp_prep(uint32_t n, const uint32_t* __restrict__ req_off, uint32_t n_req,
                                                 const uint8_t* __restrict__ msgs, const uint8_t* __restrict__ sigs,
                                                 const uint32_t* __restrict__ sig_off, const g1j* __restrict__ pk,
                                                 const uint8_t* __restrict__ seed, uint32_t* __restrict__ in16,
                                                 uint32_t* __restrict__ flags, uint8_t* __restrict__ sig_st,
                                                 uint32_t* __restrict__ set_req, uint8_t* __restrict__ valid,
                                                 uint8_t* __restrict__ req_err, uint32_t* __restrict__ cnt, uint32_t n_cnt,
                                                 unsigned long long* __restrict__ clk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  // the call's outputs and k_lp_verify's tree counters / clock stamps start at zero (here
  // instead of four memset launches ahead of a lone set's critical path)
  const uint32_t gsz = gridDim.x * blockDim.x;
  for (uint32_t j = i; j < n_req; j += gsz) {
    valid[j] = 0;
    req_err[j] = 0;
  }
  for (uint32_t j = i; j < n_cnt; j += gsz) cnt[j] = 0u;
  if (i < 4 && clk) clk[i] = 0ull;
  if (i >= n) return;
  // request of set i (binary search over the offsets)
  uint32_t lo = 0, hi = n_req;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (req_off[mid] <= i)
      lo = mid;
    else
      hi = mid;
  }
  set_req[i] = lo;
  uint32_t* rec = in16 + (size_t)i * LP_NIN * 16;
  uint32_t* fl = flags + (size_t)i * LP_NFL;
  auto put = [&](int k, const fp& v) {
#pragma unroll
    for (int j = 0; j < 12; j++) rec[16 * k + j] = v.l[j];
#pragma unroll
    for (int j = 12; j < 16; j++) rec[16 * k + j] = 0u;
  };
  uint8_t m[32];
  for (int k = 0; k < 32; k++) m[k] = msgs[(size_t)i * 32 + k];
  fp2 u[2];
  hash_to_field_fp2_2(u, m);
  put(0, u[0].c0);
  put(1, u[0].c1);
  put(2, u[1].c0);
  put(3, u[1].c1);
  // Signature.fromBytes up to the curve arithmetic (bls_curve.h g2_deserialize)
  const uint32_t a = sig_off[i], len = sig_off[i + 1] - a;
  const uint8_t* b = sigs + a;
  uint8_t st = LB_ST_OK;
  bool inf = false, comp = false, sign = false;
  fp x0, x1, y0, y1;
  fp_zero(x0);
  fp_zero(x1);
  fp_zero(y0);
  fp_zero(y1);
  if (len == 0) {
    st = LB_ST_BAD_ENCODING;
  } else {
    const uint8_t f = b[0];
    comp = (f & 0x80) != 0;
    if (len != (comp ? 96u : 192u)) {
      st = LB_ST_BAD_ENCODING;
    } else if (comp ? (f & 0x40) != 0 : (f & 0xe0) != 0) {
      if ((f & 0x40) && (f & 0x3f) == 0 && bytes_zero(b + 1, (int)len - 1))
        inf = true;
      else
        st = LB_ST_BAD_ENCODING;
    } else {
      sign = comp && (f & 0x20) != 0;
      bool ok = fp_read_masked(x1, b, comp) && fp_read_masked(x0, b + 48, false);
      if (ok && !comp) ok = fp_read_masked(y1, b + 96, false) && fp_read_masked(y0, b + 144, false);
      if (!ok) st = LB_ST_BAD_ENCODING;
    }
  }
  if (st != LB_ST_OK) {
    fp_zero(x0);
    fp_zero(x1);
    fp_zero(y0);
    fp_zero(y1);
  }
  put(4, x0);
  put(5, x1);
  put(6, y0);
  put(7, y1);
  const g1j p = pk[i];
  put(8, p.X);
  put(9, p.Y);
  put(10, p.Z);
  sig_st[i] = st;
  fl[0] = inf ? 1u : 0u;
  fl[1] = sign ? 1u : 0u;
  fl[2] = comp ? 1u : 0u;
  // the batch scalar's halves (set_batch only: a 1-set request runs set_single, which
  // reads none of them -- no SHA-256 compression on a lone set's critical path)
  uint64_t r = 0;
  if (req_off[lo + 1] - req_off[lo] != 1) {
    uint8_t sd[32];
    for (int k = 0; k < 32; k++) sd[k] = seed[k];
    r = batch_scalar(sd, i);
  }
  const uint32_t ra = (uint32_t)r, rb = (uint32_t)(r >> 32);
  for (int k = 0; k < 32; k++) {
    fl[3 + k] = (ra >> (31 - k)) & 1u;
    fl[35 + k] = (rb >> (31 - k)) & 1u;
  }
}

__global__ void __launch_bounds__(LB_LP_TPB, LB_LP_VERIFY_WPE) k_lp_verify(LpCall c) {
  __shared__ LpShared S;
  __shared__ uint32_t sh_old, sh_bad, sh_err, s_fl[4];
  const uint32_t i = blockIdx.x, tid = threadIdx.x;
  if (i >= c.n_sets) return;
  if (i == 0 && tid == 0 && c.clk) {
    c.clk[0] = __builtin_amdgcn_s_memrealtime();
    c.clk[1] = __builtin_amdgcn_s_memtime();
  }
  const uint32_t k = c.set_req[i], base = c.req_off[k], n = c.req_off[k + 1] - base;
  const bool single = n == 1;
  // one interpreter call site, run per phase (the set program, each product of the
  // tree, the final exponentiation): a single inlined copy of lp_run keeps the kernel's
  // code a third of three copies'
  enum { SET, TREE, FINAL };
  int phase = SET;
  const uint32_t* prog = single ? c.prog_single : c.prog_batch;
  const uint32_t* in_a = c.in16 + (size_t)i * LP_NIN * 16;
  const uint32_t* in_b = nullptr;
  const uint32_t* in_fl = c.flags + (size_t)i * LP_NFL;
  uint32_t split = 0xffffffffu;
  uint32_t* out = c.F + (size_t)i * 12 * 16;
  uint32_t pos = i - base, level = 0;
  for (;;) {
    lp_run(S, prog, in_a, split, in_b, in_fl, out, s_fl);
    __syncthreads();
    if (phase == FINAL) {
      if (tid == 0) {
        c.valid[k] = s_fl[0] ? 1 : 0;
        c.req_err[k] = (sh_err & 2u) ? LB_REQ_EMPTY_AGGREGATE : (sh_err & 1u) ? LB_REQ_BAD_PUBKEY : LB_REQ_OK;
        if (k == 0 && c.clk) {
          c.clk[2] = __builtin_amdgcn_s_memrealtime();
          c.clk[3] = __builtin_amdgcn_s_memtime();
        }
      }
      return;
    }
    if (phase == SET && tid == 0) {
      uint8_t st = c.sig_st[i];
      const bool sig_inf = c.flags[(size_t)i * LP_NFL] != 0;
      if (st == LB_ST_OK) {  // (the infinity encoding: no curve / subgroup test applies)
        if (sig_inf) {
          if (single) st = LB_ST_ZERO_SIGNATURE;
        } else if (!s_fl[0]) {
          st = LB_ST_NOT_ON_CURVE;
        } else if (!s_fl[1]) {
          st = LB_ST_NOT_IN_GROUP;
        }
      }
      c.sig_st[i] = st;
      uint8_t ps = c.pk_st[i];
      if (ps == LB_ST_OK && single && !s_fl[2]) ps = LB_ST_NOT_IN_GROUP;
      c.pk_st[i] = ps;
    }
    // the request's product tree: at level l the node of the positions [q, q + 2^(l+1))
    // multiplies the values at q and q + 2^l; the second of the two workgroups to
    // arrive does it and continues upward
    bool more = false;
    for (; (1u << level) < n; level++) {
      const uint32_t step = 1u << level;
      const uint32_t left = pos & ~(2 * step - 1);
      if (left + step >= n) continue;  // no right sibling: the value passes up unchanged
      __threadfence();  // every wave: its stores of this workgroup's value (and set status) at L2
      __syncthreads();
      if (tid == 0) {
        __threadfence();  // release
        sh_old = atomicAdd(c.cnt + (size_t)level * c.n_sets + base + left, 1u);
        __threadfence();
      }
      __syncthreads();
      if (sh_old == 0) return;  // the sibling's workgroup carries on
      __threadfence();          // acquire the sibling's value
      prog = c.prog_mul;
      in_a = c.F + (size_t)(base + left) * 12 * 16;
      in_b = c.F + (size_t)(base + left + step) * 12 * 16;
      split = 12;
      in_fl = nullptr;
      out = const_cast<uint32_t*>(in_a);
      pos = left;
      level++;
      more = true;
      break;
    }
    if (more) {
      phase = TREE;
      continue;
    }
    // root: the request's statuses, then its final exponentiation
    __syncthreads();
    __threadfence();
    if (tid == 0) {
      sh_bad = 0;
      sh_err = LB_REQ_OK;
    }
    __syncthreads();
    {
      uint32_t bad = 0, empty = 0, badpk = 0;
      for (uint32_t j = tid; j < n; j += LB_LP_TPB) {
        const uint8_t ss = ((volatile uint8_t*)c.sig_st)[base + j], ps = ((volatile uint8_t*)c.pk_st)[base + j];
        bad |= (ss != LB_ST_OK || ps != LB_ST_OK) ? 1u : 0u;
        empty |= ps == LB_ST_EMPTY_AGGREGATE ? 1u : 0u;
        badpk |= ps == LB_ST_BAD_ENCODING ? 1u : 0u;
      }
      if (bad) atomicOr(&sh_bad, 1u);
      if (empty) atomicOr(&sh_err, 2u);
      if (badpk) atomicOr(&sh_err, 1u);
    }
    __syncthreads();
    if (sh_bad) {
      if (tid == 0) {
        c.valid[k] = 0;
        c.req_err[k] = (sh_err & 2u) ? LB_REQ_EMPTY_AGGREGATE : (sh_err & 1u) ? LB_REQ_BAD_PUBKEY : LB_REQ_OK;
      }
      return;
    }
    phase = FINAL;
    prog = c.prog_final;
    in_a = c.F + (size_t)base * 12 * 16;
    in_b = nullptr;
    split = 0xffffffffu;
    in_fl = nullptr;
    out = nullptr;
  }
}

// The throughput pipeline's merged check (bls_host.hip run_pipeline: steps organisation
// with the bucket MSM): S_all from the MSM's bit sums, Miller(-g1, S_all) times the
// Horner value of the call's level products, final exponentiation -- ~880 rounds on one
// workgroup instead of the one-lane msm_final (1.5 ms) + lines of S_all (3.4 ms) + the
// one-wave final exponentiation (3.1 ms) on every call's serial tail.
__global__ void __launch_bounds__(LB_LP_MTAIL_ROWS * 16) k_lp_mtail(const uint32_t* __restrict__ prog,
                                                        const uint32_t* __restrict__ in16, uint8_t* __restrict__ mflag,
                                                        uint32_t* __restrict__ out16) {
  __shared__ LpSharedMtail S;
  __shared__ uint32_t s_fl[4];
  lp_run(S, prog, in16, 0xffffffffu, in16, nullptr, out16, s_fl);
  __syncthreads();
  if (mflag && threadIdx.x == 0) mflag[0] = s_fl[0] ? 1 : 0;
}

__global__ void __launch_bounds__(LB_LP_TPB) k_lp_final_lane(const uint32_t* __restrict__ prog,
                                                             const uint32_t* __restrict__ in16,
                                                             uint8_t* __restrict__ out) {
  __shared__ LpShared S;
  __shared__ uint32_t s_fl[4];
  lp_run(S, prog, in16, 0xffffffffu, in16, nullptr, nullptr, s_fl);
  __syncthreads();
  if (threadIdx.x == 0) out[0] = s_fl[0] ? 1 : 0;
}

// The merged-check program's inputs as 16-word records: the 63 level products P_l (k_level_prod)
// in the program's domain (R = 2^416: x 2^416 / 2^384, one product by the raw constant 2^416 mod
// p -- lpgen/bls.py mtail_program takes them as raw inputs), then the MSM's 33 bit sums in the
// one-lane form (converted by the program).  fp12: 12 fp in the order c0.c0.c0 ... c1.c2.c1;
// g2j: X.c0, X.c1, Y.c0, Y.c1, Z.c0, Z.c1.
__global__ void __launch_bounds__(256) k_mtail_prep(const fp12* __restrict__ Pl, const g2j* __restrict__ G,
                                                    uint32_t* __restrict__ in16) {
  constexpr uint32_t NP = 12 * LB_MTAIL_LEVELS;
  for (uint32_t i = threadIdx.x; i < (uint32_t)LB_MTAIL_NIN; i += blockDim.x) {
    fp v;
    if (i < NP) {
      fp k;
      fp_set(k, LB_LP_R416_RAW);
      fp_mul(v, (&Pl[i / 12].c0.c0.c0)[i % 12], k);
    } else {
      if (!G) break;  // (the G_p records already written by the lone call's bit-sum programs)
      v = (&G[(i - NP) / 6].X.c0)[(i - NP) % 6];
    }
#pragma unroll
    for (int j = 0; j < 12; j++) in16[16 * i + j] = v.l[j];
#pragma unroll
    for (int j = 12; j < 16; j++) in16[16 * i + j] = 0u;
  }
}

__global__ void __launch_bounds__(256) k_rtail_prep(uint32_t n_req, const fp12* __restrict__ F,
                                                    const g2a* __restrict__ S, uint32_t* __restrict__ in16,
                                                    uint32_t* __restrict__ inflag) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_req * (uint32_t)LB_RTAIL_NIN) return;
  const uint32_t k = t / LB_RTAIL_NIN, i = t % LB_RTAIL_NIN;
  const fp v = i < 12 ? (&F[k].c0.c0.c0)[i]
                      : i == 12 ? S[k].x.c0 : i == 13 ? S[k].x.c1 : i == 14 ? S[k].y.c0 : S[k].y.c1;
#pragma unroll
  for (int j = 0; j < 12; j++) in16[16 * t + j] = v.l[j];
#pragma unroll
  for (int j = 12; j < 16; j++) in16[16 * t + j] = 0u;
  if (i == 0) inflag[k] = S[k].inf ? 1u : 0u;
}

__global__ void __launch_bounds__(LB_LP_TPB, LB_LP_VERIFY_WPE) k_lp_rtail(const uint32_t* __restrict__ prog,
                                                                          uint32_t n_req,
                                                                          const uint32_t* __restrict__ in16,
                                                                          const uint32_t* __restrict__ inflag,
                                                                          const uint8_t* __restrict__ req_bad,
                                                                          uint8_t* __restrict__ valid,
                                                                          const uint8_t* __restrict__ skip) {
  __shared__ LpSharedRtail S;
  __shared__ uint32_t s_fl[4];
  const uint32_t k = blockIdx.x;
  if (k >= n_req) return;
  if (req_bad[k] || (skip && *skip)) {  // (uniform per workgroup)
    if (threadIdx.x == 0) valid[k] = req_bad[k] ? 0 : 1;
    return;
  }
  const uint32_t* in = in16 + (size_t)k * LB_RTAIL_NIN * 16;
  lp_run(S, prog, in, 0xffffffffu, in, inflag + k, nullptr, s_fl);
  __syncthreads();
  if (threadIdx.x == 0) valid[k] = s_fl[0] ? 1 : 0;
}

__global__ void __launch_bounds__(256) k_msm_bits_prep(const g2j* __restrict__ bsum, uint32_t* __restrict__ in16) {
  constexpr uint32_t PER_POS = LB_MSM_NB / 2 / LB_MSM_BITS_GROUP;  // instances per bit position
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;        // (instance, point, coordinate)
  if (t >= (uint32_t)LB_MSM_BITS_INST * LB_MSM_BITS_GROUP * 6u) return;
  const uint32_t c = t % 6u, j = (t / 6u) % LB_MSM_BITS_GROUP, inst = t / (6u * LB_MSM_BITS_GROUP);
  const uint32_t p = inst / PER_POS, m = (inst % PER_POS) * LB_MSM_BITS_GROUP + j;
  const uint32_t w = p / LB_MSM_C, k = p % LB_MSM_C;
  const uint32_t n = k < LB_MSM_C - 1 ? LB_MSM_NB / 2 : 1u;  // (k_msm_bits' enumeration)
  fp v;
  fp_zero(v);  // (a missing point: all zero, Z = 0 -- infinity to the program)
  if (m < n) {
    const uint32_t low = m & ((1u << k) - 1u), high = m >> k;
    const uint32_t d = (high << (k + 1)) | (1u << k) | low;
    v = (&bsum[w * LB_MSM_NB + d - 1].X.c0)[c];
  }
#pragma unroll
  for (int q = 0; q < 12; q++) in16[16 * t + q] = v.l[q];
#pragma unroll
  for (int q = 12; q < 16; q++) in16[16 * t + q] = 0u;
}

__global__ void __launch_bounds__(LB_LP_TPB, LB_LP_VERIFY_WPE) k_lp_msm_bits(const uint32_t* __restrict__ prog,
                                                                             uint32_t n, uint32_t n_in,
                                                                             uint32_t n_out,
                                                                             const uint32_t* __restrict__ in16,
                                                                             uint32_t* __restrict__ out16) {
  __shared__ LpSharedRtail S;
  __shared__ uint32_t s_fl[4];
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
  const uint32_t* in = in16 + (size_t)b * n_in * 16;
  lp_run(S, prog, in, 0xffffffffu, in, nullptr, out16 + (size_t)b * n_out * 16, s_fl);
}

__global__ void __launch_bounds__(256) k_sm_dec_prep(uint32_t n, const uint8_t* __restrict__ sigs,
                                                     const uint32_t* __restrict__ sig_off, uint32_t* __restrict__ in16,
                                                     uint32_t* __restrict__ fl, uint8_t* __restrict__ pre) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // g2_deserialize's encoding rules (bls_curve.h) up to its curve arithmetic
  const uint32_t a = sig_off[i], len = sig_off[i + 1] - a;
  const uint8_t* b = sigs + a;
  fp v[4];  // x.c0, x.c1, y.c0, y.c1 (one-lane Montgomery form)
#pragma unroll
  for (int c = 0; c < 4; c++) fp_zero(v[c]);
  bool inf = false, sign = false, comp = false;
  uint8_t st = LB_ST_OK;
  if (len == 0) {
    st = LB_ST_BAD_ENCODING;
  } else {
    const uint8_t f = b[0];
    comp = (f & 0x80) != 0;
    if (len != (comp ? 96u : 192u)) {
      st = LB_ST_BAD_ENCODING;
    } else if (comp) {
      if (f & 0x40) {
        if ((f & 0x3f) == 0 && bytes_zero(b + 1, 95))
          inf = true;
        else
          st = LB_ST_BAD_ENCODING;
      } else {
        if (!fp_read_masked(v[1], b, true) || !fp_read_masked(v[0], b + 48, false)) st = LB_ST_BAD_ENCODING;
        sign = (f & 0x20) != 0;
      }
    } else if (f & 0xe0) {
      if ((f & 0x40) && (f & 0x3f) == 0 && bytes_zero(b + 1, 191))
        inf = true;
      else
        st = LB_ST_BAD_ENCODING;
    } else if (!fp_read_masked(v[1], b, false) || !fp_read_masked(v[0], b + 48, false) ||
               !fp_read_masked(v[3], b + 96, false) || !fp_read_masked(v[2], b + 144, false)) {
      st = LB_ST_BAD_ENCODING;
    }
  }
  if (st != LB_ST_OK || inf) {
#pragma unroll
    for (int c = 0; c < 4; c++) fp_zero(v[c]);
  }
#pragma unroll
  for (int c = 0; c < 4; c++) {
#pragma unroll
    for (int j = 0; j < 12; j++) in16[(size_t)(4 * i + c) * 16 + j] = v[c].l[j];
#pragma unroll
    for (int j = 12; j < 16; j++) in16[(size_t)(4 * i + c) * 16 + j] = 0u;
  }
  fl[3 * i] = inf ? 1u : 0u;  // (lpgen/bls.py SIG_DECODE_FLAGS order)
  fl[3 * i + 1] = sign ? 1u : 0u;
  fl[3 * i + 2] = comp ? 1u : 0u;
  pre[i] = st;
}

__global__ void __launch_bounds__(LB_LP_DEC_ROWS * 16) k_lp_dec(const uint32_t* __restrict__ prog, uint32_t n,
                                                                const uint32_t* __restrict__ in16,
                                                                const uint32_t* __restrict__ fl,
                                                                uint32_t* __restrict__ out16,
                                                                uint32_t* __restrict__ ofl) {
  __shared__ LpSharedT<LB_LP_DEC_REGS> S;
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
  const uint32_t* in = in16 + (size_t)b * 4 * 16;
  lp_run(S, prog, in, 0xffffffffu, in, fl + 3 * (size_t)b, out16 + (size_t)b * 2 * 16, ofl + 2 * (size_t)b);
}

__global__ void __launch_bounds__(256) k_sm_dec_finish(uint32_t n, const uint8_t* __restrict__ pre,
                                                       const uint32_t* __restrict__ in16,
                                                       const uint32_t* __restrict__ fl,
                                                       const uint32_t* __restrict__ out16,
                                                       const uint32_t* __restrict__ ofl, g2j* __restrict__ sig,
                                                       uint8_t* __restrict__ status,
                                                       const uint8_t* __restrict__ single_flag) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t st = pre[i];
  // (k_decode_sigs' single-set rule: a 1-set request's core verify rejects the infinite signature)
  if (st == LB_ST_OK && fl[3 * i] && single_flag && single_flag[i]) st = LB_ST_ZERO_SIGNATURE;
  g2j P;
  jac_set_inf(P);  // (k_decode_sigs: infinity unless the encoding decoded; infinity itself is OK)
  if (st == LB_ST_OK && !fl[3 * i]) {
    if (!ofl[2 * i]) {
      st = LB_ST_NOT_ON_CURVE;
    } else {
#pragma unroll
      for (int j = 0; j < 12; j++) {
        P.X.c0.l[j] = in16[(size_t)(4 * i) * 16 + j];
        P.X.c1.l[j] = in16[(size_t)(4 * i + 1) * 16 + j];
        P.Y.c0.l[j] = out16[(size_t)(2 * i) * 16 + j];
        P.Y.c1.l[j] = out16[(size_t)(2 * i + 1) * 16 + j];
      }
      fone(P.Z);
      if (!ofl[2 * i + 1]) st = LB_ST_NOT_IN_GROUP;  // (the point kept, as k_decode_sigs keeps it)
    }
  }
  sig[i] = P;
  status[i] = st;
}

__global__ void __launch_bounds__(256) k_hf_prep(uint32_t n, const g2j* __restrict__ q, uint32_t* __restrict__ in16) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // (set, record): 12 records a set
  if (t >= n * 12u) return;
  const uint32_t i = t / 12u, c = t % 12u;
  const fp v = (&q[2 * i + c / 6u].X.c0)[c % 6u];
#pragma unroll
  for (int j = 0; j < 12; j++) in16[(size_t)t * 16 + j] = v.l[j];
#pragma unroll
  for (int j = 12; j < 16; j++) in16[(size_t)t * 16 + j] = 0u;
}

__global__ void __launch_bounds__(LB_LP_HF_ROWS * 16) k_lp_hf(const uint32_t* __restrict__ prog, uint32_t n,
                                                              const uint32_t* __restrict__ in16,
                                                              uint32_t* __restrict__ out16) {
  __shared__ LpSharedT<LB_LP_DEC_REGS> S;
  __shared__ uint32_t s_fl[4];
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
  const uint32_t* in = in16 + (size_t)b * 12 * 16;
  lp_run(S, prog, in, 0xffffffffu, in, nullptr, out16 + (size_t)b * 6 * 16, s_fl);
}

__global__ void __launch_bounds__(256) k_hu_prep(uint32_t n, const uint8_t* __restrict__ msgs,
                                                 uint32_t* __restrict__ in16) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t m[32];
  for (int k = 0; k < 32; k++) m[k] = msgs[(size_t)i * 32 + k];
  fp2 u[2];
  hash_to_field_fp2_2(u, m);
  uint32_t* rec = in16 + (size_t)i * 4 * 16;
  const fp* v[4] = {&u[0].c0, &u[0].c1, &u[1].c0, &u[1].c1};
#pragma unroll
  for (int k = 0; k < 4; k++) {
#pragma unroll
    for (int j = 0; j < 12; j++) rec[16 * k + j] = v[k]->l[j];
#pragma unroll
    for (int j = 12; j < 16; j++) rec[16 * k + j] = 0u;
  }
}

__global__ void __launch_bounds__(LB_LP_HF_ROWS * 16) k_lp_hash(const uint32_t* __restrict__ prog, uint32_t n,
                                                                const uint32_t* __restrict__ in16,
                                                                uint32_t* __restrict__ out16) {
  __shared__ LpSharedT<LB_LP_HASH_REGS> S;
  __shared__ uint32_t s_fl[4];
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
  const uint32_t* in = in16 + (size_t)b * 4 * 16;
  lp_run(S, prog, in, 0xffffffffu, in, nullptr, out16 + (size_t)b * 6 * 16, s_fl);
}

__global__ void __launch_bounds__(256) k_hf_finish(uint32_t n, const uint32_t* __restrict__ out16,
                                                   g2j* __restrict__ h) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // (set, coordinate): 6 a set
  if (t >= n * 6u) return;
  const uint32_t i = t / 6u, c = t % 6u;
  fp v;
#pragma unroll
  for (int j = 0; j < 12; j++) v.l[j] = out16[(size_t)t * 16 + j];
  (&h[i].X.c0)[c] = v;
}

// slot q -> (row i, position r) of the steps row layout (k_steps.hip slot_row)
LB_DEV void lines_slot_row(const Rows& R, uint32_t q, uint32_t& i, uint32_t& r) {
  uint32_t lo = 0, hi = R.meta[0];
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (R.rowoff[mid] <= q)
      lo = mid;
    else
      hi = mid;
  }
  i = lo;
  r = q - R.rowoff[lo];
}

__global__ void __launch_bounds__(256) k_lines_prep(uint32_t n_sets, Rows R, const uint32_t* __restrict__ req_off,
                                                    const g1j* __restrict__ P, const g2j* __restrict__ Q,
                                                    uint32_t* __restrict__ in16) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;  // (slot, record): P's 3 + H's 6
  if (t >= n_sets * 9u) return;
  const uint32_t q = t / 9u, c = t % 9u;
  uint32_t i, r;
  lines_slot_row(R, q, i, r);
  const uint32_t s = req_off[R.inv[r]] + i;
  const fp v = c < 3u ? (&P[s].X)[c] : (&Q[s].X.c0)[c - 3u];
#pragma unroll
  for (int j = 0; j < 12; j++) in16[(size_t)t * 16 + j] = v.l[j];
#pragma unroll
  for (int j = 12; j < 16; j++) in16[(size_t)t * 16 + j] = 0u;
}

__global__ void __launch_bounds__(LB_LP_HF_ROWS * 16) k_lp_lines(const uint32_t* __restrict__ prog, uint32_t n,
                                                                 const uint32_t* __restrict__ in16,
                                                                 uint32_t* __restrict__ out16) {
  __shared__ LpSharedRtail S;
  __shared__ uint32_t s_fl[4];
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
  const uint32_t* in = in16 + (size_t)b * 9 * 16;
  lp_run(S, prog, in, 0xffffffffu, in, nullptr, out16 + (size_t)b * LB_LP_LINES_NOUT * 16, s_fl);
}

__global__ void __launch_bounds__(256) k_lines_store(uint32_t n_sets, uint32_t n_pairs, const uint32_t* __restrict__ out16,
                                                     uint32_t* __restrict__ lines) {
  // thread (word w of line j, slot q): consecutive threads take consecutive slots, so the SoA
  // stores coalesce (the record reads stride by a slot's 408 records)
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)n_sets * LB_MILLER_LINES * 72) return;
  const uint32_t q = (uint32_t)(t % n_sets), jw = (uint32_t)(t / n_sets);  // jw = j * 72 + w
  const uint32_t j = jw / 72u, w = jw % 72u, e = w / 12u, limb = w % 12u;
  lines[(size_t)jw * n_pairs + q] = out16[((size_t)q * LB_LP_LINES_NOUT + j * 6u + e) * 16 + limb];
}

__global__ void __launch_bounds__(64) k_records_to_fp12(const uint32_t* __restrict__ in16, fp12* __restrict__ F) {
  const uint32_t i = threadIdx.x;
  if (i >= 12) return;
  fp v;
#pragma unroll
  for (int j = 0; j < 12; j++) v.l[j] = in16[16 * i + j];
  (&F->c0.c0.c0)[i] = v;
}

// Test / stage entry: instance b runs `prog` on in[b * in_stride ...].
__global__ void __launch_bounds__(LB_LP_TPB) k_lp_program(const uint32_t* __restrict__ prog, uint32_t n,
                                                          const uint32_t* __restrict__ in, uint32_t in_stride,
                                                          const uint32_t* __restrict__ in_flags, uint32_t flag_stride,
                                                          uint32_t* __restrict__ out, uint32_t out_stride,
                                                          uint32_t* __restrict__ out_flags, uint32_t oflag_stride,
                                                          unsigned long long* __restrict__ stamps) {
  __shared__ LpShared S;
  const uint32_t b = blockIdx.x;
  if (b >= n) return;
  const uint32_t* ia = in + (size_t)b * in_stride;
  lp_run(S, prog, ia, 0xffffffffu, ia, in_flags + (size_t)b * flag_stride, out + (size_t)b * out_stride,
         out_flags + (size_t)b * oflag_stride, b == 0 ? stamps : nullptr);
}

}  // namespace lb
