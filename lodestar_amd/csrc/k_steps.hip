// Step-major Miller accumulation ("steps" organisation of the stored lines).
// Part of the MI355X BLS verification pipeline; see bls_host.hip for the DAG.
//
// The Miller value of a request is F_k = prod_j L_{k,j}^(2^(62 - lvl(j))) with
// L_{k,j} = prod_{pairs i of k} l_{i,j} (68 lines j per pair; lvl(j) = number of
// Fp12 squarings before line j).  The pair-major accumulation (k_miller_acc)
// gives every lane a few pairs and all 68 steps, so each lane squares its
// accumulator 62 times.  Here a lane takes 68 consecutive lines of its request
// in step-major order -- lines t in [68 l, 68 l + 68) with j = t / n_k,
// i = t mod n_k -- so a lane of a >= 68-set request spans at most two steps and
// squares at most once; a request has n_k lanes (one per set, as before; a lone
// mid-size call splits each in Rows::split lanes of 68 / split lines).
// The squarings left are those of one Horner chain over the 63 levels per
// merged check (folded into the merged-check round program, k_lp_mtail; or
// k_horner_all, one wave) or per request on the failure path (k_req_horner).
// Work per pair: 68 x 11.5 Fp2 products instead of 68 x 17.5 (two pairs per
// lane) or 68 x 25 (one pair per lane).
//
// Row layout: requests are ordered by size, descending (position pos(k)); row i
// holds pair i of every request with n_k > i, so pair (k, i) lives at slot
// rowoff[i] + pos(k) and the slots are exactly [0, n_sets).  A wave of 64
// consecutive slots is 64 requests at the same lane index l: with equal sizes
// every lane reads line (j, i) of its request at the same moment and the SoA
// loads (word w of line j of slot q at lines[(j*72 + w)*n_pairs + q]) coalesce.
#include "bls_kernels.h"
#include "bls_wc12.h"

namespace lb {

// Levels of the 68 lines (loop order of miller_lines: the doubling line of bit
// i = 62..0, then the addition line when bit i of |x| is set) and the first
// line of each level (first[63] = 68).
struct StepTab {
  uint8_t lvl[LB_MILLER_LINES];
  uint8_t first[64];
};
constexpr StepTab make_step_tab() {
  StepTab t{};
  int j = 0;
  for (int i = 62; i >= 0; i--) {
    const int l = 62 - i;
    t.first[l] = (uint8_t)j;
    t.lvl[j++] = (uint8_t)l;
    if ((LB_X_ABS >> i) & 1ull) t.lvl[j++] = (uint8_t)l;
  }
  t.first[63] = (uint8_t)j;
  return t;
}
__constant__ StepTab c_steps = make_step_tab();
static_assert(make_step_tab().first[63] == LB_MILLER_LINES, "68 Miller lines");

// ---- size-descending order of the requests and the row offsets ----------
// hist[n] = number of requests of n sets (n <= n_sets; zeroed by the host)
__global__ void __launch_bounds__(256) k_rows_hist(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                   uint32_t* __restrict__ hist) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_req) atomicAdd(&hist[req_off[k + 1] - req_off[k]], 1u);
}

// gt[n] = #requests with more than n sets (= the first position of the size-n
// requests), rowoff[i] = sum_{i' < i} gt[i'] for i in [0, n_sets], meta[0] =
// number of rows (the largest request size).  One workgroup of 1024 threads.
__global__ void __launch_bounds__(1024) k_rows_scan(uint32_t n_sets, const uint32_t* __restrict__ hist,
                                                    uint32_t* __restrict__ gt, uint32_t* __restrict__ rowoff,
                                                    uint32_t* __restrict__ meta) {
  __shared__ uint32_t part[1024];
  __shared__ uint32_t rmax;
  const uint32_t m = n_sets + 1, tid = threadIdx.x;
  const uint32_t per = (m + 1023) / 1024, b = tid * per, e = b + per < m ? b + per : m;
  if (tid == 0) rmax = 0;
  // suffix sums of hist: gt[n] = sum_{n' > n} hist[n']
  uint32_t s = 0;
  for (uint32_t n = b; n < e; n++) s += hist[n];
  part[tid] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive suffix scan of part
    const uint32_t v = tid + d < 1024 ? part[tid + d] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t acc = tid + 1 < 1024 ? part[tid + 1] : 0u;  // sum over the segments after this one
  for (uint32_t n = e; n-- > b;) {
    gt[n] = acc;
    acc += hist[n];
    if (hist[n] && n > 0) atomicMax(&rmax, n);
  }
  __syncthreads();
  // prefix sums of gt: rowoff[i] = sum_{i' < i} gt[i']
  s = 0;
  for (uint32_t n = b; n < e; n++) s += gt[n];
  part[tid] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive prefix scan
    const uint32_t v = tid >= d ? part[tid - d] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  acc = tid ? part[tid - 1] : 0u;
  for (uint32_t n = b; n < e; n++) {
    rowoff[n] = acc;
    acc += gt[n];
  }
  if (tid == 0) meta[0] = rmax;
}

// pos[k] = position of request k in the size-descending order, inv[pos] = k
// (within one size the order is that of the atomics: any order keeps rows dense)
__global__ void __launch_bounds__(256) k_rows_pos(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                  const uint32_t* __restrict__ gt, uint32_t* __restrict__ cursor,
                                                  uint32_t* __restrict__ pos, uint32_t* __restrict__ inv) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_req) return;
  const uint32_t n = req_off[k + 1] - req_off[k];
  const uint32_t p = gt[n] + atomicAdd(&cursor[n], 1u);
  pos[k] = p;
  inv[p] = k;
}

// slot q -> (row i, position r): the largest i < rows with rowoff[i] <= q
LB_DEV void slot_row(const Rows& R, uint32_t q, uint32_t& i, uint32_t& r) {
  uint32_t lo = 0, hi = R.meta[0];  // rows [lo, hi)
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

// Lines of every set pair, stored at its slot: lane q is slot q (coalesced stores).
// (LB_LINES_QREGS: Q held in registers; default: the affine H(m) replaces its Jacobian
// form in Q -- which nothing reads after this kernel -- and the Miller loop re-reads it at
// its 5 addition steps, miller_lines_qmem)
template <int WAVES>
__global__ void __launch_bounds__(TPB, WAVES) k_lines_rows(uint32_t n_sets, uint32_t n_pairs, Rows R,
                                                           const uint32_t* __restrict__ req_off,
                                                           const g1j* __restrict__ P, g2j* __restrict__ Q,
                                                           uint32_t* __restrict__ lines) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_sets) return;
  uint32_t i, r;
  slot_row(R, q, i, r);
  const uint32_t s = req_off[R.inv[r]] + i;
  g1a p;
#ifdef LB_LINES_QREGS
  g2a h;
  jac_pair_to_aff(p, h, P[s], Q[s]);
  miller_lines(p, h, lines, n_pairs, q);
#else
  bool h_inf;
  {
    g2a h;
    jac_pair_to_aff(p, h, P[s], Q[s]);
    h_inf = h.inf;
    if (!p.inf && !h.inf) {
      Q[s].X = h.x;
      Q[s].Y = h.y;
    }
  }
  if (p.inf || h_inf) {
    g2a none;
    none.inf = true;
    miller_lines(p, none, lines, n_pairs, q);  // (unit lines)
  } else {
    miller_lines_qmem(p, Q + s, lines, n_pairs, q);
  }
#endif
}

// Request status of the steps organisation (what k_miller_acc reduces on the
// side): bad = empty request or any set not OK; the rejection code.  One wave
// per request, grid-stride.
__global__ void __launch_bounds__(TPB) k_req_status(uint32_t n_req, const uint32_t* __restrict__ req_off,
                                                    const uint8_t* __restrict__ sig_status,
                                                    const uint8_t* __restrict__ pk_status,
                                                    uint8_t* __restrict__ req_bad, uint8_t* __restrict__ req_err) {
  for (uint32_t k = blockIdx.x; k < n_req; k += gridDim.x) {
    const uint32_t a = req_off[k], b = req_off[k + 1];
    bool bad = false, empty_agg = false, bad_pk = false;
    for (uint32_t i = a + threadIdx.x; i < b; i += TPB) {
      const uint8_t ss = sig_status[i], ps = pk_status[i];
      bad |= ss != LB_ST_OK || ps != LB_ST_OK;
      empty_agg |= ps == LB_ST_EMPTY_AGGREGATE;
      bad_pk |= ps == LB_ST_BAD_ENCODING;
    }
    bad = __any(bad);
    empty_agg = __any(empty_agg);
    bad_pk = __any(bad_pk);
    if (threadIdx.x == 0) {
      req_bad[k] = (bad || a == b) ? 1 : 0;
      req_err[k] = empty_agg ? LB_REQ_EMPTY_AGGREGATE : bad_pk ? LB_REQ_BAD_PUBKEY : LB_REQ_OK;
    }
  }
}

// G of lane (request k, index l): the Horner product of its 68 lines, at the
// level of its last line.  SoA over slots: word w at G[w * n_sets + q].
LB_DEV void g_put(uint32_t* __restrict__ G, uint32_t n_sets, uint32_t q, const fp12& f) {
  const uint32_t* v = &f.c0.c0.c0.l[0];
#pragma unroll
  for (int w = 0; w < 144; w++) G[(size_t)w * n_sets + q] = v[w];
}
LB_DEV void g_get(fp12& f, const uint32_t* __restrict__ G, uint32_t n_sets, uint32_t q) {
  uint32_t* v = &f.c0.c0.c0.l[0];
#pragma unroll
  for (int w = 0; w < 144; w++) v[w] = G[(size_t)w * n_sets + q];
}

// The lane's 68 lines (from line t0 = 68 l of its n-set request, step-major),
// accumulated with the in-lane Horner rule; Acc holds the accumulator: registers
// (AccReg) or this lane's LDS record (AccLds: each half of f read where it is used,
// so its 144 registers leave the peak register set of the sparse product).
struct AccReg {
  fp12 f;
  LB_DEV void sqr() { fp12_sqr(f, f); }
  LB_DEV void mul_line(const fp2& l0, const fp2& l1, const fp2& l4) { fp12_mul_line(f, f, l0, l1, l4); }
  LB_DEV void mul_sparse2(const fp6& x, const fp2& y1, const fp2& y2) { fp12_mul_by_sparse2(f, f, x, y1, y2); }
  LB_DEV void set(const fp12& v) { f = v; }
  LB_DEV void get(fp12& v) const { v = f; }
};
#define LB_LDS_FENCE() asm volatile("" ::: "memory")
struct AccLds {
  fp12* A;
  LB_DEV void sqr() {
    fp12 t = *A;
    fp12_sqr(t, t);
    *A = t;
    LB_LDS_FENCE();
  }
  LB_DEV void mul_line(const fp2& l0, const fp2& l1, const fp2& l4) {
    fp12 t = *A;
    fp12_mul_line(t, t, l0, l1, l4);
    *A = t;
    LB_LDS_FENCE();
  }
  // fp12_mul_by_sparse2's formulas (17 Fp2 products), halves of f loaded per use
  LB_DEV void mul_sparse2(const fp6& x, const fp2& y1, const fp2& y2) {
    fp6 t1, s, t0, sm;
    {
      const fp6 c1 = A->c1;
      fp6_mul_12(t1, c1, y1, y2);
    }
    LB_LDS_FENCE();
    {
      const fp6 c0 = A->c0, c1 = A->c1;
      fp6_add(s, c0, c1);
    }
    sm.c0 = x.c0;
    fp2_add(sm.c1, x.c1, y1);
    fp2_add(sm.c2, x.c2, y2);
    fp6_mul(s, s, sm);
    LB_LDS_FENCE();
    {
      const fp6 c0 = A->c0;
      fp6_mul(t0, c0, x);
    }
    fp6_sub(s, s, t0);
    fp6_sub(s, s, t1);
    A->c1 = s;
    fp6_mul_v(t1, t1);
    fp6_add(t0, t0, t1);
    A->c0 = t0;
    LB_LDS_FENCE();
  }
  LB_DEV void set(const fp12& v) {
    *A = v;
    LB_LDS_FENCE();
  }
  LB_DEV void get(fp12& v) const { v = *A; }
};

template <bool PAIRED, class Acc>
LB_DEV void step_lines(Acc& acc, const uint32_t* __restrict__ lines, uint32_t n_pairs, const Rows& R, uint32_t r,
                       uint32_t n, uint32_t t0, uint32_t cnt) {
  uint32_t j = t0 / n, i = t0 - j * n;
  int lvl = c_steps.lvl[j];
  bool have = false;
  fp2 l0, l1, l4;
#pragma unroll 1
  for (uint32_t c = 0; c < cnt;) {
    const int lj = c_steps.lvl[j];
    if (lj != lvl) {  // one doubling step further: one squaring
      if (have) acc.sqr();
      lvl = lj;
    }
    const uint32_t qa = R.rowoff[i] + r;
    if (PAIRED && i + 1 < n && c + 1 < cnt) {  // two lines of the same step
      const uint32_t qb = R.rowoff[i + 1] + r;
      fp2 m0, m1, m4, y1, y2;
      fp6 x;
      line_get(lines, n_pairs, qa, (int)j, l0, l1, l4);
      line_get(lines, n_pairs, qb, (int)j, m0, m1, m4);
      line_mul_line(x, y1, y2, l0, l1, l4, m0, m1, m4);
      if (have) {
        acc.mul_sparse2(x, y1, y2);
      } else {
        fp12 v;
        v.c0 = x;
        fp2_zero(v.c1.c0);
        v.c1.c1 = y1;
        v.c1.c2 = y2;
        acc.set(v);
        have = true;
      }
      i += 2;
      c += 2;
    } else {
      line_get(lines, n_pairs, qa, (int)j, l0, l1, l4);
      if (have) {
        acc.mul_line(l0, l1, l4);
      } else {
        fp12 v;
        fp6_zero(v.c0);
        fp6_zero(v.c1);
        v.c0.c0 = l0;
        v.c0.c1 = l1;
        v.c1.c1 = l4;
        acc.set(v);
        have = true;
      }
      i += 1;
      c += 1;
    }
    if (i >= n) {
      i -= n;
      j++;
    }
  }
}

// MODE 0: accumulator in registers, two lines of a step through the sparse x sparse
// product (default); 1: the accumulator in LDS (one 592-byte record per lane, 37 KB per
// wave, four waves per CU at one wave per SIMD; LB_STEP_MODE=1); 2: registers, one line
// at a time (13 Fp2 products per line instead of 11.5, a smaller live set; LB_STEP_MODE=2).
// WAVES: the occupancy target (1: 512 registers, the accumulator in registers; 2: 256,
// spilling, but a SIMD interleaves two waves' VALU issue: one wave alone issues a VALU
// instruction every 4 cycles, two every 2 (MI355X_MICROARCH.md); LB_STEP_WAVES=2).
template <int MODE, int WAVES>
__global__ void __launch_bounds__(TPB, WAVES) k_step_acc(uint32_t n_sets, uint32_t n_pairs, Rows R,
                                                            const uint32_t* __restrict__ req_off,
                                                            const uint32_t* __restrict__ lines,
                                                            uint32_t* __restrict__ G) {
  __shared__ LdsRec<fp12> sacc[MODE == 1 ? TPB : 1];
  // thread t: part h of slot q's lane (R.split parts of 68 / split lines; G slot q split + h)
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t q = t / R.split, h = t - q * R.split;
  if (q >= n_sets) return;
  uint32_t l, r;
  slot_row(R, q, l, r);
  const uint32_t k = R.inv[r];
  const uint32_t n = req_off[k + 1] - req_off[k];
  const uint32_t L = (uint32_t)LB_MILLER_LINES / R.split, t0 = (uint32_t)LB_MILLER_LINES * l + L * h;
  fp12 out;
  if constexpr (MODE == 1) {
    AccLds acc{&sacc[threadIdx.x].v};
    step_lines<true>(acc, lines, n_pairs, R, r, n, t0, L);
    acc.get(out);
  } else {
    AccReg acc;
    step_lines<MODE == 0>(acc, lines, n_pairs, R, r, n, t0, L);
    acc.get(out);
  }
  g_put(G, n_sets * R.split, t, out);
}

// [lo, hi): the (virtual) lane indices v of an n-set request whose last line has level lvl;
// lane v covers lines [v L, v L + L) with L = 68 / split (split v-lanes per set)
LB_DEV void level_lanes(uint32_t n, int lvl, uint32_t& lo, uint32_t& hi, uint32_t split = 1) {
  const int64_t L = LB_MILLER_LINES / (int64_t)split;
  const int64_t a = (int64_t)c_steps.first[lvl] * n - (L - 1);
  const int64_t b = (int64_t)c_steps.first[lvl + 1] * n - (L - 1);
  lo = a <= 0 ? 0u : (uint32_t)((a + L - 1) / L);
  hi = b <= 0 ? 0u : (uint32_t)((b + L - 1) / L);
  if (hi > n * split) hi = n * split;
  if (lo > hi) lo = hi;
}
// G slot of lane v of the request at position r (k_step_acc: slot q's part h at q split + h)
LB_DEV uint32_t g_slot(const Rows& R, uint32_t v, uint32_t r) {
  const uint32_t l = v / R.split;
  return (R.rowoff[l] + r) * R.split + (v - l * R.split);
}

// Merged check: P[lvl] = prod over the good requests' lanes at level lvl of G,
// times the lines of level lvl of the merged pair (-g1, S_all) (slot s_pair).
// One workgroup of LB_LVL_TPB threads per level: strided products, LDS tree.
static constexpr int LB_LVL_TPB = 256;
__global__ void __launch_bounds__(LB_LVL_TPB, 1) k_level_prod(uint32_t n_req, uint32_t n_sets, uint32_t n_pairs,
                                                              uint32_t s_pair, Rows R,
                                                              const uint32_t* __restrict__ req_off,
                                                              const uint32_t* __restrict__ G,
                                                              const uint8_t* __restrict__ req_bad,
                                                              const uint32_t* __restrict__ lines,
                                                              fp12* __restrict__ Pl) {
  __shared__ LdsRec<fp12> sh[LB_LVL_TPB];
  __shared__ uint8_t has[LB_LVL_TPB];
  const int lvl = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  fp12 acc;
  bool have = false;
  auto take = [&](uint32_t q) {
    fp12 g;
    g_get(g, G, n_sets * R.split, q);
    if (have) {
      fp12_mul(acc, acc, g);
    } else {
      acc = g;
      have = true;
    }
  };
  // requests in size-descending order: the large ones first, their lanes of this level
  // spread over all threads (a request of thousands of sets has tens of lanes per level),
  // then one request per thread
  uint32_t r0 = 0;
  for (; r0 < n_req; r0++) {
    const uint32_t k = R.inv[r0], n = req_off[k + 1] - req_off[k];
    if (n * R.split <= 16u * LB_MILLER_LINES) break;
    if (req_bad[k]) continue;
    uint32_t lo, hi;
    level_lanes(n, lvl, lo, hi, R.split);
    for (uint32_t l = lo + tid; l < hi; l += LB_LVL_TPB) take(g_slot(R, l, r0));
  }
  for (uint32_t r = r0 + tid; r < n_req; r += LB_LVL_TPB) {
    const uint32_t k = R.inv[r];
    if (req_bad[k]) continue;
    uint32_t lo, hi;
    level_lanes(req_off[k + 1] - req_off[k], lvl, lo, hi, R.split);
    for (uint32_t l = lo; l < hi; l++) take(g_slot(R, l, r));
  }
  if (have) sh[tid].v = acc;
  has[tid] = have ? 1 : 0;
  __syncthreads();
  for (uint32_t s = LB_LVL_TPB / 2; s > 0; s >>= 1) {
    if (tid < s && has[tid + s]) {
      fp12 o = sh[tid + s].v;
      if (has[tid]) {
        fp12 m = sh[tid].v;
        fp12_mul(m, m, o);
        sh[tid].v = m;
      } else {
        sh[tid].v = o;
        has[tid] = 1;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    have = has[0] != 0;
    if (have) acc = sh[0].v;
    if (s_pair != 0xffffffffu) {
      for (int j = c_steps.first[lvl]; j < c_steps.first[lvl + 1]; j++) {
        fp2 l0, l1, l4;
        line_get(lines, n_pairs, s_pair, j, l0, l1, l4);
        if (have) {
          fp12_mul_line(acc, acc, l0, l1, l4);
        } else {
          fp6_zero(acc.c0);
          fp6_zero(acc.c1);
          acc.c0.c0 = l0;
          acc.c0.c1 = l1;
          acc.c1.c1 = l4;
          have = true;
        }
      }
    }
    if (!have) fp12_one(acc);
    Pl[lvl] = acc;
  }
}

// The level products in two stages (round 6; LB_LEVEL=0 restores k_level_prod).  k_level_prod's
// 256 threads per level end in an LDS tree of eight single-lane Fp12 products (~150 us each on
// one lane): ~11 dependent lane products, 1.7 ms for a 65,536-set call.  Here:
//   k_level_part, grid (B, 63): the level's per = 256 B threads dealt over the requests (per /
//     n_req threads each, each taking every (per / n_req)-th lane of its request at this level;
//     one request per thread when there are more) -- one or two lane products -- and stores
//     its product, or nothing, at part[lvl * per + g];
//   k_level_wc, grid (ceil(per_in / 8), 63), one wave each: the product of a group of 8
//     partials as wave-cooperative Fp12 products (~10 us each, bls_wc12.h), until one value
//     per level is left; the last pass (Pl given) multiplies in the merged pair's lines of
//     the level (s_pair, unless the round program does) and writes P[lvl].
__global__ void __launch_bounds__(256, 1) k_level_part(uint32_t n_req, uint32_t n_sets, Rows R,
                                                       const uint32_t* __restrict__ req_off,
                                                       const uint32_t* __restrict__ G,
                                                       const uint8_t* __restrict__ req_bad, uint32_t per,
                                                       fp12* __restrict__ part, uint8_t* __restrict__ has) {
  const int lvl = blockIdx.y;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= per) return;
  fp12 acc;
  bool have = false;
  auto take = [&](uint32_t q) {
    fp12 v;
    g_get(v, G, n_sets * R.split, q);
    if (have) {
      fp12_mul(acc, acc, v);
    } else {
      acc = v;
      have = true;
    }
  };
  // T = per / n_req threads per request (consecutive threads: consecutive requests at the same
  // lane index -- coalesced G loads), thread j of a request taking its lanes j, j + T, ...; with
  // more requests than threads, one request per thread and all its lanes of the level
  const uint32_t T = per >= n_req ? per / n_req : 0u;
  if (T) {
    if (g < n_req * T) {
      const uint32_t r = g % n_req, j = g / n_req, k = R.inv[r];
      if (!req_bad[k]) {
        uint32_t lo, hi;
        level_lanes(req_off[k + 1] - req_off[k], lvl, lo, hi, R.split);
        for (uint32_t l = lo + j; l < hi; l += T) take(g_slot(R, l, r));
      }
    }
  } else {
    for (uint32_t r = g; r < n_req; r += per) {
      const uint32_t k = R.inv[r];
      if (req_bad[k]) continue;
      uint32_t lo, hi;
      level_lanes(req_off[k + 1] - req_off[k], lvl, lo, hi, R.split);
      for (uint32_t l = lo; l < hi; l++) take(g_slot(R, l, r));
    }
  }
  const size_t o = (size_t)lvl * per + g;
  if (have) part[o] = acc;
  has[o] = have ? 1 : 0;
}

__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_level_wc(uint32_t per_in, const fp12* __restrict__ in,
                                                             const uint8_t* __restrict__ in_has, uint32_t per_out,
                                                             fp12* __restrict__ out, uint8_t* __restrict__ out_has,
                                                             uint32_t n_pairs, uint32_t s_pair,
                                                             const uint32_t* __restrict__ lines, fp12* __restrict__ Pl) {
  __shared__ wc_smem S;
  const int lvl = blockIdx.y;
  const uint32_t c = blockIdx.x;
  const uint32_t a = c * LB_LVL_GROUP, b = a + LB_LVL_GROUP < per_in ? a + LB_LVL_GROUP : per_in;
  wc_init_tables(S);
  bool have = false;
#pragma unroll 1
  for (uint32_t i = a; i < b; i++) {
    const size_t o = (size_t)lvl * per_in + i;
    if (!in_has[o]) continue;  // (uniform: one wave per group)
    wc_load12(S, have ? WC_T0 : WC_ACC, in[o]);
    if (have) wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, WC_T0);
    have = true;
  }
  if (!Pl) {
    if (have && threadIdx.x < 12) (&out[(size_t)lvl * per_out + c].c0.c0.c0)[threadIdx.x] = S.slot[WC_ACC][threadIdx.x];
    if (threadIdx.x == 0) out_has[(size_t)lvl * per_out + c] = have ? 1 : 0;
    return;
  }
  if (s_pair != 0xffffffffu) {
    if (!have) wc_set_one(S, WC_ACC);
    have = true;
#pragma unroll 1
    for (int j = c_steps.first[lvl]; j < c_steps.first[lvl + 1]; j++) {
      if (threadIdx.x < 6) {
        const uint32_t* p = lines + ((size_t)j * 72 + 12 * threadIdx.x) * n_pairs + s_pair;
        fp v;
        for (int w = 0; w < 12; w++) v.l[w] = p[(size_t)w * n_pairs];
        S.slot[WC_LINE][threadIdx.x] = v;
      }
      __syncthreads();
      wc_apply(S, LB_WC_LINE, WC_ACC, WC_ACC, WC_LINE);
    }
  }
  if (!have) wc_set_one(S, WC_ACC);
  if (threadIdx.x < 12) (&Pl[lvl].c0.c0.c0)[threadIdx.x] = S.slot[WC_ACC][threadIdx.x];
}

// F_all = conj(Horner over the 63 levels of P[lvl]) (x < 0): one wave, wave-
// cooperative Fp12 (62 squarings + 62 products on the merged check's path).
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_horner_all(const fp12* __restrict__ Pl, fp12* __restrict__ F_all) {
  __shared__ wc_smem S;
  wc_init_tables(S);
  wc_load12(S, WC_ACC, Pl[0]);
#pragma unroll 1
  for (int l = 1; l < 63; l++) {
    wc_apply(S, LB_WC_SQR, WC_ACC, WC_ACC, WC_ACC);
    wc_load12(S, WC_T0, Pl[l]);
    wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, WC_T0);
  }
  wc_apply(S, LB_WC_CONJ, WC_ACC, WC_ACC, WC_ACC);
  if (threadIdx.x < 12) (&F_all->c0.c0.c0)[threadIdx.x] = S.slot[WC_ACC][threadIdx.x];
}

// Per-request F_k (the failure path of a merged check, or every request of an
// unmerged call): one wave per request, Horner over its lanes' G values.
// skip (optional): nonzero when the merged check passed -> nothing to do.
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_req_horner(uint32_t n_req, uint32_t n_sets, Rows R,
                                                             const uint32_t* __restrict__ req_off,
                                                             const uint32_t* __restrict__ G,
                                                             const uint8_t* __restrict__ req_bad,
                                                             fp12* __restrict__ F, const uint8_t* __restrict__ skip) {
  // (a split accumulation: one wave per (request, part h) over the lanes v = h mod split -- the
  // conjugated Horner value is multiplicative over any partition of the lanes, so each wave
  // runs the squaring chain of its share and k_req_join multiplies the parts; F: split per request)
  __shared__ wc_smem S;
  const uint32_t k = blockIdx.x / R.split, h = blockIdx.x - k * R.split;
  if (k >= n_req || (skip && *skip) || req_bad[k]) return;  // (uniform per workgroup)
  const uint32_t n = req_off[k + 1] - req_off[k], r = R.pos[k];
  wc_init_tables(S);
  bool started = false;
#pragma unroll 1
  for (int lvl = 0; lvl < 63; lvl++) {
    if (started) wc_apply(S, LB_WC_SQR, WC_ACC, WC_ACC, WC_ACC);
    uint32_t lo, hi;
    level_lanes(n, lvl, lo, hi, R.split);
    for (uint32_t l = lo + (h + R.split - lo % R.split) % R.split; l < hi; l += R.split) {
      const int dst = started ? WC_T0 : WC_ACC;
      if (threadIdx.x < 12) {
        fp v;
        const size_t q = g_slot(R, l, r);
#pragma unroll
        for (int w = 0; w < 12; w++) v.l[w] = G[(size_t)(12 * threadIdx.x + w) * n_sets * R.split + q];
        S.slot[dst][threadIdx.x] = v;
      }
      __syncthreads();
      if (started) wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, WC_T0);
      started = true;
    }
  }
  if (!started) wc_set_one(S, WC_ACC);
  wc_apply(S, LB_WC_CONJ, WC_ACC, WC_ACC, WC_ACC);
  if (threadIdx.x < 12) (&F[blockIdx.x].c0.c0.c0)[threadIdx.x] = S.slot[WC_ACC][threadIdx.x];
}

// F[k] = the product of k_req_horner's `split` parts of request k (one wave per request)
__global__ void __launch_bounds__(TPB, LB_W_TAIL) k_req_join(uint32_t n_req, uint32_t split,
                                                           const fp12* __restrict__ parts,
                                                           const uint8_t* __restrict__ req_bad,
                                                           fp12* __restrict__ F, const uint8_t* __restrict__ skip) {
  __shared__ wc_smem S;
  const uint32_t k = blockIdx.x;
  if (k >= n_req || (skip && *skip) || req_bad[k]) return;  // (uniform per workgroup)
  wc_init_tables(S);
  wc_load12(S, WC_ACC, parts[(size_t)k * split]);
#pragma unroll 1
  for (uint32_t h = 1; h < split; h++) {
    wc_load12(S, WC_T0, parts[(size_t)k * split + h]);
    wc_apply(S, LB_WC_MUL, WC_ACC, WC_ACC, WC_T0);
  }
  if (threadIdx.x < 12) (&F[k].c0.c0.c0)[threadIdx.x] = S.slot[WC_ACC][threadIdx.x];
}

#define LB_INST_STEP(M, W)                                                                                      \
  template __global__ void k_step_acc<M, W>(uint32_t, uint32_t, Rows, const uint32_t* __restrict__,               \
                                            const uint32_t* __restrict__, uint32_t* __restrict__);
LB_INST_STEP(0, 1)
LB_INST_STEP(1, 1)
LB_INST_STEP(2, 1)
LB_INST_STEP(0, 2)
LB_INST_STEP(2, 2)
#define LB_INST_LINES_ROWS(W)                                                                                    \
  template __global__ void k_lines_rows<W>(uint32_t, uint32_t, Rows, const uint32_t* __restrict__,                \
                                           const g1j* __restrict__, g2j* __restrict__, uint32_t* __restrict__);
LB_INST_LINES_ROWS(1)
LB_INST_LINES_ROWS(2)

}  // namespace lb
