// qoc_run_blk.hip — the block chains and block gradient (qoc_blk.hpp): detection of the generators' invariant
// blocks, and the launches of one propagate / grape_sensitivity / concurrent eval on them.
#include <cstring>
#include <numeric>

#include "qoc_blk.hpp"
#include "qoc_blkp.hpp"
#include "qoc_blkseg.hpp"
#include "qoc_blku.hpp"
#include "qoc_internal.hpp"

namespace qoc_host {

static int blku_forward(qoc_ctx* c);
static int blku_backward(qoc_ctx* c, int order, double* d_dJdu);
static int blku_eval_concurrent(qoc_ctx* c, int order, double* d_dJdu);

// Connected components of the union sparsity pattern of A_0..A_nu (host copy, c->h_gen): rows i and k share a block
// whenever some A_j[i, k] or A_j[k, i] is nonzero.  Blocks of at most BLK_NBMAX rows turn the block path on
// (QOC_BLOCKS=0 keeps the dense chains); d_brow lists each block's rows in increasing order, blocks ordered by
// their first row, padded with -1 to NB = 2, 3 or 4.
int blk_detect(qoc_ctx* c) {
  c->blk_nb = 0;
  c->nblk = 0;
  c->blk_jr = 0;
  c->blk_real = false;
  c->nwb = 0;
  const char* env = getenv("QOC_BLOCKS");
  if (env && !std::strcmp(env, "0")) return QOC_OK;
  const bool valu = env && !std::strcmp(env, "valu");  // blocks of <= 4 rows on the VALU lanes (k_blk_*)
  // blocks of <= 2 rows on their real embedding (JR = 0, QOC_BLOCKS=real): one MFMA per term and no DPP swap, but
  // 4 columns per wave and 5 waves per cavity seed instead of 3; measured the same as the complex slots (cavity
  // chain 0.79 vs 0.78 ms), so the complex slots stay the default
  const bool real_req = env && !std::strcmp(env, "real");
  const int N = c->N;
  const size_t NN = (size_t)N * N;
  std::vector<int> par(N);
  std::iota(par.begin(), par.end(), 0);
  auto find = [&](int x) {
    while (par[x] != x) x = par[x] = par[par[x]];
    return x;
  };
  for (int j = 0; j <= c->nu; ++j)
    for (int col = 0; col < N; ++col)
      for (int row = 0; row < N; ++row) {
        const double* v = c->h_gen.data() + 2 * (j * NN + row + (size_t)N * col);
        if (row != col && (v[0] != 0.0 || v[1] != 0.0)) {
          const int a = find(row), b = find(col);
          if (a != b) par[std::max(a, b)] = std::min(a, b);
        }
      }
  std::vector<std::vector<int>> blocks;
  std::vector<int> id(N, -1);
  for (int row = 0; row < N; ++row) {
    const int root = find(row);
    if (id[root] < 0) {
      id[root] = (int)blocks.size();
      blocks.emplace_back();
    }
    blocks[id[root]].push_back(row);
  }
  size_t mx = 0;
  for (const auto& bl : blocks) mx = std::max(mx, bl.size());
  // blocks of <= 4 rows: packed into the aligned 4-row slots of MFMA block waves (JR = 1), or one VALU lane per
  // (block, column) with QOC_BLOCKS=valu; 5..16 rows: one MFMA wave per block (JR = 4), only when the dense state
  // needs more than one 16-row group (N > 16: at N <= 16 the dense register chain already runs one wave per column
  // pair)
  if (mx > 16 || (mx > (size_t)BLK_NBMAX && N <= 16)) return QOC_OK;
  const int NB = mx <= 2 ? 2 : mx <= 3 ? 3 : mx <= 4 ? 4 : 16;
  const int nblk = (int)blocks.size();
  std::vector<int> brow((size_t)nblk * NB, -1);
  for (int b = 0; b < nblk; ++b)
    for (size_t i = 0; i < blocks[b].size(); ++i) brow[(size_t)b * NB + i] = blocks[b][i];
  // the MFMA waves' 16-row states
  std::vector<int> wrow;
  int jr = 0;
  bool real = false;
  if (NB == 16) {
    jr = 4;
    wrow = brow;
  } else if (real_req && mx <= 2) {
    // real embedding: a block of <= 2 complex rows is one 4-row slot [Re r0, Re r1, Im r0, Im r1] (two 1-row blocks
    // share a slot); entries row * 2 + part, so that each element's partner part sits 32 lanes away
    real = true;
    std::vector<int> rows;  // complex rows in slot order, 2 per slot (-1 padding)
    for (const auto& bl : blocks) {
      if (bl.size() == 2 && rows.size() % 2) rows.push_back(-1);  // a 2-row block starts a slot
      for (int r : bl) rows.push_back(r);
    }
    if (rows.size() % 2) rows.push_back(-1);
    for (size_t q = 0; q < rows.size(); q += 2) {
      const int r0 = rows[q], r1 = rows[q + 1];
      wrow.push_back(r0 >= 0 ? 2 * r0 : -1);
      wrow.push_back(r1 >= 0 ? 2 * r1 : -1);
      wrow.push_back(r0 >= 0 ? 2 * r0 + 1 : -1);
      wrow.push_back(r1 >= 0 ? 2 * r1 + 1 : -1);
    }
    while (wrow.size() % 16) wrow.push_back(-1);
  } else if (!valu) {
    jr = 1;
    std::vector<int> slot;  // rows of the 4-row slots, in order (a block never straddles two slots)
    int fill = 0;
    for (const auto& bl : blocks) {
      if (fill + (int)bl.size() > 4) {
        for (; fill < 4; ++fill) slot.push_back(-1);
        fill = 0;
      }
      for (int r : bl) slot.push_back(r);
      fill += (int)bl.size();
      if (fill == 4) fill = 0;
    }
    while (slot.size() % 16) slot.push_back(-1);
    wrow = slot;
  }
  c->h_wrow = wrow;
  c->h_wrow_live.clear();
  c->h_dead_rows.clear();
  c->dead_dirty = true;
  for (int** p : {&c->d_brow, &c->d_wrow, &c->d_wrow_live, &c->d_dead_rows})
    if (*p) {
      HIPCHK(c, hipFree(*p));
      *p = nullptr;
    }
  c->dev_bytes -= c->blk_dev_bytes;  // the row lists of a previous qoc_set_generators
  c->blk_dev_bytes = 0;
  HIPCHK(c, hipMalloc((void**)&c->d_brow, brow.size() * sizeof(int)));
  HIPCHK(c, hipMemcpy(c->d_brow, brow.data(), brow.size() * sizeof(int), hipMemcpyHostToDevice));
  c->blk_dev_bytes += brow.size() * sizeof(int);
  if (jr || real) {
    HIPCHK(c, hipMalloc((void**)&c->d_wrow, wrow.size() * sizeof(int)));
    HIPCHK(c, hipMemcpy(c->d_wrow, wrow.data(), wrow.size() * sizeof(int), hipMemcpyHostToDevice));
    c->blk_dev_bytes += wrow.size() * sizeof(int);
  }
  c->dev_bytes += c->blk_dev_bytes;
  c->blk_nb = NB;
  c->nblk = nblk;
  c->blk_jr = jr;
  c->blk_real = real;
  c->nwb = (int)(wrow.size() / 16);
  return QOC_OK;
}

// The block path runs the Taylor-action chains' fp64 scheme (step records, shifted generators) on unpacked states
bool blk_active(const qoc_ctx* c) {
  if (c->blk_nb <= 0 || c->prec != QOC_FP64 || c->chain_mode != 1 || c->prop_method != QOC_PROP_EXPM || c->big ||
      c->packed || c->nu > 2)
    return false;
  // MFMA block waves: <= 8 per workgroup (the 512-thread launch bound keeps 256 VGPRs per wave)
  if (c->blk_real) return c->nwb * ((c->m + 3) / 4) <= 8;
  if (c->blk_jr) return c->nwb * ((c->m + 1) / 2) <= 8 && (c->blk_nb < 16 || tchain_mf(c));
  return c->nblk * c->m <= BLK_MAXT && c->nblk <= 256;
}
// MFMA block waves (k_blkrot_*): the chain kernels; blocks of 16 rows also take the dense gradient kernels
bool blk_rot(const qoc_ctx* c) { return c->blk_jr > 0 || c->blk_real; }
static bool blk_big(const qoc_ctx* c) { return c->blk_nb == 16; }

// Block propagators (qoc_blku.hpp), the default for blocks of <= 4 rows: formed per (slice, block) apart from the
// serial chain, which then runs one NB x NB matvec per slice.  QOC_BLKU=0 keeps the polynomial-in-the-chain kernels
// (k_blkrot_* / k_blk_*).  The gradient packs 64 / nblk slices per wave (nblk <= 32); the chain lanes take
// nblk m <= 256 (block, column) pairs.
bool blku_on(const qoc_ctx* c) {
  // QOC_BLOCKS=valu / real ask for those kernel variants explicitly (blk_jr != 1): they keep them
  if (!blk_active(c) || c->blk_jr != 1 || c->blk_nb > BLK_NBMAX || c->nu < 1 || c->nu > 2 || c->nblk > 32 ||
      c->nblk * c->m * (c->blk_nb == 2 ? 2 : 4) > 64 * (c->blk_nb == 4 ? 2 : 4))
    return false;
  // an explicit QOC_BLOCKS=valu / real keeps the polynomial-in-the-chain kernels, also where it falls back to the
  // complex MFMA slots (real with blocks of more than 2 rows)
  const char* bl = getenv("QOC_BLOCKS");
  if (bl && (!std::strcmp(bl, "valu") || !std::strcmp(bl, "real"))) return false;
  const char* env = getenv("QOC_BLKU");
  return !(env && !std::strcmp(env, "0"));
}

struct BlkuShape {
  int C, CW, W, S, ustg;
  size_t lds;
};
// Waves per workgroup: CW chain waves (one lane per state element), in the fused backward one staging wave, and FW
// worker waves (formation, in the fused backward also the contraction).  The workers are the critical path (their
// chunk of formation + contraction takes longer than the chain's C matvecs), so FW takes every wave slot left:
// 8 waves per CU at the kernels' > 128 VGPRs (2 per SIMD), shared by the B / CUs workgroups a CU holds at once
// (QOC_BLKU_FW / QOC_BLKU_GFW override FW).  C: the most slices per chunk (a power of two <= 64: chunks never
// straddle k_blku_rec's 64-slice (J, P) groups) whose LDS fits those workgroups (QOC_BLKU_C / QOC_BLKU_GC override
// it).  S: the prefix-product group (QOC_BLKU_S; 1 by default: the chains are store- or latency-bound at S = 1 and
// the scans cost the workers more than they save).
static BlkuShape blku_shape(const qoc_ctx* c, bool fused, bool storeu = false) {
  BlkuShape s{};
  const int NB = c->blk_nb;
  s.CW = (c->nblk * c->m * (NB == 2 ? 2 : 4) + 63) / 64;  // one chain lane per state element (qoc_blku.hpp)
  const int per_cu = std::max(1, std::min(3, (c->B + c->ncu - 1) / std::max(1, c->ncu)));
  // the fused backward's staging waves: with stored propagators one more, unless one wave can hold a chunk's records,
  // x_k and propagators (QOC_BLKU_USTG=1: then the freed wave slot is a worker's)
  const char* us = getenv("QOC_BLKU_USTG");
  s.ustg = storeu && us && atoi(us) == 1 ? 1 : 2;
  int stg = fused ? (storeu && s.ustg == 2 ? 2 : 1) : 0;
  // waves per workgroup at most: the kernels' launch bound (blku_max_threads: 12 waves for blocks of 2 rows), shared
  // by the workgroups of a CU
  const int wcap = blku_max_threads(NB) / 64;
  // the fused backward needs at least one worker wave (the contraction runs on workers only): with the second
  // staging wave that would not fit (blocks of 4 rows, nblk m > 16: CW = 2 within 4 waves), one stager copies all
  if (fused && stg == 2 && s.CW + stg + 1 > wcap) {
    s.ustg = 1;
    stg = 1;
  }
  const int wmax = std::max(s.CW + stg + 1, wcap / per_cu);
  int fw = wmax - s.CW - stg;
  if (const char* env = getenv(fused ? "QOC_BLKU_GFW" : "QOC_BLKU_FW")) fw = atoi(env);
  fw = std::max(1, std::min(fw, wcap - s.CW - stg));
  s.W = s.CW + stg + fw;
  s.S = 1;
  if (const char* env = getenv("QOC_BLKU_S")) s.S = atoi(env) >= 2 && NB < 4 ? 2 : 1;
  const size_t budget = (size_t)156 * 1024 / per_cu;
  const int gw = fused ? fw : 0;
  s.C = 64;
  // the stager's registers: x_k and the stored propagators of one chunk
  auto stage_ok = [&](int C) { return !fused || std::max(C * c->N * c->m, C * NB * NB * c->nblk) <= BLKU_XMAX * 64; };
  auto fits = [&](int C) { return blku_lds(c->N, c->m, NB, c->nblk, C, gw) <= budget && stage_ok(C); };
  if (!fused) {
    while (s.C > 4 && !fits(s.C)) s.C >>= 1;
  } else {
    // the fused backward: the largest C that fits, then within [Cmax / 2, Cmax] the C whose wave-iterations of the
    // contraction (ceil(C / UPW), UPW = 64 / nblk slices each) come out most even over the fw workers: the fewest
    // iterations of the busiest worker per slice (ties: the larger C, fewer chunk barriers)
    while (s.C > 4 && !fits(s.C)) --s.C;
    const int upw = std::max(1, 64 / std::max(1, c->nblk)), cmax = s.C;
    auto per_slice = [&](int C) { return (double)(((C + upw - 1) / upw + fw - 1) / fw) / C; };
    for (int C = cmax; C >= std::max(4, cmax / 2); --C)
      if (per_slice(C) < per_slice(s.C) - 1e-12) s.C = C;
  }
  if (const char* env = getenv(fused ? "QOC_BLKU_GC" : "QOC_BLKU_C")) {
    // an override is clamped to what fits (the stager's registers and the LDS budget), never an invalid launch
    int q = 1;
    if (fused) {
      q = std::max(1, std::min(atoi(env), 64));
      while (q > 1 && !fits(q)) --q;
    } else {
      while (q * 2 <= std::min(atoi(env), 64) && fits(q * 2)) q *= 2;
    }
    s.C = q;
  }
  s.C = std::max(s.C, s.S);
  s.lds = blku_lds(c->N, c->m, NB, c->nblk, s.C, gw);
  s.W = std::min(s.W, wcap);  // never above the launch bound (a larger launch faults)
  if (fused && s.W < s.CW + stg + 1) s.W = 0;  // no worker wave: not launchable (blku_fused_ok refuses it)
  return s;
}

static int blku_ntp(const qoc_ctx* c) { return (c->Nt + BLKU_RECBLK - 1) / BLKU_RECBLK * BLKU_RECBLK; }

static BlkuParams blku_params(const qoc_ctx* c, const BlkuShape& s, double* d_dJdu = nullptr) {
  BlkuParams p{};
  for (int j = 0; j < 3; ++j) {
    const bool on = j <= c->nu;
    // skew-Hermitian generators: spectral half-widths (the 2-norm bound of Ã_k); otherwise the shifted 1-norms
    p.rad[j] = on ? (c->cheb_ok ? c->tprm.rad[j] : c->tprm.nrm[j]) : 0.0;
    p.mur[j] = on ? c->tprm.mur[j] : 0.0;
    p.mui[j] = on ? c->tprm.mui[j] : 0.0;
  }
  p.theta_cap = c->tprm.theta[17];
  p.C = s.C;
  p.CW = s.CW;
  p.Ntp = blku_ntp(c);
  p.rec = c->d_blkrec;
  p.terms = c->d_terms;
  p.dJdu = d_dJdu;
  return p;
}

// the step records of every (seed, slice) of the current u (k_blku_rec); count: add Σ P 2^J to the terms counter
static int blku_records(qoc_ctx* c, BlkuParams& bp, bool count, const double* d_u = nullptr) {
  const long long total = (long long)c->B * blku_ntp(c);
  if (!c->d_blkrec) {
    const size_t bytes = (size_t)total * BLKU_REC * sizeof(double);
    HIPCHK(c, hipMalloc((void**)&c->d_blkrec, bytes));
    c->dev_bytes += bytes;
  }
  bp.rec = c->d_blkrec;
  BlkuParams rp = bp;
  rp.terms = count ? c->d_terms : nullptr;
  const int mk = mark_begin(c, 0);
  hipLaunchKernelGGL(k_blku_rec, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c->stream, rp,
                     d_u ? d_u : (const double*)c->d_u, c->nu, c->Nt, total, c->d_blkrec);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}

static BlkArgs blk_args(const qoc_ctx* c) {
  BlkArgs bk{};
  bk.brow = c->d_brow;
  bk.A = c->d_A;
  bk.nblk = c->nblk;
  bk.wrow = c->d_wrow;
  bk.nwb = c->nwb;
  return bk;
}

static int blk_threads(const qoc_ctx* c, int nwb = -1) {
  if (nwb < 0) nwb = c->nwb;
  if (c->blk_real) return 64 * nwb * ((c->m + 3) / 4);  // 4 state columns per real-embedded wave
  return blk_rot(c) ? 64 * nwb * ((c->m + 1) / 2) : 64 * ((c->nblk * c->m + 63) / 64);
}
static size_t blk_lds_of(const qoc_ctx* c, int nwb = -1) {
  return blk_rot(c) ? blkrot_lds(c->N, c->m, blk_threads(c, nwb) / 64) : blk_lds(c->N, c->m);
}

// Blocks of 5..16 rows that carry no state: x_0 (every seed) and X_target are zero on all their rows.  The generators
// keep every block invariant, so such a block's x_k and μ_k are exactly zero at every k, and it adds nothing to J
// (its overlaps are zero) or to dJ/du (each generator's contribution is λ_β^H A_jβ x_β = 0).  The reference exploits
// the same structure by hand with compress_states (src/utils.jl:96-109; the tunable bus' parity blocks,
// test/test_utils.jl:23): here the concurrent eval launches waves for the live blocks only and k_zero_rows writes
// the dead rows' zeros into the state-shaped buffers, so every output (x_k, λ_k, J, dJ/du) is what the full launch
// gives.  The tunable bus (m = 1, |110> -> |200>) carries its state in the 14-row even-parity block only.
// QOC_BLK_DEAD=0 launches every block.  Sets bk.wrow / bk.nwb; leaves them when every block is live.
static int blk_live(qoc_ctx* c, BlkArgs& bk) {
  if (!blk_big(c) || c->h_wrow.empty() || c->h_Xt.empty() || !c->have_x0) return QOC_OK;
  const char* env = getenv("QOC_BLK_DEAD");
  if (env && atoi(env) == 0) return QOC_OK;
  const int N = c->N, mu = c->m_user;
  const size_t cnt = c->x0_per_seed ? (size_t)c->B : 1, Nmu = (size_t)N * mu;
  if (c->h_x0.size() < 2 * Nmu * cnt || c->h_Xt.size() < 2 * Nmu) return QOC_OK;
  std::vector<char> live(N, 0);
  auto mark = [&](const double* v) {
    for (size_t e = 0; e < Nmu; ++e)
      if (v[2 * e] != 0.0 || v[2 * e + 1] != 0.0) live[e % N] = 1;
  };
  for (size_t q = 0; q < cnt; ++q) mark(c->h_x0.data() + 2 * Nmu * q);
  mark(c->h_Xt.data());
  std::vector<int> wl, dead;
  for (int w = 0; w < c->nwb; ++w) {
    bool lv = false;
    for (int i = 0; i < 16; ++i) {
      const int r = c->h_wrow[16 * w + i];
      lv = lv || (r >= 0 && live[r]);
    }
    for (int i = 0; i < 16; ++i) {
      const int r = c->h_wrow[16 * w + i];
      if (lv) wl.push_back(r);
      else if (r >= 0) dead.push_back(r);
    }
  }
  if (dead.empty() || wl.empty()) return QOC_OK;
  if (wl != c->h_wrow_live || dead != c->h_dead_rows) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int** p : {&c->d_wrow_live, &c->d_dead_rows})
      if (*p) {
        HIPCHK(c, hipFree(*p));
        *p = nullptr;
      }
    HIPCHK(c, hipMalloc((void**)&c->d_wrow_live, wl.size() * sizeof(int)));
    HIPCHK(c, hipMemcpy(c->d_wrow_live, wl.data(), wl.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(c, hipMalloc((void**)&c->d_dead_rows, dead.size() * sizeof(int)));
    HIPCHK(c, hipMemcpy(c->d_dead_rows, dead.data(), dead.size() * sizeof(int), hipMemcpyHostToDevice));
    c->h_wrow_live = wl;
    c->h_dead_rows = dead;
  }
  bk.wrow = c->d_wrow_live;
  bk.nwb = (int)(wl.size() / 16);
  return QOC_OK;
}
// the dead rows' zeros (blk_live) in up to six state-shaped buffers of B (Nt + 1) m columns.  Skipped when the same
// buffers already hold zeros on the same rows: every exact recurrence keeps rows whose x0 and target are zero at zero
// (the generators keep the blocks invariant), so only a backward with an external λ_N or a co-state source
// (dead_dirty), new generators or a reallocated buffer can put anything else there.
static int blk_zero_dead(qoc_ctx* c, std::initializer_list<void*> bufs) {
  ZeroRows z{};
  for (void* p : bufs)
    if (p && z.nbuf < 6) z.buf[z.nbuf++] = (double2*)p;
  bool same = !c->dead_dirty && c->h_dead_zeroed == c->h_dead_rows;
  for (int i = 0; i < 6; ++i) same = same && c->dead_bufs[i] == (i < z.nbuf ? (const void*)z.buf[i] : nullptr);
  if (same) return QOC_OK;
  const long long cols = (long long)c->B * (c->Nt + 1) * c->m;
  const long long total = cols * (long long)c->h_dead_rows.size();
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(k_zero_rows, dim3(grid), dim3(256), 0, c->stream, z, cols, c->N, c->d_dead_rows,
                     (int)c->h_dead_rows.size());
  HIPCHK(c, hipGetLastError());
  c->h_dead_zeroed = c->h_dead_rows;
  for (int i = 0; i < 6; ++i) c->dead_bufs[i] = i < z.nbuf ? (const void*)z.buf[i] : nullptr;
  c->dead_dirty = false;
  return QOC_OK;
}
// dynamic LDS above the 64 KiB default (up to 16 MFMA block waves of staging)
template <typename K>
static hipError_t blk_lds_attr(K kern, size_t lds) {
  return lds > 65536 ? hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
                     : hipSuccess;
}

// f(kernel-selector, Chebyshev): selector 1 / 4 = k_blkrot_*<JR>, 2 / 3 / 4 + 100 = k_blk_*<NB> (VALU lanes)
template <typename F>
static hipError_t blk_dispatch(const qoc_ctx* c, F&& f) {
  using std::integral_constant;
  auto ch = [&](auto K_) { return c->cheb_ran ? f(K_, std::true_type()) : f(K_, std::false_type()); };
  if (c->blk_real) return ch(integral_constant<int, 0>());
  if (c->blk_jr == 1) return ch(integral_constant<int, 1>());
  if (c->blk_jr == 4) return ch(integral_constant<int, 4>());
  switch (c->blk_nb) {
    case 2: return ch(integral_constant<int, 102>());
    case 3: return ch(integral_constant<int, 103>());
    case 4: return ch(integral_constant<int, 104>());
  }
  return hipErrorInvalidValue;
}

int blk_forward(qoc_ctx* c) {
  if (blku_on(c)) return blku_forward(c);
  int r = blkp_forward(c);  // blocks of 5..16 rows: stored propagators (1: not applicable)
  if (r != 1) return r;
  r = tchain_prep(c);
  if (r) return r;
  const TChainArgs g = tchain_args(c);
  const BlkArgs bk = blk_args(c);
  const size_t lds = blk_lds_of(c);
  const int mk = mark_begin(c, 1);
  const hipError_t e = blk_dispatch(c, [&](auto NB_, auto CH_) {
    constexpr int NB = decltype(NB_)::value;
    constexpr bool CH = decltype(CH_)::value;
    if constexpr (NB < 100) {
      const hipError_t q = blk_lds_attr(k_blkrot_fwd<NB, CH>, lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL((k_blkrot_fwd<NB, CH>), dim3(c->B), dim3(blk_threads(c)), lds, c->stream, g, bk);
    }
    else hipLaunchKernelGGL((k_blk_fwd<NB - 100, CH>), dim3(c->B), dim3(blk_threads(c)), lds, c->stream, g, bk);
    return hipGetLastError();
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blk_fwd launch: %s", hipGetErrorString(e));
  c->fwd_captured = false;
  c->props_since_reset++;
  return QOC_OK;
}

// the order-o gradient from d_X and d_L (mu_mode: d_L holds μ, λ = coef ⊙ μ with the coefficients in d_coef)
static int blk_grad(qoc_ctx* c, int order, bool mu_mode, double* d_dJdu) {
  const TChainArgs g = tchain_args(c);
  const BlkArgs bk = blk_args(c);
  const long long units = (long long)c->B * c->Nt;
  const int upw = 256 / c->nblk;
  if (upw < 1) return fail(c, QOC_ERR_UNSUPPORTED, "block gradient: %d blocks exceed one workgroup", c->nblk);
  const unsigned blocks = (unsigned)((units + upw - 1) / upw);
  const int mk = mark_begin(c, 3);
  hipError_t e = hipSuccess;
  auto launch = [&](auto NB_) {
    constexpr int NB = decltype(NB_)::value;
    switch (order) {
      case 1: hipLaunchKernelGGL((k_blk_grad<NB, 1>), dim3(blocks), dim3(256), 0, c->stream, g, bk, units, (int)mu_mode, d_dJdu); break;
      case 2: hipLaunchKernelGGL((k_blk_grad<NB, 2>), dim3(blocks), dim3(256), 0, c->stream, g, bk, units, (int)mu_mode, d_dJdu); break;
      case 3: hipLaunchKernelGGL((k_blk_grad<NB, 3>), dim3(blocks), dim3(256), 0, c->stream, g, bk, units, (int)mu_mode, d_dJdu); break;
      default: hipLaunchKernelGGL((k_blk_grad<NB, 4>), dim3(blocks), dim3(256), 0, c->stream, g, bk, units, (int)mu_mode, d_dJdu); break;
    }
    return hipGetLastError();
  };
  if (c->blk_nb == 2) e = launch(std::integral_constant<int, 2>());
  else if (c->blk_nb == 3) e = launch(std::integral_constant<int, 3>());
  else e = launch(std::integral_constant<int, 4>());
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blk_grad launch: %s", hipGetErrorString(e));
  return QOC_OK;
}

// grape_sensitivity: λ by the block backward chain (penalty, co-state source and an external λ_N included), then the
// block gradient for orders 1..4; the exact (Fréchet) gradient runs its own dense kernel on the same λ.
int blk_backward(qoc_ctx* c, int order, double* d_dJdu) {
  if (blku_on(c)) return blku_backward(c, order, d_dJdu);
  if (c->steps_stale) {  // the last forward was the stored-propagator eval (blkp): this u's step records first
    if (int r0 = tchain_prep(c)) return r0;
  }
  const TChainArgs g = tchain_args(c);
  const BlkArgs bk = blk_args(c);
  const size_t lds = blk_lds_of(c);
  int mk = mark_begin(c, 2);
  const hipError_t e = blk_dispatch(c, [&](auto NB_, auto CH_) {
    constexpr int NB = decltype(NB_)::value;
    constexpr bool CH = decltype(CH_)::value;
    if constexpr (NB < 100) {
      const hipError_t q = blk_lds_attr(k_blkrot_bwd<NB, CH>, lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL((k_blkrot_bwd<NB, CH>), dim3(c->B), dim3(blk_threads(c)), lds, c->stream, g, bk);
    }
    else hipLaunchKernelGGL((k_blk_bwd<NB - 100, CH>), dim3(c->B), dim3(blk_threads(c)), lds, c->stream, g, bk);
    return hipGetLastError();
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blk_bwd launch: %s", hipGetErrorString(e));
  if (order == QOC_DUKDP_EXACT || blk_big(c)) return dense_gradient<double>(c, order, d_dJdu);
  return blk_grad(c, order, false, d_dJdu);
}

// qoc_eval_dev with a built-in cost, no penalty and no co-state source: the forward chain and the μ recurrence
// (λ_k = coef ⊙ μ_k, src/penalty_fcns.jl:19-22, 35-40) in one launch, then the gradient with the coefficients.
bool blk_concurrent_ok(const qoc_ctx* c, int order) {
  // MFMA block waves: the contraction from the chains' captures (k_grad_rr_c, order 3)
  if (blk_big(c) && !(order == 3 && tchain_cap_ok(c))) return false;
  return blk_active(c) && c->concurrent && order >= 1 && order <= BLK_ORDMAX &&
         (c->cost_kind == QOC_COST_TRACE || c->cost_kind == QOC_COST_ZCAL) && c->mu == 0.0 && !c->src_on;
}

// ---- stored propagators for blocks of 5..16 rows (qoc_blkp.hpp) ------------------------------------------------------
// The tunable bus' parity blocks: U_k per (seed, slice, live block) -- interpolated in u for one control
// (k_blkp_int), else on MFMA (k_blkp_exp) --, then the one-matvec chains (k_blkp_dual / k_blkp_chain) and the order-3
// gradient on MFMA (k_blkp_grad).  QOC_BLKP=0 keeps the Chebyshev-action chains (k_blkrot_dual).
bool blkp_on(const qoc_ctx* c) {
  if (!blk_active(c) || !blk_big(c) || c->nu < 1 || c->nu > 2) return false;
  const char* env = getenv("QOC_BLKP");
  return !(env && atoi(env) == 0);
}

// the propagator store d_blkU of at least `bytes` (reallocated when a larger batch part or block layout needs more);
// soft: a failed allocation is no error (returns 1: the caller takes the Chebyshev block chains instead)
static int blkp_ensure_store(qoc_ctx* c, size_t bytes, bool soft) {
  if (c->blkU_bytes >= bytes) return QOC_OK;
  if (c->d_blkU) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->stream2) HIPCHK(c, hipStreamSynchronize(c->stream2));
    HIPCHK(c, hipFree(c->d_blkU));
    c->d_blkU = nullptr;
    c->dev_bytes -= c->blkU_bytes;
    c->blkU_bytes = 0;
  }
  const hipError_t e = hipMalloc((void**)&c->d_blkU, bytes);
  if (e != hipSuccess) {
    c->d_blkU = nullptr;
    (void)hipGetLastError();  // clear the sticky error of the failed allocation
    if (soft) return 1;
    return fail(c, QOC_ERR_HIP, "stored block propagators (%zu bytes): %s", bytes, hipGetErrorString(e));
  }
  c->blkU_bytes = bytes;
  c->dev_bytes += bytes;
  return QOC_OK;
}

// θ[r][s] of BlkpArgs::tail: the largest ρ with Σ_{k > 4r} ρ^k / k! <= 2^-53 2^-(s + tail) (bisection; the tail sum from
// its first term, exp((4r + 1) ln ρ - lgamma(4r + 2)), 40 terms)
static void blkp_theta_table(int tail, double (&theta)[BLKP_RMAX + 1][16]) {
  for (int r = 0; r <= BLKP_RMAX; ++r)
    for (int s = 0; s < 16; ++s) {
      if (r < BLKP_RMIN) {
        theta[r][s] = 0.0;
        continue;
      }
      const int m = 4 * r;
      const double tol = std::ldexp(1.0, -53 - s - tail);
      auto tailsum = [&](double rho) {
        double t = std::exp((m + 1) * std::log(rho) - std::lgamma(m + 2.0)), sum = 0.0;
        for (int k = m + 1; k < m + 41; ++k) {
          sum += t;
          t *= rho / (k + 1);
        }
        return sum;
      };
      double lo = 0.0, hi = 16.0;
      for (int it = 0; it < 200; ++it) {
        const double mid = 0.5 * (lo + hi);
        (tailsum(mid) <= tol ? lo : hi) = mid;
      }
      theta[r][s] = lo;
    }
}

// The Chebyshev form's table (qoc_blkp.hpp blkp_cheb) for block size cm up to ρ_c = crmax: per grid point
// ρ_c = 2^((g - BLKP_CT_G0) / 4) the Bessel values J_k(ρ_c) (Miller's backward recurrence in long double, normalised
// by J_0 + 2 Σ J_2k = 1), the degree n with Σ_{k>n} 2 |J_k| <= 2^-57, and the series rewritten for block Clenshaw in
// Z = T_cm: c_k = (2 - δ_k0) (-i)^k J_k, then from the top block down a_{q,j} = 2 c_{cm q + j}, c_{cm q - j} -= c_{cm q + j}
// (j = 1..cm-1), a_{q,0} = c_{cm q}; β_{q,j} = i^j a_{q,j} is real for even cm.
static int blkp_cheb_table(qoc_ctx* c, int cm, double crmax) {
  if (c->d_blkp_ctab && c->ctab_cm == cm && c->ctab_rmax == crmax) return QOC_OK;
  const int gn = BLKP_CT_G0 + (int)std::lround(4.0 * std::log2(crmax)) + 1;
  std::vector<double> tab((size_t)gn * BLKP_CT_STRIDE, 0.0);
  typedef long double LD;
  for (int g = 0; g < gn; ++g) {
    const LD rc = std::pow((LD)2, (LD)(g - BLKP_CT_G0) / 4);
    const int K = 100, M = K + 60 + (int)(4 * rc);
    std::vector<LD> jb(M + 2, 0.0L);
    jb[M] = 1e-300L;
    for (int k = M; k >= 1; --k) jb[k - 1] = (2.0L * k / rc) * jb[k] - jb[k + 1];
    LD nrm = jb[0];
    for (int k = 2; k <= M; k += 2) nrm += 2 * jb[k];
    std::vector<LD> J(K + 1);
    for (int k = 0; k <= K; ++k) J[k] = jb[k] / nrm;
    int n = K;
    LD tail = 0;
    while (n > 0 && tail + 2 * std::fabs(J[n]) <= std::ldexp(1.0L, -57)) tail += 2 * std::fabs(J[n--]);
    const int Q = n <= cm - 1 ? 0 : (n - (cm - 1) + cm - 1) / cm;
    if (4 + (Q + 1) * cm > BLKP_CT_STRIDE) return fail(c, QOC_ERR_UNSUPPORTED, "Chebyshev table: degree %d at rho %g", n, (double)rc);
    const int L = cm * (Q + 1);
    std::vector<LD> cr(L, 0.0L), ci(L, 0.0L);  // c_k = (2 - δ) (-i)^k J_k
    for (int k = 0; k <= n && k < L; ++k) {
      const LD v = (k ? 2 : 1) * J[k];
      switch (k & 3) {
        case 0: cr[k] = v; break;
        case 1: ci[k] = -v; break;
        case 2: cr[k] = -v; break;
        default: ci[k] = v; break;
      }
    }
    double* row = tab.data() + (size_t)g * BLKP_CT_STRIDE;
    row[0] = (double)rc;
    row[1] = (double)(1.0L / rc);
    row[2] = Q;
    for (int qq = Q; qq >= 0; --qq)
      for (int jj = cm - 1; jj >= 0; --jj) {
        const int k = cm * qq + jj;
        LD ar = cr[k], ai = ci[k];
        if (qq > 0 && jj > 0) {
          ar *= 2;
          ai *= 2;
          cr[cm * qq - jj] -= cr[k];
          ci[cm * qq - jj] -= ci[k];
        }
        // β = i^j a (real)
        LD br = ar, bi = ai;
        for (int t = 0; t < (jj & 3); ++t) {
          const LD nr = -bi, ni = br;
          br = nr;
          bi = ni;
        }
        if (std::fabs(bi) > 1e-12L * (std::fabs(br) + 1e-300L) && std::fabs(bi) > 1e-300L)
          return fail(c, QOC_ERR_UNSUPPORTED, "Chebyshev table: complex coefficient (g %d, q %d, j %d)", g, qq, jj);
        row[4 + qq * cm + jj] = (double)br;
      }
  }
  if (c->d_blkp_ctab) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->d_blkp_ctab));
    c->d_blkp_ctab = nullptr;
  }
  HIPCHK(c, hipMalloc((void**)&c->d_blkp_ctab, tab.size() * sizeof(double)));
  HIPCHK(c, hipMemcpy(c->d_blkp_ctab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
  c->ctab_cm = cm;
  c->ctab_rmax = crmax;
  return QOC_OK;
}

// ---- one control: the propagators interpolated in u (qoc_blkp.hpp k_blkp_int) ----
typedef long double LD;
// exp(X) of an n x n complex matrix in long double (row-major, re / im apart): scaling to ||X||_1 <= 1/2, Taylor
// degree 30 (tail < 1e-40), squarings; 64-bit mantissas, so its own error (~1e-18) is far below the fp64 result
static void ld_expm(int n, const std::vector<LD>& Xr, const std::vector<LD>& Xi, std::vector<LD>& Er, std::vector<LD>& Ei) {
  LD n1 = 0;
  for (int c = 0; c < n; ++c) {
    LD sum = 0;
    for (int r = 0; r < n; ++r) sum += std::hypot(Xr[r * n + c], Xi[r * n + c]);
    n1 = std::max(n1, sum);
  }
  int s = 0;
  while (n1 > 0.5L && s < 60) {
    n1 *= 0.5L;
    ++s;
  }
  const LD sc = std::ldexp(1.0L, -s);
  std::vector<LD> Yr(n * n), Yi(n * n), Tr(n * n, 0), Ti(n * n, 0), Nr(n * n), Ni(n * n);
  for (int e = 0; e < n * n; ++e) {
    Yr[e] = Xr[e] * sc;
    Yi[e] = Xi[e] * sc;
  }
  Er.assign(n * n, 0);
  Ei.assign(n * n, 0);
  for (int d = 0; d < n; ++d) Tr[d * n + d] = Er[d * n + d] = 1;
  auto mul = [&](const std::vector<LD>& Ar, const std::vector<LD>& Ai, const std::vector<LD>& Br, const std::vector<LD>& Bi) {
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < n; ++c) {
        LD sr = 0, si = 0;
        for (int q = 0; q < n; ++q) {
          sr += Ar[r * n + q] * Br[q * n + c] - Ai[r * n + q] * Bi[q * n + c];
          si += Ar[r * n + q] * Bi[q * n + c] + Ai[r * n + q] * Br[q * n + c];
        }
        Nr[r * n + c] = sr;
        Ni[r * n + c] = si;
      }
  };
  for (int k = 1; k <= 30; ++k) {
    mul(Tr, Ti, Yr, Yi);
    for (int e = 0; e < n * n; ++e) {
      Tr[e] = Nr[e] / k;
      Ti[e] = Ni[e] / k;
      Er[e] += Tr[e];
      Ei[e] += Ti[e];
    }
  }
  for (int t = 0; t < s; ++t) {
    mul(Er, Ei, Er, Ei);
    Er = Nr;
    Ei = Ni;
  }
}

// the control range [lo, hi] of the batch in d_u (nu = 1): a partial min / max per block, finished on the host
static int blkp_urange(qoc_ctx* c, double& lo, double& hi) {
  const long long n = (long long)c->B * c->Nt * c->nu;
  const int grid = (int)std::max<long long>(1, std::min<long long>(256, (n + 255) / 256));
  if (!c->d_minmax) {
    HIPCHK(c, hipMalloc((void**)&c->d_minmax, 512 * sizeof(double)));
    HIPCHK(c, hipHostMalloc((void**)&c->h_minmax, 512 * sizeof(double), hipHostMallocDefault));
  }
  hipLaunchKernelGGL(k_minmax, dim3(grid), dim3(256), 0, c->stream, (const double*)c->d_u, n, c->d_minmax);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(c->h_minmax, c->d_minmax, 2 * grid * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  lo = c->h_minmax[0];
  hi = c->h_minmax[1];
  for (int b = 1; b < grid; ++b) {
    lo = std::min(lo, c->h_minmax[2 * b]);
    hi = std::max(hi, c->h_minmax[2 * b + 1]);
  }
  return QOC_OK;
}

// The coefficient matrices of exp(Ã_0 + u Ã_1) on [lo, hi] for every live wave block: the exponentials at NI
// Chebyshev points θ_k = π (k + 1/2) / NI in long double, M_i = (2 - δ_i0) / NI Σ_k F_k cos(i θ_k), D the last index
// whose tail max_{i > D} |M_i| is <= 2^-56 (the coefficients of an entire function fall super-exponentially; the
// aliasing of the NI-point transform is below the last ones).  Returns 1 when the series has not converged within NI
// points (a control range too wide) or the coefficients exceed the LDS.
static int blkp_interp_coeffs(qoc_ctx* c, const std::vector<int>& wrow, double lo, double hi) {
  constexpr int NI = 40;
  const int N = c->N, nwb = (int)(wrow.size() / 16);
  const size_t NN = (size_t)N * N;
  const LD pi = std::acos(-1.0L), mid = ((LD)lo + hi) / 2, half = ((LD)hi - lo) / 2;
  std::vector<std::vector<LD>> Mr((size_t)nwb * NI, std::vector<LD>(256, 0)), Mi = Mr;
  std::vector<LD> Xr(256), Xi(256), Er, Ei;
  for (int b = 0; b < nwb; ++b)
    for (int k = 0; k < NI; ++k) {
      const LD th = pi * (k + 0.5L) / NI, u = mid + half * std::cos(th);
      for (int r = 0; r < 16; ++r)
        for (int q = 0; q < 16; ++q) {
          const int row = wrow[16 * b + r], col = wrow[16 * b + q];
          LD vr = 0, vi = 0;
          if (row >= 0 && col >= 0) {
            for (int j = 0; j <= 1; ++j) {
              const double* a = c->h_gen.data() + 2 * (j * NN + row + (size_t)N * col);
              LD ar = a[0], ai = a[1];
              if (row == col) {
                ar -= c->tprm.mur[j];
                ai -= c->tprm.mui[j];
              }
              const LD f = j ? u : 1.0L;
              vr += f * ar;
              vi += f * ai;
            }
          }
          Xr[r * 16 + q] = vr;
          Xi[r * 16 + q] = vi;
        }
      ld_expm(16, Xr, Xi, Er, Ei);
      for (int i = 0; i < NI; ++i) {
        const LD w = std::cos(i * th) * (i ? 2.0L : 1.0L) / NI;
        auto& mr = Mr[(size_t)b * NI + i];
        auto& mi = Mi[(size_t)b * NI + i];
        for (int e = 0; e < 256; ++e) {
          mr[e] += w * Er[e];
          mi[e] += w * Ei[e];
        }
      }
    }
  // complex-symmetric generators on a block's rows (A_j^T = A_j: -i H Δt with H real symmetric) give symmetric
  // propagators: the coefficients are symmetrised (the long-double transform leaves the two triangles a rounding
  // apart), so every form gives U[r][c] = U[c][r] bit for bit, and the interpolating chains may form the upper triangle
  // alone (k_blkp_ichain SYM: block 0, its nl live rows first in the wave block, nl (nl + 1) / 2 <= 128)
  std::vector<char> bsym(nwb, 1);
  for (int b = 0; b < nwb; ++b) {
    for (int r = 0; r < 16 && bsym[b]; ++r)
      for (int q = r + 1; q < 16 && bsym[b]; ++q) {
        const int row = wrow[16 * b + r], col = wrow[16 * b + q];
        if (row < 0 || col < 0) continue;
        for (int j = 0; j <= 1; ++j) {
          const double* x = c->h_gen.data() + 2 * (j * NN + row + (size_t)N * col);
          const double* y = c->h_gen.data() + 2 * (j * NN + col + (size_t)N * row);
          if (x[0] != y[0] || x[1] != y[1]) bsym[b] = 0;
        }
      }
    if (!bsym[b]) continue;
    for (int i = 0; i < NI; ++i) {
      auto& mr = Mr[(size_t)b * NI + i];
      auto& mi = Mi[(size_t)b * NI + i];
      for (int r = 0; r < 16; ++r)
        for (int q = r + 1; q < 16; ++q) {
          const LD ar = (mr[r * 16 + q] + mr[q * 16 + r]) / 2, ai = (mi[r * 16 + q] + mi[q * 16 + r]) / 2;
          mr[r * 16 + q] = mr[q * 16 + r] = ar;
          mi[r * 16 + q] = mi[q * 16 + r] = ai;
        }
    }
  }
  int nl = 0;
  while (nl < 16 && wrow[nl] >= 0) ++nl;
  bool sym = nwb == 1 && bsym[0] && nl * (nl + 1) / 2 <= 128;
  for (int r = nl; r < 16 && sym; ++r) sym = wrow[r] < 0;
  // per block (its own degree: a block's propagators do not depend on the other blocks of the launch); the long-double
  // transform's own rounding leaves a floor near 1e-18 under the converged coefficients
  const LD tol = std::ldexp(1.0L, -56);
  if (nwb > 8) return 1;
  std::vector<int> Db(nwb);
  int D = 0;
  for (int b = 0; b < nwb; ++b) {
    std::vector<LD> mx(NI, 0);
    for (int i = 0; i < NI; ++i)
      for (int e = 0; e < 256; ++e)
        mx[i] = std::max(mx[i], std::max(std::fabs(Mr[(size_t)b * NI + i][e]), std::fabs(Mi[(size_t)b * NI + i][e])));
    if (mx[NI - 1] > tol || mx[NI - 2] > tol) return 1;
    int d = NI - 1;
    while (d > 0 && mx[d] <= tol) --d;
    Db[b] = d;
    D = std::max(D, d);
  }
  if (blkp_int_lds(1, D) > (size_t)150 * 1024) return 1;  // one block's coefficients per launch at least
  std::vector<double2> h((size_t)nwb * (D + 1) * 256);
  for (int b = 0; b < nwb; ++b)
    for (int i = 0; i <= D; ++i)
      for (int p = 0; p < 256; ++p) {  // store position p = blkp_upos(r, col): col = 4 ((p >> 4) & 3) + (p >> 6)
        const int col = 4 * ((p >> 4) & 3) + (p >> 6), row = (p & 15) ^ col, ent = row * 16 + col;
        h[((size_t)b * (D + 1) + i) * 256 + p] =
            make_double2((double)Mr[(size_t)b * NI + i][ent], (double)Mi[(size_t)b * NI + i][ent]);
      }
  const size_t nfull = h.size();
  if (sym) {  // block 0's packed upper triangle after the full layout: [i][slot], slots past nl (nl + 1) / 2 zero
    h.resize(nfull + (size_t)(D + 1) * 128, make_double2(0.0, 0.0));
    for (int i = 0; i <= D; ++i)
      for (int a = 0; a < nl; ++a)
        for (int b2 = a; b2 < nl; ++b2)
          h[nfull + (size_t)i * 128 + blkp_sym_slot(a, b2, nl)] =
              make_double2((double)Mr[i][a * 16 + b2], (double)Mi[i][a * 16 + b2]);
  }
  const size_t bytes = h.size() * sizeof(double2);
  if (c->blkp_M_bytes < bytes) {
    if (c->d_blkp_M) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (c->stream2) HIPCHK(c, hipStreamSynchronize(c->stream2));
      HIPCHK(c, hipFree(c->d_blkp_M));
      c->d_blkp_M = nullptr;
    }
    HIPCHK(c, hipMalloc((void**)&c->d_blkp_M, bytes));
    c->blkp_M_bytes = bytes;
  }
  HIPCHK(c, hipMemcpy(c->d_blkp_M, h.data(), bytes, hipMemcpyHostToDevice));
  c->int_D = D;
  c->int_Db = Db;
  c->int_sym = sym;
  c->int_nl = nl;
  c->int_nfull = nfull;
  c->int_lo = lo;
  c->int_hi = hi;
  c->int_wrow = wrow;
  c->int_ok = true;
  return QOC_OK;
}

// the interpolation's launch arguments from the cached coefficients (c->int_*: valid for bk's layout)
static void blkp_interp_args(const qoc_ctx* c, const BlkArgs& bk, BlkpIntArgs& ia) {
  ia = BlkpIntArgs{};
  ia.nwb = bk.nwb;
  ia.D = c->int_D;
  for (int b = 0; b < bk.nwb && b < 8; ++b) ia.Db[b] = c->int_Db[b];
  ia.u = c->d_u;
  ia.xa = 2.0 / (c->int_hi - c->int_lo);
  ia.xb = -(c->int_hi + c->int_lo) / (c->int_hi - c->int_lo);
  for (int j = 0; j < 2; ++j) {
    ia.mur[j] = c->tprm.mur[j];
    ia.mui[j] = c->tprm.mui[j];
  }
  ia.skew = c->skew_exact && c->tprm.mur[0] == 0.0 && c->tprm.mur[1] == 0.0;
  ia.M = c->d_blkp_M;
  ia.Msym = c->int_sym && bk.nwb == 1 ? c->d_blkp_M + c->int_nfull : nullptr;
  ia.nl = ia.Msym ? c->int_nl : 0;
}

// 0: the formation interpolates (ia filled), 1: it forms the exponentials.  One control (nu = 1) and
// QOC_BLKP_INTERP != 0; the coefficients are recomputed when the batch's control range leaves the one they were made
// for (then widened by 5 % each side, so that an optimiser's drifting controls rarely trigger it) or the generators
// or the live-block layout changed.
static int blkp_interp_setup(qoc_ctx* c, const BlkArgs& bk, BlkpIntArgs& ia) {
  const char* env = getenv("QOC_BLKP_INTERP");
  if (c->nu != 1 || (env && atoi(env) == 0)) return 1;
  double lo, hi;
  int r = blkp_urange(c, lo, hi);
  if (r) return r;
  if (!std::isfinite(lo) || !std::isfinite(hi)) return 1;
  const std::vector<int>& wrow = bk.wrow == c->d_wrow_live ? c->h_wrow_live : c->h_wrow;  // the host copy of bk's rows
  if (wrow.size() != 16 * (size_t)bk.nwb) return 1;
  if (!(c->int_ok && lo >= c->int_lo && hi <= c->int_hi && wrow == c->int_wrow)) {
    // a range already found too wide (within the failed one, same layout and generators): no second attempt
    if (c->int_failed && lo <= c->int_fail_lo && hi >= c->int_fail_hi && wrow == c->int_wrow) return 1;
    const double w = std::max(hi - lo, 1e-3 * std::max(1.0, std::max(std::fabs(lo), std::fabs(hi))));
    r = blkp_interp_coeffs(c, wrow, lo - 0.05 * w, hi + 0.05 * w);
    if (r == 1) r = blkp_interp_coeffs(c, wrow, lo, hi);  // without the margin
    if (r) {
      c->int_ok = false;
      if (r == 1) {
        c->int_failed = true;
        c->int_fail_lo = lo;
        c->int_fail_hi = hi;
        c->int_wrow = wrow;
      }
      return r;
    }
    c->int_failed = false;
  }
  blkp_interp_args(c, bk, ia);
  return QOC_OK;
}

// The formation's arguments and launch shape, the chain kernels' chunk size
struct BlkpPlan {
  BlkpArgs a;
  void (*kern)(BlkpArgs);
  size_t lds;
  int per_cu;
  int ch;
  size_t clds;
  bool interp;  // the formation interpolates (k_blkp_int)
  BlkpIntArgs ia;
};
// form: the plan of a launch that forms propagators (the interpolation's setup reads the control range)
static int blkp_plan(qoc_ctx* c, const BlkArgs& bk, int parts, BlkpPlan& pl, bool form = true) {
  BlkpArgs& a = pl.a;
  a = BlkpArgs{};
  a.N = c->N;
  a.nu = c->nu;
  a.nwb = bk.nwb;
  a.skew = c->skew_exact && c->tprm.mur[0] == 0.0 && c->tprm.mur[1] == 0.0 && c->tprm.mur[2] == 0.0;
  a.four = getenv("QOC_BLKP_4M") && atoi(getenv("QOC_BLKP_4M")) != 0;
  // one product more for one squaring fewer (default): each squaring doubles the rounding error a slice carries over
  // 2000 chained slices (tunable bus, all 512 seeds against the C port: max |ΔJ| 4.7e-12 with the fewest products,
  // 9.1e-13 with slack 1 at 11.75 instead of 10.75 products per unit; tools/blkp_accuracy.py)
  a.slack = getenv("QOC_BLKP_SLACK") ? std::max(0, atoi(getenv("QOC_BLKP_SLACK"))) : 1;
  // the accurate (r, s) choice by default (BlkpArgs::rcap): pieces of norm <= 1, truncation 2^-3 ulp after the
  // squarings; QOC_BLKP_RCAP=0 keeps the fewest-products choice (QOC_BLKP_SLACK, QOC_BLKP_TAIL)
  a.rcap = getenv("QOC_BLKP_RCAP") ? std::max(0.0, atof(getenv("QOC_BLKP_RCAP"))) : 1.0;
  a.tail = getenv("QOC_BLKP_TAIL") ? std::max(0, atoi(getenv("QOC_BLKP_TAIL"))) : a.rcap > 0.0 ? 3 : 0;
  if (a.tail > 0) blkp_theta_table(a.tail, a.theta);
  a.wrow = bk.wrow;
  a.At = (const cx<double>*)c->d_At;
  a.u = c->d_u;
  for (int j = 0; j < 3; ++j) {
    a.mur[j] = j <= c->nu ? c->tprm.mur[j] : 0.0;
    a.mui[j] = j <= c->nu ? c->tprm.mui[j] : 0.0;
  }
  a.prods = c->d_terms;  // qoc_chain_terms: executed 16 x 16 complex products on this path
  pl.lds = (size_t)bk.nwb * 768 * sizeof(double2) + (size_t)(BLKP_WG / 64) * BLKP_TP * sizeof(double2);
  const char* oc = getenv("QOC_BLKP_OCC");
  const bool occ3 = !(oc && atoi(oc) == 2);
  pl.kern = c->nu == 1 ? (occ3 ? k_blkp_exp<1, 3> : k_blkp_exp<1, 2>) : (occ3 ? k_blkp_exp<2, 3> : k_blkp_exp<2, 2>);
  // skew-Hermitian blocks: the Chebyshev form (QOC_BLKP_CHEB = block size 4 or 6, 0 off; QOC_BLKP_CRMAX the largest
  // ρ_c before a squaring, 8 or 16)
  int cm = 0;
  if (const char* ce = getenv("QOC_BLKP_CHEB")) cm = atoi(ce);
  if (cm != 4 && cm != 6) cm = 0;
  if (!a.skew) cm = 0;
  if (cm) {
    const double crmax = getenv("QOC_BLKP_CRMAX") && atof(getenv("QOC_BLKP_CRMAX")) >= 16.0 ? 16.0 : 8.0;
    if (int r = blkp_cheb_table(c, cm, crmax)) return r;
    a.ctab = c->d_blkp_ctab;
    a.cgn = BLKP_CT_G0 + (int)std::lround(4.0 * std::log2(crmax)) + 1;
    a.crmax = crmax;
    pl.kern = cm == 4 ? (c->nu == 1 ? k_blkp_exp<1, 3, 4> : k_blkp_exp<2, 3, 4>)
                      : (c->nu == 1 ? k_blkp_exp<1, 2, 6> : k_blkp_exp<2, 2, 6>);
  }
  HIPCHK(c, blk_lds_attr(pl.kern, pl.lds));
  const int waves = bk.nwb * c->m;
  int ch = blkp_chunk(waves, parts);
  if (const char* ce = getenv("QOC_BLKP_CH")) {
    const int v = atoi(ce);
    if (v == 1 || v == 2 || v == 4 || v == 8) ch = v;
  }
  if (blkp_chain_lds(c->N, c->m, waves, ch) > 160 * 1024) ch = blkp_chunk(waves);
  pl.ch = ch;
  pl.clds = blkp_chain_lds(c->N, c->m, waves, ch);
  pl.per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pl.per_cu, (const void*)pl.kern, BLKP_WG, pl.lds) != hipSuccess ||
      pl.per_cu < 1)
    pl.per_cu = 2;
  if (parts > 1) pl.per_cu = std::min(pl.per_cu, 2);  // a chain workgroup fits beside the formation
  pl.interp = false;
  if (form) {
    const int ri = blkp_interp_setup(c, bk, pl.ia);
    if (ri > 1 || ri < 0) return ri;
    pl.interp = ri == 0;
    c->last_int_D = pl.interp ? pl.ia.D : 0;
  }
  return QOC_OK;
}
// the formation of units [unit0, units) into UF (which holds unit ubase at its start)
static int blkp_launch_exp(qoc_ctx* c, BlkpPlan& pl, long long unit0, long long units, double2* UF, long long ubase) {
  if (pl.interp) {  // seed groups cover whole (seed, slice) slots: units are multiples of nwb
    BlkpIntArgs& ia = pl.ia;
    ia.slot0 = unit0 / ia.nwb;
    ia.slots = units / ia.nwb;
    ia.ubase = ubase;
    ia.UF = UF;
    // as many blocks per launch as their coefficients fit the LDS
    const int per = std::max(1, std::min(ia.nwb, (int)((size_t)150 * 1024 / blkp_int_lds(1, ia.D))));
    for (int b0 = 0; b0 < ia.nwb; b0 += per) {
      ia.beta0 = b0;
      ia.nb = std::min(per, ia.nwb - b0);
      // workgroups of 4 waves (QOC_BLKP_INT_WG=8: 8 waves), 4 units per wave (QOC_BLKP_INT_UPW=8: 8), up to 4
      // workgroups per CU in the grid (one holds the LDS at a time when the coefficients exceed 80 KB)
      const bool w8 = getenv("QOC_BLKP_INT_WG") && atoi(getenv("QOC_BLKP_INT_WG")) == 8;
      const bool u8 = getenv("QOC_BLKP_INT_UPW") && atoi(getenv("QOC_BLKP_INT_UPW")) == 8;
      const int iw = w8 ? 8 : 4, upw = u8 ? 8 : 4;
      auto kern = u8 ? (w8 ? k_blkp_int<8, 512> : k_blkp_int<8, 256>) : (w8 ? k_blkp_int<4, 512> : k_blkp_int<4, 256>);
      HIPCHK(c, blk_lds_attr(kern, blkp_int_lds(ia.nb, ia.D)));
      const long long items = (ia.slots - ia.slot0 + upw - 1) / upw * ia.nb;
      const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>((items + iw - 1) / iw, (long long)c->ncu * 4));
      const int mk = mark_begin(c, 0);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * iw), blkp_int_lds(ia.nb, ia.D), c->stream, ia);
      mark_end(c, mk);
      HIPCHK(c, hipGetLastError());
    }
    return QOC_OK;
  }
  pl.a.unit0 = unit0;
  pl.a.units = units;
  pl.a.UF = UF;
  pl.a.ubase = ubase;
  const unsigned grid = (unsigned)std::max<long long>(
      1, std::min<long long>((units - unit0 + BLKP_WG / 64 - 1) / (BLKP_WG / 64), (long long)c->ncu * pl.per_cu));
  const int mk = mark_begin(c, 0);
  hipLaunchKernelGGL(pl.kern, dim3(grid), dim3(BLKP_WG), pl.lds, c->stream, pl.a);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}
// one direction's chains for seeds [s0, s1) from the propagators in U (seed useed0's first)
template <bool FWD>
static int blkp_launch_chain(qoc_ctx* c, const BlkpPlan& pl, const TChainArgs& g, const BlkArgs& bk, const double2* U,
                             int s0, int s1, int useed0, hipStream_t st, const int* stale) {
  auto chain = pl.ch == 8   ? k_blkp_chain<FWD, 8>
               : pl.ch == 4 ? k_blkp_chain<FWD, 4>
               : pl.ch == 2 ? k_blkp_chain<FWD, 2>
                            : k_blkp_chain<FWD, 1>;
  HIPCHK(c, blk_lds_attr(chain, pl.clds));
  const int mk = mark_begin(c, FWD ? 1 : 2, st);
  hipLaunchKernelGGL(chain, dim3(s1 - s0), dim3(64 * bk.nwb * c->m), pl.clds, st, g, bk, U, s0, useed0, stale);
  mark_end(c, mk, st);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}
// the order-3 gradient from x_k, μ_{k+1} and the λ_N coefficients
static int blkp_launch_grad(qoc_ctx* c, const BlkArgs& bk, double* d_dJdu, const int* stale, cx<double>* coef_out) {
  BlkpGradArgs ga{};
  ga.N = c->N;
  ga.m = c->m;
  ga.Nt = c->Nt;
  ga.nwb = bk.nwb;
  ga.wrow = bk.wrow;
  ga.A = (const cx<double>*)c->d_A;
  ga.u = c->d_u;
  ga.X = (const cx<double>*)c->d_X;
  ga.L = (const cx<double>*)c->d_L;
  ga.coef = c->d_coef;
  ga.dJdu = d_dJdu;
  ga.tiles = (long long)c->B * ((c->Nt + 15) / 16);
  ga.stale = stale;
  ga.coef_out = coef_out;
  // generators diagonal on the live wave blocks' rows (QOC_BLKP_GDIAG=0: every product on MFMA)
  ga.diag = 0;
  if (!(getenv("QOC_BLKP_GDIAG") && atoi(getenv("QOC_BLKP_GDIAG")) == 0)) {
    const std::vector<int>& wrow = bk.wrow == c->d_wrow_live ? c->h_wrow_live : c->h_wrow;
    const size_t NN = (size_t)c->N * c->N;
    for (int j = 1; j <= c->nu && wrow.size() == 16 * (size_t)bk.nwb; ++j) {
      bool dg = true;
      for (int w = 0; w < bk.nwb && dg; ++w)
        for (int r = 0; r < 16 && dg; ++r)
          for (int q = 0; q < 16 && dg; ++q) {
            const int row = wrow[16 * w + r], col = wrow[16 * w + q];
            if (row < 0 || col < 0 || row == col) continue;
            const double* z = c->h_gen.data() + 2 * (j * NN + row + (size_t)c->N * col);
            dg = z[0] == 0.0 && z[1] == 0.0;
          }
      if (dg) ga.diag |= 1u << j;
    }
  }
  const size_t glds = blkp_grad_lds(bk.nwb, c->nu);
  auto gk = c->nu == 1 ? k_blkp_grad<1> : k_blkp_grad<2>;
  HIPCHK(c, blk_lds_attr(gk, glds));
  int gpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&gpc, (const void*)gk, 256, glds) != hipSuccess || gpc < 1) gpc = 2;
  const unsigned ggrid = (unsigned)std::max<long long>(1, std::min<long long>((ga.tiles + 3) / 4, (long long)c->ncu * gpc));
  const int mg = mark_begin(c, 3);
  hipLaunchKernelGGL(gk, dim3(ggrid), dim3(256), glds, c->stream, ga);
  mark_end(c, mg);
  HIPCHK(c, hipGetLastError());
  return QOC_OK;
}
// the interpolating chains (k_blkp_ichain) apply: the interpolation (one control), one live wave block, one state
// column, and the block's coefficients in the LDS beside four waves' rows (QOC_BLKP_ICHAIN=0: the stored form)
constexpr int BLKP_ISL = 8;  // slices per chunk
static bool blkp_ichain_sym(const BlkpIntArgs& ia) {  // complex-symmetric generators: the upper triangle alone
  return ia.Msym && !(getenv("QOC_BLKP_ISYM") && atoi(getenv("QOC_BLKP_ISYM")) == 0);
}
// 0: the stored form, 1: the interpolating chains (every entry), 2: the same on the upper triangle
static int blkp_ichain_on(const qoc_ctx* c, const BlkArgs& bk, const BlkpPlan& pl) {
  const char* env = getenv("QOC_BLKP_ICHAIN");
  if (env && atoi(env) == 0) return 0;
  const bool sym = pl.interp && blkp_ichain_sym(pl.ia);
  if (!(pl.interp && bk.nwb == 1 && c->m == 1 && blkp_ichain_lds(pl.ia.D, BLKP_ISL, 4, sym) <= 160 * 1024)) return 0;
  return sym ? 2 : 1;
}
// dual: the forward chain and the μ recurrence of every seed (one launch), else direction dir alone; the forward's
// terminal cost and λ_N coefficients by k_terminal_cost (64 threads: chain_costs as the one-wave chain workgroups run
// it, the same sums); stale: a queued stale-u flag (nonzero: nothing is written)
static int blkp_launch_ichain(qoc_ctx* c, const TChainArgs& gf, const TChainArgs& gb, const BlkArgs& bk,
                              const BlkpIntArgs& ia0, bool dual, int dir, const int* stale) {
  // the slices' e^{μ(u_k)} first (one sincos per (seed, slice) instead of one per chain wave)
  const size_t nph = (size_t)c->B * c->Nt;
  if (c->blkp_ph_n < nph) {
    if (c->d_blkp_ph) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipFree(c->d_blkp_ph));
      c->d_blkp_ph = nullptr;
    }
    HIPCHK(c, hipMalloc((void**)&c->d_blkp_ph, nph * sizeof(double2)));
    c->blkp_ph_n = nph;
  }
  BlkpIntArgs ia = ia0;
  ia.ph = c->d_blkp_ph;
  hipLaunchKernelGGL(k_blkp_phase, dim3((unsigned)std::min<size_t>((nph + 255) / 256, 4096)), dim3(256), 0, c->stream, ia,
                     (long long)nph);
  HIPCHK(c, hipGetLastError());
  // (the next chunk's interpolation interleaved with this chunk's steps measured slower: 2.45 ms at SL = 4, 2.68 ms at
  // SL = 8 with AGPR spills, against 1.95 ms in sequence; profiles/r06v_ichain_ab.txt)
  // complex-symmetric generators: the upper triangle alone (QOC_BLKP_ISYM=0: every entry)
  const bool sym = blkp_ichain_sym(ia);
  // two waves per (seed, direction) on one SIMD, taking alternate chunks (QOC_BLKP_IPAIR=0: one wave)
  const int pairs = (dual ? 2 : 1) * c->B;
  // pairs per workgroup: 4 (the two waves of a pair on one SIMD) unless that leaves CUs without one, then 2
  int npw = pairs >= 4 * c->ncu ? 4 : 2;
  // (QOC_BLKP_IPW=2 on the dual launch: two workgroups per CU, the pairs' waves on different SIMDs)
  if (const char* e = getenv("QOC_BLKP_IPW")) npw = atoi(e) == 4 ? 4 : 2;  // (tests: force either)
  const bool pair = !(getenv("QOC_BLKP_IPAIR") && atoi(getenv("QOC_BLKP_IPAIR")) == 0) &&
                    blkp_ipair_lds(ia.D, BLKP_ISL, sym, npw) <= 160 * 1024;
  auto kern = pair ? (sym ? k_blkp_ichain2<BLKP_ISL, true> : k_blkp_ichain2<BLKP_ISL, false>)
                   : (sym ? k_blkp_ichain<BLKP_ISL, true> : k_blkp_ichain<BLKP_ISL, false>);
  const size_t lds = pair ? blkp_ipair_lds(ia.D, BLKP_ISL, sym, npw) : blkp_ichain_lds(ia.D, BLKP_ISL, 4, sym);
  HIPCHK(c, blk_lds_attr(kern, lds));
  const int per = pair ? npw : 4;  // (seed, direction) pairs per workgroup
  const int mk = mark_begin(c, dual || dir == 0 ? 1 : 2);
  hipLaunchKernelGGL(kern, dim3((pairs + per - 1) / per), dim3(pair ? 128 * npw : 256), lds, c->stream, gf, gb, bk, ia,
                     0, c->B, dual ? 1 : 0, dir, stale);
  mark_end(c, mk);
  HIPCHK(c, hipGetLastError());
  if (dual || dir == 0) {
    hipLaunchKernelGGL(k_terminal_cost<double>, dim3(c->B), dim3(64), 0, c->stream, c->N, c->m, c->Nt,
                       (const cx<double>*)gf.X, (const cx<double>*)gf.Xt, gf.cost_kind, gf.n_norm, 0, gf.J, gf.coef,
                       gf.sc);
    HIPCHK(c, hipGetLastError());
  }
  return QOC_OK;
}
static int blkp_parts(const qoc_ctx* c) {
  int parts = 4;
  if (const char* pe = getenv("QOC_BLKP_PARTS")) parts = atoi(pe);
  return std::max(1, std::min(parts, c->B));
}

// qoc_eval_dev: U_k per (seed, slice, live block) on MFMA, the forward chain and the μ recurrence from the stored
// propagators, then the order-3 gradient.  The formation is MFMA-bound and the chains are bound by their propagator
// reads: the seeds go in `parts` groups, the chains of group p (second stream) beside the formation of group p + 1, with
// the formation at two workgroups per CU so that a chain workgroup fits beside them (QOC_BLKP_PARTS, default 4; 1: one
// formation, then the chains).  The propagators of two groups are held at a time (the formation of group p + 2 waits
// for the chains of group p): 2.1 GB at the tunable bus' B = 512 instead of every seed's 4.2 GB.  Returns 1 (nothing
// launched) when even that does not fit in the free HBM: the Chebyshev block chains then run.
static int blkp_eval_concurrent(qoc_ctx* c, double* d_dJdu, const BlkArgs& bk) {
  TChainArgs gf = tchain_args(c);
  TChainArgs gb = tchain_args(c);
  gb.mu_mode = 1;
  int r;
  const int parts = blkp_parts(c);
  const long long per_seed = (long long)c->Nt * bk.nwb;  // units per seed
  const int gmax = (c->B + parts - 1) / parts;           // seeds of the largest group
  const int nslab = parts > 1 ? 2 : 1;
  const size_t slab = (size_t)gmax * per_seed * 256;      // double2 per slab
  BlkpPlan pl;
  if ((r = blkp_plan(c, bk, parts, pl))) return r;
  c->ichain_last = blkp_ichain_on(c, bk, pl);
  if (c->ichain_last) {  // both chains interpolate their own propagators: nothing stored
    if (bk.nwb != c->nwb) {
      if ((r = blk_zero_dead(c, {c->d_X, c->d_L}))) return r;
    }
    if ((r = blkp_launch_ichain(c, gf, gb, bk, pl.ia, true, 0, nullptr))) return r;
    c->fwd_captured = false;
    c->props_since_reset++;
    c->steps_stale = true;
    if ((r = blkp_launch_grad(c, bk, d_dJdu, nullptr, c->d_coef_mu))) return r;
    c->L_is_mu = true;
    c->last_eval_mode = 7;
    return QOC_OK;
  }
  if ((r = blkp_ensure_store(c, nslab * slab * sizeof(double2), true))) return r;  // 1: does not fit
  if (bk.nwb != c->nwb) {
    if ((r = blk_zero_dead(c, {c->d_X, c->d_L}))) return r;
  }
  // events: [p] group p formed, [parts + p] group p's chains done, [2 parts] everything queued before
  if (parts > 1) {
    if ((r = ensure_stream2(c, 2 * parts + 1))) return r;
    HIPCHK(c, hipEventRecord(c->sync_ev[2 * parts], c->stream));  // the second stream after everything queued so far
    HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[2 * parts], 0));
  }
  hipStream_t cs = parts > 1 ? c->stream2 : c->stream;
  // QOC_BLKP_PRIO=1: the chain waves at the top issue priority.  Measured: each group's chains 1.63 -> 1.07 ms, the
  // formation beside them 1.85 -> 1.97 ms per group, and the formation is the critical path (8.72 vs 8.93 ms per
  // eval), so off by default
  const int cprio = getenv("QOC_BLKP_PRIO") ? atoi(getenv("QOC_BLKP_PRIO")) : 0;
  auto chain = pl.ch == 8 ? k_blkp_dual<8> : pl.ch == 4 ? k_blkp_dual<4> : pl.ch == 2 ? k_blkp_dual<2> : k_blkp_dual<1>;
  HIPCHK(c, blk_lds_attr(chain, pl.clds));
  const int waves = bk.nwb * c->m;
  for (int p = 0; p < parts; ++p) {
    const int s0 = (int)((long long)c->B * p / parts), s1 = (int)((long long)c->B * (p + 1) / parts);
    if (s1 <= s0) continue;
    double2* const U = (double2*)c->d_blkU + (size_t)(p % nslab) * slab;
    if (p >= 2) HIPCHK(c, hipStreamWaitEvent(c->stream, c->sync_ev[parts + p - 2], 0));  // slab p % 2 read out
    if ((r = blkp_launch_exp(c, pl, (long long)s0 * per_seed, (long long)s1 * per_seed, U, (long long)s0 * per_seed)))
      return r;
    if (parts > 1) {
      HIPCHK(c, hipEventRecord(c->sync_ev[p], c->stream));
      HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[p], 0));
    }
    const int mk = mark_begin(c, 1, cs);
    hipLaunchKernelGGL(chain, dim3(2 * (s1 - s0)), dim3(64 * waves), pl.clds, cs, gf, gb, bk, (const double2*)U, s0, s0,
                       cprio);
    mark_end(c, mk, cs);
    HIPCHK(c, hipGetLastError());
    if (parts > 1) HIPCHK(c, hipEventRecord(c->sync_ev[parts + p], c->stream2));
  }
  if (parts > 1) {  // the gradient (and everything after it on the engine stream) after the last chains
    HIPCHK(c, hipEventRecord(c->sync_ev[2 * parts], c->stream2));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->sync_ev[2 * parts], 0));
  }
  c->fwd_captured = false;
  c->props_since_reset++;
  c->steps_stale = true;  // d_steps still holds the last k_tchain_prep's records, not this u's
  if ((r = blkp_launch_grad(c, bk, d_dJdu, nullptr, c->d_coef_mu))) return r;
  c->L_is_mu = true;
  c->last_eval_mode = 7;
  return QOC_OK;
}

// the stored-propagator eval applies (blocks of 5..16 rows with a live-wave layout that fits the chain and gradient
// kernels)
static bool blkp_fits(qoc_ctx* c, const BlkArgs& bk) {
  const int waves = bk.nwb * c->m;
  return waves <= 8 && blkp_chain_lds(c->N, c->m, waves, blkp_chunk(waves)) <= 160 * 1024 &&
         blkp_grad_lds(bk.nwb, c->nu) <= 160 * 1024;
}

// propagate on stored propagators (the reference's own structure, src/gradient_computations.jl:17-29): every U_k of
// the live blocks formed on MFMA, the forward chain from them (seed groups pipelined as in the eval), states in d_X;
// the propagators stay for grape_sensitivity (every seed's: 4.2 GB at the tunable bus' B = 512).  Built-in costs, no
// penalty; QOC_BLKP_SPLIT=0 keeps the Chebyshev block chains.  Returns 1 (nothing launched) when it does not apply.
int blkp_forward(qoc_ctx* c) {
  const char* env = getenv("QOC_BLKP_SPLIT");
  if ((env && atoi(env) == 0) || !blkp_on(c) || c->mu != 0.0 ||
      (c->cost_kind != QOC_COST_TRACE && c->cost_kind != QOC_COST_ZCAL))
    return 1;
  BlkArgs bk = blk_args(c);
  int r = blk_live(c, bk);
  if (r) return r;
  if (!blkp_fits(c, bk)) return 1;
  const long long per_seed = (long long)c->Nt * bk.nwb;
  const int parts = blkp_parts(c);
  BlkpPlan pl;
  if ((r = blkp_plan(c, bk, parts, pl))) return r;
  const TChainArgs gf = tchain_args(c);
  c->ichain_last = blkp_ichain_on(c, bk, pl);
  c->ichain_fwd = c->ichain_last != 0;
  if (c->ichain_fwd) {  // the forward chain interpolates its propagators; grape_sensitivity's μ recurrence will too
    if (bk.nwb != c->nwb) {
      if ((r = blk_zero_dead(c, {c->d_X, c->d_L}))) return r;
    }
    if ((r = blkp_launch_ichain(c, gf, gf, bk, pl.ia, false, 0, nullptr))) return r;
    c->fwd_captured = false;
    c->props_since_reset++;
    c->steps_stale = true;
    c->fwd_kind = 2;
    return QOC_OK;
  }
  if ((r = blkp_ensure_store(c, (size_t)c->B * per_seed * 256 * sizeof(double2), true))) return r;
  if (bk.nwb != c->nwb) {
    if ((r = blk_zero_dead(c, {c->d_X, c->d_L}))) return r;
  }
  if (parts > 1) {
    if ((r = ensure_stream2(c, parts + 1))) return r;
    HIPCHK(c, hipEventRecord(c->sync_ev[parts], c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[parts], 0));
  }
  hipStream_t cs = parts > 1 ? c->stream2 : c->stream;
  double2* const U = (double2*)c->d_blkU;
  for (int p = 0; p < parts; ++p) {
    const int s0 = (int)((long long)c->B * p / parts), s1 = (int)((long long)c->B * (p + 1) / parts);
    if (s1 <= s0) continue;
    if ((r = blkp_launch_exp(c, pl, (long long)s0 * per_seed, (long long)s1 * per_seed, U, 0))) return r;
    if (parts > 1) {
      HIPCHK(c, hipEventRecord(c->sync_ev[p], c->stream));
      HIPCHK(c, hipStreamWaitEvent(c->stream2, c->sync_ev[p], 0));
    }
    if ((r = blkp_launch_chain<true>(c, pl, gf, bk, U, s0, s1, 0, cs, nullptr))) return r;
  }
  if (parts > 1) {
    HIPCHK(c, hipEventRecord(c->sync_ev[parts], c->stream2));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->sync_ev[parts], 0));
  }
  c->fwd_captured = false;
  c->props_since_reset++;
  c->steps_stale = true;  // d_steps holds another u's step records (the Chebyshev backward re-preps first)
  c->fwd_kind = 2;
  return QOC_OK;
}

bool blkp_backward_ok(const qoc_ctx* c, int order) {
  return c->fwd_kind == 2 && order == 3 && c->mu == 0.0 && !c->src_on &&
         (c->cost_kind == QOC_COST_TRACE || c->cost_kind == QOC_COST_ZCAL) && (c->ichain_fwd || c->d_blkU);
}

// grape_sensitivity after blkp_forward: the μ recurrence from the stored propagators (μ_N = X_target, λ_k = coef ⊙ μ_k,
// src/penalty_fcns.jl:19-22, 35-40), then the order-3 gradient; stale: the device flag of a queued stale-u check
int blkp_backward(qoc_ctx* c, double* d_dJdu, const int* stale) {
  BlkArgs bk = blk_args(c);
  int r = blk_live(c, bk);
  if (r) return r;
  if (!c->d_coef_mu) {
    HIPCHK(c, hipMalloc((void**)&c->d_coef_mu, (size_t)c->B * 2 * c->m_user * sizeof(cx<double>)));
    c->dev_bytes += (size_t)c->B * 2 * c->m_user * sizeof(cx<double>);
  }
  TChainArgs gb = tchain_args(c);
  gb.mu_mode = 1;
  if (c->ichain_fwd) {  // the propagate interpolated: the μ recurrence from the same coefficients (the same u)
    BlkpIntArgs ia;
    blkp_interp_args(c, bk, ia);
    if ((r = blkp_launch_ichain(c, gb, gb, bk, ia, false, 1, stale))) return r;
  } else {
    BlkpPlan pl;
    if ((r = blkp_plan(c, bk, 1, pl, false))) return r;
    if ((r = blkp_launch_chain<false>(c, pl, gb, bk, (const double2*)c->d_blkU, 0, c->B, 0, c->stream, stale)))
      return r;
  }
  if ((r = blkp_launch_grad(c, bk, d_dJdu, stale, c->d_coef_mu))) return r;
  c->L_is_mu = true;
  c->last_eval_mode = 7;
  return QOC_OK;
}

int blk_eval_concurrent(qoc_ctx* c, int order, double* d_dJdu) {
  if (blku_on(c)) return blku_eval_concurrent(c, order, d_dJdu);
  if (!c->d_coef_mu) {
    HIPCHK(c, hipMalloc((void**)&c->d_coef_mu, (size_t)c->B * 2 * c->m_user * sizeof(cx<double>)));
    c->dev_bytes += (size_t)c->B * 2 * c->m_user * sizeof(cx<double>);
  }
  int r;
  if (blkp_on(c)) {
    BlkArgs bk = blk_args(c);
    if ((r = blk_live(c, bk))) return r;
    if (blkp_fits(c, bk)) {
      r = blkp_eval_concurrent(c, d_dJdu, bk);
      if (r != 1) return r;  // 1: the propagators do not fit in HBM: the Chebyshev block chains below
    }
  }
  if ((r = blk_big(c) ? ensure_pws(c) : QOC_OK)) return r;
  if ((r = tchain_prep(c))) return r;
  TChainArgs gf = tchain_args(c);
  TChainArgs gb = tchain_args(c);
  gb.mu_mode = 1;
  if (blk_big(c)) {  // the first two products of every slice for k_grad_rr_c (forward -> d_pws, μ -> d_gws)
    const size_t bufN = (size_t)c->N * ((size_t)c->B * (c->Nt + 1) * c->m);
    gf.cap1 = c->d_pws;
    gf.cap2 = (cx<double>*)c->d_pws + bufN;
    gb.cap1 = c->d_gws;
    gb.cap2 = (cx<double>*)c->d_gws + bufN;
  }
  BlkArgs bk = blk_args(c);
  if ((r = blk_live(c, bk))) return r;
  const bool skip = bk.nwb != c->nwb;
  const size_t lds = blk_lds_of(c, bk.nwb);
  const int thr = blk_threads(c, bk.nwb);
  if (skip) {
    if ((r = blk_zero_dead(c, {c->d_X, c->d_L, (void*)gf.cap1, (void*)gf.cap2, (void*)gb.cap1, (void*)gb.cap2})))
      return r;
  }
  const int mk = mark_begin(c, 1);
  const hipError_t e = blk_dispatch(c, [&](auto NB_, auto CH_) {
    constexpr int NB = decltype(NB_)::value;
    constexpr bool CH = decltype(CH_)::value;
    if constexpr (NB < 100) {
      const hipError_t q = blk_lds_attr(k_blkrot_dual<NB, CH>, lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL((k_blkrot_dual<NB, CH>), dim3(2 * c->B), dim3(thr), lds, c->stream, gf, gb, bk);
    }
    else hipLaunchKernelGGL((k_blk_dual<NB - 100, CH>), dim3(2 * c->B), dim3(thr), lds, c->stream, gf, gb, bk);
    return hipGetLastError();
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blk_dual launch: %s", hipGetErrorString(e));
  c->fwd_captured = false;  // the block backward recomputes its own products
  c->props_since_reset++;
  if (blk_big(c)) {
    const int mg = mark_begin(c, 3);
    r = grad_rr_cap(c, d_dJdu, c->stream, 0, c->Nt, true);
    mark_end(c, mg);
  } else {
    r = blk_grad(c, order, true, d_dJdu);
  }
  if (r) return r;
  HIPCHK(c, hipMemcpyAsync(c->d_coef_mu, c->d_coef, (size_t)c->B * 2 * c->m * sizeof(cx<double>),
                           hipMemcpyDeviceToDevice, c->stream));
  c->L_is_mu = true;
  c->last_eval_mode = 4;
  return QOC_OK;
}

// ---- block propagators (qoc_blku.hpp) ----------------------------------------------------------------------------
template <typename F>
static hipError_t blku_dispatch(const qoc_ctx* c, F&& f) {
  using std::integral_constant;
  switch (c->blk_nb) {
    case 2: return f(integral_constant<int, 2>());
    case 3: return f(integral_constant<int, 3>());
    case 4: return f(integral_constant<int, 4>());
  }
  return hipErrorInvalidValue;
}

// the gradient order 1..4 as a compile-time constant
template <typename F>
static hipError_t blk_order_dispatch(int order, F&& f) {
  using std::integral_constant;
  switch (order) {
    case 1: return f(integral_constant<int, 1>());
    case 2: return f(integral_constant<int, 2>());
    case 3: return f(integral_constant<int, 3>());
    default: return f(integral_constant<int, 4>());
  }
}

// the prefix-product group size as a compile-time constant (1, or 2 for blocks of <= 3 rows)
template <int NB, typename F>
static hipError_t blku_sdispatch(int S, F&& f) {
  using std::integral_constant;
  if constexpr (NB <= 3)
    if (S == 2) return f(integral_constant<int, 2>());
  return f(integral_constant<int, 1>());
}

static hipError_t blku_launch_fwd_g(qoc_ctx* c, const TChainArgs& g, const BlkuShape& s, const BlkuParams& bp) {
  const BlkArgs bk = blk_args(c);
  return blku_dispatch(c, [&](auto NB_) {
    constexpr int NB = decltype(NB_)::value;
    return blku_sdispatch<NB>(s.S, [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      const hipError_t q = blk_lds_attr(k_blku_fwd<NB, S>, s.lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL((k_blku_fwd<NB, S>), dim3(c->B), dim3(64 * s.W), s.lds, c->stream, g, bk, bp);
      return hipGetLastError();
    });
  });
}

static hipError_t blku_launch_fwd(qoc_ctx* c, const BlkuShape& s, const BlkuParams& bp) {
  return blku_launch_fwd_g(c, tchain_args(c), s, bp);
}

static int blku_forward(qoc_ctx* c) {
  const BlkuShape s = blku_shape(c, false);
  BlkuParams bp = blku_params(c, s);
  int r = blku_records(c, bp, true);
  if (r) return r;
  const int mk = mark_begin(c, 1);
  const hipError_t e = blku_launch_fwd(c, s, bp);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_fwd launch: %s", hipGetErrorString(e));
  c->fwd_captured = false;
  c->props_since_reset++;
  return QOC_OK;
}

// the order-o gradient from d_X and d_L (mu_mode: d_L holds μ, λ = coef ⊙ μ with the coefficients in d_coef)
static int blku_grad(qoc_ctx* c, int order, bool mu_mode, double* d_dJdu) {
  const TChainArgs g = tchain_args(c);
  const BlkArgs bk = blk_args(c);
  const long long units = (long long)c->B * c->Nt;
  const int upw = 64 / blku_nbp(c->nblk);  // units per wave (blocks on power-of-two lane groups)
  if (upw < 1) return fail(c, QOC_ERR_UNSUPPORTED, "block gradient: %d blocks exceed one wave", c->nblk);
  const long long waves = (units + upw - 1) / upw;
  const unsigned blocks = (unsigned)std::max<long long>(1, std::min<long long>((waves + 3) / 4, (long long)c->ncu * 8));
  const size_t glds = blku_grad_lds(c->blk_nb, c->nblk);
  const int mk = mark_begin(c, 3);
  // the column count as a compile-time constant (operand prefetch) for blocks of 2 rows with m = 2 (cavity)
  const char* pf = getenv("QOC_BLKU_GRAD_PF");
  const bool m2 = c->blk_nb == 2 && c->m == 2 && !(pf && !std::strcmp(pf, "0"));
  const hipError_t e = blku_dispatch(c, [&](auto NB_) {
    constexpr int NB = decltype(NB_)::value;
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), glds, c->stream, g, bk, units, (int)mu_mode, d_dJdu);
      return hipGetLastError();
    };
    auto by_m = [&](auto ORD_) {
      constexpr int ORD = decltype(ORD_)::value;
      if constexpr (NB == 2) {
        if (m2) return launch(k_blku_grad<NB, ORD, 2>);
      }
      return launch(k_blku_grad<NB, ORD, 0>);
    };
    return blk_order_dispatch(order, by_m);
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_grad launch: %s", hipGetErrorString(e));
  return QOC_OK;
}

// the plain backward chain (λ_Nt -> λ_0 into d_L; add: the penalty / co-state source after every slice)
static hipError_t blku_launch_bwd(qoc_ctx* c, const TChainArgs& g, const BlkuShape& s, const BlkuParams& bp, bool add) {
  const BlkArgs bk = blk_args(c);
  return blku_dispatch(c, [&](auto NB_) {
    constexpr int NB = decltype(NB_)::value;
    auto launch = [&](auto kern) {
      const hipError_t q = blk_lds_attr(kern, s.lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL(kern, dim3(c->B), dim3(64 * s.W), s.lds, c->stream, g, bk, bp);
      return hipGetLastError();
    };
    if (add) return launch(k_blku_bwd<NB, 1, true>);  // additions after every slice: no prefix groups
    return blku_sdispatch<NB>(s.S, [&](auto S_) { return launch(k_blku_bwd<NB, decltype(S_)::value, false>); });
  });
}

// The fused backward (k_blku_bwdg): orders 1..4 without a penalty or co-state source.  λ stays in the workgroups;
// qoc_get_costates recomputes it on demand from a copy of this evaluation's u and λ_N coefficients (blku_costates).
static bool blku_fused_ok(const qoc_ctx* c, int order) {
  const char* env = getenv("QOC_BLKU_FUSED");
  return order >= 1 && order <= BLK_ORDMAX && c->mu == 0.0 && !c->src_on && !(env && !std::strcmp(env, "0")) &&
         blku_shape(c, true, false).W > 0;
}

static int blku_bwdg(qoc_ctx* c, int order, double* d_dJdu, const double2* Uin = nullptr) {
  const TChainArgs g = tchain_args(c);
  const BlkArgs bk = blk_args(c);
  const BlkuShape s = blku_shape(c, true, Uin != nullptr);
  if (s.W <= 0) return fail(c, QOC_ERR_UNSUPPORTED, "fused block backward: no worker wave fits the launch bound");
  BlkuParams bp = blku_params(c, s, d_dJdu);  // the records are current (the caller's)
  bp.Uin = Uin;
  bp.ustg = s.ustg;
  const int mk = mark_begin(c, 2);
  const hipError_t e = blku_dispatch(c, [&](auto NB_) {
    constexpr int NB = decltype(NB_)::value;
    return blku_sdispatch<NB>(s.S, [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      return blk_order_dispatch(order, [&](auto ORD_) {
        constexpr int ORD = decltype(ORD_)::value;
        const hipError_t q = blk_lds_attr(k_blku_bwdg<NB, S, ORD>, s.lds);
        if (q != hipSuccess) return q;
        hipLaunchKernelGGL((k_blku_bwdg<NB, S, ORD>), dim3(c->B), dim3(64 * s.W), s.lds, c->stream, g, bk, bp);
        return hipGetLastError();
      });
    });
  });
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_bwdg launch: %s", hipGetErrorString(e));
  // what qoc_get_costates needs to rebuild λ: this u and the λ_N coefficients (external λ_N stays in d_L)
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt, ncf = (size_t)c->B * 2 * c->m;
  if (!c->d_u_lam) {
    HIPCHK(c, hipMalloc((void**)&c->d_u_lam, nu_t * sizeof(double)));
    HIPCHK(c, hipMalloc((void**)&c->d_coef_lam, ncf * sizeof(cx<double>)));
    c->dev_bytes += nu_t * sizeof(double) + ncf * sizeof(cx<double>);
  }
  HIPCHK(c, hipMemcpyAsync(c->d_u_lam, c->d_u, nu_t * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_coef_lam, c->d_coef, ncf * sizeof(cx<double>), hipMemcpyDeviceToDevice, c->stream));
  c->L_lazy = true;
  c->last_eval_mode = 5;
  return QOC_OK;
}

// qoc_get_costates after a fused backward: the plain backward chain from the saved u and coefficients into d_L
int blku_costates(qoc_ctx* c) {
  if (!c->L_lazy) return QOC_OK;
  TChainArgs g = tchain_args(c);
  g.coef = c->d_coef_lam;
  g.u = c->d_u_lam;
  const BlkuShape s = blku_shape(c, false);
  BlkuParams bp = blku_params(c, s);
  int r = blku_records(c, bp, false, c->d_u_lam);
  if (r) return r;
  const hipError_t e = blku_launch_bwd(c, g, s, bp, false);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_bwd launch: %s", hipGetErrorString(e));
  c->L_lazy = false;
  return QOC_OK;
}

// grape_sensitivity: the fused backward when it applies; otherwise λ by the plain backward chain (penalty, co-state
// source and an external λ_N included), then the block gradient for orders 1..4 or the dense exact (Fréchet) one
static int blku_backward(qoc_ctx* c, int order, double* d_dJdu) {
  const TChainArgs g = tchain_args(c);
  const BlkuShape s = blku_shape(c, false);
  BlkuParams bp = blku_params(c, s);
  int r = blku_records(c, bp, false);  // the u of the last propagate (stale-checked by the caller)
  if (r) return r;
  if (blku_fused_ok(c, order)) return blku_bwdg(c, order, d_dJdu);
  const int mk = mark_begin(c, 2);
  const hipError_t e = blku_launch_bwd(c, g, s, bp, g.pmask || g.src);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_bwd launch: %s", hipGetErrorString(e));
  if (order == QOC_DUKDP_EXACT) return dense_gradient<double>(c, order, d_dJdu);
  return blku_grad(c, order, false, d_dJdu);
}

// qoc_eval_dev (built-in cost, no penalty, no co-state source): the step records once, the forward chain (J and the
// λ_N coefficients), then the fused backward -- x_k is written once and read once, λ never leaves the workgroups
static int blku_eval_concurrent(qoc_ctx* c, int order, double* d_dJdu) {
  BlkuShape s = blku_shape(c, false);
  // the forward's prefix groups apart from the backward's (QOC_BLKU_FS; the stored propagators are the plain ones)
  if (const char* fs = getenv("QOC_BLKU_FS")) {
    s.S = atoi(fs) >= 2 && c->blk_nb < 4 ? 2 : 1;
    s.C = std::max(s.C, s.S);
  }
  BlkuParams bp = blku_params(c, s);
  int r = blku_records(c, bp, true);
  if (r) return r;
  // the forward also stores the block propagators for the fused backward (which then forms none; its S = 1 only:
  // with prefix groups its chunks hold products); QOC_BLKU_STOREU=0 keeps the backward forming its own
  const char* su = getenv("QOC_BLKU_STOREU");
  const bool fused = blku_fused_ok(c, order);
  const bool storeu = fused && blku_shape(c, true, true).S == 1 && !(su && !std::strcmp(su, "0"));
  const size_t ubytes = (size_t)c->B * c->Nt * c->blk_nb * c->blk_nb * c->nblk * sizeof(double2);
  if (storeu && c->blkU_bytes < ubytes) {  // a new block layout (qoc_set_generators) may need more
    if (c->d_blkU) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipFree(c->d_blkU));
      c->d_blkU = nullptr;
      c->dev_bytes -= c->blkU_bytes;
      c->blkU_bytes = 0;
    }
    HIPCHK(c, hipMalloc((void**)&c->d_blkU, ubytes));
    c->blkU_bytes = ubytes;
    c->dev_bytes += ubytes;
  }
  bp.Uout = storeu ? (double2*)c->d_blkU : nullptr;
  const int mk = mark_begin(c, 1);
  const hipError_t e = blku_launch_fwd(c, s, bp);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_fwd launch: %s", hipGetErrorString(e));
  c->fwd_captured = false;
  c->props_since_reset++;
  if (fused) {
    r = blku_bwdg(c, order, d_dJdu, storeu ? (const double2*)c->d_blkU : nullptr);
  } else {
    const int mb = mark_begin(c, 2);
    const hipError_t eb = blku_launch_bwd(c, tchain_args(c), s, bp, false);
    mark_end(c, mb);
    if (eb != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_bwd launch: %s", hipGetErrorString(eb));
    r = blku_grad(c, order, false, d_dJdu);
    c->last_eval_mode = 4;  // the block chains' eval, λ in HBM
  }
  if (r) return r;
  c->L_is_mu = false;
  return QOC_OK;
}

// ---- segmented block eval (qoc_blkseg.hpp) -------------------------------------------------------------------------
struct BlksegShape {
  int W, S, L, UPW, RB;
  size_t lds;
};
// One workgroup per seed with W waves (8 at one seed per CU, fewer when several seeds share a CU: 8 wave slots at the
// kernel's <= 256 VGPRs), UPW = 64 / nblk segments per wave, S = W UPW segments of L = ceil(Nt / S) slices (then S
// trimmed so that no segment is empty).  QOC_BLKSEG_W / QOC_BLKSEG_S override the waves / cap the segments.
static BlksegShape blkseg_shape(const qoc_ctx* c) {
  BlksegShape s{};
  const int per_cu = std::max(1, std::min(8, (c->B + c->ncu - 1) / std::max(1, c->ncu)));
  s.W = std::max(1, 8 / per_cu);
  if (const char* env = getenv("QOC_BLKSEG_W")) s.W = std::max(1, std::min(8, atoi(env)));
  s.UPW = 64 / std::max(1, c->nblk);
  int S = std::max(1, std::min(s.W * s.UPW, c->Nt));
  if (const char* env = getenv("QOC_BLKSEG_S")) S = std::max(1, std::min(S, atoi(env)));
  s.L = (c->Nt + S - 1) / S;
  s.S = (c->Nt + s.L - 1) / s.L;
  s.W = (s.S + s.UPW - 1) / s.UPW;
  s.RB = blkseg_rb(s.UPW, c->nu);
  // blocks of 2 rows: up to 8 slice-steps per reduction when the LDS holds them (cavity: 0.0727 -> 0.0715 ms per launch,
  // the same sums in the same order, profiles/bench_r06zl_*); QOC_BLKSEG_RB overrides (up to 64 / (UPW nu))
  const int rbmax = std::max(1, 64 / (s.UPW * std::max(1, c->nu)));
  if (c->blk_nb == 2) {
    const int rb8 = std::min(8, rbmax);
    if (blkseg_lds(c->N, c->m, c->nu, c->blk_nb, c->nblk, c->Nt, s.S, s.W, rb8) <= (size_t)160 * 1024) s.RB = rb8;
  }
  if (const char* e = getenv("QOC_BLKSEG_RB")) s.RB = std::max(1, std::min(atoi(e), rbmax));
  s.lds = blkseg_lds(c->N, c->m, c->nu, c->blk_nb, c->nblk, c->Nt, s.S, s.W, s.RB);
  return s;
}

// The segmented eval applies to block propagators of blocks of <= 3 rows with exactly skew-Hermitian generators
// (unitary slices), the built-in costs, no penalty and no co-state source; QOC_BLKSEG=0 keeps the forward + fused
// backward of k_blku_*.
bool blkseg_ok(const qoc_ctx* c, int order) {
  if (!blku_on(c) || (c->blk_nb != 2 && c->blk_nb != 3) || !c->skew_exact || c->nblk > 32) return false;
  if (order < 1 || order > BLK_ORDMAX || c->mu != 0.0 || c->src_on) return false;
  if (c->cost_kind != QOC_COST_TRACE && c->cost_kind != QOC_COST_ZCAL) return false;
  const char* env = getenv("QOC_BLKSEG");
  if (env && !std::strcmp(env, "0")) return false;
  return blkseg_shape(c).lds <= (size_t)160 * 1024;
}

template <typename F>
static hipError_t blkseg_dispatch(int NB, int order, F&& f) {
  return blk_order_dispatch(order, [&](auto ORD_) {
    if (NB == 2) return f(std::integral_constant<int, 2>(), ORD_);
    return f(std::integral_constant<int, 3>(), ORD_);
  });
}

static int ensure_lazy_bufs(qoc_ctx* c) {
  const size_t nu_t = (size_t)c->B * c->nu * c->Nt, ncf = (size_t)c->B * 2 * c->m_user;
  if (!c->d_u_lam) {
    HIPCHK(c, hipMalloc((void**)&c->d_u_lam, nu_t * sizeof(double)));
    HIPCHK(c, hipMalloc((void**)&c->d_coef_lam, ncf * sizeof(cx<double>)));
    c->dev_bytes += nu_t * sizeof(double) + ncf * sizeof(cx<double>);
  }
  return QOC_OK;
}

// the launch parameters every mode shares; the best-(J, seed) epilogue's buffers on first use
static int blkseg_params(qoc_ctx* c, const BlksegShape& s, BlksegParams& sp) {
  sp = BlksegParams{};
  for (int j = 0; j < 3; ++j) {
    const bool on = j <= c->nu;
    sp.rad[j] = on ? c->tprm.rad[j] : 0.0;  // skew-Hermitian: spectral half-widths of the shifted generators
    sp.mur[j] = on ? c->tprm.mur[j] : 0.0;
    sp.mui[j] = on ? c->tprm.mui[j] : 0.0;
  }
  sp.theta_cap = c->tprm.theta[17];
  sp.S = s.S;
  sp.L = s.L;
  sp.UPW = s.UPW;
  sp.RB = s.RB;
  sp.terms = c->d_terms;
  // the best (J, seed) for qoc_allgather_best_dev, found by the launch's last workgroup
  if (!c->d_best) {  // no communicator yet: this context alone (the epilogue's own layout)
    HIPCHK(c, hipMalloc((void**)&c->d_best, 6 * sizeof(double)));
    c->world = 1;
    c->rank = 0;
  }
  if (!c->d_done) {
    HIPCHK(c, hipMalloc((void**)&c->d_done, sizeof(unsigned int)));
    HIPCHK(c, hipMemsetAsync(c->d_done, 0, sizeof(unsigned int), c->stream));
  }
  sp.done = c->d_done;
  sp.best = c->d_best + 2 + 2 * c->rank;
  sp.seed_offset = c->seed_offset;
  // one rank: the pick after the (identity) exchange is done here, when a buffer is registered
  const bool direct = c->world == 1 && c->best_out;
  sp.best_res = direct ? c->d_best + 2 + 2 * c->world : nullptr;
  sp.best_out = direct ? c->best_out : nullptr;
  c->best_direct = direct;
  return QOC_OK;
}

template <int MODE>
static hipError_t blkseg_launch(qoc_ctx* c, int order, const BlksegShape& s, const BlksegParams& sp) {
  const TChainArgs g = tchain_args(c);
  const BlkArgs bk = blk_args(c);
  return blkseg_dispatch(c->blk_nb, MODE == BLKSEG_FWD ? 1 : order, [&](auto NB_, auto ORD_) {
    constexpr int NB = decltype(NB_)::value, ORD = decltype(ORD_)::value;
    // the forward half has no gradient: one instantiation (ORD 1) serves every order
    if constexpr (MODE == BLKSEG_FWD && ORD != 1) {
      return hipErrorInvalidValue;
    } else {
      auto kern = k_blkseg_eval<NB, ORD, 8, MODE>;
      const hipError_t q = blk_lds_attr(kern, s.lds);
      if (q != hipSuccess) return q;
      hipLaunchKernelGGL(kern, dim3(c->B), dim3(64 * s.W), s.lds, c->stream, g, bk, sp);
      return hipGetLastError();
    }
  });
}

int blkseg_eval(qoc_ctx* c, int order, const double* d_u, double* d_J, double* d_dJdu) {
  const BlksegShape s = blkseg_shape(c);
  int r = ensure_lazy_bufs(c);
  if (r) return r;
  BlksegParams sp;
  if ((r = blkseg_params(c, s, sp))) return r;
  sp.u = d_u;
  sp.u_copy = d_u != c->d_u ? c->d_u : nullptr;
  sp.u_copy2 = c->d_u_lam;  // the co-states' rebuild (blku_costates) reads this copy and d_coef_lam
  sp.J2 = d_J && d_J != c->d_J ? d_J : nullptr;
  sp.coef2 = c->d_coef_lam;
  sp.dJdu = d_dJdu;
  const int mk = mark_begin(c, 2);
  const hipError_t e = blkseg_launch<BLKSEG_FUSED>(c, order, s, sp);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blkseg_eval launch: %s", hipGetErrorString(e));
  c->fwd_captured = false;
  c->L_is_mu = false;
  c->X_lazy = true;
  c->L_lazy = true;
  c->best_ready = true;
  c->last_eval_mode = 6;
  return QOC_OK;
}

// propagate on the segmented eval (the reference's f, examples/ipopt_callbacks_exp.jl:11-19): J, the λ_N coefficients
// and G at every segment's end, x_k rebuilt on demand.  Applies where the fused eval does (any order: the forward half
// has none) unless QOC_BLKSEG_SPLIT=0.
bool blkseg_split_ok(const qoc_ctx* c) {
  const char* env = getenv("QOC_BLKSEG_SPLIT");
  if (env && !std::strcmp(env, "0")) return false;
  return blkseg_ok(c, 3);
}

int blkseg_forward(qoc_ctx* c, const double* d_u, double* d_J) {
  const BlksegShape s = blkseg_shape(c);
  int r = ensure_lazy_bufs(c);
  if (r) return r;
  const size_t gbytes = (size_t)c->B * s.S * c->nblk * c->blk_nb * c->blk_nb * sizeof(double2);
  if (c->gseg_bytes < gbytes) {  // a new block layout (qoc_set_generators) may need more
    if (c->d_gseg) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipFree(c->d_gseg));
      c->d_gseg = nullptr;
      c->dev_bytes -= c->gseg_bytes;
      c->gseg_bytes = 0;
    }
    HIPCHK(c, hipMalloc((void**)&c->d_gseg, gbytes));
    c->gseg_bytes = gbytes;
    c->dev_bytes += gbytes;
  }
  BlksegParams sp;
  if ((r = blkseg_params(c, s, sp))) return r;
  sp.u = d_u;
  sp.u_copy = d_u != c->d_u ? c->d_u : nullptr;  // the backward half and the stale check read d_u
  sp.J2 = d_J && d_J != c->d_J ? d_J : nullptr;
  sp.gseg = c->d_gseg;  // (the co-states' rebuild source stays the last grape_sensitivity's: the backward writes it)
  const int mk = mark_begin(c, 1);
  const hipError_t e = blkseg_launch<BLKSEG_FWD>(c, 1, s, sp);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blkseg_eval (forward) launch: %s", hipGetErrorString(e));
  c->fwd_captured = false;
  c->X_lazy = true;
  c->best_ready = true;
  c->fwd_kind = 1;
  c->props_since_reset++;
  return QOC_OK;
}

// grape_sensitivity after blkseg_forward (the reference's f_grad, :21-31): phase 3 from the stored G; the co-states are
// rebuilt on demand from the forward's copies of u and the λ_N coefficients
int blkseg_backward(qoc_ctx* c, int order, double* d_dJdu, const int* stale) {
  const BlksegShape s = blkseg_shape(c);
  BlksegParams sp;
  int r = blkseg_params(c, s, sp);
  if (r) return r;
  if ((r = ensure_lazy_bufs(c))) return r;
  sp.u = c->d_u;
  sp.u_copy2 = c->d_u_lam;  // λ_k rebuilt on demand from this u and the forward's λ_N coefficients
  sp.coef2 = c->d_coef_lam;
  sp.dJdu = d_dJdu;
  sp.gseg = c->d_gseg;
  sp.stale = stale;
  const int mk = mark_begin(c, 2);
  const hipError_t e = blkseg_launch<BLKSEG_BWD>(c, order, s, sp);
  mark_end(c, mk);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blkseg_eval (backward) launch: %s", hipGetErrorString(e));
  c->L_is_mu = false;
  c->L_lazy = true;
  c->last_eval_mode = 6;
  return QOC_OK;
}

// x_k of the last segmented eval: the block forward chain on the u it left in d_u, J and the coefficients into
// scratch (the eval's own values stay as they were)
int blku_states(qoc_ctx* c) {
  if (!c->X_lazy) return QOC_OK;
  if (!c->d_J_scr) {
    HIPCHK(c, hipMalloc((void**)&c->d_J_scr, (size_t)c->B * sizeof(double)));
    HIPCHK(c, hipMalloc((void**)&c->d_coef_scr, (size_t)c->B * 2 * c->m_user * sizeof(cx<double>)));
    c->dev_bytes += (size_t)c->B * (sizeof(double) + 2 * c->m_user * sizeof(cx<double>));
  }
  TChainArgs g = tchain_args(c);
  g.J = c->d_J_scr;
  g.coef = c->d_coef_scr;
  g.pmask = nullptr;
  const BlkuShape s = blku_shape(c, false);
  BlkuParams bp = blku_params(c, s);
  int r = blku_records(c, bp, false);
  if (r) return r;
  const hipError_t e = blku_launch_fwd_g(c, g, s, bp);
  if (e != hipSuccess) return fail(c, QOC_ERR_HIP, "k_blku_fwd launch (states): %s", hipGetErrorString(e));
  c->X_lazy = false;
  return QOC_OK;
}

int blk_materialize(qoc_ctx* c) {
  int r = QOC_OK;
  if (c->X_lazy) r = blku_states(c);
  if (r == QOC_OK && c->L_lazy) r = blku_costates(c);
  return r;
}

}  // namespace qoc_host
