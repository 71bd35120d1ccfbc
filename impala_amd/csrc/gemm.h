// Two MFMA GEMM skeletons cover every contraction of the learner step.
//
//  gemm_rc  : D[r][c] = sum_k A[r][k] * B(c, k)      (forward convs, FC, heads, all dgrads)
//             Both operands are k-contiguous, so every lane loads its fragment straight from
//             HBM/L2 with one 16-byte load (no LDS round trip); rows = output channels,
//             cols = pixels/frames, so each lane ends up with 4 consecutive channels of one
//             pixel -> one vector store into the channels-last activation.
//  gemm_wg  : D[r][c] = sum_m X(m, r) * Y(m, c)      (all weight gradients)
//             Reduction over pixels m; operands are m-strided in HBM, so a 32-deep m-chunk of
//             both is staged through LDS transposed ([r][m], [c][m]) and fragments are read
//             k-contiguous from LDS.  The m range is split over blockIdx.z; each split writes
//             an fp32 partial slab that reduce_grads() sums in a fixed order (deterministic).
#pragma once
#include "common.h"

template <typename T, int TR, int TC, class Op>
__global__ __launch_bounds__(256) void gemm_rc(const Op op) {
  using F = Frag<T>;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r0 = blockIdx.y * (16 * TR);
  const int cw = (blockIdx.x * 4 + wave) * (16 * TC);
  const int kl = F::KPL * (lane >> 4);
  typename Op::ColCtx cc[TC];
#pragma unroll
  for (int j = 0; j < TC; ++j) cc[j] = op.col_ctx(min(cw + 16 * j + (lane & 15), op.C - 1));
  const T* arow[TR];
#pragma unroll
  for (int i = 0; i < TR; ++i) arow[i] = op.a_row(r0 + 16 * i + (lane & 15), min(cw, op.C - 1));
  f32x4 acc[TR][TC];
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int j = 0; j < TC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int k = 0; k < Op::K; k += F::KSTEP) {
    typename F::vec a[TR], b[TC];
#pragma unroll
    for (int i = 0; i < TR; ++i) a[i] = F::load(arow[i] + k + kl);
#pragma unroll
    for (int j = 0; j < TC; ++j) b[j] = op.load_b(cc[j], k + kl);
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int j = 0; j < TC; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
  }
#pragma unroll
  for (int j = 0; j < TC; ++j) {
    const int c = cw + 16 * j + (lane & 15);
    if (c >= op.C) continue;
#pragma unroll
    for (int i = 0; i < TR; ++i) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      op.store(r0 + 16 * i + 4 * (lane >> 4), c, v);
    }
  }
}

// LDS fragment read along the k (= m) dimension of a row-major [m][col] tile:
//  bf16: two ds_read_b64_tr_b16 (hardware transpose, 4 rows x 16 cols per 16-lane group):
//        lane l gets S[k0 + 8*(l>>4) + j][c0 + (l&15)], j = 0..7.
//  f32 : four ds_read_b32 for the lane-permuted k of Frag<float>: S[k0 + 4*(l>>4) + j][...].
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4;

DEV Frag<__bf16>::vec lds_frag_k(const __bf16* tile, int ld, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const __bf16* a0 = tile + (8 * g + q) * ld + 4 * pp;
  const bf16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  const bf16x4_t y = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0 + 4 * ld));
  Frag<__bf16>::vec v;
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
  return v;
}
DEV Frag<float>::vec lds_frag_k(const float* tile, int ld, int lane) {
  const float* a0 = tile + 4 * (lane >> 4) * ld + (lane & 15);
  return f32x4{a0[0], a0[ld], a0[2 * ld], a0[3 * ld]};
}
// The same fragment from a tile whose rows are stored bit-2 / bit-3 swapped (wg_row): the
// 32 lanes of one transposing read then cover physical rows 0..7 (logical 0..3 and 8..11),
// and with a row pitch of 16 k + 16 elements, k even (row step = 8 mod 16 dwords), their
// 8-dword pieces tile the 64 banks (tools/ldsbank.py: 2.0x -> 1.0x).  A plain pitch cannot:
// rows r and r + 8 of the read are 8 pitches apart, which is 0 or 32 dwords mod 64 and
// either lands on the same banks or breaks the 8-dword alignment of the other rows.
DEV int wg_row(int r) { return (r & ~12) | ((r >> 2) & 1) << 3 | ((r >> 3) & 1) << 2; }
DEV Frag<__bf16>::vec lds_frag_k_sw(const __bf16* tile, int ld, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const __bf16* a0 = tile + (q + 4 * (g & 1) + 16 * (g >> 1)) * ld + 4 * pp;
  const bf16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
  const bf16x4_t y = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0 + 8 * ld));
  Frag<__bf16>::vec v;
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
  v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
  return v;
}
DEV Frag<float>::vec lds_frag_k_sw(const float* tile, int ld, int lane) { return lds_frag_k(tile, ld, lane); }

// epilogue operand types of a gemm_tile op: per-tile Epi for store(), or per-workgroup
// EpiConst for a TILE_EPI tile_epilogue()
template <class Op, bool TE = Op::TILE_EPI> struct EpiTypes {
  typedef typename Op::Epi Epi;
  struct EpiConst {};
};
template <class Op> struct EpiTypes<Op, true> {
  struct Epi {};
  typedef typename Op::EpiConst EpiConst;
};

// LDS-staged, persistent tile GEMM for the same operand definitions as gemm_rc:
//   D[r][c] = sum_k A[r][k] * B(c, k),  WG tile BR x BC, K chunk BK.
// A persistent grid walks the (row-tile, col-tile) list; every K chunk of A (weights) and B
// (im2col / activation gather, 16-byte runs along k) is loaded into registers one chunk
// ahead -- across tile boundaries too, so a workgroup never waits on a cold prologue --
// stored k-contiguous into one of two LDS buffers with 16-byte writes (rows padded by 16 B),
// and every wave reads its fragments with ds_read_b128: operand reuse across the WG's waves
// comes from LDS instead of L1.  WR x WC waves, each owning (BR/WR) x (BC/WC) of the tile.
// Op::A_KMAJOR: A is stored transposed (a_kptr(k, r, c0) -> 16-byte run along r; e.g. the
// forward weight consumed by a dgrad); its chunk is staged [k][r] and the A fragments are
// read with the LDS transpose read, so no transposed weight copy is kept in HBM.
// Requires K % BK == 0, R % BR == 0 and no A dependence on columns inside one BC tile.
// The body runs on NT = 64 * WR * WC threads as virtual workgroup `vbid` of `vgrid`, with the
// LDS passed in (gemm_tile_smem elements), so a launch can host it beside another body.
// bf16 rows are padded by 16 elements: the k-contiguous ds_read_b128 fragment reads are then
// conflict-free (row step 8 mod 64 dwords; + 8 is 2.0x by tools/ldsbank.py), and the k-major
// A tile also stores its rows bit-2/3 swapped for the transposing read (wg_row).
template <typename T> DEV int wg_prow(int r) { if constexpr (sizeof(T) == 2) return wg_row(r); else return r; }
// fp32 k-contiguous rows (LD = BK + 8 floats: the row step is 2 16-byte slots mod the 256-byte
// bank row, so each of ds_read_b128's 16-lane groups -- lanes {0-3, 12-15, 20-27} etc., rows
// lane & 15 at k offset 4 (lane >> 4) -- reads 16 distinct slots; at + 4 floats (1 slot per
// row) rows r, g and r - 1, g + 1 shared a slot: 33 % of the FC forward's LDS cycles were
// conflicts, profiles/r04pmc).  The k-major A tile keeps + 4.
constexpr int F32_ROW_PAD = 8;
template <typename T> constexpr int tile_pad() { return sizeof(T) == 2 ? 16 : F32_ROW_PAD; }
template <typename T> constexpr int tile_pad_ak() { return sizeof(T) == 2 ? 16 : 4; }
template <typename T, int BR, int BC, int BK, int WR, int WC, class Op, int NP = 1>
constexpr int gemm_tile_smem() {
  constexpr int LD = BK + tile_pad<T>();
  constexpr int ASZ = Op::A_KMAJOR ? BK * (BR + tile_pad_ak<T>()) : BR * LD;
  return 2 * NP * (ASZ + BC * LD);
}
// Split-plane products (NP = 3, bf16): an fp32 operand x is held as three bf16 planes
// x = hi + mid + lo (split3, exact), plane p of every operand at a fixed element stride from
// plane 0 (Op::a_ps / b_ps, x_ps / y_ps).  a * b is then the sum of the plane products with
// (p, q) pairs in the order below, smallest terms first; each plane product is exact in
// fp32 (8 x 8 significant bits), the MFMA accumulates them in fp32.  kSplitPairs[0..kSplitN)
// lists (p, q).  9 terms: every product (a * b exact before the fp32 accumulation).
// Measured for the fp32 FC forward (tools/probe/fc_split.hip, profiles/r06z): 13.6-19.8 us
// against 12.3 for the f32 MFMA, and 2.4x its rel-L2 error against fp64 (the 9 terms' extra
// fp32 roundings) -- the three planes triple the staged bytes.  Not used by the library.
constexpr int kSplitN = 9;
constexpr int kSplitPairs[9][2] = {{2, 2}, {2, 1}, {1, 2}, {2, 0}, {1, 1}, {0, 2}, {1, 0}, {0, 1}, {0, 0}};
// PF: K chunks held in registers ahead of the one being computed (1: the next chunk; 2: the
// next two, for a K loop whose chunks are too short to cover the L2 latency of one fetch).
// KACC: accumulator chains per output fragment over alternating k-steps, their elements
// interleaved (Frag::mma_e) so consecutive MFMAs never wait on each other's result (a lone
// 16x16x4 fp32 chain issues every 40 cycles instead of 32); summed in chain order at the end.
// KW (KACC == 1): the NW waves split each chunk's k-steps instead of the tile -- wave w
// computes every fragment of the tile over k-steps w, w + NW, ... -- so a wave runs
// (BR/16)*(BC/16) independent accumulator chains and reads each A / B fragment once for all of
// them; the NW partial tiles are summed in wave order through LDS at the end of the tile,
// and fragment f's epilogue runs on wave f % NW.  Any BR, BC multiple of 16 (e.g. 32 x 48:
// 216 tiles of the FC forward at N = 1280, one per CU, instead of 320 32 x 32 tiles).
// NP = 3: split-plane operands (above; plain k loop only: KACC 1, no KW, no TILE_EPI).
template <typename T, int BR, int BC, int BK, int WR, int WC, class Op, int PF = 1, int KACC = 1,
          bool KW = false, int NP = 1>
DEV void gemm_tile_body(const Op& op, int n_rtiles, int vbid, int vgrid, T* __restrict__ smem) {
  constexpr int NT = 64 * WR * WC;
  constexpr bool AK = Op::A_KMAJOR;
  using F = Frag<T>;
  typedef typename F::vec V;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int KV = BK / VEC;            // 16-byte vectors per tile row per chunk
  constexpr int LD = BK + tile_pad<T>();  // padded row (elements)
  // (KW: the per-wave split is unused, but the arrays sized by it must not be empty)
  constexpr int TRW = BR / 16 / WR > 0 ? BR / 16 / WR : 1, TCW = BC / 16 / WC > 0 ? BC / 16 / WC : 1;
  constexpr int NA = BR * KV / NT, NB = BC * KV / NT;
  constexpr int RV = BR / VEC;            // (A_KMAJOR) 16-byte vectors per k row
  constexpr int LDA = AK ? BR + tile_pad_ak<T>() : LD;  // A tile row length (elements)
  constexpr int ASZ = AK ? BK * LDA : BR * LD;
  constexpr int NK = Op::K / BK;
  static_assert((WR * WC == 4 || (WR * WC == 8 && !Op::TILE_EPI)) && (KW || (BR / 16 / WR >= 1 && BC / 16 / WC >= 1)),
                "tile");
  static_assert(BR * KV % NT == 0 && BC * KV % NT == 0, "staging");
  static_assert(Op::K % BK == 0 && BK % F::KSTEP == 0, "K chunking");
  static_assert((PF == 1 || PF == 2) && (KACC == 1 || KACC == 2) && (BK / F::KSTEP) % KACC == 0, "PF / KACC");
  static_assert(PF == 1 || NK % 2 == 0, "two chunks ahead: an even chunk count per tile");
  constexpr int FR = BR / 16, FC = BC / 16;  // KW: fragments of the tile, all on every wave
  constexpr int NW = WR * WC;                   // waves (KW: each takes every NW-th k-step)
  constexpr int NOWN = (FR * FC + NW - 1) / NW;  // KW: fragments whose epilogue a wave runs
  static_assert(!KW || (KACC == 1 && !Op::TILE_EPI && BR % 16 == 0 && BC % 16 == 0 &&
                        (BK / F::KSTEP) % NW == 0), "KW: whole k-steps per wave per chunk");
  static_assert(NP == 1 || (NP == 3 && sizeof(T) == 2 && KACC == 1 && !KW && !Op::TILE_EPI), "split planes");
  constexpr int PSZ = ASZ + BC * LD;  // one plane of a buffer (A then B)
  constexpr int SMEM = 2 * NP * PSZ;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WC, wc = wave % WC;
  // staging element e = tid + i*256 of a chunk -> (tile row e / KV, 16-byte vector e % KV)
  auto srow = [&](int i) { return (tid + i * NT) / KV; };
  auto skv = [&](int i) { return (tid + i * NT) % KV; };
  const int n_tiles = n_rtiles * ((op.C + BC - 1) / BC);
  const int ft = xcd_swizzle(vbid, vgrid);  // first tile of this workgroup
  if (ft >= n_tiles) return;
  // per-thread staging contexts of the fetch tile
  const T* arow[NA];
  typename Op::ColCtx bctx[NB];
  int fr0 = 0, fc0 = 0, fcw = 0;
  auto set_ctx = [&](int t) {
    fr0 = (t % n_rtiles) * BR;
    fc0 = (t / n_rtiles) * BC;
    fcw = min(fc0, op.C - 1);
    if constexpr (!AK) {
#pragma unroll
      for (int i = 0; i < NA; ++i) arow[i] = op.a_row(fr0 + srow(i), fcw);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) bctx[i] = op.col_ctx(min(fc0 + srow(i), op.C - 1));
  };
  V ra[PF][NP][NA], rb[PF][NP][NB];
  auto fetch = [&](int k0, int sl) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if constexpr (AK) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int e = tid + i * NT, kr = e / RV, rv = e % RV;
          const T* ap = op.a_kptr(k0 + kr, fr0 + rv * VEC, fcw);
          if constexpr (NP > 1) ap += p * op.a_ps;
          ra[sl][p][i] = F::load(ap);
        }
      } else {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const T* ap = arow[i] + k0 + skv(i) * VEC;
          if constexpr (NP > 1) ap += p * op.a_ps;
          ra[sl][p][i] = F::load(ap);
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        if constexpr (NP > 1)
          rb[sl][p][i] = op.load_b(bctx[i], k0 + skv(i) * VEC, p);
        else
          rb[sl][p][i] = op.load_b(bctx[i], k0 + skv(i) * VEC);
      }
    }
  };
  auto stash = [&](int buf, int sl) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      T* As = smem + (buf * NP + p) * PSZ;
      T* Bs = As + ASZ;
      if constexpr (AK) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int e = tid + i * NT, kr = e / RV, rv = e % RV;
          *reinterpret_cast<V*>(As + wg_prow<T>(kr) * LDA + rv * VEC) = ra[sl][p][i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < NA; ++i) *reinterpret_cast<V*>(As + srow(i) * LD + skv(i) * VEC) = ra[sl][p][i];
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) *reinterpret_cast<V*>(Bs + srow(i) * LD + skv(i) * VEC) = rb[sl][p][i];
    }
  };
  const int kl = F::KPL * (lane >> 4);
  set_ctx(ft);
  fetch(0, 0);
  if constexpr (PF == 2) fetch(BK, 1);
  [[maybe_unused]] typename EpiTypes<Op>::EpiConst econst{};
  if constexpr (Op::TILE_EPI) econst = op.epi_const(tid);
  for (int t = ft; t < n_tiles; t += vgrid) {
    const int cr0 = fr0, cc0 = fc0;  // coordinates of tile t (the fetch cursor is on it)
    // the epilogue's global reads, issued now so they land under the K loop
    [[maybe_unused]] typename EpiTypes<Op>::Epi ep[TRW][TCW];
    [[maybe_unused]] typename EpiTypes<Op>::Epi epw[KW ? NOWN : 1];
    if constexpr (KW) {
#pragma unroll
      for (int u = 0; u < NOWN; ++u) {
        const int f = min(wave + NW * u, FR * FC - 1), i = f / FC, j = f % FC;
        epw[u] = op.epi(cr0 + i * 16 + 4 * (lane >> 4), min(cc0 + j * 16 + (lane & 15), op.C - 1));
      }
    } else if constexpr (!Op::TILE_EPI) {
#pragma unroll
      for (int j = 0; j < TCW; ++j)
#pragma unroll
        for (int i = 0; i < TRW; ++i)
          ep[i][j] = op.epi(cr0 + (wr * TRW + i) * 16 + 4 * (lane >> 4),
                            min(cc0 + (wc * TCW + j) * 16 + (lane & 15), op.C - 1));
    }
    f32x4 acc[TRW][TCW], acc2[KACC > 1 ? TRW : 1][KACC > 1 ? TCW : 1];
    f32x4 accw[KW ? FR : 1][KW ? FC : 1];
    if constexpr (KW) {
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) accw[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < TRW; ++i)
#pragma unroll
      for (int j = 0; j < TCW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (KACC > 1) {
#pragma unroll
      for (int i = 0; i < TRW; ++i)
#pragma unroll
        for (int j = 0; j < TCW; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kc = 0; kc < NK; ++kc) {
      const int buf = kc & 1;  // NK is even or the next tile restarts at buffer 0 after a sync
      // PF == 2: chunk kc sits in register slot kc & 1 (NK is even: a tile starts at slot 0)
      const int sl = PF == 2 ? (kc & 1) : 0;
      stash(buf, sl);
      __syncthreads();
      if (kc + PF < NK) {
        fetch((kc + PF) * BK, sl);
      } else if (t + vgrid < n_tiles) {
        // prefetch the next tile's first chunk(s) under this compute
        if (kc + PF == NK) set_ctx(t + vgrid);
        fetch((kc + PF - NK) * BK, sl);
      }
      const T* As = smem + buf * NP * PSZ;
      const T* Bs = As + ASZ;
      auto frags = [&](int kk, V (&a)[TRW], V (&b)[TCW]) {
#pragma unroll
        for (int i = 0; i < TRW; ++i) {
          if constexpr (AK)
            a[i] = lds_frag_k_sw(As + kk * LDA + (wr * TRW + i) * 16, LDA, lane);
          else
            a[i] = *reinterpret_cast<const V*>(As + ((wr * TRW + i) * 16 + (lane & 15)) * LD + kk + kl);
        }
#pragma unroll
        for (int j = 0; j < TCW; ++j)
          b[j] = *reinterpret_cast<const V*>(Bs + ((wc * TCW + j) * 16 + (lane & 15)) * LD + kk + kl);
      };
      if constexpr (KW) {
#pragma unroll
        for (int kk = wave * F::KSTEP; kk < BK; kk += NW * F::KSTEP) {
          V a[FR], b[FC];
#pragma unroll
          for (int i = 0; i < FR; ++i)
            a[i] = *reinterpret_cast<const V*>(As + (i * 16 + (lane & 15)) * LD + kk + kl);
#pragma unroll
          for (int j = 0; j < FC; ++j)
            b[j] = *reinterpret_cast<const V*>(Bs + (j * 16 + (lane & 15)) * LD + kk + kl);
#pragma unroll
          for (int e = 0; e < F::NE; ++e)
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
              for (int j = 0; j < FC; ++j) accw[i][j] = F::mma_e(e, a[i], b[j], accw[i][j]);
        }
      } else if constexpr (NP > 1) {
#pragma unroll
        for (int kk = 0; kk < BK; kk += F::KSTEP) {
          V a[NP][TRW], b[NP][TCW];
#pragma unroll
          for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int i = 0; i < TRW; ++i) {
              const T* Ap = As + p * PSZ;
              if constexpr (AK)
                a[p][i] = lds_frag_k_sw(Ap + kk * LDA + (wr * TRW + i) * 16, LDA, lane);
              else
                a[p][i] = *reinterpret_cast<const V*>(Ap + ((wr * TRW + i) * 16 + (lane & 15)) * LD + kk + kl);
            }
#pragma unroll
            for (int j = 0; j < TCW; ++j)
              b[p][j] = *reinterpret_cast<const V*>(Bs + p * PSZ + ((wc * TCW + j) * 16 + (lane & 15)) * LD + kk + kl);
          }
#pragma unroll
          for (int q = 0; q < kSplitN; ++q)
#pragma unroll
            for (int i = 0; i < TRW; ++i)
#pragma unroll
              for (int j = 0; j < TCW; ++j)
                acc[i][j] = F::mma(a[kSplitPairs[q][0]][i], b[kSplitPairs[q][1]][j], acc[i][j]);
        }
      } else if constexpr (KACC == 1) {
#pragma unroll
        for (int kk = 0; kk < BK; kk += F::KSTEP) {
          V a[TRW], b[TCW];
          frags(kk, a, b);
#pragma unroll
          for (int i = 0; i < TRW; ++i)
#pragma unroll
            for (int j = 0; j < TCW; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2 * F::KSTEP) {
          V a[TRW], b[TCW], a2[TRW], b2[TCW];
          frags(kk, a, b);
          frags(kk + F::KSTEP, a2, b2);
#pragma unroll
          for (int e = 0; e < F::NE; ++e)
#pragma unroll
            for (int i = 0; i < TRW; ++i)
#pragma unroll
              for (int j = 0; j < TCW; ++j) {
                acc[i][j] = F::mma_e(e, a[i], b[j], acc[i][j]);
                acc2[i][j] = F::mma_e(e, a2[i], b2[j], acc2[i][j]);
              }
        }
      }
    }
    if constexpr (KACC > 1) {
#pragma unroll
      for (int i = 0; i < TRW; ++i)
#pragma unroll
        for (int j = 0; j < TCW; ++j) acc[i][j] += acc2[i][j];
    }
    if constexpr (KW) {
      // the waves' partial tiles through LDS: [wave][fragment][lane] f32x4, summed in wave order;
      // fragment f's epilogue on wave f % NW
      static_assert((size_t)NW * FR * FC * 64 * sizeof(f32x4) <= SMEM * sizeof(T), "KW partials");
      f32x4* part = reinterpret_cast<f32x4*>(smem);
      __syncthreads();  // every wave is done with the staging buffers
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FC; ++j) part[((wave * FR + i) * FC + j) * 64 + lane] = accw[i][j];
      __syncthreads();
#pragma unroll
      for (int u = 0; u < NOWN; ++u) {
        const int f = wave + NW * u;
        if (f < FR * FC) {
          f32x4 sum = part[f * 64 + lane];
#pragma unroll
          for (int w = 1; w < NW; ++w) sum += part[(w * FR * FC + f) * 64 + lane];
          const int i = f / FC, j = f % FC, c = cc0 + j * 16 + (lane & 15);
          if (c < op.C) {
            float v[4] = {sum[0], sum[1], sum[2], sum[3]};
            op.store(cr0 + i * 16 + 4 * (lane >> 4), c, v, epw[u]);
          }
        }
      }
      __syncthreads();  // the next tile's stash reuses the LDS
    }
    if constexpr (Op::TILE_EPI) {
      // workgroup epilogue: fp32 tile [BC][BR+4] in (reused) LDS, then op.tile_epilogue
      static_assert((size_t)BC * (BR + 4) * sizeof(float) <= SMEM * sizeof(T), "epilogue tile");
      __syncthreads();  // all waves are done reading the staging buffers
      float* et = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int j = 0; j < TCW; ++j)
#pragma unroll
        for (int i = 0; i < TRW; ++i) {
          const int cl = (wc * TCW + j) * 16 + (lane & 15);
          const int rl0 = (wr * TRW + i) * 16 + 4 * (lane >> 4);
          *reinterpret_cast<f32x4*>(et + cl * (BR + 4) + rl0) = acc[i][j];
        }
      __syncthreads();
      op.tile_epilogue(et, BR + 4, cr0, cc0, tid, econst);
      __syncthreads();  // the next tile's stash reuses the LDS
    } else if constexpr (!KW) {
      if constexpr (NK % 2 == 1) __syncthreads();  // next tile reuses buffer 0 first
#pragma unroll
      for (int j = 0; j < TCW; ++j) {
        const int c = cc0 + (wc * TCW + j) * 16 + (lane & 15);
        if (c < op.C) {
#pragma unroll
          for (int i = 0; i < TRW; ++i) {
            float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            op.store(cr0 + (wr * TRW + i) * 16 + 4 * (lane >> 4), c, v, ep[i][j]);
          }
        }
      }
    }
  }
}

template <typename T, int BR, int BC, int BK, int WR, int WC, class Op, int PF = 1, int KACC = 1,
          bool KW = false, int NP = 1>
__global__ __launch_bounds__(64 * WR * WC) void gemm_tile(const Op op, int n_rtiles) {
  __shared__ __attribute__((aligned(16))) T smem[gemm_tile_smem<T, BR, BC, BK, WR, WC, Op, NP>()];
  gemm_tile_body<T, BR, BC, BK, WR, WC, Op, PF, KACC, KW, NP>(op, n_rtiles, (int)blockIdx.x, (int)gridDim.x, smem);
}

// Weight-gradient GEMM  D[r][c] = sum_m X[m][r] * Y(m, c)  over the m range of split
// blockIdx.z.  X is a row-major [M][x_ld] matrix (the channels-last output gradient); Y is a
// gather (im2col of the layer input) given as element offsets y_roff(m) + y_coff(c) of 16-byte
// runs along c.  Each BM-row chunk of both is staged row-major into LDS with 16-byte stores and
// the MFMA fragments are read along m with the hardware transpose read (bf16).  A workgroup
// holds G independent 4-wave groups on interleaved chunks, and every group keeps PD chunks in
// flight in a register ring (the chunk it multiplies was issued PD chunks earlier): the MFMA
// work per chunk is a few hundred cycles against a ~2 us loaded memory round trip, so the
// kernel is bound by how many chunk loads are in flight per CU.  All loads are buffer loads
// issued unconditionally: rows past the split's end and chunks past the group's last one carry
// an out-of-range offset and read as zero without touching memory (no branch around a load,
// so the compiler's counted vmcnt waits stay exact).  The groups' accumulators are summed in
// a fixed order at the end.  Output: fp32 partial slab [split][R][C] (+ per-split bias sums),
// or, for an Op with DIRECT (one split: the tile is final), the canonical gradient itself plus
// the workgroup's sum of squares in op.sumsq[workgroup].
template <class Op, class = void> struct wg_direct { static constexpr bool value = false; };
template <class Op> struct wg_direct<Op, decltype(void(Op::DIRECT))> {
  static constexpr bool value = Op::DIRECT;
};
// The body runs as virtual workgroup `lin` of a gx x gy x gz grid on 256 * G threads, with the
// LDS passed in (gemm_wg_smem elements).
// bf16 rows are stored bit-2/3 swapped (wg_row) at a pitch of BR / BC + 16 (conflict-free
// transposing fragment reads); fp32 rows in order at + 4.
template <class Op, class = void> struct wg_ycur { static constexpr bool value = false; };
template <class Op> struct wg_ycur<Op, decltype(void(Op::YCUR))> {
  static constexpr bool value = Op::YCUR;
};
template <class Op, bool = wg_ycur<Op>::value> struct WgYCur { struct type { int n, p; }; };
template <class Op> struct WgYCur<Op, true> { typedef typename Op::YCur type; };
template <typename T> constexpr int wg_pad() { return sizeof(T) == 2 ? 16 : 4; }
template <typename T, int BR, int BC, int BM, int G>
constexpr int gemm_wg_smem() {
  return (BM * (BR + wg_pad<T>()) + BM * (BC + wg_pad<T>())) * 2 * G;
}
template <typename T, int BR, int BC, int WR, int WC, int BM, int G, class Op, int PD = 2>
DEV void gemm_wg_body(const Op& op, float* __restrict__ slab, float* __restrict__ slab_bias,
                      int m_per_split, int lin, int gx, int gy, int gz, T* __restrict__ smem) {
  using F = Frag<T>;
  typedef typename F::vec V;  // 16 bytes of T
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int LDX = BR + wg_pad<T>(), LDY = BC + wg_pad<T>();
  constexpr int TRW = BR / 16 / WR, TCW = BC / 16 / WC;
  constexpr int NACC = TRW * TCW * 4;
  constexpr int STAGE = BM * LDX + BM * LDY;  // elements of T per buffer
  constexpr int NXV = BM * (BR / VEC);
  constexpr int NX = (NXV + 255) / 256;
  // Y staging: vector v = t + i*256 of a chunk is row v / (BC/VEC), column vector v % (BC/VEC),
  // so consecutive lanes read one contiguous run of a row (the BC columns of a tile are one
  // contiguous run of the im2col row: 4 taps x 32 channels of conv2, one tap of conv3, an FC
  // row slice).  A wave instruction then touches a few whole 128-B lines instead of one 32-B
  // piece of a line per row: the TA's per-line rate, not bytes, bounded the row-per-lane form
  // (24 B/cycle per CU, profiles/r02c).
  constexpr int YV = BC / VEC, NYV = BM * YV, NY = (NYV + 255) / 256;
  constexpr int OOB = 0x7ffffff0;  // buffer offset past any extent: the load returns zero
  static_assert(256 % BM == 0, "Y staging");
  static_assert(WR * WC == 4, "4 waves per group");
  static_assert(TRW >= 1 && TCW >= 1 && BR % 16 == 0 && BC % 16 == 0, "tile");
  static_assert(BM % F::KSTEP == 0, "chunk");
  static_assert(PD >= 1, "prefetch depth");
  // the LDS is reused for the fixed-order group reduction (G > 1) and the bias / sum-of-squares
  // combines (256 floats)
  static_assert((G == 1 || (size_t)STAGE * 2 * G * sizeof(T) >= (size_t)256 * (NACC + 1) * sizeof(float)) &&
                    (size_t)STAGE * 2 * G * sizeof(T) >= 256 * sizeof(float),
                "LDS reuse for the group reduction");
  static_assert(STAGE * 2 * G == gemm_wg_smem<T, BR, BC, BM, G>(), "LDS size");
  const int grp = threadIdx.x >> 8, tid = threadIdx.x & 255, lane = tid & 63, wave = tid >> 6;
  // work item (column tile fastest) from the XCD-swizzled dispatch id
  const int nwg = gx * gy * gz;
  const int wid = xcd_swizzle(lin, nwg);
  const int bx = wid % gx, by = (wid / gx) % gy, split = wid / (gx * gy);
  const int c0 = bx * BC, r0 = by * BR;
  const int m_beg = split * m_per_split;
  const int m_end = min(op.M, m_beg + m_per_split);
  const int wr = wave / WC, wc = wave % WC;
  constexpr bool DIRECT = wg_direct<Op>::value;
  const bool do_bias = (DIRECT || slab_bias != nullptr) && bx == 0;
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(op.x), 0, op.M * op.x_ld * (int)sizeof(T), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(op.ybase()), 0, op.y_bytes(), 0x00020000);
  f32x4 acc[TRW][TCW];
#pragma unroll
  for (int i = 0; i < TRW; ++i)
#pragma unroll
    for (int j = 0; j < TCW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bias_acc = 0.f;
  // per-thread constant parts of the staging addresses (bytes)
  int xcol[NX], ycol[NY];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int e = min(tid + i * 256, NXV - 1);
    xcol[i] = (r0 + (e % (BR / VEC)) * VEC) * (int)sizeof(T);
  }
#pragma unroll
  for (int i = 0; i < NY; ++i) ycol[i] = op.y_coff(c0 + ((tid + i * 256) % YV) * VEC) * (int)sizeof(T);
  V rx[PD][NX], ry[PD][NY];
  // YCUR ops: the Y rows this thread stages, as cursors advanced by one chunk (BM * G rows) per
  // fetch -- fetch(d, it) is called with it = 0, 1, 2, ... in order -- instead of y_roff's
  // divisions per load (which the compiler put behind a branch each: 4 of them per chunk)
  constexpr bool YC = wg_ycur<Op>::value;
  typename WgYCur<Op>::type ycur[YC ? NY : 1];
  int ym[YC ? NY : 1];
  if constexpr (YC) {
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      ym[i] = m_beg + grp * BM + min(tid + i * 256, NYV - 1) / YV;
      ycur[i] = op.ycur(ym[i]);
    }
  }
  // chunk `it` of this group -> ring slot d.  Offsets are computed for a clamped row and
  // replaced by OOB with a select afterwards (unsigned: OOB + a column offset stays out of
  // range), so no load sits behind a branch.
  auto fetch = [&](int d, int it) {
    const int m0 = m_beg + (it * G + grp) * BM;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int m = m0 + (tid + i * 256) / (BR / VEC);
      const uint32_t off = (uint32_t)(min(m, m_end - 1) * op.x_ld * (int)sizeof(T) + xcol[i]);
      rx[d][i] = __builtin_bit_cast(
          V, __builtin_amdgcn_raw_buffer_load_b128(rs_x, (int)(m < m_end ? off : (uint32_t)OOB), 0, 0));
    }
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      uint32_t yr;
      if constexpr (YC) {
        // rows past the split's end read as zero (OOB), whatever the cursor's offset
        const uint32_t o = (uint32_t)(op.ycur_off(ycur[i]) * (int)sizeof(T));
        yr = ym[i] < m_end ? o : (uint32_t)OOB;
        ym[i] += BM * G;
        op.template ycur_adv<BM * G>(ycur[i]);
      } else {
        const int m = m0 + min(tid + i * 256, NYV - 1) / YV;
        yr = m < m_end ? (uint32_t)(op.y_roff(min(m, m_end - 1)) * (int)sizeof(T)) : (uint32_t)OOB;
      }
      ry[d][i] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs_y, (int)(yr + (uint32_t)ycol[i]), 0, 0));
    }
  };
  auto stash = [&](int d, T* Xs) {
    T* Ys = Xs + BM * LDX;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = tid + i * 256, mm = e / (BR / VEC), rr = (e % (BR / VEC)) * VEC;
      if (e < NXV) *reinterpret_cast<V*>(Xs + wg_prow<T>(mm) * LDX + rr) = rx[d][i];
    }
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const int v = tid + i * 256;
      if (v < NYV) *reinterpret_cast<V*>(Ys + wg_prow<T>(v / YV) * LDY + (v % YV) * VEC) = ry[d][i];
    }
  };
  const int n_it = (m_end - m_beg + BM * G - 1) / (BM * G);
  // sched_barrier(0) keeps the ring slots' loads in issue order (the scheduler otherwise
  // interleaves the prologue's fetches, and the first stash then waits for all of them)
#pragma unroll
  for (int d = 0; d < PD; ++d) {
    fetch(d, d);
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int it0 = 0; it0 < n_it; it0 += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const int it = it0 + d;
      // no early exit: the trip count is padded to a multiple of PD and chunks past n_it are
      // all-OOB (zero, no memory traffic, MFMAs skipped).  An exit from the middle of the
      // unrolled ring is funnelled through the loop latch by the CFG structurizer, which merges
      // a rotated ring state into the loop header and forces vmcnt(0) at every stash.
      const int m0 = m_beg + (it * G + grp) * BM;
      const bool active = m0 < m_end;
      T* Xs = smem + (grp * 2 + (it & 1)) * STAGE;
      const T* Ys = Xs + BM * LDX;
      stash(d, Xs);
      __syncthreads();
      fetch(d, it + PD);  // in flight under the next PD - 1 chunks
      __builtin_amdgcn_sched_barrier(0);
      if (active) {
        if (do_bias) {  // (256/BR) row groups x BR channels; summed across groups at the end
          constexpr int RG = 256 / BR;
          const int rch = tid % BR, rg = tid / BR;
          float s0 = 0.f;
#pragma unroll
          for (int mm = rg; mm < BM; mm += RG) s0 += (float)Xs[wg_prow<T>(mm) * LDX + rch];
          bias_acc += s0;
        }
#pragma unroll
        for (int kk = 0; kk < BM; kk += F::KSTEP) {
          V a[TRW], b[TCW];
#pragma unroll
          for (int i = 0; i < TRW; ++i)
            a[i] = lds_frag_k_sw(Xs + kk * LDX + (wr * TRW + i) * 16, LDX, lane);
#pragma unroll
          for (int j = 0; j < TCW; ++j)
            b[j] = lds_frag_k_sw(Ys + kk * LDY + (wc * TCW + j) * 16, LDY, lane);
#pragma unroll
          for (int i = 0; i < TRW; ++i)
#pragma unroll
            for (int j = 0; j < TCW; ++j) acc[i][j] = F::mma(a[i], b[j], acc[i][j]);
        }
      }
    }
  }
  __syncthreads();
  // fixed-order reduction of the G groups' accumulators through (reused) LDS
  if constexpr (G > 1) {
    float* red = reinterpret_cast<float*>(smem);
    for (int g = 1; g < G; ++g) {
      if (grp == g) {
#pragma unroll
        for (int i = 0; i < TRW; ++i)
#pragma unroll
          for (int j = 0; j < TCW; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[((i * TCW + j) * 4 + q) * 256 + tid] = acc[i][j][q];
        red[NACC * 256 + tid] = bias_acc;
      }
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int i = 0; i < TRW; ++i)
#pragma unroll
          for (int j = 0; j < TCW; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[i][j][q] += red[((i * TCW + j) * 4 + q) * 256 + tid];
        bias_acc += red[NACC * 256 + tid];
      }
      __syncthreads();
    }
  }
  float bias_sq = 0.f;  // DIRECT: this thread's final bias element, squared
  if (do_bias) {  // combine the (256/BR) row groups of group 0's bias sums, fixed order
    constexpr int RG = 256 / BR;
    float* redb = reinterpret_cast<float*>(smem);
    if (grp == 0) redb[tid] = bias_acc;
    __syncthreads();
    if (grp == 0 && tid < BR) {
      float bsum = 0.f;
#pragma unroll
      for (int g = 0; g < RG; ++g) bsum += redb[g * BR + tid];
      if constexpr (DIRECT) {
        op.grads[op.bias_canon(r0 + tid)] = bsum;
        bias_sq = bsum * bsum;
      } else {
        slab_bias[(size_t)split * op.R + r0 + tid] = bsum;
      }
    }
  }
  if constexpr (DIRECT) {
    __syncthreads();  // the bias sums above are read from smem before it is reused below
    float sq = 0.f;
    if (grp == 0) {
#pragma unroll
      for (int j = 0; j < TCW; ++j) {
        const int c = c0 + (wc * TCW + j) * 16 + (lane & 15);
#pragma unroll
        for (int i = 0; i < TRW; ++i) {
          const int r = r0 + (wr * TRW + i) * 16 + 4 * (lane >> 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = acc[i][j][q] * op.out_scale;
            if (c < op.C) {
              op.grads[op.canon(r + q, c)] = v;
              sq += v * v;
            }
          }
        }
      }
      sq = wave_sum(sq + bias_sq);
    }
    float* redq = reinterpret_cast<float*>(smem);
    if (grp == 0 && lane == 0) redq[wave] = sq;
    __syncthreads();
    if (threadIdx.x == 0) op.sumsq[lin] = (redq[0] + redq[1]) + (redq[2] + redq[3]);
    return;
  }
  if (grp != 0) return;
  const float sc = op.out_scale;
#pragma unroll
  for (int j = 0; j < TCW; ++j) {
    const int c = c0 + (wc * TCW + j) * 16 + (lane & 15);
    if (c >= op.C) continue;
#pragma unroll
    for (int i = 0; i < TRW; ++i) {
      const int r = r0 + (wr * TRW + i) * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        slab[((size_t)split * op.R + r + q) * op.C + c] = acc[i][j][q] * sc;
    }
  }
}

template <typename T, int BR, int BC, int WR, int WC, int BM, int G, class Op, int PD = 2>
__global__ __launch_bounds__(256 * G) void gemm_wg(const Op op, float* __restrict__ slab,
                                                   float* __restrict__ slab_bias,
                                                   int m_per_split) {
  __shared__ __attribute__((aligned(16))) T smem[gemm_wg_smem<T, BR, BC, BM, G>()];
  gemm_wg_body<T, BR, BC, WR, WC, BM, G, Op, PD>(
      op, slab, slab_bias, m_per_split,
      (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)), (int)gridDim.x,
      (int)gridDim.y, (int)gridDim.z, smem);
}
