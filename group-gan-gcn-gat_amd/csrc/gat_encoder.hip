// The whole group GAT encoder of a scene in one workgroup (GATEncoder,
// reference sgan/models.py:254-294, with GAT :222-237 and
// GraphAttentionLayer :184-220), forward and backward.
//
// Per scene (n <= 64 peds, the workgroup's LDS holds everything):
//   groups      M_ij = (i == j) | (lab_i == lab_j != 0) on the last-observed
//               labels (:263-266); group g(i) = index of i's first member
//   intra GAT   per head h: Wh = X W_h (40 -> 72), masked softmax attention,
//               ELU; heads concatenated; out layer (72 nh -> 16) + ELU +
//               log_softmax over features                      (:269, :231-237)
//   group mean  gin = R intra, R the row-normalised distinct rows of M
//                                                               (:271-280)
//   inter GAT   the same GAT (16 -> 72 -> 16) on the complete graph of the
//               scene's groups                                  (:282-285)
//   un-pool     inter_i = gout[g(i)] / |g(i)|  (R^T with R normalised, :286)
//   out         Linear(32, 24)([intra, inter])                   (:288-289)
//
// One launch replaces the ~14 launches of the per-op path (sgg_xw +
// sgg_gat_fwd per layer, group pooling kernels, concat, Linear).  The
// backward recomputes the forward in LDS (it is ~0.3 MFLOP per 20-ped scene)
// and back-propagates through every layer in the same workgroup; each
// scene's parameter gradients go to its own row of a slab (no atomics) that
// sgg_slab_reduce sums in scene order (deterministic).
//
// Attention: e_ij = LeakyReLU(a[:F].Wh_i + a[F:].Wh_j) (the s_i + t_j
// decomposition of the reference's (N, N, 2F) concatenation), masked to
// -inf outside the graph, softmax over j; one wavefront per attention row
// with lane j (n <= 64), row max / sum by wave shuffles.
#include <string.h>

#include "sgg_common.h"



namespace sgg {

namespace {

// forward 1024 threads (16 waves: attention rows and output elements of a
// 20-ped scene are ~1 per wave / thread, so the dependent chains overlap);
// the same for the backward
constexpr int kFwdThreads = 1024, kBwdThreads = 1024;
#ifndef SGG_GATENC_GRID_CAP
#define SGG_GATENC_GRID_CAP 65536
#endif
constexpr int kGridCap = SGG_GATENC_GRID_CAP;   // workgroups (scenes loop over them); a probe build lowers it
constexpr int FI = 40, FH = 72, FO = 16, FE = 24;   // GATEncoder dims (models.py:242-244)
constexpr int P40 = FI + 1, P72 = FH + 1, P16 = FO + 1;

// LDS image of the weights: W (K x N) rows at pitch N + 1 (odd: a column walk
// across rows, lane = row, is bank-conflict free; a row walk is contiguous)
constexpr int PW72 = FH + 1, PW16 = FO + 1, PWE = 2 * FO + 1;
__host__ __device__ constexpr int weights_floats(int nh) {
  return nh * (FI * PW72 + 2 * FH) + (FH * nh * PW16 + 2 * FO) + nh * (FO * PW72 + 2 * FH) + (FH * nh * PW16 + 2 * FO) +
         FE * PWE + FE;
}

struct LW {
  const float* Wi[kGatEncMaxHeads];
  const float* ai[kGatEncMaxHeads];
  const float* Wio;
  const float* aio;
  const float* Wg[kGatEncMaxHeads];
  const float* ag[kGatEncMaxHeads];
  const float* Wgo;
  const float* ago;
  const float* Woe;
  const float* boe;
};

// The module's weights to LDS in ONE memory round trip.  The host lays the
// 22 segments (per head Wi, ai; Wio, aio; per head Wg, ag; Wgo, ago; Woe,
// boe -- unused heads have length 0) out as 8-float chunks (a segment starts
// on a chunk); thread c copies chunk c: 8 loads in flight, then the stores
// into the LDS image (matrices at pitch N + 1, vectors packed).
constexpr int kSegs = 4 * kGatEncMaxHeads + 6;
constexpr int kChunk = 8;
// the per-batch fields of a forward (the second batch of sgg_gatenc_fwd2)
struct GatEncSet {
  const float* X;
  const float* X2;
  const float* labels;
  const int32_t* scene_off;
  float* y;
  float* saved;
  int ldx, ldx2, kx1, S, ldy;
};

struct StageTab {
  const float* src[kSegs];
  int coff[kSegs];   // first chunk (non-decreasing)
  int len[kSegs];    // floats
  int dst[kSegs];    // LDS image offset
  int rowN[kSegs];   // matrix row length (pitch rowN + 1); 0: vector
  int nchunks;
  int floats;        // LDS image size
};

inline StageTab make_stage_tab(const SggGatEncWeights& w, int nh) {
  StageTab T = {};
  int q = 0, ch = 0;
  auto put = [&](int sl, const float* sp, int K, int N, bool mat, bool live) {
    T.src[sl] = sp;
    T.coff[sl] = ch;
    T.len[sl] = live ? K * N : 0;
    T.dst[sl] = q;
    T.rowN[sl] = mat ? N : 0;
    if (live) {
      ch += (K * N + kChunk - 1) / kChunk;
      q += mat ? K * (N + 1) : K * N;
    }
  };
  for (int h = 0; h < kGatEncMaxHeads; ++h) {
    put(2 * h, w.Wi[h], FI, FH, true, h < nh);
    put(2 * h + 1, w.ai[h], 2 * FH, 1, false, h < nh);
  }
  put(2 * kGatEncMaxHeads, w.Wio, FH * nh, FO, true, true);
  put(2 * kGatEncMaxHeads + 1, w.aio, 2 * FO, 1, false, true);
  for (int h = 0; h < kGatEncMaxHeads; ++h) {
    put(2 * kGatEncMaxHeads + 2 + 2 * h, w.Wg[h], FO, FH, true, h < nh);
    put(2 * kGatEncMaxHeads + 3 + 2 * h, w.ag[h], 2 * FH, 1, false, h < nh);
  }
  put(4 * kGatEncMaxHeads + 2, w.Wgo, FH * nh, FO, true, true);
  put(4 * kGatEncMaxHeads + 3, w.ago, 2 * FO, 1, false, true);
  put(4 * kGatEncMaxHeads + 4, w.Woe, FE, 2 * FO, true, true);
  put(4 * kGatEncMaxHeads + 5, w.boe, FE, 1, false, true);
  T.nchunks = ch;
  T.floats = q;
  return T;
}

__device__ inline void stage_weights(float* base, const StageTab& T, LW& lw) {
  lw.Wi[0] = base + T.dst[0];
  lw.ai[0] = base + T.dst[1];
  lw.Wio = base + T.dst[2 * kGatEncMaxHeads];
  lw.aio = base + T.dst[2 * kGatEncMaxHeads + 1];
  lw.Wg[0] = base + T.dst[2 * kGatEncMaxHeads + 2];
  lw.ag[0] = base + T.dst[2 * kGatEncMaxHeads + 3];
  lw.Wgo = base + T.dst[4 * kGatEncMaxHeads + 2];
  lw.ago = base + T.dst[4 * kGatEncMaxHeads + 3];
  lw.Woe = base + T.dst[4 * kGatEncMaxHeads + 4];
  lw.boe = base + T.dst[4 * kGatEncMaxHeads + 5];
  for (int c = threadIdx.x; c < T.nchunks; c += blockDim.x) {
    int seg = 0;
#pragma unroll
    for (int k = 1; k < kSegs; ++k)
      if (c >= T.coff[k]) seg = k;
    const float* sp = T.src[0];
    int len = 0, dst = 0, N = 0, c0 = 0;
#pragma unroll
    for (int k = 0; k < kSegs; ++k)
      if (seg == k) {
        sp = T.src[k];
        len = T.len[k];
        dst = T.dst[k];
        N = T.rowN[k];
        c0 = T.coff[k];
      }
    const int r0 = (c - c0) * kChunk;
    float v[kChunk];
#pragma unroll
    for (int u = 0; u < kChunk; ++u) v[u] = r0 + u < len ? sp[r0 + u] : 0.f;
    int row = N ? r0 / N : 0, col = N ? r0 - row * N : r0;
    int d = dst + (N ? row * (N + 1) + col : r0);
#pragma unroll
    for (int u = 0; u < kChunk; ++u)
      if (r0 + u < len) {
        base[d++] = v[u];
        if (N && ++col == N) {   // next row (chunks are shorter than a row)
          col = 0;
          ++d;
        }
      }
  }
}

// stage_weights for a kernel built for NH heads: only the NH-head table's
// segments are looked up (fewer scalar registers than the 4-head table)
template <int NH>
__host__ __device__ constexpr int live_slot(int q) {
  return q < 2 * NH ? q
         : q < 2 * NH + 2 ? 2 * kGatEncMaxHeads + (q - 2 * NH)
         : q < 4 * NH + 2 ? 2 * kGatEncMaxHeads + 2 + (q - 2 * NH - 2)
                          : 4 * kGatEncMaxHeads + 2 + (q - 4 * NH - 2);
}
// the weight matrices' / vectors' places in an LDS image at base
template <int NH>
__device__ __forceinline__ void set_lw(float* base, const StageTab& T, LW& lw) {
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    lw.Wi[h] = base + T.dst[2 * h];
    lw.ai[h] = base + T.dst[2 * h + 1];
    lw.Wg[h] = base + T.dst[2 * kGatEncMaxHeads + 2 + 2 * h];
    lw.ag[h] = base + T.dst[2 * kGatEncMaxHeads + 3 + 2 * h];
  }
  lw.Wio = base + T.dst[2 * kGatEncMaxHeads];
  lw.aio = base + T.dst[2 * kGatEncMaxHeads + 1];
  lw.Wgo = base + T.dst[4 * kGatEncMaxHeads + 2];
  lw.ago = base + T.dst[4 * kGatEncMaxHeads + 3];
  lw.Woe = base + T.dst[4 * kGatEncMaxHeads + 4];
  lw.boe = base + T.dst[4 * kGatEncMaxHeads + 5];
}

template <int NH>
__device__ inline void stage_weights_t(float* base, const StageTab& T, LW& lw) {
  constexpr int NL = 4 * NH + 6;
  set_lw<NH>(base, T, lw);
  for (int c = threadIdx.x; c < T.nchunks; c += blockDim.x) {
    int q = 0;
#pragma unroll
    for (int k = 1; k < NL; ++k)
      if (c >= T.coff[live_slot<NH>(k)]) q = k;
    const float* sp = T.src[0];
    int len = 0, dst = 0, N = 0, c0 = 0;
#pragma unroll
    for (int k = 0; k < NL; ++k)
      if (q == k) {
        const int sl = live_slot<NH>(k);
        sp = T.src[sl];
        len = T.len[sl];
        dst = T.dst[sl];
        N = T.rowN[sl];
        c0 = T.coff[sl];
      }
    const int r0 = (c - c0) * kChunk;
    float v[kChunk];
#pragma unroll
    for (int u = 0; u < kChunk; ++u) v[u] = r0 + u < len ? sp[r0 + u] : 0.f;
    int row = N ? r0 / N : 0, col = N ? r0 - row * N : r0;
    int d = dst + (N ? row * (N + 1) + col : r0);
#pragma unroll
    for (int u = 0; u < kChunk; ++u)
      if (r0 + u < len) {
        base[d++] = v[u];
        if (N && ++col == N) {
          col = 0;
          ++d;
        }
      }
  }
}

// int region of a scene: lab (float), gidl, grank, cnt, ginv (float), M, then
// the groups' member masks (64-bit, 8-byte aligned)
__host__ __device__ inline int gm_offset(int np) { return (5 * np + 4 + 1) & ~1; }
__host__ __device__ inline int ints_floats(int np) { return gm_offset(np) + 2 * np; }
// attention matrix pitch: >= the 4-padded row count (the aggregation's
// reduction reads columns up to it), odd
__host__ __device__ inline int att_pitch(int np) { return (((np + 3) & ~3)) | 1; }
constexpr int kScoreTiles = (FH + 15) / 16;   // score partial sums: one per 16-column tile

struct Layout {
  // float offsets into the workgroup's LDS
  int X, H1, yI, preI, gin, G1, preG, gout, Wh, s, t, sp, tp, attm;   // forward
  int dWh, dH, dI, dG, dpre, dz, ds, dt;                             // backward
  int WhIs, stIs, WhIOs, stIOs, WhGs, stGs, WhGOs, stGOs;              // backward: the saved layer state
  int ints;       // see ints_floats
  int wts;        // the module's weights, staged once per workgroup (odd row pitches)
  int total;      // floats
  int PH, NP, NPP;
  int compact;    // backward plan for scenes past the full plan (see make_compact_layout)
};

constexpr int kLdsFloats = 160 * 1024 / 4;

// The backward's plan when the full one (every forward activation resident
// beside the gradients) exceeds the LDS -- scenes of 49 .. 64 peds with one
// head.  It needs the forward's saved state and keeps only what the phase at
// hand reads, aliased by lifetime:
//   * yI / gout (the out embedding's input), preG / preI (the epilogue
//     backwards) are read straight from the saved state in global memory,
//     once per element;
//   * one region U holds the inter layers' operands -- G1 | dH | gin | dpre --
//     during the inter backward, then the intra layers' -- H1 | dH | X --
//     loaded after the group-mean backward (H1 over the dead G1, X over the
//     dead gin / dpre; dH at the same offset in both).  The extra memory
//     round trip of H1 / X is the price (the inter operands arrive with dy).
__host__ __device__ inline Layout make_compact_layout(int np, int nh) {
  Layout L;
  L.NP = np;
  L.PH = FH * nh + 1;
  L.NPP = att_pitch(np);
  L.compact = 1;
  int o = 0;
  auto take = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
  L.s = take(np);
  L.t = take(np);
  L.ds = take(np);
  L.dt = take(np);
  L.attm = take(np * L.NPP);
  L.dz = take(np * L.NPP);
  L.Wh = take(np * P72);
  L.dWh = take(np * P72);
  L.dI = take(np * P16);
  L.dG = take(np * P16);
  const int ph = (np * L.PH + 3) & ~3, p16 = (np * P16 + 3) & ~3;
  const int u = take(2 * ph + (np * P40 > 2 * p16 ? np * P40 : 2 * p16));
  L.G1 = L.H1 = u;
  L.dH = u + ph;
  L.gin = L.X = u + 2 * ph;
  L.dpre = u + 2 * ph + p16;
  L.yI = L.preI = L.preG = L.gout = L.sp = L.tp = 0;   // (not resident)
  L.WhIs = L.stIs = L.WhIOs = L.stIOs = L.WhGs = L.stGs = L.WhGOs = L.stGOs = 0;
  L.ints = take(ints_floats(np));
  L.wts = take(weights_floats(nh));
  L.total = o;
  return L;
}

// full: every buffer of either direction resident (bwd 2: this plan even
// when it does not fit -- the recompute backward has no other)
__host__ __device__ inline Layout make_layout(int np, int nh, int bwd) {
  Layout L;
  L.NP = np;
  L.PH = FH * nh + 1;
  L.NPP = att_pitch(np);
  L.compact = 0;
  int o = 0;
  auto take = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
  L.X = take(np * P40);
  L.H1 = take(np * L.PH);
  L.yI = take(np * P16);
  L.preI = take(np * P16);
  L.gin = take(np * P16);
  L.G1 = take(np * L.PH);
  L.preG = take(np * P16);
  L.gout = take(np * P16);
  L.Wh = take(np * P72);
  L.s = take(np);
  L.t = take(np);
  L.sp = take(kScoreTiles * np);
  L.tp = take(kScoreTiles * np);
  L.attm = take(np * L.NPP);
  if (bwd) {
    L.dWh = take(np * P72);
    L.dH = take(np * L.PH);
    L.dI = take(np * P16);
    L.dG = take(np * P16);
    L.dpre = take(np * P16);
    L.dz = take(np * L.NPP);
    L.ds = take(np);
    L.dt = take(np);
    // every layer's Wh and scores s | t, loaded with the inputs (one round
    // trip per scene instead of one per layer) -- when they fit beside the
    // rest of the plan (else 0: loaded per layer into the Wh scratch)
    const int rest = ((ints_floats(np) + 3) & ~3) + ((weights_floats(nh) + 3) & ~3);
    const int pre = 2 * (((nh * np * P72 + 3) & ~3) + ((nh * 2 * np + 3) & ~3) + ((np * P16 + 3) & ~3) + ((2 * np + 3) & ~3));
    if (o + pre + rest <= kLdsFloats) {
      L.WhIs = take(nh * np * P72);
      L.stIs = take(nh * 2 * np);
      L.WhIOs = take(np * P16);
      L.stIOs = take(2 * np);
      L.WhGs = take(nh * np * P72);
      L.stGs = take(nh * 2 * np);
      L.WhGOs = take(np * P16);
      L.stGOs = take(2 * np);
    } else {
      L.WhIs = L.stIs = L.WhIOs = L.stIOs = L.WhGs = L.stGs = L.WhGOs = L.stGOs = 0;
    }
  } else {
    L.dWh = L.dH = L.dI = L.dG = L.dpre = L.dz = L.ds = L.dt = 0;
    L.WhIs = L.stIs = L.WhIOs = L.stIOs = L.WhGs = L.stGs = L.WhGOs = L.stGOs = 0;
  }
  L.ints = take(ints_floats(np));
  L.wts = take(weights_floats(nh));
  L.total = o;
  if (bwd == 1 && L.total > kLdsFloats) return make_compact_layout(np, nh);
  return L;
}

// parameter-gradient slab layout (floats per scene)
struct PLayout {
  int Wi[kGatEncMaxHeads], ai[kGatEncMaxHeads], Wio, aio, Wg[kGatEncMaxHeads], ag[kGatEncMaxHeads], Wgo, ago, Woe,
      boe, total;
};

__host__ __device__ inline PLayout make_playout(int nh) {
  PLayout P;
  int o = 0;
#pragma unroll
  for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
    if (h >= nh) break;
    P.Wi[h] = o; o += FI * FH;
    P.ai[h] = o; o += 2 * FH;
  }
  P.Wio = o; o += FH * nh * FO;
  P.aio = o; o += 2 * FO;
#pragma unroll
  for (int h = 0; h < kGatEncMaxHeads; ++h) {  // static head index: the LW / PLayout arrays stay in registers
    if (h >= nh) break;
    P.Wg[h] = o; o += FO * FH;
    P.ag[h] = o; o += 2 * FH;
  }
  P.Wgo = o; o += FH * nh * FO;
  P.ago = o; o += 2 * FO;
  P.Woe = o; o += FE * 2 * FO;
  P.boe = o; o += FE;
  P.total = o;
  return P;
}

// forward state of one scene kept for the backward (floats; written by the
// forward when args.saved != NULL, read back by the backward instead of
// recomputing the four attention layers): every layer's Wh and attention
// scores s | t, the head / out activations, the group structure
struct SLayout {
  int Whi[kGatEncMaxHeads], Whio, Whg[kGatEncMaxHeads], Whgo;
  int sti[kGatEncMaxHeads], stio, stg[kGatEncMaxHeads], stgo;
  int H1, yI, preI, gin, G1, preG, gout, ints, total;
};

__host__ __device__ inline SLayout make_slayout(int np, int nh) {
  SLayout S;
  int o = 0;
  for (int h = 0; h < kGatEncMaxHeads; ++h) {
    S.Whi[h] = o;
    S.sti[h] = o + np * FH;
    if (h < nh) o += np * FH + 2 * np;
  }
  S.Whio = o; o += np * FO;
  S.stio = o; o += 2 * np;
  for (int h = 0; h < kGatEncMaxHeads; ++h) {
    S.Whg[h] = o;
    S.stg[h] = o + np * FH;
    if (h < nh) o += np * FH + 2 * np;
  }
  S.Whgo = o; o += np * FO;
  S.stgo = o; o += 2 * np;
  S.H1 = o; o += np * FH * nh;
  S.yI = o; o += np * FO;
  S.preI = o; o += np * FO;
  S.gin = o; o += np * FO;
  S.G1 = o; o += np * FH * nh;
  S.preG = o; o += np * FO;
  S.gout = o; o += np * FO;
  S.ints = (o + 1) & ~1; o = S.ints + ints_floats(np);
  S.total = (o + 3) & ~3;
  return S;
}

// rows x cols between an LDS image at pitch ld and a dense global block
__device__ inline void rows_to_global(float* __restrict__ dst, const float* src, int ld, int rows, int cols) {
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int r = e / cols, c = e - r * cols;
    dst[e] = src[r * ld + c];
  }
}
__device__ inline void rows_from_global(float* dst, int ld, const float* __restrict__ src, int rows, int cols) {
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    const int r = e / cols, c = e - r * cols;
    dst[r * ld + c] = src[e];
  }
}

// Several rows x cols global blocks (source row pitch sld, 0: dense) into LDS
// images (pitch dld, 0: dense) with every block's loads of a round issued
// before any of its stores: one memory round trip per round of 2 x blockDim
// elements of each block, where a rows_from_global per block waits out one
// round trip per block (and per element of a thread).  Element pairs: every
// block's cols, row pitch and source offset are even (8-byte loads; a pair
// never crosses a row), so a round is one 8-byte load per thread and block.
// The loads are clamped, not guarded (a guard's branches break the batch up
// with waits); lanes past a block reload its last pair and do not store.
struct GSeg {
  float* dst;
  int dld;
  const float* src;
  int sld, rows, cols;
};
// (cols are compile-time constants at every call: the lane's row / column
// per distinct width is one multiply-shift, shared by the blocks of that
// width; a lane past a block clamps its row, and a block of 0 rows reads
// its source's first pair)
template <int NS>
__device__ __forceinline__ void segs_load(const GSeg (&g)[NS], float2 (&v)[NS], int base) {
  const int e = base + 2 * (int)threadIdx.x;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int r0 = e / g[s].cols, c = e - r0 * g[s].cols;
    const int r = max(min(r0, g[s].rows - 1), 0);
    v[s] = *reinterpret_cast<const float2*>(g[s].src + (g[s].sld ? r * g[s].sld : r * g[s].cols) + c);
  }
}
template <int NS>
__device__ __forceinline__ void segs_store(const GSeg (&g)[NS], const float2 (&v)[NS], int base) {
  const int e = base + 2 * (int)threadIdx.x;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int r = e / g[s].cols, c = e - r * g[s].cols;
    if (r < g[s].rows) {
      float* d = g[s].dst + (g[s].dld ? r * g[s].dld : r * g[s].cols) + c;
      d[0] = v[s].x;
      d[1] = v[s].y;
    }
  }
}
template <int NS>
__device__ __forceinline__ int segs_most(const GSeg (&g)[NS]) {
  int most = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s) most = max(most, g[s].rows * g[s].cols);
  return most;
}
template <int NS>
__device__ __forceinline__ void segs_from_global(const GSeg (&g)[NS]) {
  const int most = segs_most(g);
  for (int base = 0; base < most; base += 2 * (int)blockDim.x) {
    float2 v[NS];
    segs_load(g, v, base);
    segs_store(g, v, base);
  }
}

__device__ __forceinline__ float lrelu(float x, float a) { return x > 0.f ? x : a * x; }

// ---------------------------------------------------------------------------
// cross-lane reductions on DPP lane moves (VALU; the shuffle forms cost an LDS
// round trip per step).  Every lane ends with the bitwise-same value (each
// step adds a lane pair in both orders, and + / max commute exactly).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ float dpp(float v, float old) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROWS, 0xF, false));
}
// over each row of 16 lanes
__device__ __forceinline__ float row_sum(float v) {
  v += dpp<0xB1>(v, 0.f);    // quad_perm [1, 0, 3, 2]
  v += dpp<0x4E>(v, 0.f);    // quad_perm [2, 3, 0, 1]
  v += dpp<0x141>(v, 0.f);   // row_half_mirror
  v += dpp<0x140>(v, 0.f);   // row_mirror
  return v;
}
__device__ __forceinline__ float row_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v, -INFINITY));
  v = fmaxf(v, dpp<0x4E>(v, -INFINITY));
  v = fmaxf(v, dpp<0x141>(v, -INFINITY));
  v = fmaxf(v, dpp<0x140>(v, -INFINITY));
  return v;
}
__device__ __forceinline__ float lane63(float v) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// over the wave: rows, then row_bcast:15 into rows 1 / 3 and row_bcast:31
// into rows 2 / 3; lane 63 holds the total, broadcast by readlane
__device__ __forceinline__ float wsum(float v) {
  v = row_sum(v);
  v += dpp<0x142, 0xA>(v, 0.f);
  v += dpp<0x143, 0xC>(v, 0.f);
  return lane63(v);
}
__device__ __forceinline__ float wmax(float v) {
  v = row_max(v);
  v = fmaxf(v, dpp<0x142, 0xA>(v, -INFINITY));
  v = fmaxf(v, dpp<0x143, 0xC>(v, -INFINITY));
  return lane63(v);
}

// ---------------------------------------------------------------------------
// Matrix products on the f32 MFMA (v_mfma_f32_16x16x4_f32): 16 x 16 output
// tiles, one wavefront per tile (tiles dealt round-robin over the
// workgroup's waves, starting at wave `first` so that two products issued in
// one phase share the waves out).  Operand lanes: A[i = lane & 15][k = lane >>
// 4], B[k = lane >> 4][j = lane & 15]; the D lane holds rows 4 (lane >> 4) + r,
// column lane & 15.  Rows / columns past the edge read a clamped (valid)
// element and are not stored; a reduction over rows masks them to zero.
// k-steps per operand batch of lin / lin_t / wgrad (template NB): the forward
// kernel batches 4 (its 1024-thread workgroups leave it registers); the
// backward sits at the 128-VGPR cap and keeps the plain loop (NB = 1)
__device__ __forceinline__ int mm_wave(int first) {
  const int nw = blockDim.x >> 6;
  return ((int)(threadIdx.x >> 6) + nw - first % nw) % nw;
}

// out[r][c] = sum_k in[r][k] W[k][c]   (W: K x N in LDS at pitch ldw, K % 4 == 0).
// With a (2N: a_src | a_dst), also the attention score partials of the tile:
// sp[tile column][r] = sum over its 16 columns of out[r][c] a[c], tp the same
// with a[N + c] (att_rows sums the column tiles).
template <int kMmB = 1>
__device__ __forceinline__ void lin(const float* in, int ldi, int rows, int K, const float* W, int ldw, int N, float* out, int ldo,
                    int first = 0, const float* a = nullptr, float* sp = nullptr, float* tp = nullptr, int np = 0) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6, i = lane & 15, kq = lane >> 4;
  const int ct = (N + 15) >> 4, nt = ((rows + 15) >> 4) * ct;
  for (int tile = mm_wave(first); tile < nt; tile += nw) {
    const int r0 = (tile / ct) << 4, c0 = (tile % ct) << 4;
    const float* pa = in + min(r0 + i, rows - 1) * ldi + kq;
    const float* pb = W + kq * ldw + min(c0 + i, N - 1);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    // batches of kMmB k-steps: the batch's LDS operands are read before its
    // MFMAs (one LDS latency per batch, not per k-step); k-steps past K
    // multiply zeros (the sum is unchanged, bit for bit)
    if constexpr (kMmB == 1) {
#pragma unroll 2
      for (int k = 0; k < K; k += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[k], pb[k * ldw], acc, 0, 0, 0);
    } else
    for (int k = 0; k < K; k += 4 * kMmB) {
      float av[kMmB], bv[kMmB];
#pragma unroll
      for (int u = 0; u < kMmB; ++u) {
        const int kk = min(k + 4 * u, K - 4);
        av[u] = k + 4 * u < K ? pa[kk] : 0.f;
        bv[u] = k + 4 * u < K ? pb[kk * ldw] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kMmB; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
    const int col = c0 + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * kq + r;
      if (row < rows && col < N) out[row * ldo + col] = acc[r];
    }
    if (a) {
      const float as = col < N ? a[col] : 0.f, at = col < N ? a[N + col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ps = row_sum(acc[r] * as), pt = row_sum(acc[r] * at);
        const int row = r0 + 4 * kq + r;
        if (i == 0 && row < rows) {
          sp[(c0 >> 4) * np + row] = ps;
          tp[(c0 >> 4) * np + row] = pt;
        }
      }
    }
  }
}

// out[r][k] (+)= sum_c d[r][c] W[k][c]   (input gradient of lin; N % 4 == 0;
// out may be global memory)
// (out2: columns >= ksplit go to out2 at pitch ldo2 instead)
template <int kMmB = 1>
__device__ __forceinline__ void lin_t(const float* d, int ldd, int rows, int N, const float* W, int ldw, int K, float* out, int ldo,
                      bool accum, int first = 0, float* out2 = nullptr, int ldo2 = 0, int ksplit = 0) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6, i = lane & 15, kq = lane >> 4;
  const int ct = (K + 15) >> 4, nt = ((rows + 15) >> 4) * ct;
  for (int tile = mm_wave(first); tile < nt; tile += nw) {
    const int r0 = (tile / ct) << 4, k0 = (tile % ct) << 4;
    const float* pa = d + min(r0 + i, rows - 1) * ldd + kq;
    const float* pb = W + min(k0 + i, K - 1) * ldw + kq;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (kMmB == 1) {
#pragma unroll 2
      for (int c = 0; c < N; c += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[c], pb[c], acc, 0, 0, 0);
    } else
    for (int c = 0; c < N; c += 4 * kMmB) {   // batched as in lin
      float av[kMmB], bv[kMmB];
#pragma unroll
      for (int u = 0; u < kMmB; ++u) {
        const int cc = min(c + 4 * u, N - 4);
        av[u] = c + 4 * u < N ? pa[cc] : 0.f;
        bv[u] = c + 4 * u < N ? pb[cc] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kMmB; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
    const int col = k0 + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * kq + r;
      if (row < rows && col < K) {
        float* po = out2 && col >= ksplit ? out2 + row * ldo2 + (col - ksplit) : out + row * ldo + col;
        *po = accum ? *po + acc[r] : acc[r];
      }
    }
  }
}

// dst[k][c] = sum_r x[r][k] d[r][c]  (weight gradient of lin: to the slab,
// ldo = N; or an LDS image)
template <int kMmB = 1>
__device__ __forceinline__ void wgrad(const float* x, int ldx, int rows, int K, const float* d, int ldd, int N, float* dst, int ldo,
                      int first = 0) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6, i = lane & 15, kq = lane >> 4;
  const int ct = (N + 15) >> 4, nt = ((K + 15) >> 4) * ct;
  for (int tile = mm_wave(first); tile < nt; tile += nw) {
    const int k0 = (tile / ct) << 4, c0 = (tile % ct) << 4;
    const float* pa = x + min(k0 + i, K - 1);
    const float* pb = d + min(c0 + i, N - 1);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    // the lane's row r; a step covers rows r - kq .. r - kq + 3; batched as in lin
    if constexpr (kMmB == 1) {
      for (int r = kq; r < rows + kq; r += 4) {
        const bool ok = r < rows;
        const float av = ok ? pa[r * ldx] : 0.f, bv = ok ? pb[r * ldd] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
    } else
    for (int r = kq; r < rows + kq; r += 4 * kMmB) {
      float av[kMmB], bv[kMmB];
#pragma unroll
      for (int u = 0; u < kMmB; ++u) {
        const int rr = r + 4 * u;
        const bool ok = rr < rows;
        av[u] = ok ? pa[rr * ldx] : 0.f;
        bv[u] = ok ? pb[rr * ldd] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kMmB; ++u)
        if (r + 4 * u < rows + kq) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
    const int col = c0 + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = k0 + 4 * kq + r;
      if (row < K && col < N) dst[row * ldo + col] = acc[r];
    }
  }
}

__device__ __forceinline__ bool edge(const int* gidl, int i, int j) { return gidl == nullptr || gidl[i] == gidl[j]; }

// s_i / t_i from lin's score partials (ct column tiles)
__device__ __forceinline__ float score_of(const float* part, int ct, int np, int i) {
  float v = part[i];
  for (int c = 1; c < ct; ++c) v += part[c * np + i];
  return v;
}

// attention rows (one wavefront per row i, lane j; rows <= 64): att_ij =
// softmax_j(LeakyReLU(s_i + t_j)) over the graph's edges, to attm (columns
// up to the 4-padded row count, zero past the rows).  s / t from lin's
// partials (ct >= 1) or, ct == 0, already in s / t.  Writes s / t (and the
// saved copy sv: s | t, when given).
__device__ void att_rows(int rows, int ct, const float* sp, const float* tp, int np, const int* gidl, float alpha,
                         float* s, float* t, float* attm, int npp, float* sv) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int cols = (rows + 3) & ~3;
  for (int i = threadIdx.x >> 6; i < rows; i += nw) {
    const int j = min(lane, rows - 1);
    const float si = ct ? score_of(sp, ct, np, i) : s[i];
    const float tj = ct ? score_of(tp, ct, np, j) : t[j];
    const bool ok = lane < rows && edge(gidl, i, lane);
    const float e = ok ? lrelu(si + tj, alpha) : -INFINITY;
    const float m = wmax(e);
    const float pe = ok ? __expf(e - m) : 0.f;
    const float sum = wsum(pe);
    if (lane < cols) attm[i * npp + lane] = pe / sum;
    if (ct) {
      if (lane == 0) s[i] = si;
      if (lane == i) t[i] = tj;
      if (sv) {
        if (lane == 0) sv[i] = si;
        if (lane == i) sv[np + i] = tj;
      }
    }
  }
}

// out = epi(att Wh) on the MFMA (reduction over the rows' 4-padded columns
// of attm; B rows past the edge clamp, their A columns are zero).  epi 1:
// ELU; epi 2 (F == 16: a row is one lane row): pre = att Wh, out =
// log_softmax(ELU(pre)) over the 16 features
__device__ void att_agg(const float* attm, int npp, int rows, const float* Wh, int ldw, int F, int epi, float* out,
                        int ldo, float* pre, int ldp) {
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6, i = lane & 15, kq = lane >> 4;
  const int ct = (F + 15) >> 4, nt = ((rows + 15) >> 4) * ct;
  const int K = (rows + 3) & ~3;
  for (int tile = threadIdx.x >> 6; tile < nt; tile += nw) {
    const int r0 = (tile / ct) << 4, c0 = (tile % ct) << 4;
    const float* pa = attm + min(r0 + i, rows - 1) * npp + kq;
    const float* pb = Wh + min(c0 + i, F - 1);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; k += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[k], pb[min(k + kq, rows - 1) * ldw], acc, 0, 0, 0);
    const int col = c0 + i;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + 4 * kq + r;
      const float z = elu(acc[r]);
      float v = z;
      if (epi == 2) {
        const float zm = row_max(z);
        const float lse = zm + __logf(row_sum(__expf(z - zm)));
        v = z - lse;
      }
      if (row < rows && col < F) {
        out[row * ldo + col] = v;
        if (pre) pre[row * ldp + col] = acc[r];
      }
    }
  }
}

// gradient through the epilogue: d (in: d out, out: d pre), one wave per row
__device__ void epi_bwd(float* d, int ldd, const float* pre, int ldp, int rows, int F, int epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = wave; i < rows; i += (int)(blockDim.x >> 6)) {
    float dv[2], hv[2], zv[2];
    float zmax = -INFINITY, sdy = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = lane + 64 * c;
      dv[c] = f < F ? d[i * ldd + f] : 0.f;
      hv[c] = f < F ? pre[i * ldp + f] : 0.f;
      zv[c] = elu(hv[c]);
      if (f < F) {
        zmax = fmaxf(zmax, zv[c]);
        sdy += dv[c];
      }
    }
    float lse = 0.f;
    if (epi == 2) {
      zmax = wmax(zmax);
      sdy = wsum(sdy);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (lane + 64 * c < F) se += __expf(zv[c] - zmax);
      lse = zmax + __logf(wsum(se));
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int f = lane + 64 * c;
      if (f < F) {
        float v = dv[c];
        if (epi == 2) v -= __expf(zv[c] - lse) * sdy;
        d[i * ldd + f] = v * elu_grad(hv[c]);
      }
    }
  }
}

#ifdef SGG_GATENC_PROF
__device__ long long g_gatenc_prof[2][64];   // phase timestamps (tools/gatenc_probe.hip)
#endif

// The backward's preloaded blocks of one scene (the full plan with every
// layer's state resident; 1 - 2 heads): group structure, activations, every
// layer's Wh / scores, and dy when it is one copy at an 8-byte aligned pitch
// (dy_pairs; else its block is empty and the caller sums the copies)
template <int NH>
__device__ __forceinline__ void preload_segs(GSeg (&g)[12 + 4 * NH + 1], float* sm, const Layout& L,
                                             const SLayout& SL, const float* saved, const float* dyg, int lddy, int n,
                                             bool dy_pairs) {
  const int NP = L.NP, PH = L.PH, SLH = NP * FH + 2 * NP;
  int ns = 0;
  g[ns++] = {sm + L.ints, 0, saved + SL.ints, 0, ints_floats(NP) / 2, 2};
  g[ns++] = {sm + L.H1, PH, saved + SL.H1, 0, n, FH * NH};
  g[ns++] = {sm + L.yI, P16, saved + SL.yI, 0, n, FO};
  g[ns++] = {sm + L.preI, P16, saved + SL.preI, 0, n, FO};
  g[ns++] = {sm + L.gin, P16, saved + SL.gin, 0, n, FO};
  g[ns++] = {sm + L.G1, PH, saved + SL.G1, 0, n, FH * NH};
  g[ns++] = {sm + L.preG, P16, saved + SL.preG, 0, n, FO};
  g[ns++] = {sm + L.gout, P16, saved + SL.gout, 0, n, FO};
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    g[ns++] = {sm + L.WhIs + h * NP * P72, P72, saved + (SL.Whi[0] + h * SLH), 0, n, FH};
    g[ns++] = {sm + L.stIs + h * 2 * NP, 0, saved + (SL.sti[0] + h * SLH), 0, NP, 2};
    g[ns++] = {sm + L.WhGs + h * NP * P72, P72, saved + (SL.Whg[0] + h * SLH), 0, n, FH};
    g[ns++] = {sm + L.stGs + h * 2 * NP, 0, saved + (SL.stg[0] + h * SLH), 0, NP, 2};
  }
  g[ns++] = {sm + L.WhIOs, P16, saved + SL.Whio, 0, n, FO};
  g[ns++] = {sm + L.stIOs, 0, saved + SL.stio, 0, NP, 2};
  g[ns++] = {sm + L.WhGOs, P16, saved + SL.Whgo, 0, n, FO};
  g[ns++] = {sm + L.stGOs, 0, saved + SL.stgo, 0, NP, 2};
  g[ns++] = {sm + L.Wh, FE + 1, dy_pairs ? dyg : saved, lddy, dy_pairs ? n : 0, FE};
}

// stage_weights_t with the image's blocks at compile-time shapes (1 - 2
// heads; every parameter 8-byte aligned): one batch of pair loads, then the
// stores at the matrices' pitches -- a few VALU operations per pair instead of
// the per-chunk segment search and row walk (the 16 waves of a workgroup share
// 4 SIMDs, so the staging's VALU count is its time)
template <int NH>
__device__ __forceinline__ bool stage_fast_ok(const StageTab& T) {
  size_t a = 0;
#pragma unroll
  for (int k = 0; k < 4 * NH + 6; ++k) a |= reinterpret_cast<size_t>(T.src[live_slot<NH>(k)]);
  return NH <= 2 && (a & 7) == 0;
}
template <int NH>
__device__ __forceinline__ void stage_weights_fast(float* base, const StageTab& T, LW& lw) {
  set_lw<NH>(base, T, lw);
  constexpr int NS = 5 * NH + 6 + (NH > 1 ? 2 : 0);
  constexpr int HI = FI / 2;   // Wi in two row halves (<= 2 x 1024 floats each)
  constexpr int RO = NH > 1 ? FH : FH * NH;   // Wio / Wgo row blocks
  GSeg g[NS];
  int ns = 0;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int si = live_slot<NH>(2 * h), sa = live_slot<NH>(2 * h + 1);
    g[ns++] = {base + T.dst[si], PW72, T.src[si], 0, HI, FH};
    g[ns++] = {base + T.dst[si] + HI * PW72, PW72, T.src[si] + HI * FH, 0, HI, FH};
    g[ns++] = {base + T.dst[sa], 0, T.src[sa], 0, FH, 2};
  }
  {
    const int so = live_slot<NH>(2 * NH), sa = live_slot<NH>(2 * NH + 1);
#pragma unroll
    for (int b = 0; b < (NH > 1 ? 2 : 1); ++b)
      g[ns++] = {base + T.dst[so] + b * RO * PW16, PW16, T.src[so] + b * RO * FO, 0, NH > 1 ? FH * NH / 2 : RO, FO};
    g[ns++] = {base + T.dst[sa], 0, T.src[sa], 0, FO, 2};
  }
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int sw = live_slot<NH>(2 * NH + 2 + 2 * h), sa = live_slot<NH>(2 * NH + 3 + 2 * h);
    g[ns++] = {base + T.dst[sw], PW72, T.src[sw], 0, FO, FH};
    g[ns++] = {base + T.dst[sa], 0, T.src[sa], 0, FH, 2};
  }
  {
    const int so = live_slot<NH>(4 * NH + 2), sa = live_slot<NH>(4 * NH + 3);
#pragma unroll
    for (int b = 0; b < (NH > 1 ? 2 : 1); ++b)
      g[ns++] = {base + T.dst[so] + b * RO * PW16, PW16, T.src[so] + b * RO * FO, 0, NH > 1 ? FH * NH / 2 : RO, FO};
    g[ns++] = {base + T.dst[sa], 0, T.src[sa], 0, FO, 2};
    const int se = live_slot<NH>(4 * NH + 4), sb = live_slot<NH>(4 * NH + 5);
    g[ns++] = {base + T.dst[se], PWE, T.src[se], 0, FE, 2 * FO};
    g[ns++] = {base + T.dst[sb], 0, T.src[sb], 0, FE / 2, 2};
  }
  segs_from_global(g);
}

__device__ __forceinline__ bool dy_pairs_ok(const GatEncArgs& p) {
  return p.dy_copies <= 1 && (p.lddy & 1) == 0 && (reinterpret_cast<size_t>(p.dy) & 7) == 0;
}

// attention layer backward, s / t / Wh in LDS.  dpre: gradient of the
// aggregate (rows x F).  Writes dWh (rows x F) and starts the a-gradient
// (2F, to da) in the last phase WITHOUT a closing barrier: the caller adds
// its weight / input gradient products to that phase.  attm, dz: scratch
// rows x npp.
__device__ __forceinline__ void att_bwd(const float* Wh, int ldw, int rows, int F, const int* gidl, const float* s, const float* t,
                        float alpha, const float* a, const float* dpre, int ldd, float* dWh, int lddw, float* ds,
                        float* dt, float* attm, float* dz, int npp, float* da, int mk = 0) {
#ifdef SGG_GATENC_PROF
#define AMARK(i) \
  if (mk && threadIdx.x == 0 && blockIdx.x == 0) g_gatenc_prof[1][mk + (i)] = wall_clock64();
#else
#define AMARK(i)
#endif
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  att_rows(rows, 0, nullptr, nullptr, 0, gidl, alpha, const_cast<float*>(s), const_cast<float*>(t), attm, npp,
           nullptr);
  lds_barrier(); AMARK(0);
  // dWh = att^T dpre; datt = dpre Wh^T (to dz)
  wgrad(attm, npp, rows, rows, dpre, ldd, F, dWh, lddw, 0);
  lin_t(dpre, ldd, rows, F, Wh, ldw, rows, dz, npp, false, 8);
  lds_barrier(); AMARK(1);
  // softmax + LeakyReLU backward, row i: dz_ij = lrelu'(.) att_ij (datt_ij - sum_k att_ik datt_ik)
  for (int i = threadIdx.x >> 6; i < rows; i += nw) {
    const bool ok = lane < rows;
    const float at = ok ? attm[i * npp + lane] : 0.f, dv = ok ? dz[i * npp + lane] : 0.f;
    const float dot = wsum(at * dv);
    const float de = at * (dv - dot);
    const float z = ok ? ((s[i] + t[lane]) > 0.f ? de : alpha * de) : 0.f;
    if (ok) dz[i * npp + lane] = z;
    const float dsum = wsum(z);
    if (lane == 0) ds[i] = dsum;
  }
  lds_barrier(); AMARK(2);
  // column j: dt_j = sum_i dz_ij; dWh_j += ds_j a[:F] + dt_j a[F:]
  for (int j = threadIdx.x >> 6; j < rows; j += nw) {
    const float dtj = wsum(lane < rows ? dz[lane * npp + j] : 0.f);
    if (lane == 0) dt[j] = dtj;
    const float dsj = ds[j];
    for (int f = lane; f < F; f += 64) dWh[j * lddw + f] += dsj * a[f] + dtj * a[F + f];
  }
  lds_barrier(); AMARK(3);
  // da[f] = sum_i ds_i Wh_i[f], da[F + f] = sum_j dt_j Wh_j[f]: four
  // interleaved partial sums per output (one chain over the rows waited an
  // LDS latency per row: ~1 us at F = 72, 20 rows)
  for (int e = threadIdx.x; e < 2 * F; e += blockDim.x) {
    const int w = e / F, f = e - w * F;
    const float* g = w ? dt : ds;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int r = 0;
    for (; r + 4 <= rows; r += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = fmaf(g[r + u], Wh[(r + u) * ldw + f], acc[u]);
    }
    for (; r < rows; ++r) acc[0] = fmaf(g[r], Wh[r * ldw + f], acc[0]);
    da[e] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  AMARK(4);
#undef AMARK
}

// phase timestamps of workgroup 0's first scene (tools/gatenc_probe.hip)
#ifdef SGG_GATENC_PROF
#define PMARK(i) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_gatenc_prof[BWD][i] = wall_clock64();
#define PMARKW(i) \
  if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) g_gatenc_prof[BWD][(i) + (threadIdx.x >> 6)] = wall_clock64();
#else
#define PMARK(i)
#define PMARKW(i)
#endif

// the scene set of virtual scene vs: p's scenes first, then s2's (a
// forward over two independent batches with the same weights and np in one
// launch, sgg_gatenc_fwd2); per-field uniform selects, no struct copy
__device__ __forceinline__ GatEncSet pick_set(const GatEncArgs& p, const GatEncSet& s2, bool two) {
  GatEncSet q;
  q.X = two ? s2.X : p.X;
  q.ldx = two ? s2.ldx : p.ldx;
  q.X2 = two ? s2.X2 : p.X2;
  q.ldx2 = two ? s2.ldx2 : p.ldx2;
  q.kx1 = two ? s2.kx1 : p.kx1;
  q.labels = two ? s2.labels : p.labels;
  q.scene_off = two ? s2.scene_off : p.scene_off;
  q.S = two ? s2.S : p.S;
  q.y = two ? s2.y : p.y;
  q.ldy = two ? s2.ldy : p.ldy;
  q.saved = two ? s2.saved : p.saved;
  return q;
}

template <bool BWD, int NH>
__global__ void __launch_bounds__(BWD ? kBwdThreads : kFwdThreads) gatenc_kernel(GatEncArgs p, StageTab tab,
                                                                                  GatEncSet s2) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int nh = NH;
  // per-head strides of the weight image, the slab row and the saved state
  constexpr int SEGI = FI * PW72 + 2 * FH, SEGG = FO * PW72 + 2 * FH, PLI = FI * FH + 2 * FH, PLG = FO * FH + 2 * FH;
  const int tid = threadIdx.x;
  // element e = r * FI + k of a scene's input rows (the split input: X2)
  auto xval = [&](const GatEncSet& q, int o, int e) -> float {
    const int r = e / FI, k = e - r * FI;
    return q.X2 && k >= q.kx1 ? q.X2[(size_t)(o + r) * q.ldx2 + (k - q.kx1)] : q.X[(size_t)(o + r) * q.ldx + k];
  };
  const int nvs = p.S + (BWD ? 0 : s2.S);   // virtual scenes (the backward: p's only)
  // the first scene's inputs are loaded before the weight staging so their
  // latency hides under it (registers; stored after the staging)
  constexpr int kXPre = 3;
  const bool two0 = !BWD && (int)blockIdx.x >= p.S;
  const GatEncSet q0 = pick_set(p, s2, two0);
  const int sc0 = two0 ? (int)blockIdx.x - p.S : (int)blockIdx.x;
  const int o0 = q0.scene_off[sc0], n0 = q0.scene_off[sc0 + 1] - o0;
  const bool pre = n0 > 0 && n0 * FI <= kXPre * (int)blockDim.x;   // uniform
  float xp[kXPre];
  float lp = 0.f;
  if (pre) {
#pragma unroll
    for (int m = 0; m < kXPre; ++m) {
      const int e = tid + m * (int)blockDim.x;
      xp[m] = e < n0 * FI ? xval(q0, o0, e) : 0.f;
    }
    if (tid < n0) lp = q0.labels[o0 + tid];
  }
  PMARK(40);
  PMARKW(42);
  // the first scene's backward preload (1 - 2 heads, when one round covers
  // it): its loads go out with the weight staging's, its stores follow them
  constexpr int NSEG = 12 + 4 * NH + 1;
  bool pre0 = false;
  GSeg g0[NSEG];
  float2 v0[NSEG];
  if constexpr (BWD && NH <= 2) {
    const Layout L0 = make_layout(p.np, NH, BWD);
    pre0 = p.saved && !L0.compact && L0.WhIs > 0 && n0 > 0 && n0 * FH * NH <= 2 * (int)blockDim.x;   // uniform
    if (pre0) {
      const SLayout SL0 = make_slayout(p.np, NH);
      preload_segs<NH>(g0, sm, L0, SL0, p.saved + (size_t)sc0 * SL0.total, p.dy + (size_t)o0 * p.lddy, p.lddy, n0,
                       dy_pairs_ok(p));
      segs_load(g0, v0, 0);
    }
  }
  // The weights' LDS image.  The backward with the forward's saved state
  // copies the image that forward's workgroup 0 left after the saved blocks
  // (contiguous, 16-byte loads, no per-element placement); otherwise each
  // workgroup stages it from the parameters (stage_weights_t)
  LW lw;
  float* const wbase = sm + make_layout(p.np, NH, BWD).wts;
  constexpr int WF4 = (weights_floats(NH) + 3) / 4, WQ = (WF4 + kBwdThreads - 1) / kBwdThreads;
  const bool wimg = BWD && p.saved != nullptr;   // uniform
  if (wimg) {
    set_lw<NH>(wbase, tab, lw);
    const floatx4* img = reinterpret_cast<const floatx4*>(p.saved + (size_t)p.S * make_slayout(p.np, NH).total);
    floatx4 wv[WQ];
#pragma unroll
    for (int m = 0; m < WQ; ++m) wv[m] = img[min(tid + m * (int)blockDim.x, WF4 - 1)];
#pragma unroll
    for (int m = 0; m < WQ; ++m)
      if (tid + m * (int)blockDim.x < WF4) reinterpret_cast<floatx4*>(wbase)[tid + m * (int)blockDim.x] = wv[m];
  } else {
    // (the forward only: in the backward the dead branch costs the preload's
    // schedule ~1 us, measured)
    bool fast = false;
    if constexpr (!BWD) fast = stage_fast_ok<NH>(tab);
    if (fast)
      stage_weights_fast<NH>(wbase, tab, lw);
    else
      stage_weights_t<NH>(wbase, tab, lw);
  }
  if constexpr (BWD && NH <= 2)
    if (pre0) segs_store(g0, v0, 0);
  // (the first scene's input stores are followed by a barrier before any use)
  PMARK(41);

  for (int vs = blockIdx.x; vs < nvs; vs += gridDim.x) {
    const bool two = !BWD && vs >= p.S;   // uniform
    const GatEncSet q = pick_set(p, s2, two);
    const int sc = two ? vs - p.S : vs;
    // the LDS plan derived per scene from an opaque copy of np: hoisted out
    // of the scene loop, the per-lane addresses spill to scratch
    int NPo = p.np;
    __asm__ volatile("" : "+s"(NPo));
    const Layout L = make_layout(NPo, NH, BWD);
    const PLayout PL = make_playout(NH);
    const SLayout SL = make_slayout(NPo, NH);
    const int PH = L.PH, NP = L.NP, NPP = L.NPP;
    const bool compact = BWD && L.compact;   // uniform (the host requires the saved state for it)
    const int SLH = NP * FH + 2 * NP;
    float* X = sm + L.X;
    float* H1 = sm + L.H1;
    float* yI = sm + L.yI;
    float* preI = sm + L.preI;
    float* gin = sm + L.gin;
    float* G1 = sm + L.G1;
    float* preG = sm + L.preG;
    float* gout = sm + L.gout;
    float* Wh = sm + L.Wh;
    float* s = sm + L.s;
    float* t = sm + L.t;
    float* sp = sm + L.sp;
    float* tp = sm + L.tp;
    float* attm = sm + L.attm;
    float* lab = sm + L.ints;
    int* gidl = reinterpret_cast<int*>(lab + NP);
    int* grank = gidl + NP;
    int* cnt = grank + NP;
    float* ginv = reinterpret_cast<float*>(cnt + NP);
    int* Mp = reinterpret_cast<int*>(ginv + NP);
    unsigned long long* gm = reinterpret_cast<unsigned long long*>(lab + gm_offset(NP));
    // (the first scene's offsets were read at entry: no second dependent load)
    const bool first_vs = vs == (int)blockIdx.x;
    const int o = first_vs ? o0 : q.scene_off[sc];
    const int n = first_vs ? n0 : q.scene_off[sc + 1] - o;
    if (n <= 0) continue;   // uniform over the workgroup
    PMARK(0);
    const bool first = pre && vs == (int)blockIdx.x;   // uniform
    float* saved = q.saved ? q.saved + (size_t)sc * SL.total : nullptr;
    // ---- inputs and group structure (one phase) ------------------------
    if (compact) {
      // (X arrives with H1 before the intra backward)
    } else if (first) {
#pragma unroll
      for (int m = 0; m < kXPre; ++m) {
        const int e = tid + m * (int)blockDim.x;
        if (e < n * FI) {
          const int r = e / FI;
          X[r * P40 + (e - r * FI)] = xp[m];
        }
      }
    } else {
      for (int e = tid; e < n * FI; e += blockDim.x) {
        const int r = e / FI;
        X[r * P40 + (e - r * FI)] = xval(q, o, e);
      }
    }
    PMARK(37);
    const bool preload = BWD && saved && L.WhIs > 0;   // uniform
    if (BWD && saved && !preload) rows_from_global(lab, 0, saved + SL.ints, 1, ints_floats(NP));
    if (preload) {
      // the backward's whole input in ONE memory round trip: group structure,
      // activations, every layer's Wh / scores (n rows: the group-side rows
      // past M are never read), dy (+ its copies)
      constexpr int PDY = FE + 1;
      const float* dyg = p.dy + (size_t)o * p.lddy;
      const int ncp = p.dy_copies > 1 ? p.dy_copies : 1;
      const bool dy_pairs = NH <= 2 && dy_pairs_ok(p);
      if constexpr (NH <= 2) {
        if (!(pre0 && first_vs)) {   // (the first scene's came with the weights)
          GSeg g[NSEG];
          preload_segs<NH>(g, sm, L, SL, saved, dyg, p.lddy, n, dy_pairs);
          segs_from_global(g);
        }
        PMARK(38);
      } else {   // (3 - 4 heads: one block at a time -- all in flight would spill)
        rows_from_global(lab, 0, saved + SL.ints, 1, ints_floats(NP));
        rows_from_global(H1, PH, saved + SL.H1, n, FH * nh);
        rows_from_global(yI, P16, saved + SL.yI, n, FO);
        rows_from_global(preI, P16, saved + SL.preI, n, FO);
        rows_from_global(gin, P16, saved + SL.gin, n, FO);
        rows_from_global(G1, PH, saved + SL.G1, n, FH * nh);
        rows_from_global(preG, P16, saved + SL.preG, n, FO);
        rows_from_global(gout, P16, saved + SL.gout, n, FO);
        for (int h = 0; h < nh; ++h) {
          rows_from_global(sm + L.WhIs + h * NP * P72, P72, saved + (SL.Whi[0] + h * SLH), n, FH);
          rows_from_global(sm + L.stIs + h * 2 * NP, 0, saved + (SL.sti[0] + h * SLH), 1, 2 * NP);
          rows_from_global(sm + L.WhGs + h * NP * P72, P72, saved + (SL.Whg[0] + h * SLH), n, FH);
          rows_from_global(sm + L.stGs + h * 2 * NP, 0, saved + (SL.stg[0] + h * SLH), 1, 2 * NP);
        }
        rows_from_global(sm + L.WhIOs, P16, saved + SL.Whio, n, FO);
        rows_from_global(sm + L.stIOs, 0, saved + SL.stio, 1, 2 * NP);
        rows_from_global(sm + L.WhGOs, P16, saved + SL.Whgo, n, FO);
        rows_from_global(sm + L.stGOs, 0, saved + SL.stgo, 1, 2 * NP);
      }
      if (!dy_pairs) {
        for (int e = tid; e < n * FE; e += blockDim.x) {
          const int i = e / FE, k = e - i * FE;
          float v = dyg[(size_t)i * p.lddy + k];
          for (int c = 1; c < ncp; ++c) v += dyg[(size_t)c * p.dy_cstride + (size_t)i * p.lddy + k];
          Wh[i * PDY + k] = v;   // dy (see below)
        }
      }
    } else if (!(BWD && saved)) {
      // group structure (models.py:263-278) in ONE wave, lane = ped (n <= 64),
      // from the labels in global memory (no barrier after the X stores): a
      // ped's group is every ped with its non-zero label (a zero label: itself
      // alone), led by its lowest member; groups are ranked by their leaders,
      // as the reference's unique rows.  Each lane builds its own member mask
      // over the n labels (broadcast by readlane, no dependence between the
      // steps) -- the former walk over the groups was a serial chain of
      // ballots, ~1.5 us of the forward's first phase
      if (tid < 64) {
        const int i = tid;
        const bool in = i < n;
        const float li = !in ? 0.f : first ? lp : q.labels[o + i];
        if (in) lab[i] = li;
        unsigned long long same = 0ull;
        for (int j = 0; j < n; ++j) {   // (n: uniform)
          const float lj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(li), j));
          if (lj == li) same |= 1ull << j;
        }
        if (li == 0.f || !in) same = 1ull << i;
        same |= 1ull << i;   // (a label that equals nothing, e.g. NaN: itself alone)
        const int g = __ffsll((long long)same) - 1;   // the leader (in lanes: same has bit i)
        const unsigned long long leaders = __ballot(in && g == i);
        const int r = __popcll(leaders & ((1ull << g) - 1ull));
        const int c = __popcll(same);
        if (in) {
          gidl[i] = g;
          grank[i] = r;
          ginv[i] = 1.f / (float)c;
          if (g == i) {
            cnt[r] = c;
            gm[r] = same;
          }
        }
        if (i == 0) *Mp = __popcll(leaders);
      }
    }
    lds_barrier(); PMARK(1); PMARK(2);
    const int M = *Mp;

    if (!BWD || !saved) {
      // ---- intra GAT: heads (40 -> 72, ELU), out (72 nh -> 16, ELU, log_softmax)
      for (int h = 0; h < nh; ++h) {   // per-head offsets are strides (no indexed arrays)
        lin<BWD ? 1 : 4>(X, P40, n, FI, (lw.Wi[0] + h * SEGI), PW72, FH, Wh, P72, 0, (lw.ai[0] + h * SEGI), sp, tp, NP);
        lds_barrier(); PMARK(3);
        att_rows(n, kScoreTiles, sp, tp, NP, gidl, p.alpha, s, t, attm, NPP, saved ? saved + (SL.sti[0] + h * SLH) : nullptr);
        if (saved) rows_to_global(saved + (SL.Whi[0] + h * SLH), Wh, P72, n, FH);
        lds_barrier(); PMARK(4);
        att_agg(attm, NPP, n, Wh, P72, FH, 1, H1 + h * FH, PH, nullptr, 0);
        lds_barrier(); PMARK(5);
      }
      lin<BWD ? 1 : 4>(H1, PH, n, FH * nh, lw.Wio, PW16, FO, Wh, P72, 0, lw.aio, sp, tp, NP);
      lds_barrier(); PMARK(6);
      att_rows(n, 1, sp, tp, NP, gidl, p.alpha, s, t, attm, NPP, saved ? saved + SL.stio : nullptr);
      if (saved) rows_to_global(saved + SL.Whio, Wh, P72, n, FO);
      lds_barrier(); PMARK(7);
      att_agg(attm, NPP, n, Wh, P72, FO, 2, yI, P16, preI, P16);
      lds_barrier(); PMARK(8);
      // ---- group mean (R intra): members in ascending ped order ---------
      for (int e = tid; e < M * FO; e += blockDim.x) {
        const int g = e / FO, f = e - g * FO;
        unsigned long long mk = gm[g];
        float acc = 0.f;
        while (mk) {
          const int i = __ffsll((long long)mk) - 1;
          mk &= mk - 1;
          acc = fmaf(ginv[i], yI[i * P16 + f], acc);
        }
        gin[g * P16 + f] = acc;
      }
      lds_barrier(); PMARK(9);
      // ---- inter GAT on the complete graph of the M groups ----------------
      for (int h = 0; h < nh; ++h) {   // per-head offsets are strides (no indexed arrays)
        lin<BWD ? 1 : 4>(gin, P16, M, FO, (lw.Wg[0] + h * SEGG), PW72, FH, Wh, P72, 0, (lw.ag[0] + h * SEGG), sp, tp, NP);
        lds_barrier(); PMARK(10);
        att_rows(M, kScoreTiles, sp, tp, NP, nullptr, p.alpha, s, t, attm, NPP, saved ? saved + (SL.stg[0] + h * SLH) : nullptr);
        if (saved) rows_to_global(saved + (SL.Whg[0] + h * SLH), Wh, P72, M, FH);
        lds_barrier(); PMARK(11);
        att_agg(attm, NPP, M, Wh, P72, FH, 1, G1 + h * FH, PH, nullptr, 0);
        lds_barrier(); PMARK(12);
      }
      lin<BWD ? 1 : 4>(G1, PH, M, FH * nh, lw.Wgo, PW16, FO, Wh, P72, 0, lw.ago, sp, tp, NP);
      lds_barrier(); PMARK(13);
      att_rows(M, 1, sp, tp, NP, nullptr, p.alpha, s, t, attm, NPP, saved ? saved + SL.stgo : nullptr);
      if (saved) rows_to_global(saved + SL.Whgo, Wh, P72, M, FO);
      lds_barrier(); PMARK(14);
      att_agg(attm, NPP, M, Wh, P72, FO, 2, gout, P16, preG, P16);
      lds_barrier(); PMARK(15);
      if (saved) {   // the activations and the group structure for the backward
        rows_to_global(saved + SL.H1, H1, PH, n, FH * nh);
        rows_to_global(saved + SL.yI, yI, P16, n, FO);
        rows_to_global(saved + SL.preI, preI, P16, n, FO);
        rows_to_global(saved + SL.gin, gin, P16, M, FO);
        rows_to_global(saved + SL.G1, G1, PH, M, FH * nh);
        rows_to_global(saved + SL.preG, preG, P16, M, FO);
        rows_to_global(saved + SL.gout, gout, P16, M, FO);
        rows_to_global(saved + SL.ints, lab, 0, 1, ints_floats(NP));
      }
    } else if (compact) {
      // the inter backward's operands (the intra ones come after it)
      rows_from_global(gin, P16, saved + SL.gin, M, FO);
      rows_from_global(G1, PH, saved + SL.G1, M, FH * nh);
      lds_barrier();
    } else if (!preload) {
      // backward with the forward's saved state: no recompute
      rows_from_global(H1, PH, saved + SL.H1, n, FH * nh);
      rows_from_global(yI, P16, saved + SL.yI, n, FO);
      rows_from_global(preI, P16, saved + SL.preI, n, FO);
      rows_from_global(gin, P16, saved + SL.gin, M, FO);
      rows_from_global(G1, PH, saved + SL.G1, M, FH * nh);
      rows_from_global(preG, P16, saved + SL.preG, M, FO);
      rows_from_global(gout, P16, saved + SL.gout, M, FO);
      lds_barrier();
    }   // (preload: everything came with the inputs)

    if (!BWD) {
      // ---- out = Woe [intra, gout[g(i)] / |g(i)|] + boe on the MFMA ------
      // (n x 32) x (32 x 24): A row i = [yI_i | gout_g(i) / |g(i)|]
      const int lane = tid & 63, nw = blockDim.x >> 6, i16 = lane & 15, kq = lane >> 4;
      const int nt = ((n + 15) >> 4) * 2;
      for (int tile = tid >> 6; tile < nt; tile += nw) {
        const int r0 = (tile >> 1) << 4, c0 = (tile & 1) << 4;
        const int ar = min(r0 + i16, n - 1);
        const float* gi = gout + grank[ar] * P16;
        const float sci = ginv[ar];
        const int col = c0 + i16;
        const float* wr = lw.Woe + min(col, FE - 1) * PWE;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 2 * FO; k += 4) {
          const int kk = k + kq;
          const float av = kk < FO ? yI[ar * P16 + kk] : gi[kk - FO] * sci;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wr[kk], acc, 0, 0, 0);
        }
        if (col < FE) {
          const float bc = lw.boe[col];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = r0 + 4 * kq + r;
            if (row < n) q.y[(size_t)(o + row) * q.ldy + col] = acc[r] + bc;
          }
        }
      }
      lds_barrier(); PMARK(16);
      continue;
    }

    // ================= backward ===========================================
    float* dWh = sm + L.dWh;
    float* dH = sm + L.dH;
    float* dI = sm + L.dI;
    float* dG = sm + L.dG;
    float* dpre = sm + L.dpre;
    float* dz = sm + L.dz;
    float* ds = sm + L.ds;
    float* dt = sm + L.dt;
    float* slab = p.slab + (size_t)sc * PL.total;
    // dy rows and the out embedding's input v = [yI | gout_g(i) / |g(i)|] to
    // LDS (the Wh scratch: dy at pitch FE + 1, v after it at pitch 2 FO + 1)
    constexpr int PDY = FE + 1, PV = 2 * FO + 1;
    float* dy = Wh;
    float* v = Wh + NP * PDY;
    {
      if (!preload) {   // (preload: dy came with the inputs)
        const float* dyg = p.dy + (size_t)o * p.lddy;
        const int ncp = p.dy_copies > 1 ? p.dy_copies : 1;
        for (int e = tid; e < n * FE; e += blockDim.x) {
          const int i = e / FE, k = e - i * FE;
          float v = dyg[(size_t)i * p.lddy + k];
          for (int c = 1; c < ncp; ++c) v += dyg[(size_t)c * p.dy_cstride + (size_t)i * p.lddy + k];
          dy[i * PDY + k] = v;
        }
      }
      if (compact) {   // yI / gout straight from the saved state
        const float* yIg = saved + SL.yI;
        const float* goutg = saved + SL.gout;
        for (int e = tid; e < n * 2 * FO; e += blockDim.x) {
          const int i = e / (2 * FO), c = e - i * 2 * FO;
          v[i * PV + c] = c < FO ? yIg[i * FO + c] : goutg[grank[i] * FO + c - FO] * ginv[i];
        }
      } else {
        for (int e = tid; e < n * 2 * FO; e += blockDim.x) {
          const int i = e / (2 * FO), c = e - i * 2 * FO;
          v[i * PV + c] = c < FO ? yI[i * P16 + c] : gout[grank[i] * P16 + c - FO] * ginv[i];
        }
      }
    }
    lds_barrier(); PMARK(17);
    // out embedding: [d intra | d inter] = dy Woe; dWoe = dy^T v; dboe = sum dy
    lin(dy, PDY, n, FE, lw.Woe, PWE, FO, dI, P16, 0);
    lin(dy, PDY, n, FE, lw.Woe + FO, PWE, FO, dpre, P16, 4);   // d inter (scratch)
    wgrad(dy, PDY, n, FE, v, PV, 2 * FO, slab + PL.Woe, 2 * FO, 8);
    for (int k = tid; k < FE; k += blockDim.x) {
      float acc = 0.f;
      for (int i = 0; i < n; ++i) acc += dy[i * PDY + k];
      slab[PL.boe + k] = acc;
    }
    lds_barrier(); PMARK(18);
    // un-pool backward: d gout[g] = sum_{i in g} d inter_i / |g|
    for (int e = tid; e < M * FO; e += blockDim.x) {
      const int g = e / FO, f = e - g * FO;
      unsigned long long mk = gm[g];
      float acc = 0.f;
      while (mk) {
        const int i = __ffsll((long long)mk) - 1;
        mk &= mk - 1;
        acc = fmaf(ginv[i], dpre[i * P16 + f], acc);
      }
      dG[g * P16 + f] = acc;
    }
    lds_barrier(); PMARK(19);
    // ---- inter out layer ----
    if (compact)
      epi_bwd(dG, P16, saved + SL.preG, FO, M, FO, 2);
    else
      epi_bwd(dG, P16, preG, P16, M, FO, 2);
    const float* WhL = Wh;   // the layer's Wh / s / t: the preloaded copies, or the Wh scratch
    int ldL = P72;
    const float *sL = s, *tL = t;
    if (preload) {
      WhL = sm + L.WhGOs;
      ldL = P16;
      sL = sm + L.stGOs;
      tL = sL + NP;
    } else if (saved) {
      rows_from_global(Wh, P72, saved + SL.Whgo, M, FO);
      rows_from_global(s, 0, saved + SL.stgo, 1, M);
      rows_from_global(t, 0, saved + SL.stgo + NP, 1, M);
    } else {
      lin(G1, PH, M, FH * nh, lw.Wgo, PW16, FO, Wh, P72, 0, lw.ago, sp, tp, NP);
      lds_barrier();
      for (int i = tid; i < M; i += blockDim.x) {
        s[i] = score_of(sp, 1, NP, i);
        t[i] = score_of(tp, 1, NP, i);
      }
    }
    lds_barrier(); PMARK(20);
    att_bwd(WhL, ldL, M, FO, nullptr, sL, tL, p.alpha, lw.ago, dG, P16, dWh, P72, ds, dt, attm, dz, NPP, slab + PL.ago);
    wgrad(G1, PH, M, FH * nh, dWh, P72, FO, slab + PL.Wgo, FO, 0);
    lin_t(dWh, P72, M, FO, lw.Wgo, PW16, FH * nh, dH, PH, false, 8);
    lds_barrier(); PMARK(21);
    // ---- inter heads ----
    for (int e = tid; e < M * FO; e += blockDim.x) dG[(e / FO) * P16 + e % FO] = 0.f;   // becomes d gin
    for (int h = 0; h < nh; ++h) {   // per-head offsets are strides (no indexed arrays)
      // ELU backward from the stored output: elu'(x) = 1 (y > 0) | y + 1
      for (int e = tid; e < M * FH; e += blockDim.x) {
        const int r = e / FH, f = e - r * FH;
        const float yv = G1[r * PH + h * FH + f];
        dH[r * PH + h * FH + f] *= yv > 0.f ? 1.f : yv + 1.f;
      }
      const float* WhH = Wh;
      const float *sH = s, *tH = t;
      if (preload) {
        WhH = sm + L.WhGs + h * NP * P72;
        sH = sm + L.stGs + h * 2 * NP;
        tH = sH + NP;
      } else if (saved) {
        rows_from_global(Wh, P72, saved + (SL.Whg[0] + h * SLH), M, FH);
        rows_from_global(s, 0, saved + (SL.stg[0] + h * SLH), 1, M);
        rows_from_global(t, 0, saved + (SL.stg[0] + h * SLH) + NP, 1, M);
      } else {
        lin(gin, P16, M, FO, (lw.Wg[0] + h * SEGG), PW72, FH, Wh, P72, 0, (lw.ag[0] + h * SEGG), sp, tp, NP);
        lds_barrier();
        for (int i = tid; i < M; i += blockDim.x) {
          s[i] = score_of(sp, kScoreTiles, NP, i);
          t[i] = score_of(tp, kScoreTiles, NP, i);
        }
      }
      lds_barrier(); PMARK(22);
      att_bwd(WhH, P72, M, FH, nullptr, sH, tH, p.alpha, (lw.ag[0] + h * SEGG), dH + h * FH, PH, dWh, P72, ds, dt, attm, dz, NPP,
              slab + (PL.ag[0] + h * PLG));
      wgrad(gin, P16, M, FO, dWh, P72, FH, slab + (PL.Wg[0] + h * PLG), FH, 0);
      lin_t(dWh, P72, M, FH, (lw.Wg[0] + h * SEGG), PW72, FO, dG, P16, true, 8);
      lds_barrier(); PMARK(23);
    }
    // group-mean backward: d intra_i += d gin[g(i)] / |g(i)|
    for (int e = tid; e < n * FO; e += blockDim.x) {
      const int i = e / FO, f = e - i * FO;
      dI[i * P16 + f] = fmaf(ginv[i], dG[grank[i] * P16 + f], dI[i * P16 + f]);
    }
    if (compact) {   // the intra backward's operands, over the dead inter ones
      rows_from_global(H1, PH, saved + SL.H1, n, FH * nh);
      for (int e = tid; e < n * FI; e += blockDim.x) {
        const int r = e / FI;
        X[r * P40 + (e - r * FI)] = xval(q, o, e);
      }
    }
    lds_barrier(); PMARK(24);
    // ---- intra out layer ----
    if (compact)
      epi_bwd(dI, P16, saved + SL.preI, FO, n, FO, 2);
    else
      epi_bwd(dI, P16, preI, P16, n, FO, 2);
    WhL = Wh;
    ldL = P72;
    sL = s;
    tL = t;
    if (preload) {
      WhL = sm + L.WhIOs;
      ldL = P16;
      sL = sm + L.stIOs;
      tL = sL + NP;
    } else if (saved) {
      rows_from_global(Wh, P72, saved + SL.Whio, n, FO);
      rows_from_global(s, 0, saved + SL.stio, 1, n);
      rows_from_global(t, 0, saved + SL.stio + NP, 1, n);
    } else {
      lin(H1, PH, n, FH * nh, lw.Wio, PW16, FO, Wh, P72, 0, lw.aio, sp, tp, NP);
      lds_barrier();
      for (int i = tid; i < n; i += blockDim.x) {
        s[i] = score_of(sp, 1, NP, i);
        t[i] = score_of(tp, 1, NP, i);
      }
    }
    lds_barrier(); PMARK(25);
    att_bwd(WhL, ldL, n, FO, gidl, sL, tL, p.alpha, lw.aio, dI, P16, dWh, P72, ds, dt, attm, dz, NPP, slab + PL.aio);
    wgrad(H1, PH, n, FH * nh, dWh, P72, FO, slab + PL.Wio, FO, 0);
    lin_t(dWh, P72, n, FO, lw.Wio, PW16, FH * nh, dH, PH, false, 8);
    lds_barrier(); PMARK(26);
    // ---- intra heads ----
    float* dXo = p.dX + (size_t)o * p.lddx;
    float* dX2o = p.X2 ? p.dX2 + (size_t)o * p.lddx2 : nullptr;
    for (int h = 0; h < nh; ++h) {   // per-head offsets are strides (no indexed arrays)
      for (int e = tid; e < n * FH; e += blockDim.x) {
        const int r = e / FH, f = e - r * FH;
        const float yv = H1[r * PH + h * FH + f];
        dH[r * PH + h * FH + f] *= yv > 0.f ? 1.f : yv + 1.f;
      }
      const float* WhH = Wh;
      const float *sH = s, *tH = t;
      if (preload) {
        WhH = sm + L.WhIs + h * NP * P72;
        sH = sm + L.stIs + h * 2 * NP;
        tH = sH + NP;
      } else if (saved) {
        rows_from_global(Wh, P72, saved + (SL.Whi[0] + h * SLH), n, FH);
        rows_from_global(s, 0, saved + (SL.sti[0] + h * SLH), 1, n);
        rows_from_global(t, 0, saved + (SL.sti[0] + h * SLH) + NP, 1, n);
      } else {
        lin(X, P40, n, FI, (lw.Wi[0] + h * SEGI), PW72, FH, Wh, P72, 0, (lw.ai[0] + h * SEGI), sp, tp, NP);
        lds_barrier();
        for (int i = tid; i < n; i += blockDim.x) {
          s[i] = score_of(sp, kScoreTiles, NP, i);
          t[i] = score_of(tp, kScoreTiles, NP, i);
        }
      }
      lds_barrier(); PMARK(27);
      att_bwd(WhH, P72, n, FH, gidl, sH, tH, p.alpha, (lw.ai[0] + h * SEGI), dH + h * FH, PH, dWh, P72, ds, dt, attm, dz, NPP,
              slab + (PL.ai[0] + h * PLI), BWD ? 30 : 0);
      wgrad(X, P40, n, FI, dWh, P72, FH, slab + (PL.Wi[0] + h * PLI), FH, 0);
      PMARK(35);
      // dX (global) accumulates over heads in a fixed order
      lin_t(dWh, P72, n, FH, (lw.Wi[0] + h * SEGI), PW72, FI, dXo, p.lddx, h > 0, 8, dX2o, p.lddx2, p.kx1);
      PMARK(36);
      __syncthreads();   // dX read-modify-write by the next head: global ordering
      PMARK(28);
    }
  }
  if constexpr (!BWD) {
    // workgroup 0: the staged weight image after the saved blocks of each
    // batch that keeps its state (the backward copies it contiguously)
    if (blockIdx.x == 0) {
      const SLayout SLw = make_slayout(p.np, NH);
      const floatx4* im = reinterpret_cast<const floatx4*>(wbase);
      floatx4* d1 = p.saved ? reinterpret_cast<floatx4*>(p.saved + (size_t)p.S * SLw.total) : nullptr;
      floatx4* d2 = s2.saved ? reinterpret_cast<floatx4*>(s2.saved + (size_t)s2.S * SLw.total) : nullptr;
      for (int e = tid; e < WF4; e += blockDim.x) {
        const floatx4 v = im[e];
        if (d1) d1[e] = v;
        if (d2) d2[e] = v;
      }
    }
  }
}

// out[c] = sum_s slab[s][c] in a fixed order (deterministic): block = 64
// columns x 16 row phases, phase p sums rows p, p + 16, ... with 4 loads in
// flight, then the 16 phase sums in order
__global__ void __launch_bounds__(1024) slab_reduce_kernel(const float* __restrict__ slab, int rows, int cols,
                                                          float* __restrict__ out) {
  __shared__ float part[16][64];
  const int el = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + el;
  float s = 0.f;
  if (c < cols) {
    int r = ph;
    for (; r + 48 < rows; r += 64) {
      const float v0 = slab[(size_t)r * cols + c], v1 = slab[(size_t)(r + 16) * cols + c];
      const float v2 = slab[(size_t)(r + 32) * cols + c], v3 = slab[(size_t)(r + 48) * cols + c];
      s += v0;
      s += v1;
      s += v2;
      s += v3;
    }
    for (; r < rows; r += 16) s += slab[(size_t)r * cols + c];
  }
  part[ph][el] = s;
  __syncthreads();
  if (ph == 0 && c < cols) {
    float v = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) v += part[p][el];
    out[c] = v;
  }
}

}  // namespace

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_gatenc_param_size(int nh) {
  if (nh < 1 || nh > kGatEncMaxHeads) return -1;
  return make_playout(nh).total;
}

extern "C" long long sgg_gatenc_saved_floats(int S, int max_n, int nh) {
  if (S < 0 || max_n < 1 || nh < 1 || nh > kGatEncMaxHeads) return -1;
  // S per-scene blocks, then the weights' LDS image (gatenc_kernel)
  return (long long)S * make_slayout(max_n, nh).total + 4ll * ((weights_floats(nh) + 3) / 4);
}

extern "C" long long sgg_gatenc_lds_bytes(int max_n, int nh, int bwd) {
  if (max_n < 1 || nh < 1 || nh > kGatEncMaxHeads || bwd < 0 || bwd > 2) return -1;
  return 4ll * make_layout(max_n, nh, bwd).total;
}

static int gatenc_check(const char* who, const GatEncArgs* a, int bwd) {
  SGG_CHECK_ARG(a, "%s: null args", who);
  SGG_CHECK_ARG(a->X && a->labels && a->scene_off, "%s: null input", who);
  SGG_CHECK_ARG(a->nh >= 1 && a->nh <= kGatEncMaxHeads, "%s: heads %d outside [1, %d]", who, a->nh, kGatEncMaxHeads);
  SGG_CHECK_ARG(a->np >= 1 && a->np <= 64, "%s: max scene size %d outside [1, 64]", who, a->np);
  SGG_CHECK_ARG(a->S >= 0 && a->ldx >= (a->X2 ? a->kx1 : FI), "%s: bad sizes", who);
  if (a->X2) {
    SGG_CHECK_ARG(a->kx1 > 0 && a->kx1 < FI && a->ldx2 >= FI - a->kx1, "%s: bad split input (kx1 %d)", who, a->kx1);
    if (bwd)
      SGG_CHECK_ARG(a->dX2 && a->lddx2 >= FI - a->kx1 && a->lddx >= a->kx1, "%s: null / bad split gradient", who);
  }
  for (int h = 0; h < a->nh; ++h)
    SGG_CHECK_ARG(a->w.Wi[h] && a->w.ai[h] && a->w.Wg[h] && a->w.ag[h], "%s: null head weight %d", who, h);
  SGG_CHECK_ARG(a->w.Wio && a->w.aio && a->w.Wgo && a->w.ago && a->w.Woe && a->w.boe, "%s: null weight", who);
  if (bwd) {
    SGG_CHECK_ARG(a->dy && a->dX && a->slab && a->lddy >= FE && a->lddx >= (a->X2 ? a->kx1 : FI),
                  "%s: null / bad gradient buffer", who);
  } else {
    SGG_CHECK_ARG(a->y && a->ldy >= FE, "%s: null / bad output", who);
  }
  const long long lds = sgg_gatenc_lds_bytes(a->np, a->nh, bwd);
  SGG_CHECK_ARG(lds <= 160 * 1024, "%s: %d peds x %d heads need %lld B of LDS (> 160 KiB)", who, a->np, a->nh, lds);
  if (bwd)
    SGG_CHECK_ARG(a->saved || sgg_gatenc_lds_bytes(a->np, a->nh, 2) <= 160 * 1024,
                  "%s: %d peds x %d heads: the backward fits the LDS only with the forward's saved state", who, a->np,
                  a->nh);
  return 0;
}

extern "C" int sgg_gatenc_fwd(const GatEncArgs* args, void* stream) {
  const int rc = gatenc_check("sgg_gatenc_fwd", args, 0);
  if (rc) return rc;
  if (args->S == 0) return 0;
  const size_t lds = (size_t)sgg_gatenc_lds_bytes(args->np, args->nh, 0);
  const dim3 grid(args->S < kGridCap ? args->S : kGridCap);
  const StageTab tab = make_stage_tab(args->w, args->nh);
  const hipStream_t st = (hipStream_t)stream;
  const GatEncSet none = {};
  switch (args->nh) {
    case 1: hipLaunchKernelGGL((gatenc_kernel<false, 1>), grid, dim3(kFwdThreads), lds, st, *args, tab, none); break;
    case 2: hipLaunchKernelGGL((gatenc_kernel<false, 2>), grid, dim3(kFwdThreads), lds, st, *args, tab, none); break;
    case 3: hipLaunchKernelGGL((gatenc_kernel<false, 3>), grid, dim3(kFwdThreads), lds, st, *args, tab, none); break;
    default: hipLaunchKernelGGL((gatenc_kernel<false, 4>), grid, dim3(kFwdThreads), lds, st, *args, tab, none); break;
  }
  SGG_RETURN_LAUNCH("sgg_gatenc_fwd");
}

extern "C" int sgg_gatenc_fwd2(const GatEncArgs* a, const GatEncArgs* b, void* stream) {
  if (int rc = gatenc_check("sgg_gatenc_fwd2 (a)", a, 0)) return rc;
  if (int rc = gatenc_check("sgg_gatenc_fwd2 (b)", b, 0)) return rc;
  SGG_CHECK_ARG(a->nh == b->nh && a->np == b->np && a->alpha == b->alpha &&
                    memcmp(&a->w, &b->w, sizeof(a->w)) == 0,
                "sgg_gatenc_fwd2: the two batches must share the weights, heads, alpha and np (np %d / %d)", a->np,
                b->np);
  const int S = a->S + b->S;
  if (S == 0) return 0;
  const size_t lds = (size_t)sgg_gatenc_lds_bytes(a->np, a->nh, 0);
  const dim3 grid(S < kGridCap ? S : kGridCap);
  const StageTab tab = make_stage_tab(a->w, a->nh);
  const hipStream_t st = (hipStream_t)stream;
  const GatEncSet s2 = {b->X, b->X2, b->labels, b->scene_off, b->y, b->saved, b->ldx, b->ldx2, b->kx1, b->S, b->ldy};
  switch (a->nh) {
    case 1: hipLaunchKernelGGL((gatenc_kernel<false, 1>), grid, dim3(kFwdThreads), lds, st, *a, tab, s2); break;
    case 2: hipLaunchKernelGGL((gatenc_kernel<false, 2>), grid, dim3(kFwdThreads), lds, st, *a, tab, s2); break;
    case 3: hipLaunchKernelGGL((gatenc_kernel<false, 3>), grid, dim3(kFwdThreads), lds, st, *a, tab, s2); break;
    default: hipLaunchKernelGGL((gatenc_kernel<false, 4>), grid, dim3(kFwdThreads), lds, st, *a, tab, s2); break;
  }
  SGG_RETURN_LAUNCH("sgg_gatenc_fwd2");
}

extern "C" int sgg_gatenc_bwd(const GatEncArgs* args, void* stream) {
  const int rc = gatenc_check("sgg_gatenc_bwd", args, 1);
  if (rc) return rc;
  if (args->S == 0) return 0;
  const size_t lds = (size_t)sgg_gatenc_lds_bytes(args->np, args->nh, 1);
  const dim3 grid(args->S < kGridCap ? args->S : kGridCap);
  const StageTab tab = make_stage_tab(args->w, args->nh);
  const hipStream_t st = (hipStream_t)stream;
  const GatEncSet none = {};
  switch (args->nh) {
    case 1: hipLaunchKernelGGL((gatenc_kernel<true, 1>), grid, dim3(kBwdThreads), lds, st, *args, tab, none); break;
    case 2: hipLaunchKernelGGL((gatenc_kernel<true, 2>), grid, dim3(kBwdThreads), lds, st, *args, tab, none); break;
    case 3: hipLaunchKernelGGL((gatenc_kernel<true, 3>), grid, dim3(kBwdThreads), lds, st, *args, tab, none); break;
    default: hipLaunchKernelGGL((gatenc_kernel<true, 4>), grid, dim3(kBwdThreads), lds, st, *args, tab, none); break;
  }
  SGG_RETURN_LAUNCH("sgg_gatenc_bwd");
}

extern "C" int sgg_slab_reduce(const float* slab, int rows, int cols, float* out, void* stream) {
  SGG_CHECK_ARG(slab && out, "sgg_slab_reduce: null pointer");
  SGG_CHECK_ARG(rows >= 0 && cols >= 0, "sgg_slab_reduce: bad sizes");
  if (cols == 0) return 0;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((cols + 63) / 64), dim3(1024), 0, (hipStream_t)stream, slab, rows, cols,
                     out);
  SGG_RETURN_LAUNCH("sgg_slab_reduce");
}
