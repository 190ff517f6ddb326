// Weight-gradient finish of a backward pass in TWO launches (sgg_grad_finish,
// include/sgg.h): the slab row sums (SggRed) of every backward op -- the
// pooling backward (reference sgan/models.py:497-549), the LSTM backward
// (:62-92, :142-178), the discriminator head, the GAT encoder / GCN module
// slabs -- then the input-embedding fold backwards (SggFoldBwd) of all of
// them, one workgroup each.  (sgan.kernels defers the ops' finishes to the
// end of the backward pass inside the training step and issues them here
// together.)
//
// Before, the row sums took a sgg_slab_reduce and sgg_xtw's reduce pass per
// op, launches of a few microseconds of work each behind the fixed per-
// dispatch cost.  A fold job needs (dA, dbias), which are row sums of the
// same slabs: two more row-sum jobs write them to a scratch buffer and the
// fold backward (fold.hip) follows as the op's one other launch.  (Running
// the folds in the same launch needs a grid-wide handoff: a device-scope
// release fence per workgroup writes back the XCD's L2 and measured 5x
// slower than the second launch; a single workgroup re-summing the slabs
// reads up to 1.5 MB through one CU.)  Every sum keeps the order of the
// reductions it replaces, so the outputs are bit-identical to the separate
// launches.
//
// Row-sum order (shared with slab_reduce_kernel / xtw_reduce_kernel): column
// c's 16 phases p each add rows p, p + 16, p + 32, ... in row order starting
// from 0, then the 16 phase sums are added in phase order.
#include <string.h>

#include "sgg_common.h"

namespace sgg {

namespace {

constexpr int kRedJobs = SGG_RED_MAX + 2 * SGG_FOLDB_MAX;   // + each fold's (dA, dbias) row sums

struct FinishArgs {
  SggRed red[kRedJobs];
  unsigned char vec[kRedJobs];   // job j read as float4 columns (16-byte aligned rows and first column)
  int nred;
  int blk0[kRedJobs + 1];   // first workgroup of red job j (after the loss workgroup, if any); blk0[nred]: end
  SggL2Job l2[SGG_LOSSJOB_MAX];
  SggBceJob bce[SGG_LOSSJOB_MAX];
  int nl2, nbce;
};

__device__ __forceinline__ float phase_sum(const float* __restrict__ src, int rows, int ld, int col, int ph) {
  float s = 0.f;
  int r = ph;
  for (; r + 48 < rows; r += 64) {
    const float v0 = src[(size_t)r * ld + col], v1 = src[(size_t)(r + 16) * ld + col];
    const float v2 = src[(size_t)(r + 32) * ld + col], v3 = src[(size_t)(r + 48) * ld + col];
    s += v0;
    s += v1;
    s += v2;
    s += v3;
  }
  for (; r < rows; r += 16) s += src[(size_t)r * ld + col];
  return s;
}

// the same phase sums over four adjacent columns (one 16-byte load per row)
__device__ __forceinline__ floatx4 phase_sum4(const float* __restrict__ src, int rows, int ld, int col, int ph) {
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  int r = ph;
  for (; r + 48 < rows; r += 64) {
    const floatx4 v0 = *reinterpret_cast<const floatx4*>(src + (size_t)r * ld + col);
    const floatx4 v1 = *reinterpret_cast<const floatx4*>(src + (size_t)(r + 16) * ld + col);
    const floatx4 v2 = *reinterpret_cast<const floatx4*>(src + (size_t)(r + 32) * ld + col);
    const floatx4 v3 = *reinterpret_cast<const floatx4*>(src + (size_t)(r + 48) * ld + col);
    s += v0;
    s += v1;
    s += v2;
    s += v3;
  }
  for (; r < rows; r += 16) s += *reinterpret_cast<const floatx4*>(src + (size_t)r * ld + col);
  return s;
}

__device__ __forceinline__ void red_store(const SggRed& d, int c, float v) {
  if (d.map == 0) {
    d.out[c] = v;
  } else {
    const int m = c / d.N, n = c - m * d.N;
    d.out[d.trans ? (size_t)n * d.ldo + m : (size_t)m * d.ldo + n] = v;
  }
}

// a workgroup of 1024 threads = 16 row phases x 64 lanes: 64 columns per
// workgroup, or 256 when the job's rows are read as float4 (vec) -- a quarter
// of the workgroups and of the load instructions for the same bytes, and the
// same per-column order of additions (bit-identical)
__device__ void red_job(const SggRed& d, bool vec, int blk, float (*rpart)[256]) {
  const int el = threadIdx.x & 63, ph = threadIdx.x >> 6;
  if (vec) {
    const int c = blk * 256 + 4 * el;
    const floatx4 s = c < d.cols ? phase_sum4(d.src + d.col0, d.rows, d.ld, c, ph) : floatx4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<floatx4*>(&rpart[ph][4 * el]) = s;
    __syncthreads();
    if (ph == 0 && c < d.cols) {
      floatx4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 16; ++p) v += *reinterpret_cast<const floatx4*>(&rpart[p][4 * el]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (c + i < d.cols) red_store(d, c + i, v[i]);
    }
    return;
  }
  const int c = blk * 64 + el;
  const float s = c < d.cols ? phase_sum(d.src + d.col0, d.rows, d.ld, c, ph) : 0.f;
  rpart[ph][el] = s;
  __syncthreads();
  if (ph == 0 && c < d.cols) {
    float v = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) v += rpart[p][el];
    red_store(d, c, v);
  }
}

// ---- the loss values' workgroup (sgg_grad_finish_losses) -------------------
constexpr int kLossThreads = 1024;

// *loss = the scene terms summed in scene order by lane-strided partials and a
// shuffle tree (l2_sum_kernel's form); the value is also left in *lv (LDS)
// for a BCE job's addend
__device__ void l2_value(const SggL2Job& d, float* lv) {
  if (threadIdx.x < 64) {
    float a = 0.f;
    for (int s = threadIdx.x; s < d.S; s += 64) a += d.term[s];
    a = wave_sum(a);
    if (threadIdx.x == 0) {
      *d.loss = a;
      *lv = a;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float bce_term(float x, float y) {   // as loss.hip
  return fmaxf(x, 0.f) - x * y + logf(1.f + expf(-fabsf(x)));
}

// a BCE job's inputs, loaded before the L2 jobs run (one round trip for all)
struct BceIn {
  float v[8], a, b;
  int nv;
};
__device__ __forceinline__ void bce_load(const SggBceJob& d, BceIn& in) {
  in.a = *d.ya;
  in.b = *d.yb;
  in.nv = d.nvalid ? *d.nvalid : d.n;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int i = threadIdx.x + kLossThreads * m;
    in.v[m] = i < d.n ? d.x[i] : 0.f;
  }
}

// *loss = w (mean_{i < split} f(x_i, ya) + mean_{i >= split} f(x_i, yb)) over
// the first nvalid scores of each half; *total = *loss + addend (addend: an
// L2 job's value from LDS when it is that job's loss, else *d.addend)
__device__ void bce_value(const SggBceJob& d, const BceIn& in, float addend, float (*red)[kLossThreads / 64]) {
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int i = threadIdx.x + kLossThreads * m;
    const bool live = i < d.split ? i < in.nv : i - d.split < in.nv;
    if (i < d.n && live) {
      if (i < d.split) s0 += bce_term(in.v[m], in.a);
      else s1 += bce_term(in.v[m], in.b);
    }
  }
  for (int i = threadIdx.x + 8 * kLossThreads; i < d.n; i += kLossThreads) {   // past the prefetched scores
    const bool live = i < d.split ? i < in.nv : i - d.split < in.nv;
    if (live) {
      if (i < d.split) s0 += bce_term(d.x[i], in.a);
      else s1 += bce_term(d.x[i], in.b);
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = s0;
    red[1][wave] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t0 = 0.f, t1 = 0.f;
#pragma unroll
    for (int w = 0; w < kLossThreads / 64; ++w) {
      t0 += red[0][w];
      t1 += red[1][w];
    }
    const int c0 = min(d.split, in.nv), c1 = min(d.n - d.split, in.nv);
    const float m0 = c0 > 0 ? t0 / (float)c0 : 0.f;
    const float m1 = c1 > 0 ? t1 / (float)c1 : 0.f;
    const float l = d.w * (m0 + m1);
    *d.loss = l;
    if (d.total) *d.total = l + addend;
  }
  __syncthreads();
}

__device__ void loss_workgroup(const FinishArgs& a, float (*rpart)[256]) {
  __shared__ float lv[SGG_LOSSJOB_MAX];
  BceIn in[SGG_LOSSJOB_MAX];
#pragma unroll
  for (int j = 0; j < SGG_LOSSJOB_MAX; ++j)
    if (j < a.nbce) bce_load(a.bce[j], in[j]);
  // an addend that is not an L2 job's value: read with the inputs
  float ad[SGG_LOSSJOB_MAX];
#pragma unroll
  for (int j = 0; j < SGG_LOSSJOB_MAX; ++j) {
    ad[j] = 0.f;
    if (j < a.nbce && a.bce[j].total) {
      bool fromL2 = false;
      for (int k = 0; k < a.nl2; ++k) fromL2 |= a.bce[j].addend == a.l2[k].loss;
      if (!fromL2) ad[j] = *a.bce[j].addend;
    }
  }
  for (int k = 0; k < a.nl2; ++k) l2_value(a.l2[k], lv + k);
#pragma unroll
  for (int j = 0; j < SGG_LOSSJOB_MAX; ++j)
    if (j < a.nbce) {
      float addend = ad[j];
      for (int k = 0; k < a.nl2; ++k)
        if (a.bce[j].total && a.bce[j].addend == a.l2[k].loss) addend = lv[k];
      bce_value(a.bce[j], in[j], addend, reinterpret_cast<float(*)[kLossThreads / 64]>(&rpart[0][0]));
    }
}

// workgroups = (with loss jobs) the loss workgroup, then the red jobs' 64-column
// blocks (1024 threads: 64 columns x 16 row phases)
__global__ void __launch_bounds__(1024) grad_finish_kernel(FinishArgs a) {
  __shared__ __attribute__((aligned(16))) float rpart[16][256];
  const int lw = a.nl2 + a.nbce > 0;   // (the loss workgroup is block 0: dispatched first, beside the row sums)
  const int b = (int)blockIdx.x - lw;
  if (b < 0) {   // the loss values: every L2 job, then every BCE job (an addend may be an L2 loss)
    loss_workgroup(a, rpart);
    return;
  }
  int j = 0;
  while (j + 1 < a.nred && b >= a.blk0[j + 1]) ++j;
  red_job(a.red[j], a.vec[j] != 0, b - a.blk0[j], rpart);
}

}  // namespace

}  // namespace sgg

using namespace sgg;

extern "C" int sgg_grad_finish(const SggRed* reds, int nred, const SggFoldBwd* folds, int nfold, float* scratch,
                               size_t scratch_bytes, void* stream) {
  return sgg_grad_finish_losses(reds, nred, folds, nfold, scratch, scratch_bytes, nullptr, 0, nullptr, 0, stream);
}

extern "C" int sgg_grad_finish_losses(const SggRed* reds, int nred, const SggFoldBwd* folds, int nfold,
                                      float* scratch, size_t scratch_bytes, const SggL2Job* l2, int nl2,
                                      const SggBceJob* bce, int nbce, void* stream) {
  SGG_CHECK_ARG(nl2 >= 0 && nl2 <= SGG_LOSSJOB_MAX && nbce >= 0 && nbce <= SGG_LOSSJOB_MAX &&
                    (nl2 == 0 || l2) && (nbce == 0 || bce),
                "sgg_grad_finish_losses: 0 <= nl2, nbce <= %d (got %d, %d)", SGG_LOSSJOB_MAX, nl2, nbce);
  for (int j = 0; j < nl2; ++j) {
    const SggL2Job& d = l2[j];
    SGG_CHECK_ARG(d.loss && (d.S == 0 || d.term) && d.S >= 0, "sgg_grad_finish_losses: bad L2 job %d", j);
  }
  for (int j = 0; j < nbce; ++j) {
    const SggBceJob& d = bce[j];
    SGG_CHECK_ARG(d.ya && d.yb && d.loss && (d.n == 0 || d.x) && (!d.total || d.addend),
                  "sgg_grad_finish_losses: null pointer in BCE job %d", j);
    SGG_CHECK_ARG(d.n >= 0 && d.split >= 0 && d.split <= d.n, "sgg_grad_finish_losses: BCE job %d: bad sizes", j);
  }
  SGG_CHECK_ARG(nred >= 0 && nred <= SGG_RED_MAX && nfold >= 0 && nfold <= SGG_FOLDB_MAX,
                "sgg_grad_finish: 0 <= nred <= %d, 0 <= nfold <= %d (got %d, %d)", SGG_RED_MAX, SGG_FOLDB_MAX, nred,
                nfold);
  SGG_CHECK_ARG((nred == 0 || reds) && (nfold == 0 || (folds && scratch)), "sgg_grad_finish: null job list or scratch");
  FinishArgs a;
  memset(&a, 0, sizeof(a));
  int nj = 0;
  auto add_red = [&](const SggRed& d) {
    a.red[nj] = d;
    ++nj;
  };
  for (int j = 0; j < nred; ++j) {
    const SggRed& d = reds[j];
    SGG_CHECK_ARG(d.src && d.out && d.rows >= 0 && d.cols >= 1 && d.col0 >= 0 && d.ld >= d.col0 + d.cols,
                  "sgg_grad_finish: bad reduction job %d (rows %d ld %d col0 %d cols %d)", j, d.rows, d.ld, d.col0,
                  d.cols);
    SGG_CHECK_ARG(d.map == 0 || (d.map == 1 && d.N >= 1 && d.cols % d.N == 0 &&
                                 d.ldo >= (d.trans ? d.cols / d.N : d.N)),
                  "sgg_grad_finish: bad output map of reduction job %d", j);
    add_red(d);
  }
  size_t need = 0;
  for (int k = 0; k < nfold; ++k) need += sizeof(float) * 3 * (size_t)folds[k].R;
  SGG_CHECK_ARG(scratch_bytes >= need, "sgg_grad_finish: scratch %zu < %zu bytes", scratch_bytes, need);
  float* g = scratch;
  for (int k = 0; k < nfold; ++k) {
    const SggFoldBwd& d = folds[k];
    SGG_CHECK_ARG(d.W && d.We && d.be && d.dA_src && d.db_src && d.dW && d.dWe && d.dbe,
                  "sgg_grad_finish: null pointer in fold job %d", k);
    SGG_CHECK_ARG(d.R >= 1 && d.R <= 512 && d.E >= 1 && d.E <= 128 && d.ldw >= d.E && d.lddw >= d.E,
                  "sgg_grad_finish: bad fold sizes in job %d (R %d E %d)", k, d.R, d.E);
    SGG_CHECK_ARG(d.dA_rows >= 0 && d.db_rows >= 0 && d.dA_col0 >= 0 && d.db_col0 >= 0 &&
                      d.dA_ld >= d.dA_col0 + 2 * d.R && d.db_ld >= d.db_col0 + d.R,
                  "sgg_grad_finish: bad (dA, dbias) sources in fold job %d", k);
    add_red(SggRed{d.dA_src, d.dA_rows, d.dA_ld, d.dA_col0, 2 * d.R, g, 0, 0, 0, 0});
    add_red(SggRed{d.db_src, d.db_rows, d.db_ld, d.db_col0, d.R, g + 2 * d.R, 0, 0, 0, 0});
    g += 3 * (size_t)d.R;
  }
  a.nred = nj;
  int blk = 0;
  for (int j = 0; j < nj; ++j) {
    const SggRed& d = a.red[j];
    a.vec[j] = d.ld % 4 == 0 && d.col0 % 4 == 0 && (reinterpret_cast<uintptr_t>(d.src) & 15) == 0;
    a.blk0[j] = blk;
    blk += a.vec[j] ? (d.cols + 255) / 256 : (d.cols + 63) / 64;
  }
  a.blk0[nj] = blk;
  for (int j = 0; j < nl2; ++j) a.l2[j] = l2[j];
  for (int j = 0; j < nbce; ++j) a.bce[j] = bce[j];
  a.nl2 = nl2;
  a.nbce = nbce;
  if (nl2 + nbce > 0) ++blk;   // the loss workgroup
  hipStream_t st = (hipStream_t)stream;
  if (blk > 0) hipLaunchKernelGGL(grad_finish_kernel, dim3(blk), dim3(1024), 0, st, a);
  if (nfold > 0) {   // the fold backwards on the summed (dA, dbias), one workgroup each
    SggFoldBwd f[SGG_FOLDB_MAX];
    g = scratch;
    for (int k = 0; k < nfold; ++k) {
      f[k] = folds[k];
      f[k].dA_src = g;              // (the row-sum launch's outputs: dA, then dbias)
      f[k].db_src = g + 2 * folds[k].R;
      g += 3 * (size_t)folds[k].R;
    }
    fold_bwd_multi(f, nfold, st);
  }
  SGG_RETURN_LAUNCH("sgg_grad_finish");
}
