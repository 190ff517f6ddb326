/*
 * sgg.h -- C ABI of libsgg.so, the MI355X (gfx950) kernels behind the
 * group-aware Social-GAN hot path (reference: peaceminusones/Group-GAN-GCN-GAT).
 *
 * The reference has no native boundary: its "operator API" is the PyTorch
 * module code in sgan/models.py.  Each entry point below replaces a sequence
 * of ATen ops inside one of those modules; the replaced reference lines are
 * cited per function (paths relative to the reference root).
 *
 * Conventions (every function):
 *   - all pointers are DEVICE pointers owned by the caller (the library never
 *     allocates); fp32 tensors are row-major and contiguous unless an explicit
 *     leading dimension is given;
 *   - scenes / segments are CSR ranges: `off[k] .. off[k+1]` (int32, off[0] = 0);
 *   - launches go on `stream` (a hipStream_t passed as void*); nothing blocks,
 *     nothing synchronises, so every call is hipGraph-capturable;
 *   - return 0 on success, SGG_E_ARG (-1) for a bad argument (nothing
 *     launched), or a positive hipError_t from the launch.  sgg_last_error()
 *     describes the last failure of the calling thread.
 */
#ifndef SGG_H
#define SGG_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGG_E_ARG (-1)

/* Library version / self description.  sgg_source_hash(): SHA-256 (hex) of
 * the kernel sources (csrc: .hip and .h files) and this header the library was built from
 * (build_native.py); the Python loader refuses a library whose hash differs
 * from the tree it runs in. */
int sgg_version(void);
const char* sgg_last_error(void);
const char* sgg_source_hash(void);

/* Upper bounds the kernels are built for (checked on every call). */
#define SGG_POOL_MAX_PEDS 64   /* peds per scene held LDS-resident by the pooling kernel      */
#define SGG_GAT_MAX_NODES 128  /* nodes per segment held LDS-resident by the attention kernel */

/* ------------------------------------------------------------------------
 * Dense node-feature transform on MFMA (v_mfma_f32_16x16x4_f32, exact fp32):
 *   Y[m, n] = act( sum_k X[m, k] * Wop[k, n] + bias[n] )
 * Wop = W (K x N row-major) when trans_w = 0, or W^T for a W stored N x K when
 * trans_w = 1.  act: bit 0 ReLU; bit 1 accumulate, Y = act(..) + Y (the
 * pooling backward adds its dh into the GAT encoder's input gradient in
 * place of an autograd sum).  bias may be NULL.  ldx / ldw / ldy are
 * the row strides of X, W (as stored) and Y (elements); a column block of a
 * wider weight (the h-half W1[:, E:] of the pooling layer) is passed in place.
 * Replaces the per-node `torch.mm(h, W)` / nn.Linear calls of
 * models.py:199 (GAT Wh = hW), :576 ((AH)W of the GCN), :289 / :706
 * (out_embedding), and the h_j half of the pooling MLP's first layer :538.
 * Xmask (may be NULL, row stride ldm): X[m, k] enters only where
 * Xmask[m, k] > 0 -- the ReLU backward dY * (Y > 0) of a transform with a
 * fused ReLU, without materialising the masked gradient.
 */
int sgg_xw(const float* X, int ldx, const float* Xmask, int ldm, const float* W, int ldw, int trans_w,
           const float* bias, float* Y, int ldy, int M, int K, int N, int act, void* stream);

/* The same transform with X and W rounded to bf16 (round-to-nearest-even) on
 * v_mfma_f32_16x16x32_bf16, fp32 accumulation and output: the opt-in "bf16 +
 * MFMA XW" precision of BASELINE configs 3 and 5 (sgan.kernels.set_precision). */
int sgg_xw_bf16(const float* X, int ldx, const float* Xmask, int ldm, const float* W, int ldw, int trans_w,
                const float* bias, float* Y, int ldy, int M, int K, int N, int act, void* stream);

/* ------------------------------------------------------------------------
 * Social pooling (PoolHiddenNet.forward, models.py:497-549), factored:
 *   hidden(i,j,k) = ReLU( U[j,k] + A[k,0]*(p_j - p_i)_x + A[k,1]*(p_j - p_i)_y )
 *   out[i,c]      = max_j ReLU( sum_k W2[c,k] * hidden(i,j,k) + b2[c] )
 * where U = h W1h^T + (W1e be + b1) (one sgg_xw) and A = W1e We, i.e. the
 * reference's Linear(2,E) -> cat[., h_j] -> Linear(E+H,512) with the
 * embedding folded into the first layer.  The (N^2 x 512) pair tensor is
 * never materialised; the 512 -> bn layer runs on fp32 MFMA.  argmax[i,c]
 * receives the GLOBAL ped index j that attains the max (smallest j on ties)
 * for the backward.
 *   U: B x 512, pos: B x 2, A: 512 x 2, W2: bn x 512 (nn.Linear layout), b2: bn
 *   out: B x bn, argmax: B x bn (int32).  bn in {8, 16, 32, 48, 64}.
 *   max_n = largest scene size in the batch (<= SGG_POOL_MAX_PEDS).
 * Work is split into chunks of whole i-rows of one scene; the chunk table
 * (int32 x 4 per chunk: scene, i0, i1, gpw) is built on the HOST by
 * sgg_pool_plan from the host copy of scene_off and copied to the device by
 * the caller (once per batch).  sgg_pool_plan returns the number of chunks
 * (<= cap) or SGG_E_ARG, the largest chunk height in *max_rows and the
 * 16-pair groups per wave in *gpw (1, 2, 4 or 8: the widest that still gives
 * >= target_chunks workgroups, capped by max_gpw when > 0; ~2-4x the CU
 * count keeps small batches busy).
 * Pass max_rows and gpw unchanged to sgg_pool_fwd.  A chunk with i1 <= i0 is
 * skipped.  nchunks_dev (optional, one device int32): the number of chunks
 * the workgroups walk (grid-stride) is read on the device, while nchunks
 * sizes the grid and picks the kernel form -- a fixed-capacity plan whose
 * chunk count varies between graph replays (sgan.scene.PaddedScenes).
 */
int sgg_pool_plan(const int32_t* host_scene_off, int S, int bn, int target_chunks, int max_gpw,
                  int32_t* host_chunks, int cap, int* max_rows, int* gpw);
int sgg_pool_fwd(const float* U, const float* pos, const float* A, const float* W2,
                 const float* b2, const int32_t* scene_off, const int32_t* chunks, int nchunks,
                 int max_rows, int gpw, int B, int bn, int max_n, float* out, int32_t* argmax,
                 const int32_t* nchunks_dev, void* stream);

/* sgg_pool_fwd in the opt-in bf16 precision (BASELINE configs 3 and 5,
 * sgan.kernels.set_precision("bf16")): the same arguments and argmax
 * contract; the 512 -> bn contraction runs on v_mfma_f32_16x16x32_bf16 with
 * the hidden units (formed in fp32, 2 FMA + max) and W2 rounded to bf16
 * (round-to-nearest-even), fp32 accumulation, bias, ReLU and max.  Any chunk
 * table is accepted (a chunk runs in passes of up to 8 x 16 gpw pairs); the
 * efficient one comes from sgg_pool_plan_bf16 (up to 1024 pairs per chunk,
 * >= target_chunks chunks -- one per CU fills the persistent grid).  The
 * backward (sgg_pool_bwd) is the fp32 one at the argmax this forward chose. */
int sgg_pool_plan_bf16(const int32_t* host_scene_off, int S, int bn, int target_chunks, int32_t* host_chunks,
                       int cap, int* max_rows, int* gpw);
int sgg_pool_fwd_bf16(const float* U, const float* pos, const float* A, const float* W2,
                      const float* b2, const int32_t* scene_off, const int32_t* chunks, int nchunks,
                      int max_rows, int gpw, int B, int bn, int max_n, float* out, int32_t* argmax,
                      const int32_t* nchunks_dev, void* stream);

/* Two batches through ONE pooling net in one launch: sgg_pool_fwd (bf16 = 0)
 * or sgg_pool_fwd_bf16 (bf16 != 0) of batch a and of batch b, the same
 * weights (A, W2, b2, bn) -- the discriminator step's generator pooling
 * (scripts/train.py:400, no autograd) and the generator step's (:443) run
 * together (sgan.models.TrajectoryGenerator.context_pair).  Each batch's
 * fields are sgg_pool_fwd's arguments of the same name; both plans must have
 * the same gpw.  The workgroups walk a's chunks, then b's: each output is
 * bitwise what the single-batch call writes. */
typedef struct SggPoolBatch {
  const float* U;
  const float* pos;
  const int32_t* scene_off;
  const int32_t* chunks;
  int nchunks;
  int max_rows;
  int gpw;
  int B;
  int max_n;
  float* out;
  int32_t* argmax;
  const int32_t* nchunks_dev;
} SggPoolBatch;
int sgg_pool_fwd2(const SggPoolBatch* a, const SggPoolBatch* b, const float* A, const float* W2, const float* b2,
                  int bn, int bf16, void* stream);

/* The pooling backward's two products of dU (B x 512, row stride ldu) in ONE
 * launch (models.py:538's Linear: the h half of the first layer): dh = dU W
 * (W = W1[:, E:], 512 x H at row stride ldw; accumulate != 0 adds to dh) and
 * the split-K partials of h^T dU plus the column sums of dU into ws, laid
 * out exactly as sgg_xtw_partial(h, dU, colsum = 1) lays them out
 * (sgg_xtw_splits(B, H, 512) splits; ws >= splits (512 H + 512) floats), for
 * sgg_grad_finish to sum.  H <= 64. */
int sgg_pool_dh_dw(const float* dU, int ldu, const float* W, int ldw, float* dh, int ldh, int accumulate,
                   const float* h, int ldx, int B, int H, float* ws, size_t ws_bytes, void* stream);

/* Backward of sgg_pool_fwd.  Only the (i, argmax[i,c]) pairs carry gradient
 * (torch.max(dim) backward, models.py:541).  Writes dU (B x 512, every row),
 * and one row per workgroup of the parameter-gradient slab `part`
 * (grid x (bn*512 + 1024 + bn), grid = sgg_pool_bwd_grid(S)): the
 * workgroup's partial sums of [dW2 (bn x 512) | dA (512 x 2) | db2 (bn)];
 * sgg_slab_reduce sums the rows (fixed order => deterministic).  part may be
 * NULL (frozen weights, e.g. the G-step's discriminator): dU only.
 * pos gets no gradient (it is an input trajectory in every caller). */
int sgg_pool_bwd_grid(int S);
int sgg_pool_bwd(const float* U, const float* pos, const float* A, const float* W2,
                 const float* out, const int32_t* argmax, const float* dout,
                 const int32_t* scene_off, int S, int B, int bn, int max_n,
                 float* dU, float* part, void* stream);

/* ------------------------------------------------------------------------
 * Graph attention over the nodes of each segment (GraphAttentionLayer,
 * models.py:198-220, and the ELU / log_softmax of GAT.forward :236-237):
 *   s_i = Wh_i . a[:F],  t_j = Wh_j . a[F:]
 *   e_ij = LeakyReLU_alpha(s_i + t_j) on the mask, softmax over j,
 *   hp_i = sum_j att_ij Wh_j
 *   y_i  = epilogue(hp_i): 0 identity, 1 ELU, 2 log_softmax(ELU(.)) over F
 * mask_mode 0: (i == j) or (lab_i == lab_j and lab_i != 0)   (models.py:263-267)
 * mask_mode 1: complete graph                                (models.py:282-283)
 * Multi-head (the batched GAT of the sgangat family, sgan/GAT.py:6-55 text,
 * attention over the complete scene graph = mask_mode 1): Wh is n x heads*F
 * (heads side by side), a is heads x 2F ([a_src | a_dst] per head), head h
 * writes columns [hF, hF + F) of y (the head concat of GAT.py:86), and bias
 * (F, may be NULL) is added to every head's aggregate before the epilogue
 * (GAT.py:41).  heads = 1, bias = NULL is the GraphAttentionLayer above.
 * y is written with row stride ldy (>= heads*F; single-head layers of the
 * group GAT write straight into their concat slot, models.py:234); hp
 * (n x heads*F, pre-epilogue, bias included) is written when epilogue != 0
 * (needed by the backward).  Epilogue 2 requires heads == 1 and ldy == F.
 * Rows [seg_off[nseg], n) (zero-padded group buffers no segment covers)
 * get zero y / hp.  Segments larger than SGG_GAT_MAX_NODES are rejected.
 */
int sgg_gat_fwd(const float* Wh, int heads, const float* a, const float* bias, const float* labels,
                const int32_t* seg_off, int nseg, int n, int F, float alpha, int mask_mode,
                int epilogue, int max_seg, float* hp, float* y, int ldy, void* stream);

/* Backward of sgg_gat_fwd (bias excluded: its gradient is the column sum of
 * the pre-epilogue gradient, formed by the caller).  dy: head h at columns
 * [hF, hF + F) of row stride lddy; y / hp as written by the forward.  Writes
 * dWh (n x heads*F) and ds, dt (n x heads), zero on the rows past the last
 * segment; the caller finishes
 * da_h = [Wh_h^T ds_h ; Wh_h^T dt_h], dX = dWh W^T, dW = X^T dWh. */
int sgg_gat_bwd(const float* Wh, int heads, const float* a, const float* labels, const int32_t* seg_off,
                int nseg, int n, int F, float alpha, int mask_mode, int epilogue, int max_seg,
                const float* hp, const float* y, const float* dy, int lddy,
                float* dWh, float* ds, float* dt, void* stream);

/* sgg_gat_fwd with the attention vectors as the module holds them: a_src
 * and a_dst heads x F each (the batched GAT's (heads, F, 1) parameters,
 * GAT.py:38-39 text) instead of one heads x 2F array -- no concatenation. */
int sgg_gat_fwd_ex(const float* Wh, int heads, const float* a_src, const float* a_dst, const float* bias,
                   const float* labels, const int32_t* seg_off, int nseg, int n, int F, float alpha, int mask_mode,
                   int epilogue, int max_seg, float* hp, float* y, int ldy, void* stream);

/* Backward of sgg_gat_fwd_ex with the parameter gradients finished on the
 * device: dWh (n x heads*F, zero past the last segment), da_src / da_dst
 * (heads x F: Wh_h^T ds_h, Wh_h^T dt_h) and, when dbias != NULL, dbias (F:
 * the column sum over nodes and heads of the pre-epilogue gradient,
 * accumulated in fp64).  Per-(segment, head) partials go to `work` (16-byte
 * aligned, sgg_gat_bwd_ex_work_bytes) and a second launch sums them in a
 * fixed order (deterministic). */
size_t sgg_gat_bwd_ex_work_bytes(int nseg, int heads, int F);
int sgg_gat_bwd_ex(const float* Wh, int heads, const float* a_src, const float* a_dst, const float* labels,
                   const int32_t* seg_off, int nseg, int n, int F, float alpha, int mask_mode, int epilogue,
                   int max_seg, const float* hp, const float* y, const float* dy, int lddy, float* dWh,
                   float* da_src, float* da_dst, float* dbias, void* work, void* stream);

/* One layer of the sgangat family's batched GAT in one launch (GAT.py:71-86
 * text): InstanceNorm1d over each segment's rows (biased variance, eps; the
 * statistics of sgg_seg_norm_fwd), Wh = xn [w_0 | .. | w_{H-1}] with w in
 * the module's (heads, K, F) layout -- fp32, or with bf16 != 0 the operands
 * rounded to bf16 as sgg_xw_bf16 does (fp32 accumulate) -- then the
 * multi-head attention of sgg_gat_fwd_ex on the complete segment graph
 * (epilogue 0 or 1).  The input is one row block x1 (n x K1, stride ld1) or
 * two, [x1 | x2] (x2: n x K2, stride ld2; NULL for one): K = K1 + K2 <= 256.
 * When wh != NULL (training) also writes the backward's operands: xn (n x
 * K, the normalised input), rstd (nseg x K) and wh (n x heads*F) -- with
 * them the backward is sgg_gat_bwd_ex, the transform's products and
 * sgg_seg_norm_bwd.  Rows past the last segment get zeros.  The LDS plan
 * (sgg_gat_layer_lds_bytes(K, F, max_seg)) must fit 160 KiB. */
size_t sgg_gat_layer_lds_bytes(int K, int F, int max_seg);
int sgg_gat_layer_fwd(const float* x1, int ld1, int K1, const float* x2, int ld2, int K2, const float* w,
                      const float* a_src, const float* a_dst, const float* bias, const int32_t* seg_off, int nseg,
                      int n, int heads, int F, float alpha, float eps, int epilogue, int max_seg, int bf16,
                      float* xn, float* rstd, float* wh, float* hp, float* y, int ldy, void* stream);

/* The same layer over TWO batches in one launch (the sgangat generator's two
 * contexts of one training iteration, G.context_pair: the discriminator
 * step's, without saved operands, and the generator step's, with them).  A
 * set is one batch's inputs, segments and outputs, with the fields of
 * sgg_gat_layer_fwd; the weights and layer shape are shared.  Both sets use
 * one LDS plan (the larger max_seg); each set's results are those of its
 * own sgg_gat_layer_fwd launch. */
typedef struct SggGatLayerSet {
  const float* x1;
  int ld1, K1;
  const float* x2;
  int ld2, K2;
  const int32_t* seg_off;
  int nseg, n, max_seg;
  float *xn, *rstd, *wh, *hp, *y;
  int ldy;
} SggGatLayerSet;
int sgg_gat_layer_fwd2(const SggGatLayerSet* a, const SggGatLayerSet* b, const float* w, const float* a_src,
                       const float* a_dst, const float* bias, int heads, int F, float alpha, float eps,
                       int epilogue, int bf16, void* stream);

/* ------------------------------------------------------------------------
 * Instance normalisation over the rows of each segment (InstanceNorm1d,
 * affine = False, of the sgangat GAT, GAT.py:71-74, 80: each scene's
 * (1, F, N) view is normalised per feature over its N peds):
 *   y_ij = (x_ij - mean_j) * rstd_j,  rstd_j = 1 / sqrt(var_j + eps)
 * with the biased variance over the segment.  rstd (nseg x F) is saved for
 * the backward.  A 1-row segment normalises to 0 (torch raises for it; the
 * reference's loader never produces one-ped scenes, trajectories_GCN.py).
 */
int sgg_seg_norm_fwd(const float* x, int ldx, int F, const int32_t* seg_off, int nseg, float eps,
                     float* y, int ldy, float* rstd, void* stream);

/* dx = rstd * (dy - mean(dy) - y * mean(dy * y)) per segment and feature. */
int sgg_seg_norm_bwd(const float* y, int ldy, const float* dy, int lddy, int F, const int32_t* seg_off,
                     int nseg, const float* rstd, float* dx, int lddx, void* stream);

/* ------------------------------------------------------------------------
 * Group structure of each scene from the last observed group labels
 * (models.py:263-278 / 654-680: M_intra, torch.unique rows, R = D^-1 rows):
 * group = one non-zero label value of the scene, label 0 = singleton.
 * Groups are numbered scene by scene, in order of their first member.
 * Outputs (device):
 *   ped_gid[B]        global group index of each ped
 *   ped_scene[B]      scene of each ped
 *   group_off[S+1]    CSR of groups per scene (group_off[S] = total groups G)
 *   group_scene[B]    scene of group g        (valid for g < G)
 *   group_count[B]    members of group g      (valid for g < G)
 * max_n = largest scene (<= 1024).  workspace: >= sgg_group_index_ws(S, B) bytes.
 */
size_t sgg_group_index_ws(int S, int B);
int sgg_group_index(const float* labels, const int32_t* scene_off, int S, int B, int max_n,
                    int32_t* ped_gid, int32_t* ped_scene, int32_t* group_off,
                    int32_t* group_scene, int32_t* group_count, void* workspace, void* stream);

/* Segmented reduction with deterministic (row-ascending) order:
 *   out[k, f] = post_k * sum_{i in [lo_k, hi_k), seg_of_row[i] == k} row_scale_i * x[i, f]
 * lo_k = range_off[r_k], hi_k = range_off[r_k + 1], r_k = seg_range ? seg_range[k] : k.
 * post_k = 1 / count_k when mean != 0 (count = matching rows), else 1.
 * row_scale may be NULL (= 1).  Rows k >= nseg_valid(*) are zero-filled up to
 * nseg_cap, where nseg_valid is read on the DEVICE from *nseg_dev (no host sync).
 * Replaces R @ X (group mean-pool, models.py:280 / :683), the row-normalised
 * A @ H aggregations of the GCN (:576), and (with mean = 0, row_scale = 1/|g|)
 * the backward of R^T (:286 / :699). */
int sgg_seg_reduce(const float* x, int ldx, int F, const int32_t* seg_of_row,
                   const float* row_scale, const int32_t* range_off, const int32_t* seg_range,
                   const int32_t* nseg_dev, int nseg_cap, int mean, float* out, int ldo,
                   void* stream);

/* out[i, f] = src[seg_of_row[i], f] * (row_scale ? row_scale[i] : 1) for
 * i < nvalid, 0 for nvalid <= i < n, nvalid = nrow_dev ? *nrow_dev : n (read on
 * the device).  Replaces R^T @ G (un-pool, models.py:286 / :699) and the
 * broadcast half of the GCN's A @ H (:576). */
int sgg_seg_gather(const float* src, int lds, int F, const int32_t* seg_of_row,
                   const float* row_scale, const int32_t* nrow_dev, int n, float* out, int ldo,
                   void* stream);

/* ------------------------------------------------------------------------
 * Parameter-gradient reduction C = X^T Y over R rows (X: R x M, Y: R x N,
 * row strides ldx / ldy; C: M x N, or C^T (N x M) when trans_c = 1, row
 * stride ldc -- nn.Linear-layout weights take their gradient transposed, so
 * it lands in place), and optionally colsum = sum_r Y[r, :] (bias gradient).  Split-K over sgg_xtw_splits(R, M, N)
 * workgroup slabs summed in a fixed order (deterministic); ws must hold
 * splits * (M*N + N) floats.  Replaces the library GEMMs of every weight
 * gradient (dW = X^T dY of the node transforms, W_hh / W_ih / hidden2pos of the
 * LSTMs summed over T x B, W1h of the pooling, `a` of the attention).
 * Ymask (may be NULL, row stride ldm): Y[r, n] enters (C and colsum) only where
 * Ymask[r, n] > 0 (the fused ReLU's backward). */
int sgg_xtw_splits(int R, int M, int N);
int sgg_xtw(const float* X, int ldx, const float* Y, int ldy, const float* Ymask, int ldm, int R, int M, int N,
            float* C, int ldc, int trans_c, float* colsum, float* ws, size_t ws_bytes, void* stream);
/* sgg_xtw's first pass alone: the split partials land in ws (C partials:
 * splits rows of M*N floats; then, when colsum != 0, the column-sum partials:
 * splits rows of N floats at ws + splits*M*N).  The row sums join the
 * backward's one sgg_grad_finish launch (SggRed jobs, map 1 for C). */
int sgg_xtw_partial(const float* X, int ldx, const float* Y, int ldy, const float* Ymask, int ldm, int R, int M,
                    int N, int colsum, float* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Weight-gradient finish of the backward ops of one backward pass (the
 * pooling backward of models.py:497-549, the LSTM backward of :62-92 /
 * :142-178, the discriminator head, the GAT encoder / GCN module slabs):
 * every slab row sum the op needs (SggRed: the kernels' per-workgroup slab
 * rows, sgg_xtw_partial's split partials) and the input-embedding fold
 * backwards (SggFoldBwd, the algebra of sgg_fold_bwd) whose (dA, dbias) are
 * themselves row sums of such slabs (summed into `scratch` by the row-sum
 * launch).  Every sum keeps
 * the fixed order of sgg_slab_reduce, so every output is bit-identical to
 * sgg_slab_reduce / sgg_xtw / sgg_fold_bwd run one after the other.
 * SggRed: out_c = sum_{s < rows} src[s * ld + col0 + c], c < cols, summed as
 * sgg_slab_reduce does (16 row phases, then the phases in order); map 0:
 * out[c]; map 1 (sgg_xtw's C, c = m * N + n): out[m * ldo + n], or
 * out[n * ldo + m] when trans != 0. */
#define SGG_RED_MAX 24
#define SGG_FOLDB_MAX 6
typedef struct {
  const float* src;
  int rows;
  int ld;
  int col0;
  int cols;
  float* out;
  int map;
  int N;
  int ldo;
  int trans;
} SggRed;
/* dA[r][j] = row sum of dA_src at column dA_col0 + 2 r + j, dbias[r] = row sum
 * of db_src at column db_col0 + r; then, as sgg_fold_bwd: dW (R x E, row
 * stride lddw), dWe (E x 2), dbe (E), dbias_copy (may be NULL).  R <= 512,
 * E <= 128. */
typedef struct {
  const float* W;
  int ldw;
  int R;
  int E;
  const float* We;
  const float* be;
  const float* dA_src;
  int dA_rows;
  int dA_ld;
  int dA_col0;
  const float* db_src;
  int db_rows;
  int db_ld;
  int db_col0;
  float* dW;
  int lddw;
  float* dWe;
  float* dbe;
  float* dbias_copy;
} SggFoldBwd;
/* scratch: 3 R floats per fold job (its (dA, dbias) row sums).  Launches:
 * one for all row sums, then (with fold jobs) one for every fold backward
 * (a workgroup per fold, fold_bwd's algebra and order). */
int sgg_grad_finish(const SggRed* reds, int nred, const SggFoldBwd* folds, int nfold, float* scratch,
                    size_t scratch_bytes, void* stream);

/* Loss VALUES of a training step, formed in the row-sum launch of
 * sgg_grad_finish (one extra workgroup) instead of launches of their own: in
 * the step the values are only reported (the gradients come from the
 * backward kernels), so they are due with the weight gradients, before the
 * optimizer and the data-parallel all-reduce.
 * SggL2Job: *loss = the value of sgg_l2_loss_fwd (the best-of-k L2 term,
 *   train.py:459-464): the sum in scene order of the per-scene terms
 *   w * masked SE / mask sum that sgg_l2_loss_bwd_scenes wrote (term != NULL)
 *   in the backward -- no second pass over the predictions.
 * SggBceJob: *loss = the value of sgg_bce_fwd (gan_d_loss / gan_g_loss,
 *   losses.py:24-49), *total = *loss + *addend when total != NULL.
 * The workgroup runs every L2 job, then every BCE job (an addend may be an L2
 * job's loss).  The sums keep the separate kernels' orders (bit-identical
 * values). */
#define SGG_LOSSJOB_MAX 2
typedef struct {
  const float* term;
  int S;
  float* loss;
} SggL2Job;
typedef struct {
  const float* x;
  int n;
  int split;
  const float* ya;
  const float* yb;
  float w;
  float* loss;
  const float* addend;
  float* total;
  const int32_t* nvalid;
} SggBceJob;
int sgg_grad_finish_losses(const SggRed* reds, int nred, const SggFoldBwd* folds, int nfold, float* scratch,
                           size_t scratch_bytes, const SggL2Job* l2, int nl2, const SggBceJob* bce, int nbce,
                           void* stream);

/* ------------------------------------------------------------------------
 * The discriminator's scoring head real_classifier = make_mlp([K, N1, 1])
 * (models.py:958-965 with make_mlp :7-20, applied at :991):
 *   hid = act1(X W1^T + b1)  (M x N1),   Y = act2(hid . w2 + b2)  (M)
 * act: bit 0 act1 = ReLU, bit 1 act2 = ReLU.  W1: N1 x K contiguous (nn.Linear),
 * w2: N1, b1: N1, b2: 1 (device).  hid is written for the backward.  One
 * launch: the hidden layer on v_mfma_f32_16x16x4_f32, the N1 -> 1 layer from
 * the accumulator tiles.  X and W1 16-byte aligned, ldx % 4 == 0.  Shapes: sgg_head_ok(K, N1) (K in {16, 32, 48, 64},
 * N1 in {16, 32, 64}).
 * Backward: dX (row stride lddx) and, when wslab != NULL, one slab row per 64
 * rows ((M + 63) / 64 rows of sgg_head_slab_cols(K, N1) floats):
 * [dW1 (N1 x K) | db1 (N1) | dW2 (N1) | db2], summed by sgg_grad_finish. */
int sgg_head_ok(int K, int N1);
int sgg_head_slab_cols(int K, int N1);
int sgg_head_fwd(const float* X, int ldx, int M, int K, int N1, const float* W1, const float* b1, const float* w2,
                 const float* b2, int act, float* hid, float* Y, void* stream);
/* bce_g != NULL: dY is not read; the head's output gradient is formed in the
 * launch from the BCE loss on Y that sgg_bce_fwd computed (losses.py:5-21):
 * dY[m] = (bce_g * bce_w / count) * d bce(Y[m], m < bce_split ? ya : yb) / dY,
 * count = bce_split or M - bce_split -- sgg_bce_bwd's expression (with
 * bce_nvalid, as sgg_bce_bwd: the real rows of each range only). */
int sgg_head_bwd(const float* X, int ldx, int M, int K, int N1, const float* W1, const float* w2, const float* hid,
                 const float* Y, const float* dY, int act, float* dX, int lddx, float* wslab, const float* bce_g,
                 const float* bce_ya, const float* bce_yb, int bce_split, float bce_w, const int32_t* bce_nvalid,
                 void* stream);
/* sgg_head_fwd and sgg_head_bwd with the BCE loss's gradient (bce_g != NULL
 * required) in ONE launch: Y is written (the loss value's input), hid is not
 * (the backward's ReLU masks come from the forward's own registers), dX and
 * the slab row are what the two calls write, bitwise, when *bce_g holds the
 * same value.  The trainer issues it at the BCE forward with bce_g = its
 * backward seed (1.0), which the loss's backward then confirms it received
 * (sgan.kernels.BceLink). */
int sgg_head_fwdbwd(const float* X, int ldx, int M, int K, int N1, const float* W1, const float* b1, const float* w2,
                    const float* b2, int act, float* Y, float* dX, int lddx, float* wslab, const float* bce_g,
                    const float* bce_ya, const float* bce_yb, int bce_split, float bce_w, const int32_t* bce_nvalid,
                    void* stream);

/* ------------------------------------------------------------------------
 * Input-embedding fold (a Linear(2, E) displacement embedding feeding a
 * linear layer: the LSTM input weights, models.py:52-59 / 121-125, and the
 * pooling MLP's first layer, :477-481 / 530-538):
 *   A = W We (R x 2),  bias = W be + b1 (+ b2; b2 may be NULL)
 * W: R x E with row stride ldw (W1[:, :E] in place), We: E x 2, be, b1, b2.
 * Backward: dW = dA We^T + dbias be^T (R x E, row stride lddw),
 * dWe = W^T dA (E x 2), dbe = W^T dbias (E); db1 = db2 = dbias. */
int sgg_fold_fwd(const float* W, int ldw, int R, int E, const float* We, const float* be,
                 const float* b1, const float* b2, float* A, float* bias, void* stream);
/* Several folds (a module set's: encoder, pooling, decoder) in ONE launch,
 * one workgroup each; the descriptors are copied into the kernel arguments. */
#define SGG_FOLD_MAX 8
typedef struct {
  const float* W;
  int ldw;
  int R;
  int E;
  const float* We;
  const float* be;
  const float* b1;
  const float* b2;
  float* A;
  float* bias;
} SggFold;
int sgg_fold_fwd_multi(const SggFold* folds, int n, void* stream);
/* dbias_copy (may be NULL) receives a copy of dbias: the LSTM's second bias
 * leaf b_hh gets its own gradient tensor without an extra launch.
 * R <= 512, E <= 128. */
int sgg_fold_bwd(const float* W, int ldw, int R, int E, const float* We, const float* be, const float* dA,
                 const float* dbias, float* dW, int lddw, float* dWe, float* dbe, float* dbias_copy, void* stream);

/* ------------------------------------------------------------------------
 * Fused LSTM sequence (Encoder.forward models.py:62-92; Decoder.forward
 * :142-178 with pool_every_timestep = 0), one launch for all T steps:
 *   gates_t = A r_t + W_hh h_{t-1} + bias   (A = W_ih We, bias = W_ih be + b_ih + b_hh:
 *                                           the Linear(2, E) input embedding folded in)
 *   i, f, o = sigmoid, g = tanh;  c_t = f c_{t-1} + i g;  h_t = o tanh(c_t)
 * encoder (decoder = 0): r_t = rel[t] (T x B x 2); h_{-1} = h0, c_{-1} = c0 (NULL = 0).
 * decoder (decoder = 1): r_0 = rel (B x 2), r_t = Wp h_{t-1} + bp (hidden2pos) for
 *   t >= 1; rel_out[t] = Wp h_t + bp (T x B x 2) is the predicted displacement.
 * H in {16, 32, 48, 64}.  h_all: (T+1) x B x H with index 0 the initial state.
 * act_all (gate activations) and c_all (cells) are the saved states the
 * backward reads, in a layout private to the kernel family the dispatcher
 * picks for (H, B): allocate sgg_lstm_state_floats(T, B, H, 0) floats for
 * act_all and (.., 1) for c_all.  act_all may be NULL (inference: then only
 * h_all[T] is written) and is required by the backward.
 */
long long sgg_lstm_state_floats(int T, int B, int H, int which);
int sgg_lstm_fwd(const float* rel, const float* A, const float* Whh, const float* bias,
                 const float* h0, const float* c0, const float* Wp, const float* bp, int T, int B, int H,
                 int decoder, float* h_all, float* c_all, float* act_all, float* rel_out,
                 void* stream);
/* The decoder's initial state built in the sequence kernel's prologue
 * instead of by sgg_decoder_init (add_noise, 'global' mix, models.py:827-850,
 * and the decoder's first input, :909-925; one launch fewer per rollout):
 * column p = r Bper + i (copy r, ped i) starts from
 *   h0[p] = [ctx[i] (Dc floats, row stride ldc) | z[k][scene(i)] (nz floats)],
 *   k = best[scene(i)] for r == 0 when best != NULL, else first_k + r - (best ? 1 : 0)
 *   (z: K x S x nz), rel0[p] = last_rel[i];
 * ped_scene: Bper int32 scene indices.  Everything else as sgg_lstm_fwd with
 * decoder = 1, c0 = 0; rel0_out (may be NULL) receives rel0 (B x 2) -- the
 * backward's first input -- when act_all != NULL.  Without act_all (no
 * saved states) h_all and c_all may both be NULL: the final state (h_T, c_T)
 * is then not written -- the best-of-k rollout's consumers read rel_out only
 * (models.py:925 discards the decoder state).  Returns SGG_E_ARG where
 * no kernel family takes the fused start (the caller then runs
 * sgg_decoder_init + sgg_lstm_fwd). */
typedef struct {
  const float* ctx;
  int ldc;
  int Dc;
  const float* z;
  int nz;
  const int64_t* best;
  int first_k;
  const int32_t* ped_scene;
  int S;
  int Bper;
  const float* last_rel;
} SggDecInit;
/* The discriminator input traj_rel = cat(head, the decoder's output) (and the
 * start positions) written by the same decoder launch (SggTrajOut, may be
 * NULL): sgg_traj_cat's result (train.py:409-415, 468-470) without its own
 * launch.  out is (T0 + T) x NB x 2; decoder columns col0 .. col0 + ncol - 1
 * become out's columns 0 .. ncol - 1 at steps T0 .. T0 + T - 1, head (T0
 * steps of ncol peds, step stride ldh floats) fills their first T0 steps;
 * with b != NULL (NB = 2 ncol) columns ncol .. 2 ncol - 1 hold head again,
 * then b (T steps, stride ldb); with start != NULL, start (1 x NB x 2) gets
 * pos0 (ncol x 2) for either half.  Taken by the four-wave decoder family
 * and, without saved or final states (h_all NULL), by the batch-MFMA family
 * (its second-segment form of sgg_lstm_fwd_dec2 with an empty first
 * segment); SGG_E_ARG otherwise, as for a start no family takes. */
typedef struct {
  float* out;
  int NB;
  int T0;
  int col0;
  int ncol;
  const float* head;
  int ldh;
  const float* b;
  int ldb;
  const float* pos0;
  float* start;
} SggTrajOut;
int sgg_lstm_fwd_dec(const SggDecInit* di, const float* A, const float* Whh, const float* bias, const float* Wp,
                     const float* bp, int T, int B, int H, float* h_all, float* c_all, float* act_all,
                     float* rel_out, float* rel0_out, const SggTrajOut* to, void* stream);
/* Two no-grad decoder rollouts of the same decoder weights in ONE launch on
 * the batch-MFMA family (no saved or final states): di's B sequences (the
 * generator step's best-of-k samples, B >= the family's minimum) and di2's
 * B2 (the discriminator step's generator decoder), the latter also writing
 * its discriminator input (to2, may be NULL) as sgg_lstm_fwd_dec would.  As
 * in the four-wave family the hidden2pos feedback is folded into the
 * recurrence from step 1 on (W_hh + A Wp, b + A bp), here with the weights
 * pre-scaled for v_exp_f32 and the bias as the accumulators' start: the same
 * values up to fp32 reassociation. */
int sgg_lstm_fwd_dec2(const SggDecInit* di, const SggDecInit* di2, const float* A, const float* Whh,
                      const float* bias, const float* Wp, const float* bp, int T, int B, int B2, int H,
                      float* rel_out, float* rel_out2, const SggTrajOut* to2, void* stream);

/* Encoder sequence (decoder = 0) with the pooling MLP's h-half fused into the
 * kernel's epilogue (models.py:538): also writes U = h_T Wu^T + cu (B x NU,
 * Wu: NU x H with row stride ldwu -- W1[:, E:] in place; cu: NU), computed
 * while h_T is still in LDS.  Available where sgg_lstm_u_ok says so (the
 * four-wave family; NU a multiple of 16); the other arguments and outputs are
 * those of sgg_lstm_fwd (act_all = NULL: no saved states). */
int sgg_lstm_u_ok(int T, int B, int H, int decoder, int save, int NU);
int sgg_lstm_fwd_u(const float* rel, const float* A, const float* Whh, const float* bias, const float* h0,
                   const float* c0, int T, int B, int H, float* h_all, float* c_all, float* act_all,
                   const float* Wu, int ldwu, const float* cu, int NU, float* U, void* stream);

/* Backward of sgg_lstm_fwd (BPTT).  encoder: dh_last = dL/dh_{T-1} (B x H, may
 * be NULL); decoder: dout = dL/drel_out (T x B x 2) (the decoder feedback
 * r_t -> step t+1 is included).  Writes drel_in (T x B x 2, dL/dr_t of the
 * step inputs), dh0 (B x H, may be NULL; no gradient is produced for c0)
 * and, for the decoder, drel_tot (T x B x 2, total dL/d rel_out[t]).
 * Weight gradients, two forms:
 *  - sgg_lstm_wpart_rows(H, B) > 0 (the four-wave MFMA family): pass wpart
 *    (rows x (4H*H + 4H + 8H) floats; the decoder's rows are 2H + 2 wider)
 *    and the kernel accumulates, per workgroup, one slab row [dW_hh (4H x H)
 *    | dbias (4H) | dA (4H x 2)] = sum over its peds and all steps of
 *    dG_t^T [h_{t-1} | 1 | r_in(t)] (h_all and rel -- and rel_out for the
 *    decoder, r_in(t) = rel_out[t-1] -- are read for that), followed for the
 *    decoder by [dWp (2 x H) | dbp (2)] = sum of drel_tot[t] [h_{t+1}^T | 1];
 *    sgg_slab_reduce / sgg_grad_finish sum the rows.  wpart = NULL: input
 *    gradients only (frozen weights).  dG is not used (may be NULL).
 *  - otherwise dG (T x B x 4H, gradient of the gate pre-activations) is
 *    written and the caller forms the outer-product sums (sgg_xtw); wpart
 *    must be NULL.
 * In the dG form dWp / dbp of the decoder are X^T sums of drel_tot and h_all,
 * left to the caller. */
int sgg_lstm_wpart_rows(int H, int B);
/* Name of the kernel sgg_lstm_fwd (bwd = 0; save = act_all != NULL) or
 * sgg_lstm_bwd (bwd = 1) launches for these sizes, as rocprofv3 lists it
 * (bench.py's per-kernel timing). */
const char* sgg_lstm_kernel_name(int H, int B, int decoder, int save, int bwd);
/* The decoder backward (the four-wave family, sgg_lstm_wpart_rows > 0) with
 * the output gradient in two blocks: peds < bsplit from dout (T x bsplit x 2),
 * the rest from dout2 (T x (B - bsplit) x 2) -- the best-of-k step's best and
 * last samples, whose gradients come from the L2 and the adversarial loss,
 * without concatenating them first.  Other arguments as sgg_lstm_bwd. */
int sgg_lstm_bwd_split(const float* A, const float* Whh, const float* Wp, const float* h_all, const float* c_all,
                       const float* act_all, const float* rel, const float* rel_out, const float* dout,
                       const float* dout2, int bsplit, int T, int B, int H, float* dh0, float* drel_in,
                       float* drel_tot, float* wpart, void* stream);
/* Encoder backward (the four-wave family) of steps t_stop .. T-1 only, input
 * gradients only: drel_in rows t >= t_stop are computed, rows below are set
 * to zero (their gradient is not wanted), no weight gradients, no dh0 -- the generator step's pass through
 * the frozen discriminator, whose observed-part inputs need no gradient.
 * Other arguments as sgg_lstm_bwd (decoder = 0). */
int sgg_lstm_bwd_tail(const float* A, const float* Whh, const float* h_all, const float* c_all,
                      const float* act_all, const float* rel, const float* dh_last, int T, int B, int H,
                      int t_stop, float* drel_in, void* stream);
int sgg_lstm_bwd(const float* A, const float* Whh, const float* Wp, const float* h_all, const float* c_all,
                 const float* act_all, const float* rel, const float* rel_out, const float* dh_last,
                 const float* dout, int T, int B, int H, int decoder, float* dG, float* dh0,
                 float* drel_in, float* drel_tot, float* wpart, void* stream);

/* Encoder sequence SEGMENTS of the four-wave family (sgg_lstm_u_ok's family,
 * T <= 64): steps t0 .. t0 + T - 1 of a Tl-step sequence whose states are
 * saved at their Tl-layout positions -- the discriminator encoder's observed
 * steps (models.py:976-980: Encoder(traj_rel), whose first obs_len inputs are
 * obs_rel for the real and the fake trajectories alike) run ONCE, beside the
 * generator's encoder of the same obs_rel (sgg_lstm_fwd_seg2: one launch),
 * and the discriminator's forward runs only the remaining steps on both
 * halves (sgg_lstm_fwd_seg with t0 = obs_len, Bsrc = the prefix's peds).
 *   rel      (rows t0 .. t0+T-1 of a (t0+T) x B x 2 input; t0 = 0: T x B x 2)
 *   A, Whh, bias, h0, c0 (t0 = 0 only), Wu / ldwu / cu / NU / U: as sgg_lstm_fwd_u (U NULL: none)
 *   h_all    (Tl + 1) x Bl x H, rows Bl apart (Bl >= B); c_all / act_all the
 *            tile-native saved states sized sgg_lstm_state_floats(Tl, Bl, H, .)
 *            (act_all NULL: no saved states; only h_all[t0 + T] is written)
 *   t0 > 0:  the state entering step t0 of ped p is ped (p mod Bsrc)'s,
 *            read from h_all[t0] and c_all (Bsrc = B, or a multiple of 16
 *            dividing B); h0 / c0 must be NULL.
 * The backward of the whole Tl-step sequence is sgg_lstm_bwd_shared (or
 * sgg_lstm_bwd / _tail when Bsrc = B: the layout is then complete). */
typedef struct {
  const float* rel;
  const float* A;
  const float* Whh;
  const float* bias;
  const float* h0;
  const float* c0;
  int T, B, Bl, t0, Tl, Bsrc;
  float* h_all;
  float* c_all;
  float* act_all;
  const float* Wu;
  int ldwu;
  const float* cu;
  int NU;
  float* U;
} SggLstmSeg;
int sgg_lstm_fwd_seg(const SggLstmSeg* seg, int H, void* stream);
/* Two independent segments in ONE launch (a's workgroups first); one launch
 * for (Ha, Hb) = (32, 48) with b saving states, two launches otherwise. */
int sgg_lstm_fwd_seg2(const SggLstmSeg* a, int Ha, const SggLstmSeg* b, int Hb, void* stream);
/* Three independent segments in ONE launch (a's workgroups, then b's, then
 * c's): the discriminator step's generator encoder (a, no saved states), the
 * discriminator's observed-steps prefix (b) and the generator step's encoder
 * (c, saved states) -- G.context_pair forms both steps' contexts at the
 * discriminator step (G's weights do not change in between).  One launch
 * for (Ha, Hb, Hc) = (32, 48, 32) with a not saving and b, c saving; else
 * sgg_lstm_fwd_seg2(a, b) + c. */
int sgg_lstm_fwd_seg3(const SggLstmSeg* a, int Ha, const SggLstmSeg* b, int Hb, const SggLstmSeg* c, int Hc,
                      void* stream);
/* sgg_lstm_fwd_dec (saving, four-wave family) with an independent encoder
 * segment in the same launch: the generator step's best / last samples
 * beside the discriminator's observed-steps prefix of that step (pre: the
 * SggLstmSeg sgg_lstm_fwd_seg2 would carry as b; it needs D's weights after
 * the discriminator step, so it rides with the first launch of the
 * generator step that follows them).  One launch for (H, Hp) = (32, 48),
 * two otherwise. */
int sgg_lstm_fwd_dec_seg(const SggDecInit* di, const float* A, const float* Whh, const float* bias, const float* Wp,
                         const float* bp, int T, int B, int H, float* h_all, float* c_all, float* act_all,
                         float* rel_out, float* rel0_out, const SggTrajOut* to, const SggLstmSeg* pre, int Hp,
                         void* stream);
/* sgg_lstm_bwd (encoder) of a Tl = T step sequence whose steps < t_sh were
 * saved once for Bsrc peds (sgg_lstm_fwd_seg with t0 = t_sh): ped p reads the
 * saved states of steps < t_sh (cells and h up to t_sh) of ped p mod Bsrc.
 * Bsrc a multiple of 16 dividing B; results identical to sgg_lstm_bwd on the
 * complete layout. */
int sgg_lstm_bwd_shared(const float* A, const float* Whh, const float* h_all, const float* c_all,
                        const float* act_all, const float* rel, const float* dh_last, int T, int B, int H,
                        int t_sh, int Bsrc, float* drel_in, float* wpart, void* stream);

/* ------------------------------------------------------------------------
 * Adversarial loss (losses.py:5-21 bce_loss; gan_d_loss :36-49 sums two of
 * them, gan_g_loss :24-33 is one), shard-weighted:
 *   loss = w * (mean_{i < split} f(x_i, *ya) + mean_{i >= split} f(x_i, *yb))
 *   f(x, y) = max(x, 0) - x y + log(1 + exp(-|x|))
 * An empty range contributes 0.  ya, yb are device scalars (graph-capturable
 * label smoothing); loss is one device float.  total (optional, with the
 * device scalar addend): *total = *loss + *addend -- the generator's total
 * loss (gan_g_loss + the L2 term, train.py:471-474) in the same launch.
 * nvalid (optional, one device int32): a padded batch (the fixed-capacity
 * scene index of the graph-replayed real-data path): only the first *nvalid
 * scores of each range are real; the means run over them. */
int sgg_bce_fwd(const float* x, int n, int split, const float* ya, const float* yb, float w, float* loss,
                const float* addend, float* total, const int32_t* nvalid, void* stream);

/* dx_i = *gout * w / |range(i)| * df/dx(x_i, y_range(i)) with torch's
 * subgradients at 0 (clamp passes x >= 0, d|x| = sign(x) = 0 at 0); with
 * nvalid, |range| counts the real scores and the padding scores get 0. */
int sgg_bce_bwd(const float* x, int n, int split, const float* ya, const float* yb, float w,
                const float* gout, float* dx, const int32_t* nvalid, void* stream);

/* ------------------------------------------------------------------------
 * Optimizer step of the training loop (scripts/train.py:418-427 and :472-482:
 * optional nn.utils.clip_grad_norm_(params, max_norm), then optim.Adam.step()
 * without weight decay / amsgrad).  params[i], grads[i], exp_avg[i],
 * exp_avg_sq[i] are device fp32 buffers of numel[i] elements and step[i] the
 * tensor's device fp32 step counter (torch's capturable Adam state['step']),
 * incremented first (host arrays of n <= 48 pointers).  max_norm <= 0: no clipping; otherwise the
 * clipped gradient is written back, as clip_grad_norm_ does.  ws holds
 * sgg_adam_parts(sum numel) floats: ws[0] is the one-launch path's ticket
 * word (zero when ws is first used; every call leaves it at zero and nothing
 * else writes it, whatever the tensor list or clipping of a call), then the
 * partial norms and the per-tensor step scalars.  Two launches with clipping, one without; graph-capturable. */
int sgg_adam_parts(long long total);
int sgg_adam_step(float* const* params, float* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
                  const long long* numel, int n, double lr, double beta1, double beta2, float eps, float max_norm,
                  float* const* step, float* ws, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------
 * The group GAT encoder of every scene in ONE launch (GATEncoder.forward,
 * models.py:254-294, with GAT.forward :231-237 and GraphAttentionLayer
 * :198-220): per scene (workgroup) the group mask of the last-observed labels
 * (:263-266), the intra-group GAT 40 -> 72 (x nh heads, ELU) -> 16 (ELU,
 * log_softmax), the group mean R.intra (:271-280), the inter-group GAT
 * 16 -> 72 -> 16 on the complete graph of the scene's groups (:282-285), the
 * un-pool R^T (:286) and out_embedding Linear(32, 24) (:288-289), all in LDS.
 * Replaces the per-op sequence sgg_xw / sgg_gat_fwd / sgg_group_index /
 * sgg_seg_reduce / sgg_seg_gather / concat / Linear (~14 launches).
 *
 * Weights are the module's own tensors: Wi[h] (40 x 72), ai[h] (144),
 * Wio (72 nh x 16), aio (32) of gat_intra; Wg[h] (16 x 72), ag[h], Wgo, ago of
 * gat_inter; Woe (24 x 32, nn.Linear layout), boe (24).  X: B x 40 rows
 * (stride ldx), labels: B floats, scene_off: S + 1, np = the largest scene
 * (<= 64; the LDS plan is sized by it, sgg_gatenc_lds_bytes <= 160 KiB).
 * Forward writes y (B x 24, stride ldy).  Backward (reads the forward's
 * saved state, or recomputes it when saved == NULL) reads dy and writes dX (B x 40, stride lddx) and, per scene s, the
 * parameter gradients into slab row s (sgg_gatenc_param_size(nh) floats, in
 * the order Wi[0], ai[0], .., Wio, aio, Wg[0], ag[0], .., Wgo, ago, Woe, boe);
 * sgg_slab_reduce sums the rows in scene order.
 */
#define SGG_GATENC_MAX_HEADS 4
typedef struct {
  const float* Wi[SGG_GATENC_MAX_HEADS];
  const float* ai[SGG_GATENC_MAX_HEADS];
  const float* Wio;
  const float* aio;
  const float* Wg[SGG_GATENC_MAX_HEADS];
  const float* ag[SGG_GATENC_MAX_HEADS];
  const float* Wgo;
  const float* ago;
  const float* Woe;
  const float* boe;
} SggGatEncWeights;

typedef struct {
  const float* X;
  int ldx;
  const float* labels;
  const int32_t* scene_off;
  int S;
  int np;
  int nh;
  float alpha;
  SggGatEncWeights w;
  float* y;
  int ldy;
  const float* dy;
  int lddy;
  float* dX;
  int lddx;
  float* slab;
  float* saved;   /* may be NULL: sgg_gatenc_saved_floats(S, np, nh) floats of forward state
                     (S per-scene blocks, then the staged weights the backward copies) */
  /* optional second input block: when X2 != NULL a row of the 40-wide input
   * is [X[r][0 .. kx1) | X2[r][0 .. 40 - kx1)] (the encoder state and the
   * pooled vector without a concatenation copy), and the backward writes the
   * input gradient split the same way into dX (kx1 columns) and dX2 */
  const float* X2;
  int ldx2;
  int kx1;
  float* dX2;
  int lddx2;
  /* backward: dy of the scene rows is the sum of dy_copies blocks dy_cstride
   * floats apart (the decoder's initial-state gradient of the best-of-k
   * copies, summed here instead of in a separate launch); 0 or 1: one block */
  int dy_copies;
  int dy_cstride;
} SggGatEncArgs;

int sgg_gatenc_param_size(int nh);
/* Forward state kept for the backward: when args->saved != NULL the forward
 * writes every scene's layer inputs / activations and group structure there
 * and the backward reads them instead of recomputing the forward (it must
 * then be called with the same saved buffer, np, nh and weights: after the S
 * scene blocks the buffer holds the weights' LDS image, written by the
 * forward's workgroup 0 and copied by the backward instead of restaging the
 * parameters). */
long long sgg_gatenc_saved_floats(int S, int max_n, int nh);
/* LDS bytes of a launch's plan (<= 160 KiB to run): bwd 0 the forward, 1 the
 * backward with the forward's saved state (scenes past the full plan, e.g.
 * 49 .. 64 peds with one head, take a compact plan that aliases the inter /
 * intra layers' operands and reads the epilogue inputs from the saved
 * state), 2 the backward without it (recomputing the forward: the full plan
 * only).  sgg_gatenc_bwd refuses a launch whose plan needs the saved state
 * when args->saved is NULL. */
long long sgg_gatenc_lds_bytes(int max_n, int nh, int bwd);
int sgg_gatenc_fwd(const SggGatEncArgs* args, void* stream);
/* Two independent batches through the same GATEncoder in ONE launch (a's
 * scenes first, then b's): the discriminator step's generator forward (no
 * saved state) beside the generator step's context (saved state for its
 * backward) -- the weights do not change between them (scripts/train.py:
 * 395-429 updates D only).  Both must have the same weights, heads, alpha
 * and np; each batch keeps its own X / X2 / labels / scene_off / S / y /
 * saved, exactly as two sgg_gatenc_fwd calls would write them. */
int sgg_gatenc_fwd2(const SggGatEncArgs* a, const SggGatEncArgs* b, void* stream);
int sgg_gatenc_bwd(const SggGatEncArgs* args, void* stream);

/* ------------------------------------------------------------------------
 * The group GCN module of every scene in ONE launch per direction
 * (GCNModule.forward, models.py:628-712, with GCN.forward :573-580 and
 * normalize :607-613): per scene (workgroup) the group mask of the
 * last-observed labels (:651-657), gcn_intra (fin -> 72 -> 16, A = D^-1 M,
 * ReLU((A H) W) per layer), the group pool R.intra (:667-686), gcn_inter
 * (16 -> 72 -> 16 on the complete group graph, A = 1/G), the un-pool R^T
 * (:700) and out_embedding Linear(32, fe) (:703-708).  Replaces the per-op
 * sequence sgg_group_index / sgg_seg_reduce / sgg_seg_gather / sgg_xw x 4 /
 * concat / Linear (~14 launches forward, more backward).
 *
 * Weights are the module's own tensors: W0i (fin x 72), W1i (72 x 16) of
 * gcn_intra, W0g (16 x 72), W1g (72 x 16) of gcn_inter, Woe (fe x 32, nn.Linear
 * layout), boe (fe).  X: B rows of fin floats (stride ldx), or two column
 * blocks [X (kx1) | X2 (fin - kx1)] as in SggGatEncArgs; labels: B floats;
 * scene_off: S + 1; np = the largest scene (<= 64; sgg_gcnmod_lds_bytes).
 * bf16 != 0: the forward node transforms take bf16 operands (round to nearest
 * even) with fp32 accumulation on the bf16 MFMA (set_precision("bf16")).
 * Forward writes y (B x fe, stride ldy).  Backward recomputes the forward,
 * reads dy (dy_copies blocks dy_cstride floats apart, summed) and writes dX
 * (/ dX2) and, per workgroup w < sgg_gcnmod_slab_rows(S), the parameter
 * gradients of its scenes into slab row w (sgg_gcnmod_param_size floats in
 * the order W0i, W1i, W0g, W1g, Woe, boe); sgg_slab_reduce sums the rows.
 */
typedef struct {
  const float* X;
  int ldx;
  const float* X2;
  int ldx2;
  int kx1;
  const float* labels;
  const int32_t* scene_off;
  int S;
  int np;
  int fin;
  int fe;
  int bf16;
  const float* W0i;
  const float* W1i;
  const float* W0g;
  const float* W1g;
  const float* Woe;
  const float* boe;
  float* y;
  int ldy;
  const float* dy;
  int lddy;
  int dy_copies;
  int dy_cstride;
  float* dX;
  int lddx;
  float* dX2;
  int lddx2;
  float* slab;
} SggGcnModArgs;

int sgg_gcnmod_param_size(int fin, int fe);
int sgg_gcnmod_slab_rows(int S);
long long sgg_gcnmod_lds_bytes(int max_n, int fin, int fe, int bwd);
int sgg_gcnmod_fwd(const SggGcnModArgs* args, void* stream);
/* Two independent batches through the same GCNModule in ONE launch (a's
 * scenes first): the discriminator step's generator forward beside the
 * generator step's context (G's weights do not change in between).  Same
 * weights, np, fin, fe and precision; each batch's own X / X2 / labels /
 * scene_off / S / y, exactly as two sgg_gcnmod_fwd calls would write them. */
int sgg_gcnmod_fwd2(const SggGcnModArgs* a, const SggGcnModArgs* b, void* stream);
int sgg_gcnmod_bwd(const SggGcnModArgs* args, void* stream);

/* out[c] = sum_r slab[r][c] (rows x cols, row-major), rows summed in order. */
int sgg_slab_reduce(const float* slab, int rows, int cols, float* out, void* stream);

/* ------------------------------------------------------------------------
 * Training-step glue (scripts/train.py:395-484, sgan/losses.py:52-71,
 * sgan/models.py:814-850), one launch each.  Trajectory tensors are
 * time-major rows of (x, y) pairs; ld* are floats per time step.
 *
 * sgg_traj_cat: out ((T0 + T1) x NB x 2, NB = B, or 2B when b != NULL) =
 *   cat over time of head (T0 steps, B peds; repeated for both halves) and
 *   a (T1 steps, B peds) | b (T1 steps, B peds) side by side -- the
 *   discriminator input traj_rel of the fake and real trajectories
 *   (train.py:409-415, 468-470).  start (optional, NB x 2): the same launch
 *   writes pos0 (B x 2) for every column (traj[0] of the D input, both halves
 *   start where the observation starts).
 */
int sgg_traj_cat(const float* head, int ldh, int T0, const float* a, int lda, const float* b, int ldb, int T1, int B,
                 float* out, const float* pos0, float* start, void* stream);

/* sgg_decoder_init: add_noise ('global' mix, models.py:827-850) for `copies`
 * sample-major copies of the batch: h0[r*B + p] = [ctx[p] (Dc) | z[k, s(p)] (nz)]
 * with k = best[s] for r = 0 when best != NULL (then k = first_k + r - 1
 * for r > 0), else k = first_k + r; z is (K x S x nz).  rel0[r*B + p] =
 * last_rel[p] (the decoder's first input, models.py:915). */
int sgg_decoder_init(const float* ctx, int ldc, int Dc, const float* z, int nz, const int64_t* best, int first_k,
                     int copies, const int32_t* ped_scene, int S, int B, const float* last_rel, float* h0,
                     float* rel0, void* stream);

/* sgg_l2_select: best-of-k (train.py:443-464): pred (T x k*B x 2, sample-major),
 * gt (T x B x 2), mask (B rows of ldm floats, the pred_len steps); best[s] =
 * argmin_k sum_{peds of s, t} mask (gt - pred)^2 (first minimum). */
int sgg_l2_select(const float* pred, const float* gt, const float* mask, int ldm, const int32_t* scene_off, int S,
                  int T, int B, int k, int64_t* best, void* stream);

/* sgg_l2_loss_fwd: loss = sum_s w * sum_{i in s, t} mask (gt - pred)^2 / msum_s,
 * msum_s = sum_{i in s, t} mask (train.py:459-464, losses.py:52-71 'raw');
 * a scene with msum_s = 0 (only padding scenes) adds 0 and gets 0 gradient;
 * writes msum (S) and uses term_ws (S floats).  sgg_l2_loss_bwd: dpred =
 * gout * w * -2 mask (gt - pred) / msum_{s(i)}. */
int sgg_l2_loss_fwd(const float* pred, int ldp, const float* gt, const float* mask, int ldm, const int32_t* scene_off,
                    int S, int T, int B, float w, float* loss, float* msum, float* term_ws, void* stream);
int sgg_l2_loss_bwd(const float* pred, int ldp, const float* gt, const float* mask, int ldm, const int32_t* ped_scene,
                    const float* msum, int T, int B, float w, const float* gout, float* dpred, int ldd, void* stream);
/* sgg_l2_loss_bwd without the forward: one workgroup per scene forms the
 * scene's masked squared error and mask sum (sgg_l2_loss_fwd's order) and
 * writes the scene's rows of dpred and, when term != NULL, the scene's loss
 * term (sgg_l2_loss_fwd's term_ws values), which a SggL2Job of
 * sgg_grad_finish_losses sums into the loss value. */
int sgg_l2_loss_bwd_scenes(const float* pred, int ldp, const float* gt, const float* mask, int ldm,
                           const int32_t* scene_off, int S, int T, int B, float w, const float* gout, float* dpred,
                           int ldd, float* term, void* stream);

/* ------------------------------------------------------------------------
 * Device-resident data path (sgan/data/device.py): a split's peds live in
 * HBM as one table of `rec` floats per ped
 *   [abs x, y (T x 2) | rel x, y (T x 2) | group label (T) | loss mask (T) | non_linear]
 * (T = obs_len + pred_len); one launch gathers the B ped rows of a batch
 * (`rows`, int32, the scenes' peds in batch order) into the time-major
 * 11-tuple of seq_collate (trajectories_GCN.py:15-42) packed in `out`
 * (sgg_gather_batch_floats(B, ..) floats): obs_traj, pred_traj,
 * obs_traj_rel, pred_traj_rel, obs_vel, pred_vel ((T_part x B x 2) each;
 * velocity = 2.5 x displacement), obs_traj_g, pred_traj_g (T_part x B),
 * non_linear_ped (B), loss_mask (B x T).  seq_start_end stays on the host.
 * rows[b] < 0: a padding ped, written as zeros (loss mask included). */
long long sgg_gather_batch_floats(int B, int obs_len, int pred_len);
int sgg_gather_batch(const float* table, int rec, const int32_t* rows, int B, int obs_len, int pred_len, float* out,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SGG_H */
