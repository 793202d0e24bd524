/*
 * edet.h — C-ABI of libedet.so, the MI355X (gfx950) kernels behind the EfficientDet
 * call()/train_step() hot path of tfwcn/tensorflow2-machine-vision.
 *
 * Boundary rules
 *   - plain pointers, sizes and POD descriptors only; no torch / HIP C++ types;
 *   - every entry point returns 0 on success or a negative EDET_E* code, and
 *     edet_last_error() returns a thread-local message describing the last failure;
 *   - the library never allocates or frees device memory: every buffer (activations,
 *     fp32 statistic / gradient accumulators, workspaces) is caller-owned;
 *   - every kernel is enqueued on the caller's HIP stream (`stream`, a hipStream_t
 *     passed as void*), is graph-capturable (no allocation, no host sync) and is
 *     re-entrant (no mutable global state);
 *   - activations are NHWC, row-major [rows][ld] with rows = batch*H*W;
 *     `dtype` selects the storage type: EDET_F32 or EDET_BF16; accumulation is fp32;
 *   - *_accumulate* outputs: 0 = overwrite, 1 = add into the existing contents;
 *     weight-gradient and statistic outputs are fp32 and always accumulated
 *     (atomics) into caller-zeroed buffers.
 *
 * Reference interfaces each group replaces (paths relative to
 * AIServer/ai_api/ai_models/ of the reference):
 *   stem            layers/stem.py:37-38            (Conv2D 3x3 s2 SAME + BN + swish)
 *   conv1x1         layers/mb_conv_block.py:143-154 (expand / project Conv2D 1x1),
 *                   layers/resample_feature_map.py:24-27, layers/bifpn.py:16-21,
 *                   layers/class_net.py:54-76, layers/box_net.py:49-78 (pointwise halves)
 *   dwconv          layers/mb_conv_block.py:85-91,147 (DepthwiseConv2D k3/k5 s1/s2 SAME),
 *                   SeparableConv2D depthwise halves (bifpn.py:16, class_net.py:46, box_net.py:52)
 *   lazy BN/act     every BatchNormalization(training=True) + tf.nn.swish;
 *                   the normalisation is applied in the consumer's load path
 *   se              layers/se.py:35-39
 *   maxpool/fuse    layers/resample_feature_map.py:35-51, layers/bifpn.py:59-66
 *   residual        layers/class_net.py:93-96, layers/box_net.py:93-95 + utils/drop_connect.py:4-18
 *   loss            losses/focal_loss.py:26-52, losses/box_loss.py:21-30,
 *                   efficientnet/efficientdet_net_train.py:41-52
 *   optimizer       efficientdet_net_train.py:21-28,129-131, efficientnet/train.py:35-63,114-120
 *   anchors         efficientnet/utils/anchors.py:47-84 (_generate_boxes), :91-138
 *                   (generate_targets + iou.py:27-69), :245-274 (_boxes_decoder)
 */
#ifndef EDET_H_
#define EDET_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* edet_stream_t; /* hipStream_t */

enum { EDET_F32 = 0, EDET_BF16 = 1 };
enum { EDET_ACT_NONE = 0, EDET_ACT_SWISH = 1 };
enum { EDET_MODE_SAME = 0, EDET_MODE_UPSAMPLE = 1, EDET_MODE_MAXPOOL = 2 };
enum { EDET_OK = 0, EDET_EINVAL = -1, EDET_EUNSUPPORTED = -2, EDET_EHIP = -3 };

#define EDET_MAX_SEG 5

/* Statistics vectors (ABI 9): the fp64 per-channel BN statistics (edet_bn.sum / .sq,
 * edet_statout) and BN-backward sums (edet_bngrad64) are stored REPLICATED: channel c of
 * replica r (r < EDET_STAT_REPLICAS) lives at element
 *     (c / 16) * 16 * EDET_STAT_REPLICAS + r * 16 + c % 16
 * and its value is the sum of its replicas (r = 0, 1, 2, 3, in that order, paired (0+1)+(2+3)).
 * A vector of C channels therefore takes ceil(C / 16) * 16 * EDET_STAT_REPLICAS doubles
 * (EDET_STAT_LEN(C)); producers add each block's sums into one replica, so an address sees a
 * quarter of the adders (contended fp64 atomics cost the D0 step ~0.3 ms).  Accumulators are
 * caller-zeroed as before; a caller that writes a value itself puts it in replica 0 and zeroes
 * the others. */
#define EDET_STAT_REPLICAS 4
#define EDET_STAT_LEN(C) ((((C) + 15) / 16) * 16 * EDET_STAT_REPLICAS)

/* Row layout of a (possibly multi-level) NHWC activation buffer.  Segment s holds
 * batch*H[s]*W[s] rows starting at row_off[s] (a multiple of 128).  A plain tensor
 * is one segment at offset 0.  The feature pyramid P3..P7 is five segments. */
typedef struct edet_pyramid {
  int32_t nseg;
  int32_t batch;
  int32_t row_off[EDET_MAX_SEG];
  int32_t H[EDET_MAX_SEG];
  int32_t W[EDET_MAX_SEG];
} edet_pyramid;

/* Training-mode batch normalisation of a raw tensor (per segment). sum/sq are the fp64
 * per-channel sums of x and x^2 over the segment's rows, produced by the tensor's
 * producer kernel (blocks reduce in fp32, then one fp64 atomic per channel: the order of
 * the cross-block additions no longer reaches the fp32 affine, so forward values are
 * reproducible run to run, and var = E[x^2] - mean^2 keeps its precision over 2M rows).
 * y = (x - mean) * rsqrt(var + eps) * gamma + beta, var biased. */
typedef struct edet_bn {
  const double* sum[EDET_MAX_SEG];
  const double* sq[EDET_MAX_SEG];
  const float* gamma[EDET_MAX_SEG];
  const float* beta[EDET_MAX_SEG];
  float eps;
  int32_t enabled;
} edet_bn;

/* A value that is stored raw and materialised on load:
 *   v = act(bn(x)) * gate[image][c]        (bn / act / gate each optional) */
typedef struct edet_lazy {
  const void* x;        /* raw [rows][ld] in `dtype` */
  const float* gate;    /* [batch][C] SE gate or NULL */
  edet_bn bn;
  int32_t ld;
  int32_t act;
} edet_lazy;

/* per-segment fp32 outputs (BN gamma / beta gradients) */
typedef struct edet_segout {
  float* a[EDET_MAX_SEG];
  float* b[EDET_MAX_SEG];
} edet_segout;

/* per-segment fp64 BN-backward sums (dgamma = sum du * xhat, dbeta = sum du), see
 * edet_lazy_bwd_reduce */
typedef struct edet_bngrad64 {
  double* dgamma[EDET_MAX_SEG];
  double* dbeta[EDET_MAX_SEG];
} edet_bngrad64;

/* The gradient of a lazy value's RAW tensor left unmaterialised (ABI 8): its consumer computes
 *   d(raw y) = sc*du + kb*y + kc,  du = (dv * gate[n][c] + dsq[n][c]) * act'(bn(y))
 * (kb, kc from acc: edet_lazy_bwd_apply's formula, element for element) while it loads it, so
 * the apply pass over (dv, y) and the write + re-read of d(raw y) disappear.
 *   dv   : d(value) [rows][C] in the storage dtype (the value's own row layout)
 *   y    : the value's descriptor (raw y, training BN statistics, act, SE gate or null)
 *   dsq  : [batch][C] SE squeeze-path gradient (edet_se_bwd*), nullable
 *   acc  : the final fp64 (dgamma, dbeta) sums of y's BatchNorm (y.bn.enabled)
 *   grads: fp32 gamma / beta parameter gradients, += (float)acc once by the consumer (a[s] null:
 *          not written) */
typedef struct edet_dgrad_lazy {
  const void* dv;
  edet_lazy y;
  const float* dsq;
  edet_bngrad64 acc;
  edet_segout grads;
} edet_dgrad_lazy;

/* per-segment fp64 BN statistics outputs of a producer: sum and sum of squares */
typedef struct edet_statout {
  double* sum[EDET_MAX_SEG];
  double* sq[EDET_MAX_SEG];
} edet_statout;

typedef struct edet_fuse_input {
  edet_lazy v;          /* input value (lazy BN of a resampled conv, or a node output) */
  void* dx;             /* backward: gradient w.r.t. the input value (same layout) */
  int32_t H, W;         /* input spatial size */
  int32_t mode;         /* EDET_MODE_* : same / nearest upsample / maxpool 3x3 s2 SAME */
  int32_t accumulate;   /* backward: accumulate into dx */
  uint8_t* pool_arg;    /* MAXPOOL, optional: [B*H_out*W_out][C] window tap (0..8, row-major) of
                           each output's max.  fwd writes it, bwd reads it instead of
                           re-evaluating the windows (null: recompute) */
} edet_fuse_input;

typedef struct edet_sched {
  float adjusted_lr, warmup_init;
  int32_t warmup_steps, total_steps;
  float momentum, ema_decay, clip_norm, l2_weight;
  float fixed_lr;       /* >0: constant learning rate instead of the cosine schedule */
  int32_t skip_nonfinite; /* 1: a step whose gradient norm is NaN / Inf leaves w, v, ema, the
                             compute copy and the step counter unchanged (scalars[6] = 1); 0 (the
                             reference's behaviour, efficientdet_net_train.py:129-130): applied */
} edet_sched;

/* ---- library ---- */
const char* edet_last_error(void);
int edet_abi_version(void);
int edet_memset_async(void* p, int value, size_t bytes, edet_stream_t stream);
int edet_memcpy_async(void* dst, const void* src, size_t bytes, edet_stream_t stream);
/* round 6: zero up to EDET_ZERO_MAX 16-byte aligned device ranges in one launch (the step's
 * per-step accumulators: gradients, BN statistics, loss scalars) */
#define EDET_ZERO_MAX 8
int edet_zero_ranges(int n, void* const* ptrs, const size_t* bytes, edet_stream_t stream);
/* Register device scratch used by split reductions (weight gradients write per-split partials
 * and sum them in a fixed order instead of issuing atomics).  The buffer must stay valid while
 * kernels that may use it are queued; NULL unregisters (atomics fallback).  Not thread-safe:
 * one registered workspace per process. */
int edet_set_workspace(void* ptr, size_t bytes);
/* ABI 10: deferred split sums.  Between edet_partials_defer and edet_partials_flush, every
 * weight-gradient split reduction (1x1 wgrad partials, wave-streaming wgrad, stem wgrad) writes
 * its partials into a fresh region of `arena` (256-B aligned bump allocation) and its fixed-order
 * sum into dW / db is recorded instead of launched; edet_partials_flush launches every recorded
 * sum (one launch per 40 jobs) and closes the window.  The gradients those sums complete must not
 * be read before the flush.  A region that does not fit falls back to the ordinary workspace and
 * an immediate sum; *needed (nullable) receives the arena size the window would have used. */
int edet_partials_defer(void* arena, size_t bytes);
int edet_partials_flush(size_t* needed, edet_stream_t stream);
/* launch-duration probe (measurement): end = 0 stores the wall clock in slot[0]; end = 1 adds
 * (now - slot[0]) to slot[1] and 1 to slot[2].  Capturable in HIP graphs. */
int edet_probe(uint64_t* slot, int end, edet_stream_t stream);
int edet_wall_clock_khz(int* khz);
/* measurement: the kernels this thread launched through the library since the previous call,
 * comma-separated base names (e.g. "k_wgrad_tr,k_sum_partials") into buf; returns the number
 * of launches (not a status). */
int edet_launched_kernels(char* buf, size_t size);
/* development: A/B slots 0..63 read by some launchers' plan choices (0 = the production plan),
 * compiled only into the EDET_DEV build (`make dev` -> lib/libedet_dev.so, for
 * scripts/kbench.py --dev).  Returns EDET_OK there (EDET_EINVAL for a slot outside 0..63); the
 * production library has no slots and returns EDET_EUNSUPPORTED. */
int edet_dev_set(int slot, int value);

/* ---- pointwise (1x1) convolution: y[m][n] = sum_k v(a)[m][k] * wt[n][k] + bias[n] ----
 * wt is [N][K] in `dtype`.  `stats` (nullable) receives per-segment column sums of y.
 * accumulate = 1 needs a plain A (a->bn disabled, no act, no gate): EDET_EINVAL otherwise. */
int edet_conv1x1_fwd(int dtype, const edet_lazy* a, const edet_pyramid* rows, int K,
                     const void* wt, int N, const float* bias, void* y, int ldy,
                     int accumulate, const edet_statout* stats, edet_stream_t stream);
/* dx[m][k] = sum_n dy[m][n] * w[n][k]; wkn is the transposed compute copy [K][roundup(N,8)]
 * written by edet_transpose_cast */
int edet_conv1x1_dgrad(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                       const void* wkn, int K, void* dx, int lddx, int accumulate,
                       edet_stream_t stream);
/* edet_conv1x1_dgrad (accumulate = 0) with the BN-backward fold of the value dx is the gradient
 * of (ABI 7): xv is that value's lazy descriptor (raw x [rows][xv->ld], BN enabled, act, no gate)
 * and, per segment s and channel k over the valid rows,
 *   du = dx * act'(bn(x)),  fold->dbeta[s][k] += sum du,  fold->dgamma[s][k] += sum du * xhat
 * (fp64, caller-zeroed) -- the sums edet_lazy_bwd_reduce(xv, dv = dx) would take, from the stored
 * dx, in the GEMM's epilogue instead of a pass over (x, dx).  Replaces the reduce of
 * mb_conv_block.py:143-154's BatchNormalization backward behind the expand conv's dgrad. */
int edet_conv1x1_dgrad_fold(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                            const void* wkn, int K, void* dx, int lddx, const edet_lazy* xv,
                            const edet_bngrad64* fold, edet_stream_t stream);
/* dwt[n][k] += sum_m dy[m][n] * v(a)[m][k];  dbias[n] += sum_m dy[m][n]  (valid rows only) */
/* The MBConv project conv's dgrad (mb_conv_block.py:150-154 backward) with the SE-gated
 * depthwise output's backward sums taken from its own output tile (ABI 8): dx = dy * W as
 * edet_conv1x1_dgrad (accumulate 0), and sums5 += edet_gate_bn_reduce(yv, dv = dx)'s five
 * per-image sums ([5][batch][K] fp64, zeroed by the caller).  yv: the gated value's descriptor
 * (raw y, BN with batch statistics, swish; its gate is ignored), one segment.  Shapes the
 * K-loop epilogue does not take run the two passes (same results, same destinations). */
int edet_conv1x1_dgrad_sesum(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                             const void* wkn, int K, void* dx, int lddx, const edet_lazy* yv, double* sums5,
                             edet_stream_t stream);
int edet_conv1x1_wgrad(int dtype, const edet_lazy* a, const edet_pyramid* rows, int K,
                       const void* dy, int lddy, int N, float* dwt, float* dbias,
                       edet_stream_t stream);

/* ---- depthwise k x k, stride s, TF 'SAME' padding; w is [k*k][C] in `dtype` ---- */
int edet_dwconv_fwd(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                    int stride, const void* w, void* y, const edet_pyramid* pout,
                    const edet_statout* stats, edet_stream_t stream);
/* inference: edet_dwconv_fwd (no statistics) and the SE squeeze of the output in the same pass,
 *   s[n][c] += mean_hw v(y)  with v = yv's lazy transform act(bn(y)) (yv->x is ignored; no
 *   gate) into a zeroed fp64 [B][C] -- edet_se_squeeze over y without its own pass.  In
 *   call(training=False) y's BN uses moving statistics, so its affine is known before the
 *   launch (layers/se.py:35-39 on mb_conv_block.py:147-150).  Single tensors (nseg 1). */
int edet_dwconv_fwd_squeeze(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                            int stride, const void* w, void* y, const edet_pyramid* pout,
                            const edet_lazy* yv, double* s, edet_stream_t stream);
int edet_dwconv_dgrad(int dtype, const void* dy, const edet_pyramid* pout, int C, int k,
                      int stride, const void* w, void* dx, const edet_pyramid* pin,
                      int accumulate, edet_stream_t stream);
/* edet_dwconv_dgrad (accumulate = 0) with the BN-backward fold of the value dx is the gradient of
 * (ABI 7): xv = that value's lazy descriptor (raw x on pin's rows, BN enabled, act, no gate);
 * fold->dbeta[s][c] += sum du, fold->dgamma[s][c] += sum du * xhat with du = dx * act'(bn(x)) from
 * the stored dx (fp64, caller-zeroed) -- edet_lazy_bwd_reduce(xv, dv = dx) without its pass where
 * that is faster (measured per shape; elsewhere the library runs the dgrad and the reduce pass).
 * Used for the stride-2 MBConv depthwise convs (mb_conv_block.py:143-147), whose backward is not
 * fused. */
int edet_dwconv_dgrad_fold(int dtype, const void* dy, const edet_pyramid* pout, int C, int k,
                           int stride, const void* w, void* dx, const edet_pyramid* pin,
                           const edet_lazy* xv, const edet_bngrad64* fold, edet_stream_t stream);
int edet_dwconv_wgrad(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                      int stride, const void* dy, const edet_pyramid* pout, float* dw,
                      edet_stream_t stream);

/* ---- stem: 3x3 s2 SAME, Cin = 3, no bias; w is [3][3][3][Cout] in `dtype` ---- */
int edet_stem_fwd(int dtype, const void* x, int B, int H, int W, const void* w, int Cout,
                  void* y, double* sum, double* sq, edet_stream_t stream);
int edet_stem_wgrad(int dtype, const void* x, int B, int H, int W, const void* dy, int Cout,
                    float* dw, edet_stream_t stream);

/* ---- lazy-value backward: dx = d v / d x  (BN training backward, swish', SE gate) ----
 * dv_scale [nseg][batch] (nullable) multiplies dv per image (drop-connect);
 * dsq [batch][C] (nullable) is added to d(pre-gate value) (SE squeeze path, already / HW).
 * reduce: acc->dgamma[s] += sum du * xhat, acc->dbeta[s] += sum du   (fp64, zeroed by caller:
 *         the sums feed every dx of the apply pass, so their cross-block order must not
 *         reach the bf16 rounding of dx — see edet_bn)
 * apply : dx = scale * (du - dbeta/M - xhat * dgamma/M)   (or du when BN is off);
 *         block 0 also adds the fp32 parameter gradients grads->a[s] += dgamma,
 *         grads->b[s] += dbeta when `grads` is non-NULL */
int edet_lazy_bwd_reduce(int dtype, const edet_lazy* x, const edet_pyramid* p, int C,
                         const void* dv, const float* dv_scale, const float* dsq,
                         const edet_bngrad64* acc, edet_stream_t stream);
int edet_lazy_bwd_apply(int dtype, const edet_lazy* x, const edet_pyramid* p, int C,
                        const void* dv, const float* dv_scale, const float* dsq,
                        const edet_bngrad64* acc, const edet_segout* grads, void* dx,
                        int accumulate, edet_stream_t stream);

/* ---- fused depthwise backward, stride 1: one pass over dy and x gives
 *   dx (= edet_dwconv_dgrad, `accumulate` as there), dw += (= edet_dwconv_wgrad), and, when
 *   `fold` is non-NULL, x's BN-backward sums fold->dbeta[s] += sum du,
 *   fold->dgamma[s] += sum du * xhat with du = dx * act'(bn(x)) (= edet_lazy_bwd_reduce with
 *   dv = dx, no dv_scale / dsq; needs accumulate == 0, no gate on x and x->bn enabled).
 *   stride != 1 returns EDET_EUNSUPPORTED. */
int edet_dwconv_bwd(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                    int stride, const void* dy, const edet_pyramid* pout, const void* w,
                    void* dx, int accumulate, float* dw, const edet_bngrad64* fold,
                    edet_stream_t stream);
/* edet_dwconv_bwd with dy given lazily (ABI 8): dy = d(raw y) of the edet_dgrad_lazy `dyl`
 * (the SE-gated swish(BN) depthwise output's gradient of an MBConv block, mb_conv_block.py:
 * 147-150 with se.py:35-39), built while the dy window is loaded, rounded to the storage dtype
 * as edet_lazy_bwd_apply would store it.  Also writes dyl->grads (y's gamma / beta gradients).
 * Stride 1, C % 16 == 0, dyl->y.ld == C; same results as edet_lazy_bwd_apply + edet_dwconv_bwd. */
int edet_dwconv_bwd_lazy(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                         const edet_dgrad_lazy* dyl, const edet_pyramid* pout, const void* w,
                         void* dx, int accumulate, float* dw, const edet_bngrad64* fold,
                         edet_stream_t stream);

/* ---- squeeze-excitation ---- */
/* s += mean_hw v(x) into a zeroed fp64 [B][C] (fp64 cross-block sums: the squeeze feeds the
 * forward, so it is kept reproducible like the BN statistics) */
int edet_se_squeeze(int dtype, const edet_lazy* x, int B, int HW, int C, double* s,
                    edet_stream_t stream);
int edet_se_fwd(int B, int C, int R, const double* s, const float* w1, const float* b1,
                const float* w2, const float* b2, float* z1, float* gate, edet_stream_t stream);
/* dgate += sum_hw dv * v(x) into a zeroed fp64 [B][C] (feeds dx through se_bwd -> dsq) */
int edet_gate_grad(int dtype, const edet_lazy* x, int B, int HW, int C, const void* dv,
                   double* dgate, edet_stream_t stream);
/* SE-gated BN value v = swish(bn(x)) * gate: one pass over (x, dv) giving, per image and
 * channel, sums5[q][n][c] (fp64, accumulated) for q = 0: dv*swish(u) (the gate gradient),
 * 1: dv*swish'(u), 2: swish'(u), 3: dv*swish'(u)*xhat, 4: swish'(u)*xhat; then
 * edet_se_bn_combine folds gate and dsq in: dbeta += sum_n gate*[1] + dsq*[2], dgamma +=
 * sum_n gate*[3] + dsq*[4] -- the edet_lazy_bwd_reduce result, without its pass over x, dv.
 * (layers/se.py:35-39 + mb_conv_block.py:147-150 backward; C <= 2048.) */
int edet_gate_bn_reduce(int dtype, const edet_lazy* x, int B, int HW, int C, const void* dv,
                        double* sums5, edet_stream_t stream);
int edet_se_bn_combine(int B, int C, const float* gate, const float* dsq, const double* sums5,
                       const edet_bngrad64* acc, edet_stream_t stream);
int edet_se_bwd(int B, int C, int R, int HW, const double* s, const float* z1,
                const float* gate, const double* dgate, const float* w1, const float* w2,
                float* dw1, float* db1, float* dw2, float* db2, float* dsq, float* dz1,
                edet_stream_t stream); /* dz1: [B][R] scratch; weight grads accumulate (+=) */
/* edet_se_bwd followed by edet_se_bn_combine(B, C, gate, dsq, sums5, acc) in the same two
 * launches (the combine's sums over the images ride in the weight-gradient pass) */
int edet_se_bwd_bn(int B, int C, int R, int HW, const double* s, const float* z1,
                   const float* gate, const double* dgate, const float* w1, const float* w2,
                   float* dw1, float* db1, float* dw2, float* db2, float* dsq, float* dz1,
                   const double* sums5, const edet_bngrad64* acc, edet_stream_t stream);

/* ---- out[rows][C] = v(x) = act(bn(x)) * gate: the SE-gated depthwise output written once for
 * the MBConv project conv (mb_conv_block.py:150-154), whose forward GEMM and weight gradient
 * both read it ---- */
int edet_lazy_materialize(int dtype, const edet_lazy* x, const edet_pyramid* p, int C, void* out,
                          edet_stream_t stream);

/* ---- heads: out = v(x) * scale[seg][n] + v(res) (drop-connect + residual) ---- */
int edet_residual_fwd(int dtype, const edet_lazy* x, const edet_lazy* res,
                      const edet_pyramid* p, int C, const float* scale, void* out,
                      edet_stream_t stream);

/* ---- resampling & BiFPN weighted fusion ---- */
int edet_maxpool_fwd(int dtype, const edet_lazy* x, int B, int H, int W, int C, void* y,
                     edet_stream_t stream);
int edet_maxpool_bwd(int dtype, const edet_lazy* x, int B, int H, int W, int C,
                     const void* dy, void* dx, int accumulate, edet_stream_t stream);
/* round 6: the forward records each output's window tap (0..8, row-major) per channel in
 * taps [B*ceil(H/2)*ceil(W/2)][C] (uint8); the backward then routes dy by the taps alone -- no
 * input values, no BN tables, no window re-evaluation.  Same results as edet_maxpool_bwd. */
int edet_maxpool_fwd_taps(int dtype, const edet_lazy* x, int B, int H, int W, int C, void* y,
                          uint8_t* taps, edet_stream_t stream);
int edet_maxpool_bwd_taps(int dtype, int B, int H, int W, int C, const uint8_t* taps,
                          const void* dy, void* dx, int accumulate, edet_stream_t stream);
int edet_bifpn_fuse_fwd(int dtype, int n_in, const edet_fuse_input* ins, const float* w,
                        int B, int H, int W, int C, void* out, edet_stream_t stream);
int edet_bifpn_fuse_bwd(int dtype, int n_in, const edet_fuse_input* ins, const float* w,
                        int B, int H, int W, int C, const void* out, const void* dout,
                        float* dw, edet_stream_t stream);

/* ABI 10: the fusion backward in one pass from the gradient of the node's VALUE
 * (bifpn.py:59-66 with OpAfterCombine's swish, bifpn.py:26): dv = d act(F) [B*H*W][C], out = the
 * raw fused F the forward wrote, out_act = act (0 none, 1 swish).  d(raw F) is formed in
 * registers, so the caller runs no d(value) -> d(raw) pass over the output.  dx of every input as
 * edet_bifpn_fuse_bwd (accumulate honoured).  The weight gradient leaves as per-block sums in
 * part[nparts][4] floats (no atomics); edet_bifpn_fuse_fold adds them into dw.
 * edet_bifpn_fuse_bwd_dv_parts sets *nparts to the number of float4 records the launch writes,
 * or 0 when the node is not covered (bf16 only; the input-mode combinations of the BiFPN; an
 * upsampled input must be exactly x2; a max-pooled input needs the forward's pool_arg taps):
 * the caller then uses edet_bifpn_fuse_bwd. */
int edet_bifpn_fuse_bwd_dv_parts(int dtype, int n_in, const edet_fuse_input* ins, int B, int H,
                                 int W, int C, int* nparts);
int edet_bifpn_fuse_bwd_dv(int dtype, int n_in, const edet_fuse_input* ins, const float* w,
                           int B, int H, int W, int C, const void* out, const void* dv,
                           int out_act, float* part, int nparts, edet_stream_t stream);

/* one node's weight-gradient records: dw[i] += (sum_b part[b][i]) / (sum_i w[i] + 1e-4),
 * i < n_in, the records summed in a fixed order in fp64 (reproducible) */
typedef struct edet_fuse_fold {
  const float* part;    /* [nparts][4] from edet_bifpn_fuse_bwd_dv */
  const float* w;       /* the node's n_in fusion weights */
  float* dw;            /* their gradient (added to) */
  int32_t nparts, n_in;
} edet_fuse_fold;
#define EDET_FUSE_FOLD_MAX 64  /* items per launch; longer lists take several launches */
int edet_bifpn_fuse_fold(int n, const edet_fuse_fold* items, edet_stream_t stream);

/* ---- detection loss (focal + Huber), forward and backward in one pass ----
 * cls: [rows][ldc] logits (A*NC used), box: [rows][ldb] (A*4 used).
 * cls_t [rows][A] class index, box_t [rows][A][4], npos_sum = sum of positive masks
 * (the kernel adds the reference's +1).  loss += sum_l (box_weight*box_l + focal_l).
 * focal_count_scale multiplies the per-level element count of the focal mean (data-parallel
 * replicas pass the world size so the summed replica gradients equal the global-batch ones).
 * dcls may alias cls and dbox may alias box (each element is read before it is written).
 * dcls/dbox (nullable) receive d loss / d logits (pad columns written as 0). */
int edet_detection_loss(int dtype, const void* cls, int ldc, const void* box, int ldb,
                        const edet_pyramid* p, int A, int NC, const int32_t* cls_t,
                        const float* box_t, const float* npos_sum, float alpha, float gamma,
                        float delta, float box_weight, float focal_count_scale, void* dcls,
                        void* dbox, float* loss, float* level_parts, edet_stream_t stream);
int edet_count_positives(const uint8_t* mask, int64_t n, float* out, edet_stream_t stream);
int edet_onehot_to_index(const float* onehot, int64_t n, int NC, int32_t* out,
                         edet_stream_t stream);

/* ---- anchors / targets / decode (bit-exact fp32 index work) ---- */
int edet_anchor_boxes(int fh, int fw, float start_y, float delta_y, float start_x,
                      float delta_x, int A, const float* half_yx, float* out,
                      edet_stream_t stream);
int edet_generate_targets(const float* anchors, const edet_pyramid* p, int A,
                          const float* gt, const int32_t* gt_cls, const int32_t* n_gt,
                          int max_gt, float iou_thr, float* box_t, int32_t* cls_t,
                          uint8_t* mask, edet_stream_t stream);
int edet_decode_boxes(int dtype, const float* anchors, const edet_pyramid* p, int A,
                      const void* rel, int ld, float* out, edet_stream_t stream);

/* Detection post-processing of a batch (the test_step / inference path): per image, the
 * anchors whose first-argmax class over the NC logits is not class 0 and whose max logit is
 * >= score_thr, greedy DIoU-NMS in descending logit order (ties: lower flat index) with
 * suppression at DIoU >= iou_thr, at most max_out kept; scores returned as sigmoid(logit).
 * boxes: decoded [rows][A][4] fp32 (edet_decode_boxes); cls: logits [rows][ldc] in dtype,
 * channel a*NC + c; scratch: batch * N * 8 bytes with N = sum_l H_l*W_l*A.
 * Outputs [batch][max_out][4], [batch][max_out], [batch][max_out], [batch].
 * Replaces Anchors.convert_outputs_one (anchors.py:161-202) + get_nms (nms.py:5-61). */
int edet_detect_nms(int dtype, const float* boxes, const void* cls, int ldc, const edet_pyramid* p, int A,
                    int NC, int max_out, float iou_thr, float score_thr, void* scratch,
                    float* out_boxes, int32_t* out_cls, float* out_scores, int32_t* out_count,
                    edet_stream_t stream);

/* ---- optimizer: L2 + clip_by_global_norm + SGD momentum + EMA, fused ----
 * scalars: [0] loss  [1] sum g^2  [2] sum w^2 (L2 params)  [3] gnorm  [4] lr  [5] npos
 *          [6] 1 when edet_opt_apply skipped a non-finite step (sched->skip_nonfinite), else 0
 * step: device int32 step counter (incremented by edet_opt_apply). */
/* norm pass: writes EDET_OPT_NORM_BLOCKS per-block partial sums of (g + l2*w)^2 and of
 * w^2 over the L2 prefix to partials[0..255] / partials[256..511] (fp64, device; no atomics);
 * also writes scalars[4] = lr(step) and increments *step. */
#define EDET_OPT_NORM_BLOCKS 256
int edet_opt_norm(const float* w, const float* g, int64_t n, int64_t n_l2,
                  const edet_sched* sched, float* scalars, double* partials, int32_t* step,
                  edet_stream_t stream);
/* apply pass: folds the partials in one fixed order (bit-identical gnorm on every data-parallel
 * replica), clip, SGD momentum, EMA; writes the `dtype` compute copy of w (nullable),
 * scalars[1] = sum g^2, scalars[2] = sum w^2, scalars[3] = gnorm (pre-clip),
 * scalars[0] += l2 * sum w^2 / 2, scalars[6] = skipped (0/1).  `step` (nullable): the counter
 * edet_opt_norm advanced, stepped back when the update is skipped (ABI 7). */
int edet_opt_apply(float* w, const float* g, float* v, float* ema, int64_t n, int64_t n_l2,
                   const edet_sched* sched, float* scalars, const double* partials, int dtype, void* wcompute,
                   int32_t* step, edet_stream_t stream);
int edet_cast_f32(int dtype, const float* src, void* dst, int64_t n, edet_stream_t stream);
/* fp32 [N][K] 1x1 kernels -> `dtype` [K][roundup(N,8)] copies; table[e] = {src_off, dst_off, N, K}
 * (int64, device memory); grid = max_tiles (32x32 tiles of the largest entry) x n_entries */
int edet_transpose_cast(int dtype, const float* src, void* dst, const int64_t* table, int n_entries,
                        int max_tiles, edet_stream_t stream);
/* inference-mode BN: express moving mean/var as the sums the lazy loaders expect */
int edet_bn_inference_stats(int64_t n, const float* mmean, const float* mvar, const float* count,
                            double* sum, double* sq, edet_stream_t stream);
/* Keras moving statistics from the step's batch sums.  `skip` (nullable, device): the
 * optimizer's scalars[6]; when it is non-zero (edet_opt_apply skipped a non-finite step) the
 * moving statistics are left unchanged (ABI 8). */
int edet_bn_update_moving(int64_t n, const double* sum, const double* sq, const float* count,
                          float momentum, const float* skip, float* mmean, float* mvar,
                          edet_stream_t stream);
int edet_dropmask(float* out, int n, float survival, uint64_t seed, const int32_t* step,
                  edet_stream_t stream);

/* ---- input pipeline: training augmentation (datasets/coco_dataset_one.py:99-135) ----
 * One image, HWC uint8 in the caller's channel order: box blur -> perspective warp (+ noise)
 * -> proportional resize into an out_w x out_h frame with a border -> /255 in `dtype` (or raw
 * uint8 with out_raw).  The restated OpenCV algorithms and their parity status are described in
 * csrc/augment.hip; the random draws and the box-corner geometry are host-side (augment.py).
 * scratch: 2 * H * W * 3 bytes of device memory. */
typedef struct edet_aug_params {
  double warp[9];            /* destination -> source map of the warp, row-major (identity: none) */
  uint64_t noise_seed;
  int32_t blur;              /* box-blur window 0..31 (0 or 1: none) */
  int32_t warp_border;       /* 0: constant warp_bg, 1: replicate */
  int32_t noise;             /* 1: + U{0..39} - 20 per element, clipped to [0, 255] */
  int32_t rw, rh, top, left; /* the resized image's size and its place in the output frame */
  int32_t pad_border;        /* 0: constant pad_bg, 1: replicate the resized image's edge */
  int32_t out_raw;           /* 1: out is uint8 [out_h][out_w][3] without the /255 */
  uint8_t warp_bg[4];        /* border values in the image's channel order ([3] unused) */
  uint8_t pad_bg[4];
} edet_aug_params;
int edet_augment_image(int dtype, const uint8_t* src, int H, int W, const edet_aug_params* p,
                       uint8_t* scratch, void* out, int out_h, int out_w, edet_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* EDET_H_ */
