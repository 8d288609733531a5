/* fastscnn.h — C ABI of libfastscnn_hip.so, the MI355X (gfx950) Fast-SCNN hot path.
 *
 * Plain pointers and sizes only (no torch types).  Every function returns 0 on success or a
 * negative status (-1 invalid argument, -2 unsupported, -3 HIP error); fscnn_last_error()
 * returns the thread-local message of the last failure.  The library never allocates device
 * memory: the caller passes arenas and workspaces.  Launches go to the caller's hipStream_t
 * (passed as void*), so calls are graph-capturable and overlap with RCCL on other streams.
 *
 * dtype codes: 0 = fp32, 1 = bf16, 2 = fp16 (a plan's arithmetic, and image / logit dtypes).
 * Activations are NHWC; images and logits are NCHW.
 *
 * Thread safety: every entry point may be called concurrently from several host threads (the
 * reference's torch.nn.DataParallel, train.py:170-171, runs one replica per device from its own
 * worker thread); a plan may be shared by calls on the device it was first used on.  The launch
 * profiler (fscnn_prof_*) is process-global and meant for single-threaded measurement.
 *
 * Reference interfaces replaced (Shinokawa/Fast-SCNN-pytorch):
 *   fscnn_net_* / fscnn_plan_* / fscnn_forward   FastSCNN.__init__ / forward
 *                                                 (models/fast_scnn.py:16-46)
 *   fscnn_backward                                autograd backward of that forward
 *                                                 (train.py:273 / :280 loss.backward())
 *   fscnn_ce_fwd / fscnn_ce_bwd                   nn.CrossEntropyLoss(ignore_index=-1)
 *                                                 (utils/loss.py:103-124, train.py:191)
 *   fscnn_sgd                                     torch.optim.SGD.step (train.py:195-198,274)
 *   fscnn_conv0_fwd                               _ConvBNReLU(3,32,3,2) (models/fast_scnn.py:153)
 *   fscnn_dw3x3_*                                 nn.Conv2d(groups=C, k=3, pad=1) (:70, :86)
 *   fscnn_pw_gemm / fscnn_pw_wgrad                nn.Conv2d(k=1) (:73, :103, :107, :124-128,
 *                                                 :198, :202, :230)
 *   fscnn_bn_*                                    nn.BatchNorm2d (:56, :71, :74, :87, :108)
 *   fscnn_bilinear_ac_*                           F.interpolate(bilinear, align_corners=True)
 *                                                 (:40, :135, :212)
 *   fscnn_pyramid_pool_*                          AdaptiveAvgPool2d(1,2,3,6) (:130-132)
 */
#ifndef FASTSCNN_H
#define FASTSCNN_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fscnn_net fscnn_net;
typedef struct fscnn_plan fscnn_plan;

const char* fscnn_version(void);
const char* fscnn_last_error(void);

/* ---- network: layer table + arena layout ------------------------------------------------ */
int fscnn_net_create(int num_classes, int aux, fscnn_net** out);
void fscnn_net_destroy(fscnn_net* net);
/* parameter arena (fp32, 64-B aligned tensors, named_parameters() order) */
int fscnn_net_param_count(const fscnn_net* net, int* count, long long* total_floats);
int fscnn_net_param_info(const fscnn_net* net, int i, const char** name, long long* offset,
                         long long* numel);
/* buffer arena: running_mean / running_var in a fp32 arena, num_batches_tracked in an int64
 * arena (for those entries *offset is the index into the int64 arena) */
int fscnn_net_buffer_count(const fscnn_net* net, int* count, long long* total_floats, int* num_bn);
int fscnn_net_buffer_info(const fscnn_net* net, int i, const char** name, long long* offset,
                          long long* numel);
/* backward stage s (0..3) finalises the gradients of parameters [begin, end) of the arena */
int fscnn_net_stage_range(const fscnn_net* net, int stage, long long* begin, long long* end);

/* ---- plan: shapes + workspace sizes for one (N, H, W, dtype, mode) ----------------------
 * train: 0 inference (BatchNorm folded, fused blocks), 1 training (batch statistics, running-stat
 * update, Dropout, staged backward), 2 differentiable inference (the training dataflow with
 * running-statistics BatchNorm: model.eval() under autograd) */
int fscnn_plan_create(const fscnn_net* net, int N, int H, int W, int dtype, int train,
                      fscnn_plan** out);
void fscnn_plan_destroy(fscnn_plan* plan);
int fscnn_plan_workspace(const fscnn_plan* plan, long long* fwd_bytes, long long* bwd_bytes);
int fscnn_plan_shapes(const fscnn_plan* plan, int* dims /* 10: H1 W1 H2 W2 H3 W3 H4 W4 H5 W5 */);
/* debug / stage-level parity: location of a named activation (e.g. "c2pw.a", "g_logits") in
 * the forward (in_bws = 0) or backward (in_bws = 1) workspace; rows x cols with row stride ld */
int fscnn_plan_buffer(const fscnn_plan* plan, const char* name, long long* offset, long long* rows,
                      int* cols, int* ld, int* in_bws);

/* ---- whole-network forward / backward ----------------------------------------------------- */
int fscnn_forward(const fscnn_plan* plan, const void* x, int x_dtype, void* out, int out_dtype,
                  const float* params, float* running, long long* nbt, void* ws,
                  unsigned long long dropout_seed, float dropout_p, float momentum,
                  void* stream);
int fscnn_backward(const fscnn_plan* plan, const void* dout, const void* x, int x_dtype,
                   const float* params, float* grads, void* ws, void* bws,
                   unsigned long long dropout_seed, float dropout_p, int stage_from,
                   int stage_to, void* stream);

/* General backward (any of the three heads above) that can also return the gradient of the input
 * image: autograd of x through the whole network (models/fast_scnn.py:33-46; the reference module
 * is differentiable in its input like any nn.Module).  Exactly one of dout (d logits, with daux for
 * an aux net) or grad_loss + loss2 (the fused loss head) is given.  dx: NCHW [N][3][H][W] in
 * dx_dtype (0 fp32, 1 bf16, 2 fp16), written by the stage-3 call, or null.
 * Plans: train = 1 (train-mode BatchNorm, batch statistics) or 2 (eval-mode autograd: every
 * BatchNorm normalised by its running statistics, Dropout off, no running-stat update; the
 * reference's model.eval() with grad enabled, e.g. eval.py:43). */
int fscnn_backward_dx(const fscnn_plan* plan, const void* dout, const void* daux,
                      const float* grad_loss, const float* loss2, const void* x, int x_dtype,
                      void* dx, int dx_dtype, const float* params, float* grads, void* ws,
                      void* bws, unsigned long long dropout_seed, float dropout_p, int stage_from,
                      int stage_to, void* stream);

/* FastSCNN(aux=True) (models/fast_scnn.py:24-31, 42-45): the same forward / backward plus the
 * auxiliary head (3x3 conv 64->32 + BN + ReLU + Dropout + 1x1 on the LearningToDownsample output,
 * upsampled like the main logits).  aux_out / daux: NCHW [N][C][H][W] in out_dtype.  Plans of an
 * aux net must use these entry points (fscnn_forward / fscnn_backward return -1;
 * fscnn_forward_loss covers the main output only and returns -2). */
int fscnn_forward_aux(const fscnn_plan* plan, const void* x, int x_dtype, void* out, void* aux_out,
                      int out_dtype, const float* params, float* running, long long* nbt,
                      void* ws, unsigned long long dropout_seed, float dropout_p, float momentum,
                      void* stream);
int fscnn_backward_aux(const fscnn_plan* plan, const void* dout, const void* daux, const void* x,
                       int x_dtype, const float* params, float* grads, void* ws, void* bws,
                       unsigned long long dropout_seed, float dropout_p, int stage_from,
                       int stage_to, void* stream);

/* Eval prediction (eval.py:43-45, demo.py:43-48 consume only torch.argmax(outputs[0], 1)):
 * forward of an inference plan whose final bilinear upsample is fused with the argmax over classes;
 * labels [N][H][W] (label_dtype 0: int64 like torch.argmax, 1: uint8).  No logits are written. */
int fscnn_predict(const fscnn_plan* plan, const void* x, int x_dtype, void* labels,
                  int label_dtype, const float* params, float* running, long long* nbt, void* ws,
                  void* stream);
/* SegmentationMetric counters (utils/metric.py:73-105, batch_pix_accuracy +
 * batch_intersection_union) of n predictions (pred_dtype 0 int64, 1 uint8) against int64 labels,
 * ACCUMULATED into counts[2 + 3*nclass] (int64): [correct, labeled, inter[C], area_pred[C],
 * area_lab[C]]; union = area_pred + area_lab - inter.  Exact integer counts. */
int fscnn_seg_metric(const void* pred, int pred_dtype, const long long* target, long long n,
                     int nclass, long long* counts, void* stream);

/* OHEM cross entropy (SoftmaxCrossEntropyOHEMLoss, utils/loss.py:127-176, the criterion of
 * train.py:190-191):
 * fscnn_ohem_prob: prob[i] = softmax probability of the label of pixel i (2.0 for ignored
 *   pixels); counts[0] += #labelled, counts[1] += #(prob <= thresh)  (device uint64 x 2).
 * fscnn_ohem_threshold: the whole threshold rule of utils/loss.py:159-170 on the device, from
 *   fscnn_ohem_prob's counters: *thr (device float) = inf when min_kept >= #labelled, else thresh,
 *   raised to the k-th smallest label probability (k = min(#labelled, min_kept)) when fewer than
 *   k labelled pixels have prob <= thresh.  work: 2056 uint32 device scratch.  No host sync
 *   (the reference's print of the label count on the first branch is not reproduced).
 * fscnn_ce_weighted_fwd / _bwd: nn.CrossEntropyLoss(weight, ignore_index) over the pixels with
 *   prob <= *thr (thr a device float; prob null: all labelled pixels; weight null: unweighted);
 *   out2 = (weighted mean loss, sum of weights); part as for fscnn_ce_fwd. */
int fscnn_ohem_prob(const void* logits, int dtype, const long long* target, int N, int C,
                    long long HW, long long ignore_index, float thresh, float* prob,
                    unsigned long long* counts, void* stream);
int fscnn_ohem_threshold(const float* prob, long long n, const unsigned long long* counts,
                         long long min_kept, float thresh, unsigned* work, float* thr, void* stream);
/* Deprecated (round 3): the host-driven k-th smallest of the OHEM rule was replaced by
 * fscnn_ohem_threshold, which keeps the threshold on the device.  Kept so old callers still link;
 * always returns -2 (unsupported) with a message naming the replacement. */
int fscnn_kth_smallest(const float* values, long long n, long long k, unsigned* hist, float* out,
                       void* stream);
int fscnn_ce_weighted_fwd(const void* logits, int dtype, const long long* target, int N, int C,
                          long long HW, long long ignore_index, const float* weight,
                          const float* prob, const float* thr, float* part, float* out2,
                          void* stream);
int fscnn_ce_weighted_bwd(const void* logits, int dtype, const long long* target, int N, int C,
                          long long HW, long long ignore_index, const float* weight,
                          const float* prob, const float* thr, const float* grad_out,
                          const float* out2, void* dlogits, void* stream);

/* Dice / Focal+Dice criteria (utils/loss.py:12-100; train.py:183-188, binary lane segmentation):
 * fscnn_dice_fwd writes stats[4] (device fp64) = (sum p1*t, sum p1, sum t, sum focal_i) with
 *   p1 = softmax(logits)[:, 1] (C > 1) or sigmoid (C == 1), t = float(target), focal_i =
 *   alpha (1 - pt)^gamma ce_i (only when focal != 0; C > 1); part: ce_parts(N, HW) * 4 floats.
 * fscnn_dice_bwd: d/dlogits of dice_weight * (1 - dice) + focal_weight * mean(focal), scaled by
 *   *grad_out (device). */
int fscnn_dice_fwd(const void* logits, int dtype, const long long* target, int N, int C,
                   long long HW, float alpha, float gamma, int focal, float* part, double* stats,
                   void* stream);
int fscnn_dice_bwd(const void* logits, int dtype, const long long* target, int N, int C,
                   long long HW, float alpha, float gamma, int focal, const double* stats,
                   const float* grad_out, float smooth, float dice_weight, float focal_weight,
                   void* dlogits, void* stream);

/* GPU input path.
 * fscnn_normalize_u8: transforms.ToTensor() + transforms.Normalize(mean, std) (train.py:104-107,
 *   eval.py:22-25, demo.py:37-40) of N uint8 HWC RGB images into the NCHW network input
 *   ((x / 255 - mean[c]) / std[c], torchvision's fp32 operation order); mean/std are HOST arrays
 *   of 3 floats; H*W must be a multiple of 4; out_dtype 0 fp32, 1 bf16.
 * fscnn_remap_labels: dataset label ids -> train ids through a device lookup table
 *   (data_loader/cityscapes.py:56-71 `_class_to_index` is lut = _key, offset = 1); ids outside
 *   the table become `invalid`. */
int fscnn_normalize_u8(const unsigned char* images, int N, int H, int W, const float* mean,
                       const float* std, void* out, int out_dtype, void* stream);
int fscnn_remap_labels(const unsigned char* labels, long long n, const long long* lut, int lut_size,
                       int offset, long long invalid, long long* out, void* stream);

/* Fused training step head (train plans only): forward + bilinear upsample + CE(ignore_index)
 * evaluated at low resolution; loss2[0] = mean loss, loss2[1] = valid pixel count.  Computes
 * exactly criterion(model(x)[0], target) of train.py:270-271 without materialising the
 * full-resolution logits.  backward_loss then takes d(loss) (device scalar) instead of
 * d(logits). */
int fscnn_forward_loss(const fscnn_plan* plan, const void* x, int x_dtype, const long long* target,
                       long long ignore_index, float* loss2, const float* params, float* running,
                       long long* nbt, void* ws, unsigned long long dropout_seed, float dropout_p,
                       float momentum, void* stream);
int fscnn_backward_loss(const fscnn_plan* plan, const float* grad_loss, const float* loss2,
                        const void* x, int x_dtype, const float* params, float* grads, void* ws,
                        void* bws, unsigned long long dropout_seed, float dropout_p,
                        int stage_from, int stage_to, void* stream);

/* ---- fused blocks (inference) ---------------------------------------------------------------
 * fscnn_block_ir_fwd: one stride-1 LinearBottleneck (models/fast_scnn.py:95-115) with its three
 * BatchNorms folded (eval): y = BN_p(W_p * relu(BN_d(dw3x3(relu(BN_e(W_e * x)))))) (+ x when
 * residual, which needs cin == cout).  x, y NHWC [N][H][W] with row strides ldx / ldy elements
 * (ldy may exceed cout: the PPM concat buffer); w_expand [expand][cin] and w_project
 * [cout][expand] in dtype (the nn.Conv2d weight layouts); w_dw [expand][9] fp32; scale_* / shift_*
 * fp32 per channel (BN folded as gamma/sqrt(var+eps), beta - mean*scale).  cin in {64, 96, 128},
 * expand a multiple of 64, cout a multiple of 16 <= 128.  The 6x-expanded tensor stays in LDS.
 * Replaces the three conv+BN(+ReLU) modules of LinearBottleneck.block (:103-108) and the
 * shortcut add (:113-114). */
int fscnn_block_ir_fwd(const void* x, int ldx, int dtype, int N, int H, int W, int cin, int expand,
                       int cout, const void* w_expand, const float* w_dw, const void* w_project,
                       const float* scale_e, const float* shift_e, const float* scale_d,
                       const float* shift_d, const float* scale_p, const float* shift_p,
                       int residual, void* y, int ldy, void* stream);

/* fscnn_block_ir_s2_fwd: the stride-2 LinearBottleneck (models/fast_scnn.py:95-115 with
 * stride 2: bottleneck1.0 and bottleneck2.0, no shortcut) in one inference launch:
 * y = BN_p(W_p * relu(BN_d(dw3x3_s2_p1(relu(BN_e(W_e * x)))))), every BN folded.  x NHWC
 * [N][H][W] x cin (row stride ldx), y NHWC [N][(H-1)/2+1][(W-1)/2+1] x cout (row stride ldy);
 * weights and BN tables as fscnn_block_ir_fwd.  The expanded tensor never reaches memory; the
 * executor uses it for the two stride-2 blocks of every eval plan with >= 128 output tiles. */
int fscnn_block_ir_s2_fwd(const void* x, int ldx, int dtype, int N, int H, int W, int cin,
                          int expand, int cout, const void* w_expand, const float* w_dw,
                          const void* w_project, const float* scale_e, const float* shift_e,
                          const float* scale_d, const float* shift_d, const float* scale_p,
                          const float* shift_p, void* y, int ldy, void* stream);

/* fscnn_block_ltd_fwd: the inference LearningToDownsample stem up to dsconv1 in one launch
 * (models/fast_scnn.py:153-154): y = BN_p(W_p * relu(BN_d(dw3x3_s2_p1(relu(BN_0(conv3x3_s2_p0(x)))))))
 * followed by ReLU, every BN folded (scale, shift fp32 per channel).  x NCHW [N][3][H][W] of
 * x_dtype (0 fp32, 1 bf16, 2 fp16; 16-B aligned, W a multiple of 16 B / element size); w_conv
 * [32][3][3][3] fp32, w_dw [32][9] fp32, w_pw [48][32] in dtype (the plan's storage type);
 * y NHWC [N][H2][W2] x 48 channels with row stride ldy elements (>= 48, multiple of 4), where
 * H1 = (H-3)/2+1, H2 = (H1-1)/2+1 (same for W).  conv0's and the depthwise output never reach
 * memory.  Replaces LearningToDownsample.conv (_ConvBNReLU, :52) and .dsconv1 (_DSConv, :64-78);
 * the executor uses it for every eval plan whose image fits these constraints. */
int fscnn_block_ltd_fwd(const void* x, int x_dtype, int dtype, int N, int H, int W,
                        const float* w_conv, const float* scale_0, const float* shift_0,
                        const float* w_dw, const float* scale_d, const float* shift_d,
                        const void* w_pw, const float* scale_p, const float* shift_p, void* y,
                        int ldy, void* stream);

/* fscnn_block_dsconv_fwd: an inference _DSConv (models/fast_scnn.py:64-79; the Classifer's
 * dsconv1 / dsconv2, :228-231) in one launch: y = relu(BN_p(W_p * relu(BN_d(dw3x3_s1_p1(x))))),
 * every BN folded (scale, shift fp32 per channel).  x NHWC [N][H][W] x C in dtype (rows of C
 * contiguous elements, 16-B aligned); w_dw [C][9] fp32, w_pw [Co][C] in dtype; y NHWC with row
 * stride ldy elements (>= Co, multiple of 4, 16-B aligned).  C = Co = 128 (E_UNSUPPORTED
 * otherwise).  The depthwise output never reaches memory.  Replaces _DSConv's dw conv + BN + ReLU
 * and pw conv + BN + ReLU (two launches of the unfused eval path); the executor uses it for the
 * classifier's two DSConvs of every eval plan. */
int fscnn_block_dsconv_fwd(const void* x, int dtype, int N, int H, int W, int C, int Co,
                           const float* w_dw, const float* scale_d, const float* shift_d,
                           const void* w_pw, const float* scale_p, const float* shift_p, void* y,
                           int ldy, void* stream);

/* fscnn_block_dsconv_res_fwd: the same with a residual added after the pointwise BN, before the
 * final ReLU: y = relu(BN_p(W_p * relu(BN_d(dw3x3(up(x))))) + res) -- the FeatureFusionModule's
 * F.interpolate(scale 4, bilinear, align_corners) + dwconv + conv_lower_res + the high-res branch
 * (models/fast_scnn.py:207-218).  Hi > 0: x is [N][Hi][Wi] x C and up() its bilinear
 * align_corners resize to H x W, formed in LDS and never stored (same arithmetic as the unfused
 * up_nhwc); Hi = 0: up() is the identity and x is [N][H][W] x C.  res NHWC with row stride ldres
 * (>= Co, multiple of 4, 16-B aligned); res may alias y (each element is read before it is
 * written, by the same thread). */
int fscnn_block_dsconv_res_fwd(const void* x, int dtype, int N, int H, int W, int C, int Co,
                               int Hi, int Wi, const float* w_dw, const float* scale_d, const float* shift_d,
                               const void* w_pw, const float* scale_p, const float* shift_p,
                               const void* res, int ldres, void* y, int ldy, void* stream);

/* fscnn_block_cls_fwd: the inference Classifer (models/fast_scnn.py:221-237; Dropout is the
 * identity in eval) in two launches: tmp = dsconv1(x) (fscnn_block_dsconv_fwd), then dsconv2 and
 * the 1x1 classifier conv (+ bias) in one launch whose 128-channel dsconv2 output never reaches
 * memory: logits = W_cls * dsconv2(tmp) + b_cls.  x and tmp NHWC [N][H][W] x 128 in dtype
 * (16-B aligned); w_dw* [128][9] fp32, w_pw* [128][128] and w_cls [ncls][128] in dtype, b_cls
 * [ncls] fp32, every BN folded to (scale, shift) fp32; logits NHWC [N][H][W] x ncls with row
 * stride ldl (>= ncls; ncls <= 32), only the first ncls columns written.  Replaces the
 * Classifer's dw / pw / dw / pw / conv launches of the unfused eval path; bit-identical to them. */
int fscnn_block_cls_fwd(const void* x, int dtype, int N, int H, int W, const float* w_dw1,
                        const float* scale_d1, const float* shift_d1, const void* w_pw1,
                        const float* scale_p1, const float* shift_p1, const float* w_dw2,
                        const float* scale_d2, const float* shift_d2, const void* w_pw2,
                        const float* scale_p2, const float* shift_p2, const void* w_cls,
                        const float* b_cls, int ncls, void* tmp, void* logits, int ldl,
                        void* stream);

/* fscnn_block_ffm_fwd: the inference FeatureFusionModule (models/fast_scnn.py:200-218) in one
 * launch: y = relu(BN_l(W_l * relu(BN_d(dw3x3(up(low))))) + BN_h(W_h * high)).  low NHWC
 * [N][Hi][Wi] x 128 (the global feature extractor's output; up() its bilinear align_corners resize
 * to H x W, formed in LDS); high NHWC [N][H][W] x 64 with row stride ldhigh (>= 64, multiple of
 * 8, 16-B aligned; LearningToDownsample's output); w_dw [128][9] fp32, w_low [128][128] and
 * w_high [128][64] in dtype; every BN folded to (scale, shift) fp32.  Neither the upsampled
 * input, the depthwise output nor the high-res branch's output reaches memory.  Replaces
 * F.interpolate + dwconv + conv_lower_res + conv_higher_res + add + ReLU (four launches of the
 * unfused eval path); the executor uses it for the FFM of every eval plan (FSCNN_FFM_HI=0 keeps
 * the high-res branch as its own GEMM and fscnn_block_dsconv_res_fwd), bit-identical to them. */
int fscnn_block_ffm_fwd(const void* low, int dtype, int N, int Hi, int Wi, int H, int W,
                        const void* high, int ldhigh, const float* w_dw, const float* scale_d,
                        const float* shift_d, const void* w_low, const float* scale_l,
                        const float* shift_l, const void* w_high, const float* scale_h,
                        const float* shift_h, void* y, int ldy, void* stream);

/* ---- launch profiler (bench.py roofline, tools/layer_report.py) ----------------------------
 * kind: 1 conv0_fwd, 2 dw_fwd, 3 dw_dgrad, 4 dw_wgrad, 5 gemm_nt, 6 gemm_tn, 7 bn_apply,
 * 8 bn_bwd (apply), 9 upsample, 10 upsample_bwd, 11 cross_entropy / fused loss head,
 * 12 conv0_wgrad, 13 bn_bwd_reduce, 14 bn_finalize, 15 ppm_branches (the four pyramid-pooling
 * branch convs + BN + ReLU, one launch each way), 16 ir_block (fused inference bottleneck),
 * 17 ltd_stem (fused inference stem), 18 dsconv (fused inference DSConv);
 * 100 = every kind.
 * Between begin and end every launch of that kernel family is bracketed by hipEvents bound to its
 * dispatch (hipExtLaunchKernelGGL); end synchronises and returns summed kernel ms,
 * launch count and the algorithmic bytes
 * and flops of those launches (SURVEY.md §8(d) formulas); fscnn_prof_launch then returns launch
 * i's kind, ms, bytes, flops and layer (reference module name; issue order). */
int fscnn_prof_begin(int kind, int max_launches);
int fscnn_prof_end(double* total_ms, long long* launches, double* bytes, double* flops);
int fscnn_prof_launch(long long i, int* kind, float* ms, double* bytes, double* flops,
                      const char** layer);
const char* fscnn_prof_kind_name(int kind);
/* Debug: phase stamps of the next launches of the instrumented kernels (pointwise GEMMs, depthwise
 * forward / stride-1 dgrad): per-wave 100 MHz wall clock at fixed points of the kernel
 * (tools/stamp_probe.py).  Launch i writes buf + i * 262144 uint64 (8192 workgroups x 4 waves x
 * 8 slots), up to max_launches; null: off.  fscnn_debug_stamp_count / _tag: launches recorded and
 * each one's layer label.  Process-global, single-threaded measurement only. */
int fscnn_debug_stamps(void* buf, int max_launches);
int fscnn_debug_stamp_count(void);
const char* fscnn_debug_stamp_tag(int i);

/* ---- loss / optimizer ------------------------------------------------------------------- */
/* out2[0] = mean loss over valid pixels, out2[1] = valid count; part: ce_parts*2 floats */
long long fscnn_ce_parts(int N, long long HW);
int fscnn_ce_fwd(const void* logits, int dtype, const long long* target, int N, int C,
                 long long HW, long long ignore_index, float* part, float* out2, void* stream);
int fscnn_ce_bwd(const void* logits, int dtype, const long long* target, int N, int C,
                 long long HW, long long ignore_index, const float* grad_out,
                 const float* out2, void* dlogits, void* stream);
int fscnn_sgd(float* p, const float* g, float* buf, long long n, float lr, float momentum,
              float dampening, float weight_decay, int nesterov, int first, float grad_scale,
              void* stream);

/* ---- individual kernels (per-op parity tests) ------------------------- */
int fscnn_conv0_fwd(const void* x, int x_dtype, int N, int H, int W, const float* w,
                    const float* scale, const float* shift, int relu, void* y, int y_dtype,
                    void* stream);
/* dW [32][3][3][3] of the first conv from the NCHW image and NHWC dZ [N][Ho][Wo][32]
 * (autograd of models/fast_scnn.py:153); slab: fscnn_conv0_wgrad_slab_floats floats */
long long fscnn_conv0_wgrad_slab_floats(int N, int H, int W);
int fscnn_conv0_wgrad(const void* x, int x_dtype, int N, int H, int W, const void* dz,
                      int dz_dtype, float* slab, float* dw, void* stream);
int fscnn_dw3x3_fwd(const void* x, int dtype, int N, int H, int W, int C, int stride,
                    const float* w, const float* scale, const float* shift, int relu, void* y,
                    void* stream);
int fscnn_dw3x3_dgrad(const void* dy, int dtype, int N, int H, int W, int C, int stride,
                      const float* w, void* dx, void* stream);
long long fscnn_dw3x3_wgrad_slab_floats(int N, int H, int W, int C, int stride, int dtype);
int fscnn_dw3x3_wgrad(const void* x, const void* dy, int dtype, int N, int H, int W, int C,
                      int stride, float* slab, float* dw, void* stream);
/* C[M][N] = act((A[M][K] . B^T) * scale + shift (+ R)); B is [N][K] (b_trans=0) or [K][N].
 * stats_part (train BN statistics of the output, before R / relu): room for ceil(M/128)
 * records [P][3][N]; the call writes fscnn_pw_gemm_stats_parts(...) of them (pass that count as
 * P to fscnn_bn_finalize). */
int fscnn_pw_gemm_stats_parts(int M, int N, int K, int lda, int ldc, int dtype);
int fscnn_pw_gemm(int M, int N, int K, const void* A, int lda, const void* B, int ldb,
                  int b_trans, const float* scale, const float* shift, const void* R, int ldr,
                  int relu, void* C, int ldc, float* stats_part, int dtype, void* stream);
/* Training dgrad of a 1x1 conv whose output is the dy of a BatchNorm (the form the executor runs
 * for every LinearBottleneck expand dgrad, models/fast_scnn.py:103-104 autograd):
 *   dX[M][N] = D[M][K] . B^T (+ R), B [N][K] (the transposed conv weight, row stride ldb),
 * plus that BN's backward reduction over the STORED (rounded) dX, finished in the same call:
 *   dbeta[n] = sum_m dX*mask, dgamma[n] = sum_m dX*mask*(z - mean[n])*invstd[n],
 *   coef[n] = dbeta[n] / M, coef[N + n] = dgamma[n] / M,
 * mask = 1 (relu_mode 0) or (z*scale[n] + shift[n] > 0) (relu_mode 2: the BN feeds a ReLU).
 * z [M][N] (ld ldz) is the BN's forward input.  Scratch: part >= ceil(M/128)*2*N floats,
 * counters 512 zeroed uint32 (left zero), tsum 32*3*1024 doubles.  *path (nullable): 1 when the
 * streaming kernel ran (deep-K form for 16-bit K = 384 / 512 / 576 at M >= 131072), 0 tiled. */
int fscnn_pw_dgrad_bnbwd(int M, int N, int K, const void* D, int ldd, const void* B, int ldb,
                         const void* R, int ldr, void* dX, int lddx, const void* z, int ldz,
                         const float* mean, const float* invstd, const float* scale,
                         const float* shift, int relu_mode, float* part, unsigned* counters,
                         double* tsum, float* dgamma, float* dbeta, float* coef, int dtype,
                         int* path, void* stream);
long long fscnn_pw_wgrad_slab_floats(int M, int N, int K);
/* dW[N][K] = sum_m D[m][n] X[m][k] */
int fscnn_pw_wgrad(int M, int N, int K, const void* D, int ldd, const void* X, int ldx,
                   float* slab, float* dW, int dtype, void* stream);
/* part [P][3][C] is consumed (folded in place) */
int fscnn_bn_finalize(float* part, int P, int C, const float* gamma, const float* beta,
                      float* rmean, float* rvar, long long* nbt, float momentum, float* mean,
                      float* invstd, float* scale, float* shift, void* stream);
int fscnn_bilinear_ac_fwd(const void* x, int dtype, int N, int Hi, int Wi, int C, int Ho, int Wo,
                          void* y, int out_nchw, int out_dtype, void* stream);
/* NHWC grad wrt output [N][Ho][Wo][C] -> NHWC grad wrt input [N][Hi][Wi][C] (fp32 tmp) */
int fscnn_bilinear_ac_bwd(const void* dy, int dtype, int N, int Hi, int Wi, int C, int Ho, int Wo,
                          float* tmp, void* dx, void* stream);
int fscnn_pyramid_pool_fwd(const void* x, int dtype, int N, int H, int W, int C, int ldx,
                           void* pooled, void* stream);
int fscnn_pyramid_pool_bwd(const void* dpooled, int dtype, int N, int H, int W, int C, void* dx,
                           int lddx, int accumulate, void* stream);

#ifdef __cplusplus
}
#endif
#endif
