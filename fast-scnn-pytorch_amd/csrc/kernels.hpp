// Argument structs and host launchers of every Fast-SCNN HIP kernel (csrc/*.hip).
// The executor (net.cpp) and the C ABI (capi.cpp) call these; each returns 0 or a negative
// fscnn::Status with the message available from fscnn::last_error().
#pragma once
#include "common.hpp"

namespace fscnn {

constexpr int MAX_FOLD = 48;  // (45 BatchNorms with the aux head; the table is a kernel argument)
// BN-backward element count of a BatchNorm normalised with its running statistics (plans with
// train == 2, eval-mode autograd): bn_bwd_finish then drops the batch-mean terms
constexpr double BN_FROZEN_COUNT = -1.0;


struct Conv0Args {
  const void* x;       // NCHW [N,3,H,W]
  int x_bf16;          // input dtype code: 0 fp32, 1 bf16, 2 fp16
  int N, H, W, Ho, Wo;
  const float* w;      // [32][3][3][3]
  const float* scale;  // [32] or null (eval BN fold)
  const float* shift;  // [32] or null
  int relu;
  void* y;             // NHWC [N,Ho,Wo,32]
  float* part;         // BN partial records [part][3][32] or null
  unsigned long long* stamps = nullptr;  // (set by the launcher) phase stamps
};

struct Conv0WgradArgs {
  const void* x;
  int x_bf16;          // input dtype code: 0 fp32, 1 bf16, 2 fp16
  int N, H, W, Ho, Wo;
  const void* dz;  // NHWC [N,Ho,Wo,32] (dy when zz is set)
  float* slab;     // [parts][864]
  int rows_per_block;
  const void* zz = nullptr;   // BN backward applied on load: z [N,Ho,Wo,32], tab [32][8]
  const float* tab = nullptr;
};

struct BnFinalizeArgs {
  float* part;        // [P][3][C] (mean, M2, count); consumed (folded in place)
  int P, C;
  const float* gamma;
  const float* beta;
  float* rmean;       // running stats, updated in place (or null)
  float* rvar;
  long long* nbt;     // num_batches_tracked (or null)
  float momentum;
  const float* bias;  // conv bias to add to the batch mean (stats taken before the bias) or null
  float* mean;        // [C] saved for backward
  float* invstd;      // [C]
  float* scale;       // [C] gamma*invstd
  float* shift;       // [C] beta - mean*scale
  unsigned* counters = nullptr;  // >= cdiv(C,64) zeroed arrival counters: one-launch fold+finalize
};

struct BnBwdTab {
  float* tab = nullptr;
  const float* scale = nullptr;
  const float* shift = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  int relu = 0;
};

// In-kernel BatchNorm finish of a GEMM producer: the last-arriving workgroup of each column
// group folds that group's records and writes the finished per-channel values, so no separate
// finalize launch sits between producer and consumer.  Forward (GemmArgs::part): fwd's gamma ..
// shift (part / P / C / counters are the GEMM's own).  Backward (GemmArgs::bpart): dgamma /
// dbeta into the gradient arena, the apply coefficients coef [2][C] and, when tab.tab is set,
// the BN-backward operand table.  When gemm_nt takes its tiled path it runs the separate
// finalize itself, so callers see the same result either way.
constexpr int BN_COUNTERS = 512;  // arrival counters per direction (zeroed each step)
struct BnTail {
  unsigned* counters = nullptr;  // BN_COUNTERS zeroed counters; null: no finish (records only)
  BnFinalizeArgs fwd{};
  double count = 0.0;
  float* dgamma = nullptr;
  float* dbeta = nullptr;
  float* coef = nullptr;
  BnBwdTab tab{};
  // fp64 team sums of the generic in-kernel finish (bn_finish.hpp tail_finish), >= TAIL_TMAX *
  // 3 * C doubles; null: that finish is not used (the producer falls back to a finalize launch)
  double* tsum = nullptr;
};

// BatchNorm-backward partial sums of a dgrad's OUTPUT, when that output is the dy of a BN
// (the mirror of GemmArgs::bpart): per workgroup, s1[c] = sum g*mask, s2[c] = sum
// g*mask*(z-mean)*invstd of the stored (rounded) output g, the mask recomputed from that BN's z
struct BnBwdPart {
  float* part = nullptr;        // [P][2][C] or null
  const void* z = nullptr;      // that BN's pre-BN tensor, NHWC with ld C
  const float* mean = nullptr;
  const float* invstd = nullptr;
  const float* scale = nullptr;  // forward BN affine (mode 2: mask = fmaf(z, scale, shift) > 0)
  const float* shift = nullptr;
  int mode = 0;                  // 0 no ReLU, 2 relu_z
};

struct DwArgs {
  int N, H, W, C, Ho, Wo, stride;
  const void* x;   // NHWC [N,H,W,C] (input activation)
  const float* w;  // [C][3][3] fp32 master weights
  const float* scale;  // eval BN fold, or null
  const float* shift;
  int relu;
  void* y;         // NHWC [N,Ho,Wo,C]
  float* part;     // BN partial records [parts][3][C] or null
  // lazily applied BN+ReLU of x (train: x is the producer's raw conv output z) or null
  const float* in_scale = nullptr;
  const float* in_shift = nullptr;
  BnBwdPart bs{};  // stride-1 dgrad (the flipped forward): BN-backward partials of y
  // BN finish of the records this launch writes (part: forward statistics; bs.part: stride-1
  // dgrad partials): tail.counters set -> dw_fwd finishes the BN, in the kernel's last
  // workgroups when the records fit (tail_ink, set by the launcher) or as its own launch
  BnTail tail{};
  int tail_ink = 0;
  unsigned long long* stamps = nullptr;  // (set by the launcher) phase stamps
};

struct DwBwdArgs {
  int N, H, W, C, Ho, Wo, stride;
  const void* x;    // forward input activation (wgrad)
  const void* dy;   // NHWC [N,Ho,Wo,C]
  const float* w;   // [C][9]
  void* dx;         // NHWC [N,H,W,C] (dgrad)
  float* slab;      // [parts][9][C] (wgrad)
  const float* x_scale = nullptr;  // lazily applied BN+ReLU of x (wgrad) or null
  const float* x_shift = nullptr;
  BnBwdPart bs{};  // dgrad: BN-backward partials of dx (dw_dgrad_parts records)
  BnTail tail{};     // dgrad: finish of the bs.part BN (see DwArgs::tail)
  int tail_ink = 0;
};

struct GemmArgs {
  int M, N, K;
  const void* A;
  int lda;
  const void* B;
  int ldb;
  int b_trans;          // 0: Bk(n,k) = B[n*ldb+k]   1: Bk(n,k) = B[k*ldb+n]
  const float* scale;   // [N] or null
  const float* shift;   // [N] or null
  const void* R;        // residual [M][N] (ldr) or null; may alias C
  int ldr;
  int relu;
  void* C;
  int ldc;
  float* part;          // BN partial records [gridDim.x][3][N] or null
  // Fused BatchNorm-backward partial sums of the OUTPUT, when this GEMM produces the dy of a BN
  // (dgrad): per 128-row tile, s1[n] = sum g*mask, s2[n] = sum g*mask*(z-mean)*invstd with g the
  // stored (rounded) output.  bpart [cdiv(M,128)][2][N] or null.
  float* bpart = nullptr;
  const void* bz = nullptr; int ldbz = 0;        // z of that BN (pre-BN forward tensor)
  const float* bmean = nullptr; const float* binvstd = nullptr;
  const float* bscale = nullptr; const float* bshift = nullptr;  // forward BN affine (mode 2)
  int bmode = 0;        // 0 no ReLU, 2 relu_z: mask = fmaf(z, bscale, bshift) > 0
  // lazily applied BN+ReLU of the A operand (train forward: A is the producer's raw conv output
  // z, the GEMM consumes relu(fmaf(z, a_scale[k], a_shift[k]))) or null
  const float* a_scale = nullptr;
  const float* a_shift = nullptr;
  BnTail tail{};        // in-kernel finish of the BN whose records this GEMM writes
  int tail_ink = 0;     // (set by the launcher) the tiled kernel runs the finish itself (tail_finish)
  // Dropout of the OUTPUT (train backward of the classifier's Dropout, models/fast_scnn.py:235:
  // the dgrad stores keep ? round(out) / (1 - drop_p) : 0, the dropout kernel's law, so its BN
  // partials (bpart) are those of the dropped gradient).  The mask hashes the NCHW index of
  // output element (m = n * drop_hw + hw, channel c); drop_hw 0: none.  Streaming kernel only.
  int drop_hw = 0;
  uint32_t drop_thr = 0;
  float drop_p = 0.f;
  uint64_t drop_seed = 0;                    // seed (+ drop_seed_add) or the device slot below
  const uint64_t* drop_seed_ptr = nullptr;
  uint64_t drop_seed_add = 0;
  unsigned long long* stamps = nullptr;  // (set by the launcher from g_stamps) phase stamps
};

struct GemmTnArgs {
  int M, N, K;
  const void* D;
  int ldd;
  const void* X;
  int ldx;
  float* slab;   // [splits][N][K]
  int rows_per_split;
  int splits;
  const float* x_scale = nullptr;  // lazily applied BN+ReLU of X (see GemmArgs::a_scale) or null
  const float* x_shift = nullptr;
};

struct FoldEntry {
  const float* gamma;
  const float* beta;
  const float* rmean;
  const float* rvar;
  const float* bias;  // conv bias folded in, or null
  float* scale;
  float* shift;
  int C;
  // running-statistics BN of a differentiable eval forward (train == 2 plans): the constants
  // the backward's x_hat uses, mean = running_mean, invstd = 1 / sqrt(running_var + eps), or null
  float* mean = nullptr;
  float* invstd = nullptr;
};

struct FoldTable {
  int n;
  FoldEntry e[MAX_FOLD];
};


struct BnApplyArgs {
  long long M;
  int C;
  const void* z;  int ldz;
  const float* scale; const float* shift;
  const void* z2; int ldz2;           // optional second affine branch (FFM)
  const float* scale2; const float* shift2;
  const void* res; int ldres;         // optional residual (LinearBottleneck shortcut)
  int relu;
  void* y; int ldy;
};

struct BnBwdArgs {
  long long M;
  int C;
  const void* dy; int lddy;
  const void* mask; int ldmask;   // null: no ReLU (unless relu_z)
  const void* z; int ldz;
  const float* mean; const float* invstd; const float* scale;
  const float* shift;             // forward shift (relu_z)
  int relu_z;                     // mask = fmaf(z, scale, shift) > 0, recomputed (no mask read)
  float* part;                    // [P][2][C]: sum dy_r, sum dy_r*xhat
  int rows_per_block;
  // apply
  const float* coef;              // [2][C]: mean(dy_r), mean(dy_r*xhat) (train) — null in eval
  void* dz; int lddz;
  // a second BN with the same dy and mask (FeatureFusionModule: relu(BN_l(z_l) + BN_h(z_h))):
  // z2 / mean2 / invstd2 / scale2 [C], records part2 [P][2][C] (its s1 equals the first BN's),
  // coef2 and dz2 (ld lddz) — one pass reads dy and the mask once for both BNs (mask mode only)
  const void* z2 = nullptr;
  const float* mean2 = nullptr; const float* invstd2 = nullptr; const float* scale2 = nullptr;
  float* part2 = nullptr;
  const float* coef2 = nullptr;
  void* dz2 = nullptr;
};

struct UpArgs {
  int N, Hi, Wi, C, Ho, Wo;
  const void* x; int ldx;   // NHWC, ldx = row stride (elements) >= C
  void* y; int ldy;         // NHWC slice, ldy >= C
};

struct AxisBwdArgs {
  long long n_o1;
  int n_o2;
  int Lout, Lin;
  long long n_in;
  const void* g;
  long long g_s1, g_s2, g_idx, g_in;
  void* d;
  long long d_s1, d_s2, d_idx, d_in;
  int accumulate;
};

struct PoolArgs {
  int N, H, W, C;
  const void* x; int ldx;   // NHWC (channel slice)
  void* pooled;             // bin-major [50][N][C], storage type
};

struct PoolBwdArgs {
  int N, H, W, C;
  const void* dpooled;  // bin-major [50][N][C]
  void* dx; int lddx;
  int accumulate;
};

struct PpmUpArgs {
  int N, H, W, CF;
  const void* feats;
  void* y; int ldy; int coff;
};

// PPM branch convs in one launch (ppm.hip): training, one workgroup per branch; inference, one
// wave per 16-row tile
struct PpmBranchFwd {
  BnFinalizeArgs f;  // gamma / beta / running statistics -> mean / invstd / scale / shift
  const void* x;     // pooled rows [M][K]
  const void* w;     // [32][K], storage type
  void* z;           // [M][32] conv output
  void* y;           // relu(BN(z)) [M][ldy]
  int ldy, M;
};
struct PpmFwdArgs {
  PpmBranchFwd b[4];
  int nb, K, C;
  int eval = 0;  // inference: y = relu(z * f.scale + f.shift) (folded BN), no z, no statistics
  unsigned long long* stamps = nullptr;  // phase stamps (tools/stamp_probe.py)
};
struct PpmBranchBwd {
  const void* dy; int lddy;  // gradient of y
  const void* y; int ldy;    // forward output (its ReLU mask)
  const void* z;             // [M][32]
  const float *mean, *invstd, *scale;  // (the forward's; the backward recomputes them in fp64)
  const float* gamma;        // BN weight [32]
  const void* x;             // pooled rows [M][K]
  const void* w;             // [32][K], storage type
  float *dgamma, *dbeta;     // [32]
  float* dw;                 // [32][K] fp32, stored
  void* dx;                  // [M][K]
  int M;
};
struct PpmBwdArgs {
  PpmBranchBwd b[4];
  int nb, K, C;
  int wg0[5] = {0, 0, 0, 0, 0};  // (set by the launcher) first workgroup of each branch
  unsigned long long* stamps = nullptr;  // phase stamps (tools/stamp_probe.py)
};

struct CeArgs {
  int N, C;
  long long HW;
  const void* logits;     // [N][C][HW]
  const long long* target;  // [N][HW]
  long long ignore_index;
  float* part;            // [P][2]: sum of loss, count of valid pixels
  // backward
  const float* scale;     // device scalar: grad_out / count (computed by ce_finalize)
  void* dlogits;          // [N][C][HW] or null
  // OHEM (utils/loss.py:127-176): class weights [C] (weighted mean: sum w*nll / sum w) and the
  // kept mask prob[i] <= *thr (prob from ohem_prob, thr a device scalar); null = plain CE
  const float* weight = nullptr;
  const float* prob = nullptr;
  const float* thr = nullptr;
};

// Fused training head: bilinear(align_corners) upsample of the low-res logits to the input
// resolution + cross-entropy(ignore_index) + its gradient back to the low-res logits, without
// materialising full-resolution logits.  g_raw receives sum_pixels w * (softmax - onehot)
// (unscaled); loss partials per workgroup.
struct CeHeadArgs {
  int N, C, Hl, Wl, H, W;
  const void* logits;        // NHWC [N][Hl][Wl][ldl]
  int ldl;
  const long long* target;   // [N][H][W]
  long long ignore_index;
  float* g_raw;              // 2 planes NHWC [N][Hl][Wl][ldl] fp32: own row, spill from row above
  float* part;               // [N * Hl][2]
  unsigned long long* stamps = nullptr;
  // optional: the targets packed to int8 (class or -1; ce_pack_targets), read by the 16-bit
  // kernels 4 rows ahead instead of the int64 rows
  const signed char* tgt8 = nullptr;
};

struct DropArgs {
  int N, H, W, C;
  const void* x; int ldx;
  void* y; int ldy;
  uint64_t seed;
  float p;
  const uint64_t* seed_ptr = nullptr;  // device slot holding the seed (graph-replayable), or null
  uint64_t seed_add = 0;               // mask seed = seed + seed_add (aux head Dropout: +1)
  // x is the raw conv output z of a BN+ReLU that is never stored: the kernel drops out
  // relu(fmaf(z, x_scale[c], x_shift[c])) (bn_apply's arithmetic), or null
  const float* x_scale = nullptr;
  const float* x_shift = nullptr;
};

// aux head 3x3 conv as im2col + GEMM (aux.hip): col[m][c*9 + kh*3 + kw], pad 1, stride 1
struct Im2ColArgs {
  int N, H, W, C;
  const void* x; int ldx;    // NHWC [N][H][W][ldx]
  void* col; int ldcol;      // [N*H*W][ldcol], ldcol >= 9*C
};
struct Col2ImArgs {
  int N, H, W, C;
  const void* dcol; int ldcol;
  void* dx; int lddx;
  int accumulate;            // dx += (else dx =)
};

struct SgdArgs {
  long long n;
  float* p;
  const float* g;
  float* buf;
  float lr, momentum, dampening, weight_decay;
  int nesterov, first;
  float grad_scale;  // multiply g first (e.g. 1/world_size); 1 = none
};

// ---- launchers ----------------------------------------------------------------------------
// fused stride-1 inverted-residual block, inference (ir.hip; models/fast_scnn.py:95-115)
struct IrArgs {
  int N, H, W;                 // output map (stride 1: = the input map)
  int stride = 1;              // 1, or 2 (bottleneck1.0 / 2.0: no residual)
  int Hi = 0, Wi = 0;          // input map (0: = H, W)
  int Cin, E, Cout;            // block input, expanded (6 Cin), output channels
  const void* x; int ldx;      // NHWC block input (storage dtype)
  void* y; int ldy;            // NHWC block output
  const void* we;              // expand weights [E][Cin] (storage dtype)
  const float* wd;             // depthwise weights [E][9] (fp32)
  const void* wp;              // project weights [Cout][E] (storage dtype)
  const float *sc_e, *sh_e, *sc_d, *sh_d, *sc_p, *sh_p;  // folded eval BatchNorms
  int residual;                // + x (stride 1, Cin == Cout)
  // fp32 plans: the expand / project weights already split into three bf16 planes
  // ([3][E][Cin], [3][Cout][E]; weights_prep mode 3), or null (the kernel splits them)
  const uint16_t* we3 = nullptr;
  const uint16_t* wp3 = nullptr;
  // training form (ir_train_fwd: expand recomputed + depthwise, no project): the input's lazily
  // applied BN + ReLU (or null), sc_e / sh_e = BN_e's batch-statistics table, y = the depthwise's
  // pre-BN output [N,H,W][ldy] and part = its BN records [tiles][3][E]
  const float* x_scale = nullptr;
  const float* x_shift = nullptr;
  float* part = nullptr;
};
bool ir_block_ok(const IrArgs& a, int dtype);
int ir_block_fwd(const IrArgs& a, int dtype, hipStream_t st);
bool ir_train_ok(const IrArgs& a, int dtype);
long long ir_train_parts(int N, int H, int W, int stride);
int ir_train_fwd(const IrArgs& a, int dtype, hipStream_t st);

// inference LearningToDownsample stem (stem.hip): conv0 + BN + ReLU -> dsconv1.dw + BN + ReLU ->
// dsconv1.pw + BN + ReLU in one launch (models/fast_scnn.py:153-154), BatchNorms folded
struct StemArgs {
  const void* x; int x_dtype;  // NCHW [N,3,H,W] image: 0 fp32, 1 bf16, 2 fp16 (16-B aligned, W % 16 B)
  int N, H, W;
  int H1, W1, H2, W2;          // conv0 (3x3 s2 p0) and dsconv1 (3x3 s2 p1) output maps
  const float* w0;             // conv0 weights [32][27] fp32
  const float *sc0, *sh0;      // folded BN of conv0
  const float* wd;             // dsconv1.dw weights [32][9] fp32
  const float *scd, *shd;      // folded BN of dsconv1.dw
  const void* wp;              // dsconv1.pw weights [48][32] in the storage dtype
  const float *scp, *shp;      // folded BN of dsconv1.pw
  void* y; int ldy;            // NHWC [N,H2,W2] x 48 channels (row stride ldy elements)
  unsigned long long* stamps = nullptr;  // (set by the launcher) phase stamps
};
bool stem_ok(const StemArgs& a);
int stem_fwd(const StemArgs& a, int dtype, hipStream_t st);

// ---- inference DSConv: dw 3x3 s1 p1 + BN + ReLU -> 1x1 + BN + ReLU in one launch (dsconv.hip) --
struct DsArgs {
  const void* x;               // NHWC [N,H,W] x C (contiguous rows of C elements), storage dtype
  int N, H, W, C, Co;          // C = Co = 128 (the Classifer's _DSConv)
  const float* wd;             // depthwise weights [C][9] fp32
  const float *scd, *shd;      // folded BN of the depthwise
  const void* wp;              // pointwise weights [Co][C] in the storage dtype
  const float *scp, *shp;      // folded BN of the pointwise
  void* y; int ldy;            // NHWC [N,H,W] x Co (row stride ldy elements)
  const void* r = nullptr;     // optional residual added after the pointwise BN, before its ReLU
  int ldr = 0;                 // (the FFM: relu(BN_l(conv_l(dw)) + f), :213-218); may alias y
                               // (or xh below)
  int rs;                      // output rows walked per workgroup (ds_rows)
  // optional classifier 1x1 (+ bias) on the pointwise output (the Classifer's last conv,
  // :233-236, Dropout the identity in eval): logits [N,H,W] x ncls (row stride ldl) written
  // instead of y; the pointwise output never reaches memory
  const void* wc = nullptr;    // [ncls][Co] in the storage dtype (ncls <= 32)
  const float* bc = nullptr;   // [ncls] fp32 bias
  int ncls = 0;
  void* logits = nullptr; int ldl = 0;
  int Hi = 0, Wi = 0;          // > 0: x is [N,Hi,Wi] x C and the depthwise input is its bilinear
                               // align_corners upsample to H x W (the FFM's F.interpolate, :212),
                               // formed in LDS, never stored (up_nhwc's arithmetic)
  // optional high-resolution branch computed in the launch and used as the residual (the FFM's
  // conv_higher_res + BN, :214-215; requires Hi > 0 and r == nullptr): BN_h(W_h * xh), its
  // 128-channel output never stored
  const void* xh = nullptr;    // NHWC [N,H,W] x 64 (row stride ldxh elements), storage dtype
  int ldxh = 0;
  const void* wh = nullptr;    // [Co][64] in the storage dtype
  const float *sch = nullptr, *shh = nullptr;  // folded BN of the high-res branch
  unsigned long long* stamps = nullptr;  // (set by the launcher) phase stamps
};
bool ds_ok(const DsArgs& a);
// inference LearningToDownsample.dsconv2 (dsconv.hip ds2_fwd): depthwise 3x3 s2 p1 over 48
// channels + folded BN + ReLU, pointwise 48 -> 64 + folded BN + ReLU, one launch
struct Ds2Args {
  const void* x;             // NHWC [N,H,W] x 48, contiguous, storage dtype
  int N, H, W, Ho, Wo;
  const float* wd;           // depthwise weights [48][9] fp32
  const float *scd, *shd;    // its folded BN
  const void* wp;            // pointwise weights [64][48], storage dtype
  const float *scp, *shp;    // its folded BN
  void* y; int ldy;          // NHWC [N,Ho,Wo] x 64 (row stride ldy)
  unsigned long long* stamps = nullptr;
};
bool ds2_ok(const Ds2Args& a);
int ds2_fwd(const Ds2Args& a, int dtype, hipStream_t st);
int ds_rows(int N, int H, int W);
int ds_fwd(const DsArgs& a, int dtype, hipStream_t st);

// input gradient of conv0 (autograd of the image through models/fast_scnn.py:153)
struct Conv0DgradArgs {
  const void* dz;  // NHWC [N,Ho,Wo,32] in the plan dtype (conv0's BN-backward output)
  const float* w;  // [32][3][3][3] fp32 master weights
  int N, H, W, Ho, Wo;
  void* dx;        // NCHW [N,3,H,W] in dx_dtype (0 fp32, 1 bf16, 2 fp16)
  int dx_dtype;
};
int conv0_dgrad(const Conv0DgradArgs& a, int dz_dtype, hipStream_t st);
int conv0_parts(int N, int Ho, int Wo);
int conv0_fwd(const Conv0Args& a, int y_dtype, hipStream_t st);
int conv0_wgrad_parts(int N, int Ho, int Wo, int rows_per_block);
int conv0_wgrad(const Conv0WgradArgs& a, int dz_dtype, hipStream_t st);

// LearningToDownsample.dsconv1.dw input gradient (stride 2) fused with the conv0 weight gradient
// (conv0.hip ltd_c0_bwd).  The dgrad's output g is the gradient of conv0's BN output; the launch
// emits that BN's backward records and finish (bs / tail, as dw_dgrad does) and, instead of
// storing g, per-workgroup conv0 partials [P][LC0_SLAB] = (A = sum g x^T, Zx = sum z x^T,
// B = sum x) over the conv0 patches x.  With the finished BN's operand table (common.hpp
// bwdx_apply: dz = al*g + gz*z + be), conv0_wgrad_combine forms dW = al*A + gz*Zc + (be+gz*mean)*B.
constexpr int LC0_SLAB = 2 * 864 + 27;  // [A: co*27+tap][Zx: 864 + co*27+tap][B: 1728 + tap]
struct LtdC0BwdArgs {
  int N, H, W;     // conv0 output = the depthwise layer's input (dx) dims
  int Ho, Wo;      // depthwise output (dy) dims
  const void* dy;  // NHWC [N,Ho,Wo,32]
  const float* w;  // depthwise taps [32][9] (16-B aligned)
  BnBwdPart bs{};  // conv0's BN (z, mean, invstd, scale, shift, mode); part [P][2][32]
  BnTail tail{};   // its finish
  const void* x;   // NCHW [N,3,XH,XW] image
  int x_dtype, XH, XW;
  float* slab;     // [P][LC0_SLAB]
};
int ltd_c0_bwd_parts(int N, int H, int W);
bool ltd_c0_bwd_ok(int dtype, int x_dtype, int XW, const void* x);
int ltd_c0_bwd(const LtdC0BwdArgs& a, int dtype, hipStream_t st);
// dW[co][tap] = al*A + gz*Zc + (be + gz*mean)*B from the reduced LC0_SLAB sums (Zc over z - mean)
// and the table (BWDX_STRIDE)
int conv0_wgrad_combine(const float* sums, const float* tab, const float* mean, float* dw,
                        hipStream_t st);

int dw_parts(int N, int Ho, int Wo, int C, int dtype, int stride);
int dw_fwd(const DwArgs& a, int dtype, hipStream_t st);
int dw_dgrad(const DwBwdArgs& a, int dtype, hipStream_t st);
int dw_dgrad_parts(int N, int H, int W, int C, int dtype, int stride);  // BnBwdPart records
int dw_wgrad_parts(int N, int Ho, int Wo, int C, int dtype, int stride);
int dw_wgrad(const DwBwdArgs& a, int dtype, hipStream_t st);
int dw_wgrad_reduce(float* slab, int P, int C, float* dw, hipStream_t st);

int gemm_parts(int M);
int gemm_nt(const GemmArgs& a, int dtype, hipStream_t st);
bool gemm_stream_ok(const GemmArgs& a, int dtype);
int gemm_stream(const GemmArgs& a, int dtype, hipStream_t st);  // streaming gemm_nt (gemm_stream.hip)
int gemm_stream_parts(const GemmArgs& a, int dtype);  // its workgroups per column group
int gemm_nt_parts(const GemmArgs& a, int dtype);      // BN records gemm_nt(a) writes
int gemm_tn_splits(int M, int N, int K);
int gemm_tn(GemmTnArgs a, int splits, int dtype, hipStream_t st);
// slab is consumed (folded in place)
int reduce_slabs(float* slab, int S, long long stride, long long count, float* out,
                 int accumulate, hipStream_t st);
int reduce_slabs_ex(float* slab, int S, long long stride, long long count, float* out,
                    int accumulate, int C9, hipStream_t st);
// Deferred weight-gradient reductions: the slab reductions of a backward stage are queued and run
// by two launches (fold + final) over the whole job table instead of two per weight tensor.
constexpr int RED_MAXJOBS = 64;  // a whole step's weight-gradient jobs (one multi-stage call)
struct RedJob {
  float* slab;   // [S][stride] partials (consumed)
  float* out;
  long long stride;
  int S, count, accumulate, C9;
  int Q = 0;     // fold fan-out (set by reduce_slabs_multi): S > RED_Q partials fold into Q
};
struct RedTable {
  int n = 0;
  int blocks = 0;                 // 256-element blocks over all jobs
  int blk0[RED_MAXJOBS + 1] = {};  // first block of each job
  RedJob j[RED_MAXJOBS];
};
int reduce_slabs_multi(const RedTable& t, hipStream_t st);
int colsum_parts(int M);
int colsum(const void* D, int M, int N, int ld, float* part, int dtype, hipStream_t st);

int bn_fold(const FoldTable& t, hipStream_t st);
int bn_finalize(const BnFinalizeArgs& a, hipStream_t st);
// FSCNN_TAIL_INK bitmask of the producers that finish their BN in-kernel (A/B, bisection):
// 1 tiled gemm_nt, 2 depthwise forward, 4 depthwise stride-1 dgrad, 8 stride-2 dgrad
int bn_apply(const BnApplyArgs& a, int dtype, hipStream_t st);
int bn_bwd_parts(long long M, int C, int dtype, int* rows_per_block);
int bn_bwd_reduce(const BnBwdArgs& a, int dtype, hipStream_t st);
// tab (optional): the per-channel operand-transform table of common.hpp bwdx_apply, built from
// the forward BN (scale, shift, mean, invstd; relu: the ReLU mask is recomputed from z)
int bn_bwd_finalize(float* part, int P, int C, double count, float* dgamma, float* dbeta,
                    float* coef, hipStream_t st, unsigned* counters = nullptr,
                    const BnBwdTab& tab = BnBwdTab());
int bn_bwd_apply(const BnBwdArgs& a, int dtype, hipStream_t st);

int up_nhwc(const UpArgs& a, int dtype, hipStream_t st);
int up_nchw(const UpArgs& a, int in_dtype, int out_dtype, hipStream_t st);
// final upsample + argmax over classes -> labels [N][Ho][Wo] (int64, or uint8 when label_u8)
int up_argmax(const UpArgs& a, int in_dtype, void* labels, int label_u8, hipStream_t st);
// SegmentationMetric counters [2 + 3C] (int64, accumulated); see misc.hip
int seg_metric(const void* pred, int pred_u8, const long long* target, long long n, int C,
               long long* counts, hipStream_t st);
int axis_bwd(const AxisBwdArgs& a, int g_dtype, int d_dtype, hipStream_t st);
int pyramid_pool(const PoolArgs& a, int dtype, hipStream_t st);
int pyramid_pool_bwd(const PoolBwdArgs& a, int dtype, hipStream_t st);
int ppm_up_fwd(const PpmUpArgs& a, int dtype, hipStream_t st);
int ppm_up_bwd(const PpmUpArgs& a, void* dfeats, int dtype, hipStream_t st);

bool ppm_branches_ok(int maxM, int K, int dtype);
int ppm_branches_fwd(const PpmFwdArgs& a, int dtype, hipStream_t st);
int ppm_branches_bwd(const PpmBwdArgs& a, int dtype, hipStream_t st);

int ce_parts(int N, long long HW);
int ce_fwd(const CeArgs& a, float* out, int dtype, hipStream_t st);
int ce_bwd(const CeArgs& a, const float* gout, const float* stats, int dtype, hipStream_t st);
// OHEM: label probabilities + counters [#labelled, #(prob <= thresh)] (accumulated), and the
// k-th smallest of n non-negative floats (host-synchronising radix select; hist: 2048 uint32)
int ohem_prob(const CeArgs& a, float thresh, float* prob, unsigned long long* counts, int dtype,
              hipStream_t st);
// the whole OHEM threshold on the device from ohem_prob's counters (no host synchronisation):
// *thr = inf (keep all labelled) / thresh / the k-th smallest label probability; work: 2056 uint32
int ohem_threshold_dev(const float* key, long long n, const unsigned long long* counts,
                       long long min_kept, float thresh, unsigned* work, float* thr,
                       hipStream_t st);
// Dice / Focal+Dice criteria (misc.hip): stats = (sum p1 t, sum p1, sum t, sum focal) in fp64
int dice_loss_fwd(const void* logits, int dtype, const long long* target, int N, int C, long long HW,
                  float alpha, float gamma, int focal, float* part, double* stats, hipStream_t st);
int dice_loss_bwd(const void* logits, int dtype, const long long* target, int N, int C, long long HW,
                  float alpha, float gamma, int focal, const double* stats, const float* gout,
                  float smooth, float wd, float wf, void* dlogits, hipStream_t st);
int ce_head_parts(int N, int Hl, int Wl);
int ce_head(const CeHeadArgs& a, float* out2, int dtype, hipStream_t st);
// the 16-bit loss-head kernel (ce_head2_kernel) takes these shapes; it reads CeHeadArgs::tgt8
// (when given) only where ce_head_reads_tgt8 holds, so only then are the targets packed
bool ce_head2_form(int C, int ldl, int dtype);
bool ce_head_reads_tgt8(int C, int ldl, int W, int dtype);
// targets [n] int64 -> int8: t if 0 <= t < C and t != ignore_index, else -1 (C <= 127)
int ce_pack_targets(const long long* t, long long n, int C, long long ignore_index,
                    signed char* out, hipStream_t st);
// g[m][c] = g_raw[m][c] * gout / count  (c < C; pad columns zeroed)
int ce_head_scale(const float* g_raw, void* g, long long M, int C, int ld, const float* gout,
                  const float* out2, int dtype, hipStream_t st);
int dropout(const DropArgs& a, int dtype, hipStream_t st);
// GPU input path: ToTensor + Normalize of uint8 HWC images into NCHW (fp32 / bf16)
int normalize_u8(const uint8_t* x, int N, int H, int W, const float* mean, const float* std,
                 void* y, int out_dtype, hipStream_t st);
// label-id -> train-id lookup (out-of-table ids -> invalid)
int remap_labels(const uint8_t* in, long long n, const long long* lut, int lut_size, int offset,
                 long long invalid, long long* out, hipStream_t st);
int im2col3(const Im2ColArgs& a, int dtype, hipStream_t st);
int col2im3(const Col2ImArgs& a, int dtype, hipStream_t st);
// *p = v (one thread): per-call scalars that captured graphs read from device memory
int set_u64(uint64_t* p, uint64_t v, hipStream_t st);
int sgd(const SgdArgs& a, hipStream_t st);
int cast_f32_bf16(const float* x, void* y, long long n, hipStream_t st);
// per-step weight operands from the fp32 arena: plain casts and zero-padded transposes (misc.hip)
constexpr int PREP_MAXJOBS = 48;
struct PrepJob {
  long long src;   // P offset (floats)
  long long dst;   // element offset in the destination
  int R, Cc;       // source [R][Cc] (row-major)
  int ld;          // trans: destination [Cc][ld] with ld >= R (columns >= R zero)
  int trans;       // 0 cast, 1 transpose, 2 zero fill of R*Cc elements, 3 split (below)
  // 3: the three-term bf16 truncation split of an fp32 [R][Cc] (common.hpp gs_split3) as planes
  //    [3][R][Cc] of uint16, dst counted in uint16 elements of the destination buffer
};
struct PrepTable {
  int n = 0;
  long long total = 0;
  long long start[PREP_MAXJOBS + 1] = {};
  int cstart[PREP_MAXJOBS + 1] = {};  // (set by weights_prep) first 2048-element chunk of each job
  PrepJob j[PREP_MAXJOBS];
};
int weights_prep(PrepTable& t, const float* P, void* dst, int dtype, hipStream_t st);
int fill_f32(float* x, long long n, float v, hipStream_t st);

}  // namespace fscnn
