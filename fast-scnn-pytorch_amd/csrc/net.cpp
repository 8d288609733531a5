// Native executor: builds the layer table, plans the workspace for a (N, H, W, dtype, mode)
// and issues the forward / backward kernel sequences on the caller's stream.
//
// Forward dataflow (models/fast_scnn.py:33-46), NHWC activations:
//   conv0 → dsconv1 → dsconv2 (= higher_res_features)        LearningToDownsample :157-161
//   9 × LinearBottleneck                                     GlobalFeatureExtractor :182-187
//   PPM: pool(1,2,3,6) → 4 × 1x1 → upsample into concat[:,128:256]; out 1x1(256→128)  :137-145
//   FFM: up(x4, ac) → dw → 1x1+bias+BN  (+)  1x1+bias+BN(higher) → ReLU    :207-218
//   Classifier: 2 × DSConv → Dropout → 1x1(+bias) → final bilinear to NCHW   :233-237, :40
// eval : BN folded into every producer's epilogue (one bn_fold launch per forward)
// train: producer writes raw z + per-block statistics → bn_finalize → bn_apply (+res / ReLU)
#include "net.hpp"
#include "bn_finish.hpp"

#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <vector>

#include <cstdio>
#include <cstring>

namespace fscnn {

// ======================================================================================
// layer table
// ======================================================================================
namespace {
struct Builder {
  Net& n;
  explicit Builder(Net& net) : n(net) {}
  long long palloc(const std::string& name, std::vector<int> shape) {
    long long numel = 1;
    for (int s : shape) numel *= s;
    long long off = (n.p_total + 15) / 16 * 16;  // 64-B aligned tensors (16-B vector loads)
    n.params.push_back({name, shape, off, numel});
    n.p_total = off + numel;
    return off;
  }
  long long ralloc(const std::string& name, int C) {
    long long off = (n.r_total + 15) / 16 * 16;
    n.buffers.push_back({name, {C}, off, C});
    n.r_total = off + C;
    return off;
  }
  ConvL conv(const std::string& key, int cin, int cout, int k = 1, int groups = 1, bool bias = false) {
    ConvL c;
    c.cin = cin; c.cout = cout; c.k = k; c.groups = groups;
    c.w = palloc(key + ".weight", {cout, cin / groups, k, k});
    if (bias) c.b = palloc(key + ".bias", {cout});
    if (groups == 1 && !(k == 3 && cin == 3)) {  // dense convs with a dgrad (not conv0)
      c.ldt = (cout + 7) / 8 * 8;
      c.wt = n.wt_total;
      n.wt_total += (long long)cin * k * k * c.ldt;
    }
    return c;
  }
  BnL bn(const std::string& key, int C) {
    BnL b;
    b.C = C;
    b.g = palloc(key + ".weight", {C});
    b.b = palloc(key + ".bias", {C});
    b.rm = ralloc(key + ".running_mean", C);
    b.rv = ralloc(key + ".running_var", C);
    b.nbt = n.n_bn;
    b.id = n.n_bn;
    n.buffers.push_back({key + ".num_batches_tracked", {}, (long long)n.n_bn, 1});
    n.n_bn++;
    return b;
  }
  DsL dsconv(const std::string& p, int cin, int cout) {
    DsL d;
    d.dw = conv(p + ".conv.0", cin, cin, 3, cin);
    d.bdw = bn(p + ".conv.1", cin);
    d.pw = conv(p + ".conv.3", cin, cout);
    d.bpw = bn(p + ".conv.4", cout);
    return d;
  }
};
}  // namespace

int net_build(int num_classes, int aux, Net& net) {
  if (num_classes < 1 || num_classes > 1024) {
    set_error("net_build: num_classes=%d out of range", num_classes);
    return E_INVALID;
  }
  net = Net();
  net.num_classes = num_classes;
  net.aux = aux;
  Builder b(net);
  // models/fast_scnn.py:20 LearningToDownsample(32, 48, 64)
  net.c0 = b.conv("learning_to_downsample.conv.conv.0", 3, 32, 3);
  net.b0 = b.bn("learning_to_downsample.conv.conv.1", 32);
  net.ltd1 = b.dsconv("learning_to_downsample.dsconv1", 32, 48);
  net.ltd2 = b.dsconv("learning_to_downsample.dsconv2", 48, 64);
  // :21 GlobalFeatureExtractor(64, [64, 96, 128], 128, 6, [3, 3, 3])
  static const int cin_[9] = {64, 64, 64, 64, 96, 96, 96, 128, 128};
  static const int cout_[9] = {64, 64, 64, 96, 96, 96, 128, 128, 128};
  static const int s_[9] = {2, 1, 1, 2, 1, 1, 1, 1, 1};
  net.stage_p_begin[3] = 0;
  for (int i = 0; i < 9; ++i) {
    char pfx[128];
    snprintf(pfx, sizeof pfx, "global_feature_extractor.bottleneck%d.%d", i / 3 + 1, i % 3);
    std::string p(pfx);
    int e = cin_[i] * 6;
    if (i == 3) net.stage_p_begin[2] = (net.p_total + 15) / 16 * 16;
    if (i == 6) net.stage_p_begin[1] = (net.p_total + 15) / 16 * 16;
    LbL& l = net.lb[i];
    l.cin = cin_[i]; l.cout = cout_[i]; l.stride = s_[i];
    l.e = b.conv(p + ".block.0.conv.0", cin_[i], e);
    l.be = b.bn(p + ".block.0.conv.1", e);
    l.d = b.conv(p + ".block.1.conv.0", e, e, 3, e);
    l.bd = b.bn(p + ".block.1.conv.1", e);
    l.p = b.conv(p + ".block.2", e, cout_[i]);
    l.bp = b.bn(p + ".block.3", cout_[i]);
  }
  net.stage_p_begin[0] = (net.p_total + 15) / 16 * 16;
  for (int i = 0; i < 4; ++i) {
    char pfx[128];
    snprintf(pfx, sizeof pfx, "global_feature_extractor.ppm.conv%d.conv", i + 1);
    std::string p(pfx);
    net.ppm_c[i] = b.conv(p + ".0", 128, 32);
    net.ppm_b[i] = b.bn(p + ".1", 32);
  }
  net.ppm_o = b.conv("global_feature_extractor.ppm.out.conv.0", 256, 128);
  net.ppm_ob = b.bn("global_feature_extractor.ppm.out.conv.1", 128);
  // :22 FeatureFusionModule(64, 128, 128)
  net.ffm_dw = b.conv("feature_fusion.dwconv.conv.0", 128, 128, 3, 128);
  net.ffm_bdw = b.bn("feature_fusion.dwconv.conv.1", 128);
  net.ffm_low = b.conv("feature_fusion.conv_lower_res.0", 128, 128, 1, 1, true);
  net.ffm_blow = b.bn("feature_fusion.conv_lower_res.1", 128);
  net.ffm_high = b.conv("feature_fusion.conv_higher_res.0", 64, 128, 1, 1, true);
  net.ffm_bhigh = b.bn("feature_fusion.conv_higher_res.1", 128);
  // :23 Classifer(128, num_classes)
  net.cls1 = b.dsconv("classifier.dsconv1", 128, 128);
  net.cls2 = b.dsconv("classifier.dsconv2", 128, 128);
  net.cls_out = b.conv("classifier.conv.1", 128, num_classes, 1, 1, true);
  if (aux) {
    net.aux0 = b.conv("auxlayer.0", 64, 32, 3);
    net.aux1 = b.bn("auxlayer.1", 32);
    net.aux4 = b.conv("auxlayer.4", 32, num_classes, 1, 1, true);
  }
  net.p_total = (net.p_total + 15) / 16 * 16;
  net.r_total = (net.r_total + 15) / 16 * 16;
  return OK;
}

// ======================================================================================
// planning
// ======================================================================================
namespace {
struct Alloc {
  size_t top = 0;
  size_t get(size_t bytes) {
    size_t off = (top + 255) / 256 * 256;
    top = off + (bytes ? bytes : 1);
    return off;
  }
};

int dwout(int h, int s) { return (h - 1) / s + 1; }

}  // namespace

// FSCNN_IR_S2=0: the stride-2 bottlenecks (1.0, 2.0) as three unfused launches in inference
static bool ir_stride2_enabled() {
  static const bool on = [] {
    const char* e = getenv("FSCNN_IR_S2");
    return !(e && e[0] == '0');
  }();
  return on;
}
// shape of bottleneck i as one fused inference launch (ir.hip); false when the block runs as
// its three unfused units (training plans, unsupported shapes)
bool ir_block_shape(const Net& net, const Plan& pl, int i, IrArgs& b) {
  const LbL& l = net.lb[i];
  if (pl.train || (l.stride != 1 && l.stride != 2)) return false;
  b = IrArgs{};
  b.N = pl.N;
  b.stride = l.stride;
  b.H = i < 3 ? pl.H4 : pl.H5;
  b.W = i < 3 ? pl.W4 : pl.W5;
  // input map: the previous block's output, or (block 0) the LearningToDownsample output
  b.Hi = i == 0 ? pl.H3 : (i < 4 ? pl.H4 : pl.H5);
  b.Wi = i == 0 ? pl.W3 : (i < 4 ? pl.W4 : pl.W5);
  b.Cin = l.cin; b.E = l.cin * 6; b.Cout = l.cout;
  b.ldx = i == 0 ? pl.l2pw.ld : pl.lbp[i - 1].ld; b.ldy = pl.lbp[i].ld;
  b.residual = l.stride == 1 && l.cin == l.cout;
  // one output tile per workgroup (8 x 8; stride 2: 4 x 8): below ~128 tiles (cfg1's 24 x 24
  // bottleneck3 map is 9 tiles) the fused launch leaves most CUs idle and the three unfused
  // launches are faster
  const int th = l.stride == 2 ? 4 : 8;
  const long long tiles = (long long)b.N * ((b.H + th - 1) / th) * ((b.W + 7) / 8);
  return ir_stride2_enabled() || l.stride == 1 ? tiles >= 128 && ir_block_ok(b, pl.dtype) : false;
}

// FSCNN_IR_TRAIN: training plans recompute the 6x-expanded tensor of these bottlenecks instead
// of storing it (ir.hip ir_train_fwd + a statistics-only expand pass; the backward recomputes it):
// 0 none (default), 1 bottleneck1 (the 201 / 50 / 50 MB tensors at cfg3), 2 every bottleneck.
// Measured r06 (cfg3 bf16, same box, two pairs): 6.028 / 6.035 ms per step with bottleneck1
// recomputed vs 5.815 / 5.815 stored -- the statistics-only expand costs 76 of the stored
// expand's 103 us (its epilogue's statistics, not its stores, dominate), the fused tile kernel
// 113 us against the depthwise's 91, and the backward's recompute another 137 us
static int ir_train_blocks() {
  static const int v = [] {
    const char* e = getenv("FSCNN_IR_TRAIN");
    return e ? atoi(e) : 0;
  }();
  return v;
}

int plan_build(const Net& net, int N, int H, int W, int dtype, int train, Plan& pl) {
  if (N < 1 || H < 3 || W < 3) {
    set_error("plan_build: bad input shape N=%d H=%d W=%d", N, H, W);
    return E_INVALID;
  }
  if (dtype != DT_F32 && dtype != DT_BF16 && dtype != DT_F16) {
    set_error("plan_build: unsupported dtype %d", dtype);
    return E_UNSUPPORTED;
  }
  if (train < 0 || train > 2) {
    set_error("plan_build: train must be 0 (inference), 1 (training) or 2 (differentiable "
              "inference: running-statistics BatchNorm)");
    return E_INVALID;
  }
  pl = Plan();
  pl.net = &net;
  pl.N = N; pl.H = H; pl.W = W; pl.dtype = dtype; pl.train = train;
  pl.H1 = (H - 3) / 2 + 1; pl.W1 = (W - 3) / 2 + 1;  // first conv, padding 0
  pl.H2 = dwout(pl.H1, 2); pl.W2 = dwout(pl.W1, 2);
  pl.H3 = dwout(pl.H2, 2); pl.W3 = dwout(pl.W2, 2);
  pl.H4 = dwout(pl.H3, 2); pl.W4 = dwout(pl.W3, 2);
  pl.H5 = dwout(pl.H4, 2); pl.W5 = dwout(pl.W4, 2);
  const int V = dtype == DT_F32 ? 4 : 8;
  const size_t E = dtype == DT_F32 ? 4 : 2;
  pl.Cp = (net.num_classes + V - 1) / V * V;
  Alloc A, B;  // forward (saved) and backward (scratch) workspaces
  auto unit = [&](Unit& u, long long M, int C, int nparts, size_t a_override = (size_t)-1,
                  int ld = 0) {
    u.M = M; u.C = C; u.ld = ld ? ld : C;
    u.a = a_override != (size_t)-1 ? a_override : A.get((size_t)M * u.ld * E);
    u.z = train ? A.get((size_t)M * C * E) : u.a;
    u.nparts = nparts;
    if (train) u.part = A.get((size_t)nparts * 3 * C * 4);
    u.mean = A.get(C * 4); u.invstd = A.get(C * 4);
    u.scale = A.get(C * 4); u.shift = A.get(C * 4);
  };
  auto gunit = [&](Unit& u, size_t ga_override = (size_t)-1, int ld = 0) {
    u.ga_ld = ld ? ld : u.C;
    u.ga = ga_override != (size_t)-1 ? ga_override : B.get((size_t)u.M * u.ga_ld * E);
  };
  const long long M0 = (long long)N * pl.H1 * pl.W1, M1 = (long long)N * pl.H2 * pl.W2,
                  M2 = (long long)N * pl.H3 * pl.W3, M4 = (long long)N * pl.H4 * pl.W4,
                  M5 = (long long)N * pl.H5 * pl.W5;
  if (M0 > 0x7fffffffLL / 32) {
    set_error("plan_build: batch too large for 32-bit row indexing");
    return E_INVALID;
  }
  if (dtype != DT_F32) pl.pbf = A.get((size_t)net.p_total * 2);  // 16-bit weight copy
  if (train) pl.wt = A.get((size_t)net.wt_total * E);
  unit(pl.c0, M0, 32, conv0_parts(N, pl.H1, pl.W1));
  unit(pl.l1dw, M1, 32, dw_parts(N, pl.H2, pl.W2, 32, dtype, 2));
  unit(pl.l1pw, M1, 48, gemm_parts((int)M1));
  unit(pl.l2dw, M2, 48, dw_parts(N, pl.H3, pl.W3, 48, dtype, 2));
  unit(pl.l2pw, M2, 64, gemm_parts((int)M2));
  pl.concat = A.get((size_t)M5 * 256 * E);
  for (int i = 0; i < 9; ++i) {
    const LbL& l = net.lb[i];
    long long Min = i == 0 ? M2 : (i <= 3 ? M4 : M5);
    long long Mout = i < 3 ? M4 : M5;
    int Ho = i < 3 ? pl.H4 : pl.H5, Wo = i < 3 ? pl.W4 : pl.W5;
    int e = l.cin * 6;
    unit(pl.lbe[i], Min, e, gemm_parts((int)Min));
    // (the training form of ir.hip writes one BN_d record per output tile)
    unit(pl.lbd[i], Mout, e, std::max<int>(dw_parts(N, Ho, Wo, e, dtype, l.stride),
                                          (int)ir_train_parts(N, Ho, Wo, l.stride)));
    if (i == 8) unit(pl.lbp[i], Mout, l.cout, gemm_parts((int)Mout), pl.concat, 256);
    else unit(pl.lbp[i], Mout, l.cout, gemm_parts((int)Mout));
  }
  // PPM: pooled / feats are bin-major [50][N][C]
  pl.pooled = A.get((size_t)50 * N * 128 * E);
  pl.feats_a = A.get((size_t)50 * N * 32 * E);
  static const int kk[4] = {1, 2, 3, 6}, base[4] = {0, 1, 5, 14};
  for (int i = 0; i < 4; ++i) {
    long long M = (long long)kk[i] * kk[i] * N;
    unit(pl.ppk[i], M, 32, gemm_parts((int)M), pl.feats_a + (size_t)base[i] * N * 32 * E, 32);
  }
  unit(pl.po, M5, 128, gemm_parts((int)M5));
  pl.up_low = A.get((size_t)M2 * 128 * E);
  unit(pl.fdw, M2, 128, dw_parts(N, pl.H3, pl.W3, 128, dtype, 1));
  pl.f = A.get((size_t)M2 * 128 * E);
  unit(pl.flow, M2, 128, gemm_parts((int)M2), pl.f);    // a = f (combined), z own
  unit(pl.fhigh, M2, 128, gemm_parts((int)M2), pl.f);
  unit(pl.c1dw, M2, 128, dw_parts(N, pl.H3, pl.W3, 128, dtype, 1));
  unit(pl.c1pw, M2, 128, gemm_parts((int)M2));
  unit(pl.c2dw, M2, 128, dw_parts(N, pl.H3, pl.W3, 128, dtype, 1));
  unit(pl.c2pw, M2, 128, gemm_parts((int)M2));
  pl.drop = train ? A.get((size_t)M2 * 128 * E) : pl.c2pw.a;
  pl.logits = A.get((size_t)M2 * pl.Cp * E);
  if (net.aux) {  // models/fast_scnn.py:24-31: 3x3 conv on im2col columns, BN, ReLU, Dropout, 1x1
    unit(pl.aux0, M2, 32, gemm_parts((int)M2));
    pl.aux_col = A.get((size_t)M2 * 576 * E);
    pl.aux_drop = train ? A.get((size_t)M2 * 32 * E) : pl.aux0.a;
    pl.aux_logits = A.get((size_t)M2 * pl.Cp * E);
  }
  // labels: models/fast_scnn.py module paths
  pl.c0.name = "learning_to_downsample.conv";
  pl.l1dw.name = "learning_to_downsample.dsconv1.dw"; pl.l1pw.name = "learning_to_downsample.dsconv1.pw";
  pl.l2dw.name = "learning_to_downsample.dsconv2.dw"; pl.l2pw.name = "learning_to_downsample.dsconv2.pw";
  for (int i = 0; i < 9; ++i) {
    const std::string b = "global_feature_extractor.bottleneck" + std::to_string(i / 3 + 1) + "." +
                          std::to_string(i % 3);
    pl.lbe[i].name = b + ".expand"; pl.lbd[i].name = b + ".dw"; pl.lbp[i].name = b + ".project";
    pl.lbp[i].block_name = b + " (fused block)";
  }
  for (int i = 0; i < 4; ++i) pl.ppk[i].name = "global_feature_extractor.ppm.conv" + std::to_string(i + 1);
  pl.po.name = "global_feature_extractor.ppm.out";
  pl.fdw.name = "feature_fusion.dwconv"; pl.flow.name = "feature_fusion.conv_lower_res";
  pl.fhigh.name = "feature_fusion.conv_higher_res";
  pl.c1dw.name = "classifier.dsconv1.dw"; pl.c1pw.name = "classifier.dsconv1.pw";
  pl.c2dw.name = "classifier.dsconv2.dw"; pl.c2pw.name = "classifier.dsconv2.pw";
  pl.aux0.name = "auxlayer";
  if (train) {
    pl.g_raw = A.get((size_t)2 * M2 * pl.Cp * 4);  // own-row plane + row-spill plane
    pl.head_part = A.get((size_t)ce_head_parts(N, pl.H3, pl.W3) * 2 * 4);
    if (train == 1 && ce_head_reads_tgt8(net.num_classes, pl.Cp, pl.W, dtype))
      pl.tgt8 = A.get((size_t)N * pl.H * pl.W);
  }
  if (train) {
    pl.seed_slot = A.get(64);
    // arrival counters of the one-launch BN fold+finalize (forward and backward), zeroed by the
    // step's weights_prep launch and left zero by every launch that uses them
    pl.fcnt = A.get(2 * BN_COUNTERS * 4);
    pl.bcnt = pl.fcnt + BN_COUNTERS * 4;
  }
  if (train) {
    // BN+ReLU outputs whose only consumers are GEMM / depthwise operands (and the wgrads reading
    // them again in the backward) are never stored: bn_apply is skipped and the consumers apply
    // relu(fmaf(z, scale, shift)) while staging.  Saves a read + write of each tensor per step.
    pl.c0.lazy = pl.l1dw.lazy = pl.l1pw.lazy = pl.l2dw.lazy = true;
    for (int i = 0; i < 9; ++i) pl.lbe[i].lazy = pl.lbd[i].lazy = true;
    pl.fdw.lazy = pl.c1dw.lazy = pl.c1pw.lazy = pl.c2dw.lazy = true;
    // LearningToDownsample's output: read by bottleneck1.0's expand and the FFM's high-res
    // branch (both GEMM operands) — unless the aux head's im2col reads it as well
    if (!net.aux) pl.l2pw.lazy = true;
  }
  // fp32 inference: the fused bottlenecks' expand / project weights as three bf16 split planes
  // (weights_prep mode 3, once per forward), so the fused kernel does no split arithmetic
  if (!train && dtype == DT_F32) {
    for (int i = 0; i < 9; ++i) {
      IrArgs b;
      if (!ir_block_shape(net, pl, i, b)) continue;
      pl.lb_we3[i] = A.get((size_t)3 * b.E * b.Cin * 2);
      pl.lb_wp3[i] = A.get((size_t)3 * b.Cout * b.E * 2);
    }
  }
  // fp64 team sums of the in-kernel BN finishes (last, so the activation offsets above do not move)
  if (train) pl.tsum = A.get((size_t)TAIL_TMAX * 3 * TAIL_CMAX * 8);
  if (train) pl.tsum2 = A.get((size_t)TAIL_TMAX * 3 * TAIL_CMAX * 8);
  pl.ws_bytes = A.top;
  auto nm = [&](const char* n, size_t off, long long rows, int cols, int ld, int bws) {
    pl.named.push_back({n, off, rows, cols, ld, bws});
  };
  auto nu = [&](const std::string& n, const Unit& u) {
    pl.named.push_back({n + ".a", u.a, u.M, u.C, u.ld, 0});
    pl.named.push_back({n + ".z", u.z, u.M, u.C, u.C, 0});
    pl.named.push_back({n + ".scale", u.scale, 1, u.C, u.C, 0});
    pl.named.push_back({n + ".shift", u.shift, 1, u.C, u.C, 0});
    pl.named.push_back({n + ".mean", u.mean, 1, u.C, u.C, 0});
    pl.named.push_back({n + ".invstd", u.invstd, 1, u.C, u.C, 0});
  };
  nu("c0", pl.c0); nu("l1dw", pl.l1dw); nu("l1pw", pl.l1pw); nu("l2dw", pl.l2dw); nu("l2pw", pl.l2pw);
  for (int i = 0; i < 9; ++i) {
    nu("lbe" + std::to_string(i), pl.lbe[i]);
    nu("lbd" + std::to_string(i), pl.lbd[i]);
    nu("lbp" + std::to_string(i), pl.lbp[i]);
  }
  for (int i = 0; i < 4; ++i) nu("ppk" + std::to_string(i), pl.ppk[i]);
  nu("po", pl.po); nu("fdw", pl.fdw); nu("flow", pl.flow); nu("fhigh", pl.fhigh);
  nu("c1dw", pl.c1dw); nu("c1pw", pl.c1pw); nu("c2dw", pl.c2dw); nu("c2pw", pl.c2pw);
  if (net.aux) nu("aux0", pl.aux0);
  nm("concat", pl.concat, M5, 256, 256, 0);
  nm("up_low", pl.up_low, M2, 128, 128, 0);
  nm("f", pl.f, M2, 128, 128, 0);
  nm("drop", pl.drop, M2, 128, 128, 0);
  nm("logits", pl.logits, M2, net.num_classes, pl.Cp, 0);

  if (train) {
    const int C = net.num_classes;
    pl.g_logits = B.get((size_t)M2 * pl.Cp * E);
    pl.t_up = B.get((size_t)N * C * H * pl.W3 * 4);
    pl.g_drop = B.get((size_t)M2 * 128 * E);
    gunit(pl.c2pw);
    gunit(pl.c2dw);
    gunit(pl.c1pw);
    gunit(pl.c1dw);
    pl.g_f = B.get((size_t)M2 * 128 * E);
    gunit(pl.fdw);
    pl.g_up = B.get((size_t)M2 * 128 * E);
    pl.t_up2 = B.get((size_t)N * pl.H3 * pl.W5 * 128 * 4);
    gunit(pl.po);
    pl.g_concat = B.get((size_t)M5 * 256 * E);
    pl.g_feats = B.get((size_t)50 * N * 32 * E);
    for (int i = 0; i < 4; ++i)
      gunit(pl.ppk[i], pl.g_feats + (size_t)base[i] * N * 32 * E, 32);
    pl.g_pooled = B.get((size_t)50 * N * 128 * E);
    for (int i = 8; i >= 0; --i) {
      gunit(pl.lbd[i]);
      gunit(pl.lbe[i]);
      if (i == 8) gunit(pl.lbp[i], pl.g_concat, 256);
      else gunit(pl.lbp[i]);
    }
    gunit(pl.l2pw);
    gunit(pl.l2dw);
    gunit(pl.l1pw);
    gunit(pl.l1dw);
    gunit(pl.c0);
    if (net.aux) {
      gunit(pl.aux0);
      pl.g_auxlog = B.get((size_t)M2 * pl.Cp * E);
      pl.g_aux = B.get((size_t)M2 * 32 * E);
      pl.aux_dcol = B.get((size_t)M2 * 576 * E);
    }
    // scratch sized for the largest consumer
    long long max_mc = 0;
    auto upd = [&](const Unit& u) { if (u.M * u.C > max_mc) max_mc = u.M * u.C; };
    upd(pl.c0); upd(pl.l1dw); upd(pl.l1pw); upd(pl.l2dw); upd(pl.l2pw);
    for (int i = 0; i < 9; ++i) { upd(pl.lbe[i]); upd(pl.lbd[i]); upd(pl.lbp[i]); }
    upd(pl.po); upd(pl.fdw); upd(pl.flow); upd(pl.c1dw); upd(pl.c1pw);
    if (net.aux) upd(pl.aux0);
    // BN-backward outputs: one slot per unit per backward call (Exec::dz_buf), so a wgrad
    // queued for the side stream never races a later rewrite
    size_t dzs = 0;
    auto dzu = [&](const Unit& u) { dzs += ((size_t)u.M * u.C * E + 255) / 256 * 256; };
    dzu(pl.c0); dzu(pl.l1dw); dzu(pl.l1pw); dzu(pl.l2dw); dzu(pl.l2pw);
    for (int i = 0; i < 9; ++i) { dzu(pl.lbe[i]); dzu(pl.lbd[i]); dzu(pl.lbp[i]); }
    for (int i = 0; i < 4; ++i) dzu(pl.ppk[i]);
    dzu(pl.po); dzu(pl.fdw); dzu(pl.flow); dzu(pl.fhigh); dzu(pl.c1dw); dzu(pl.c1pw);
    dzu(pl.c2dw); dzu(pl.c2pw);
    if (net.aux) dzu(pl.aux0);
    (void)max_mc;
    pl.dz_bytes = dzs;
    pl.dz = B.get(dzs);
    // weight-gradient partial slabs: the reductions of a backward stage are deferred to one
    // multi-job launch pair (Exec::flush_reduce), so every job keeps its own slab until then;
    // the arena holds the whole step's (sum over jobs, 64-float aligned each)
    size_t slab = 0;
    auto add_slab = [&](size_t floats) { slab += (floats + 63) / 64 * 64; };
    auto pw_slab = [&](long long M, int n, int k, bool bias = false) {
      add_slab((size_t)gemm_tn_splits((int)M, n, k) * n * k);
      if (bias) add_slab((size_t)colsum_parts((int)M) * n);
    };
    auto dw_slab = [&](int Ho, int Wo, int Cc, int st) {
      add_slab((size_t)dw_wgrad_parts(N, Ho, Wo, Cc, dtype, st) * 9 * Cc);
    };
    pw_slab(M1, 48, 32); pw_slab(M2, 64, 48);
    dw_slab(pl.H2, pl.W2, 32, 2); dw_slab(pl.H3, pl.W3, 48, 2);
    for (int i = 0; i < 9; ++i) {
      const LbL& l = net.lb[i];
      long long Min = pl.lbe[i].M, Mout = pl.lbd[i].M;
      int Ho = i < 3 ? pl.H4 : pl.H5, Wo = i < 3 ? pl.W4 : pl.W5;
      pw_slab(Min, l.cin * 6, l.cin);
      pw_slab(Mout, l.cout, l.cin * 6);
      dw_slab(Ho, Wo, l.cin * 6, l.stride);
    }
    for (int i = 0; i < 4; ++i) pw_slab(pl.ppk[i].M, 32, 128);
    pw_slab(M5, 128, 256);
    for (int i = 0; i < 3; ++i) dw_slab(pl.H3, pl.W3, 128, 1);  // FFM dw, classifier dw x2
    pw_slab(M2, 128, 128, true); pw_slab(M2, 128, 64, true);   // FFM low / high (bias)
    pw_slab(M2, 128, 128); pw_slab(M2, 128, 128);              // classifier dsconv pw x2
    pw_slab(M2, C, 128, true);                                 // classifier 1x1 (bias)
    if (net.aux) { pw_slab(M2, 32, 576); pw_slab(M2, C, 32, true); }
    add_slab((size_t)conv0_wgrad_parts(N, pl.H1, pl.W1, 8) * 864);
    add_slab((size_t)ltd_c0_bwd_parts(N, pl.H1, pl.W1) * LC0_SLAB);  // (the fused form's)
    pl.slab_floats = slab;
    pl.slab = B.get(slab * 4);
    // BN backward partials: max P*2*C
    size_t bnp = 0;
    auto bn_upd = [&](const Unit& u) {
      int rpb;
      size_t s = (size_t)bn_bwd_parts(u.M, u.C, dtype, &rpb) * 2 * u.C;
      if (s > bnp) bnp = s;
      s = (size_t)gemm_parts((int)u.M) * 2 * u.C;  // fused dgrad-epilogue records
      if (s > bnp) bnp = s;
    };
    bn_upd(pl.c0); bn_upd(pl.l1dw); bn_upd(pl.l1pw); bn_upd(pl.l2dw); bn_upd(pl.l2pw);
    for (int i = 0; i < 9; ++i) { bn_upd(pl.lbe[i]); bn_upd(pl.lbd[i]); bn_upd(pl.lbp[i]); }
    for (int i = 0; i < 4; ++i) bn_upd(pl.ppk[i]);
    bn_upd(pl.po); bn_upd(pl.fdw); bn_upd(pl.flow); bn_upd(pl.c1dw); bn_upd(pl.c1pw);
    if (net.aux) bn_upd(pl.aux0);
    // depthwise dgrads producing a BN's dy write dw_dgrad_parts records (Executor::dw_bwd)
    auto dw_upd = [&](int H, int W, int Cc, int stride) {
      const size_t s = (size_t)dw_dgrad_parts(N, H, W, Cc, dtype, stride) * 2 * Cc;
      if (s > bnp) bnp = s;
    };
    dw_upd(pl.H1, pl.W1, 32, 2); dw_upd(pl.H2, pl.W2, 48, 2);
    for (int i = 0; i < 9; ++i) {
      const int Hin = i == 0 ? pl.H3 : (i <= 3 ? pl.H4 : pl.H5);
      const int Win = i == 0 ? pl.W3 : (i <= 3 ? pl.W4 : pl.W5);
      dw_upd(Hin, Win, net.lb[i].cin * 6, net.lb[i].stride);
    }
    dw_upd(pl.H3, pl.W3, 128, 1);
    {  // the FFM pair (Exec::bn_bwd_pair) keeps both BNs' records side by side
      int rpb;
      const size_t s = (size_t)2 * bn_bwd_parts(pl.flow.M, 128, dtype, &rpb) * 2 * 128;
      if (s > bnp) bnp = s;
    }
    pl.bnpart = B.get(bnp * 4);
    pl.bnpart_floats = bnp;
    pl.coef = B.get(2 * 1024 * 4);
    pl.xtab = B.get((size_t)pl.c0.C * BWDX_STRIDE * 4);  // Exec::tab_slot (conv0's BN)
    pl.c0sum = B.get((size_t)LC0_SLAB * 4);  // reduced conv0 partials of the fused LTD backward
    pl.cspart = B.get((size_t)colsum_parts((int)M2) * (C > 128 ? C : 128) * 4);
    pl.bws_bytes = B.top;
    auto gu = [&](const std::string& n, const Unit& u) {
      pl.named.push_back({n + ".ga", u.ga, u.M, u.C, u.ga_ld, 1});
    };
    gu("c0", pl.c0); gu("l1dw", pl.l1dw); gu("l1pw", pl.l1pw); gu("l2dw", pl.l2dw); gu("l2pw", pl.l2pw);
    for (int i = 0; i < 9; ++i) {
      gu("lbe" + std::to_string(i), pl.lbe[i]);
      gu("lbd" + std::to_string(i), pl.lbd[i]);
      gu("lbp" + std::to_string(i), pl.lbp[i]);
    }
    gu("po", pl.po); gu("fdw", pl.fdw); gu("c1dw", pl.c1dw); gu("c1pw", pl.c1pw);
    gu("c2dw", pl.c2dw); gu("c2pw", pl.c2pw);
    nm("g_logits", pl.g_logits, M2, C, pl.Cp, 1);
    nm("g_f", pl.g_f, M2, 128, 128, 1);
    nm("g_up", pl.g_up, M2, 128, 128, 1);
    nm("g_concat", pl.g_concat, M5, 256, 256, 1);
    nm("dz", pl.dz, M0, 32, 32, 1);
  }
  return OK;
}

// ======================================================================================
// execution
// ======================================================================================
// The backward's weight gradients (gemm_tn, colsum, depthwise / conv0 wgrad) only feed the
// deferred slab reduction at the end of their stage, so they run on a second stream, beside
// the dgrad -> BN-backward chain that carries the critical path: many of those launches are
// latency-bound and leave HBM idle.  Every event recorded on a stream costs that stream ~5-7 us
// of idle time on MI355X (measured: 61 such gaps = 0.43 ms of a 7.05 ms step; r06: two extra
// forks per flush +0.41 ms per step; forking every 2nd / 3rd flush +0.28 / +0.35 ms: the wgrads
// start later), less without the events' system-scope fence (SideStream::init), so events are
// kept to one fork per wgrad launch (Exec::side_launch) and one join before the stage's slab
// reduction: every BN-backward output dz and operand table a wgrad reads has its own slot in
// the step's arenas (no reuse, so no release events; 7.08 -> 7.00 ms/step).
// FSCNN_SIDE_STREAM=0 keeps one stream.
// Thread safety (DataParallel replicas, train.py:170-171, call the backward from one worker
// thread per device; two replicas may share a device and so this plan): the stream lives on the
// device of the caller's stream at its creation and is only used from calls whose stream AND
// current device are that device (a call on another device's stream while a different device is
// current runs on one stream: a side stream of the current device would run the weight gradients
// against the other device's memory); every (record, wait) pair on the shared fork / join events
// is one critical section, so a fork always orders the side stream after the CALLER's
// main-stream work (a concurrent record in between would hand it another thread's point in time).
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  int dev = -1;
  bool ready = false, failed = false;
  std::mutex mu;
  // device of the caller's stream, when it is also the current device; -1 otherwise
  static int caller_device(hipStream_t main) {
    int cur = -1, sd = -1;
    if (hipGetDevice(&cur) != hipSuccess) return -1;
    if (hipStreamGetDevice(main, &sd) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    return sd == cur ? cur : -1;
  }
  bool init(hipStream_t main) {
    const int cd = caller_device(main);
    if (cd < 0) return false;
    std::lock_guard<std::mutex> lock(mu);
    if (ready || failed) return ready && cd == dev;
    failed = true;
    dev = cd;
    // the side stream at the lowest priority the device offers (FSCNN_SIDE_PRIO: 0 = plain
    // stream, 2 = the highest): measured r04 5.944-5.957 ms/step vs 5.984-5.985 (plain) and
    // 5.993-5.995 (highest) -- the main stream's latency-bound chain gets the CUs first
    static const int prio_mode = [] {
      const char* e = getenv("FSCNN_SIDE_PRIO");
      return e ? atoi(e) : 1;
    }();
    // (a CU-masked side stream, hipExtStreamCreateWithCUMask on 1/2 or 1/4 of the CUs, measured
    // r04 10.6 / 12.3 ms per step: not an option)
    if (prio_mode) {
      int lo = 0, hi = 0;  // numerically: greatest = lowest priority
      if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
          hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio_mode == 1 ? lo : hi) != hipSuccess)
        return false;
    } else if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      return false;
    }
    // fork / join events without the system-scope fence: a default event record writes back and
    // invalidates the L2s (host visibility) and the next kernels start cold.  Both ends of these
    // events are kernels of this device, whose dispatch packets carry their own agent-scope
    // acquire / release (the cross-XCD coherence every same-stream kernel pair already relies
    // on), and no host code inspects them.  Measured r06: 5.585 / 5.599 vs 5.677 / 5.692 ms per
    // cfg3 step (same box; device-scope-release events 5.693 / 5.696); every side-stream path stays
    // bit-identical to one stream (test_switch_train_steps_bit_identical_with_dropout).
    // FSCNN_SIDE_FENCE=1 restores the default (fenced) events.
    static const unsigned evf = [] {
      const char* e = getenv("FSCNN_SIDE_FENCE");
      return (unsigned)hipEventDisableTiming |
             (e && e[0] == '1' ? 0u : (unsigned)hipEventDisableSystemFence);
    }();
    hipEvent_t* ev[2] = {&fork, &join};
    for (auto* e : ev)
      if (hipEventCreateWithFlags(e, evf) != hipSuccess) return false;
    ready = true;
    failed = false;
    return true;
  }
  // the side stream waits for everything enqueued on `main` so far
  bool fork_from(hipStream_t main) {
    const double t0 = g_host_prof ? host_now_us() : 0.0;
    std::lock_guard<std::mutex> lock(mu);
    const bool ok = hipEventRecord(fork, main) == hipSuccess && hipStreamWaitEvent(s, fork, 0) == hipSuccess;
    if (g_host_prof) host_prof_add(1, host_now_us() - t0);
    return ok;
  }
  // `main` waits for everything enqueued on the side stream so far
  bool join_into(hipStream_t main) {
    const double t0 = g_host_prof ? host_now_us() : 0.0;
    std::lock_guard<std::mutex> lock(mu);
    const bool ok = hipEventRecord(join, s) == hipSuccess && hipStreamWaitEvent(main, join, 0) == hipSuccess;
    if (g_host_prof) host_prof_add(2, host_now_us() - t0);
    return ok;
  }
  ~SideStream() {
    hipEvent_t ev[2] = {fork, join};
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
  }
};
std::shared_ptr<SideStream> make_side_stream() { return std::make_shared<SideStream>(); }

namespace {

#define TRY(x)                 \
  do {                         \
    int rc__ = (x);            \
    if (rc__) return rc__;     \
  } while (0)

bool graphs_enabled();

// FSCNN_SIDE_STREAM=0: every weight gradient on the caller's stream (one stream; debugging and
// A/B; tests/test_gpu_switches.py keeps it parity-green)
bool side_stream_enabled() {
  static const bool on = [] {
    const char* e = getenv("FSCNN_SIDE_STREAM");
    return !(e && e[0] == '0');
  }();
  return on;
}

// FSCNN_LTD_FUSED=0: LTD.dsconv1.dw's input gradient stored and conv0's weight gradient as its
// own launch (conv0_wgrad) instead of the fused ltd_c0_bwd (A/B; tests/test_gpu_switches.py)
bool ltd_fused_enabled() {
  static const bool on = [] {
    const char* e = getenv("FSCNN_LTD_FUSED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// FSCNN_DROP_FUSED=0: the classifier's Dropout backward as its own launch and dsconv2 pw's
// BN-backward reduce as its own pass, instead of both in the classifier conv's dgrad epilogue
// (A/B; tests/test_gpu_switches.py)
bool drop_dgrad_on() {
  static const bool on = [] {
    const char* e = getenv("FSCNN_DROP_FUSED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// fused BN-backward partials: the dgrad GEMM producing the dy of unit `u` emits its records
struct BTarget {
  const Unit* u = nullptr;
  const BnL* bn = nullptr;
  int mode = 0;  // 0 no ReLU, 2 relu_z (mask recomputed from z)
};

struct Exec {
  const Plan& pl;
  const Net& net;
  const RunArgs& r;
  char* ws;
  char* bws;
  int dt;
  size_t E;
  bool train;
  // train == 2 plans (eval-mode autograd): the training dataflow (pre-BN z stored, BN applied by
  // the consumers, the staged backward) with every BatchNorm normalised by its running statistics
  // (fold_all before the forward): no batch statistics, no running-stat update, no Dropout, and
  // the BN backward without its batch-mean terms (BN_FROZEN_COUNT)
  bool frozen;
  Exec(const Plan& p, const RunArgs& ra)
      : pl(p), net(*p.net), r(ra), ws((char*)ra.ws), bws((char*)ra.bws), dt(p.dtype),
        E(p.dtype == DT_F32 ? 4 : 2), train(p.train != 0), frozen(p.train == 2) {}
  // element count of unit u's BN backward (frozen: the running-statistics form)
  double bcount(const Unit& u) const { return frozen ? BN_FROZEN_COUNT : (double)u.M; }
  // every return path (a TRY() failure between a fork and its join included) leaves the caller's
  // stream ordered after the side-stream work already issued: the workspaces it writes are
  // freed by the caller once the call returns, and a graph capture needs the fork joined
  ~Exec() {
    if (side && forked) (void)side->join_into(r.st);
  }

  // ---- side stream for the weight gradients (backward only; see SideStream) ----------------
  SideStream* side = nullptr;
  bool forked = false;  // side-stream work issued since the last join
  std::vector<std::function<int(hipStream_t)>> sideq;  // wgrads waiting for the next fork
  void use_side() {
    if (train && side_stream_enabled() && pl.side && pl.side->init(r.st)) side = pl.side.get();
  }
  // the PPM branches as one fused launch each way (ppm.hip) wherever the branch shapes fit it;
  // the general per-branch GEMM / BN kernels otherwise
  bool ppm_fused() const { return train && !frozen && ppm_branches_ok((int)pl.ppk[3].M, 128, dt); }
  // a weight-gradient launch: queued for the side stream (issued by flush_side), or run now on
  // the main stream without one
  int side_launch(std::function<int(hipStream_t)> f) {
    if (!side) return f(r.st);
    const char* tag = g_prof_tag;  // the launch keeps its layer label (per-launch profile)
    sideq.push_back([tag, f](hipStream_t s) {
      const char* o = g_prof_tag;
      g_prof_tag = tag;
      const int rc = f(s);
      g_prof_tag = o;
      return rc;
    });
    return OK;
  }
  // the wgrads of one conv (gemm_tn + bias colsum, or the depthwise wgrad) behind one fork:
  // issued as soon as their dz exists, they fill the idle issue slots of the latency-bound
  // dgrad chain (queueing a whole block's behind one fork measured slower: 7.24 vs 7.00 ms/step)
  // one fork: everything enqueued on the main stream so far happens before the queued wgrads
  int flush_side() {
    if (!side || sideq.empty()) return OK;
    if (!side->fork_from(r.st)) {
      set_error("side stream: fork failed");
      return E_HIP;
    }
    forked = true;
    for (auto& f : sideq) TRY(f(side->s));
    sideq.clear();
    return OK;
  }
  // the loss head's targets as int8 (the side stream packs them during the global feature
  // extractor; the FFM join orders them before the head), where the head reads them
  bool ce_head_packs() const { return pl.tgt8 != 0; }
  int pack_targets(hipStream_t s) {
    g_prof_tag = "head (targets to int8)";
    return ce_pack_targets(r.target, (long long)pl.N * pl.H * pl.W, net.num_classes,
                           r.ignore_index, (signed char*)W(pl.tgt8), s);
  }
  int join() {
    if (!side) return OK;
    TRY(flush_side());
    if (!forked) return OK;
    if (!side->join_into(r.st)) {
      set_error("side stream: join failed");
      return E_HIP;
    }
    forked = false;
    return OK;
  }
  // BN-backward output dz of unit u: its own slot of the step's dz arena (a queued wgrad may
  // read it after the main stream has moved on)
  size_t dz_top = 0;
  void* dz_buf(const Unit& u) {
    const size_t bytes = ((size_t)u.M * u.C * E + 255) / 256 * 256;
    if (dz_top + bytes > pl.dz_bytes) return nullptr;
    void* p = (char*)Bw(pl.dz) + dz_top;
    dz_top += bytes;
    return p;
  }
  // BN-backward operand table of unit u, written by its dy producer's BN finish and read by the
  // consumer of the fused dz (bn_bwd_x): only conv0's BN has such a consumer (its streaming
  // weight gradient), so only that unit owns a table — a fixed slot of the plan, valid across
  // the separate per-stage backward calls; every other producer writes none
  float* tab_slot(const Unit& u) const { return &u == &pl.c0 ? (float*)Bw(pl.xtab) : nullptr; }

  // the dropout seed: a device slot only when the launches may be captured into a hipGraph
  // (replays must see a new seed); otherwise a kernel argument (no set_u64 launch per step)
  const uint64_t* seed_ptr() const {
    return graphs_enabled() ? reinterpret_cast<const uint64_t*>(W(pl.seed_slot)) : nullptr;
  }
  void* W(size_t off) const { return ws + off; }
  void* Bw(size_t off) const { return bws + off; }
  float* Wf(size_t off) const { return (float*)(ws + off); }
  const float* P(long long off) const { return off < 0 ? nullptr : r.P + off; }
  float* G(long long off) const { return off < 0 ? nullptr : r.G + off; }
  // GEMM weight operand in the storage dtype
  const void* Wg(const ConvL& c) const {
    if (dt == DT_F32) return r.P + c.w;
    return ws + pl.pbf + (size_t)c.w * 2;
  }
  // W^T [cin*k*k][ldt] in the storage dtype (train plans): the dgrad's B operand
  const void* WT(const ConvL& c) const { return ws + pl.wt + (size_t)c.wt * E; }

  // bf16 cast of the arena and the transposed dgrad weights, one launch per step
  int prep_weights() {
    PrepTable t;
    if (dt != DT_F32) {
      PrepJob& j = t.j[t.n++];
      j.src = 0; j.dst = (long long)(pl.pbf / 2); j.R = 1; j.Cc = (int)net.p_total; j.ld = 0;
      j.trans = 0;
    }
    for (int i = 0; i < 9; ++i) {  // fp32 inference: split planes of the fused bottlenecks
      if (!pl.lb_we3[i]) continue;
      const LbL& l = net.lb[i];
      const ConvL* cs[2] = {&l.e, &l.p};
      const size_t offs[2] = {pl.lb_we3[i], pl.lb_wp3[i]};
      for (int k = 0; k < 2; ++k) {
        PrepJob& j = t.j[t.n++];
        j.src = cs[k]->w; j.dst = (long long)(offs[k] / 2); j.R = cs[k]->cout; j.Cc = cs[k]->cin;
        j.ld = 0; j.trans = 3;
      }
    }
    if (train) {
      auto add = [&](const ConvL& c) {
        PrepJob& j = t.j[t.n++];
        j.src = c.w; j.dst = (long long)(pl.wt / E) + c.wt; j.R = c.cout;
        j.Cc = c.cin * c.k * c.k; j.ld = c.ldt; j.trans = 1;
      };
      add(net.ltd1.pw); add(net.ltd2.pw);
      for (int i = 0; i < 9; ++i) { add(net.lb[i].e); add(net.lb[i].p); }
      for (int i = 0; i < 4; ++i) add(net.ppm_c[i]);
      add(net.ppm_o); add(net.ffm_low); add(net.ffm_high);
      add(net.cls1.pw); add(net.cls2.pw); add(net.cls_out);
      if (net.aux) { add(net.aux0); add(net.aux4); }
      PrepJob& z = t.j[t.n++];  // BN arrival counters (fcnt, bcnt: 2 x BN_COUNTERS uint32)
      z.src = 0; z.dst = (long long)(pl.fcnt / E); z.R = 1; z.Cc = (int)(2 * BN_COUNTERS * 4 / E);
      z.ld = 0;
      z.trans = 2;
    }
    if (!t.n) return OK;
    return weights_prep(t, r.P, ws, dt, r.st);
  }

  // ---- deferred weight-gradient reductions ----------------------------------------------
  RedTable red;
  size_t slab_top = 0;  // floats of the plan's slab arena in use
  float* slab_alloc(size_t floats) {
    const size_t n = (floats + 63) / 64 * 64;
    if (slab_top + n > pl.slab_floats) return nullptr;
    float* p = (float*)Bw(pl.slab) + slab_top;
    slab_top += n;
    return p;
  }
  int defer_reduce(float* slab, int S, long long count, float* out, int C9) {
    if (red.n == RED_MAXJOBS) {  // (a stage has <= ~20 jobs; flushing here would let later
      set_error("defer_reduce: more than %d jobs in one call", RED_MAXJOBS);  // slabs overlap)
      return E_INVALID;
    }
    if (count <= 0 || count > 0x7fffffff) {
      set_error("defer_reduce: bad count %lld", count);
      return E_INVALID;
    }
    RedJob& J = red.j[red.n];
    J.slab = slab; J.out = out; J.stride = count; J.S = S; J.count = (int)count;
    J.accumulate = 0; J.C9 = C9;
    red.blk0[red.n] = red.blocks;
    red.blocks += cdiv(count, 256);
    red.n++;
    red.blk0[red.n] = red.blocks;
    return OK;
  }
  // slabs are reused only by kernels enqueued after these launches (same stream)
  // (on the side stream instead, behind the stage's wgrads, it measured no faster: 7.11 vs
  // 7.08-7.10 ms/step)
  bool c0_combine = false;  // the stage's reduce produced the fused conv0 sums (ltd1_c0_bwd)
  int flush_reduce() {
    TRY(join());  // every wgrad slab of the table is written
    const int rc = reduce_slabs_multi(red, r.st);
    red = RedTable();
    slab_top = 0;
    if (rc || !c0_combine) return rc;
    c0_combine = false;
    g_prof_tag = "learning_to_downsample.conv (weight gradient)";
    return conv0_wgrad_combine((const float*)Bw(pl.c0sum), (const float*)Bw(pl.xtab),
                               Wf(pl.c0.mean), G(net.c0.w), r.st);
  }
  int slab_oom() {
    set_error("backward: weight-gradient slab arena exhausted");
    return E_INVALID;
  }

  // ---- operands: an activation buffer, or a lazy unit's z with its BN+ReLU applied on load --
  struct In {
    const void* p;
    int ld;
    const float* sc;
    const float* sh;
  };
  In act(const Unit& u) const {
    if (u.lazy) return {W(u.z), u.C, Wf(u.scale), Wf(u.shift)};
    return {W(u.a), u.ld, nullptr, nullptr};
  }
  static In raw(const void* p, int ld) { return {p, ld, nullptr, nullptr}; }

  // ---- BN glue -----------------------------------------------------------------------
  BnFinalizeArgs fin_args(const Unit& u, const BnL& bn) const {
    BnFinalizeArgs f{};
    f.part = Wf(u.part); f.P = u.nparts; f.C = u.C;
    f.gamma = P(bn.g); f.beta = P(bn.b);
    f.rmean = r.R + bn.rm; f.rvar = r.R + bn.rv;
    f.nbt = r.NBT ? r.NBT + bn.nbt : nullptr;
    f.momentum = r.momentum;
    f.bias = nullptr;
    f.mean = Wf(u.mean); f.invstd = Wf(u.invstd); f.scale = Wf(u.scale); f.shift = Wf(u.shift);
    f.counters = (unsigned*)W(pl.fcnt);  // one launch (fold + last-arriver finalize)
    return f;
  }
  int finalize(const Unit& u, const BnL& bn) {
    g_prof_tag = u.name.c_str();
    return bn_finalize(fin_args(u, bn), r.st);
  }
  // a GEMM producer finishes its BN itself (gemm_nt: in-kernel, or its own finalize launch)
  void gemm_fin(GemmArgs& g, const Unit& u, const BnL& bn) const {
    g.part = Wf(u.part);
    g.tail.counters = (unsigned*)W(pl.fcnt);
    g.tail.fwd = fin_args(u, bn);
    g.tail.tsum = (double*)W(pl.tsum);
  }
  int apply(const Unit& u, bool relu, const void* res = nullptr, int ldres = 0) {
    BnApplyArgs a{};
    a.M = u.M; a.C = u.C;
    a.z = W(u.z); a.ldz = u.C;
    a.scale = Wf(u.scale); a.shift = Wf(u.shift);
    a.res = res; a.ldres = ldres;
    a.relu = relu;
    a.y = W(u.a); a.ldy = u.ld;
    return bn_apply(a, dt, r.st);
  }

  // ---- conv + BN (+ReLU) producers -------------------------------------------------------
  // pointwise conv on X [M][K] (ld ldx); eval: fused BN(+res,+relu); train: stats → apply
  // store_out = false (train): the BN+ReLU output is applied by its only consumer instead
  int pw(const Unit& u, const ConvL& c, const BnL* bn, In x, bool relu,
         const void* res = nullptr, int ldres = 0, bool store_out = true) {
    g_prof_tag = u.name.c_str();
    GemmArgs g{};
    const int K = c.cin * c.k * c.k;  // 1x1 convs; the aux 3x3 runs on its im2col columns
    g.M = (int)u.M; g.N = c.cout; g.K = K;
    g.A = x.p; g.lda = x.ld; g.a_scale = x.sc; g.a_shift = x.sh;
    g.B = Wg(c); g.ldb = K; g.b_trans = 0;
    if (!train || !bn) {
      g.scale = bn ? Wf(u.scale) : nullptr;
      g.shift = bn ? Wf(u.shift) : P(c.b);
      g.R = res; g.ldr = ldres;
      g.relu = relu;
      g.C = W(u.a); g.ldc = u.ld;
      return gemm_nt(g, dt, r.st);
    }
    g.scale = nullptr; g.shift = P(c.b);
    g.C = W(u.z); g.ldc = u.C;
    if (!frozen) gemm_fin(g, u, *bn);
    TRY(gemm_nt(g, dt, r.st));
    return (u.lazy || !store_out) ? OK : apply(u, relu, res, ldres);
  }
  int dw(const Unit& u, const ConvL& c, const BnL& bn, In x, int H, int Wd, int Ho, int Wo,
         int stride) {
    g_prof_tag = u.name.c_str();
    DwArgs d{};
    d.N = pl.N; d.H = H; d.W = Wd; d.C = u.C; d.Ho = Ho; d.Wo = Wo; d.stride = stride;
    d.x = x.p; d.w = P(c.w); d.in_scale = x.sc; d.in_shift = x.sh;
    if (x.ld != u.C) {
      set_error("dw: strided input (ld %d, C %d) not supported", x.ld, u.C);
      return E_UNSUPPORTED;
    }
    if (!train) {
      d.scale = Wf(u.scale); d.shift = Wf(u.shift); d.relu = 1; d.y = W(u.a);
      return dw_fwd(d, dt, r.st);
    }
    d.relu = 0; d.y = W(u.z);
    if (!frozen) {
      d.part = Wf(u.part);
      d.tail.counters = (unsigned*)W(pl.fcnt);  // dw_fwd finishes the BN (in-kernel when it fits)
      d.tail.fwd = fin_args(u, bn);
      d.tail.tsum = (double*)W(pl.tsum);
    }
    TRY(dw_fwd(d, dt, r.st));
    return u.lazy ? OK : apply(u, true);
  }

  // inference stem fusion (stem.hip); FSCNN_STEM_FUSED=0 runs the three unfused launches (the
  // bit-identity test, tests/test_gpu_switches.py)
  static bool stem_enabled() {
    static const bool on = [] {
      const char* e = getenv("FSCNN_STEM_FUSED");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // inference LearningToDownsample.dsconv2 in one launch (dsconv.hip ds2_fwd);
  // FSCNN_LTD2_FUSED=0 runs its depthwise and pointwise launches (the bit-identity test,
  // tests/test_gpu_switches.py)
  static bool ltd2_enabled() {
    static const bool on = [] {
      const char* e = getenv("FSCNN_LTD2_FUSED");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // inference PPM branch convs in one launch (ppm.hip); FSCNN_PPM_FUSED=0 runs the four pointwise
  // launches (the bit-identity test, tests/test_gpu_switches.py)
  static bool ppm_eval_enabled() {
    static const bool on = [] {
      const char* e = getenv("FSCNN_PPM_FUSED");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // inference DSConv fusion (dsconv.hip: the classifier's two DSConvs, the FFM's dwconv +
  // conv_lower_res); FSCNN_DSCONV_FUSED=0 runs dw + pw as two launches (the bit-identity test,
  // tests/test_gpu_switches.py)
  static bool ds_enabled() {
    static const bool on = [] {
      const char* e = getenv("FSCNN_DSCONV_FUSED");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  // FSCNN_FFM_HI=0: the FFM's high-res branch runs as its own GEMM (the fused launch then adds its
  // stored output as a residual)
  static bool ffm_hi_enabled() {
    static const bool on = [] {
      const char* e = getenv("FSCNN_FFM_HI");
      return !(e && e[0] == '0');
    }();
    return on;
  }
  int fold_all() {
    FoldTable t{};
    auto add = [&](const BnL& bn, const Unit& u, const ConvL* conv) {
      FoldEntry& e = t.e[t.n++];
      e.gamma = P(bn.g); e.beta = P(bn.b); e.rmean = r.R + bn.rm; e.rvar = r.R + bn.rv;
      // (frozen: the stored z already carries the conv bias, as in training plans)
      e.bias = (!frozen && conv && conv->b >= 0) ? P(conv->b) : nullptr;
      e.scale = Wf(u.scale); e.shift = Wf(u.shift); e.C = bn.C;
      if (frozen) { e.mean = Wf(u.mean); e.invstd = Wf(u.invstd); }
    };
    add(net.b0, pl.c0, nullptr);
    add(net.ltd1.bdw, pl.l1dw, nullptr); add(net.ltd1.bpw, pl.l1pw, nullptr);
    add(net.ltd2.bdw, pl.l2dw, nullptr); add(net.ltd2.bpw, pl.l2pw, nullptr);
    for (int i = 0; i < 9; ++i) {
      add(net.lb[i].be, pl.lbe[i], nullptr);
      add(net.lb[i].bd, pl.lbd[i], nullptr);
      add(net.lb[i].bp, pl.lbp[i], nullptr);
    }
    for (int i = 0; i < 4; ++i) add(net.ppm_b[i], pl.ppk[i], nullptr);
    add(net.ppm_ob, pl.po, nullptr);
    add(net.ffm_bdw, pl.fdw, nullptr);
    add(net.ffm_blow, pl.flow, &net.ffm_low);
    add(net.ffm_bhigh, pl.fhigh, &net.ffm_high);
    add(net.cls1.bdw, pl.c1dw, nullptr); add(net.cls1.bpw, pl.c1pw, nullptr);
    add(net.cls2.bdw, pl.c2dw, nullptr); add(net.cls2.bpw, pl.c2pw, nullptr);
    if (net.aux) add(net.aux1, pl.aux0, nullptr);
    return bn_fold(t, r.st);
  }

  // ================================ forward ================================================
  int forward() {
    const int N = pl.N;
    g_prof_tag = "weights_prep";
    TRY(prep_weights());
    if (!train || frozen) TRY(fold_all());
    g_prof_tag = pl.c0.name.c_str();
    // ---- LearningToDownsample ----
    StemArgs sa{};
    if (!train) {  // inference: conv + dsconv1 (dw, pw) in one launch (stem.hip) when it fits
      sa.x = r.x; sa.x_dtype = r.x_dtype;
      sa.N = N; sa.H = pl.H; sa.W = pl.W; sa.H1 = pl.H1; sa.W1 = pl.W1; sa.H2 = pl.H2; sa.W2 = pl.W2;
      sa.w0 = P(net.c0.w); sa.sc0 = Wf(pl.c0.scale); sa.sh0 = Wf(pl.c0.shift);
      sa.wd = P(net.ltd1.dw.w); sa.scd = Wf(pl.l1dw.scale); sa.shd = Wf(pl.l1dw.shift);
      sa.wp = Wg(net.ltd1.pw); sa.scp = Wf(pl.l1pw.scale); sa.shp = Wf(pl.l1pw.shift);
      sa.y = W(pl.l1pw.a); sa.ldy = pl.l1pw.ld;
    }
    if (!train && stem_enabled() && stem_ok(sa)) {
      g_prof_tag = "learning_to_downsample.conv + dsconv1 (fused stem)";
      TRY(stem_fwd(sa, dt, r.st));
    } else {
      Conv0Args c{};
      c.x = r.x; c.x_bf16 = r.x_dtype;
      c.N = N; c.H = pl.H; c.W = pl.W; c.Ho = pl.H1; c.Wo = pl.W1;
      c.w = P(net.c0.w);
      if (!train) { c.scale = Wf(pl.c0.scale); c.shift = Wf(pl.c0.shift); c.relu = 1; c.y = W(pl.c0.a); }
      else { c.relu = 0; c.y = W(pl.c0.z); c.part = frozen ? nullptr : Wf(pl.c0.part); }
      TRY(conv0_fwd(c, dt, r.st));
      if (train) {
        if (!frozen) TRY(finalize(pl.c0, net.b0));
        if (!pl.c0.lazy) TRY(apply(pl.c0, true));
      }
      TRY(dw(pl.l1dw, net.ltd1.dw, net.ltd1.bdw, act(pl.c0), pl.H1, pl.W1, pl.H2, pl.W2, 2));
      TRY(pw(pl.l1pw, net.ltd1.pw, &net.ltd1.bpw, act(pl.l1dw), true));
    }
    {
      // inference: dsconv2's depthwise s2 + pointwise in one launch (dsconv.hip ds2_fwd), its
      // 48-channel depthwise output never stored; FSCNN_LTD2_FUSED=0 runs the two launches
      Ds2Args d2{};
      const In xin = act(pl.l1pw);
      d2.x = xin.p; d2.N = N; d2.H = pl.H2; d2.W = pl.W2; d2.Ho = pl.H3; d2.Wo = pl.W3;
      d2.wd = P(net.ltd2.dw.w); d2.scd = Wf(pl.l2dw.scale); d2.shd = Wf(pl.l2dw.shift);
      d2.wp = Wg(net.ltd2.pw); d2.scp = Wf(pl.l2pw.scale); d2.shp = Wf(pl.l2pw.shift);
      d2.y = W(pl.l2pw.a); d2.ldy = pl.l2pw.ld;
      if (!train && ltd2_enabled() && !xin.sc && xin.ld == 48 && ds2_ok(d2)) {
        g_prof_tag = "learning_to_downsample.dsconv2 (dw + pw, fused)";
        TRY(ds2_fwd(d2, dt, r.st));
      } else {
        TRY(dw(pl.l2dw, net.ltd2.dw, net.ltd2.bdw, xin, pl.H2, pl.W2, pl.H3, pl.W3, 2));
        TRY(pw(pl.l2pw, net.ltd2.pw, &net.ltd2.bpw, act(pl.l2dw), true));
      }
    }
    // train: the FeatureFusionModule's high-res branch (conv_higher_res + its BN statistics, on
    // the LTD output only) runs on the side stream beside the latency-bound global feature
    // extractor; its BN finish uses the backward's counters and its own team-sum scratch, so it
    // never shares arrival state with the main stream's producers; joined before the FFM apply
    const bool fhigh_side = train && side != nullptr;
    // the loss head's int8 targets: on the side stream from the start of bottleneck2, beside its
    // latency-bound launches, or on the main stream without a side stream.  (Measured r04, cfg3
    // A/B: the head reading int64 targets 6.07 ms per step, packed beside bottleneck1's HBM-bound
    // launches 6.03, beside bottleneck2/3 6.015; the alternatives were retired as switches in r05.)
    const bool pack = train && !frozen && r.target && ce_head_packs();
    const int pack_at = pack ? 3 : -1;
    if (fhigh_side) {
      TRY(fhigh_fwd(true));
      TRY(flush_side());
    } else if (pack) {
      TRY(pack_targets(r.st));
    }
    // ---- bottlenecks ----
    const void* x = W(pl.l2pw.a);
    int xld = 64;
    int Hc = pl.H3, Wc = pl.W3;
    for (int i = 0; i < 9; ++i) {
      if (fhigh_side && i == pack_at) {
        TRY(side_launch([this](hipStream_t s) { return pack_targets(s); }));
        TRY(flush_side());
      }
      const LbL& l = net.lb[i];
      int Ho = dwout(Hc, l.stride), Wo = dwout(Wc, l.stride);
      IrArgs b;
      if (ir_block_shape(net, pl, i, b)) {
        // inference: the whole stride-1 block in one launch (ir.hip), the 6x-expanded tensor
        // never leaves LDS
        b.x = x; b.ldx = xld; b.y = W(pl.lbp[i].a);
        b.we = Wg(l.e); b.wd = P(l.d.w); b.wp = Wg(l.p);
        b.sc_e = Wf(pl.lbe[i].scale); b.sh_e = Wf(pl.lbe[i].shift);
        b.sc_d = Wf(pl.lbd[i].scale); b.sh_d = Wf(pl.lbd[i].shift);
        b.sc_p = Wf(pl.lbp[i].scale); b.sh_p = Wf(pl.lbp[i].shift);
        if (pl.lb_we3[i]) {
          b.we3 = (const uint16_t*)W(pl.lb_we3[i]);
          b.wp3 = (const uint16_t*)W(pl.lb_wp3[i]);
        }
        g_prof_tag = pl.lbp[i].block_name.c_str();
        TRY(ir_block_fwd(b, dt, r.st));
        x = W(pl.lbp[i].a);
        xld = pl.lbp[i].ld;
        Hc = Ho; Wc = Wo;
        continue;
      }
      IrArgs tb;
      const In xin = i == 0 ? act(pl.l2pw) : raw(x, xld);
      if (irt_shape(i, xin, tb)) {
        TRY(irt_forward(i, xin, tb));
      } else {
        TRY(pw(pl.lbe[i], l.e, &l.be, xin, true));
        TRY(dw(pl.lbd[i], l.d, l.bd, act(pl.lbe[i]), Hc, Wc, Ho, Wo, l.stride));
      }
      bool shortcut = l.stride == 1 && l.cin == l.cout;
      TRY(pw(pl.lbp[i], l.p, &l.bp, act(pl.lbd[i]), false, shortcut ? x : nullptr,
             shortcut ? xld : 0));
      x = W(pl.lbp[i].a);
      xld = pl.lbp[i].ld;
      Hc = Ho; Wc = Wo;
    }
    // ---- PPM ----
    {
      g_prof_tag = "global_feature_extractor.ppm.pool";
      PoolArgs p{};
      p.N = N; p.H = pl.H5; p.W = pl.W5; p.C = 128; p.x = W(pl.concat); p.ldx = 256;
      p.pooled = W(pl.pooled);
      TRY(pyramid_pool(p, dt, r.st));
      static const int base[4] = {0, 1, 5, 14};
      if (ppm_fused()) {
        // the four branch convs + BN + ReLU in one launch (block-local batch statistics)
        g_prof_tag = "global_feature_extractor.ppm.conv1-4";
        PpmFwdArgs f{};
        f.nb = 4; f.K = 128; f.C = 32;
        for (int i = 0; i < 4; ++i) {
          const Unit& u = pl.ppk[i];
          PpmBranchFwd& b = f.b[i];
          b.f = fin_args(u, net.ppm_b[i]);
          b.x = (char*)W(pl.pooled) + (size_t)base[i] * N * 128 * E;
          b.w = Wg(net.ppm_c[i]);
          b.z = W(u.z); b.y = W(u.a); b.ldy = u.ld; b.M = (int)u.M;
        }
        TRY(ppm_branches_fwd(f, dt, r.st));
      } else if (!train && ppm_eval_enabled()) {
        // inference: the four branch convs + folded BN + ReLU as one launch of 16-row tiles,
        // bit-identical to the four pointwise launches (FSCNN_PPM_FUSED=0)
        g_prof_tag = "global_feature_extractor.ppm.conv1-4";
        PpmFwdArgs f{};
        f.nb = 4; f.K = 128; f.C = 32; f.eval = 1;
        for (int i = 0; i < 4; ++i) {
          const Unit& u = pl.ppk[i];
          PpmBranchFwd& b = f.b[i];
          b.f.scale = Wf(u.scale); b.f.shift = Wf(u.shift);
          b.x = (char*)W(pl.pooled) + (size_t)base[i] * N * 128 * E;
          b.w = Wg(net.ppm_c[i]);
          b.y = W(u.a); b.ldy = u.ld; b.M = (int)u.M;
        }
        TRY(ppm_branches_fwd(f, dt, r.st));
      } else {
        for (int i = 0; i < 4; ++i) {
          const void* xin = (char*)W(pl.pooled) + (size_t)base[i] * N * 128 * E;
          TRY(pw(pl.ppk[i], net.ppm_c[i], &net.ppm_b[i], raw(xin, 128), true));
        }
      }
      g_prof_tag = "global_feature_extractor.ppm.upsample";
      PpmUpArgs u{};
      u.N = N; u.H = pl.H5; u.W = pl.W5; u.CF = 32; u.feats = W(pl.feats_a);
      u.y = W(pl.concat); u.ldy = 256; u.coff = 128;
      TRY(ppm_up_fwd(u, dt, r.st));
      TRY(pw(pl.po, net.ppm_o, &net.ppm_ob, raw(W(pl.concat), 256), true));
    }
    // ---- FFM ----
    {
      g_prof_tag = "feature_fusion.upsample";
      UpArgs u{};
      u.N = N; u.Hi = pl.H5; u.Wi = pl.W5; u.C = 128; u.Ho = pl.H3; u.Wo = pl.W3;
      u.x = W(pl.po.a); u.ldx = 128; u.y = W(pl.up_low); u.ldy = 128;
      if (!train) {
        // f = BN_h(conv_h(hr)) ; f = relu(BN_l(conv_l(dw)) + f), the dw and conv_l in one
        // launch (dsconv.hip) when it fits
        DsArgs fa{};  // the upsample too: the depthwise reads the PPM output through it
        fa.x = W(pl.po.a); fa.Hi = pl.H5; fa.Wi = pl.W5;
        fa.N = N; fa.H = pl.H3; fa.W = pl.W3; fa.C = 128; fa.Co = 128;
        fa.wd = P(net.ffm_dw.w); fa.scd = Wf(pl.fdw.scale); fa.shd = Wf(pl.fdw.shift);
        fa.wp = Wg(net.ffm_low); fa.scp = Wf(pl.flow.scale); fa.shp = Wf(pl.flow.shift);
        fa.y = W(pl.flow.a); fa.ldy = pl.flow.ld;
        fa.rs = ds_rows(N, pl.H3, pl.W3);
        // and the high-res branch (conv_higher_res + BN) as a second GEMM in the same launch
        DsArgs fh = fa;
        fh.xh = W(pl.l2pw.a); fh.ldxh = 64; fh.wh = Wg(net.ffm_high);
        fh.sch = Wf(pl.fhigh.scale); fh.shh = Wf(pl.fhigh.shift);
        fa.r = W(pl.f); fa.ldr = 128;
        const bool hi_fused = ds_enabled() && ffm_hi_enabled() && ds_ok(fh);
        if (!hi_fused) TRY(pw(pl.fhigh, net.ffm_high, &net.ffm_bhigh, raw(W(pl.l2pw.a), 64), false));
        if (hi_fused) {
          g_prof_tag = "feature_fusion (upsample + dwconv + conv_lower_res + conv_higher_res, fused)";
          TRY(ds_fwd(fh, dt, r.st));
        } else if (ds_enabled() && ds_ok(fa)) {
          g_prof_tag = "feature_fusion.upsample + dwconv + conv_lower_res (fused)";
          TRY(ds_fwd(fa, dt, r.st));
        } else {
          g_prof_tag = "feature_fusion.upsample";
          TRY(up_nhwc(u, dt, r.st));
          TRY(dw(pl.fdw, net.ffm_dw, net.ffm_bdw, raw(W(pl.up_low), 128), pl.H3, pl.W3, pl.H3, pl.W3, 1));
          TRY(pw(pl.flow, net.ffm_low, &net.ffm_blow, act(pl.fdw), true, W(pl.f), 128));
        }
      } else {
        TRY(up_nhwc(u, dt, r.st));
        TRY(dw(pl.fdw, net.ffm_dw, net.ffm_bdw, raw(W(pl.up_low), 128), pl.H3, pl.W3, pl.H3, pl.W3, 1));
        g_prof_tag = pl.flow.name.c_str();
        GemmArgs g{};
        const In fin = act(pl.fdw);
        g.M = (int)pl.flow.M; g.N = 128; g.K = 128; g.A = fin.p; g.lda = fin.ld;
        g.a_scale = fin.sc; g.a_shift = fin.sh;
        g.B = Wg(net.ffm_low); g.ldb = 128; g.shift = P(net.ffm_low.b);
        g.C = W(pl.flow.z); g.ldc = 128;
        if (!frozen) gemm_fin(g, pl.flow, net.ffm_blow);
        TRY(gemm_nt(g, dt, r.st));
        if (fhigh_side) TRY(join());
        else TRY(fhigh_fwd(false));
        BnApplyArgs a{};
        a.M = pl.flow.M; a.C = 128;
        a.z = W(pl.flow.z); a.ldz = 128; a.scale = Wf(pl.flow.scale); a.shift = Wf(pl.flow.shift);
        a.z2 = W(pl.fhigh.z); a.ldz2 = 128; a.scale2 = Wf(pl.fhigh.scale); a.shift2 = Wf(pl.fhigh.shift);
        a.relu = 1; a.y = W(pl.f); a.ldy = 128;
        TRY(bn_apply(a, dt, r.st));
      }
    }
    // ---- Classifier ----
    // inference: each DSConv (dw + BN + ReLU, pw + BN + ReLU) in one launch (dsconv.hip)
    auto ds_args = [&](const DsL& d, const Unit& udw, const Unit& upw, const void* xin) {
      DsArgs s{};
      s.x = xin; s.N = N; s.H = pl.H3; s.W = pl.W3; s.C = 128; s.Co = 128;
      s.wd = P(d.dw.w); s.scd = Wf(udw.scale); s.shd = Wf(udw.shift);
      s.wp = Wg(d.pw); s.scp = Wf(upw.scale); s.shp = Wf(upw.shift);
      s.y = W(upw.a); s.ldy = upw.ld; s.rs = ds_rows(N, pl.H3, pl.W3);
      return s;
    };
    const bool ds_fuse = !train && ds_enabled() && pl.c1pw.ld == 128;
    const DsArgs ds1 = ds_fuse ? ds_args(net.cls1, pl.c1dw, pl.c1pw, W(pl.f)) : DsArgs{};
    if (ds_fuse && ds_ok(ds1)) {
      g_prof_tag = "classifier.dsconv1 (fused)";
      TRY(ds_fwd(ds1, dt, r.st));
    } else {
      TRY(dw(pl.c1dw, net.cls1.dw, net.cls1.bdw, raw(W(pl.f), 128), pl.H3, pl.W3, pl.H3, pl.W3, 1));
      TRY(pw(pl.c1pw, net.cls1.pw, &net.cls1.bpw, act(pl.c1dw), true));
    }
    // train with Dropout: the dsconv2 pw BN+ReLU output is only read by the dropout, which
    // applies the BN itself (c2pw.a is never stored: one 128-channel write + read fewer)
    const bool drop_fused = train && r.dropout_p > 0.f;
    // (inference: the classifier conv rides in the same launch -- Dropout is the identity -- and
    // the dsconv2 output is never stored)
    DsArgs ds2 = ds_fuse ? ds_args(net.cls2, pl.c2dw, pl.c2pw, W(pl.c1pw.a)) : DsArgs{};
    if (ds_fuse) {
      ds2.wc = Wg(net.cls_out); ds2.bc = P(net.cls_out.b); ds2.ncls = net.num_classes;
      ds2.logits = W(pl.logits); ds2.ldl = pl.Cp;
    }
    const bool cls_fused = ds_fuse && ds_ok(ds2);
    if (cls_fused) {
      g_prof_tag = "classifier.dsconv2 + conv (fused)";
      TRY(ds_fwd(ds2, dt, r.st));
    } else {
      TRY(dw(pl.c2dw, net.cls2.dw, net.cls2.bdw, act(pl.c1pw), pl.H3, pl.W3, pl.H3, pl.W3, 1));
      TRY(pw(pl.c2pw, net.cls2.pw, &net.cls2.bpw, act(pl.c2dw), true, nullptr, 0, !drop_fused));
    }
    const void* cls_in = W(pl.c2pw.a);
    if (drop_fused) {
      DropArgs d{};
      d.N = N; d.H = pl.H3; d.W = pl.W3; d.C = 128; d.x = W(pl.c2pw.z); d.ldx = 128;
      d.x_scale = Wf(pl.c2pw.scale); d.x_shift = Wf(pl.c2pw.shift);
      d.y = W(pl.drop); d.ldy = 128; d.seed = r.seed; d.p = r.dropout_p;
      d.seed_ptr = seed_ptr();
      TRY(dropout(d, dt, r.st));
      cls_in = W(pl.drop);
    }
    g_prof_tag = "classifier.conv";
    if (!cls_fused) {
      GemmArgs g{};
      g.M = (int)pl.c2pw.M; g.N = net.num_classes; g.K = 128; g.A = cls_in; g.lda = 128;
      g.B = Wg(net.cls_out); g.ldb = 128; g.shift = P(net.cls_out.b);
      g.C = W(pl.logits); g.ldc = pl.Cp;
      TRY(gemm_nt(g, dt, r.st));
    }
    if (net.aux && r.aux_out) TRY(forward_aux());
    if (r.target) {
      // ---- fused training head: upsample + CE + gradient at low resolution ----
      if (!train || frozen) {
        set_error("forward_loss needs a training plan (train=1)");
        return E_INVALID;
      }
      g_prof_tag = "head (upsample + cross entropy)";
      CeHeadArgs h{};
      h.N = N; h.C = net.num_classes; h.Hl = pl.H3; h.Wl = pl.W3; h.H = pl.H; h.W = pl.W;
      h.logits = W(pl.logits); h.ldl = pl.Cp; h.target = r.target; h.ignore_index = r.ignore_index;
      h.g_raw = Wf(pl.g_raw); h.part = Wf(pl.head_part);
      if (pack) h.tgt8 = (const signed char*)W(pl.tgt8);
      return ce_head(h, r.loss2, dt, r.st);
    }
    // ---- final bilinear (align_corners) to NCHW ----
    g_prof_tag = "head (upsample)";
    UpArgs u{};
    if (r.labels) {  // eval.py:45 / demo.py:48: only torch.argmax(outputs[0], 1) is consumed
      u.N = N; u.Hi = pl.H3; u.Wi = pl.W3; u.C = net.num_classes; u.Ho = pl.H; u.Wo = pl.W;
      u.x = W(pl.logits); u.ldx = pl.Cp;
      return up_argmax(u, dt, r.labels, r.label_u8, r.st);
    }
    u.N = N; u.Hi = pl.H3; u.Wi = pl.W3; u.C = net.num_classes; u.Ho = pl.H; u.Wo = pl.W;
    u.x = W(pl.logits); u.ldx = pl.Cp; u.y = r.out; u.ldy = 0;
    return up_nchw(u, dt, r.out_dtype, r.st);
  }

  // ---- training bottleneck with the expanded tensor recomputed (ir.hip ir_train_fwd) ----------
  // (models/fast_scnn.py:102-107) 16-bit training plans, the blocks ir_train_blocks() selects
  bool irt_shape(int i, const In& xin, IrArgs& b) const {
    const int sel = ir_train_blocks();
    if (pl.train != 1 || frozen || dt == DT_F32 || sel == 0 || (sel == 1 && i >= 3)) return false;
    const LbL& l = net.lb[i];
    b = IrArgs{};
    b.N = pl.N; b.stride = l.stride;
    b.H = i < 3 ? pl.H4 : pl.H5; b.W = i < 3 ? pl.W4 : pl.W5;
    b.Hi = i == 0 ? pl.H3 : (i < 4 ? pl.H4 : pl.H5);
    b.Wi = i == 0 ? pl.W3 : (i < 4 ? pl.W4 : pl.W5);
    b.Cin = l.cin; b.E = l.cin * 6; b.Cout = l.cout;
    b.x = xin.p; b.ldx = xin.ld; b.x_scale = xin.sc; b.x_shift = xin.sh;
    b.we = Wg(l.e); b.wd = P(l.d.w);
    b.sc_e = Wf(pl.lbe[i].scale); b.sh_e = Wf(pl.lbe[i].shift);
    b.y = W(pl.lbd[i].z); b.ldy = b.E; b.part = Wf(pl.lbd[i].part);
    // the statistics-only pass needs the streaming GEMM (M >= 4096 pixels)
    GemmArgs g = expand_args(i, xin);
    g.part = Wf(pl.lbe[i].part);
    return ir_train_parts(b.N, b.H, b.W, b.stride) <= pl.lbd[i].nparts && ir_train_ok(b, dt) &&
           gemm_stream_ok(g, dt);
  }
  // the expand conv as a GEMM over the block input (statistics only, or the recompute)
  GemmArgs expand_args(int i, const In& xin) const {
    const LbL& l = net.lb[i];
    const Unit& ue = pl.lbe[i];
    GemmArgs g{};
    g.M = (int)ue.M; g.N = ue.C; g.K = l.cin;
    g.A = xin.p; g.lda = xin.ld; g.a_scale = xin.sc; g.a_shift = xin.sh;
    g.B = Wg(l.e); g.ldb = l.cin;
    g.shift = P(l.e.b);
    g.ldc = ue.C;
    return g;
  }
  int irt_forward(int i, const In& xin, IrArgs& b) {
    const LbL& l = net.lb[i];
    const Unit &ue = pl.lbe[i], &ud = pl.lbd[i];
    // BN_e's batch statistics: the expand GEMM with no output (its records + in-kernel finish)
    g_prof_tag = ue.name.c_str();
    GemmArgs g = expand_args(i, xin);
    g.C = nullptr;
    gemm_fin(g, ue, l.be);
    TRY(gemm_nt(g, dt, r.st));
    // expand recomputed per tile -> BN_e + ReLU -> depthwise: only its pre-BN output stored
    g_prof_tag = ud.name.c_str();
    TRY(ir_train_fwd(b, dt, r.st));
    BnFinalizeArgs f = fin_args(ud, l.bd);
    f.P = (int)ir_train_parts(b.N, b.H, b.W, b.stride);
    return bn_finalize(f, r.st);
  }
  // the backward's copy of the expand output the forward never stored: the same GEMM (same MFMA
  // k order, rounded to the storage type) as the statistics pass, with its output
  int irt_recompute(int i) {
    const In xin = i == 0 ? act(pl.l2pw) : raw(W(pl.lbp[i - 1].a), pl.lbp[i - 1].ld);
    IrArgs tb;
    if (!irt_shape(i, xin, tb)) return OK;
    g_prof_tag = pl.lbe[i].name.c_str();
    GemmArgs g = expand_args(i, xin);
    g.C = W(pl.lbe[i].z);
    return gemm_nt(g, dt, r.st);
  }

  // FFM conv_higher_res (models/fast_scnn.py:202) + its BN statistics (train): on the side
  // stream (queued for the next fork) or the caller's
  int fhigh_fwd(bool on_side) {
    g_prof_tag = pl.fhigh.name.c_str();
    GemmArgs g{};
    const In hin = act(pl.l2pw);
    g.M = (int)pl.fhigh.M; g.N = 128; g.K = 64; g.A = hin.p; g.lda = hin.ld;
    g.a_scale = hin.sc; g.a_shift = hin.sh;
    g.B = Wg(net.ffm_high); g.ldb = 64; g.shift = P(net.ffm_high.b);
    g.C = W(pl.fhigh.z); g.ldc = 128;
    if (!frozen) gemm_fin(g, pl.fhigh, net.ffm_bhigh);
    if (!on_side) return gemm_nt(g, dt, r.st);
    if (!frozen) {
      g.tail.counters = (unsigned*)W(pl.bcnt);
      g.tail.tsum = (double*)W(pl.tsum2);
    }
    const int dtc = dt;
    return side_launch([g, dtc](hipStream_t s) { return gemm_nt(g, dtc, s); });
  }

  // aux head (models/fast_scnn.py:24-31,42-45) on the LearningToDownsample output l2pw.a
  int forward_aux() {
    const Unit& u = pl.aux0;
    Im2ColArgs ic{};
    ic.N = pl.N; ic.H = pl.H3; ic.W = pl.W3; ic.C = 64; ic.x = W(pl.l2pw.a); ic.ldx = 64;
    ic.col = W(pl.aux_col); ic.ldcol = 576;
    TRY(im2col3(ic, dt, r.st));
    TRY(pw(u, net.aux0, &net.aux1, raw(W(pl.aux_col), 576), true));
    const void* ain = W(u.a);
    if (train && r.dropout_p > 0.f) {  // Dropout(0.1): the classifier's mask law with seed + 1
      DropArgs d{};
      d.N = pl.N; d.H = pl.H3; d.W = pl.W3; d.C = 32; d.x = W(u.a); d.ldx = 32;
      d.y = W(pl.aux_drop); d.ldy = 32; d.seed = r.seed; d.p = r.dropout_p; d.seed_add = 1;
      d.seed_ptr = seed_ptr();
      TRY(dropout(d, dt, r.st));
      ain = W(pl.aux_drop);
    }
    GemmArgs g{};
    g.M = (int)u.M; g.N = net.num_classes; g.K = 32; g.A = ain; g.lda = 32;
    g.B = Wg(net.aux4); g.ldb = 32; g.shift = P(net.aux4.b);
    g.C = W(pl.aux_logits); g.ldc = pl.Cp;
    TRY(gemm_nt(g, dt, r.st));
    UpArgs up{};
    up.N = pl.N; up.Hi = pl.H3; up.Wi = pl.W3; up.C = net.num_classes; up.Ho = pl.H; up.Wo = pl.W;
    up.x = W(pl.aux_logits); up.ldx = pl.Cp; up.y = r.aux_out; up.ldy = 0;
    return up_nchw(up, dt, r.out_dtype, r.st);
  }

  // aux head backward from d(aux_out); its input gradient is added into l2pw.ga (which the FFM
  // high-res dgrad has written and bottleneck 1's expand dgrad later accumulates into)
  int backward_aux() {
    g_prof_tag = "auxlayer (backward)";
    const int N = pl.N, C = net.num_classes;
    const Unit& u = pl.aux0;
    AxisBwdArgs a{};
    a.n_o1 = (long long)N * C * pl.H; a.n_o2 = 1; a.Lout = pl.W; a.Lin = pl.W3; a.n_in = 1;
    a.g = r.daux; a.g_s1 = pl.W; a.g_s2 = 0; a.g_idx = 1; a.g_in = 0;
    a.d = Bw(pl.t_up); a.d_s1 = pl.W3; a.d_s2 = 0; a.d_idx = 1; a.d_in = 0;
    TRY(axis_bwd(a, dt, DT_F32, r.st));
    AxisBwdArgs b{};
    b.n_o1 = N; b.n_o2 = C; b.Lout = pl.H; b.Lin = pl.H3; b.n_in = pl.W3;
    b.g = Bw(pl.t_up); b.g_s1 = (long long)C * pl.H * pl.W3; b.g_s2 = (long long)pl.H * pl.W3;
    b.g_idx = pl.W3; b.g_in = 1;
    b.d = Bw(pl.g_auxlog); b.d_s1 = (long long)pl.H3 * pl.W3 * pl.Cp; b.d_s2 = 1;
    b.d_idx = (long long)pl.W3 * pl.Cp; b.d_in = pl.Cp;
    TRY(axis_bwd(b, DT_F32, dt, r.st));
    const bool drop = r.dropout_p > 0.f;
    TRY(pw_bwd(net.aux4, u.M, plain(Bw(pl.g_auxlog), pl.Cp), raw(drop ? W(pl.aux_drop) : W(u.a), 32),
               drop ? Bw(pl.g_aux) : Bw(u.ga), 32));
    if (drop) {
      DropArgs d{};
      d.N = N; d.H = pl.H3; d.W = pl.W3; d.C = 32; d.x = Bw(pl.g_aux); d.ldx = 32;
      d.y = Bw(u.ga); d.ldy = 32; d.seed = r.seed; d.p = r.dropout_p; d.seed_add = 1;
      d.seed_ptr = seed_ptr();
      TRY(dropout(d, dt, r.st));
    }
    Dz d;
    TRY(bn_bwd_x(u, net.aux1, Bw(u.ga), 32, true, dz_buf(u), d));
    TRY(pw_bwd(net.aux0, u.M, d, raw(W(pl.aux_col), 576), Bw(pl.aux_dcol), 576));
    Col2ImArgs cc{};
    cc.N = N; cc.H = pl.H3; cc.W = pl.W3; cc.C = 64; cc.dcol = Bw(pl.aux_dcol); cc.ldcol = 576;
    cc.dx = Bw(pl.l2pw.ga); cc.lddx = 64; cc.accumulate = 1;
    return col2im3(cc, dt, r.st);
  }

  // ================================ backward ===============================================
  // BN backward of unit u: dy = u.ga (ld u.ga_ld), mask = relu output (or null) → dz scratch.
  // u.bdone: the dgrad that produced dy already reduced and finished this BN (coef / dgamma /
  // dbeta written, set_btarget), so only the apply runs.
  // dz operand of a conv backward: a materialised tensor, or dy + z + transform table
  struct Dz {
    const void* p;
    int ld;
    const void* z;
    const float* tab;
  };
  static Dz plain(const void* p, int ld) { return {p, ld, nullptr, nullptr}; }
  // reduce + finalize of u's BN backward unless its dy producer did both
  int bn_bwd_stats(const Unit& u, const BnL& bn, const void* dy, int lddy, const void* mask,
                   int ldmask, bool relu_z, const BnBwdTab& tb) {
    if (u.bdone.get()) return OK;
    BnBwdArgs b{};
    b.M = u.M; b.C = u.C;
    b.dy = dy; b.lddy = lddy; b.mask = mask; b.ldmask = ldmask;
    b.z = W(u.z); b.ldz = u.C;
    b.mean = Wf(u.mean); b.invstd = Wf(u.invstd); b.scale = Wf(u.scale);
    b.shift = Wf(u.shift); b.relu_z = relu_z;
    b.part = (float*)Bw(pl.bnpart);
    TRY(bn_bwd_reduce(b, dt, r.st));
    int rpb;
    const int P = bn_bwd_parts(u.M, u.C, dt, &rpb);
    return bn_bwd_finalize((float*)Bw(pl.bnpart), P, u.C, bcount(u), G(bn.g), G(bn.b),
                           (float*)Bw(pl.coef), r.st, (unsigned*)W(pl.bcnt), tb);
  }
  // Where a BN-backward dz is formed: by bn_bwd_apply (materialised), or — `streaming`, only
  // conv0's weight gradient, a bandwidth-efficient streaming consumer — by the consumer while it
  // stages its operand (common.hpp bwdx_apply): measured on MI355X (cfg3), conv0's wgrad absorbs
  // the extra z read at ~5.4 TB/s (c0's 800 MB apply, 189 us, becomes +49 us), while the
  // latency-bound pointwise / depthwise consumers slowed down by more than the apply they replaced
  // (+0.89 ms vs -0.58 ms over 15 BNs), so they read a materialised dz.
  // fused form: reduce + finalize only; the consumer applies it on load
  int bn_bwd_x(const Unit& u, const BnL& bn, const void* dy, int lddy, bool relu_z, void* dz,
               Dz& out, bool streaming = false) {
    g_prof_tag = u.name.c_str();
    if (!train || !streaming) {
      TRY(bn_bwd(u, bn, dy, lddy, nullptr, 0, dz, relu_z));
      out = plain(dz, u.C);
      return OK;
    }
    const BnBwdTab tb = bwd_tab(u, relu_z, tab_slot(u));  // written by u's dy producer
    TRY(bn_bwd_stats(u, bn, dy, lddy, nullptr, 0, relu_z, tb));
    out = {dy, lddy, W(u.z), tb.tab};
    return OK;
  }
  int bn_bwd(const Unit& u, const BnL& bn, const void* dy, int lddy, const void* mask,
             int ldmask, void* dz, bool relu_z = false) {
    g_prof_tag = u.name.c_str();
    if (!dz) {
      set_error("backward: dz arena exhausted (%s)", u.name.c_str());
      return E_INVALID;
    }
    TRY(bn_bwd_stats(u, bn, dy, lddy, mask, ldmask, relu_z, BnBwdTab()));
    BnBwdArgs b{};
    b.M = u.M; b.C = u.C;
    b.dy = dy; b.lddy = lddy; b.mask = mask; b.ldmask = ldmask;
    b.z = W(u.z); b.ldz = u.C;
    b.mean = Wf(u.mean); b.invstd = Wf(u.invstd); b.scale = Wf(u.scale);
    b.shift = Wf(u.shift); b.relu_z = relu_z;
    b.coef = (float*)Bw(pl.coef);
    b.dz = dz; b.lddz = u.C;
    return bn_bwd_apply(b, dt, r.st);
  }
  // the FeatureFusionModule's two BNs, f = relu(BN_l(z_l) + BN_h(z_h)) (models/fast_scnn.py
  // :207-218): the same dy (g_f) and ReLU mask (f) for both, so one reduce pass and one apply
  // pass read them once (the reduce's sum of dy_r is shared; the finishes stay per BN)
  int bn_bwd_pair(const Unit& u1, const BnL& bn1, const Unit& u2, const BnL& bn2, const void* dy,
                  int lddy, const void* mask, int ldmask, void* dz1, void* dz2) {
    g_prof_tag = "feature_fusion (BN backward, both branches)";
    int rpb;
    const int P = bn_bwd_parts(u1.M, u1.C, dt, &rpb);
    if (!dz1 || !dz2 || u1.M != u2.M || u1.C != u2.C || 4 * u1.C > 2048 ||
        (size_t)P * 4 * u1.C > pl.bnpart_floats) {
      set_error("bn_bwd_pair: units do not pair or the record arena is too small");
      return E_INVALID;
    }
    BnBwdArgs b{};
    b.M = u1.M; b.C = u1.C;
    b.dy = dy; b.lddy = lddy; b.mask = mask; b.ldmask = ldmask;
    b.z = W(u1.z); b.ldz = u1.C;
    b.mean = Wf(u1.mean); b.invstd = Wf(u1.invstd); b.scale = Wf(u1.scale); b.shift = Wf(u1.shift);
    b.z2 = W(u2.z); b.mean2 = Wf(u2.mean); b.invstd2 = Wf(u2.invstd); b.scale2 = Wf(u2.scale);
    b.part = (float*)Bw(pl.bnpart);
    b.part2 = b.part + (size_t)P * 2 * u1.C;
    TRY(bn_bwd_reduce(b, dt, r.st));
    float* coef = (float*)Bw(pl.coef);
    float* coef2 = coef + 2 * u1.C;
    TRY(bn_bwd_finalize(b.part, P, u1.C, bcount(u1), G(bn1.g), G(bn1.b), coef, r.st,
                        (unsigned*)W(pl.bcnt), BnBwdTab()));
    TRY(bn_bwd_finalize(b.part2, P, u2.C, bcount(u2), G(bn2.g), G(bn2.b), coef2, r.st,
                        (unsigned*)W(pl.bcnt), BnBwdTab()));
    b.coef = coef; b.coef2 = coef2;
    b.dz = dz1; b.dz2 = dz2; b.lddz = u1.C;
    return bn_bwd_apply(b, dt, r.st);
  }
  // BN whose output is relu(BN(z)) with no second branch: the ReLU mask is recomputed from z
  int bn_bwd_relu(const Unit& u, const BnL& bn, const void* dy, int lddy, void* dz) {
    return bn_bwd(u, bn, dy, lddy, nullptr, 0, dz, true);
  }
  // the dgrad producing the dy of BN (u, bn) also reduces and finishes that BN's backward
  // (gemm_nt: in-kernel, or its own finalize launch); its bn_bwd then only applies
  void set_btarget(GemmArgs& g, const BTarget& t) {
    const Unit& u = *t.u;
    g.bpart = (float*)Bw(pl.bnpart);
    g.bz = W(u.z); g.ldbz = u.C;
    g.bmean = Wf(u.mean); g.binvstd = Wf(u.invstd); g.bscale = Wf(u.scale); g.bshift = Wf(u.shift);
    g.bmode = t.mode;
    g.tail.counters = (unsigned*)W(pl.bcnt);
    g.tail.tsum = (double*)W(pl.tsum);
    g.tail.count = bcount(u);
    g.tail.dgamma = G(t.bn->g);
    g.tail.dbeta = G(t.bn->b);
    g.tail.coef = (float*)Bw(pl.coef);
    // the operand table too: a fused consumer (depthwise, or every pointwise one in mode 2)
    // reads it instead of a materialised dz (the target's own slot, see bn_bwd_x)
    g.tail.tab = bwd_tab(u, t.mode == 2, tab_slot(u));
  }
  BnBwdTab bwd_tab(const Unit& u, bool relu, float* tab) const {
    BnBwdTab tb;
    tb.tab = tab;
    tb.scale = Wf(u.scale); tb.shift = Wf(u.shift); tb.mean = Wf(u.mean); tb.invstd = Wf(u.invstd);
    tb.relu = relu;
    return tb;
  }
  // pw conv backward given dz [M][cout]: wgrad into G, dgrad into dX (ld lddx) (+R)
  GemmArgs pw_dgrad_args(const ConvL& c, long long M, Dz dz, void* dX, int lddx, const void* R,
                         int ldr, BTarget bt, const DropArgs* dro) {
    GemmArgs g{};
    g.M = (int)M; g.N = c.cin * c.k * c.k; g.K = c.cout; g.A = dz.p; g.lda = dz.ld;
    g.B = WT(c); g.ldb = c.ldt; g.b_trans = 0;
    g.R = R; g.ldr = ldr;
    g.C = dX; g.ldc = lddx;
    if (bt.u && train) set_btarget(g, bt);
    if (dro) {
      g.drop_hw = dro->H * dro->W; g.drop_thr = dropout_threshold(dro->p); g.drop_p = dro->p;
      g.drop_seed = dro->seed; g.drop_seed_ptr = dro->seed_ptr; g.drop_seed_add = dro->seed_add;
    }
    return g;
  }
  // dro: a Dropout between this conv's input and the BN that bt names (the classifier): the
  // dgrad applies its mask to dX (GemmArgs::drop_hw), so the BN partials are the dropped ones
  int pw_bwd(const ConvL& c, long long M, Dz dz, In X, void* dX, int lddx,
             const void* R = nullptr, int ldr = 0, BTarget bt = BTarget(),
             const DropArgs* dro = nullptr) {
    const int K = c.cin * c.k * c.k;
    GemmTnArgs t{};
    t.M = (int)M; t.N = c.cout; t.K = K; t.D = dz.p; t.ldd = dz.ld; t.X = X.p; t.ldx = X.ld;
    t.x_scale = X.sc; t.x_shift = X.sh;
    if (dz.tab) {  // (bn_bwd_x forms a fused dz for conv0's wgrad only)
      set_error("pw_bwd: a fused BN-backward operand is not supported here");
      return E_UNSUPPORTED;
    }
    int S = gemm_tn_splits((int)M, c.cout, K);
    t.slab = slab_alloc((size_t)S * c.cout * K);
    if (!t.slab) return slab_oom();
    const int dtc = dt;
    TRY(side_launch([t, S, dtc](hipStream_t s) { return gemm_tn(t, S, dtc, s); }));
    TRY(defer_reduce(t.slab, S, (long long)c.cout * K, G(c.w), 0));
    if (c.b >= 0) {
      float* part = slab_alloc((size_t)colsum_parts((int)M) * c.cout);
      if (!part) return slab_oom();
      const void* dp = dz.p;
      const int Mi = (int)M, co = c.cout, ld = dz.ld;
      TRY(side_launch([dp, Mi, co, ld, part, dtc](hipStream_t s) {
        return colsum(dp, Mi, co, ld, part, dtc, s);
      }));
      TRY(defer_reduce(part, colsum_parts((int)M), c.cout, G(c.b), 0));
    }
    TRY(flush_side());
    if (!dX) return OK;
    const GemmArgs g = pw_dgrad_args(c, M, dz, dX, lddx, R, ldr, bt, dro);
    TRY(gemm_nt(g, dt, r.st));
    if (bt.u && train) bt.u->bdone.set();
    return OK;
  }
  static BTarget relu_target(const Unit& u, const BnL& bn) {
    BTarget t; t.u = &u; t.bn = &bn; t.mode = 2; return t;
  }
  static BTarget plain_target(const Unit& u, const BnL& bn) {
    BTarget t; t.u = &u; t.bn = &bn; t.mode = 0; return t;
  }
  // dw conv backward given dz [M][C]: wgrad into G, dgrad into dX
  // bt: the BN whose dy the dgrad produces — its reduce pass is folded into the dgrad (records
  // in bnpart; that BN's backward then only finalizes and applies)
  // dz: this dw's BN-backward output, materialised or as (dy, z, table) applied on load
  int dw_bwd(const ConvL& c, int C, Dz dz, In X, int H, int Wd, int Ho, int Wo,
             int stride, void* dX, BTarget bt = BTarget()) {
    if (dz.ld != C) {
      set_error("dw_bwd: strided dz (ld %d, C %d) not supported", dz.ld, C);
      return E_UNSUPPORTED;
    }
    DwBwdArgs d{};
    d.N = pl.N; d.H = H; d.W = Wd; d.C = C; d.Ho = Ho; d.Wo = Wo; d.stride = stride;
    d.x = X.p; d.x_scale = X.sc; d.x_shift = X.sh; d.dy = dz.p; d.w = P(c.w); d.dx = dX;
    if (dz.tab) {
      set_error("dw_bwd: a fused BN-backward operand is not supported here");
      return E_UNSUPPORTED;
    }
    const int S = dw_wgrad_parts(pl.N, Ho, Wo, C, dt, stride);
    d.slab = slab_alloc((size_t)S * 9 * C);
    if (!d.slab) return slab_oom();
    {
      const DwBwdArgs dw = d;
      const int dtc = dt;
      TRY(side_launch([dw, dtc](hipStream_t s) { return dw_wgrad(dw, dtc, s); }));
      TRY(flush_side());
    }
    TRY(defer_reduce(d.slab, S, 9LL * C, G(c.w), C));
    if (!dX) return OK;  // input gradient formed elsewhere (ltd1_c0_bwd)
    const bool br = bt.u && train;
    if (br) {
      const Unit& u = *bt.u;
      d.bs.part = (float*)Bw(pl.bnpart);
      d.bs.z = W(u.z);
      d.bs.mean = Wf(u.mean); d.bs.invstd = Wf(u.invstd);
      d.bs.scale = Wf(u.scale); d.bs.shift = Wf(u.shift);
      d.bs.mode = bt.mode;
      // and finishes that BN's backward (dgamma, dbeta, coefficients, operand table): in the
      // kernel's last workgroups when its records fit the counters, else its own launch
      d.tail.counters = (unsigned*)W(pl.bcnt);
      d.tail.tsum = (double*)W(pl.tsum);
      d.tail.count = bcount(u);
      d.tail.dgamma = G(bt.bn->g);
      d.tail.dbeta = G(bt.bn->b);
      d.tail.coef = (float*)Bw(pl.coef);
      d.tail.tab = bwd_tab(u, bt.mode == 2, tab_slot(u));
    }
    TRY(dw_dgrad(d, dt, r.st));
    if (br) bt.u->bdone.set();
    return OK;
  }

  int backward_head() {
    g_prof_tag = "head (backward) + classifier.conv";
    const int N = pl.N, C = net.num_classes;
    if (r.gloss) {
      // fused head: the low-res logits gradient was gathered in the forward; scale by dL/dloss / count
      TRY(ce_head_scale(Wf(pl.g_raw), Bw(pl.g_logits), pl.c2pw.M, C, pl.Cp, r.gloss, r.loss2, dt,
                        r.st));
    } else {
      // final upsample: W pass (NCHW rows) then H pass into NHWC low-res logits grad
      AxisBwdArgs a{};
      a.n_o1 = (long long)N * C * pl.H; a.n_o2 = 1; a.Lout = pl.W; a.Lin = pl.W3; a.n_in = 1;
      a.g = r.dout; a.g_s1 = pl.W; a.g_s2 = 0; a.g_idx = 1; a.g_in = 0;
      a.d = Bw(pl.t_up); a.d_s1 = pl.W3; a.d_s2 = 0; a.d_idx = 1; a.d_in = 0;
      TRY(axis_bwd(a, dt, DT_F32, r.st));
      AxisBwdArgs b{};
      b.n_o1 = N; b.n_o2 = C; b.Lout = pl.H; b.Lin = pl.H3; b.n_in = pl.W3;
      b.g = Bw(pl.t_up); b.g_s1 = (long long)C * pl.H * pl.W3; b.g_s2 = (long long)pl.H * pl.W3;
      b.g_idx = pl.W3; b.g_in = 1;
      b.d = Bw(pl.g_logits); b.d_s1 = (long long)pl.H3 * pl.W3 * pl.Cp; b.d_s2 = 1;
      b.d_idx = (long long)pl.W3 * pl.Cp; b.d_in = pl.Cp;
      TRY(axis_bwd(b, DT_F32, dt, r.st));
    }
    // classifier 1x1 (+bias), dropout
    const bool drop = r.dropout_p > 0.f;
    // train: the dgrad applies the dropout mask itself and folds dsconv2 pw's BN-backward reduce
    // (one 128-channel write + read and the dropout and reduce launches fewer)
    // (the streaming kernel only: not for the small test shapes, M < 4096)
    DropArgs dd{};
    dd.N = N; dd.H = pl.H3; dd.W = pl.W3; dd.C = 128; dd.seed = r.seed; dd.p = r.dropout_p;
    dd.seed_ptr = seed_ptr();
    const BTarget dbt = relu_target(pl.c2pw, net.cls2.bpw);
    const bool dfuse = drop && train && drop_dgrad_on() &&
                       gemm_stream_ok(pw_dgrad_args(net.cls_out, pl.c2pw.M, plain(Bw(pl.g_logits), pl.Cp),
                                                    Bw(pl.c2pw.ga), 128, nullptr, 0, dbt, &dd),
                                      dt);
    if (dfuse) {
      TRY(pw_bwd(net.cls_out, pl.c2pw.M, plain(Bw(pl.g_logits), pl.Cp), raw(W(pl.drop), 128),
                 Bw(pl.c2pw.ga), 128, nullptr, 0, dbt, &dd));
    } else {
      TRY(pw_bwd(net.cls_out, pl.c2pw.M, plain(Bw(pl.g_logits), pl.Cp),
                 raw(drop ? W(pl.drop) : W(pl.c2pw.a), 128), drop ? Bw(pl.g_drop) : Bw(pl.c2pw.ga),
                 128));
    }
    if (drop && !dfuse) {
      DropArgs d{};
      d.N = N; d.H = pl.H3; d.W = pl.W3; d.C = 128; d.x = Bw(pl.g_drop); d.ldx = 128;
      d.y = Bw(pl.c2pw.ga); d.ldy = 128; d.seed = r.seed; d.p = r.dropout_p;
      d.seed_ptr = seed_ptr();
      TRY(dropout(d, dt, r.st));
    }
    // classifier dsconv2, dsconv1
    Dz d;
    TRY(bn_bwd_x(pl.c2pw, net.cls2.bpw, Bw(pl.c2pw.ga), 128, true, dz_buf(pl.c2pw), d));
    TRY(pw_bwd(net.cls2.pw, pl.c2pw.M, d, act(pl.c2dw), Bw(pl.c2dw.ga), 128, nullptr, 0,
               relu_target(pl.c2dw, net.cls2.bdw)));
    TRY(bn_bwd_x(pl.c2dw, net.cls2.bdw, Bw(pl.c2dw.ga), 128, true, dz_buf(pl.c2dw), d));
    TRY(dw_bwd(net.cls2.dw, 128, d, act(pl.c1pw), pl.H3, pl.W3, pl.H3, pl.W3, 1, Bw(pl.c1pw.ga),
               relu_target(pl.c1pw, net.cls1.bpw)));
    TRY(flush_side());
    TRY(bn_bwd_x(pl.c1pw, net.cls1.bpw, Bw(pl.c1pw.ga), 128, true, dz_buf(pl.c1pw), d));
    TRY(pw_bwd(net.cls1.pw, pl.c1pw.M, d, act(pl.c1dw), Bw(pl.c1dw.ga), 128, nullptr, 0,
               relu_target(pl.c1dw, net.cls1.bdw)));
    TRY(bn_bwd_x(pl.c1dw, net.cls1.bdw, Bw(pl.c1dw.ga), 128, true, dz_buf(pl.c1dw), d));
    TRY(dw_bwd(net.cls1.dw, 128, d, raw(W(pl.f), 128), pl.H3, pl.W3, pl.H3, pl.W3, 1, Bw(pl.g_f)));
    TRY(flush_side());
    // FFM: f = relu(BN_l(z_l) + BN_h(z_h))
    // (low branch first so the low 1x1 dgrad can hand its BN-backward partials straight to
    //  the FFM dwconv BN; the high branch only needs g_f and writes l2pw.ga)
    void* zl = dz_buf(pl.flow);
    void* zh = dz_buf(pl.fhigh);
    // both branch BNs in one reduce and one apply (same dy g_f and mask f)
    TRY(bn_bwd_pair(pl.flow, net.ffm_blow, pl.fhigh, net.ffm_bhigh, Bw(pl.g_f), 128, W(pl.f), 128,
                    zl, zh));
    TRY(pw_bwd(net.ffm_low, pl.flow.M, plain(zl, 128), act(pl.fdw), Bw(pl.fdw.ga), 128, nullptr, 0,
               relu_target(pl.fdw, net.ffm_bdw)));
    TRY(bn_bwd_x(pl.fdw, net.ffm_bdw, Bw(pl.fdw.ga), 128, true, dz_buf(pl.fdw), d));
    TRY(dw_bwd(net.ffm_dw, 128, d, raw(W(pl.up_low), 128), pl.H3, pl.W3, pl.H3, pl.W3, 1,
               Bw(pl.g_up)));
    TRY(flush_side());
    TRY(pw_bwd(net.ffm_high, pl.fhigh.M, plain(zh, 128), act(pl.l2pw), Bw(pl.l2pw.ga), 64));
    TRY(flush_side());
    if (net.aux) TRY(backward_aux());
    // upsample (x4, ac) backward: W pass then H pass → grad of ppm.out activation
    g_prof_tag = "feature_fusion.upsample (backward)";
    {
      AxisBwdArgs a{};
      a.n_o1 = (long long)N * pl.H3; a.n_o2 = 1; a.Lout = pl.W3; a.Lin = pl.W5; a.n_in = 128;
      a.g = Bw(pl.g_up); a.g_s1 = (long long)pl.W3 * 128; a.g_s2 = 0; a.g_idx = 128; a.g_in = 1;
      a.d = Bw(pl.t_up2); a.d_s1 = (long long)pl.W5 * 128; a.d_s2 = 0; a.d_idx = 128; a.d_in = 1;
      TRY(axis_bwd(a, dt, DT_F32, r.st));
      AxisBwdArgs b{};
      b.n_o1 = N; b.n_o2 = 1; b.Lout = pl.H3; b.Lin = pl.H5; b.n_in = (long long)pl.W5 * 128;
      b.g = Bw(pl.t_up2); b.g_s1 = (long long)pl.H3 * pl.W5 * 128; b.g_s2 = 0;
      b.g_idx = (long long)pl.W5 * 128; b.g_in = 1;
      b.d = Bw(pl.po.ga); b.d_s1 = (long long)pl.H5 * pl.W5 * 128; b.d_s2 = 0;
      b.d_idx = (long long)pl.W5 * 128; b.d_in = 1;
      TRY(axis_bwd(b, DT_F32, dt, r.st));
    }
    // PPM out 1x1 (256→128) over the concat buffer
    TRY(bn_bwd_x(pl.po, net.ppm_ob, Bw(pl.po.ga), 128, true, dz_buf(pl.po), d));
    TRY(pw_bwd(net.ppm_o, pl.po.M, d, raw(W(pl.concat), 256), Bw(pl.g_concat), 256));
    TRY(flush_side());
    {
      PpmUpArgs u{};
      u.N = N; u.H = pl.H5; u.W = pl.W5; u.CF = 32; u.feats = nullptr;
      u.y = Bw(pl.g_concat); u.ldy = 256; u.coff = 128;
      g_prof_tag = "global_feature_extractor.ppm.upsample (backward)";
      TRY(ppm_up_bwd(u, Bw(pl.g_feats), dt, r.st));
      static const int base[4] = {0, 1, 5, 14};
      if (ppm_fused()) {
        g_prof_tag = "global_feature_extractor.ppm.conv1-4 (backward)";
        PpmBwdArgs f{};
        f.nb = 4; f.K = 128; f.C = 32;
        for (int i = 0; i < 4; ++i) {
          const Unit& u4 = pl.ppk[i];
          const size_t off = (size_t)base[i] * N;
          PpmBranchBwd& b = f.b[i];
          b.dy = (char*)Bw(pl.g_feats) + off * 32 * E; b.lddy = 32;
          b.y = (char*)W(pl.feats_a) + off * 32 * E; b.ldy = 32;
          b.z = W(u4.z);
          b.mean = Wf(u4.mean); b.invstd = Wf(u4.invstd); b.scale = Wf(u4.scale);
          b.gamma = P(net.ppm_b[i].g);
          b.x = (char*)W(pl.pooled) + off * 128 * E;
          b.w = Wg(net.ppm_c[i]);
          b.dgamma = G(net.ppm_b[i].g); b.dbeta = G(net.ppm_b[i].b);
          b.dw = G(net.ppm_c[i].w);
          b.dx = (char*)Bw(pl.g_pooled) + off * 128 * E;
          b.M = (int)u4.M;
        }
        TRY(ppm_branches_bwd(f, dt, r.st));
      }
      for (int i = 0; i < 4 && !ppm_fused(); ++i) {
        const Unit& u4 = pl.ppk[i];
        size_t off = (size_t)base[i] * N;
        void* zp = dz_buf(u4);
        TRY(bn_bwd(u4, net.ppm_b[i], (char*)Bw(pl.g_feats) + off * 32 * E, 32,
                   (char*)W(pl.feats_a) + off * 32 * E, 32, zp));
        TRY(pw_bwd(net.ppm_c[i], u4.M, plain(zp, 32), raw((char*)W(pl.pooled) + off * 128 * E, 128),
                   (char*)Bw(pl.g_pooled) + off * 128 * E, 128));
      }
      PoolBwdArgs p{};
      p.N = N; p.H = pl.H5; p.W = pl.W5; p.C = 128; p.dpooled = Bw(pl.g_pooled);
      p.dx = Bw(pl.g_concat); p.lddx = 256; p.accumulate = 1;
      g_prof_tag = "global_feature_extractor.ppm.pool (backward)";
      TRY(pyramid_pool_bwd(p, dt, r.st));
    }
    return OK;
  }

  int backward_block(int i) {
    const LbL& l = net.lb[i];
    const Unit &ue = pl.lbe[i], &ud = pl.lbd[i], &up = pl.lbp[i];
    int Hin = i == 0 ? pl.H3 : (i <= 3 ? pl.H4 : pl.H5);
    int Win = i == 0 ? pl.W3 : (i <= 3 ? pl.W4 : pl.W5);
    int Ho = i < 3 ? pl.H4 : pl.H5, Wo = i < 3 ? pl.W4 : pl.W5;
    const void* x = i == 0 ? W(pl.l2pw.a) : W(pl.lbp[i - 1].a);
    int xld = i == 0 ? 64 : pl.lbp[i - 1].ld;
    void* gx = i == 0 ? Bw(pl.l2pw.ga) : Bw(pl.lbp[i - 1].ga);
    int gxld = i == 0 ? 64 : pl.lbp[i - 1].ga_ld;
    bool shortcut = l.stride == 1 && l.cin == l.cout;
    const int e = l.cin * 6;
    TRY(irt_recompute(i));  // (the expanded tensor, when the forward did not store it)
    // up's dy was produced by block i+1's expand dgrad with fused partials (not for the last
    // block: its dy is the PPM concat gradient)
    Dz d;
    TRY(bn_bwd_x(up, l.bp, Bw(up.ga), up.ga_ld, false, dz_buf(up), d));
    TRY(pw_bwd(l.p, up.M, d, act(ud), Bw(ud.ga), e, nullptr, 0, relu_target(ud, l.bd)));
    TRY(bn_bwd_x(ud, l.bd, Bw(ud.ga), e, true, dz_buf(ud), d));
    TRY(dw_bwd(l.d, e, d, act(ue), Hin, Win, Ho, Wo, l.stride, Bw(ue.ga), relu_target(ue, l.be)));
    TRY(bn_bwd_x(ue, l.be, Bw(ue.ga), e, true, dz_buf(ue), d));
    // grad wrt x: dgrad (+ identity path of the shortcut, or + FFM's contribution for hr)
    const void* R = shortcut ? Bw(up.ga) : (i == 0 ? gx : nullptr);
    int ldr = shortcut ? up.ga_ld : (i == 0 ? gxld : 0);
    // the dgrad is the dy of the previous block's project BN (or of LTD.dsconv2's pw BN)
    const BTarget bt = i == 0 ? relu_target(pl.l2pw, net.ltd2.bpw)
                              : plain_target(pl.lbp[i - 1], net.lb[i - 1].bp);
    TRY(pw_bwd(l.e, ue.M, d, i == 0 ? act(pl.l2pw) : raw(x, xld), gx, gxld, R, ldr, bt));
    return flush_side();  // the block's three wgrads behind one fork
  }

  // LTD.dsconv1.dw input gradient + conv0's BN backward + conv0 weight gradient in one pass
  // (conv0.hip ltd_c0_bwd); dW is formed from the reduced sums after the stage's reduce
  int ltd1_c0_bwd(const Dz& d) {
    g_prof_tag = "learning_to_downsample.dsconv1.dw + conv (backward, fused)";
    const Unit& u = pl.c0;
    LtdC0BwdArgs f{};
    f.N = pl.N; f.H = pl.H1; f.W = pl.W1; f.Ho = pl.H2; f.Wo = pl.W2;
    f.dy = d.p; f.w = P(net.ltd1.dw.w);
    f.bs.part = (float*)Bw(pl.bnpart);
    f.bs.z = W(u.z);
    f.bs.mean = Wf(u.mean); f.bs.invstd = Wf(u.invstd);
    f.bs.scale = Wf(u.scale); f.bs.shift = Wf(u.shift);
    f.bs.mode = 2;
    f.tail.counters = (unsigned*)W(pl.bcnt);
    f.tail.tsum = (double*)W(pl.tsum);
    f.tail.count = bcount(u);
    f.tail.dgamma = G(net.b0.g);
    f.tail.dbeta = G(net.b0.b);
    f.tail.coef = (float*)Bw(pl.coef);
    f.tail.tab = bwd_tab(u, true, tab_slot(u));
    f.x = r.x; f.x_dtype = r.x_dtype; f.XH = pl.H; f.XW = pl.W;
    const int S = ltd_c0_bwd_parts(pl.N, pl.H1, pl.W1);
    f.slab = slab_alloc((size_t)S * LC0_SLAB);
    if (!f.slab) return slab_oom();
    TRY(ltd_c0_bwd(f, dt, r.st));
    u.bdone.set();
    TRY(defer_reduce(f.slab, S, LC0_SLAB, (float*)Bw(pl.c0sum), 0));
    c0_combine = true;
    return OK;
  }

  int backward_ltd() {
    Dz d;
    TRY(bn_bwd_x(pl.l2pw, net.ltd2.bpw, Bw(pl.l2pw.ga), 64, true, dz_buf(pl.l2pw), d));
    TRY(pw_bwd(net.ltd2.pw, pl.l2pw.M, d, act(pl.l2dw), Bw(pl.l2dw.ga), 48, nullptr, 0,
               relu_target(pl.l2dw, net.ltd2.bdw)));
    TRY(bn_bwd_x(pl.l2dw, net.ltd2.bdw, Bw(pl.l2dw.ga), 48, true, dz_buf(pl.l2dw), d));
    TRY(dw_bwd(net.ltd2.dw, 48, d, act(pl.l1pw), pl.H2, pl.W2, pl.H3, pl.W3, 2, Bw(pl.l1pw.ga),
               relu_target(pl.l1pw, net.ltd1.bpw)));
    TRY(flush_side());
    TRY(bn_bwd_x(pl.l1pw, net.ltd1.bpw, Bw(pl.l1pw.ga), 48, true, dz_buf(pl.l1pw), d));
    TRY(pw_bwd(net.ltd1.pw, pl.l1pw.M, d, act(pl.l1dw), Bw(pl.l1dw.ga), 32, nullptr, 0,
               relu_target(pl.l1dw, net.ltd1.bdw)));
    TRY(bn_bwd_x(pl.l1dw, net.ltd1.bdw, Bw(pl.l1dw.ga), 32, true, dz_buf(pl.l1dw), d));
    // the fused pass never forms conv0's dz, which the input gradient needs
    const bool want_dx = r.dx != nullptr;
    if (!want_dx && ltd_fused_enabled() && ltd_c0_bwd_ok(dt, r.x_dtype, pl.W, r.x)) {
      // (LTD.dsconv1.dw's weight gradient runs beside the fused pass at the side stream's low
      // priority; a normal-priority stream for it alone measured r05 5.888 vs 5.823 ms per step)
      TRY(dw_bwd(net.ltd1.dw, 32, d, act(pl.c0), pl.H1, pl.W1, pl.H2, pl.W2, 2, nullptr));
      TRY(ltd1_c0_bwd(d));
      return flush_side();
    }
    TRY(dw_bwd(net.ltd1.dw, 32, d, act(pl.c0), pl.H1, pl.W1, pl.H2, pl.W2, 2, Bw(pl.c0.ga),
               relu_target(pl.c0, net.b0)));
    TRY(flush_side());
    TRY(bn_bwd_x(pl.c0, net.b0, Bw(pl.c0.ga), 32, true, dz_buf(pl.c0), d, !want_dx));
    if (want_dx) {  // d is conv0's materialised dz
      g_prof_tag = "learning_to_downsample.conv (input gradient)";
      Conv0DgradArgs c{};
      c.dz = d.p; c.w = P(net.c0.w);
      c.N = pl.N; c.H = pl.H; c.W = pl.W; c.Ho = pl.H1; c.Wo = pl.W1;
      c.dx = r.dx; c.dx_dtype = r.dx_dtype;
      TRY(conv0_dgrad(c, dt, r.st));
    }
    Conv0WgradArgs c{};
    c.x = r.x; c.x_bf16 = r.x_dtype;
    c.N = pl.N; c.H = pl.H; c.W = pl.W; c.Ho = pl.H1; c.Wo = pl.W1;
    const int S = conv0_wgrad_parts(pl.N, pl.H1, pl.W1, 8);
    c.dz = d.p; c.zz = d.z; c.tab = d.tab; c.slab = slab_alloc((size_t)S * 864);
    c.rows_per_block = 8;
    if (!c.slab) return slab_oom();
    const int dtc = dt;
    TRY(side_launch([c, dtc](hipStream_t s) { return conv0_wgrad(c, dtc, s); }));
    TRY(defer_reduce(c.slab, S, 864, G(net.c0.w), 0));
    return flush_side();
  }
};

}  // namespace

// ================================ hipGraph replay =============================================
// A whole forward (~100 launches) or backward stage (~100-200 launches) is captured once into a
// hipGraph on an internal stream and replayed with one hipGraphLaunch while its arguments (all
// pointers and scalars; the dropout seed lives in device memory, written before each replay) are
// unchanged.  The caller's stream is chained in and out with events, so ordering with the
// caller's other work (and RCCL on other streams) is preserved.  Enabled with FSCNN_GRAPHS=1;
// bypassed while the launch profiler is active or when the caller's stream is being captured.
struct GraphCache {
  std::mutex mu;
  int dev = -1;
  hipStream_t gs = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  struct Entry {
    std::vector<uint64_t> key;
    hipGraphExec_t exec;
  };
  std::vector<Entry> entries;  // least recently used first
  ~GraphCache() {
    for (auto& e : entries) (void)hipGraphExecDestroy(e.exec);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    if (gs) (void)hipStreamDestroy(gs);
  }
};

std::shared_ptr<GraphCache> make_graph_cache() { return std::make_shared<GraphCache>(); }


namespace {

// Opt-in (FSCNN_GRAPHS=1): measured on MI355X / ROCm 7.2, replaying the captured chains ran
// slower than direct stream launches (9.46 vs 8.94 ms per cfg3 step) while the host enqueue
// time (2.0 vs 3.6 ms) was never the bottleneck.
bool graphs_enabled() {
  static const bool on = [] {
    const char* e = getenv("FSCNN_GRAPHS");
    return e && e[0] == '1';
  }();
  return on;
}

uint64_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

std::vector<uint64_t> run_key(int kind, int s0, int s1, const RunArgs& r) {
  auto P = [](const void* p) { return (uint64_t)(uintptr_t)p; };
  return {(uint64_t)kind, (uint64_t)s0, (uint64_t)s1, P(r.x), (uint64_t)r.x_dtype, P(r.out),
          (uint64_t)r.out_dtype, P(r.aux_out), P(r.labels), (uint64_t)r.label_u8, P(r.P), P(r.R), P(r.NBT), P(r.G), P(r.ws),
          P(r.bws), P(r.dout), P(r.daux), fbits(r.dropout_p), fbits(r.momentum), P(r.target),
          (uint64_t)r.ignore_index, P(r.loss2), P(r.gloss), P(r.dx), (uint64_t)r.dx_dtype};
}

template <typename F>
int run_graphed(const Plan& pl, std::vector<uint64_t> key, hipStream_t st, F&& body) {
  if (!graphs_enabled() || g_prof_kind != PK_NONE || !pl.graphs) return body(st);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return body(st);
  }
  GraphCache& gc = *pl.graphs;
  std::lock_guard<std::mutex> lock(gc.mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return body(st);
  if (!gc.gs) {
    if (hipStreamCreateWithFlags(&gc.gs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&gc.ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&gc.ev_out, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      return body(st);
    }
    gc.dev = dev;
  } else if (dev != gc.dev) {
    return body(st);
  }
  hipGraphExec_t exec = nullptr;
  for (size_t i = 0; i < gc.entries.size(); ++i) {
    if (gc.entries[i].key == key) {
      GraphCache::Entry e = gc.entries[i];
      gc.entries.erase(gc.entries.begin() + i);
      gc.entries.push_back(e);
      exec = e.exec;
      break;
    }
  }
  // order: caller's prior work -> graph stream
  if (hipEventRecord(gc.ev_in, st) != hipSuccess || hipStreamWaitEvent(gc.gs, gc.ev_in, 0) != hipSuccess) {
    set_error("graph: event chaining failed");
    return E_HIP;
  }
  if (!exec) {
    if (hipStreamBeginCapture(gc.gs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
      (void)hipGetLastError();
      return body(st);
    }
    const int rc = body(gc.gs);
    hipGraph_t g = nullptr;
    const hipError_t e1 = hipStreamEndCapture(gc.gs, &g);
    hipError_t e2 = hipErrorUnknown;
    if (!rc && e1 == hipSuccess && g) e2 = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (rc) return rc;
    if (e1 != hipSuccess || e2 != hipSuccess) {  // capture unsupported: run directly
      (void)hipGetLastError();
      return body(st);
    }
    gc.entries.push_back({std::move(key), exec});
    if (gc.entries.size() > 16) {
      (void)hipGraphExecDestroy(gc.entries.front().exec);
      gc.entries.erase(gc.entries.begin());
    }
  }
  if (hipGraphLaunch(exec, gc.gs) != hipSuccess || hipEventRecord(gc.ev_out, gc.gs) != hipSuccess ||
      hipStreamWaitEvent(st, gc.ev_out, 0) != hipSuccess) {
    set_error("graph: launch failed: %s", hipGetErrorString(hipGetLastError()));
    return E_HIP;
  }
  return OK;
}

}  // namespace

int net_forward_impl(const Plan& pl, const RunArgs& r);
int net_forward(const Plan& pl, const RunArgs& r) {
  const double t0 = g_host_prof ? host_now_us() : 0.0;
  const int rc = net_forward_impl(pl, r);
  if (g_host_prof) host_prof_add(3, host_now_us() - t0);
  return rc;
}
int net_forward_impl(const Plan& pl, const RunArgs& r) {
  if (r.x_dtype < DT_F32 || r.x_dtype > DT_F16 || r.out_dtype < DT_F32 || r.out_dtype > DT_F16) {
    set_error("fscnn_forward: input / output dtype codes must be 0 (fp32), 1 (bf16) or 2 (fp16)");
    return E_INVALID;
  }
  if (pl.net->aux && r.target) {
    set_error("forward_loss: the fused loss head covers the main output only (aux net)");
    return E_UNSUPPORTED;
  }
  if (pl.net->aux && !r.aux_out && !r.labels) {
    set_error("fscnn_forward: this net has the aux head; use fscnn_forward_aux");
    return E_INVALID;
  }
  if (r.dx_dtype < DT_F32 || r.dx_dtype > DT_F16) {
    set_error("input gradient dtype code must be 0 (fp32), 1 (bf16) or 2 (fp16)");
    return E_INVALID;
  }
  if (pl.train == 1 && r.dropout_p > 0.f && graphs_enabled())  // read by the dropout kernels
    TRY(set_u64(reinterpret_cast<uint64_t*>((char*)r.ws + pl.seed_slot), r.seed, r.st));
  return run_graphed(pl, run_key(0, 0, 0, r), r.st, [&](hipStream_t st) -> int {
    RunArgs rr = r;
    rr.st = st;
    if (pl.train == 2) rr.dropout_p = 0.f;  // differentiable inference: Dropout is the identity
    Exec ex(pl, rr);
    ex.use_side();
    return ex.forward();
  });
}

// stages: 0 = head (upsample, classifier, FFM, PPM), 1 = bottleneck3, 2 = bottleneck2,
//         3 = bottleneck1 + LearningToDownsample
int net_backward_impl(const Plan& pl, const RunArgs& r, int stage_from, int stage_to);
int net_backward(const Plan& pl, const RunArgs& r, int stage_from, int stage_to) {
  const double t0 = g_host_prof ? host_now_us() : 0.0;
  const int rc = net_backward_impl(pl, r, stage_from, stage_to);
  if (g_host_prof) host_prof_add(3, host_now_us() - t0);
  return rc;
}
int net_backward_impl(const Plan& pl, const RunArgs& r, int stage_from, int stage_to) {
  if (!pl.train) {
    set_error("net_backward: the plan was built for inference (train=0)");
    return E_INVALID;
  }
  if (pl.net->aux && !r.daux) {
    set_error("fscnn_backward: this net has the aux head; use fscnn_backward_aux");
    return E_INVALID;
  }
  for (int s = stage_from; s <= stage_to; ++s)
    if (s < 0 || s > 3) {
      set_error("net_backward: bad stage %d", s);
      return E_INVALID;
    }
  if (r.dx_dtype < DT_F32 || r.dx_dtype > DT_F16) {
    set_error("input gradient dtype code must be 0 (fp32), 1 (bf16) or 2 (fp16)");
    return E_INVALID;
  }
  if (r.gloss && pl.train != 1) {
    // the fused loss head's gradient exists only after fscnn_forward_loss, which needs a
    // training plan (train = 1): an eval-autograd plan (train = 2) never wrote it
    set_error("net_backward: grad_loss / loss2 need a training plan (train=1), got train=%d",
              pl.train);
    return E_INVALID;
  }
  return run_graphed(pl, run_key(1, stage_from, stage_to, r), r.st, [&](hipStream_t st) -> int {
    RunArgs rr = r;
    rr.st = st;
    if (pl.train == 2) rr.dropout_p = 0.f;
    Exec ex(pl, rr);
    ex.use_side();
    for (int s = stage_from; s <= stage_to; ++s) {
      switch (s) {
        case 0: TRY(ex.backward_head()); break;
        case 1: for (int i = 8; i >= 6; --i) TRY(ex.backward_block(i)); break;
        case 2: for (int i = 5; i >= 3; --i) TRY(ex.backward_block(i)); break;
        default:
          for (int i = 2; i >= 0; --i) TRY(ex.backward_block(i));
          TRY(ex.backward_ltd());
          break;
      }
      // the stage's gradient bucket is complete after its reduction; a call covering several
      // stages (no per-stage consumer between them: fast_scnn.py without a grad_stage_hook)
      // reduces every stage's slabs once at its end, so the main stream never waits for the
      // side stream's weight gradients mid-step (the slab arena holds the whole step's slabs)
      if (s == stage_to) TRY(ex.flush_reduce());
    }
    return ex.join();  // the caller's stream sees every gradient
  });
}

}  // namespace fscnn
