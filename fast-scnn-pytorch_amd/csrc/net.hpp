// Native executor of the Fast-SCNN hot path: layer table (state_dict schema of
// models/fast_scnn.py), workspace planning and the forward / backward launch sequences.
// It never allocates device memory: the caller passes the parameter / buffer / gradient arenas
// and workspaces (see include/fastscnn.h).
#pragma once
#include <atomic>
#include <string>
#include <memory>
#include <vector>

#include "kernels.hpp"

namespace fscnn {

struct TSpec {
  std::string name;
  std::vector<int> shape;
  long long off;    // element offset in its arena
  long long numel;
};

struct ConvL {
  long long w = -1, b = -1;  // offsets into P (floats), -1 = none
  int cin = 0, cout = 0, k = 1, groups = 1;
  // dense convs: W^T [cin*k*k][ldt] (zero-padded to ldt = cout rounded up to 8) in the compute
  // dtype at element offset wt of the plan's transposed-weight arena (the dgrad's B operand)
  long long wt = -1;
  int ldt = 0;
};
struct BnL {
  long long g = -1, b = -1;   // P offsets
  long long rm = -1, rv = -1; // R offsets
  int nbt = -1;               // index into the num_batches_tracked arena
  int C = 0;
  int id = -1;                // BN ordinal
};
struct DsL { ConvL dw; BnL bdw; ConvL pw; BnL bpw; };
struct LbL { ConvL e; BnL be; ConvL d; BnL bd; ConvL p; BnL bp; int cin, cout, stride; };

struct Net {
  int num_classes = 0, aux = 0;
  std::vector<TSpec> params;   // P arena (fp32), named_parameters() order
  std::vector<TSpec> buffers;  // R arena (fp32 running_mean/var) + nbt entries (off = index)
  long long p_total = 0, r_total = 0;
  int n_bn = 0;
  ConvL c0; BnL b0;
  DsL ltd1, ltd2, cls1, cls2;
  LbL lb[9];
  ConvL ppm_c[4]; BnL ppm_b[4];
  ConvL ppm_o; BnL ppm_ob;
  ConvL ffm_dw; BnL ffm_bdw;
  ConvL ffm_low; BnL ffm_blow;
  ConvL ffm_high; BnL ffm_bhigh;
  ConvL cls_out;
  ConvL aux0; BnL aux1; ConvL aux4;
  long long stage_p_begin[4];  // P offset where each backward stage's parameters start
  long long wt_total = 0;      // elements of the transposed-weight arena
};

int net_build(int num_classes, int aux, Net& net);

// A conv(+BN) output in the workspace.
struct Unit {
  long long M = 0;
  int C = 0, ld = 0;
  size_t z = 0, a = 0;      // raw conv output / activation (same in eval)
  size_t part = 0;          // BN partial records
  int nparts = 0;           // record slots (gemm_parts(M) for GEMM producers: an upper bound)
  // the dgrad producing this unit's dy (GEMM or depthwise) also reduces and finishes its BN
  // backward (set when that dgrad is issued; fixed per plan): the BN backward then only applies
  // (an atomic: concurrent backward calls of DataParallel replicas set it; always to true)
  struct Flag {
    std::atomic<bool> v{false};
    Flag() = default;
    Flag(const Flag& o) : v(o.v.load(std::memory_order_relaxed)) {}
    Flag& operator=(const Flag& o) {
      v.store(o.v.load(std::memory_order_relaxed), std::memory_order_relaxed);
      return *this;
    }
    bool get() const { return v.load(std::memory_order_relaxed); }
    void set() const { const_cast<std::atomic<bool>&>(v).store(true, std::memory_order_relaxed); }
  };
  Flag bdone;
  size_t mean = 0, invstd = 0, scale = 0, shift = 0;  // fp32 [C]
  size_t ga = 0;            // backward: grad wrt a (bwd workspace)
  int ga_ld = 0;
  // train: the BN+ReLU output is never stored; every consumer (forward GEMM / depthwise and the
  // backward wgrads) applies relu(fmaf(z, scale, shift)) to z while staging its operand
  bool lazy = false;
  std::string name;         // reference module path (per-launch profile label)
  std::string block_name;   // label of a fused whole-block launch (inference bottlenecks)
};

struct GraphCache;
struct SideStream;

struct Plan {
  const Net* net = nullptr;
  int N = 0, H = 0, W = 0, dtype = DT_F32, train = 0;
  int H1, W1, H2, W2, H3, W3, H4, W4, H5, W5;
  int Cp = 0;   // padded class count (row stride of the low-res logits)
  size_t ws_bytes = 0, bws_bytes = 0;
  size_t slab_floats = 0;  // weight-gradient partial arena (every job of a step has its own slab)
  // forward units
  Unit c0, l1dw, l1pw, l2dw, l2pw;
  Unit lbe[9], lbd[9], lbp[9];
  Unit ppk[4], po;
  Unit fdw, flow, fhigh;
  Unit c1dw, c1pw, c2dw, c2pw;
  Unit aux0;
  size_t concat = 0, pooled = 0, feats_a = 0, feats_z = 0, up_low = 0, f = 0, drop = 0,
         logits = 0, aux_drop = 0, aux_logits = 0, aux_col = 0, pbf = 0, fold_tmp = 0;
  size_t wt = 0;                    // transposed weights (train plans), net.wt_total elements
  size_t lb_we3[9] = {}, lb_wp3[9] = {};  // fp32 inference: split planes of fused bottlenecks
  size_t g_raw = 0, head_part = 0;  // fused loss head (train plans)
  size_t tgt8 = 0;                    // the loss head's int8 targets (train plans)
  size_t seed_slot = 0;             // dropout seed (device copy read by the dropout kernels)
  size_t fcnt = 0, bcnt = 0;        // BN arrival counters (ws), BN_COUNTERS each
  size_t tsum = 0;                  // fp64 team sums of the in-kernel BN finishes (ws)
  size_t tsum2 = 0;                 // ... of the forward's side-stream producer (FFM high-res)
  // backward workspace
  size_t g_logits = 0, t_up = 0, g_drop = 0, g_f = 0, g_up = 0, t_up2 = 0, g_concat = 0,
         g_feats = 0, g_pooled = 0, dz = 0, slab = 0, bnpart = 0, coef = 0, cspart = 0,
         g_aux = 0, g_auxlog = 0, aux_dcol = 0, xtab = 0, c0sum = 0;
  size_t dz_bytes = 0;             // the dz arena (one slot per unit, Exec::dz_buf)
  size_t bnpart_floats = 0;        // capacity of the BN-backward record arena (bnpart)
  // named buffers for debugging / stage-level parity: name -> (offset, rows, cols, ld, in_bws)
  struct Named { std::string name; size_t off; long long rows; int cols, ld, bws; };
  std::vector<Named> named;
  // captured hipGraphs of whole forward / backward-stage calls, keyed by their arguments
  std::shared_ptr<GraphCache> graphs;
  // second stream for the weight-gradient launches of the backward (created on first use)
  std::shared_ptr<SideStream> side;
};

int plan_build(const Net& net, int N, int H, int W, int dtype, int train, Plan& pl);
bool ir_block_shape(const Net& net, const Plan& pl, int i, IrArgs& b);
std::shared_ptr<GraphCache> make_graph_cache();
std::shared_ptr<SideStream> make_side_stream();

struct RunArgs {
  const void* x; int x_dtype;     // NCHW input image
  void* out; int out_dtype;       // NCHW logits [N][C][H][W]
  void* aux_out;                  // NCHW aux logits or null
  const float* P;                 // parameter arena
  float* R;                       // running stats arena
  long long* NBT;                 // num_batches_tracked arena
  float* G;                       // gradient arena (backward)
  void* ws;                       // forward workspace (persists until backward)
  void* bws;                      // backward workspace
  const void* dout;               // grad wrt out (backward)
  const void* daux;               // grad wrt aux_out (backward) or null
  unsigned long long seed;        // dropout seed
  float dropout_p;
  float momentum;
  hipStream_t st;
  // fused loss head: forward with target != null computes the CE loss into loss2[0..1]
  // (mean, count) instead of writing full-resolution logits; backward with gloss != null
  // starts from d(loss) instead of d(logits).
  const long long* target = nullptr;
  long long ignore_index = -1;
  float* loss2 = nullptr;
  const float* gloss = nullptr;
  // eval prediction: forward with labels != null writes argmax(upsampled logits) instead of out
  void* labels = nullptr;
  int label_u8 = 0;
  // backward: gradient of the input image, NCHW [N][3][H][W] in dx_dtype (autograd of x through
  // conv0, models/fast_scnn.py:153), or null
  void* dx = nullptr;
  int dx_dtype = 0;
};

int net_forward(const Plan& pl, const RunArgs& r);
int net_backward(const Plan& pl, const RunArgs& r, int stage_from, int stage_to);

}  // namespace fscnn
