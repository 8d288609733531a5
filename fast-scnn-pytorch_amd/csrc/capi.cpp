// extern "C" boundary of libfastscnn_hip.so (declared in include/fastscnn.h).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "../../include/fastscnn.h"
#include "net.hpp"

namespace fscnn {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return E_HIP;
  }
  return OK;
}

// ---- launch profiler --------------------------------------------------------------------
unsigned long long* g_stamps = nullptr;
int g_prof_kind = PK_NONE;
thread_local const char* g_prof_tag = "";
namespace {
struct ProfState {
  std::vector<hipEvent_t> ev;  // pairs
  std::vector<int> kind;       // per recorded launch
  std::vector<std::string> tag;
  std::vector<double> lbytes, lflops;
  size_t used = 0;
  double bytes = 0, flops = 0;
  long long launches = 0;
  bool overflow = false;
  bool armed = false, taken = false;  // the open scope's events (prof_start / prof_take_ext)
  hipStream_t arm_st = nullptr;
} g_prof;
}  // namespace

bool g_host_prof = [] {
  const char* e = getenv("FSCNN_HOST_PROF");
  return e && e[0] == '1';
}();
namespace {
struct HostProf {
  double us[4] = {0, 0, 0, 0};
  long long n[4] = {0, 0, 0, 0};
  ~HostProf() {
    if (!g_host_prof) return;
    static const char* names[4] = {"kernel launches", "side-stream forks", "side-stream joins",
                                   "C entry points (total)"};
    for (int i = 0; i < 4; ++i)
      fprintf(stderr, "FSCNN_HOST_PROF %-24s %10lld calls %12.1f us  (%.2f us each)\n", names[i],
              n[i], us[i], n[i] ? us[i] / n[i] : 0.0);
  }
} g_hostp;
}  // namespace
double host_now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
void host_prof_add(int what, double us) {
  g_hostp.us[what] += us;
  g_hostp.n[what]++;
}

// A scope arms its event pair for the first prof_launch inside it (kernel-bound events); a scope
// whose launch does not take them (none issued) falls back to marker events around the scope.
void prof_start(hipStream_t st) {
  if (g_prof.used + 2 > g_prof.ev.size()) { g_prof.overflow = true; return; }
  g_prof.armed = true;
  g_prof.taken = false;
  g_prof.arm_st = st;
}
bool prof_take_ext(hipEvent_t& e0, hipEvent_t& e1) {
  if (!g_prof.armed || g_prof.taken) return false;
  e0 = g_prof.ev[g_prof.used];
  e1 = g_prof.ev[g_prof.used + 1];
  g_prof.taken = true;
  return true;
}
void prof_stop(hipStream_t st, int kind, double bytes, double flops) {
  if (g_prof.used + 2 > g_prof.ev.size()) return;
  const bool taken = g_prof.armed && g_prof.taken;
  g_prof.armed = false;
  if (!taken) {  // no kernel launched in the scope: a zero-length marker pair
    (void)hipEventRecord(g_prof.ev[g_prof.used], st);
    (void)hipEventRecord(g_prof.ev[g_prof.used + 1], st);
  }
  g_prof.used += 2;
  g_prof.kind.push_back(kind);
  g_prof.tag.emplace_back(g_prof_tag ? g_prof_tag : "");
  g_prof.lbytes.push_back(bytes);
  g_prof.lflops.push_back(flops);
  g_prof.bytes += bytes;
  g_prof.flops += flops;
  g_prof.launches++;
}

}  // namespace fscnn

using namespace fscnn;

extern "C" int fscnn_prof_begin(int kind, int max_launches) {
  if ((kind <= PK_NONE || kind >= PK_COUNT) && kind != PK_ALL) {
    set_error("fscnn_prof_begin: bad kind %d", kind);
    return E_INVALID;
  }
  if (max_launches <= 0) {
    set_error("fscnn_prof_begin: bad kind %d", kind);
    return E_INVALID;
  }
  size_t need = (size_t)max_launches * 2;
  while (g_prof.ev.size() < need) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) { set_error("hipEventCreate failed"); return E_HIP; }
    g_prof.ev.push_back(e);
  }
  g_prof.used = 0; g_prof.bytes = 0; g_prof.flops = 0; g_prof.launches = 0;
  g_prof.kind.clear(); g_prof.tag.clear(); g_prof.lbytes.clear(); g_prof.lflops.clear();
  g_prof.overflow = false;
  g_prof_kind = kind;
  return OK;
}

// Synchronises on the recorded events; returns summed kernel time (ms), launches and the
// algorithmic bytes / flops of those launches.
extern "C" int fscnn_prof_end(double* total_ms, long long* launches, double* bytes, double* flops) {
  g_prof_kind = PK_NONE;
  double tot = 0;
  for (size_t i = 0; i + 1 < g_prof.used; i += 2) {
    float ms = 0;
    if (hipEventSynchronize(g_prof.ev[i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, g_prof.ev[i], g_prof.ev[i + 1]) != hipSuccess) {
      set_error("fscnn_prof_end: event query failed");
      return E_HIP;
    }
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = g_prof.launches;
  if (bytes) *bytes = g_prof.bytes;
  if (flops) *flops = g_prof.flops;
  if (g_prof.overflow) { set_error("fscnn_prof_end: event pool overflow"); return E_INVALID; }
  return OK;
}

// One recorded launch of the last fscnn_prof_begin / _end window (after _end): its kind, kernel
// time, algorithmic bytes / flops and the executor's layer label.
extern "C" int fscnn_prof_launch(long long i, int* kind, float* ms, double* bytes, double* flops,
                                 const char** tag) {
  if (i < 0 || (size_t)i >= g_prof.kind.size()) {
    set_error("fscnn_prof_launch: index %lld out of range (%zu recorded)", i, g_prof.kind.size());
    return E_INVALID;
  }
  float t = 0;
  if (hipEventElapsedTime(&t, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]) != hipSuccess) {
    set_error("fscnn_prof_launch: event query failed");
    return E_HIP;
  }
  if (kind) *kind = g_prof.kind[i];
  if (ms) *ms = t;
  if (bytes) *bytes = g_prof.lbytes[i];
  if (flops) *flops = g_prof.lflops[i];
  if (tag) *tag = g_prof.tag[i].c_str();  // valid until the next fscnn_prof_begin
  return OK;
}

// Phase stamps of the next launches of the instrumented kernels (pointwise GEMMs, depthwise
// forward / stride-1 dgrad): launch i writes buf + i * STAMP_STRIDE (max_launches regions; null:
// off).  Debug / tools only (process-global, single thread).
namespace fscnn {
static int g_stamp_max = 0, g_stamp_used = 0;
static std::vector<std::string> g_stamp_tags;
unsigned long long* stamp_region() {
  if (!g_stamps || g_stamp_used >= g_stamp_max) return nullptr;
  g_stamp_tags.emplace_back(g_prof_tag ? g_prof_tag : "");
  return g_stamps + (size_t)(g_stamp_used++) * STAMP_STRIDE;
}
}  // namespace fscnn
extern "C" int fscnn_debug_stamps(void* buf, int max_launches) {
  g_stamps = reinterpret_cast<unsigned long long*>(buf);
  g_stamp_max = buf ? max_launches : 0;
  g_stamp_used = 0;
  g_stamp_tags.clear();
  return OK;
}
extern "C" int fscnn_debug_stamp_count(void) { return g_stamp_used; }
extern "C" const char* fscnn_debug_stamp_tag(int i) {
  return (i >= 0 && i < (int)g_stamp_tags.size()) ? g_stamp_tags[i].c_str() : "";
}

extern "C" const char* fscnn_prof_kind_name(int kind) {
  static const char* names[PK_COUNT] = {"none", "conv0_fwd", "dw_fwd", "dw_dgrad", "dw_wgrad",
                                        "gemm_nt", "gemm_tn", "bn_apply", "bn_bwd", "upsample",
                                        "upsample_bwd", "cross_entropy", "conv0_wgrad",
                                        "bn_bwd_reduce", "bn_finalize", "ppm_branches",
                                        "ir_block", "ltd_stem", "dsconv"};
  return (kind >= 0 && kind < PK_COUNT) ? names[kind] : "?";
}

struct fscnn_net {
  Net net;
};
struct fscnn_plan {
  Plan plan;
};

#define GUARD(expr)                                   \
  try {                                               \
    return (expr);                                    \
  } catch (const std::exception& e) {                 \
    set_error("exception: %s", e.what());             \
    return E_INVALID;                                 \
  }

static hipStream_t S(void* s) { return (hipStream_t)s; }

extern "C" {

const char* fscnn_version(void) { return "fastscnn-hip 0.1 (gfx950)"; }
const char* fscnn_last_error(void) { return last_error(); }

int fscnn_net_create(int num_classes, int aux, fscnn_net** out) {
  if (!out) { set_error("fscnn_net_create: null out"); return E_INVALID; }
  fscnn_net* n = new (std::nothrow) fscnn_net();
  if (!n) { set_error("fscnn_net_create: out of host memory"); return E_INVALID; }
  int rc = net_build(num_classes, aux, n->net);
  if (rc) { delete n; return rc; }
  *out = n;
  return OK;
}
void fscnn_net_destroy(fscnn_net* net) { delete net; }

int fscnn_net_param_count(const fscnn_net* net, int* count, long long* total) {
  if (!net) { set_error("null net"); return E_INVALID; }
  if (count) *count = (int)net->net.params.size();
  if (total) *total = net->net.p_total;
  return OK;
}
int fscnn_net_param_info(const fscnn_net* net, int i, const char** name, long long* offset,
                         long long* numel) {
  if (!net || i < 0 || i >= (int)net->net.params.size()) { set_error("bad param index %d", i); return E_INVALID; }
  const TSpec& t = net->net.params[i];
  if (name) *name = t.name.c_str();
  if (offset) *offset = t.off;
  if (numel) *numel = t.numel;
  return OK;
}
int fscnn_net_buffer_count(const fscnn_net* net, int* count, long long* total, int* num_bn) {
  if (!net) { set_error("null net"); return E_INVALID; }
  if (count) *count = (int)net->net.buffers.size();
  if (total) *total = net->net.r_total;
  if (num_bn) *num_bn = net->net.n_bn;
  return OK;
}
int fscnn_net_buffer_info(const fscnn_net* net, int i, const char** name, long long* offset,
                          long long* numel) {
  if (!net || i < 0 || i >= (int)net->net.buffers.size()) { set_error("bad buffer index %d", i); return E_INVALID; }
  const TSpec& t = net->net.buffers[i];
  if (name) *name = t.name.c_str();
  if (offset) *offset = t.off;
  if (numel) *numel = t.numel;
  return OK;
}
int fscnn_net_stage_range(const fscnn_net* net, int stage, long long* begin, long long* end) {
  if (!net || stage < 0 || stage > 3) { set_error("bad stage %d", stage); return E_INVALID; }
  const Net& n = net->net;
  *begin = n.stage_p_begin[stage];
  *end = stage == 0 ? n.p_total : n.stage_p_begin[stage - 1];
  return OK;
}

int fscnn_plan_create(const fscnn_net* net, int N, int H, int W, int dtype, int train,
                      fscnn_plan** out) {
  if (!net || !out) { set_error("fscnn_plan_create: null argument"); return E_INVALID; }
  fscnn_plan* p = new (std::nothrow) fscnn_plan();
  if (!p) { set_error("out of host memory"); return E_INVALID; }
  int rc = plan_build(net->net, N, H, W, dtype, train, p->plan);
  if (rc) { delete p; return rc; }
  p->plan.graphs = make_graph_cache();
  p->plan.side = make_side_stream();
  *out = p;
  return OK;
}
void fscnn_plan_destroy(fscnn_plan* plan) { delete plan; }
int fscnn_plan_workspace(const fscnn_plan* plan, long long* fwd, long long* bwd) {
  if (!plan) { set_error("null plan"); return E_INVALID; }
  if (fwd) *fwd = (long long)plan->plan.ws_bytes;
  if (bwd) *bwd = (long long)plan->plan.bws_bytes;
  return OK;
}
int fscnn_plan_shapes(const fscnn_plan* plan, int* d) {
  if (!plan || !d) { set_error("null plan"); return E_INVALID; }
  const Plan& p = plan->plan;
  int v[10] = {p.H1, p.W1, p.H2, p.W2, p.H3, p.W3, p.H4, p.W4, p.H5, p.W5};
  memcpy(d, v, sizeof v);
  return OK;
}

int fscnn_forward(const fscnn_plan* plan, const void* x, int x_dtype, void* out, int out_dtype,
                  const float* params, float* running, long long* nbt, void* ws,
                  unsigned long long seed, float dropout_p, float momentum, void* stream) {
  if (!plan || !x || !out || !params || !running || !ws) {
    set_error("fscnn_forward: null argument");
    return E_INVALID;
  }
  RunArgs r{};
  r.x = x; r.x_dtype = x_dtype; r.out = out; r.out_dtype = out_dtype;
  r.P = params; r.R = running; r.NBT = nbt; r.ws = ws;
  r.seed = seed; r.dropout_p = dropout_p; r.momentum = momentum; r.st = S(stream);
  GUARD(net_forward(plan->plan, r));
}

int fscnn_backward(const fscnn_plan* plan, const void* dout, const void* x, int x_dtype,
                   const float* params, float* grads, void* ws, void* bws,
                   unsigned long long seed, float dropout_p, int stage_from, int stage_to,
                   void* stream) {
  if (!plan || !dout || !x || !params || !grads || !ws || !bws) {
    set_error("fscnn_backward: null argument");
    return E_INVALID;
  }
  RunArgs r{};
  r.dout = dout; r.x = x; r.x_dtype = x_dtype; r.P = params; r.G = grads; r.ws = ws; r.bws = bws;
  r.seed = seed; r.dropout_p = dropout_p; r.st = S(stream);
  GUARD(net_backward(plan->plan, r, stage_from, stage_to));
}

int fscnn_forward_aux(const fscnn_plan* plan, const void* x, int x_dtype, void* out, void* aux_out,
                      int out_dtype, const float* params, float* running, long long* nbt,
                      void* ws, unsigned long long seed, float dropout_p, float momentum,
                      void* stream) {
  if (!plan || !x || !out || !aux_out || !params || !running || !ws) {
    set_error("fscnn_forward_aux: null argument");
    return E_INVALID;
  }
  RunArgs r{};
  r.x = x; r.x_dtype = x_dtype; r.out = out; r.aux_out = aux_out; r.out_dtype = out_dtype;
  r.P = params; r.R = running; r.NBT = nbt; r.ws = ws;
  r.seed = seed; r.dropout_p = dropout_p; r.momentum = momentum; r.st = S(stream);
  GUARD(net_forward(plan->plan, r));
}

int fscnn_backward_aux(const fscnn_plan* plan, const void* dout, const void* daux, const void* x,
                       int x_dtype, const float* params, float* grads, void* ws, void* bws,
                       unsigned long long seed, float dropout_p, int stage_from, int stage_to,
                       void* stream) {
  if (!plan || !dout || !daux || !x || !params || !grads || !ws || !bws) {
    set_error("fscnn_backward_aux: null argument");
    return E_INVALID;
  }
  RunArgs r{};
  r.dout = dout; r.daux = daux; r.x = x; r.x_dtype = x_dtype; r.P = params; r.G = grads;
  r.ws = ws; r.bws = bws; r.seed = seed; r.dropout_p = dropout_p; r.st = S(stream);
  GUARD(net_backward(plan->plan, r, stage_from, stage_to));
}

int fscnn_predict(const fscnn_plan* plan, const void* x, int x_dtype, void* labels,
                  int label_dtype, const float* params, float* running, long long* nbt, void* ws,
                  void* stream) {
  if (!plan || !x || !labels || !params || !running || !ws) {
    set_error("fscnn_predict: null argument");
    return E_INVALID;
  }
  if (plan->plan.train) {
    set_error("fscnn_predict: needs an inference plan (train=0)");
    return E_INVALID;
  }
  if (label_dtype != 0 && label_dtype != 1) {
    set_error("fscnn_predict: label_dtype %d (0 int64, 1 uint8)", label_dtype);
    return E_INVALID;
  }
  RunArgs r{};
  r.x = x; r.x_dtype = x_dtype; r.out = nullptr; r.out_dtype = plan->plan.dtype;
  r.labels = labels; r.label_u8 = label_dtype;
  r.P = params; r.R = running; r.NBT = nbt; r.ws = ws; r.momentum = 0.1f; r.st = S(stream);
  GUARD(net_forward(plan->plan, r));
}

int fscnn_seg_metric(const void* pred, int pred_dtype, const long long* target, long long n,
                     int nclass, long long* counts, void* stream) {
  if ((!pred || !target || !counts) && n > 0) {
    set_error("fscnn_seg_metric: null argument");
    return E_INVALID;
  }
  if (pred_dtype != 0 && pred_dtype != 1) {
    set_error("fscnn_seg_metric: pred_dtype %d (0 int64, 1 uint8)", pred_dtype);
    return E_INVALID;
  }
  return seg_metric(pred, pred_dtype, target, n, nclass, counts, S(stream));
}

int fscnn_normalize_u8(const unsigned char* images, int N, int H, int W, const float* mean,
                       const float* std, void* out, int out_dtype, void* stream) {
  if (!images || !mean || !std || !out) {
    set_error("fscnn_normalize_u8: null argument");
    return E_INVALID;
  }
  if (out_dtype != DT_F32 && out_dtype != DT_BF16) {
    set_error("fscnn_normalize_u8: out_dtype %d", out_dtype);
    return E_INVALID;
  }
  return normalize_u8(images, N, H, W, mean, std, out, out_dtype, S(stream));
}

int fscnn_remap_labels(const unsigned char* labels, long long n, const long long* lut, int lut_size,
                       int offset, long long invalid, long long* out, void* stream) {
  if ((!labels || !out || !lut) && n > 0) {
    set_error("fscnn_remap_labels: null argument");
    return E_INVALID;
  }
  return remap_labels(labels, n, lut, lut_size, offset, invalid, out, S(stream));
}

int fscnn_ohem_prob(const void* logits, int dtype, const long long* target, int N, int C,
                    long long HW, long long ignore_index, float thresh, float* prob,
                    unsigned long long* counts, void* stream) {
  if (!logits || !target || !prob || !counts) {
    set_error("fscnn_ohem_prob: null argument");
    return E_INVALID;
  }
  CeArgs a{};
  a.N = N; a.C = C; a.HW = HW; a.logits = logits; a.target = target; a.ignore_index = ignore_index;
  return ohem_prob(a, thresh, prob, counts, dtype, S(stream));
}

int fscnn_ohem_threshold(const float* prob, long long n, const unsigned long long* counts,
                         long long min_kept, float thresh, unsigned* work, float* thr, void* stream) {
  if (!prob || !counts || !work || !thr) {
    set_error("fscnn_ohem_threshold: null argument");
    return E_INVALID;
  }
  return ohem_threshold_dev(prob, n, counts, min_kept, thresh, work, thr, S(stream));
}

int fscnn_kth_smallest(const float*, long long, long long, unsigned*, float*, void*) {
  set_error("fscnn_kth_smallest was removed in round 3: use fscnn_ohem_threshold (the whole OHEM "
            "threshold rule on the device, no host sync)");
  return E_UNSUPPORTED;
}

int fscnn_ce_weighted_fwd(const void* logits, int dtype, const long long* target, int N, int C,
                          long long HW, long long ignore_index, const float* weight,
                          const float* prob, const float* thr, float* part, float* out2,
                          void* stream) {
  if (prob && !thr) {
    set_error("fscnn_ce_weighted_fwd: prob without thr");
    return E_INVALID;
  }
  CeArgs a{};
  a.N = N; a.C = C; a.HW = HW; a.logits = logits; a.target = target;
  a.ignore_index = ignore_index; a.part = part; a.weight = weight; a.prob = prob; a.thr = thr;
  return ce_fwd(a, out2, dtype, S(stream));
}

int fscnn_ce_weighted_bwd(const void* logits, int dtype, const long long* target, int N, int C,
                          long long HW, long long ignore_index, const float* weight,
                          const float* prob, const float* thr, const float* grad_out,
                          const float* out2, void* dlogits, void* stream) {
  if (prob && !thr) {
    set_error("fscnn_ce_weighted_bwd: prob without thr");
    return E_INVALID;
  }
  CeArgs a{};
  a.N = N; a.C = C; a.HW = HW; a.logits = logits; a.target = target;
  a.ignore_index = ignore_index; a.dlogits = dlogits; a.weight = weight; a.prob = prob; a.thr = thr;
  return ce_bwd(a, grad_out, out2, dtype, S(stream));
}

int fscnn_dice_fwd(const void* logits, int dtype, const long long* target, int N, int C,
                   long long HW, float alpha, float gamma, int focal, float* part, double* stats,
                   void* stream) {
  if (!logits || !target || !part || !stats) {
    set_error("fscnn_dice_fwd: null argument");
    return E_INVALID;
  }
  return dice_loss_fwd(logits, dtype, target, N, C, HW, alpha, gamma, focal, part, stats, S(stream));
}

int fscnn_dice_bwd(const void* logits, int dtype, const long long* target, int N, int C,
                   long long HW, float alpha, float gamma, int focal, const double* stats,
                   const float* grad_out, float smooth, float dice_weight, float focal_weight,
                   void* dlogits, void* stream) {
  if (!logits || !target || !stats || !grad_out || !dlogits) {
    set_error("fscnn_dice_bwd: null argument");
    return E_INVALID;
  }
  return dice_loss_bwd(logits, dtype, target, N, C, HW, alpha, gamma, focal, stats, grad_out,
                       smooth, dice_weight, focal_weight, dlogits, S(stream));
}

int fscnn_forward_loss(const fscnn_plan* plan, const void* x, int x_dtype, const long long* target,
                       long long ignore_index, float* loss2, const float* params, float* running,
                       long long* nbt, void* ws, unsigned long long seed, float dropout_p,
                       float momentum, void* stream) {
  if (!plan || !x || !target || !loss2 || !params || !running || !ws) {
    set_error("fscnn_forward_loss: null argument");
    return E_INVALID;
  }
  RunArgs r{};
  r.x = x; r.x_dtype = x_dtype; r.out = nullptr; r.out_dtype = plan->plan.dtype;
  r.P = params; r.R = running; r.NBT = nbt; r.ws = ws;
  r.seed = seed; r.dropout_p = dropout_p; r.momentum = momentum; r.st = S(stream);
  r.target = target; r.ignore_index = ignore_index; r.loss2 = loss2;
  GUARD(net_forward(plan->plan, r));
}

int fscnn_backward_loss(const fscnn_plan* plan, const float* grad_loss, const float* loss2,
                        const void* x, int x_dtype, const float* params, float* grads, void* ws,
                        void* bws, unsigned long long seed, float dropout_p, int stage_from,
                        int stage_to, void* stream) {
  if (!plan || !grad_loss || !loss2 || !x || !params || !grads || !ws || !bws) {
    set_error("fscnn_backward_loss: null argument");
    return E_INVALID;
  }
  RunArgs r{};
  r.gloss = grad_loss; r.loss2 = const_cast<float*>(loss2);
  r.x = x; r.x_dtype = x_dtype; r.P = params; r.G = grads; r.ws = ws; r.bws = bws;
  r.seed = seed; r.dropout_p = dropout_p; r.st = S(stream);
  GUARD(net_backward(plan->plan, r, stage_from, stage_to));
}

int fscnn_backward_dx(const fscnn_plan* plan, const void* dout, const void* daux,
                      const float* grad_loss, const float* loss2, const void* x, int x_dtype,
                      void* dx, int dx_dtype, const float* params, float* grads, void* ws,
                      void* bws, unsigned long long seed, float dropout_p, int stage_from,
                      int stage_to, void* stream) {
  if (!plan || !x || !params || !grads || !ws || !bws || (!dout && !grad_loss) ||
      (dout && grad_loss) || (grad_loss && !loss2)) {
    set_error("fscnn_backward_dx: null argument (exactly one of dout / grad_loss + loss2)");
    return E_INVALID;
  }
  RunArgs r{};
  r.dout = dout; r.daux = daux; r.gloss = grad_loss; r.loss2 = const_cast<float*>(loss2);
  r.x = x; r.x_dtype = x_dtype; r.dx = dx; r.dx_dtype = dx_dtype;
  r.P = params; r.G = grads; r.ws = ws; r.bws = bws;
  r.seed = seed; r.dropout_p = dropout_p; r.st = S(stream);
  GUARD(net_backward(plan->plan, r, stage_from, stage_to));
}

long long fscnn_ce_parts(int N, long long HW) { return ce_parts(N, HW); }

int fscnn_ce_fwd(const void* logits, int dtype, const long long* target, int N, int C,
                 long long HW, long long ignore_index, float* part, float* out2, void* stream) {
  CeArgs a{};
  a.N = N; a.C = C; a.HW = HW; a.logits = logits; a.target = target;
  a.ignore_index = ignore_index; a.part = part;
  return ce_fwd(a, out2, dtype, S(stream));
}
int fscnn_ce_bwd(const void* logits, int dtype, const long long* target, int N, int C,
                 long long HW, long long ignore_index, const float* grad_out, const float* out2,
                 void* dlogits, void* stream) {
  CeArgs a{};
  a.N = N; a.C = C; a.HW = HW; a.logits = logits; a.target = target;
  a.ignore_index = ignore_index; a.dlogits = dlogits;
  return ce_bwd(a, grad_out, out2, dtype, S(stream));
}
int fscnn_sgd(float* p, const float* g, float* buf, long long n, float lr, float momentum,
              float dampening, float weight_decay, int nesterov, int first, float grad_scale,
              void* stream) {
  SgdArgs a{};
  a.n = n; a.p = p; a.g = g; a.buf = buf; a.lr = lr; a.momentum = momentum;
  a.dampening = dampening; a.weight_decay = weight_decay; a.nesterov = nesterov; a.first = first;
  a.grad_scale = grad_scale;
  return sgd(a, S(stream));
}

int fscnn_conv0_fwd(const void* x, int x_dtype, int N, int H, int W, const float* w,
                    const float* scale, const float* shift, int relu, void* y, int y_dtype,
                    void* stream) {
  Conv0Args a{};
  a.x = x; a.x_bf16 = x_dtype; a.N = N; a.H = H; a.W = W;
  a.Ho = (H - 3) / 2 + 1; a.Wo = (W - 3) / 2 + 1; a.w = w; a.scale = scale; a.shift = shift;
  a.relu = relu; a.y = y;
  return conv0_fwd(a, y_dtype, S(stream));
}

long long fscnn_conv0_wgrad_slab_floats(int N, int H, int W) {
  return (long long)conv0_wgrad_parts(N, (H - 3) / 2 + 1, (W - 3) / 2 + 1, 0) * 864;
}
int fscnn_conv0_wgrad(const void* x, int x_dtype, int N, int H, int W, const void* dz,
                      int dz_dtype, float* slab, float* dw, void* stream) {
  Conv0WgradArgs a{};
  a.x = x; a.x_bf16 = x_dtype; a.N = N; a.H = H; a.W = W;
  a.Ho = (H - 3) / 2 + 1; a.Wo = (W - 3) / 2 + 1; a.dz = dz; a.slab = slab;
  int rc = conv0_wgrad(a, dz_dtype, S(stream));
  if (rc) return rc;
  return reduce_slabs(slab, conv0_wgrad_parts(N, a.Ho, a.Wo, 0), 864, 864, dw, 0, S(stream));
}

int fscnn_dw3x3_fwd(const void* x, int dtype, int N, int H, int W, int C, int stride,
                    const float* w, const float* scale, const float* shift, int relu, void* y,
                    void* stream) {
  DwArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.stride = stride;
  a.Ho = (H - 1) / stride + 1; a.Wo = (W - 1) / stride + 1;
  a.x = x; a.w = w; a.scale = scale; a.shift = shift; a.relu = relu; a.y = y;
  return dw_fwd(a, dtype, S(stream));
}
int fscnn_dw3x3_dgrad(const void* dy, int dtype, int N, int H, int W, int C, int stride,
                      const float* w, void* dx, void* stream) {
  DwBwdArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.stride = stride;
  a.Ho = (H - 1) / stride + 1; a.Wo = (W - 1) / stride + 1;
  a.dy = dy; a.w = w; a.dx = dx;
  return dw_dgrad(a, dtype, S(stream));
}
long long fscnn_dw3x3_wgrad_slab_floats(int N, int H, int W, int C, int stride, int dtype) {
  int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  return (long long)dw_wgrad_parts(N, Ho, Wo, C, dtype, stride) * 9 * C;
}
int fscnn_dw3x3_wgrad(const void* x, const void* dy, int dtype, int N, int H, int W, int C,
                      int stride, float* slab, float* dw, void* stream) {
  DwBwdArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.stride = stride;
  a.Ho = (H - 1) / stride + 1; a.Wo = (W - 1) / stride + 1;
  a.x = x; a.dy = dy; a.slab = slab;
  int rc = dw_wgrad(a, dtype, S(stream));
  if (rc) return rc;
  return dw_wgrad_reduce(slab, dw_wgrad_parts(N, a.Ho, a.Wo, C, dtype, stride), C, dw, S(stream));
}

int fscnn_pw_gemm_stats_parts(int M, int N, int K, int lda, int ldc, int dtype) {
  GemmArgs a{};
  static float dummy;  // only the presence of the statistics pointer matters
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = K; a.ldc = ldc; a.part = &dummy;
  return gemm_nt_parts(a, dtype);
}
int fscnn_pw_gemm(int M, int N, int K, const void* A, int lda, const void* B, int ldb,
                  int b_trans, const float* scale, const float* shift, const void* R, int ldr,
                  int relu, void* C, int ldc, float* stats_part, int dtype, void* stream) {
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.b_trans = b_trans;
  a.scale = scale; a.shift = shift; a.R = R; a.ldr = ldr; a.relu = relu; a.C = C; a.ldc = ldc;
  a.part = stats_part;
  return gemm_nt(a, dtype, S(stream));
}
int fscnn_pw_dgrad_bnbwd(int M, int N, int K, const void* D, int ldd, const void* B, int ldb,
                         const void* R, int ldr, void* dX, int lddx, const void* z, int ldz,
                         const float* mean, const float* invstd, const float* scale,
                         const float* shift, int relu_mode, float* part, unsigned* counters,
                         double* tsum, float* dgamma, float* dbeta, float* coef, int dtype,
                         int* path, void* stream) {
  if (!D || !B || !dX || !z || !mean || !invstd || !scale || !shift || !part || !counters ||
      !tsum || !dgamma || !dbeta || !coef) {
    set_error("fscnn_pw_dgrad_bnbwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || (relu_mode != 0 && relu_mode != 2)) {
    set_error("fscnn_pw_dgrad_bnbwd: dtype %d / relu_mode %d", dtype, relu_mode);
    return E_INVALID;
  }
  // the executor's form (net.cpp Exec::pw_bwd + set_btarget)
  GemmArgs a{};
  a.M = M; a.N = N; a.K = K; a.A = D; a.lda = ldd; a.B = B; a.ldb = ldb; a.b_trans = 0;
  a.R = R; a.ldr = ldr; a.C = dX; a.ldc = lddx;
  a.bpart = part; a.bz = z; a.ldbz = ldz;
  a.bmean = mean; a.binvstd = invstd; a.bscale = scale; a.bshift = shift; a.bmode = relu_mode;
  a.tail.counters = counters; a.tail.tsum = tsum; a.tail.count = (double)M;
  a.tail.dgamma = dgamma; a.tail.dbeta = dbeta; a.tail.coef = coef;
  if (path) *path = gemm_stream_ok(a, dtype) ? 1 : 0;
  return gemm_nt(a, dtype, S(stream));
}
long long fscnn_pw_wgrad_slab_floats(int M, int N, int K) {
  return (long long)gemm_tn_splits(M, N, K) * N * K;
}
int fscnn_pw_wgrad(int M, int N, int K, const void* D, int ldd, const void* X, int ldx,
                   float* slab, float* dW, int dtype, void* stream) {
  GemmTnArgs a{};
  a.M = M; a.N = N; a.K = K; a.D = D; a.ldd = ldd; a.X = X; a.ldx = ldx; a.slab = slab;
  int s = gemm_tn_splits(M, N, K);
  int rc = gemm_tn(a, s, dtype, S(stream));
  if (rc) return rc;
  return reduce_slabs(slab, s, (long long)N * K, (long long)N * K, dW, 0, S(stream));
}

int fscnn_bn_finalize(float* part, int P, int C, const float* gamma, const float* beta,
                      float* rmean, float* rvar, long long* nbt, float momentum, float* mean,
                      float* invstd, float* scale, float* shift, void* stream) {
  BnFinalizeArgs a{};
  a.part = part; a.P = P; a.C = C; a.gamma = gamma; a.beta = beta; a.rmean = rmean;
  a.rvar = rvar; a.nbt = nbt; a.momentum = momentum; a.mean = mean; a.invstd = invstd;
  a.scale = scale; a.shift = shift;
  return bn_finalize(a, S(stream));
}

int fscnn_bilinear_ac_fwd(const void* x, int dtype, int N, int Hi, int Wi, int C, int Ho, int Wo,
                          void* y, int out_nchw, int out_dtype, void* stream) {
  UpArgs a{};
  a.N = N; a.Hi = Hi; a.Wi = Wi; a.C = C; a.Ho = Ho; a.Wo = Wo; a.x = x; a.ldx = C; a.y = y;
  a.ldy = C;
  if (out_nchw) return up_nchw(a, dtype, out_dtype, S(stream));
  return up_nhwc(a, dtype, S(stream));
}
int fscnn_bilinear_ac_bwd(const void* dy, int dtype, int N, int Hi, int Wi, int C, int Ho, int Wo,
                          float* tmp, void* dx, void* stream) {
  AxisBwdArgs a{};
  a.n_o1 = (long long)N * Ho; a.n_o2 = 1; a.Lout = Wo; a.Lin = Wi; a.n_in = C;
  a.g = dy; a.g_s1 = (long long)Wo * C; a.g_idx = C; a.g_in = 1;
  a.d = tmp; a.d_s1 = (long long)Wi * C; a.d_idx = C; a.d_in = 1;
  int rc = axis_bwd(a, dtype, DT_F32, S(stream));
  if (rc) return rc;
  AxisBwdArgs b{};
  b.n_o1 = N; b.n_o2 = 1; b.Lout = Ho; b.Lin = Hi; b.n_in = (long long)Wi * C;
  b.g = tmp; b.g_s1 = (long long)Ho * Wi * C; b.g_idx = (long long)Wi * C; b.g_in = 1;
  b.d = dx; b.d_s1 = (long long)Hi * Wi * C; b.d_idx = (long long)Wi * C; b.d_in = 1;
  return axis_bwd(b, DT_F32, dtype, S(stream));
}
int fscnn_pyramid_pool_fwd(const void* x, int dtype, int N, int H, int W, int C, int ldx,
                           void* pooled, void* stream) {
  PoolArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.x = x; a.ldx = ldx; a.pooled = pooled;
  return pyramid_pool(a, dtype, S(stream));
}
int fscnn_pyramid_pool_bwd(const void* dpooled, int dtype, int N, int H, int W, int C, void* dx,
                           int lddx, int accumulate, void* stream) {
  PoolBwdArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.dpooled = dpooled; a.dx = dx; a.lddx = lddx;
  a.accumulate = accumulate;
  return pyramid_pool_bwd(a, dtype, S(stream));
}

int fscnn_block_ir_fwd(const void* x, int ldx, int dtype, int N, int H, int W, int cin, int expand,
                       int cout, const void* w_expand, const float* w_dw, const void* w_project,
                       const float* scale_e, const float* shift_e, const float* scale_d,
                       const float* shift_d, const float* scale_p, const float* shift_p,
                       int residual, void* y, int ldy, void* stream) {
  if (!x || !y || !w_expand || !w_dw || !w_project || !scale_e || !shift_e || !scale_d ||
      !shift_d || !scale_p || !shift_p) {
    set_error("fscnn_block_ir_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16) {
    set_error("fscnn_block_ir_fwd: dtype %d", dtype);
    return E_INVALID;
  }
  IrArgs a{};
  a.N = N; a.H = H; a.W = W; a.Cin = cin; a.E = expand; a.Cout = cout;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy;
  a.we = w_expand; a.wd = w_dw; a.wp = w_project;
  a.sc_e = scale_e; a.sh_e = shift_e; a.sc_d = scale_d; a.sh_d = shift_d;
  a.sc_p = scale_p; a.sh_p = shift_p; a.residual = residual;
  return ir_block_fwd(a, dtype, S(stream));
}

int fscnn_block_ir_s2_fwd(const void* x, int ldx, int dtype, int N, int H, int W, int cin,
                          int expand, int cout, const void* w_expand, const float* w_dw,
                          const void* w_project, const float* scale_e, const float* shift_e,
                          const float* scale_d, const float* shift_d, const float* scale_p,
                          const float* shift_p, void* y, int ldy, void* stream) {
  if (!x || !y || !w_expand || !w_dw || !w_project || !scale_e || !shift_e || !scale_d ||
      !shift_d || !scale_p || !shift_p) {
    set_error("fscnn_block_ir_s2_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || H < 1 || W < 1) {
    set_error("fscnn_block_ir_s2_fwd: dtype %d H %d W %d", dtype, H, W);
    return E_INVALID;
  }
  IrArgs a{};
  a.stride = 2; a.Hi = H; a.Wi = W;
  a.N = N; a.H = (H - 1) / 2 + 1; a.W = (W - 1) / 2 + 1; a.Cin = cin; a.E = expand; a.Cout = cout;
  a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy;
  a.we = w_expand; a.wd = w_dw; a.wp = w_project;
  a.sc_e = scale_e; a.sh_e = shift_e; a.sc_d = scale_d; a.sh_d = shift_d;
  a.sc_p = scale_p; a.sh_p = shift_p; a.residual = 0;
  return ir_block_fwd(a, dtype, S(stream));
}

int fscnn_block_ltd_fwd(const void* x, int x_dtype, int dtype, int N, int H, int W,
                        const float* w_conv, const float* scale_0, const float* shift_0,
                        const float* w_dw, const float* scale_d, const float* shift_d,
                        const void* w_pw, const float* scale_p, const float* shift_p, void* y,
                        int ldy, void* stream) {
  if (!x || !y || !w_conv || !scale_0 || !shift_0 || !w_dw || !scale_d || !shift_d || !w_pw ||
      !scale_p || !shift_p) {
    set_error("fscnn_block_ltd_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || x_dtype < 0 || x_dtype > 2 || H < 3 || W < 3) {
    set_error("fscnn_block_ltd_fwd: dtype %d x_dtype %d H %d W %d", dtype, x_dtype, H, W);
    return E_INVALID;
  }
  StemArgs a{};
  a.x = x; a.x_dtype = x_dtype;
  a.N = N; a.H = H; a.W = W;
  a.H1 = (H - 3) / 2 + 1; a.W1 = (W - 3) / 2 + 1;
  a.H2 = (a.H1 - 1) / 2 + 1; a.W2 = (a.W1 - 1) / 2 + 1;
  a.w0 = w_conv; a.sc0 = scale_0; a.sh0 = shift_0;
  a.wd = w_dw; a.scd = scale_d; a.shd = shift_d;
  a.wp = w_pw; a.scp = scale_p; a.shp = shift_p;
  a.y = y; a.ldy = ldy;
  return stem_fwd(a, dtype, S(stream));
}

int fscnn_block_dsconv_fwd(const void* x, int dtype, int N, int H, int W, int C, int Co,
                           const float* w_dw, const float* scale_d, const float* shift_d,
                           const void* w_pw, const float* scale_p, const float* shift_p, void* y,
                           int ldy, void* stream) {
  if (!x || !y || !w_dw || !scale_d || !shift_d || !w_pw || !scale_p || !shift_p) {
    set_error("fscnn_block_dsconv_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || N <= 0 || H <= 0 || W <= 0) {
    set_error("fscnn_block_dsconv_fwd: dtype %d N %d H %d W %d", dtype, N, H, W);
    return E_INVALID;
  }
  DsArgs a{};
  a.x = x; a.N = N; a.H = H; a.W = W; a.C = C; a.Co = Co;
  a.wd = w_dw; a.scd = scale_d; a.shd = shift_d;
  a.wp = w_pw; a.scp = scale_p; a.shp = shift_p;
  a.y = y; a.ldy = ldy;
  a.rs = ds_rows(N, H, W);
  return ds_fwd(a, dtype, S(stream));
}

int fscnn_block_dsconv_res_fwd(const void* x, int dtype, int N, int H, int W, int C, int Co,
                               int Hi, int Wi, const float* w_dw, const float* scale_d, const float* shift_d,
                               const void* w_pw, const float* scale_p, const float* shift_p,
                               const void* res, int ldres, void* y, int ldy, void* stream) {
  if (!x || !y || !res || !w_dw || !scale_d || !shift_d || !w_pw || !scale_p || !shift_p) {
    set_error("fscnn_block_dsconv_res_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || N <= 0 || H <= 0 || W <= 0) {
    set_error("fscnn_block_dsconv_res_fwd: dtype %d N %d H %d W %d", dtype, N, H, W);
    return E_INVALID;
  }
  DsArgs a{};
  a.x = x; a.N = N; a.H = H; a.W = W; a.C = C; a.Co = Co;
  a.wd = w_dw; a.scd = scale_d; a.shd = shift_d;
  a.wp = w_pw; a.scp = scale_p; a.shp = shift_p;
  a.r = res; a.ldr = ldres;
  a.Hi = Hi > 0 ? Hi : 0; a.Wi = Hi > 0 ? Wi : 0;
  a.y = y; a.ldy = ldy;
  a.rs = ds_rows(N, H, W);
  return ds_fwd(a, dtype, S(stream));
}

int fscnn_block_cls_fwd(const void* x, int dtype, int N, int H, int W, const float* w_dw1,
                        const float* scale_d1, const float* shift_d1, const void* w_pw1,
                        const float* scale_p1, const float* shift_p1, const float* w_dw2,
                        const float* scale_d2, const float* shift_d2, const void* w_pw2,
                        const float* scale_p2, const float* shift_p2, const void* w_cls,
                        const float* b_cls, int ncls, void* tmp, void* logits, int ldl,
                        void* stream) {
  if (!x || !tmp || !logits || !w_dw1 || !scale_d1 || !shift_d1 || !w_pw1 || !scale_p1 ||
      !shift_p1 || !w_dw2 || !scale_d2 || !shift_d2 || !w_pw2 || !scale_p2 || !shift_p2 || !w_cls ||
      !b_cls) {
    set_error("fscnn_block_cls_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || N <= 0 || H <= 0 || W <= 0) {
    set_error("fscnn_block_cls_fwd: dtype %d N %d H %d W %d", dtype, N, H, W);
    return E_INVALID;
  }
  DsArgs a{};  // dsconv1 -> tmp
  a.x = x; a.N = N; a.H = H; a.W = W; a.C = 128; a.Co = 128;
  a.wd = w_dw1; a.scd = scale_d1; a.shd = shift_d1;
  a.wp = w_pw1; a.scp = scale_p1; a.shp = shift_p1;
  a.y = tmp; a.ldy = 128;
  a.rs = ds_rows(N, H, W);
  DsArgs b = a;  // dsconv2 + the classifier conv -> logits
  b.x = tmp;
  b.wd = w_dw2; b.scd = scale_d2; b.shd = shift_d2;
  b.wp = w_pw2; b.scp = scale_p2; b.shp = shift_p2;
  b.wc = w_cls; b.bc = b_cls; b.ncls = ncls; b.logits = logits; b.ldl = ldl;
  if (!ds_ok(a) || !ds_ok(b)) {
    set_error("fscnn_block_cls_fwd: unsupported shape N=%d H=%d W=%d ncls=%d ldl=%d", N, H, W, ncls, ldl);
    return E_UNSUPPORTED;
  }
  const int rc = ds_fwd(a, dtype, S(stream));
  return rc ? rc : ds_fwd(b, dtype, S(stream));
}

int fscnn_block_ffm_fwd(const void* low, int dtype, int N, int Hi, int Wi, int H, int W,
                        const void* high, int ldhigh, const float* w_dw, const float* scale_d,
                        const float* shift_d, const void* w_low, const float* scale_l,
                        const float* shift_l, const void* w_high, const float* scale_h,
                        const float* shift_h, void* y, int ldy, void* stream) {
  if (!low || !high || !y || !w_dw || !scale_d || !shift_d || !w_low || !scale_l || !shift_l ||
      !w_high || !scale_h || !shift_h) {
    set_error("fscnn_block_ffm_fwd: null argument");
    return E_INVALID;
  }
  if (dtype < DT_F32 || dtype > DT_F16 || N <= 0 || H <= 0 || W <= 0 || Hi <= 0 || Wi <= 0) {
    set_error("fscnn_block_ffm_fwd: dtype %d N %d Hi %d Wi %d H %d W %d", dtype, N, Hi, Wi, H, W);
    return E_INVALID;
  }
  DsArgs a{};
  a.x = low; a.N = N; a.H = H; a.W = W; a.C = 128; a.Co = 128; a.Hi = Hi; a.Wi = Wi;
  a.wd = w_dw; a.scd = scale_d; a.shd = shift_d;
  a.wp = w_low; a.scp = scale_l; a.shp = shift_l;
  a.xh = high; a.ldxh = ldhigh; a.wh = w_high; a.sch = scale_h; a.shh = shift_h;
  a.y = y; a.ldy = ldy;
  a.rs = ds_rows(N, H, W);
  return ds_fwd(a, dtype, S(stream));
}

}  // extern "C"

extern "C" int fscnn_plan_buffer(const fscnn_plan* plan, const char* name, long long* offset,
                                 long long* rows, int* cols, int* ld, int* in_bws) {
  if (!plan || !name) { set_error("fscnn_plan_buffer: null argument"); return E_INVALID; }
  for (const auto& b : plan->plan.named) {
    if (b.name == name) {
      if (offset) *offset = (long long)b.off;
      if (rows) *rows = b.rows;
      if (cols) *cols = b.cols;
      if (ld) *ld = b.ld;
      if (in_bws) *in_bws = b.bws;
      return OK;
    }
  }
  set_error("fscnn_plan_buffer: no buffer named '%s' in this plan", name);
  return E_INVALID;
}
