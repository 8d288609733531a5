// Bilinear upsampling with align_corners=True (models/fast_scnn.py:40 final logits, :135 PPM
// features, :212 FFM lower-resolution branch) and the pyramid pooling reduce
// AdaptiveAvgPool2d(1,2,3,6) (:130-132, overlapping windows).
//
// The source index / lambda law is aten's compute_source_index_and_lambda in fp32
// (common.hpp ac_lerp), so the GPU reproduces the CPU oracle's weights exactly.
// Backward passes are separable GATHERS along one axis at a time (no atomics, deterministic):
// for input index i the contributing outputs form the contiguous range [lo(i), hi(i)) found by
// binary search on the monotone i0(o).
#include "kernels.hpp"

namespace fscnn {

// ---- forward NHWC -> NHWC (optionally into a channel slice of a wider buffer) ---------------

template <typename T>
__global__ __launch_bounds__(256) void up_nhwc_kernel(UpArgs a) {
  constexpr int V = VecW<T>::V;
  const int CV = a.C / V;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)a.N * a.Ho * a.Wo * CV;
  if (i >= total) return;
  int cv = (int)(i % CV);
  long long pix = i / CV;
  int wo = (int)(pix % a.Wo);
  long long r = pix / a.Wo;
  int ho = (int)(r % a.Ho);
  int n = (int)(r / a.Ho);
  Lerp lh = ac_lerp(ho, a.Hi, a.Ho, ac_scale(a.Hi, a.Ho));
  Lerp lw = ac_lerp(wo, a.Wi, a.Wo, ac_scale(a.Wi, a.Wo));
  const T* xb = (const T*)a.x + (size_t)n * a.Hi * a.Wi * a.ldx + cv * V;
  float p00[V], p01[V], p10[V], p11[V], o[V];
  ldv(xb + ((size_t)lh.i0 * a.Wi + lw.i0) * a.ldx, p00);
  ldv(xb + ((size_t)lh.i0 * a.Wi + lw.i1) * a.ldx, p01);
  ldv(xb + ((size_t)lh.i1 * a.Wi + lw.i0) * a.ldx, p10);
  ldv(xb + ((size_t)lh.i1 * a.Wi + lw.i1) * a.ldx, p11);
#pragma unroll
  for (int j = 0; j < V; ++j)
    o[j] = lerp2(lh.l0, lerp2(lw.l0, p00[j], lw.l1, p01[j]), lh.l1, lerp2(lw.l0, p10[j], lw.l1, p11[j]));
  stv((T*)a.y + pix * a.ldy + cv * V, o);
}

int up_nhwc(const UpArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  if (a.C % V || a.ldx % V || a.ldy % V) {
    set_error("up_nhwc: C=%d ldx=%d ldy=%d must be multiples of %d", a.C, a.ldx, a.ldy, V);
    return E_INVALID;
  }
  long long total = (long long)a.N * a.Ho * a.Wo * (a.C / V);
  unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) prof_launch(up_nhwc_kernel<float>, grid, 256, 0, st, a);
  else if (dtype == DT_F16) prof_launch(up_nhwc_kernel<f16>, grid, 256, 0, st, a);
  else prof_launch(up_nhwc_kernel<bf16>, grid, 256, 0, st, a);
  return check_launch("up_nhwc");
}

// ---- forward NHWC (padded channels) -> NCHW logits (the final F.interpolate) -----------------
// One thread per output pixel; lanes run along wo so every per-class plane store is coalesced.
template <typename TI, typename TO, int CMAX>
__global__ __launch_bounds__(256) void up_nchw_kernel(UpArgs a) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)a.N * a.Ho * a.Wo;
  if (i >= total) return;
  int wo = (int)(i % a.Wo);
  long long r = i / a.Wo;
  int ho = (int)(r % a.Ho);
  int n = (int)(r / a.Ho);
  Lerp lh = ac_lerp(ho, a.Hi, a.Ho, ac_scale(a.Hi, a.Ho));
  Lerp lw = ac_lerp(wo, a.Wi, a.Wo, ac_scale(a.Wi, a.Wo));
  const TI* xb = (const TI*)a.x + (size_t)n * a.Hi * a.Wi * a.ldx;
  const TI* q00 = xb + ((size_t)lh.i0 * a.Wi + lw.i0) * a.ldx;
  const TI* q01 = xb + ((size_t)lh.i0 * a.Wi + lw.i1) * a.ldx;
  const TI* q10 = xb + ((size_t)lh.i1 * a.Wi + lw.i0) * a.ldx;
  const TI* q11 = xb + ((size_t)lh.i1 * a.Wi + lw.i1) * a.ldx;
  TO* yb = (TO*)a.y + (size_t)n * a.C * a.Ho * a.Wo + (size_t)ho * a.Wo + wo;
  const size_t plane = (size_t)a.Ho * a.Wo;
#pragma unroll 4
  for (int c = 0; c < a.C; ++c) {
    float o = lerp2(lh.l0, lerp2(lw.l0, ld1(q00 + c), lw.l1, ld1(q01 + c)),
                    lh.l1, lerp2(lw.l0, ld1(q10 + c), lw.l1, ld1(q11 + c)));
    st1(yb + c * plane, o);
  }
}

// Row-group form (the 1.27 GB fp32 write of cfg2 is the whole cost, so stores are what matter):
// a workgroup owns UPR_RS consecutive output rows of image n and UPR_COLS columns.  The source
// rows they read, [i0(first row), i1(last row)] (at most `rows` of them, bounded on the host), are
// staged once in LDS class-major [row][C][Wi+1] in fp32; then every thread produces 4
// consecutive columns of each class plane of each of the UPR_RS rows and writes them with 16-B
// (fp32) / 8-B (bf16) non-temporal stores.  Same weights and the same W-then-H expression as aten,
// so the fp32 result is bit-identical to the per-pixel kernel above.
constexpr int UPR_THREADS = 512;
constexpr int UPR_COLS = 4 * UPR_THREADS;
constexpr int UPR_R = 8;   // output rows per workgroup of up_argmax
constexpr int UPR_RS = 4;  // ... of up_nchw_rows (the logits upsample)
constexpr int UPR_MAXROWS = 4;  // staged source rows per group (host-checked)

typedef float upr_f4 __attribute__((ext_vector_type(4)));
typedef unsigned int upr_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st4_nt(float* p, const float (&v)[4]) {
  upr_f4 t = {v[0], v[1], v[2], v[3]};
  __builtin_nontemporal_store(t, (upr_f4*)p);
}
__device__ __forceinline__ void st4_nt(bf16* p, const float (&v)[4]) {
  upr_u2 t = {(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
               (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
  __builtin_nontemporal_store(t, (upr_u2*)p);
}
__device__ __forceinline__ void st4_nt(f16* p, const float (&v)[4]) {
  upr_u2 t = {(uint32_t)f2h(v[0]) | ((uint32_t)f2h(v[1]) << 16),
               (uint32_t)f2h(v[2]) | ((uint32_t)f2h(v[3]) << 16)};
  __builtin_nontemporal_store(t, (upr_u2*)p);
}

template <typename TI, typename TO, bool VEC, int RR, int MAXR = UPR_MAXROWS>
__global__ __launch_bounds__(UPR_THREADS) void up_nchw_rows_kernel(UpArgs a) {
  extern __shared__ float s_rows[];  // [rows][C][Wi + 1] (padded: the staging stores walk c)
  const int ho0 = blockIdx.y * RR, n = blockIdx.z;
  const int ho1 = min(ho0 + RR, a.Ho) - 1;
  const float sh = ac_scale(a.Hi, a.Ho);
  const int lo = ac_lerp(ho0, a.Hi, a.Ho, sh).i0;
  const int nrows = ac_lerp(ho1, a.Hi, a.Ho, sh).i1 - lo + 1;  // <= host bound
  const int WP = a.Wi + 1, CWP = a.C * WP, CW = a.C * a.Wi;
  const TI* xb = (const TI*)a.x + ((size_t)n * a.Hi + lo) * a.Wi * a.ldx;
  // stage: element e = (r, wi, c) with c fastest in global memory (NHWC), class-major in LDS;
  // 8 loads per thread in flight per batch (one element per iteration was a chain of memory
  // round trips before the first store of the workgroup)
  const int ne = nrows * CW;
  for (int e0 = threadIdx.x; e0 < ne; e0 += 8 * UPR_THREADS) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * UPR_THREADS, ec = e < ne ? e : e0;
      const int r = ec / CW;
      const int rem = ec - r * CW;
      const int wi = rem / a.C, c = rem - wi * a.C;
      v[u] = ld1(xb + ((size_t)r * a.Wi + wi) * a.ldx + c);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * UPR_THREADS;
      if (e < ne) {
        const int r = e / CW;
        const int rem = e - r * CW;
        const int wi = rem / a.C, c = rem - wi * a.C;
        s_rows[r * CWP + c * WP + wi] = v[u];
      }
    }
  }
  __syncthreads();
  const int wo0 = blockIdx.x * UPR_COLS + threadIdx.x * 4;
  if (wo0 >= a.Wo) return;
  const float sw = ac_scale(a.Wi, a.Wo);
  Lerp lw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) lw[j] = ac_lerp(min(wo0 + j, a.Wo - 1), a.Wi, a.Wo, sw);
  const size_t plane = (size_t)a.Ho * a.Wo;
  TO* yb = (TO*)a.y + (size_t)n * a.C * plane + wo0;
  // the RR output rows' H-interpolation (staged-row indices and weights), once for every class
  Lerp lh[RR];
#pragma unroll
  for (int q = 0; q < RR; ++q) {
    lh[q] = ac_lerp(min(ho0 + q, a.Ho - 1), a.Hi, a.Ho, sh);
    lh[q].i0 -= lo;
    lh[q].i1 -= lo;
  }
  for (int c = 0; c < a.C; ++c) {
    // W-interpolation of each staged source row for this thread's 4 columns (aten's inner
    // bracket), computed once and shared by the RR output rows
    float wr[MAXR][4];
#pragma unroll
    for (int r = 0; r < MAXR; ++r) {
      const float* row = s_rows + min(r, nrows - 1) * CWP + c * WP;
#pragma unroll
      for (int j = 0; j < 4; ++j) wr[r][j] = lerp2(lw[j].l0, row[lw[j].i0], lw[j].l1, row[lw[j].i1]);
    }
#pragma unroll
    for (int q = 0; q < RR; ++q) {
      const int ho = ho0 + q;
      if (ho > ho1) break;
      const int d0 = lh[q].i0, d1 = lh[q].i1;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x0 = wr[0][j], x1 = wr[0][j];
#pragma unroll
        for (int r = 1; r < MAXR; ++r) {  // register selects, no dynamic indexing
          x0 = d0 == r ? wr[r][j] : x0;
          x1 = d1 == r ? wr[r][j] : x1;
        }
        o[j] = lerp2(lh[q].l0, x0, lh[q].l1, x1);
      }
      TO* yp = yb + c * plane + (size_t)ho * a.Wo;
      if (VEC && wo0 + 4 <= a.Wo) {
        st4_nt(yp, o);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (wo0 + j < a.Wo) st1(yp + j, o[j]);
      }
    }
  }
}

// largest number of source rows any UPR_R-row group reads (host copy of the kernel's bound)
static int upr_max_rows(int Hi, int Ho, int UPR_R = fscnn::UPR_R) {
  const float sh = ac_scale(Hi, Ho);
  int mx = 0;
  for (int g0 = 0; g0 < Ho; g0 += UPR_R) {
    const int g1 = (g0 + UPR_R < Ho ? g0 + UPR_R : Ho) - 1;
    const int r = ac_lerp(g1, Hi, Ho, sh).i1 - ac_lerp(g0, Hi, Ho, sh).i0 + 1;
    mx = r > mx ? r : mx;
  }
  return mx;
}

int up_nchw(const UpArgs& a, int in_dtype, int out_dtype, hipStream_t st) {
  long long total = (long long)a.N * a.Ho * a.Wo;
  unsigned grid = (unsigned)((total + 255) / 256);
  ProfScope ps(PK_UP, st,
               (in_dtype == DT_F32 ? 4.0 : 2.0) * a.N * a.C * a.Hi * a.Wi +
                   (out_dtype == DT_F32 ? 4.0 : 2.0) * (double)a.N * a.C * a.Ho * a.Wo,
               7.0 * a.N * a.C * a.Ho * a.Wo);
  // 4 output rows per workgroup: 2048 workgroups at cfg2 (r06 rocprof: 254 vs 262 us with 8 rows,
  // 255 with 2; 16 / 24 rows leave the chip underfilled, +350 us)
  constexpr int RR = UPR_RS;
  const size_t lds = (size_t)upr_max_rows(a.Hi, a.Ho, RR) * a.C * (a.Wi + 1) * sizeof(float);
  if (lds <= 64 * 1024 && a.N <= 65535 && upr_max_rows(a.Hi, a.Ho, RR) <= UPR_MAXROWS) {
    dim3 g((unsigned)cdiv(a.Wo, UPR_COLS), (unsigned)cdiv(a.Ho, RR), (unsigned)a.N);
    const bool vec = a.Wo % 4 == 0;
    // staged rows per group (3 at cfg2's x8): the W-interpolations and selects of that many
    const int mr = upr_max_rows(a.Hi, a.Ho, RR);
#define UPR_LAUNCH(TI, TO)                                                              \
  do {                                                                                  \
    if (vec && mr <= 2) prof_launch(up_nchw_rows_kernel<TI, TO, true, RR, 2>, g, UPR_THREADS, lds, st, a); \
    else if (vec && mr == 3) prof_launch(up_nchw_rows_kernel<TI, TO, true, RR, 3>, g, UPR_THREADS, lds, st, a); \
    else if (vec) prof_launch(up_nchw_rows_kernel<TI, TO, true, RR>, g, UPR_THREADS, lds, st, a); \
    else prof_launch(up_nchw_rows_kernel<TI, TO, false, RR>, g, UPR_THREADS, lds, st, a);        \
  } while (0)
    if (in_dtype == DT_F32 && out_dtype == DT_F32) UPR_LAUNCH(float, float);
    else if (in_dtype == DT_F16 && out_dtype == DT_F16) UPR_LAUNCH(f16, f16);
    else if (in_dtype == DT_F16 && out_dtype == DT_F32) UPR_LAUNCH(f16, float);
    else if (in_dtype == DT_F16) UPR_LAUNCH(f16, bf16);
    else if (in_dtype == DT_BF16 && out_dtype == DT_F16) UPR_LAUNCH(bf16, f16);
    else if (in_dtype == DT_F32 && out_dtype == DT_F16) UPR_LAUNCH(float, f16);
    else if (in_dtype == DT_BF16 && out_dtype == DT_BF16) UPR_LAUNCH(bf16, bf16);
    else if (in_dtype == DT_BF16 && out_dtype == DT_F32) UPR_LAUNCH(bf16, float);
    else UPR_LAUNCH(float, bf16);
#undef UPR_LAUNCH
    return check_launch("up_nchw");
  }
  if (in_dtype == DT_F32 && out_dtype == DT_F32) prof_launch(up_nchw_kernel<float, float, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_F16 && out_dtype == DT_F16) prof_launch(up_nchw_kernel<f16, f16, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_F16 && out_dtype == DT_F32) prof_launch(up_nchw_kernel<f16, float, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_F16) prof_launch(up_nchw_kernel<f16, bf16, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_BF16 && out_dtype == DT_F16) prof_launch(up_nchw_kernel<bf16, f16, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_F32 && out_dtype == DT_F16) prof_launch(up_nchw_kernel<float, f16, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_BF16 && out_dtype == DT_BF16) prof_launch(up_nchw_kernel<bf16, bf16, 0>, grid, 256, 0, st, a);
  else if (in_dtype == DT_BF16 && out_dtype == DT_F32) prof_launch(up_nchw_kernel<bf16, float, 0>, grid, 256, 0, st, a);
  else prof_launch(up_nchw_kernel<float, bf16, 0>, grid, 256, 0, st, a);
  return check_launch("up_nchw");
}

// ---- eval: final upsample fused with the argmax over classes --------------------------------
// eval.py:45 / demo.py:48 consume only torch.argmax(outputs[0], 1).  Same staging and the same
// W-then-H arithmetic as up_nchw_rows_kernel, so each label is the argmax of exactly the values
// up_nchw writes (rounded to bf16 first when the logits are bf16), ties resolving to the lowest
// class like torch.argmax.  Only the labels are written (int64 like torch.argmax, or uint8):
// 134 / 17 MB at cfg2 instead of the 1.27 GB of fp32 logits.
template <typename TI, typename TL>
__global__ __launch_bounds__(UPR_THREADS) void up_argmax_kernel(UpArgs a, TL* labels) {
  extern __shared__ float s_rows[];
  const int ho0 = blockIdx.y * UPR_R, n = blockIdx.z;
  const int ho1 = min(ho0 + UPR_R, a.Ho) - 1;
  const float sh = ac_scale(a.Hi, a.Ho);
  const int lo = ac_lerp(ho0, a.Hi, a.Ho, sh).i0;
  const int nrows = ac_lerp(ho1, a.Hi, a.Ho, sh).i1 - lo + 1;
  const int WP = a.Wi + 1, CWP = a.C * WP, CW = a.C * a.Wi;
  const TI* xb = (const TI*)a.x + ((size_t)n * a.Hi + lo) * a.Wi * a.ldx;
  for (int e = threadIdx.x; e < nrows * CW; e += UPR_THREADS) {
    const int r = e / CW;
    const int rem = e - r * CW;
    const int wi = rem / a.C, c = rem - wi * a.C;
    s_rows[r * CWP + c * WP + wi] = ld1(xb + ((size_t)r * a.Wi + wi) * a.ldx + c);
  }
  __syncthreads();
  const int wo0 = blockIdx.x * UPR_COLS + threadIdx.x * 4;
  if (wo0 >= a.Wo) return;
  const float sw = ac_scale(a.Wi, a.Wo);
  Lerp lw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) lw[j] = ac_lerp(min(wo0 + j, a.Wo - 1), a.Wi, a.Wo, sw);
  float best[UPR_R][4];
  int arg[UPR_R][4];
#pragma unroll
  for (int rr = 0; rr < UPR_R; ++rr)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      best[rr][j] = -INFINITY;
      arg[rr][j] = 0;
    }
  for (int c = 0; c < a.C; ++c) {
    float wr[UPR_MAXROWS][4];
#pragma unroll
    for (int r = 0; r < UPR_MAXROWS; ++r) {
      const float* row = s_rows + min(r, nrows - 1) * CWP + c * WP;
#pragma unroll
      for (int j = 0; j < 4; ++j) wr[r][j] = lerp2(lw[j].l0, row[lw[j].i0], lw[j].l1, row[lw[j].i1]);
    }
#pragma unroll
    for (int rr = 0; rr < UPR_R; ++rr) {
      const Lerp lh = ac_lerp(min(ho0 + rr, ho1), a.Hi, a.Ho, sh);
      const int d0 = lh.i0 - lo, d1 = lh.i1 - lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x0 = wr[0][j], x1 = wr[0][j];
#pragma unroll
        for (int r = 1; r < UPR_MAXROWS; ++r) {
          x0 = d0 == r ? wr[r][j] : x0;
          x1 = d1 == r ? wr[r][j] : x1;
        }
        float o = lerp2(lh.l0, x0, lh.l1, x1);
        o = round_as<TI>(o);  // the logits up_nchw would store
        const bool gt = o > best[rr][j];
        best[rr][j] = gt ? o : best[rr][j];
        arg[rr][j] = gt ? c : arg[rr][j];
      }
    }
  }
#pragma unroll
  for (int rr = 0; rr < UPR_R; ++rr) {
    if (ho0 + rr > ho1) break;
    TL* lp = labels + ((size_t)n * a.Ho + ho0 + rr) * a.Wo + wo0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (wo0 + j < a.Wo) lp[j] = (TL)arg[rr][j];
  }
}

int up_argmax(const UpArgs& a, int in_dtype, void* labels, int label_u8, hipStream_t st) {
  const int rows = upr_max_rows(a.Hi, a.Ho);
  const size_t lds = (size_t)rows * a.C * (a.Wi + 1) * sizeof(float);
  if (lds > 64 * 1024 || a.N > 65535 || rows > UPR_MAXROWS || a.C < 1) {
    set_error("up_argmax: unsupported geometry (Hi=%d Ho=%d Wi=%d C=%d)", a.Hi, a.Ho, a.Wi, a.C);
    return E_UNSUPPORTED;
  }
  dim3 g((unsigned)cdiv(a.Wo, UPR_COLS), (unsigned)cdiv(a.Ho, UPR_R), (unsigned)a.N);
  if (in_dtype == DT_F32) {
    if (label_u8) prof_launch(up_argmax_kernel<float, uint8_t>, g, UPR_THREADS, lds, st, a, (uint8_t*)labels);
    else prof_launch(up_argmax_kernel<float, long long>, g, UPR_THREADS, lds, st, a, (long long*)labels);
  } else if (in_dtype == DT_F16) {
    if (label_u8) prof_launch(up_argmax_kernel<f16, uint8_t>, g, UPR_THREADS, lds, st, a, (uint8_t*)labels);
    else prof_launch(up_argmax_kernel<f16, long long>, g, UPR_THREADS, lds, st, a, (long long*)labels);
  } else {
    if (label_u8) prof_launch(up_argmax_kernel<bf16, uint8_t>, g, UPR_THREADS, lds, st, a, (uint8_t*)labels);
    else prof_launch(up_argmax_kernel<bf16, long long>, g, UPR_THREADS, lds, st, a, (long long*)labels);
  }
  return check_launch("up_argmax");
}

// ---- backward: gather along one axis --------------------------------------------------------
// Element (o1, o2, i, x) of the grad wrt the forward INPUT (i < Lin along the interpolated axis)
// is the sum over forward outputs p (< Lout) that read index i of w(p, i) * g(o1, o2, p, x).
// Every coordinate has its own stride on both sides, so the same kernel serves NCHW logits and
// NHWC activations.  Threads run fastest along x.

__device__ __forceinline__ int first_out_with_i0_ge(int i, int Lin, int Lout, float sc) {
  // smallest p with i0(p) >= i (i0 monotone non-decreasing in p)
  int lo = 0, hi = Lout;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (ac_lerp(mid, Lin, Lout, sc).i0 >= i) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// grid: x = 256-thread chunks of the (o, x) positions of one input index, y = input index i.
// The contributing output range [p_lo, p_hi) of index i is found once per workgroup.
// VX = 4: the innermost coordinate is contiguous on both sides (channels of an NHWC tensor), so a
// thread owns 4 consecutive x and every load / store is one 8-B (bf16) or 16-B (fp32) vector.
template <typename TG, typename TD, int VX>
__global__ __launch_bounds__(256) void axis_bwd_kernel(AxisBwdArgs a) {
  __shared__ int s_rng[2];
  const int i = blockIdx.y;
  const float sc = ac_scale(a.Lin, a.Lout);
  if (threadIdx.x == 0) {
    // contributors: outputs p with i0(p) in {i-1, i}  (i1 = i0 or i0+1)
    s_rng[0] = first_out_with_i0_ge(i - 1, a.Lin, a.Lout, sc);
    s_rng[1] = first_out_with_i0_ge(i + 1, a.Lin, a.Lout, sc);
  }
  __syncthreads();
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned n_o = (unsigned)(a.n_o1 * a.n_o2), n_in = (unsigned)(a.n_in / VX);
  if (t >= n_o * n_in) return;
  const unsigned o = t / n_in, x = (t - o * n_in) * VX;
  const unsigned o1 = o / (unsigned)a.n_o2, o2 = o - o1 * (unsigned)a.n_o2;
  const int p_lo = s_rng[0], p_hi = s_rng[1];
  const TG* gb = (const TG*)a.g + (long long)o1 * a.g_s1 + (long long)o2 * a.g_s2 + (long long)x * a.g_in;
  float s[VX];
#pragma unroll
  for (int j = 0; j < VX; ++j) s[j] = 0.f;
  for (int p0 = p_lo; p0 < p_hi; p0 += 4) {  // 4 independent loads per batch
    float gv[4][VX], wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + u;
      const bool ok = p < p_hi;  // clamped load + select (branch-free)
      const Lerp l = ac_lerp(ok ? p : p0, a.Lin, a.Lout, sc);
      const float w = (l.i0 == i ? l.l0 : 0.f) + (l.i1 == i ? l.l1 : 0.f);
      if constexpr (VX == 4) ld4v(gb + (size_t)(ok ? p : p0) * a.g_idx, gv[u]);
      else gv[u][0] = ld1(gb + (size_t)(ok ? p : p0) * a.g_idx);
      wv[u] = ok ? w : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < VX; ++j) s[j] += wv[u] * gv[u][j];
  }
  TD* dp = (TD*)a.d + (long long)o1 * a.d_s1 + (long long)o2 * a.d_s2 + (long long)i * a.d_idx +
           (long long)x * a.d_in;
  if constexpr (VX == 4) {
    if (a.accumulate) {
      float prev[4];
      ld4v(dp, prev);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += prev[j];
    }
    st4v(dp, s);
  } else {
    if (a.accumulate) s[0] += ld1(dp);
    st1(dp, s[0]);
  }
}

int axis_bwd(const AxisBwdArgs& a, int g_dtype, int d_dtype, hipStream_t st) {
  const long long per_i = a.n_o1 * a.n_o2 * a.n_in;
  if (per_i >= (1LL << 31) || a.Lin > 65535) {
    set_error("axis_bwd: problem too large (%lld per index, Lin %d)", per_i, a.Lin);
    return E_UNSUPPORTED;
  }
  // vector form: x contiguous and every other stride / base a whole number of 4-element vectors
  const bool vec = a.g_in == 1 && a.d_in == 1 && a.n_in % 4 == 0 && a.g_s1 % 4 == 0 &&
                   a.g_s2 % 4 == 0 && a.g_idx % 4 == 0 && a.d_s1 % 4 == 0 && a.d_s2 % 4 == 0 &&
                   a.d_idx % 4 == 0 && (uintptr_t)a.g % 16 == 0 && (uintptr_t)a.d % 16 == 0;
  const int vx = vec ? 4 : 1;
  dim3 grid((unsigned)((per_i / vx + 255) / 256), a.Lin);
#define AXB(TG, TD)                                                          \
  do {                                                                       \
    if (vec) prof_launch(axis_bwd_kernel<TG, TD, 4>, grid, 256, 0, st, a);            \
    else prof_launch(axis_bwd_kernel<TG, TD, 1>, grid, 256, 0, st, a);                \
  } while (0)
  if (g_dtype == DT_F32 && d_dtype == DT_F32) AXB(float, float);
  else if (g_dtype == DT_BF16 && d_dtype == DT_BF16) AXB(bf16, bf16);
  else if (g_dtype == DT_BF16 && d_dtype == DT_F32) AXB(bf16, float);
  else if (g_dtype == DT_F16 && d_dtype == DT_F32) AXB(f16, float);
  else if (g_dtype == DT_F32 && d_dtype == DT_F16) AXB(float, f16);
  else if (g_dtype == DT_F16 && d_dtype == DT_F16) AXB(f16, f16);
  else AXB(float, bf16);
#undef AXB
  return check_launch("axis_bwd");
}

// ---- pyramid pooling: AdaptiveAvgPool2d(1), (2), (3), (6) in one launch ----------------------
// pooled layout: [N][50 bins][C] with bins ordered level-major (1x1, 2x2, 3x3, 6x6), row-major.
constexpr int PP_LEVELS[4] = {1, 2, 3, 6};
__device__ __forceinline__ void pp_bin(int b, int& k, int& bi, int& bj) {
  if (b < 1) { k = 1; b -= 0; }
  else if (b < 5) { k = 2; b -= 1; }
  else if (b < 14) { k = 3; b -= 5; }
  else { k = 6; b -= 14; }
  bi = b / k;
  bj = b - bi * k;
}
__host__ __device__ __forceinline__ int pp_start(int i, int in, int k) { return (i * in) / k; }
__host__ __device__ __forceinline__ int pp_end(int i, int in, int k) { return ((i + 1) * in + k - 1) / k; }


// one workgroup per (bin, image, slice of CVL channel vectors): PG = 256/CVL pixel groups, every
// thread walks its pixels of the window with 8 vector loads in flight per batch; the pixel groups
// are combined by a fixed-order tree through LDS.  (r06: a workgroup per (bin, image) over all C
// left the 2048-pixel 1x1 bins on 8 CUs walking 32 dependent load batches: 34 us at cfg2, 19 us
// at cfg3; slices of 4 vectors put 8x / 4x as many workgroups on every bin.)
template <typename T>
__global__ __launch_bounds__(256) void pyramid_pool_kernel(PoolArgs a, int CVL) {
  constexpr int V = VecW<T>::V;
  __shared__ float red[256 * V];
  const int b = blockIdx.x, n = blockIdx.y;
  const int PG = 256 / CVL;
  const int cl = threadIdx.x % CVL, g = threadIdx.x / CVL;
  const int cv = blockIdx.z * CVL + cl;
  int k, bi, bj;
  pp_bin(b, k, bi, bj);
  const int h0 = pp_start(bi, a.H, k), h1 = pp_end(bi, a.H, k);
  const int w0 = pp_start(bj, a.W, k), w1 = pp_end(bj, a.W, k);
  const int ww = w1 - w0, npx = (h1 - h0) * ww;
  const float inv = 1.f / (float)npx;
  const T* xb = (const T*)a.x + (size_t)n * a.H * a.W * a.ldx + cv * V;
  float s[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = 0.f;
  if (g < PG) {
    for (int q0 = g; q0 < npx; q0 += 8 * PG) {
      float v[8][V];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = q0 + u * PG;
        const bool ok = q < npx;  // clamped load + select (branch-free)
        const int qq = ok ? q : q0;
        const int hh = qq / ww, wq = qq - hh * ww;
        ldv(xb + ((size_t)(h0 + hh) * a.W + w0 + wq) * a.ldx, v[u]);
#pragma unroll
        for (int j = 0; j < V; ++j) v[u][j] = ok ? v[u][j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < V; ++j) s[j] += v[u][j];
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[threadIdx.x * V + j] = s[j];
  __syncthreads();
  for (int st = PG >> 1; st > 0; st >>= 1) {  // PG is a power of two (host-checked)
    if (g < st) {
#pragma unroll
      for (int j = 0; j < V; ++j) red[threadIdx.x * V + j] += red[(threadIdx.x + st * CVL) * V + j];
    }
    __syncthreads();
  }
  if (g == 0) {
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = red[threadIdx.x * V + j] * inv;
    stv((T*)a.pooled + ((size_t)b * a.N + n) * a.C + cv * V, o);
  }
}

int pyramid_pool(const PoolArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  const int CV = a.C / V;
  // channel-vector slice per workgroup: 4 vectors when that divides CV (eight fp32 / four 16-bit
  // slices of C = 128; two-vector 16-bit slices measured 13.8 vs 10.3 us at cfg3), else the whole
  // row (<= 256, a power of two so the pixel groups halve evenly)
  const int CVL = CV % 4 == 0 ? 4 : CV;
  if (a.C % V || CV > 256 || (CVL & (CVL - 1)) || a.ldx % V) {
    set_error("pyramid_pool: C=%d ldx=%d", a.C, a.ldx);
    return E_UNSUPPORTED;
  }
  dim3 grid(50, a.N, CV / CVL);
  if (dtype == DT_F32) prof_launch(pyramid_pool_kernel<float>, grid, 256, 0, st, a, CVL);
  else if (dtype == DT_F16) prof_launch(pyramid_pool_kernel<f16>, grid, 256, 0, st, a, CVL);
  else prof_launch(pyramid_pool_kernel<bf16>, grid, 256, 0, st, a, CVL);
  return check_launch("pyramid_pool");
}

// backward: dx[n,h,w,c] (+)= sum_levels sum_{bins containing (h,w)} dpooled[bin,n,c] / area

// one thread per (pixel, 16-B channel vector): the bin search runs once per 4 (fp32) / 8 (16-bit)
// channels instead of once per channel (25 us -> ? at cfg3)
template <typename T>
__global__ __launch_bounds__(256) void pyramid_pool_bwd_kernel(PoolBwdArgs a) {
  constexpr int V = VecW<T>::V;
  const int CV = a.C / V;
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)a.N * a.H * a.W * CV;
  if (t >= total) return;
  const int cv = (int)(t % CV);
  long long pix = t / CV;
  int w = (int)(pix % a.W);
  long long r = pix / a.W;
  int h = (int)(r % a.H);
  int n = (int)(r / a.H);
  float s[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s[j] = 0.f;
  int base = 0;
#pragma unroll
  for (int lv = 0; lv < 4; ++lv) {
    const int k = PP_LEVELS[lv];
    // all bins whose (possibly overlapping, possibly > input size) window holds (h, w)
    for (int bi = 0; bi < k; ++bi) {
      int h0 = pp_start(bi, a.H, k), h1 = pp_end(bi, a.H, k);
      if (h < h0 || h >= h1) continue;
      for (int bj = 0; bj < k; ++bj) {
        int w0 = pp_start(bj, a.W, k), w1 = pp_end(bj, a.W, k);
        if (w < w0 || w >= w1) continue;
        float v[V];
        ldv((const T*)a.dpooled + ((size_t)(base + bi * k + bj) * a.N + n) * a.C + cv * V, v);
        const float area = (float)((h1 - h0) * (w1 - w0));
#pragma unroll
        for (int j = 0; j < V; ++j) s[j] += v[j] / area;
      }
    }
    base += k * k;
  }
  T* dp = (T*)a.dx + pix * a.lddx + cv * V;
  if (a.accumulate) {
    float o[V];
    ldv(dp, o);
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] += o[j];
  }
  stv(dp, s);
}

int pyramid_pool_bwd(const PoolBwdArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  if (a.C % V || a.lddx % V) {
    set_error("pyramid_pool_bwd: C=%d lddx=%d", a.C, a.lddx);
    return E_UNSUPPORTED;
  }
  long long total = (long long)a.N * a.H * a.W * (a.C / V);
  unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) prof_launch(pyramid_pool_bwd_kernel<float>, grid, 256, 0, st, a);
  else if (dtype == DT_F16) prof_launch(pyramid_pool_bwd_kernel<f16>, grid, 256, 0, st, a);
  else prof_launch(pyramid_pool_bwd_kernel<bf16>, grid, 256, 0, st, a);
  return check_launch("pyramid_pool_bwd");
}

// ---- PPM feature upsampling: all 4 levels into the concat buffer in one launch --------------
// feats: bin-major [50][N][CF] (CF = 32); y: concat NHWC [N,H,W] with row stride ldy, level i
// written to channels [coff + i*CF, coff + (i+1)*CF).   (models/fast_scnn.py:139-143)

// one thread per (pixel, 16-B channel vector of one level): the two lerps once per 4 / 8 channels
template <typename T>
__global__ __launch_bounds__(256) void ppm_up_fwd_kernel(PpmUpArgs a) {
  constexpr int V = VecW<T>::V;
  long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int CTV = 4 * a.CF / V;
  long long total = (long long)a.N * a.H * a.W * CTV;
  if (t >= total) return;
  const int cc = (int)(t % CTV) * V;
  long long pix = t / CTV;
  int w = (int)(pix % a.W);
  long long r = pix / a.W;
  int h = (int)(r % a.H);
  int n = (int)(r / a.H);
  const int lv = cc / a.CF, c = cc - lv * a.CF;
  const int k = PP_LEVELS[lv];
  const int base = lv == 0 ? 0 : (lv == 1 ? 1 : (lv == 2 ? 5 : 14));
  Lerp lh = ac_lerp(h, k, a.H, ac_scale(k, a.H));
  Lerp lw = ac_lerp(w, k, a.W, ac_scale(k, a.W));
  const T* f = (const T*)a.feats;
  float q[4][V];
  ldv(f + ((size_t)(base + lh.i0 * k + lw.i0) * a.N + n) * a.CF + c, q[0]);
  ldv(f + ((size_t)(base + lh.i0 * k + lw.i1) * a.N + n) * a.CF + c, q[1]);
  ldv(f + ((size_t)(base + lh.i1 * k + lw.i0) * a.N + n) * a.CF + c, q[2]);
  ldv(f + ((size_t)(base + lh.i1 * k + lw.i1) * a.N + n) * a.CF + c, q[3]);
  float o[V];
#pragma unroll
  for (int j = 0; j < V; ++j)
    o[j] = lh.l0 * (lw.l0 * q[0][j] + lw.l1 * q[1][j]) + lh.l1 * (lw.l0 * q[2][j] + lw.l1 * q[3][j]);
  stv((T*)a.y + pix * a.ldy + a.coff + cc, o);
}

int ppm_up_fwd(const PpmUpArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  if (a.CF % V || a.ldy % V || a.coff % V) {
    set_error("ppm_up_fwd: CF=%d ldy=%d coff=%d", a.CF, a.ldy, a.coff);
    return E_UNSUPPORTED;
  }
  long long total = (long long)a.N * a.H * a.W * (4 * a.CF / V);
  unsigned grid = (unsigned)((total + 255) / 256);
  if (dtype == DT_F32) prof_launch(ppm_up_fwd_kernel<float>, grid, 256, 0, st, a);
  else if (dtype == DT_F16) prof_launch(ppm_up_fwd_kernel<f16>, grid, 256, 0, st, a);
  else prof_launch(ppm_up_fwd_kernel<bf16>, grid, 256, 0, st, a);
  return check_launch("ppm_up_fwd");
}

// backward: dfeats[bin][n][c] = sum_{h,w} wy(h,bi) wx(w,bj) dy[n,h,w,coff+lv*CF+c]  (gather)
// Separable, one workgroup per (level, image, 16-B channel vector -- r06: per (level, image) the
// 32 workgroups of cfg3 took 22.7 us): phase 1 reduces every row of the level's dy slice
// onto the k column bins (rows[h][bj][c] = sum_w wx(w,bj) dy[h,w,c]), phase 2 folds the rows onto
// the k row bins (one thread per (c, bin)), fixed order throughout.  Phase 1: a thread takes one
// 16-B channel vector of one row and the columns w = s, s + 8, ... of its segment s (8 segments on
// 8 adjacent lanes): its <= 8 vector loads per batch are all in flight at once (one memory round
// trip for W <= 64; 64 rows per pass), and the 8 segments' bin sums meet in a fixed xor butterfly.
constexpr int PPB_THREADS = 512;
constexpr int PPB_MAXH = 80;  // LDS rows[H][6][8] fp32
constexpr int PPB_SEG = 8;    // column segments (adjacent lanes)

template <typename T>
__global__ __launch_bounds__(PPB_THREADS) void ppm_up_bwd_kernel(PpmUpArgs a, void* dfeats) {
  constexpr int V = VecW<T>::V;
  __shared__ float rows[PPB_MAXH * 6 * 8];  // [h][bj][one channel vector]
  const int lv = blockIdx.x, n = blockIdx.y;
  const int k = PP_LEVELS[lv];
  const int base = lv == 0 ? 0 : (lv == 1 ? 1 : (lv == 2 ? 5 : 14));
  const float sh = ac_scale(k, a.H), sw = ac_scale(k, a.W);
  const int CF = a.CF;
  const int sg = threadIdx.x % PPB_SEG, rest = threadIdx.x / PPB_SEG;
  const int cv = blockIdx.z;  // this workgroup's 16-B channel vector
  constexpr int RP = PPB_THREADS / PPB_SEG;  // rows per pass
  const T* gp = (const T*)a.y + (size_t)n * a.H * a.W * a.ldy + a.coff + lv * CF + cv * V;
  // (the pass loop is uniform across the wave's 8-lane segment groups: RP rows per pass)
  for (int h0 = 0; h0 < a.H; h0 += RP) {
    const int h = h0 + rest;
    const bool hok = h < a.H;
    float acc[6][V];
#pragma unroll
    for (int bj = 0; bj < 6; ++bj)
#pragma unroll
      for (int e = 0; e < V; ++e) acc[bj][e] = 0.f;
    const T* gr = gp + (size_t)(hok ? h : 0) * a.W * a.ldy;
    for (int w0 = sg; w0 < a.W; w0 += 8 * PPB_SEG) {
      float v[8][V];
#pragma unroll
      for (int u = 0; u < 8; ++u) {  // all loads of the batch issued, then used
        const int w = w0 + u * PPB_SEG;
        ldv(gr + (size_t)(w < a.W ? w : 0) * a.ldy, v[u]);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int w = w0 + u * PPB_SEG;
        const bool ok = hok && w < a.W;
        const Lerp lw = ac_lerp(ok ? w : 0, k, a.W, sw);
#pragma unroll
        for (int bj = 0; bj < 6; ++bj) {
          const float wt = ok ? (lw.i0 == bj ? lw.l0 : 0.f) + (lw.i1 == bj ? lw.l1 : 0.f) : 0.f;
#pragma unroll
          for (int e = 0; e < V; ++e) acc[bj][e] = fmaf(wt, v[u][e], acc[bj][e]);
        }
      }
    }
#pragma unroll
    for (int bj = 0; bj < 6; ++bj)
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float t = acc[bj][e];
        t += __shfl_xor(t, 1);
        t += __shfl_xor(t, 2);
        t += __shfl_xor(t, 4);
        acc[bj][e] = t;
      }
    if (sg == 0 && hok) {
#pragma unroll
      for (int bj = 0; bj < 6; ++bj)
        if (bj < k) {
#pragma unroll
          for (int e = 0; e < V; ++e) rows[(h * 6 + bj) * 8 + e] = acc[bj][e];
        }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < k * k * V; t += PPB_THREADS) {
    const int e = t % V, bin = t / V, bi = bin / k, bj = bin - bi * k;
    float s = 0.f;
    for (int h = 0; h < a.H; ++h) {
      const Lerp lh = ac_lerp(h, k, a.H, sh);
      const float wy = (lh.i0 == bi ? lh.l0 : 0.f) + (lh.i1 == bi ? lh.l1 : 0.f);
      s += wy * rows[(h * 6 + bj) * 8 + e];
    }
    st1((T*)dfeats + ((size_t)(base + bin) * a.N + n) * CF + cv * V + e, s);
  }
}

int ppm_up_bwd(const PpmUpArgs& a, void* dfeats, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  // the row mapping hands rest / (CF / V) rows to a pass: CF / V must divide the 64 lanes
  if (a.CF <= 0 || a.CF > 32 || a.CF % V || a.ldy % V || a.coff % V || a.H > PPB_MAXH ||
      a.N > 65535) {
    set_error("ppm_up_bwd: CF=%d H=%d unsupported", a.CF, a.H);
    return E_UNSUPPORTED;
  }
  dim3 grid(4, a.N, a.CF / V);
  if (dtype == DT_F32) prof_launch(ppm_up_bwd_kernel<float>, grid, PPB_THREADS, 0, st, a, dfeats);
  else if (dtype == DT_F16) prof_launch(ppm_up_bwd_kernel<f16>, grid, PPB_THREADS, 0, st, a, dfeats);
  else prof_launch(ppm_up_bwd_kernel<bf16>, grid, PPB_THREADS, 0, st, a, dfeats);
  return check_launch("ppm_up_bwd");
}

}  // namespace fscnn
