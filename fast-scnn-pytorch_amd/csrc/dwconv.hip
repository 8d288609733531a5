// Depthwise 3x3 convolution, pad 1, stride 1 or 2, NHWC (models/fast_scnn.py:70 _DSConv,
// :86 _DWConv; used by LTD.dsconv1/2, the 9 bottleneck expansions, FFM.dwconv and the
// classifier dsconvs — 14 layers).
//
// Workgroup = blockDim.x channel vectors (16 B each: 4 fp32 / 8 bf16 channels) x blockDim.y
// output strips; a strip is WS consecutive output pixels of one row.  Lanes run along the
// channel vectors, so every load/store of a wave is a run of contiguous 16 B vectors.  The
// WS-wide strip reuses each loaded input column for up to 3 (s=1) taps in registers; the 3x
// vertical reuse is served by L1/L2 since neighbouring rows are processed by neighbouring
// workgroups at the same time.
//
// Roofline: HBM-bound.  Algorithmic bytes per layer = e*(N*C*Hi*Wi + N*C*Ho*Wo) + 9*C*4,
// flops = 18*N*C*Ho*Wo.
#include "kernels.hpp"

namespace fscnn {


constexpr int DW_WS = 4;

__host__ __device__ inline void dw_block_shape(int C, int V, int& bx, int& by) {
  int cv = C / V;
  bx = cv < 64 ? cv : 64;
  by = 256 / bx;
  if (by < 1) by = 1;
}

template <typename T, int S>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
  constexpr int V = VecW<T>::V;
  constexpr int NIN = (DW_WS - 1) * S + 3;  // input columns touched by a strip
  extern __shared__ float s_red[];          // [blockDim.y][blockDim.x*V]
  const int cv = blockIdx.x * blockDim.x + threadIdx.x;
  const int CV = a.C / V;
  const int nstrip_w = (a.Wo + DW_WS - 1) / DW_WS;
  const long long strip = (long long)blockIdx.y * blockDim.y + threadIdx.y;
  const long long nstrips = (long long)a.N * a.Ho * nstrip_w;
  const bool active = (cv < CV) && (strip < nstrips);

  float acc[DW_WS][V];
#pragma unroll
  for (int p = 0; p < DW_WS; ++p)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[p][j] = 0.f;
  int n = 0, ho = 0, wo0 = 0;
  if (active) {
    int ws = (int)(strip % nstrip_w);
    long long r = strip / nstrip_w;
    ho = (int)(r % a.Ho);
    n = (int)(r / a.Ho);
    wo0 = ws * DW_WS;
    // taps: w[c][kh][kw] for this thread's V channels (9*V contiguous floats)
    float wt[9][V];
    const float* wp = a.w + (size_t)cv * V * 9;
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[t][j] = wp[j * 9 + t];
    const T* xb = (const T*)a.x + (size_t)n * a.H * a.W * a.C + (size_t)cv * V;
    const int wi0 = wo0 * S - 1;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      int hi = ho * S - 1 + kh;
      if (hi < 0 || hi >= a.H) continue;
      const T* xr = xb + (size_t)hi * a.W * a.C;
#pragma unroll
      for (int ci = 0; ci < NIN; ++ci) {
        int wi = wi0 + ci;
        if (wi < 0 || wi >= a.W) continue;
        float v[V];
        ldv(xr + (size_t)wi * a.C, v);
#pragma unroll
        for (int p = 0; p < DW_WS; ++p) {
          int kw = ci - p * S;
          if (kw >= 0 && kw < 3) {
#pragma unroll
            for (int j = 0; j < V; ++j) acc[p][j] = fmaf(v[j], wt[kh * 3 + kw][j], acc[p][j]);
          }
        }
      }
    }
  }
  const int npx_strip = active ? min(DW_WS, a.Wo - wo0) : 0;
  if (active) {
    float sc[V], sh[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sc[j] = a.scale ? a.scale[cv * V + j] : 1.f;
      sh[j] = a.scale ? a.shift[cv * V + j] : 0.f;
    }
    T* yb = (T*)a.y + (((size_t)n * a.Ho + ho) * a.Wo + wo0) * a.C + (size_t)cv * V;
#pragma unroll
    for (int p = 0; p < DW_WS; ++p) {
      if (p < npx_strip) {
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          float t = acc[p][j] * sc[j] + sh[j];
          o[j] = a.relu ? fmaxf(t, 0.f) : t;
          acc[p][j] = o[j];
        }
        stv(yb + (size_t)p * a.C, o);
      }
    }
  }
  if (a.part == nullptr) return;
  // ---- per-channel (mean, M2, count) over the block's pixels (train-mode BN statistics) ----
  const int BX = blockDim.x, BY = blockDim.y;
  const int tx = threadIdx.x, ty = threadIdx.y;
  float s[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    s[j] = 0.f;
#pragma unroll
    for (int p = 0; p < DW_WS; ++p) s[j] += (p < npx_strip) ? acc[p][j] : 0.f;
    s_red[ty * BX * V + tx * V + j] = s[j];
  }
  __shared__ float s_cnt[256];
  // pixels of this strip, independent of whether this thread's channel vector exists (all tx of a
  // row write the same value — no race between active and padding threads)
  int strip_px = 0;
  if (strip < nstrips) {
    int ws_ = (int)(strip % nstrip_w);
    strip_px = min(DW_WS, a.Wo - ws_ * DW_WS);
  }
  s_cnt[ty] = (float)strip_px;
  __syncthreads();
  float cnt = 0.f;
  float mean[V];
#pragma unroll
  for (int j = 0; j < V; ++j) mean[j] = 0.f;
  for (int k = 0; k < BY; ++k) {
    cnt += s_cnt[k];
#pragma unroll
    for (int j = 0; j < V; ++j) mean[j] += s_red[k * BX * V + tx * V + j];
  }
#pragma unroll
  for (int j = 0; j < V; ++j) mean[j] = cnt > 0.f ? mean[j] / cnt : 0.f;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < V; ++j) {
    float m2 = 0.f;
#pragma unroll
    for (int p = 0; p < DW_WS; ++p) {
      float d = acc[p][j] - mean[j];
      m2 += (p < npx_strip) ? d * d : 0.f;
    }
    s_red[ty * BX * V + tx * V + j] = m2;
  }
  __syncthreads();
  if (ty == 0 && cv < CV) {
    float* rec = a.part + (size_t)blockIdx.y * 3 * a.C;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float m2 = 0.f;
      for (int k = 0; k < BY; ++k) m2 += s_red[k * BX * V + tx * V + j];
      rec[cv * V + j] = mean[j];
      rec[a.C + cv * V + j] = m2;
      rec[2 * a.C + cv * V + j] = cnt;
    }
  }
}

int dw_parts(int N, int Ho, int Wo, int C, int dtype) {
  int V = dtype == DT_F32 ? 4 : 8, bx, by;
  dw_block_shape(C, V, bx, by);
  long long nstrips = (long long)N * Ho * cdiv(Wo, DW_WS);
  return (int)((nstrips + by - 1) / by);
}

int dw_fwd(const DwArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  if (a.C % V || (a.stride != 1 && a.stride != 2) || a.Ho != (a.H - 1) / a.stride + 1 ||
      a.Wo != (a.W - 1) / a.stride + 1) {
    set_error("dw_fwd: bad args C=%d stride=%d H=%d Ho=%d", a.C, a.stride, a.H, a.Ho);
    return E_INVALID;
  }
  int bx, by;
  dw_block_shape(a.C, V, bx, by);
  long long nstrips = (long long)a.N * a.Ho * cdiv(a.Wo, DW_WS);
  dim3 grid(cdiv(a.C / V, bx), (unsigned)((nstrips + by - 1) / by));
  dim3 block(bx, by);
  size_t shm = a.part ? (size_t)bx * by * V * sizeof(float) : 0;
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_FWD, st, E * (in_el + out_el) + 36.0 * a.C, 18.0 * out_el);
  if (dtype == DT_F32) {
    if (a.stride == 1) dw_fwd_kernel<float, 1><<<grid, block, shm, st>>>(a);
    else dw_fwd_kernel<float, 2><<<grid, block, shm, st>>>(a);
  } else {
    if (a.stride == 1) dw_fwd_kernel<bf16, 1><<<grid, block, shm, st>>>(a);
    else dw_fwd_kernel<bf16, 2><<<grid, block, shm, st>>>(a);
  }
  return check_launch("dw_fwd");
}

// ---- input gradient (gather form, no atomics) ----------------------------------------------
// dX[n,h,w,c] = sum_{kh,kw} dY[n,ho,wo,c] * w[c,kh,kw] with h = ho*s-1+kh, w = wo*s-1+kw.

template <typename T, int S>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(DwBwdArgs a) {
  constexpr int V = VecW<T>::V;
  const int CV = a.C / V;
  long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long total = (long long)a.N * a.H * a.W * CV;
  if (idx >= total) return;
  int cv = (int)(idx % CV);
  long long pix = idx / CV;
  int wi = (int)(pix % a.W);
  long long r = pix / a.W;
  int hi = (int)(r % a.H);
  int n = (int)(r / a.H);
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  const float* wp = a.w + (size_t)cv * V * 9;
  const T* dyb = (const T*)a.dy + (size_t)n * a.Ho * a.Wo * a.C + (size_t)cv * V;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    int hn = hi + 1 - kh;
    if (hn < 0 || (S == 2 && (hn & 1))) continue;
    int ho = hn / S;
    if (ho >= a.Ho) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      int wn = wi + 1 - kw;
      if (wn < 0 || (S == 2 && (wn & 1))) continue;
      int wo = wn / S;
      if (wo >= a.Wo) continue;
      float v[V];
      ldv(dyb + ((size_t)ho * a.Wo + wo) * a.C, v);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] = fmaf(v[j], wp[j * 9 + kh * 3 + kw], acc[j]);
    }
  }
  stv((T*)a.dx + (size_t)pix * a.C + (size_t)cv * V, acc);
}

int dw_dgrad(const DwBwdArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  long long total = (long long)a.N * a.H * a.W * (a.C / V);
  dim3 grid((unsigned)((total + 255) / 256));
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_DGRAD, st, E * (in_el + out_el) + 36.0 * a.C, 18.0 * out_el);
  if (dtype == DT_F32) {
    if (a.stride == 1) dw_dgrad_kernel<float, 1><<<grid, 256, 0, st>>>(a);
    else dw_dgrad_kernel<float, 2><<<grid, 256, 0, st>>>(a);
  } else {
    if (a.stride == 1) dw_dgrad_kernel<bf16, 1><<<grid, 256, 0, st>>>(a);
    else dw_dgrad_kernel<bf16, 2><<<grid, 256, 0, st>>>(a);
  }
  return check_launch("dw_dgrad");
}

// ---- weight gradient: per-block partial [part][9][C], reduced deterministically later --------
template <typename T, int S>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(DwBwdArgs a) {
  constexpr int V = VecW<T>::V;
  extern __shared__ float s_red[];  // [BY][BX*V]
  const int cv = blockIdx.x * blockDim.x + threadIdx.x;
  const int CV = a.C / V;
  const int nstrip_w = (a.Wo + DW_WS - 1) / DW_WS;
  const long long nstrips = (long long)a.N * a.Ho * nstrip_w;
  float acc[9][V];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[t][j] = 0.f;
  // grid-stride over strips: the number of partial records is gridDim.y (bounded), not the
  // number of strips, so the final fixed-order reduction stays short.
  for (long long strip = (long long)blockIdx.y * blockDim.y + threadIdx.y;
       cv < CV && strip < nstrips; strip += (long long)gridDim.y * blockDim.y) {
    int ws = (int)(strip % nstrip_w);
    long long r = strip / nstrip_w;
    int ho = (int)(r % a.Ho);
    int n = (int)(r / a.Ho);
    int wo0 = ws * DW_WS;
    int npx = min(DW_WS, a.Wo - wo0);
    float g[DW_WS][V];
    const T* dyb = (const T*)a.dy + (((size_t)n * a.Ho + ho) * a.Wo + wo0) * a.C + (size_t)cv * V;
#pragma unroll
    for (int p = 0; p < DW_WS; ++p) {
      if (p < npx) ldv(dyb + (size_t)p * a.C, g[p]);
      else {
#pragma unroll
        for (int j = 0; j < V; ++j) g[p][j] = 0.f;
      }
    }
    constexpr int NIN = (DW_WS - 1) * S + 3;
    const T* xb = (const T*)a.x + (size_t)n * a.H * a.W * a.C + (size_t)cv * V;
    const int wi0 = wo0 * S - 1;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      int hi = ho * S - 1 + kh;
      if (hi < 0 || hi >= a.H) continue;
      const T* xr = xb + (size_t)hi * a.W * a.C;
#pragma unroll
      for (int ci = 0; ci < NIN; ++ci) {
        int wi = wi0 + ci;
        if (wi < 0 || wi >= a.W) continue;
        float v[V];
        ldv(xr + (size_t)wi * a.C, v);
#pragma unroll
        for (int p = 0; p < DW_WS; ++p) {
          int kw = ci - p * S;
          if (kw >= 0 && kw < 3) {
#pragma unroll
            for (int j = 0; j < V; ++j) acc[kh * 3 + kw][j] = fmaf(v[j], g[p][j], acc[kh * 3 + kw][j]);
          }
        }
      }
    }
  }
  const int BX = blockDim.x, BY = blockDim.y, tx = threadIdx.x, ty = threadIdx.y;
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int j = 0; j < V; ++j) s_red[ty * BX * V + tx * V + j] = acc[t][j];
    __syncthreads();
    if (ty == 0 && cv < CV) {
      float* rec = a.slab + ((size_t)blockIdx.y * 9 + t) * a.C;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float s = 0.f;
        for (int k = 0; k < BY; ++k) s += s_red[k * BX * V + tx * V + j];
        rec[cv * V + j] = s;
      }
    }
    __syncthreads();
  }
}

int dw_wgrad_parts(int N, int Ho, int Wo, int C, int dtype) {
  int V = dtype == DT_F32 ? 4 : 8, bx, by;
  dw_block_shape(C, V, bx, by);
  long long nstrips = (long long)N * Ho * cdiv(Wo, DW_WS);
  long long gy = (nstrips + by - 1) / by;
  int gx = cdiv(C / V, bx);
  long long cap = 2048 / gx;
  if (cap < 1) cap = 1;
  return (int)(gy < cap ? gy : cap);
}

int dw_wgrad(const DwBwdArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  int bx, by;
  dw_block_shape(a.C, V, bx, by);
  dim3 grid(cdiv(a.C / V, bx), dw_wgrad_parts(a.N, a.Ho, a.Wo, a.C, dtype));
  dim3 block(bx, by);
  size_t shm = (size_t)bx * by * V * sizeof(float);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_WGRAD, st, E * (in_el + out_el), 18.0 * out_el);
  if (dtype == DT_F32) {
    if (a.stride == 1) dw_wgrad_kernel<float, 1><<<grid, block, shm, st>>>(a);
    else dw_wgrad_kernel<float, 2><<<grid, block, shm, st>>>(a);
  } else {
    if (a.stride == 1) dw_wgrad_kernel<bf16, 1><<<grid, block, shm, st>>>(a);
    else dw_wgrad_kernel<bf16, 2><<<grid, block, shm, st>>>(a);
  }
  return check_launch("dw_wgrad");
}

// slab [P][9][C] -> dW [C][9] (native PyTorch [C,1,3,3] layout), fixed-order sum over P
__global__ void dw_wgrad_reduce_kernel(const float* slab, int P, int C, float* dw) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 9 * C) return;
  int t = i / C, c = i - t * C;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += slab[((size_t)p * 9 + t) * C + c];
  dw[c * 9 + t] = s;
}

int dw_wgrad_reduce(const float* slab, int P, int C, float* dw, hipStream_t st) {
  dw_wgrad_reduce_kernel<<<cdiv(9 * C, 256), 256, 0, st>>>(slab, P, C, dw);
  return check_launch("dw_wgrad_reduce");
}

}  // namespace fscnn
