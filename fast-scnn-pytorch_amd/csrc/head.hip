// Fused training head: the final F.interpolate(bilinear, align_corners=True) of the logits
// (models/fast_scnn.py:40) + nn.CrossEntropyLoss(ignore_index=-1) (utils/loss.py:103-124) and
// its gradient back to the LOW-resolution logits, in one pass that never writes full-resolution
// logits (8 x 19 x 1024 x 2048 would be 637 MB bf16 written, read, re-written and re-read by the
// unfused path).
//
// Deterministic gather: workgroup (n, hb, wb) OWNS low-res cells [hb*TH, +TH) x [wb*TW, +TW) of
// image n.  It walks every full-res pixel whose bilinear stencil touches one of its cells
// (its support, a 1-cell halo), recomputes the interpolated logits and the softmax there, keeps
// the per-pixel gradient (softmax - onehot) of a pass in LDS, and each (cell, class) accumulator
// is owned by exactly one thread that sums its contributions in a fixed order.  A pixel's loss is
// counted by the workgroup that owns its (i0(h), i0(w)) cell, so every pixel counts once.
#include "kernels.hpp"

namespace fscnn {

constexpr int HD_TH = 4;     // owned low-res rows per workgroup
constexpr int HD_TW = 14;    // owned low-res cols per workgroup (row support <= 128 px at x8)
constexpr int HD_CMAX = 32;  // max classes
constexpr int HD_GS = HD_CMAX + 1;

__device__ __forceinline__ int hd_first_ge(int i, int Lin, int Lout, float sc) {
  int lo = 0, hi = Lout;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (ac_lerp(mid, Lin, Lout, sc).i0 >= i) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

template <typename T>
__global__ __launch_bounds__(256) void ce_head_kernel(CeHeadArgs a) {
  __shared__ float s_g[256 * HD_GS];              // per-pixel gradients of the current pass
  __shared__ float s_acc[HD_TH * HD_TW * HD_CMAX];  // owned (cell, class) accumulators
  __shared__ int s_wi0[256];
  __shared__ float s_wl0[256], s_wl1[256];
  __shared__ int s_wlo[HD_TW], s_whi[HD_TW];
  __shared__ float s_r1[256], s_r2[256];
  const int tid = threadIdx.x;
  const int n = blockIdx.z;
  const int hi0 = blockIdx.y * HD_TH, wi0 = blockIdx.x * HD_TW;
  const int nth = min(HD_TH, a.Hl - hi0), ntw = min(HD_TW, a.Wl - wi0);
  const int C = a.C;
  const float sh = ac_scale(a.Hl, a.H), sw = ac_scale(a.Wl, a.W);
  const int h_lo = hd_first_ge(hi0 - 1, a.Hl, a.H, sh), h_hi = hd_first_ge(hi0 + nth, a.Hl, a.H, sh);
  const int w_lo = hd_first_ge(wi0 - 1, a.Wl, a.W, sw), w_hi = hd_first_ge(wi0 + ntw, a.Wl, a.W, sw);
  if (tid < ntw) {
    s_wlo[tid] = hd_first_ge(wi0 + tid - 1, a.Wl, a.W, sw);
    s_whi[tid] = hd_first_ge(wi0 + tid + 1, a.Wl, a.W, sw);
  }
  for (int i = tid; i < HD_TH * HD_TW * HD_CMAX; i += 256) s_acc[i] = 0.f;
  const int npx_row = w_hi - w_lo;
  const int cw = npx_row <= 256 ? npx_row : 256;  // pixels per row per pass
  const int R = npx_row <= 256 ? max(1, 256 / max(1, npx_row)) : 1;
  const T* lg = (const T*)a.logits + (size_t)n * a.Hl * a.Wl * a.ldl;
  float loss = 0.f, cnt = 0.f;
  __syncthreads();
  for (int h0 = h_lo; h0 < h_hi; h0 += R) {
    for (int wc = w_lo; wc < w_hi; wc += cw) {
      const int ncw = min(cw, w_hi - wc);
      // ---- pass 1: gradient of each pixel of R rows x ncw cols ----------------------------
      {
        const int r = tid / max(1, cw), px = tid - r * cw;
        const int h = h0 + r, w = wc + px;
        if (r < R && h < h_hi && px < ncw) {
          Lerp lh = ac_lerp(h, a.Hl, a.H, sh);
          Lerp lw = ac_lerp(w, a.Wl, a.W, sw);
          if (r == 0) {
            s_wi0[px] = lw.i0;
            s_wl0[px] = lw.l0;
            s_wl1[px] = lw.l1;
          }
          const T* q00 = lg + ((size_t)lh.i0 * a.Wl + lw.i0) * a.ldl;
          const T* q01 = lg + ((size_t)lh.i0 * a.Wl + lw.i1) * a.ldl;
          const T* q10 = lg + ((size_t)lh.i1 * a.Wl + lw.i0) * a.ldl;
          const T* q11 = lg + ((size_t)lh.i1 * a.Wl + lw.i1) * a.ldl;
          float* gp = &s_g[(r * cw + px) * HD_GS];
          float mx = -INFINITY;
          for (int c = 0; c < C; ++c) {
            float l = lh.l0 * (lw.l0 * ld1(q00 + c) + lw.l1 * ld1(q01 + c)) +
                      lh.l1 * (lw.l0 * ld1(q10 + c) + lw.l1 * ld1(q11 + c));
            gp[c] = l;
            mx = fmaxf(mx, l);
          }
          const long long t = a.target[((size_t)n * a.H + h) * a.W + w];
          const bool valid = t != a.ignore_index && t >= 0 && t < C;
          float se = 0.f;
          for (int c = 0; c < C; ++c) se += expf(gp[c] - mx);
          const float inv = 1.f / se;
          const bool own = lh.i0 >= hi0 && lh.i0 < hi0 + nth && lw.i0 >= wi0 && lw.i0 < wi0 + ntw;
          if (valid && own) {
            loss += mx + logf(se) - gp[(int)t];
            cnt += 1.f;
          }
          for (int c = 0; c < C; ++c) {
            float p = expf(gp[c] - mx) * inv;
            gp[c] = valid ? p - (c == (int)t ? 1.f : 0.f) : 0.f;
          }
        }
      }
      __syncthreads();
      // ---- pass 2: every owned (cell column j, class c) gathers its contributions ---------
      for (int idx = tid; idx < ntw * C; idx += 256) {
        const int j = idx / C, c = idx - j * C;
        const int wi = wi0 + j;
        const int a0 = max(s_wlo[j], wc), a1 = min(s_whi[j], wc + ncw);
        for (int r = 0; r < R; ++r) {
          const int h = h0 + r;
          if (h >= h_hi) break;
          float s = 0.f;
          for (int w = a0; w < a1; ++w) {
            const int p = w - wc;
            const int i0 = s_wi0[p];
            const int i1 = i0 + (i0 < a.Wl - 1 ? 1 : 0);
            const float wx = (i0 == wi ? s_wl0[p] : 0.f) + (i1 == wi ? s_wl1[p] : 0.f);
            s += wx * s_g[(r * cw + p) * HD_GS + c];
          }
          Lerp lh = ac_lerp(h, a.Hl, a.H, sh);
          if (lh.i0 >= hi0 && lh.i0 < hi0 + nth)
            s_acc[((lh.i0 - hi0) * HD_TW + j) * HD_CMAX + c] += lh.l0 * s;
          if (lh.i1 != lh.i0 && lh.i1 >= hi0 && lh.i1 < hi0 + nth)
            s_acc[((lh.i1 - hi0) * HD_TW + j) * HD_CMAX + c] += lh.l1 * s;
        }
      }
      __syncthreads();
    }
  }
  for (int idx = tid; idx < nth * ntw * C; idx += 256) {
    const int c = idx % C, rj = idx / C;
    const int r = rj / ntw, j = rj - r * ntw;
    a.g_raw[(((size_t)n * a.Hl + hi0 + r) * a.Wl + wi0 + j) * a.ldl + c] =
        s_acc[(r * HD_TW + j) * HD_CMAX + c];
  }
  s_r1[tid] = loss;
  s_r2[tid] = cnt;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (tid < off) {
      s_r1[tid] += s_r1[tid + off];
      s_r2[tid] += s_r2[tid + off];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const size_t pi = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    a.part[2 * pi] = s_r1[0];
    a.part[2 * pi + 1] = s_r2[0];
  }
}

int ce_head_parts(int N, int Hl, int Wl) { return N * cdiv(Hl, HD_TH) * cdiv(Wl, HD_TW); }

__global__ __launch_bounds__(256) void ce_head_finalize_kernel(const float* part, int P, float* out) {
  __shared__ double r1[256], r2[256];
  double s1 = 0.0, s2 = 0.0;
  for (int p = threadIdx.x; p < P; p += 256) {
    s1 += part[2 * p];
    s2 += part[2 * p + 1];
  }
  r1[threadIdx.x] = s1;
  r2[threadIdx.x] = s2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      r1[threadIdx.x] += r1[threadIdx.x + off];
      r2[threadIdx.x] += r2[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = r2[0] > 0 ? (float)(r1[0] / r2[0]) : NAN;
    out[1] = (float)r2[0];
  }
}

int ce_head(const CeHeadArgs& a, float* out2, int dtype, hipStream_t st) {
  if (a.C < 1 || a.C > HD_CMAX) {
    set_error("ce_head: %d classes (max %d)", a.C, HD_CMAX);
    return E_UNSUPPORTED;
  }
  dim3 grid(cdiv(a.Wl, HD_TW), cdiv(a.Hl, HD_TH), a.N);
  {
    ProfScope ps(PK_CE, st, (dtype == DT_F32 ? 4.0 : 2.0) * a.N * a.Hl * a.Wl * a.ldl * 1.3 +
                                8.0 * a.N * a.H * a.W + 4.0 * a.N * a.Hl * a.Wl * a.ldl,
                 0.0);
    if (dtype == DT_F32) ce_head_kernel<float><<<grid, 256, 0, st>>>(a);
    else ce_head_kernel<bf16><<<grid, 256, 0, st>>>(a);
    int rc = check_launch("ce_head");
    if (rc) return rc;
  }
  ce_head_finalize_kernel<<<1, 256, 0, st>>>(a.part, ce_head_parts(a.N, a.Hl, a.Wl), out2);
  return check_launch("ce_head_finalize");
}

template <typename T>
__global__ __launch_bounds__(256) void ce_head_scale_kernel(const float* g_raw, T* g, int M, int C,
                                                            int ld, const float* gout,
                                                            const float* out2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * ld) return;
  const int c = i % ld;
  const float s = gout[0] / out2[1];
  st1(g + i, c < C ? g_raw[i] * s : 0.f);
}

int ce_head_scale(const float* g_raw, void* g, long long M, int C, int ld, const float* gout,
                  const float* out2, int dtype, hipStream_t st) {
  const int total = (int)(M * ld);
  if (dtype == DT_F32)
    ce_head_scale_kernel<float><<<cdiv(total, 256), 256, 0, st>>>(g_raw, (float*)g, (int)M, C, ld, gout, out2);
  else
    ce_head_scale_kernel<bf16><<<cdiv(total, 256), 256, 0, st>>>(g_raw, (bf16*)g, (int)M, C, ld, gout, out2);
  return check_launch("ce_head_scale");
}

}  // namespace fscnn
