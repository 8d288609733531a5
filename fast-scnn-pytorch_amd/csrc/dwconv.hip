// Depthwise 3x3 convolution, pad 1, stride 1 or 2, NHWC (models/fast_scnn.py:70 _DSConv,
// :86 _DWConv; LTD.dsconv1/2, the 9 bottleneck expansions, FFM.dwconv, classifier dsconvs —
// 14 layers).
//
// Workgroup = blockDim.x channel vectors (16 B: 4 fp32 / 8 bf16 channels) x blockDim.y column
// tiles.  Each thread owns a register tile of HS=2 output rows x WS=4 output columns of its
// channel vector: it streams the (HS-1)*s+3 input rows once, and every 16-B input vector it loads
// feeds all the taps of the tile that read it (stride 1: 24 loads for 8 outputs instead of 72).
// Lanes run along channels, so each wave-wide load is a run of contiguous 16-B vectors.
// Grids are 3-D (channel chunk, column tile, row band) — no 64-bit index division.
//
// dgrad, stride 1 = the same kernel with the 3x3 taps flipped (correlation of dy);
// dgrad, stride 2 = parity-aware gather (a 2x4 dx tile reads 2 dy rows x 3 dy columns).
// wgrad = per-block partial [part][9][C] sums, reduced by the deterministic two-pass reducer.
//
// Roofline: HBM-bound.  Algorithmic bytes per layer = e*(N*C*Hi*Wi + N*C*Ho*Wo) + 9*C*4,
// flops = 18*N*C*Ho*Wo.
#include "kernels.hpp"

namespace fscnn {

constexpr int DW_WS = 4;  // output columns per thread
constexpr int DW_HS = 2;  // output rows per thread

__host__ __device__ inline void dw_block_shape(int C, int V, int& bx, int& by) {
  int cv = C / V;
  bx = cv < 64 ? cv : 64;
  by = 256 / bx;
  if (by < 1) by = 1;
}

struct DwGeom {
  int gx, gy, gz;  // channel chunks, column tiles, row bands
};

// XCD-contiguous tile order (speed only): blocks L = x (mod 8) share an XCD, so residue class x
// gets the contiguous logical range [x*T/8, (x+1)*T/8) of (chunk, column tile, band) in
// chunk-fastest order — vertically adjacent bands then run on one XCD back to back and their
// shared halo rows are served by its L2 instead of being fetched from HBM twice.
__device__ __forceinline__ void dw_tile(int& cx, int& cy, int& cz) {
  const int gx = gridDim.x, gy = gridDim.y, gz = gridDim.z;
  const long long T = (long long)gx * gy * gz;
  long long L = blockIdx.x + (long long)gx * (blockIdx.y + (long long)gy * blockIdx.z);
  if ((T & 7) == 0) L = (L & 7) * (T >> 3) + (L >> 3);
  cx = (int)(L % gx);
  const long long r = L / gx;
  cy = (int)(r % gy);
  cz = (int)(r / gy);
}
static DwGeom dw_geom(int N, int Ho, int Wo, int C, int V) {
  int bx, by;
  dw_block_shape(C, V, bx, by);
  DwGeom g;
  g.gx = cdiv(C / V, bx);
  g.gy = cdiv(Wo, by * DW_WS);
  g.gz = N * cdiv(Ho, DW_HS);
  return g;
}

// ---- forward (and stride-1 dgrad with FLIP) -------------------------------------------------
template <typename T, int S, bool FLIP>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
  constexpr int V = VecW<T>::V;
  constexpr int NR = (DW_HS - 1) * S + 3;  // input rows touched
  constexpr int NC = (DW_WS - 1) * S + 3;  // input cols touched
  extern __shared__ float s_red[];         // [by][bx*V] (train statistics)
  __shared__ float s_cnt[256];
  const int tx = threadIdx.x, ty = threadIdx.y, BX = blockDim.x, BY = blockDim.y;
  int bx, by, bz;
  dw_tile(bx, by, bz);
  const int cv = bx * BX + tx;
  const int CV = a.C / V;
  const int nb = (a.Ho + DW_HS - 1) / DW_HS;
  const int n = bz / nb;
  const int ho0 = (bz - n * nb) * DW_HS;
  const int wo0 = (by * BY + ty) * DW_WS;
  const int nrow = min(DW_HS, a.Ho - ho0);
  const int ncol = wo0 < a.Wo ? min(DW_WS, a.Wo - wo0) : 0;
  const bool active = cv < CV && ncol > 0;

  float acc[DW_HS][DW_WS][V];
#pragma unroll
  for (int r = 0; r < DW_HS; ++r)
#pragma unroll
    for (int p = 0; p < DW_WS; ++p)
#pragma unroll
      for (int j = 0; j < V; ++j) acc[r][p][j] = 0.f;
  if (active) {
    float wt[9][V];
    const float* wp = a.w + (size_t)cv * V * 9;
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[FLIP ? 8 - t : t][j] = wp[j * 9 + t];
    const T* xb = (const T*)a.x + (size_t)n * a.H * a.W * a.C + (size_t)cv * V;
    const int hi0 = ho0 * S - 1, wi0 = wo0 * S - 1;
    // branch-free: out-of-image taps load a clamped in-bounds vector and are zeroed by select,
    // so the loads issue back to back (a branch around a load forces vmcnt(0) at the join)
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int hi = hi0 + rr;
      const bool rok = hi >= 0 && hi < a.H;
      const T* xr = xb + (size_t)(rok ? hi : 0) * a.W * a.C;
#pragma unroll
      for (int ci = 0; ci < NC; ++ci) {
        const int wi = wi0 + ci;
        const bool ok = rok && wi >= 0 && wi < a.W;
        float v[V];
        ldv(xr + (size_t)(ok ? wi : 0) * a.C, v);
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] = ok ? v[j] : 0.f;
#pragma unroll
        for (int r = 0; r < DW_HS; ++r) {
          const int kh = rr - r * S;
          if (kh < 0 || kh > 2) continue;
#pragma unroll
          for (int p = 0; p < DW_WS; ++p) {
            const int kw = ci - p * S;
            if (kw < 0 || kw > 2) continue;
#pragma unroll
            for (int j = 0; j < V; ++j) acc[r][p][j] = fmaf(v[j], wt[kh * 3 + kw][j], acc[r][p][j]);
          }
        }
      }
    }
    float sc[V], sh[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sc[j] = a.scale ? a.scale[cv * V + j] : 1.f;
      sh[j] = a.scale ? a.shift[cv * V + j] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < DW_HS; ++r) {
      if (r >= nrow) continue;
      T* yb = (T*)a.y + (((size_t)n * a.Ho + ho0 + r) * a.Wo + wo0) * a.C + (size_t)cv * V;
#pragma unroll
      for (int p = 0; p < DW_WS; ++p) {
        if (p >= ncol) continue;
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          float t = acc[r][p][j] * sc[j] + sh[j];
          o[j] = a.relu ? fmaxf(t, 0.f) : t;
          acc[r][p][j] = o[j];
        }
        stv(yb + (size_t)p * a.C, o);
      }
    }
  }
  if (a.part == nullptr) return;
  // ---- per-channel (mean, M2, count) over the block's outputs (train-mode BN statistics) -----
  const int npx = nrow * ncol;  // identical for every tx of this ty
#pragma unroll
  for (int j = 0; j < V; ++j) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < DW_HS; ++r)
#pragma unroll
      for (int p = 0; p < DW_WS; ++p) s += (r < nrow && p < ncol) ? acc[r][p][j] : 0.f;
    s_red[ty * BX * V + tx * V + j] = s;
  }
  s_cnt[ty] = (float)npx;
  __syncthreads();
  float cnt = 0.f, mean[V];
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
    for (int r = 0; r < DW_HS; ++r)
#pragma unroll
      for (int p = 0; p < DW_WS; ++p) {
        float d = acc[r][p][j] - mean[j];
        m2 += (r < nrow && p < ncol) ? d * d : 0.f;
      }
    s_red[ty * BX * V + tx * V + j] = m2;
  }
  __syncthreads();
  if (ty == 0 && cv < CV) {
    float* rec = a.part + ((size_t)bz * gridDim.y + by) * 3 * a.C;
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
  DwGeom g = dw_geom(N, Ho, Wo, C, dtype == DT_F32 ? 4 : 8);
  return g.gy * g.gz;
}

template <bool FLIP>
static int dw_launch_fwd(const DwArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  int bx, by;
  dw_block_shape(a.C, V, bx, by);
  DwGeom g = dw_geom(a.N, a.Ho, a.Wo, a.C, V);
  if (g.gz > 65535 || g.gy > 65535) {
    set_error("dw: grid too large (N*Ho/2=%d)", g.gz);
    return E_UNSUPPORTED;
  }
  dim3 grid(g.gx, g.gy, g.gz), block(bx, by);
  size_t shm = a.part ? (size_t)bx * by * V * sizeof(float) : 0;
  if (dtype == DT_F32) {
    if (a.stride == 1) dw_fwd_kernel<float, 1, FLIP><<<grid, block, shm, st>>>(a);
    else dw_fwd_kernel<float, 2, FLIP><<<grid, block, shm, st>>>(a);
  } else {
    if (a.stride == 1) dw_fwd_kernel<bf16, 1, FLIP><<<grid, block, shm, st>>>(a);
    else dw_fwd_kernel<bf16, 2, FLIP><<<grid, block, shm, st>>>(a);
  }
  return check_launch("dw_fwd");
}

int dw_fwd(const DwArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  if (a.C % V || (a.stride != 1 && a.stride != 2) || a.Ho != (a.H - 1) / a.stride + 1 ||
      a.Wo != (a.W - 1) / a.stride + 1) {
    set_error("dw_fwd: bad args C=%d stride=%d H=%d Ho=%d", a.C, a.stride, a.H, a.Ho);
    return E_INVALID;
  }
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_FWD, st, E * (in_el + out_el) + 36.0 * a.C, 18.0 * out_el);
  return dw_launch_fwd<false>(a, dtype, st);
}

// ---- input gradient ---------------------------------------------------------------------------
// dX[n,h,w,c] = sum_{kh,kw} dY[n,ho,wo,c] * w[c,kh,kw] with h = ho*s-1+kh, w = wo*s-1+kw.
// stride 2: a thread owns dx rows h0,h0+1 (h0 even) x cols w0..w0+3 (w0 even):
//   row h0   <- dy row h0/2 (kh=1);  row h0+1 <- dy rows h0/2+1 (kh=0) and h0/2 (kh=2)
//   col w0+q <- dy cols w0/2 + (q+1-kw)/2 for the kw of matching parity
template <typename T>
__global__ __launch_bounds__(256) void dw_dgrad_s2_kernel(DwBwdArgs a) {
  constexpr int V = VecW<T>::V;
  const int tx = threadIdx.x, ty = threadIdx.y, BX = blockDim.x, BY = blockDim.y;
  int bx, by, bz;
  dw_tile(bx, by, bz);
  const int cv = bx * BX + tx;
  const int CV = a.C / V;
  const int nb = (a.H + 1) / 2;
  const int n = bz / nb;
  const int h0 = (bz - n * nb) * 2;
  const int w0 = (by * BY + ty) * 4;
  if (cv >= CV || w0 >= a.W) return;
  float wt[9][V];
  const float* wp = a.w + (size_t)cv * V * 9;
#pragma unroll
  for (int j = 0; j < V; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t][j] = wp[j * 9 + t];
  float acc[2][4][V];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < V; ++j) acc[r][q][j] = 0.f;
  const T* gb = (const T*)a.dy + (size_t)n * a.Ho * a.Wo * a.C + (size_t)cv * V;
  const int hb = h0 / 2, wb = w0 / 2;
#pragma unroll
  for (int dr = 0; dr < 2; ++dr) {       // dy rows hb, hb+1
    const int ho = hb + dr;
#pragma unroll
    for (int dc = 0; dc < 3; ++dc) {     // dy cols wb, wb+1, wb+2
      const int wo = wb + dc;
      const bool ok = ho < a.Ho && wo < a.Wo;  // branch-free clamped load + select
      float g[V];
      ldv(gb + (ok ? (size_t)ho * a.Wo + wo : 0) * a.C, g);
#pragma unroll
      for (int j = 0; j < V; ++j) g[j] = ok ? g[j] : 0.f;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        // dx row h0+r reads dy row ho with kh = (h0 + r) + 1 - 2*ho
        const int kh = r + 1 - 2 * dr;
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kw = q + 1 - 2 * dc;
          if (kw < 0 || kw > 2) continue;
#pragma unroll
          for (int j = 0; j < V; ++j) acc[r][q][j] = fmaf(g[j], wt[kh * 3 + kw][j], acc[r][q][j]);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (h0 + r >= a.H) continue;
    T* db = (T*)a.dx + (((size_t)n * a.H + h0 + r) * a.W + w0) * a.C + (size_t)cv * V;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (w0 + q < a.W) stv(db + (size_t)q * a.C, acc[r][q]);
  }
}

int dw_dgrad(const DwBwdArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_DGRAD, st, E * (in_el + out_el) + 36.0 * a.C, 18.0 * out_el);
  if (a.stride == 1) {
    // correlation of dy with the flipped taps, same geometry as the forward
    DwArgs f{};
    f.N = a.N; f.H = a.Ho; f.W = a.Wo; f.C = a.C; f.Ho = a.H; f.Wo = a.W; f.stride = 1;
    f.x = a.dy; f.w = a.w; f.y = a.dx;
    return dw_launch_fwd<true>(f, dtype, st);
  }
  int bx, by;
  dw_block_shape(a.C, V, bx, by);
  dim3 grid(cdiv(a.C / V, bx), cdiv(a.W, by * 4), a.N * ((a.H + 1) / 2)), block(bx, by);
  if (dtype == DT_F32) dw_dgrad_s2_kernel<float><<<grid, block, 0, st>>>(a);
  else dw_dgrad_s2_kernel<bf16><<<grid, block, 0, st>>>(a);
  return check_launch("dw_dgrad");
}

// ---- weight gradient: per-block partial [part][9][C] -----------------------------------------
// Blocks walk (row band, column tile) pairs grid-stride so the partial count stays bounded.
template <typename T, int S>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(DwBwdArgs a, int gy, int gz) {
  constexpr int V = VecW<T>::V;
  constexpr int NR = (DW_HS - 1) * S + 3;
  constexpr int NC = (DW_WS - 1) * S + 3;
  extern __shared__ float s_red[];  // [BY][BX*V]
  const int tx = threadIdx.x, ty = threadIdx.y, BX = blockDim.x, BY = blockDim.y;
  const int cv = blockIdx.x * BX + tx;
  const int CV = a.C / V;
  const int nb = (a.Ho + DW_HS - 1) / DW_HS;
  float acc[9][V];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[t][j] = 0.f;
  // part p walks the contiguous tile range [p*T/P, (p+1)*T/P): consecutive bands, so the halo
  // rows it re-reads are its own recent loads (L1/L2 hits)
  const int ntiles = gy * gz;
  const int t_lo = (int)((long long)ntiles * blockIdx.y / gridDim.y);
  const int t_hi = (int)((long long)ntiles * (blockIdx.y + 1) / gridDim.y);
  for (int tile = t_lo; cv < CV && tile < t_hi; ++tile) {
    const int tz = tile / gy, tyy = tile - tz * gy;
    const int n = tz / nb;
    const int ho0 = (tz - n * nb) * DW_HS;
    const int wo0 = (tyy * BY + ty) * DW_WS;
    if (wo0 >= a.Wo) continue;
    const int nrow = min(DW_HS, a.Ho - ho0), ncol = min(DW_WS, a.Wo - wo0);
    // dy tile (unpacked once) and the input rows as raw 16-B vectors, double-buffered: row rr+1's
    // loads are in flight while row rr is consumed.  Clamped addresses + selects, no branches.
    float g[DW_HS][DW_WS][V];
    const T* gb = (const T*)a.dy + (((size_t)n * a.Ho + ho0) * a.Wo + wo0) * a.C + (size_t)cv * V;
    {
      uint4 graw[DW_HS][DW_WS];
#pragma unroll
      for (int r = 0; r < DW_HS; ++r)
#pragma unroll
        for (int p = 0; p < DW_WS; ++p) {
          const bool ok = r < nrow && p < ncol;
          graw[r][p] = sel4(ok, *reinterpret_cast<const uint4*>(gb + (ok ? (size_t)r * a.Wo + p : 0) * a.C));
        }
#pragma unroll
      for (int r = 0; r < DW_HS; ++r)
#pragma unroll
        for (int p = 0; p < DW_WS; ++p) unpackv(graw[r][p], g[r][p]);
    }
    const T* xb = (const T*)a.x + (size_t)n * a.H * a.W * a.C + (size_t)cv * V;
    const int hi0 = ho0 * S - 1, wi0 = wo0 * S - 1;
    uint4 xrow[2][NC];
    auto load_row = [&](int rr, uint4 (&dst)[NC]) {
      const int hi = hi0 + rr;
      const bool rok = hi >= 0 && hi < a.H;
      const T* xr = xb + (size_t)(rok ? hi : 0) * a.W * a.C;
#pragma unroll
      for (int ci = 0; ci < NC; ++ci) {
        const int wi = wi0 + ci;
        const bool ok = rok && wi >= 0 && wi < a.W;
        dst[ci] = sel4(ok, *reinterpret_cast<const uint4*>(xr + (size_t)(ok ? wi : 0) * a.C));
      }
    };
    load_row(0, xrow[0]);
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      if (rr + 1 < NR) load_row(rr + 1, xrow[(rr + 1) & 1]);
#pragma unroll
      for (int ci = 0; ci < NC; ++ci) {
        float v[V];
        unpackv(xrow[rr & 1][ci], v);
#pragma unroll
        for (int r = 0; r < DW_HS; ++r) {
          const int kh = rr - r * S;
          if (kh < 0 || kh > 2) continue;
#pragma unroll
          for (int p = 0; p < DW_WS; ++p) {
            const int kw = ci - p * S;
            if (kw < 0 || kw > 2) continue;
#pragma unroll
            for (int j = 0; j < V; ++j)
              acc[kh * 3 + kw][j] = fmaf(v[j], g[r][p][j], acc[kh * 3 + kw][j]);
          }
        }
      }
    }
  }
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
  DwGeom g = dw_geom(N, Ho, Wo, C, dtype == DT_F32 ? 4 : 8);
  long long tiles = (long long)g.gy * g.gz;
  long long cap = 2048 / g.gx;
  if (cap < 1) cap = 1;
  return (int)(tiles < cap ? tiles : cap);
}

int dw_wgrad(const DwBwdArgs& a, int dtype, hipStream_t st) {
  int V = dtype == DT_F32 ? 4 : 8;
  int bx, by;
  dw_block_shape(a.C, V, bx, by);
  DwGeom g = dw_geom(a.N, a.Ho, a.Wo, a.C, V);
  dim3 grid(g.gx, dw_wgrad_parts(a.N, a.Ho, a.Wo, a.C, dtype));
  dim3 block(bx, by);
  size_t shm = (size_t)bx * by * V * sizeof(float);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_WGRAD, st, E * (in_el + out_el), 18.0 * out_el);
  if (dtype == DT_F32) {
    if (a.stride == 1) dw_wgrad_kernel<float, 1><<<grid, block, shm, st>>>(a, g.gy, g.gz);
    else dw_wgrad_kernel<float, 2><<<grid, block, shm, st>>>(a, g.gy, g.gz);
  } else {
    if (a.stride == 1) dw_wgrad_kernel<bf16, 1><<<grid, block, shm, st>>>(a, g.gy, g.gz);
    else dw_wgrad_kernel<bf16, 2><<<grid, block, shm, st>>>(a, g.gy, g.gz);
  }
  return check_launch("dw_wgrad");
}

// slab [P][9][C] -> dW [C][9] (native PyTorch [C,1,3,3] layout): two-pass fixed-order reduction
int dw_wgrad_reduce(float* slab, int P, int C, float* dw, hipStream_t st) {
  return reduce_slabs_ex(slab, P, 9LL * C, 9LL * C, dw, 0, C, st);
}

}  // namespace fscnn
