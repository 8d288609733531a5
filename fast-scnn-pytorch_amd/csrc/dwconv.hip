// Depthwise 3x3 convolution, pad 1, stride 1 or 2, NHWC (models/fast_scnn.py:70 _DSConv,
// :86 _DWConv; LTD.dsconv1/2, the 9 bottleneck expansions, FFM.dwconv, classifier dsconvs —
// 14 layers).
//
// LDS-tiled: a workgroup owns cbv <= 8 channel vectors (16 B: 4 fp32 / 8 bf16 channels) of a
// spatial output tile (stride 1: 8 rows x 32 cols, stride 2: 4 x 16).  It loads the haloed input
// tile ONCE, in one batch of branch-free 16-B loads (clamped addresses + selects: a branch
// around a load makes hipcc wait vmcnt(0) at the join), into LDS; each thread then computes an
// HS x WS block of outputs for its channel vector from LDS.  Row halo 10/8 (s1) instead of the
// 2x of a per-thread register tile, one round trip per tile, ~150 VGPRs (occupancy 3).
// Tiles are mapped XCD-contiguously (dw_tile) so neighbouring tiles share an XCD's L2.
//
// dgrad, stride 1 = the same kernel with the 3x3 taps flipped (correlation of dy);
// dgrad, stride 2 = parity-aware gather (a 2x4 dx tile reads 2 dy rows x 3 dy columns).
// wgrad = same tiles; a workgroup walks tpb tiles along a row band, accumulates 9 x V taps per
// thread, reduces its 32 pixel groups in fixed order -> partial [part][9][C] (two-pass reducer).
//
// Roofline: HBM-bound.  Algorithmic bytes per layer = e*(N*C*Hi*Wi + N*C*Ho*Wo) + 9*C*4,
// flops = 18*N*C*Ho*Wo.
#include "bn_finish.hpp"

#include <optional>

namespace fscnn {

constexpr int DWL_CB = 8;  // max 16-B channel vectors per workgroup (128 B per pixel; 4 measured
                           // r04: 6.12-6.13 vs 6.02-6.06 ms per cfg3 step)

// A thread computes a channel QUAD (4 channels: 16 B fp32 / 8 B bf16 of LDS per read) for an
// HS x WS block of outputs; G = 32 / (quads per vector) pixel groups of GX x GY cover the tile.
template <typename T, int S> struct DwCfg;
template <> struct DwCfg<float, 1> { static constexpr int HS = 2, WS = 4, GX = 8, GY = 4; };
template <> struct DwCfg<float, 2> { static constexpr int HS = 1, WS = 2, GX = 8, GY = 4; };
template <> struct DwCfg<bf16, 1> { static constexpr int HS = 2, WS = 4, GX = 4, GY = 4; };
template <> struct DwCfg<bf16, 2> { static constexpr int HS = 2, WS = 2, GX = 4, GY = 4; };
template <int S> struct DwCfg<f16, S> : DwCfg<bf16, S> {};
template <typename T, int S> struct DwTile {
  static constexpr int HS = DwCfg<T, S>::HS, WS = DwCfg<T, S>::WS;
  static constexpr int GX = DwCfg<T, S>::GX, GY = DwCfg<T, S>::GY, G = GX * GY;
  static constexpr int QPV = VecW<T>::V / 4;                 // quads per 16-B vector
  static constexpr int TH = GY * HS, TW = GX * WS;           // output tile
  static constexpr int IR = (TH - 1) * S + 3, IC = (TW - 1) * S + 3;  // input tile
  static constexpr int LPT = (IR * IC + QPV * G - 1) / (QPV * G);     // 16-B loads per thread
  static constexpr int NR = (HS - 1) * S + 3, NC = (WS - 1) * S + 3;  // per-thread input window
};

// 4 channels (a quad) from LDS / registers
__device__ __forceinline__ void quad_ld(const float* p, float (&v)[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
__device__ __forceinline__ void quad_ld(const bf16* p, float (&v)[4]) {
  const uint2 t = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xFFFF0000u);
  v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xFFFF0000u);
}
__device__ __forceinline__ void quad_ld(const f16* p, float (&v)[4]) { ld4v(p, v); }
__device__ __forceinline__ void quad_st(f16* p, const float (&v)[4]) { st4v(p, v); }
__device__ __forceinline__ void quad_st(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void quad_st(bf16* p, const float (&v)[4]) {
  const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
}

// channel vectors per workgroup: the largest divisor of C/V that is <= 8
static int dw_cbv(int CV) {
  for (int b = DWL_CB; b > 1; --b)
    if (CV % b == 0) return b;
  return 1;
}

// XCD-contiguous tile order (speed only): blocks L = x (mod 8) share an XCD, so residue class x
// gets the contiguous logical range [x*T/8, (x+1)*T/8) of (chunk, column tile, band) in
// chunk-fastest order — neighbouring tiles then run on one XCD back to back and their shared
// halo rows are served by its L2.
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

// stage the haloed input tile [IR][IC][cbv] (16-B vectors) of image n into LDS; out-of-image
// positions are zero.  All loads of a thread are issued before any LDS store.
// IT: x is the raw conv output z of a BatchNorm+ReLU that is never stored (train); the staged
// value is relu(fmaf(z, isc[c], ish[c])) (bn_apply's arithmetic), padding stays zero.  A thread's
// vectors all belong to one channel vector (lv = tid % cbv), so its V pairs are loaded once.
template <typename T, int S, bool IT>
__device__ __forceinline__ void dw_stage(uint4* s_in, const T* x, int H, int W, int C, int n,
                                         int hi0, int wi0, int cvbase, int cbv, int tid, int nthr,
                                         const float* isc, const float* ish) {
  using G = DwTile<T, S>;
  constexpr int V = VecW<T>::V;
  float sc[IT ? V : 1], sh[IT ? V : 1];
  if constexpr (IT) {
    const int cb = (cvbase + tid % cbv) * V;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      sc[j] = isc[cb + j];
      sh[j] = ish[cb + j];
    }
  }
  uint4 raw[G::LPT];
#pragma unroll
  for (int k = 0; k < G::LPT; ++k) {
    const int i = tid + k * nthr;
    const int pix = i / cbv, lv = i - pix * cbv;
    const int r = pix / G::IC, col = pix - r * G::IC;
    const int hi = hi0 + r, wi = wi0 + col;
    const bool ok = pix < G::IR * G::IC && hi >= 0 && hi < H && wi >= 0 && wi < W;
    const size_t off = ok ? (((size_t)n * H + hi) * W + wi) * C + (size_t)(cvbase + lv) * V : 0;
    raw[k] = sel4(ok, *reinterpret_cast<const uint4*>(x + off));
  }
#pragma unroll
  for (int k = 0; k < G::LPT; ++k) {
    const int i = tid + k * nthr;
    if (i < G::IR * G::IC * cbv) {
      uint4 v = raw[k];
      if constexpr (IT) {
        const int pix = i / cbv;
        const int r = pix / G::IC, col = pix - r * G::IC;
        const int hi = hi0 + r, wi = wi0 + col;
        const bool ok = hi >= 0 && hi < H && wi >= 0 && wi < W;
        v = sel4(ok, bnrelu_vec<T>(v, sc, sh));
      }
      s_in[i] = v;
    }
  }
}

// ---- forward (and stride-1 dgrad with FLIP) -------------------------------------------------
// TL: the launch finishes its BN in the last workgroups (a.tail_ink; a separate instantiation so
// the other launches keep their register budget)
template <typename T, int S, bool FLIP, bool IT, bool BR = false, bool TL = false>
__global__ __launch_bounds__(256, 3) void dw_fwd_kernel(DwArgs a, int cbv) {
  using G = DwTile<T, S>;
  // LDS sized per launch (dw_shm): the staged tile of cbv channel vectors + the reduction rows
  extern __shared__ __attribute__((aligned(16))) uint4 s_dyn[];
  uint4* s_in = s_dyn;
  float* s_red = reinterpret_cast<float*>(s_dyn + G::IR * G::IC * cbv);
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int QB = cbv * G::QPV;                 // quads per workgroup
  const int q = tid % QB, grp = tid / QB;
  const int gx = grp % G::GX, gy = grp / G::GX;
  int bx, by, bz;
  dw_tile(bx, by, bz);
  const int tiles_h = cdiv(a.Ho, G::TH);
  const int n = bz / tiles_h;
  const int th0 = (bz - n * tiles_h) * G::TH, tw0 = by * G::TW;
  const int c0 = bx * cbv * VecW<T>::V + q * 4;  // first channel of the thread's quad
  stamp(a.stamps, 0);
  dw_stage<T, S, IT>(s_in, (const T*)a.x, a.H, a.W, a.C, n, th0 * S - 1, tw0 * S - 1,
                     bx * cbv, cbv, tid, nthr, a.in_scale, a.in_shift);
  float wt[9][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[FLIP ? 8 - t : t][j] = a.w[(size_t)(c0 + j) * 9 + t];
  __syncthreads();
  stamp(a.stamps, 1);

  const T* sl = reinterpret_cast<const T*>(s_in);
  const int pstride = cbv * VecW<T>::V;          // elements per staged pixel
  float acc[G::HS][G::WS][4];
#pragma unroll
  for (int r = 0; r < G::HS; ++r)
#pragma unroll
    for (int p = 0; p < G::WS; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[r][p][j] = 0.f;
  const int lr0 = gy * G::HS * S, lc0 = gx * G::WS * S;
#pragma unroll
  for (int rr = 0; rr < G::NR; ++rr) {
    // one input row of the thread's window at a time: left to itself the compiler hoists all
    // NR x NC quad loads (up to 96 live values) and the kernel drops to 3 waves per SIMD
    asm volatile("" ::: "memory");
#pragma unroll
    for (int ci = 0; ci < G::NC; ++ci) {
      float v[4];
      quad_ld(sl + ((lr0 + rr) * G::IC + lc0 + ci) * pstride + q * 4, v);
#pragma unroll
      for (int r = 0; r < G::HS; ++r) {
        const int kh = rr - r * S;
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int p = 0; p < G::WS; ++p) {
          const int kw = ci - p * S;
          if (kw < 0 || kw > 2) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[r][p][j] = fmaf(v[j], wt[kh * 3 + kw][j], acc[r][p][j]);
        }
      }
    }
  }

  const int ho0 = th0 + gy * G::HS, wo0 = tw0 + gx * G::WS;
  const int nrow = max(0, min(G::HS, a.Ho - ho0)), ncol = max(0, min(G::WS, a.Wo - wo0));
  {
    float sc[4], sh[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sc[j] = a.scale ? a.scale[c0 + j] : 1.f;
      sh[j] = a.scale ? a.shift[c0 + j] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < G::HS; ++r) {
      if (r >= nrow) continue;
      T* yb = (T*)a.y + (((size_t)n * a.Ho + ho0 + r) * a.Wo + wo0) * a.C + c0;
#pragma unroll
      for (int p = 0; p < G::WS; ++p) {
        if (p >= ncol) continue;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = acc[r][p][j] * sc[j] + sh[j];
          o[j] = a.relu ? fmaxf(t, 0.f) : t;
          acc[r][p][j] = round_as<T>(o[j]);  // (the statistics below: of the stored value)
        }
        quad_st(yb + (size_t)p * a.C, o);
      }
    }
  }
  stamp(a.stamps, 2);
  if constexpr (BR) {
    // ---- stride-1 dgrad: BN-backward partial sums of the stored dx (it is that BN's dy) -----
    const BnBwdPart& b = a.bs;
    const bool m2 = b.mode == 2;
    float bm[4], bi[4], bsc[4], bsh[4], s1[4], s2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bm[j] = b.mean[c0 + j];
      bi[j] = b.invstd[c0 + j];
      bsc[j] = m2 ? b.scale[c0 + j] : 0.f;  // mode 0: mask fmaf(z, 0, 1) > 0 always
      bsh[j] = m2 ? b.shift[c0 + j] : 1.f;
      s1[j] = s2[j] = 0.f;
    }
#pragma unroll
    for (int r = 0; r < G::HS; ++r) {
      float z[G::WS][4];  // one output row of z per batch of loads
#pragma unroll
      for (int p = 0; p < G::WS; ++p) {
        const bool ok = r < nrow && p < ncol;
        const size_t pix = ok ? ((size_t)n * a.Ho + ho0 + r) * a.Wo + wo0 + p : 0;
        quad_ld((const T*)b.z + pix * a.C + c0, z[p]);
      }
#pragma unroll
      for (int p = 0; p < G::WS; ++p) {
        const bool ok = r < nrow && p < ncol;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float gv = round_as<T>(acc[r][p][j]);
          gv = (ok && fmaf(z[p][j], bsc[j], bsh[j]) > 0.f) ? gv : 0.f;
          s1[j] += gv;
          s2[j] += gv * (z[p][j] - bm[j]) * bi[j];
        }
      }
      asm volatile("" ::: "memory");  // next row's z loads after this row's use
    }
    // the G pixel groups in fixed order, one record per workgroup
    float* rec = b.part + ((size_t)bz * gridDim.y + by) * 2 * a.C;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) s_red[(grp * QB + q) * 4 + j] = pass ? s2[j] : s1[j];
      __syncthreads();
      if (grp == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float t = 0.f;
          for (int g2 = 0; g2 < G::G; ++g2) t += s_red[(g2 * QB + q) * 4 + j];
          st_wt(rec + (size_t)pass * a.C + c0 + j, t);
        }
      }
    }
    stamp(a.stamps, 3);
    if constexpr (TL)
      tail_finish<false>(b.part, gridDim.y * gridDim.z, a.C, bz * gridDim.y + by,
                         bx * cbv * VecW<T>::V, cbv * VecW<T>::V, bx, a.tail,
                         reinterpret_cast<double*>(s_dyn));
    stamp(a.stamps, 4);
    return;
  }
  if (a.part == nullptr) return;
  // ---- per-channel (mean, M2, count) over the tile (train-mode BN statistics of the values as
  // stored: the BN normalises the rounded z, as the reference's autocast BN does) --------------
  const int trows = min(G::TH, a.Ho - th0), tcols = min(G::TW, a.Wo - tw0);
  const float cnt = (float)(trows * tcols);
  float mean[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < G::HS; ++r)
#pragma unroll
      for (int p = 0; p < G::WS; ++p) sum += (r < nrow && p < ncol) ? acc[r][p][j] : 0.f;
    s_red[(grp * QB + q) * 4 + j] = sum;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float sum = 0.f;
    for (int g = 0; g < G::G; ++g) sum += s_red[(g * QB + q) * 4 + j];
    mean[j] = sum / cnt;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float m2 = 0.f;
#pragma unroll
    for (int r = 0; r < G::HS; ++r)
#pragma unroll
      for (int p = 0; p < G::WS; ++p) {
        const float d = acc[r][p][j] - mean[j];
        m2 += (r < nrow && p < ncol) ? d * d : 0.f;
      }
    s_red[(grp * QB + q) * 4 + j] = m2;
  }
  __syncthreads();
  if (grp == 0) {
    float* rec = a.part + ((size_t)bz * gridDim.y + by) * 3 * a.C;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m2 = 0.f;
      for (int g = 0; g < G::G; ++g) m2 += s_red[(g * QB + q) * 4 + j];
      st_wt(rec + c0 + j, mean[j]);
      st_wt(rec + a.C + c0 + j, m2);
      st_wt(rec + 2 * a.C + c0 + j, cnt);
    }
  }
  stamp(a.stamps, 3);
  if constexpr (TL)
    tail_finish<true>(a.part, gridDim.y * gridDim.z, a.C, bz * gridDim.y + by,
                      bx * cbv * VecW<T>::V, cbv * VecW<T>::V, bx, a.tail,
                      reinterpret_cast<double*>(s_dyn));
  stamp(a.stamps, 4);
}

// dynamic LDS of the tile kernels: the haloed input tile of cbv vectors + 4 floats per thread
template <typename T, int S>
static size_t dw_shm(int cbv) {
  using G = DwTile<T, S>;
  return (size_t)G::IR * G::IC * cbv * 16 + (size_t)cbv * 32 * 16;
}

// one workgroup per (channel chunk, tile).  (A streaming tile-loop forward -- every workgroup
// resident, the next tile's loads in flight during the current tile's compute -- measured r04
// 6.20 vs 6.04 ms per cfg3 step: at <= 2 workgroups per CU one tile of prefetch hid less HBM
// latency than this kernel's occupancy does; removed in r05.)
static dim3 dw_grid(int N, int Ho, int Wo, int C, int V, int S, int& cbv) {
  cbv = dw_cbv(C / V);
  int TH, TW;
  if (V == 4) {
    TH = S == 1 ? DwTile<float, 1>::TH : DwTile<float, 2>::TH;
    TW = S == 1 ? DwTile<float, 1>::TW : DwTile<float, 2>::TW;
  } else {
    TH = S == 1 ? DwTile<bf16, 1>::TH : DwTile<bf16, 2>::TH;
    TW = S == 1 ? DwTile<bf16, 1>::TW : DwTile<bf16, 2>::TW;
  }
  return dim3(C / V / cbv, cdiv(Wo, TW), N * cdiv(Ho, TH));
}

int dw_parts(int N, int Ho, int Wo, int C, int dtype, int stride) {
  int cbv;
  dim3 g = dw_grid(N, Ho, Wo, C, dtype == DT_F32 ? 4 : 8, stride, cbv);
  return (int)(g.y * g.z);
}

template <typename T, bool FLIP, bool IT, bool BR>
static void dw_launch_fwd_t(const DwArgs& a, dim3 grid, int nthr, int cbv, hipStream_t st) {
  if constexpr (BR) {  // stride-1 dgrad with BN-backward partials
    if (a.tail_ink) prof_launch(dw_fwd_kernel<T, 1, true, false, true, true>, grid, nthr, dw_shm<T, 1>(cbv), st, a, cbv);
    else prof_launch(dw_fwd_kernel<T, 1, true, false, true>, grid, nthr, dw_shm<T, 1>(cbv), st, a, cbv);
    return;
  }
  if (!FLIP && a.tail_ink) {  // train forward with the in-kernel BN finish
    if (a.stride == 1) prof_launch(dw_fwd_kernel<T, 1, false, IT, false, true>, grid, nthr, dw_shm<T, 1>(cbv), st, a, cbv);
    else prof_launch(dw_fwd_kernel<T, 2, false, IT, false, true>, grid, nthr, dw_shm<T, 2>(cbv), st, a, cbv);
    return;
  }
  if (a.stride == 1) prof_launch(dw_fwd_kernel<T, 1, FLIP, IT>, grid, nthr, dw_shm<T, 1>(cbv), st, a, cbv);
  else prof_launch(dw_fwd_kernel<T, 2, FLIP, IT>, grid, nthr, dw_shm<T, 2>(cbv), st, a, cbv);
}

template <bool FLIP, bool IT, bool BR = false>
static int dw_launch_fwd(const DwArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  int cbv;
  dim3 grid = dw_grid(a.N, a.Ho, a.Wo, a.C, V, a.stride, cbv);
  if (grid.z > 65535 || grid.y > 65535) {
    set_error("dw: grid too large (%u x %u)", grid.y, grid.z);
    return E_UNSUPPORTED;
  }
  const int nthr = cbv * 32;  // = quads * groups for both dtypes
  DwArgs as = a;
  as.stamps = stamp_region();
  if (dtype == DT_F32) dw_launch_fwd_t<float, FLIP, IT, BR>(as, grid, nthr, cbv, st);
  else if (dtype == DT_F16) dw_launch_fwd_t<f16, FLIP, IT, BR>(as, grid, nthr, cbv, st);
  else dw_launch_fwd_t<bf16, FLIP, IT, BR>(as, grid, nthr, cbv, st);
  return check_launch(FLIP ? "dw_dgrad" : "dw_fwd");
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
  // (closed before a separate finalize launch: profiler scopes do not nest)
  std::optional<ProfScope> ps;
  ps.emplace(PK_DW_FWD, st, E * (in_el + out_el) + 36.0 * a.C, 18.0 * out_el);
  if (a.in_scale && !a.in_shift) {
    set_error("dw_fwd: in_scale without in_shift");
    return E_INVALID;
  }
  DwArgs b = a;
  int P = 0;
  if (a.part && a.tail.counters) {  // BN finish: in the kernel when the records fit its counters
    int cbv;
    const dim3 g = dw_grid(a.N, a.Ho, a.Wo, a.C, V, a.stride, cbv);
    P = (int)(g.y * g.z);
    b.tail_ink = a.tail.tsum && a.C <= TAIL_CMAX && tail_fits(P, (int)g.x);
  }
  const int rc = a.in_scale ? dw_launch_fwd<false, true>(b, dtype, st) : dw_launch_fwd<false, false>(b, dtype, st);
  if (rc || !a.part || !a.tail.counters || b.tail_ink) return rc;
  ps.reset();
  BnFinalizeArgs f = a.tail.fwd;
  f.part = a.part; f.P = P; f.C = a.C; f.counters = a.tail.counters;
  return bn_finalize(f, st);
}

static void dw_block_shape(int C, int V, int& bx, int& by) {
  int cv = C / V;
  bx = cv;  // channel vectors per workgroup row: all of them, or the largest divisor <= 64
  if (bx > 64) {
    bx = 64;
    while (cv % bx) --bx;
  }
  by = 256 / bx;
  if (by < 1) by = 1;
}

// ---- input gradient ---------------------------------------------------------------------------
// dX[n,h,w,c] = sum_{kh,kw} dY[n,ho,wo,c] * w[c,kh,kw] with h = ho*s-1+kh, w = wo*s-1+kw.
// stride 2: a thread owns dx rows h0,h0+1 (h0 even) x cols w0..w0+3 (w0 even) of 4 channels:
//   row h0   <- dy row h0/2 (kh=1);  row h0+1 <- dy rows h0/2+1 (kh=0) and h0/2 (kh=2)
//   col w0+q <- dy cols w0/2 + (q+1-kw)/2 for the kw of matching parity
// Four channels per thread (one 8-B vector of 16-bit data, 16 B of fp32) keep the live set near
// 100 VGPRs, so 4+ waves per SIMD hide the HBM latency; with BR (this dx is the dy of a
// BatchNorm whose backward partials the launch also emits) that BN's z loads are issued together
// with the dy loads, before any arithmetic, so the two latencies overlap.  (Measured at cfg3,
// bf16: bottleneck1.0 147 us, bottleneck2.0 56 us, against 183 / 86 us for 8 channels per thread
// and 200 / 79 us for a one-column walker over 8 rows with the taps staged in LDS.)
constexpr int DWD2_V = 4;  // channels per thread
template <typename T, bool BR, bool TL = false>
__global__ __launch_bounds__(256) void dw_dgrad_s2_kernel(DwBwdArgs a, int rpw) {
  constexpr int V = DWD2_V;
  const int tx = threadIdx.x, ty = threadIdx.y, BX = blockDim.x, BY = blockDim.y;
  int bx, by, bzg;
  dw_tile(bx, by, bzg);
  const int cv = bx * BX + tx;
  const int CV = a.C / V;
  const int nb = (a.H + 1) / 2;
  const int w0 = (by * BY + ty) * 4;
  const bool active = cv < CV && w0 < a.W;
  if (!BR && !active) return;  // (BR: every thread joins the workgroup reduction)
  const int cvc = active ? cv : 0;
  const int cb = cvc * V;
  __shared__ float s_bc[4][64 * V];  // BR: mean, invstd, mask scale, mask shift of the channels
  if constexpr (BR) {
    const BnBwdPart& b = a.bs;
    const bool m2 = b.mode == 2;
    const int c0b = bx * BX * V;
    for (int i = ty * BX + tx; i < BX * V; i += BX * BY) {
      const int c = min(c0b + i, a.C - 1);
      s_bc[0][i] = b.mean[c];
      s_bc[1][i] = b.invstd[c];
      s_bc[2][i] = m2 ? b.scale[c] : 0.f;  // mode 0: mask fmaf(z, 0, 1) > 0 always
      s_bc[3][i] = m2 ? b.shift[c] : 1.f;
    }
    __syncthreads();
  }
  float wt[9][V];
  const float4* wp = reinterpret_cast<const float4*>(a.w + (size_t)cb * 9);  // 36 floats, 16-B aligned
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float4 t4 = wp[i];
    const float tt[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int f = 4 * i + e;  // = j * 9 + tap
      wt[f % 9][f / 9] = tt[e];
    }
  }
  float s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) s1[j] = s2[j] = 0.f;
  // rpw consecutive row pairs per workgroup (one BN record for all of them: P stays within the
  // in-kernel finish's reach)
  for (int k = 0; k < rpw; ++k) {
    const int bz = bzg * rpw + k;
    if (bz >= a.N * nb) break;  // (workgroup-uniform)
    const int n = bz / nb;
    const int h0 = (bz - n * nb) * 2;
    // ---- every global load of the thread first: dy (2 x 3 vectors), BR: z (2 x 4) -----------
    const T* gb = (const T*)a.dy + (size_t)n * a.Ho * a.Wo * a.C + cb;
    const int hb = h0 / 2, wb = w0 / 2;
    float g[2][3][V];
#pragma unroll
    for (int dr = 0; dr < 2; ++dr)
#pragma unroll
      for (int dc = 0; dc < 3; ++dc) {
        const int ho = hb + dr, wo = wb + dc;
        const bool ok = active && ho < a.Ho && wo < a.Wo;  // branch-free clamped load + select
        ld4v(gb + (ok ? (size_t)ho * a.Wo + wo : 0) * a.C, g[dr][dc]);
#pragma unroll
        for (int j = 0; j < V; ++j) g[dr][dc][j] = ok ? g[dr][dc][j] : 0.f;
      }
    float z[BR ? 2 : 1][BR ? 4 : 1][V];
    if constexpr (BR) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = active && h0 + r < a.H && w0 + q < a.W;
          const size_t pix = ok ? ((size_t)n * a.H + h0 + r) * a.W + w0 + q : 0;
          ld4v((const T*)a.bs.z + pix * a.C + cb, z[r][q]);
        }
    }
    float acc[2][4][V];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < V; ++j) acc[r][q][j] = 0.f;
#pragma unroll
    for (int dr = 0; dr < 2; ++dr)
#pragma unroll
      for (int dc = 0; dc < 3; ++dc)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          // dx row h0+r reads dy row hb+dr with kh = (h0 + r) + 1 - 2*(hb+dr)
          const int kh = r + 1 - 2 * dr;
          if (kh < 0 || kh > 2) continue;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int kw = q + 1 - 2 * dc;
            if (kw < 0 || kw > 2) continue;
#pragma unroll
            for (int j = 0; j < V; ++j) acc[r][q][j] = fmaf(g[dr][dc][j], wt[kh * 3 + kw][j], acc[r][q][j]);
          }
        }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!active || h0 + r >= a.H) continue;
      T* db = (T*)a.dx + (((size_t)n * a.H + h0 + r) * a.W + w0) * a.C + cb;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (w0 + q < a.W) st4v(db + (size_t)q * a.C, acc[r][q]);
    }
    if constexpr (BR) {
      // BN-backward partial sums of the stored dx (the dy of that BN)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool ok = active && h0 + r < a.H && w0 + q < a.W;
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const int cl = tx * V + j;
            float gv = round_as<T>(acc[r][q][j]);
            gv = (ok && fmaf(z[r][q][j], s_bc[2][cl], s_bc[3][cl]) > 0.f) ? gv : 0.f;
            s1[j] += gv;
            s2[j] += gv * (z[r][q][j] - s_bc[0][cl]) * s_bc[1][cl];
          }
        }
    }
  }
  if constexpr (BR) {
    // ---- one record per workgroup: the BY column groups of a channel quad summed in fixed order
    __shared__ float s_br[256 * 2 * V];
    const BnBwdPart& b = a.bs;
    const int t = ty * BX + tx;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      s_br[t * 2 * V + j] = s1[j];
      s_br[t * 2 * V + V + j] = s2[j];
    }
    __syncthreads();
    // every thread sums whole (channel, s1|s2) columns over the BY column groups (fixed order):
    // a single row of reducers would walk BY = 64 rows alone for C = 32
    float* rec = b.part + ((size_t)bzg * gridDim.y + by) * 2 * a.C;
    for (int col = t; col < BX * 2 * V; col += BX * BY) {
      const int x = col / (2 * V), j2 = col - x * 2 * V;
      if (bx * BX + x >= CV) continue;
      float sum = 0.f;
      for (int y = 0; y < BY; ++y) sum += s_br[(y * BX + x) * 2 * V + j2];
      st_wt(rec + (j2 < V ? 0 : a.C) + (size_t)(bx * BX + x) * V + (j2 < V ? j2 : j2 - V), sum);
    }
    if constexpr (TL)
      tail_finish<false>(b.part, gridDim.y * gridDim.z, a.C, bzg * gridDim.y + by, bx * BX * V,
                         min(BX * V, a.C - bx * BX * V), bx, a.tail,
                         reinterpret_cast<double*>(s_br));  // (>= 3 x 256 doubles)
  }
}

// row pairs per workgroup of the stride-2 dgrad: the fewest that keep its BN records
// (grid.y x row-pair groups) at <= 2048 (bottleneck1.0: 13,312 -> 1,664 records, so the
// fold+finalize launch reads 5 MB instead of 41 MB)
static int dwd2_rpw(int gy, int NB) {
  int rpw = 1;
  while ((long long)gy * cdiv(NB, rpw) > 2048 && rpw < NB) ++rpw;
  return rpw;
}

int dw_dgrad(const DwBwdArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  const bool br = a.bs.part != nullptr;  // + a read of the next BN's z (dx-sized)
  std::optional<ProfScope> ps;  // (closed before a separate finalize launch)
  ps.emplace(PK_DW_DGRAD, st, E * (in_el * (br ? 2 : 1) + out_el) + 36.0 * a.C, 18.0 * out_el);
  if (a.C % V || (a.stride != 1 && a.stride != 2)) {
    set_error("dw_dgrad: bad args C=%d stride=%d", a.C, a.stride);
    return E_INVALID;
  }
  if (a.stride == 2 && (uintptr_t)a.w % 16) {
    set_error("dw_dgrad: weights must be 16-B aligned");
    return E_INVALID;
  }
  if (br && (!a.bs.z || !a.bs.mean || !a.bs.invstd || (a.bs.mode == 2 && (!a.bs.scale || !a.bs.shift)))) {
    set_error("dw_dgrad: inconsistent BN-backward partial arguments");
    return E_INVALID;
  }
  const bool fin = br && a.tail.counters;  // finish the bs.part BN (in the kernel when it fits)
  int P = 0, rc;
  bool ink = false;
  if (a.stride == 1) {
    // correlation of dy with the flipped taps, same geometry as the forward
    DwArgs f{};
    f.N = a.N; f.H = a.Ho; f.W = a.Wo; f.C = a.C; f.Ho = a.H; f.Wo = a.W; f.stride = 1;
    f.x = a.dy; f.w = a.w; f.y = a.dx;
    f.bs = a.bs;
    if (fin) {
      int cbv;
      const dim3 g = dw_grid(a.N, a.H, a.W, a.C, V, 1, cbv);
      P = (int)(g.y * g.z);
      ink = a.tail.tsum && a.C <= TAIL_CMAX && tail_fits(P, (int)g.x);
      f.tail = a.tail;
      f.tail_ink = ink;
    }
    rc = br ? dw_launch_fwd<true, false, true>(f, dtype, st) : dw_launch_fwd<true, false>(f, dtype, st);
  } else {
    int bx, by;
    dw_block_shape(a.C, DWD2_V, bx, by);
    const int gy = cdiv(a.W, by * 4), NB = a.N * ((a.H + 1) / 2);
    const int rpw = dwd2_rpw(gy, NB);
    dim3 grid(cdiv(a.C / DWD2_V, bx), gy, cdiv(NB, rpw)), block(bx, by);
    DwBwdArgs b = a;
    // its BN finish as the separate fold+finalize launch: measured 10-15 us per step faster than
    // the in-kernel finish at these record counts (the last arriver's fold sits on the tail)
    if (fin) P = (int)(grid.y * grid.z);
#define DWD2(T)                                                                 \
  do {                                                                          \
    if (br) prof_launch(dw_dgrad_s2_kernel<T, true>, grid, block, 0, st, b, rpw);              \
    else prof_launch(dw_dgrad_s2_kernel<T, false>, grid, block, 0, st, b, rpw);               \
  } while (0)
    if (dtype == DT_F32) DWD2(float);
    else if (dtype == DT_F16) DWD2(f16);
    else DWD2(bf16);
#undef DWD2
    rc = check_launch("dw_dgrad");
  }
  if (rc || !fin || ink) return rc;
  ps.reset();
  return bn_bwd_finalize(a.bs.part, P, a.C, a.tail.count, a.tail.dgamma, a.tail.dbeta,
                         a.tail.coef, st, a.tail.counters, a.tail.tab);
}

// workgroups of the dgrad launch = its BnBwdPart record count (H, W: dx = the dw's input)
int dw_dgrad_parts(int N, int H, int W, int C, int dtype, int stride) {
  const int V = dtype == DT_F32 ? 4 : 8;
  if (stride == 1) {
    int cbv;
    const dim3 g = dw_grid(N, H, W, C, V, 1, cbv);
    return (int)(g.y * g.z);
  }
  int bx, by;
  dw_block_shape(C, DWD2_V, bx, by);
  const int gy = cdiv(W, by * 4), NB = N * ((H + 1) / 2);
  return gy * cdiv(NB, dwd2_rpw(gy, NB));
}

// ---- weight gradient: per-workgroup partial [part][9][C] --------------------------------------
// grid: x = channel chunk, y = groups of tpb column tiles, z = N * row bands; part = (z, y).
template <typename T, int S, bool IT>
__global__ __launch_bounds__(256, 2) void dw_wgrad_kernel(DwBwdArgs a, int cbv, int tpb) {
  using G = DwTile<T, S>;
  extern __shared__ __attribute__((aligned(16))) uint4 s_in[];  // [IR*IC*cbv] (dw_shm)
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int QB = cbv * G::QPV;
  const int q = tid % QB, grp = tid / QB;
  const int gx = grp % G::GX, gy = grp / G::GX;
  int bx, by, bz;
  dw_tile(bx, by, bz);
  const int tiles_h = cdiv(a.Ho, G::TH), tiles_w = cdiv(a.Wo, G::TW);
  const int n = bz / tiles_h;
  const int th0 = (bz - n * tiles_h) * G::TH;
  const int c0 = bx * cbv * VecW<T>::V + q * 4;
  const int ho0 = th0 + gy * G::HS;
  const int nrow = max(0, min(G::HS, a.Ho - ho0));
  const T* sl = reinterpret_cast<const T*>(s_in);
  const int pstride = cbv * VecW<T>::V;
  float acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = 0.f;
  const int tw_lo = by * tpb, tw_hi = min(tiles_w, tw_lo + tpb);
  for (int twi = tw_lo; twi < tw_hi; ++twi) {
    const int tw0 = twi * G::TW;
    const int wo0 = tw0 + gx * G::WS;
    const int ncol = max(0, min(G::WS, a.Wo - wo0));
    // dy of the thread's outputs (clamped + selected), issued with the tile loads
    float g[G::HS][G::WS][4];
    const T* gb = (const T*)a.dy + c0;
#pragma unroll
    for (int r = 0; r < G::HS; ++r)
#pragma unroll
      for (int p = 0; p < G::WS; ++p) {
        const bool ok = r < nrow && p < ncol;
        const size_t off = ok ? (((size_t)n * a.Ho + ho0 + r) * a.Wo + wo0 + p) * a.C : 0;
        quad_ld(gb + off, g[r][p]);
      }
#pragma unroll
    for (int r = 0; r < G::HS; ++r)
#pragma unroll
      for (int p = 0; p < G::WS; ++p) {
        const bool ok = r < nrow && p < ncol;
#pragma unroll
        for (int j = 0; j < 4; ++j) g[r][p][j] = ok ? g[r][p][j] : 0.f;
      }
    __syncthreads();  // previous tile's LDS reads are done
    dw_stage<T, S, IT>(s_in, (const T*)a.x, a.H, a.W, a.C, n, th0 * S - 1, tw0 * S - 1, bx * cbv,
                       cbv, tid, nthr, a.x_scale, a.x_shift);
    __syncthreads();
    const int lr0 = gy * G::HS * S, lc0 = gx * G::WS * S;
#pragma unroll
    for (int rr = 0; rr < G::NR; ++rr)
#pragma unroll
      for (int ci = 0; ci < G::NC; ++ci) {
        float v[4];
        quad_ld(sl + ((lr0 + rr) * G::IC + lc0 + ci) * pstride + q * 4, v);
#pragma unroll
        for (int r = 0; r < G::HS; ++r) {
          const int kh = rr - r * S;
          if (kh < 0 || kh > 2) continue;
#pragma unroll
          for (int p = 0; p < G::WS; ++p) {
            const int kw = ci - p * S;
            if (kw < 0 || kw > 2) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[kh * 3 + kw][j] = fmaf(v[j], g[r][p][j], acc[kh * 3 + kw][j]);
          }
        }
      }
  }
  // ---- fixed-order reduction of the pixel groups, one tap at a time (LDS reused) ------------
  float* red = reinterpret_cast<float*>(s_in);  // [G][QB*4]
  const size_t part = (size_t)bz * gridDim.y + by;
  for (int t = 0; t < 9; ++t) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) red[(grp * QB + q) * 4 + j] = acc[t][j];
    __syncthreads();
    if (grp == 0) {
      float* rec = a.slab + (part * 9 + t) * a.C;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sum = 0.f;
        for (int g2 = 0; g2 < G::G; ++g2) sum += red[(g2 * QB + q) * 4 + j];
        rec[c0 + j] = sum;
      }
    }
  }
}

static int dw_wgrad_tpb(int N, int Ho, int Wo, int C, int V, int S, dim3& grid, int& cbv) {
  grid = dw_grid(N, Ho, Wo, C, V, S, cbv);
  const long long tiles_w = grid.y;
  const long long blocks = (long long)grid.x * grid.y * grid.z;
  // ~1024 workgroups (bounded partial count): at cfg3 6.05-6.07 ms/step against 6.10-6.11 for
  // 2048 and 6.12-6.15 for 4096 (A/B pairs on one box); 512 / 768 within noise of 1024
  long long tpb = blocks / 1024;
  if (tpb < 1) tpb = 1;
  if (tpb > tiles_w) tpb = tiles_w;
  grid.y = (unsigned)cdiv((int)tiles_w, (int)tpb);
  return (int)tpb;
}

int dw_wgrad_parts(int N, int Ho, int Wo, int C, int dtype, int stride) {
  dim3 g;
  int cbv;
  dw_wgrad_tpb(N, Ho, Wo, C, dtype == DT_F32 ? 4 : 8, stride, g, cbv);
  return (int)(g.y * g.z);
}

int dw_wgrad(const DwBwdArgs& a, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  dim3 grid;
  int cbv;
  const int tpb = dw_wgrad_tpb(a.N, a.Ho, a.Wo, a.C, V, a.stride, grid, cbv);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double in_el = (double)a.N * a.C * a.H * a.W, out_el = (double)a.N * a.C * a.Ho * a.Wo;
  ProfScope ps(PK_DW_WGRAD, st, E * (in_el + out_el), 18.0 * out_el);
  const int nthr = cbv * 32;
#define DWW_LAUNCH(T, S)                                                                      \
  do {                                                                                        \
    if (a.x_scale) prof_launch(dw_wgrad_kernel<T, S, true>, grid, nthr, dw_shm<T, S>(cbv), st, a, cbv, tpb); \
    else prof_launch(dw_wgrad_kernel<T, S, false>, grid, nthr, dw_shm<T, S>(cbv), st, a, cbv, tpb);          \
  } while (0)
  if (dtype == DT_F32) {
    if (a.stride == 1) DWW_LAUNCH(float, 1);
    else DWW_LAUNCH(float, 2);
  } else if (dtype == DT_F16) {
    if (a.stride == 1) DWW_LAUNCH(f16, 1);
    else DWW_LAUNCH(f16, 2);
  } else {
    if (a.stride == 1) DWW_LAUNCH(bf16, 1);
    else DWW_LAUNCH(bf16, 2);
  }
#undef DWW_LAUNCH
  return check_launch("dw_wgrad");
}

// slab [P][9][C] -> dW [C][9] (native PyTorch [C,1,3,3] layout): two-pass fixed-order reduction
int dw_wgrad_reduce(float* slab, int P, int C, float* dw, hipStream_t st) {
  return reduce_slabs_ex(slab, P, 9LL * C, 9LL * C, dw, 0, C, st);
}

}  // namespace fscnn
