// Pointwise 1x1 convolution as MFMA-tiled channel contractions (every nn.Conv2d(k=1) of
// models/fast_scnn.py: :73 _DSConv pw, :103/:107 bottleneck expand/project, :124-128 PPM,
// :198/:202 FFM, :230 classifier).  NHWC makes a 1x1 conv the row-major GEMM
//     C[m][n] = sum_k A[m][k] * W[n][k]      (m = pixel, k = Cin, n = Cout)
// with both operands k-contiguous ("NT"), which is exactly the operand order MFMA fragments
// want: lane l holds A[row l&15][8 consecutive k] (bf16 16x16x32) or A[row l&15][k] (fp32
// 16x16x4), so every fragment is one ds_read_b128 from a [row][k] LDS image.
//
// gemm_nt   forward and dgrad (the executor's dgrads read a per-step transposed weight copy;
//           the "b_trans" staging path remains for the C ABI).  Tile
//           128 rows x 16*NT cols, 4 waves of 32 rows, K staged in 128-B chunks (32 fp32 /
//           64 bf16), register-staged double-buffered LDS.  Epilogue fuses conv bias, BN
//           (scale/shift), residual add, ReLU and, in train mode, the per-channel BN statistics
//           (mean, M2, count) of the output tile.
// gemm_tn   weight gradient dW[n][k] = sum_m dY[m][n] X[m][k], split over m into partial
//           slabs reduced in fixed order (deterministic).
//
// fp32 storage uses v_mfma_f32_16x16x4_f32 (exact f32 products, f32 accumulate); bf16 storage
// uses v_mfma_f32_16x16x32_bf16 with f32 accumulation.  Roofline: MFMA-bound only when the
// tile's K and N are large; most Fast-SCNN 1x1 convs are HBM-bound.
#include "bn_finish.hpp"

namespace fscnn {


constexpr int G_BM = 128;
constexpr int G_VROW = 8;   // 16-B vectors per row per K chunk (128 B)
constexpr int G_VPAD = 9;   // LDS row stride in vectors
constexpr int G_ATMAX = 768;  // max K of a lazily normalised A operand (AT)

template <typename T>
struct MfmaOp;

template <>
struct MfmaOp<float> {
  // one 16-B vector per lane = 4 k-steps of 16x16x4
  static __device__ __forceinline__ void run(const uint4& a, const uint4& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};

template <>
struct MfmaOp<bf16> {
  static __device__ __forceinline__ void run(const uint4& a, const uint4& b, f32x4& acc) {
    i16x8 av, bv;
    __builtin_memcpy(&av, &a, 16);
    __builtin_memcpy(&bv, &b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
};

template <>
struct MfmaOp<f16> {  // inference plans of dtype fp16: v_mfma_f32_16x16x32_f16
  static __device__ __forceinline__ void run(const uint4& a, const uint4& b, f32x4& acc) {
    h16x8 av, bv;
    __builtin_memcpy(&av, &a, 16);
    __builtin_memcpy(&bv, &b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  }
};

template <typename T>
__device__ __forceinline__ uint4 zero_tail(uint4 v, int valid) {
  // zero the elements >= valid of a 16-B vector (valid <= 0: all, valid >= V: none); selects only
  constexpr int V = VecW<T>::V;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if (V == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = j < valid ? w[j] : 0u;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = (2 * j < valid) ? 0x0000FFFFu : 0u;
      const uint32_t hi = (2 * j + 1 < valid) ? 0xFFFF0000u : 0u;
      w[j] &= lo | hi;
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// XCD-aware block -> (major, minor) tile map.  Blocks b = x (mod 8) run on one XCD (observed
// round-robin placement; speed only, never correctness): give each residue class whole major
// indices with all `minor` tiles consecutive, so the operand shared by the minor tiles (the A
// row tile of gemm_nt, the D/X row split of gemm_tn) is fetched into that XCD's L2 once.
__device__ __forceinline__ void xcd_tile(int b, int nmajor, int nminor, int& major, int& minor) {
  if (nminor > 1 && (nmajor & 7) == 0) {
    const int x = b & 7, j = b >> 3;
    const int q = j / nminor;
    major = q * 8 + x;
    minor = j - q * nminor;
  } else {
    major = b % nmajor;
    minor = b / nmajor;
  }
}

// X3 (fp32 eval GEMMs): the MFMA step runs on the bf16 matrix cores with exact three-way
// splits of both operands (common.hpp gs_split3 / gs_mma_x3) — lane lq's two fp32 vectors of a
// 32-k chunk (k = 4lq.., 16+4lq..) form its 8 bf16 k-slots, the same permutation in A and B
// TL: the launch finishes its BN in its last workgroups (a.tail_ink; a separate instantiation so
// the other launches keep their register budget)
// The next K chunk's loads are in flight (registers) while the current chunk multiplies from LDS
// (one-ahead double buffer).  (A three-chunk register ring for the long-K low-M launches measured
// r04 6.048 vs 6.023 ms per cfg3 step -- its registers cost more occupancy than the latency it
// hid -- and was removed in r05.)
template <typename T, int NT, bool BT, bool BS, bool AT, bool X3 = false, bool TL = false>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs a) {
  constexpr int V = VecW<T>::V;
  constexpr int BN = 16 * NT;
  constexpr int KC = G_VROW * V;  // k elements per chunk
  // dynamic LDS: nbuf (1 when K fits one chunk, else 2) x (A + B tiles); the epilogue reuses it
  // for a 64-row fp32 half tile.  Single-chunk GEMMs (the K <= 64 expands) thus need ~32 KB and
  // run 4-5 workgroups per CU instead of 2.
  constexpr int CLD = BN + 4;                       // epilogue tile row stride (floats)
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  // AT kernels keep one LDS buffer (extra barrier per chunk) so their 6 KB scale/shift table
  // still leaves room for 3 workgroups per CU (double-buffered: 82 KB, 1 per CU)
  const int nbuf = ((a.K + KC - 1) / KC > 1 && !AT) ? 2 : 1;
  uint4* sAbase = reinterpret_cast<uint4*>(s_dyn);
  uint4* sBbase = sAbase + nbuf * G_BM * G_VPAD;
  auto sA = [&](int b) { return sAbase + b * G_BM * G_VPAD; };
  auto sB = [&](int b) { return sBbase + b * BN * G_VPAD; };
  float* sC = reinterpret_cast<float*>(s_dyn);      // after the main loop
  __shared__ float s_red[4][BN];
  // AT: A is the raw conv output z of a BatchNorm+ReLU whose activation is never stored (train
  // forward); the GEMM consumes relu(fmaf(z, a_scale[k], a_shift[k])), bn_apply's arithmetic
  __shared__ float s_at[AT ? 2 * G_ATMAX : 1];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  int tm, tn;
  xcd_tile(blockIdx.x, cdiv(a.M, G_BM), cdiv(a.N, BN), tm, tn);
  const int m0 = tm * G_BM;
  const int n0 = tn * BN;
  const T* A = (const T*)a.A;
  const T* B = (const T*)a.B;
  const int nchunks = (a.K + KC - 1) / KC;

  // ---- staging registers --------------------------------------------------------------------
  constexpr int A_PER = G_BM * G_VROW / 256;            // 4
  constexpr int B_PER = (BN * G_VROW + 255) / 256;      // vectors per thread (non-trans)
  uint4 ra[A_PER];
  uint4 rb[BT ? 1 : B_PER];
  // transposed-B staging: KC rows (k) x BN cols (n) of scalars, held as raw 16-B vectors along n
  constexpr int BT_VEC = KC * BN / V;                   // vectors per chunk
  constexpr int BT_PER = (BT_VEC + 255) / 256;
  uint4 rbt[BT ? BT_PER : 1];

  // Branch-free loads: every lane loads from an in-bounds (clamped) address and invalid or tail
  // elements are zeroed with selects afterwards, so all loads of a chunk issue back to back
  // (a branch around a load makes hipcc wait vmcnt(0) at the join).
  auto load_chunk = [&](int c) {
    const int k0 = c * KC;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int id = tid + 256 * i;
      int row = id >> 3, vv = id & 7;
      int m = m0 + row, k = k0 + vv * V;
      const bool ok = m < a.M && k < a.K;
      const size_t off = ok ? (size_t)m * a.lda + k : 0;
      ra[i] = *reinterpret_cast<const uint4*>(A + off);
    }
    if (!BT) {
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        int id = tid + 256 * i;
        int row = id >> 3, vv = id & 7;
        int n = n0 + row, k = k0 + vv * V;
        const bool ok = id < BN * G_VROW && n < a.N && k < a.K;
        const size_t off = ok ? (size_t)n * a.ldb + k : 0;
        rb[i] = *reinterpret_cast<const uint4*>(B + off);
      }
    } else {
#pragma unroll
      for (int i = 0; i < BT_PER; ++i) {
        int id = tid + 256 * i;
        int kk = id / (BN / V), nv = id - kk * (BN / V);
        int k = k0 + kk, n = n0 + nv * V;
        const bool ok = id < BT_VEC && k < a.K && n < a.N;
        const size_t off = ok ? (size_t)k * a.ldb + n : 0;
        rbt[i] = *reinterpret_cast<const uint4*>(B + off);
      }
    }
  };
  // Tail masks (and the lazy BN+ReLU of A) are applied when a chunk is written to LDS, i.e. after
  // the current chunk's MFMAs: applying them right after issuing the loads made every wave wait
  // for the next chunk's loads before computing (no fetch/compute overlap).
  auto store_chunk = [&](int buf, int c) {
    const int k0 = c * KC;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int id = tid + 256 * i;
      int row = id >> 3, vv = id & 7;
      int m = m0 + row, k = k0 + vv * V;
      uint4 v = ra[i];
      if constexpr (AT) {
        const int kc = k < a.K ? k : 0;
        v = bnrelu_vec<T>(v, s_at + kc, s_at + G_ATMAX + kc);
      }
      sA(buf)[row * G_VPAD + vv] = zero_tail<T>(v, m < a.M ? a.K - k : 0);
    }
    if (!BT) {
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        int id = tid + 256 * i;
        int row = id >> 3, vv = id & 7;
        int n = n0 + row, k = k0 + vv * V;
        if (id < BN * G_VROW)
          sB(buf)[row * G_VPAD + vv] = zero_tail<T>(rb[i], n < a.N ? a.K - k : 0);
      }
    } else {
      T* sbs = reinterpret_cast<T*>(sB(buf));
#pragma unroll
      for (int i = 0; i < BT_PER; ++i) {
        int id = tid + 256 * i;
        if (id < BT_VEC) {
          int kk = id / (BN / V), nv = id - kk * (BN / V);
          int k = k0 + kk, n = n0 + nv * V;
          const uint4 v = zero_tail<T>(rbt[i], k < a.K ? a.N - n : 0);
          const T* e = reinterpret_cast<const T*>(&v);
#pragma unroll
          for (int j = 0; j < V; ++j) sbs[(nv * V + j) * G_VPAD * V + kk] = e[j];
        }
      }
    }
  };

  f32x4 acc[2][NT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (AT) {
    for (int k = tid; k < G_ATMAX; k += 256) {
      s_at[k] = k < a.K ? a.a_scale[k] : 0.f;
      s_at[G_ATMAX + k] = k < a.K ? a.a_shift[k] : 0.f;
    }
  }
  stamp(a.stamps, 0);
  load_chunk(0);
  if constexpr (AT) __syncthreads();
  store_chunk(0, 0);
  __syncthreads();
  stamp(a.stamps, 1);
  {
    for (int c = 0; c < nchunks; ++c) {
      const int buf = nbuf == 2 ? (c & 1) : 0;
      if (c + 1 < nchunks) load_chunk(c + 1);
      if constexpr (X3) {
        uint4 a3[2][3];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const uint4* ar = sA(buf) + (wave * 32 + mt * 16 + li) * G_VPAD + lq;
          gs_split3(ar[0], ar[4], a3[mt]);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint4* br = sB(buf) + (nt * 16 + li) * G_VPAD + lq;
          uint4 b3[3];
          gs_split3(br[0], br[4], b3);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) gs_mma_x3(a3[mt], b3, acc[mt][nt]);
        }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int vv = lq + 4 * h;
          uint4 af[2], bfv[NT];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) af[mt] = sA(buf)[(wave * 32 + mt * 16 + li) * G_VPAD + vv];
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) bfv[nt] = sB(buf)[(nt * 16 + li) * G_VPAD + vv];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) MfmaOp<T>::run(af[mt], bfv[nt], acc[mt][nt]);
        }
      }
      if (c + 1 < nchunks) {
        if (nbuf == 1) __syncthreads();  // every wave's MFMA reads of this chunk are done
        store_chunk(nbuf == 2 ? buf ^ 1 : 0, c + 1);
      }
      __syncthreads();
    }
  }

  stamp(a.stamps, 2);
  // ---- epilogue -------------------------------------------------------------------------------
  // v = acc*scale + shift (registers; also feeds the statistics), staged through LDS as fp32 so
  // the stores (and the residual loads) are whole 16-B vectors: all residual loads are issued
  // before any store, no branches between them.
  float scv[NT], shv[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = n0 + nt * 16 + li;
    const int nc = n < a.N ? n : 0;
    scv[nt] = a.scale ? a.scale[nc] : 1.f;
    shv[nt] = a.shift ? a.shift[nc] : 0.f;
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mt][nt][r] = acc[mt][nt][r] * scv[nt] + shv[nt];
  T* Cp = (T*)a.C;
  const T* Rp = (const T*)a.R;
  constexpr int VPRow = BN / V;
  constexpr int HROWS = G_BM / 2;                // rows staged per half (waves 2h, 2h+1)
  constexpr int RG = 256 / VPRow;                // row groups; a thread keeps ONE column vector
  constexpr int NRT = (HROWS + RG - 1) / RG;     // rows per thread per half
  const int vc = tid % VPRow, rg = tid / VPRow;
  const bool tact = rg < RG;
  const int n = n0 + vc * V;
  const bool nfull = n + V <= a.N;
  constexpr bool bst = BS;  // fused BN-backward partials (dgrad producing a BN's dy)
  const T* Bz = (const T*)a.bz;
  // ReLU mask of the BN output recomputed as fmaf(z, scale, shift) > 0 (mode 2); mode 0 (no
  // ReLU) uses scale 0, shift 1 so both are the same select
  float bmu[bst ? V : 1], bis[bst ? V : 1], bsc[bst ? V : 1], bsh[bst ? V : 1];
  float s1[bst ? V : 1], s2[bst ? V : 1];
  if constexpr (bst) {
    const bool m2 = a.bmode == 2;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int nc = n + j < a.N ? n + j : 0;
      bmu[j] = a.bmean[nc];
      bis[j] = a.binvstd[nc];
      const float sc = a.bscale[nc], sh = a.bshift[nc];
      bsc[j] = m2 ? sc : 0.f;
      bsh[j] = m2 ? sh : 1.f;
      s1[j] = 0.f;
      s2[j] = 0.f;
    }
  }
  for (int half = 0; half < 2; ++half) {
    __syncthreads();  // main-loop LDS reads / previous half's reads done
    if ((wave >> 1) == half) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sC[((wave & 1) * 32 + mt * 16 + lq * 4 + r) * CLD + nt * 16 + li] = acc[mt][nt][r];
    }
    __syncthreads();
    // all global loads of the half (residual, BN z / mask) first: clamped + selected, no branch
    uint4 rr[NRT], zr[bst ? NRT : 1];
#pragma unroll
    for (int k = 0; k < NRT; ++k) {
      const int row = rg + k * RG;
      const int m = m0 + half * HROWS + row;
      const bool ok = tact && row < HROWS && m < a.M && nfull;
      if (Rp) rr[k] = sel4(ok, *reinterpret_cast<const uint4*>(Rp + (ok ? (size_t)m * a.ldr + n : 0)));
      if constexpr (bst)
        zr[k] = sel4(ok, *reinterpret_cast<const uint4*>(Bz + (ok ? (size_t)m * a.ldbz + n : 0)));
    }
#pragma unroll
    for (int k = 0; k < NRT; ++k) {
      const int row = rg + k * RG;
      const int m = m0 + half * HROWS + row;
      if (!tact || row >= HROWS || m >= a.M) continue;
      float o[V], rv[V];
      if (Rp) unpack<T>(rr[k], rv);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float v = sC[row * CLD + vc * V + j];
        if (Rp) v += rv[j];
        o[j] = a.relu ? fmaxf(v, 0.f) : v;
      }
      if (nfull) {
        stv(Cp + (size_t)m * a.ldc + n, o);
        if constexpr (bst) {  // BN-backward partials of the value as stored (rounded to T)
          float z[V];
          unpack<T>(zr[k], z);
#pragma unroll
          for (int j = 0; j < V; ++j) {
            float gv = round_as<T>(o[j]);
            gv = fmaf(z[j], bsc[j], bsh[j]) > 0.f ? gv : 0.f;
            s1[j] += gv;
            s2[j] += gv * (z[j] - bmu[j]) * bis[j];
          }
        }
      } else {
        for (int j = 0; j < V && n + j < a.N; ++j) {
          float v = sC[row * CLD + vc * V + j];
          if (Rp) v += ld1(Rp + (size_t)m * a.ldr + n + j);
          v = a.relu ? fmaxf(v, 0.f) : v;
          st1(Cp + (size_t)m * a.ldc + n + j, v);
          if constexpr (bst) {
            const float z = ld1(Bz + (size_t)m * a.ldbz + n + j);
            float gv = ld1(Cp + (size_t)m * a.ldc + n + j);
            gv = fmaf(z, bsc[j], bsh[j]) > 0.f ? gv : 0.f;
            s1[j] += gv;
            s2[j] += gv * (z - bmu[j]) * bis[j];
          }
        }
      }
    }
  }
  stamp(a.stamps, 3);
  if constexpr (bst) {
    // fixed-order column reduction over the RG row groups -> one record per 128-row tile
    __syncthreads();
    float* red = sC;  // [2][RG][BN]
    if (tact) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        red[rg * BN + vc * V + j] = s1[j];
        red[RG * BN + rg * BN + vc * V + j] = s2[j];
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.N) {
      float t1 = 0.f, t2 = 0.f;
      for (int g2 = 0; g2 < RG; ++g2) {
        t1 += red[g2 * BN + tid];
        t2 += red[RG * BN + g2 * BN + tid];
      }
      float* rec = a.bpart + (size_t)tm * 2 * a.N;
      st_wt(rec + n0 + tid, t1);
      st_wt(rec + a.N + n0 + tid, t2);
    }
    stamp(a.stamps, 4);
    if constexpr (TL)
      tail_finish<false>(a.bpart, cdiv(a.M, G_BM), a.N, tm, n0, min(BN, a.N - n0), tn, a.tail,
                         reinterpret_cast<double*>(s_dyn));
    stamp(a.stamps, 5);
    return;  // a dgrad output never carries forward statistics (acc dies with the epilogue)
  }
  if (a.part == nullptr) return;

  // ---- train-mode BN statistics of the output tile as stored (per column: mean, M2, count) -
  const int valid_rows = min(G_BM, a.M - m0);
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mt][nt][r] = round_as<T>(acc[mt][nt][r]);
  float mean_c[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    float s = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = m0 + wave * 32 + mt * 16 + lq * 4 + r;
        s += (m < a.M) ? acc[mt][nt][r] : 0.f;
      }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (lq == 0) s_red[wave][nt * 16 + li] = s;
  }
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    int col = nt * 16 + li;
    mean_c[nt] = (s_red[0][col] + s_red[1][col] + s_red[2][col] + s_red[3][col]) / (float)valid_rows;
  }
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    float s = 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int m = m0 + wave * 32 + mt * 16 + lq * 4 + r;
        float d = acc[mt][nt][r] - mean_c[nt];
        s += (m < a.M) ? d * d : 0.f;
      }
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (lq == 0) s_red[wave][nt * 16 + li] = s;
  }
  __syncthreads();
  if (wave == 0 && lq == 0) {
    float* rec = a.part + (size_t)tm * 3 * a.N;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      int col = nt * 16 + li, n = n0 + col;
      if (n < a.N) {
        st_wt(rec + n, mean_c[nt]);
        st_wt(rec + a.N + n, s_red[0][col] + s_red[1][col] + s_red[2][col] + s_red[3][col]);
        st_wt(rec + 2 * a.N + n, (float)valid_rows);
      }
    }
  }
  stamp(a.stamps, 4);
  if constexpr (TL)
    tail_finish<true>(a.part, cdiv(a.M, G_BM), a.N, tm, n0, min(BN, a.N - n0), tn, a.tail,
                      reinterpret_cast<double*>(s_dyn));
  stamp(a.stamps, 5);
}

static int pick_nt(int N) {
  if (N <= 32) return 2;
  if (N <= 48) return 3;
  if (N <= 64) return 4;
  if (N % 96 == 0) return 6;
  return 8;
}

int gemm_parts(int M) { return cdiv(M, G_BM); }

// the streaming kernel takes every shape it supports
static bool use_stream(const GemmArgs& a, int dtype) { return gemm_stream_ok(a, dtype); }

// BN partial records one gemm_nt call writes (part / bpart): one per 128-row tile, or one per
// streaming workgroup of a column group; always <= gemm_parts(M)
int gemm_nt_parts(const GemmArgs& a, int dtype) {
  return use_stream(a, dtype) ? gemm_stream_parts(a, dtype) : gemm_parts(a.M);
}

template <typename T, bool BT, bool BS, bool AT, bool X3, bool TL>
static void launch_nt_tl(const GemmArgs& a, int nt, dim3 grid, size_t shm, hipStream_t st) {
  switch (nt) {
    case 2: prof_launch(gemm_nt_kernel<T, 2, BT, BS, AT, X3, TL>, grid, 256, shm, st, a); break;
    case 3: prof_launch(gemm_nt_kernel<T, 3, BT, BS, AT, X3, TL>, grid, 256, shm, st, a); break;
    case 4: prof_launch(gemm_nt_kernel<T, 4, BT, BS, AT, X3, TL>, grid, 256, shm, st, a); break;
    case 6: prof_launch(gemm_nt_kernel<T, 6, BT, BS, AT, X3, TL>, grid, 256, shm, st, a); break;
    default: prof_launch(gemm_nt_kernel<T, 8, BT, BS, AT, X3, TL>, grid, 256, shm, st, a); break;
  }
}

template <typename T, bool BT, bool BS, bool AT = false, bool X3 = false>
static void launch_nt(const GemmArgs& a, int nt, hipStream_t st) {
  dim3 grid(cdiv(a.M, G_BM) * cdiv(a.N, 16 * nt));
  constexpr int V = VecW<T>::V;
  const int BN = 16 * nt;
  const int nbuf = (cdiv(a.K, G_VROW * V) > 1 && !AT) ? 2 : 1;
  const size_t tiles = (size_t)nbuf * (G_BM + BN) * G_VPAD * 16;
  size_t ctile = (size_t)(G_BM / 2) * (BN + 4) * 4;
  const size_t red = (size_t)2 * 256 * V * 4;  // bwd-BN column reduction (2 x RG x BN floats)
  if (a.bpart && red > ctile) ctile = red;
  const size_t shm = tiles > ctile ? tiles : ctile;
  if constexpr (!BT && !X3) {
    if (a.tail_ink) {
      launch_nt_tl<T, BT, BS, AT, X3, true>(a, nt, grid, shm, st);
      return;
    }
  }
  launch_nt_tl<T, BT, BS, AT, X3, false>(a, nt, grid, shm, st);
}

static int gemm_nt_tiled(const GemmArgs& a, int dtype, int nt, bool at, bool bs, hipStream_t st);

int gemm_nt(const GemmArgs& a, int dtype, hipStream_t st) {
  if (a.drop_hw && !gemm_stream_ok(a, dtype)) {
    set_error("gemm_nt: an output dropout needs the streaming kernel (M=%d N=%d K=%d)", a.M, a.N, a.K);
    return E_UNSUPPORTED;
  }
  const int V = dtype == DT_F32 ? 4 : 8;
  if (a.M <= 0 || a.N <= 0 || a.K <= 0) {
    set_error("gemm_nt: empty problem M=%d N=%d K=%d", a.M, a.N, a.K);
    return E_INVALID;
  }
  // C null: a statistics-only pass (the BN records of an output that is recomputed, not stored)
  if (!a.C && !(a.part && !a.R && !a.bpart && gemm_stream_ok(a, dtype))) {
    set_error("gemm_nt: no output (statistics only) needs the streaming kernel with statistics");
    return E_UNSUPPORTED;
  }
  if (a.lda % V || (uintptr_t)a.A % 16 || (uintptr_t)a.B % 16 || a.ldb % V) {
    set_error("gemm_nt: operands must be 16-B aligned with ld multiple of %d (lda=%d ldb=%d)", V,
              a.lda, a.ldb);
    return E_INVALID;
  }
  if (a.part && a.R) {
    set_error("gemm_nt: statistics with residual not supported");
    return E_UNSUPPORTED;
  }
  int nt = pick_nt(a.N);
  // small-M problems (the 16 K-row bottleneck2/3 projects and expand dgrads: 128 row tiles)
  // split the columns down to NT = 2 so ~512 workgroups (two per CU, eight waves) are in flight:
  // measured r04 5.965-5.976 ms/step vs 6.001-6.007 at a minimum grid of 256 and 6.016-6.018 at
  // 1024
  constexpr int min_tiles = 512;
  while ((long long)cdiv(a.M, G_BM) * cdiv(a.N, 16 * nt) < min_tiles &&
         (nt == 8 || nt == 6 || nt == 4 || nt == 3))
    nt = nt == 3 ? 2 : nt / 2;
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double M = a.M, N = a.N, K = a.K;
  const bool at = a.a_scale != nullptr;
  if (at && (!a.a_shift || a.b_trans || a.bpart || a.K > G_ATMAX || a.K % V)) {
    set_error("gemm_nt: lazy BN on A needs a plain GEMM with K <= %d, K %% %d == 0", G_ATMAX, V);
    return E_UNSUPPORTED;
  }
  const bool bs = a.bpart != nullptr;
  if (bs && (a.part || !a.bz || !a.bmean || !a.binvstd || !a.bscale || !a.bshift ||
             (a.bmode != 0 && a.bmode != 2) || a.ldbz % V)) {
    set_error("gemm_nt: inconsistent fused BN-backward arguments");
    return E_INVALID;
  }
  // b_trans (B read as [K][N]) stays for the C ABI's fscnn_pw_gemm; the executor's dgrads read
  // the per-step transposed weights (non-transposed B)
  if (bs && a.b_trans) {
    set_error("gemm_nt: fused BN-backward partials need a non-transposed B");
    return E_UNSUPPORTED;
  }
  if (a.tail.counters && !a.part && !a.bpart) {
    set_error("gemm_nt: a BN finish needs statistics records (part or bpart)");
    return E_INVALID;
  }
  const bool stream = use_stream(a, dtype);
  GemmArgs as = a;
  as.stamps = stamp_region();
  // tiled path: the BN finish runs in the kernel's last workgroups (bn_finish.hpp tail_finish)
  // when the records fit its counters; otherwise as its own fold + finalize launch below
  GemmArgs b = as;
  b.tail_ink = !stream && a.tail.counters && !a.b_trans &&
               a.tail.tsum && a.N <= TAIL_CMAX && tail_fits(gemm_parts(a.M), cdiv(a.N, 16 * nt));
  int rc;
  {
    ProfScope ps(PK_GEMM_NT, st,
                 E * (M * K + M * N * (a.R ? 2 : 1) + N * K + (a.bpart ? M * N : 0)),
                 2.0 * M * N * K);
    rc = stream ? gemm_stream(as, dtype, st)  // finishes the BN in-kernel (last workgroup)
                : gemm_nt_tiled(b, dtype, nt, at, bs, st);
  }
  if (rc || stream || !a.tail.counters || b.tail_ink) return rc;
  // tiled path: the BN finish as its own (fold + finalize) launch over the per-tile records
  if (a.part) {
    BnFinalizeArgs f = a.tail.fwd;
    f.part = a.part; f.P = gemm_parts(a.M); f.C = a.N; f.counters = a.tail.counters;
    return bn_finalize(f, st);
  }
  if (a.bpart)
    return bn_bwd_finalize(a.bpart, gemm_parts(a.M), a.N, a.tail.count, a.tail.dgamma,
                           a.tail.dbeta, a.tail.coef, st, a.tail.counters, a.tail.tab);
  return OK;
}

static int gemm_nt_tiled(const GemmArgs& a, int dtype, int nt, bool at, bool bs, hipStream_t st) {
  if (dtype == DT_F32) {
    static const bool x3 = [] {  // FSCNN_F32_SPLIT=0: exact fp32 MFMA (gemm_stream.hip)
      const char* e = getenv("FSCNN_F32_SPLIT");
      return !(e && e[0] == '0');
    }();
    if (x3 && !a.b_trans && !bs && !at && !a.part) launch_nt<float, false, false, false, true>(a, nt, st);
    else if (a.b_trans) launch_nt<float, true, false>(a, nt, st);
    else if (bs) launch_nt<float, false, true>(a, nt, st);
    else if (at) launch_nt<float, false, false, true>(a, nt, st);
    else launch_nt<float, false, false>(a, nt, st);
  } else if (dtype == DT_F16) {
    if (a.b_trans) launch_nt<f16, true, false>(a, nt, st);
    else if (bs) launch_nt<f16, false, true>(a, nt, st);
    else if (at) launch_nt<f16, false, false, true>(a, nt, st);
    else launch_nt<f16, false, false>(a, nt, st);
  } else {
    if (a.b_trans) launch_nt<bf16, true, false>(a, nt, st);
    else if (bs) launch_nt<bf16, false, true>(a, nt, st);
    else if (at) launch_nt<bf16, false, false, true>(a, nt, st);
    else launch_nt<bf16, false, false>(a, nt, st);
  }
  return check_launch("gemm_nt");
}

// =============================================================================================
// Weight gradient: dW[n][k] = sum_m D[m][n] * X[m][k]  (D = dY, X = layer input activation)
// =============================================================================================

constexpr int TN_T = 64;    // output tile 64 (n) x 64 (k)
constexpr int TN_MC = 64;   // rows (m) per staged chunk

// MFMA over 32 consecutive m held as 8 per lane group (k-index = 8*lq + e, same in A and B)
template <typename T>
struct TnOps;
template <>
struct TnOps<float> {
  static constexpr int LD = TN_MC + 4;
  static __device__ __forceinline__ void mma(const float* a, const float* b, f32x4& acc) {
    const float4 a0 = *reinterpret_cast<const float4*>(a), a1 = *reinterpret_cast<const float4*>(a + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(b), b1 = *reinterpret_cast<const float4*>(b + 4);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc, 0, 0, 0);
  }
};
template <>
struct TnOps<bf16> {
  static constexpr int LD = TN_MC + 8;
  static __device__ __forceinline__ void mma(const bf16* a, const bf16* b, f32x4& acc) {
    i16x8 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
};
template <>
struct TnOps<f16> {  // fp16 train plans (train.py:269's autocast arithmetic)
  static constexpr int LD = TN_MC + 8;
  static __device__ __forceinline__ void mma(const f16* a, const f16* b, f32x4& acc) {
    h16x8 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  }
};

// dW[n][k] = sum_m D[m][n] X[m][k] over the block's row split.  Chunks of 64 rows are loaded as
// 16-B vectors along n / k (coalesced), written TRANSPOSED into LDS (sDt[n][m], sXt[k][m]) so each
// MFMA operand is one or two 16-B ds_reads; the next chunk's global loads are issued before the
// current chunk's MFMAs.
template <typename T, bool XT>
__global__ __launch_bounds__(256) void gemm_tn_kernel(GemmTnArgs a) {
  constexpr int V = VecW<T>::V;
  constexpr int LD = TnOps<T>::LD;
  __shared__ __attribute__((aligned(16))) T sDt[TN_T * LD];
  __shared__ __attribute__((aligned(16))) T sXt[TN_T * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int tiles_k = cdiv(a.K, TN_T);
  int split, tile;
  xcd_tile(blockIdx.x, a.splits, cdiv(a.N, TN_T) * tiles_k, split, tile);
  const int tn = tile / tiles_k, tk = tile - tn * tiles_k;
  const int n0 = tn * TN_T, k0 = tk * TN_T;
  const int wn = (wave >> 1) * 32, wk = (wave & 1) * 32;  // wave sub-tile
  const int mb = split * a.rows_per_split;
  const int me = min(a.M, mb + a.rows_per_split);
  const T* D = (const T*)a.D;
  const T* X = (const T*)a.X;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS element (n, m) lives at n*LD + swz(n, m): the 8-element m-groups are XOR-swizzled by
  // n>>3 so the transposed pair writes below hit distinct banks; reads stay 16-B contiguous.
  auto swz = [](int n, int m) { return ((((m >> 3) ^ (n >> 3)) & 7) << 3) + (m & 7); };
  constexpr int VPR = TN_T / V;                 // vectors per staged row
  constexpr int PAIRS = TN_MC / 2 * VPR / 256;  // row pairs per thread (1 bf16 / 2 f32)
  uint4 rd[PAIRS][2], rx[PAIRS][2];
  auto load = [&](int mc) {
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      const int id = tid + 256 * i;
      const int rp = id / VPR, vv = id - rp * VPR;
      const int n = n0 + vv * V, k = k0 + vv * V;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = mc + 2 * rp + h;
        const bool okd = m < me && n < a.N, okx = m < me && k < a.K;
        rd[i][h] = *reinterpret_cast<const uint4*>(D + (okd ? (size_t)m * a.ldd + n : 0));
        rx[i][h] = *reinterpret_cast<const uint4*>(X + (okx ? (size_t)m * a.ldx + k : 0));
      }
    }
  };
  // XT: X is the raw conv output z of a BatchNorm+ReLU that is never stored (train); the operand
  // is relu(fmaf(z, x_scale[k], x_shift[k])).  A thread's X vectors all cover one k range
  // (vv = tid % VPR), so its V (scale, shift) pairs are loaded once.
  float xsc[XT ? V : 1], xsh[XT ? V : 1];
  if constexpr (XT) {
    const int kb = k0 + (tid % VPR) * V;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int k = kb + j < a.K ? kb + j : 0;
      xsc[j] = a.x_scale[k];
      xsh[j] = a.x_shift[k];
    }
  }
  // tail masks (and XT) right before the LDS stores, not right after issuing the loads (which
  // would make the wave wait for them before the current chunk's MFMAs)
  auto mask = [&](int mc) {
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      const int id = tid + 256 * i;
      const int rp = id / VPR, vv = id - rp * VPR;
      const int n = n0 + vv * V, k = k0 + vv * V;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool okm = mc + 2 * rp + h < me;
        uint4 dv = rd[i][h];
        rd[i][h] = zero_tail<T>(dv, okm ? a.N - n : 0);
        uint4 xv = rx[i][h];
        if constexpr (XT) xv = bnrelu_vec<T>(xv, xsc, xsh);
        rx[i][h] = zero_tail<T>(xv, okm ? a.K - k : 0);
      }
    }
  };
  using Pair = typename std::conditional<sizeof(T) == 2, uint32_t, uint2>::type;
  if (mb < me) load(mb);
  for (int mc = mb; mc < me; mc += TN_MC) {
    mask(mc);
    __syncthreads();  // previous chunk's MFMA reads done
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      const int id = tid + 256 * i;
      const int rp = id / VPR, vv = id - rp * VPR;
      const T* d0 = reinterpret_cast<const T*>(&rd[i][0]);
      const T* d1 = reinterpret_cast<const T*>(&rd[i][1]);
      const T* x0 = reinterpret_cast<const T*>(&rx[i][0]);
      const T* x1 = reinterpret_cast<const T*>(&rx[i][1]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int n = vv * V + j;
        const int off = n * LD + swz(n, 2 * rp);
        Pair pd, px;
        __builtin_memcpy(reinterpret_cast<T*>(&pd), d0 + j, sizeof(T));
        __builtin_memcpy(reinterpret_cast<T*>(&pd) + 1, d1 + j, sizeof(T));
        __builtin_memcpy(reinterpret_cast<T*>(&px), x0 + j, sizeof(T));
        __builtin_memcpy(reinterpret_cast<T*>(&px) + 1, x1 + j, sizeof(T));
        *reinterpret_cast<Pair*>(&sDt[off]) = pd;
        *reinterpret_cast<Pair*>(&sXt[off]) = px;
      }
    }
    __syncthreads();
    if (mc + TN_MC < me) load(mc + TN_MC);
#pragma unroll
    for (int ks = 0; ks < TN_MC / 32; ++ks) {
      const int kb = ks * 32 + 8 * lq;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int na = wn + i * 16 + li, nb = wk + j * 16 + li;
          TnOps<T>::mma(&sDt[na * LD + swz(na, kb)], &sXt[nb * LD + swz(nb, kb)], acc[i][j]);
        }
    }
  }
  // write the block's partial tile: slab[split][n][k]; acc[i][j][r]: n = wn+i*16+lq*4+r, k = wk+j*16+li
  float* sl = a.slab + (size_t)split * a.N * a.K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int n = n0 + wn + i * 16 + lq * 4 + r, k = k0 + wk + j * 16 + li;
        if (n < a.N && k < a.K) sl[(size_t)n * a.K + k] = acc[i][j][r];
      }
}

int gemm_tn_splits(int M, int N, int K) {
  // ~512 workgroups; a multiple of 8 splits so xcd_tile keeps a split's tiles on one XCD.
  // The split count sets the partial-slab volume the stage's deferred reduction reads back on
  // the main stream (366 MB per cfg3 step at ~1024 workgroups, 174 MB at ~512) while the wgrads
  // themselves run on the side stream; measured per cfg3 step: 1024 -> 6.46-6.51 ms, 512 ->
  // 6.41 ms, 256 -> 6.45-6.47 ms (the side stream then falls behind)
  constexpr int target = 512;
  int tiles = cdiv(N, TN_T) * cdiv(K, TN_T);
  int s = target / tiles;
  int smax = cdiv(M, 4 * TN_MC);
  if (s > smax) s = smax;
  if (s >= 8) s &= ~7;
  if (s < 1) s = 1;
  return s;
}

int gemm_tn(GemmTnArgs a, int splits, int dtype, hipStream_t st) {
  const int V = dtype == DT_F32 ? 4 : 8;
  if (a.ldd % V || a.ldx % V || (uintptr_t)a.D % 16 || (uintptr_t)a.X % 16) {
    set_error("gemm_tn: operands must be 16-B aligned (ldd=%d ldx=%d)", a.ldd, a.ldx);
    return E_INVALID;
  }
  a.rows_per_split = cdiv(cdiv(a.M, splits), TN_MC) * TN_MC;
  a.splits = splits;
  dim3 grid(cdiv(a.N, TN_T) * cdiv(a.K, TN_T) * splits);
  const double E = dtype == DT_F32 ? 4.0 : 2.0;
  const double M = a.M, N = a.N, K = a.K;
  ProfScope ps(PK_GEMM_TN, st, E * (M * N + M * K) + 4.0 * N * K, 2.0 * M * N * K);
  const bool xt = a.x_scale != nullptr;
  if (xt && (!a.x_shift || a.K % V)) {
    set_error("gemm_tn: lazy BN on X needs x_shift and K %% %d == 0", V);
    return E_UNSUPPORTED;
  }
#define TN_LAUNCH(T)                                        \
  do {                                                      \
    if (xt) prof_launch(gemm_tn_kernel<T, true>, grid, 256, 0, st, a); \
    else prof_launch(gemm_tn_kernel<T, false>, grid, 256, 0, st, a);   \
  } while (0)
  if (dtype == DT_F32) TN_LAUNCH(float);
  else if (dtype == DT_F16) TN_LAUNCH(f16);
  else TN_LAUNCH(bf16);
#undef TN_LAUNCH
  return check_launch("gemm_tn");
}

// Deterministic two-pass reduction of S partial slabs: out[i] = sum_{s<S} slab[s*stride + i].
// Pass 1 folds slab k into slab (k mod Q) IN PLACE (thread (i, q) owns every slab[k*stride+i]
// with k = q mod Q, so there is no race), giving Q*count-way parallelism; pass 2 sums the Q
// survivors.  Fixed assignment and order => bitwise reproducible.  `transpose9` writes
// out[(i % C9) * 9 + i / C9] (depthwise [9][C] partials -> PyTorch [C][3][3]).
constexpr int RED_Q = 64;

__global__ void reduce_fold_kernel(float* slab, int S, int Q, long long stride, int count) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  int q = blockIdx.y;
  if (i >= count) return;
  float s = 0.f;
  for (int k0 = q; k0 < S; k0 += 8 * Q) {  // 8 independent loads in flight per batch
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u * Q;
      const float t = slab[(size_t)(k < S ? k : q) * stride + i];  // clamped: branch-free
      v[u] = k < S ? t : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  slab[(size_t)q * stride + i] = s;
}

__global__ void reduce_final_kernel(const float* slab, int S, long long stride, int count,
                                    float* out, int accumulate, int C9) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  float s = 0.f;
  for (int k0 = 0; k0 < S; k0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float t = slab[(size_t)(k0 + u < S ? k0 + u : 0) * stride + i];
      v[u] = k0 + u < S ? t : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  int o = C9 ? (i % C9) * 9 + i / C9 : i;
  out[o] = accumulate ? out[o] + s : s;
}

int reduce_slabs_ex(float* slab, int S, long long stride, long long count, float* out,
                    int accumulate, int C9, hipStream_t st) {
  if (count <= 0 || count > 0x7fffffff) { set_error("reduce_slabs: bad count"); return E_INVALID; }
  int n = (int)count;
  int S2 = S;
  if (S > RED_Q) {
    dim3 g1(cdiv(n, 256), RED_Q);
    prof_launch(reduce_fold_kernel, g1, 256, 0, st, slab, S, RED_Q, stride, n);
    S2 = RED_Q;
  }
  prof_launch(reduce_final_kernel, cdiv(n, 256), 256, 0, st, slab, S2, stride, n, out, accumulate, C9);
  return check_launch("reduce_slabs");
}

int reduce_slabs(float* slab, int S, long long stride, long long count, float* out,
                 int accumulate, hipStream_t st) {
  return reduce_slabs_ex(slab, S, stride, count, out, accumulate, 0, st);
}

// Multi-job form: block b of the flattened job table belongs to the job whose [blk0, blk0')
// range holds b; every job is folded / summed exactly as reduce_slabs_ex does it (same
// assignment and order, so the result is bit-identical).
__device__ __forceinline__ int red_job(const RedTable& t, int b) {
  int lo = 0, hi = t.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t.blk0[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// fold: job j's blocks are (q, column block) pairs, q < J.Q, thread (i, q) sums slabs q, q + Q,
// ... into slab q.  Q = cdiv(S, 16) (<= RED_Q): ~16 partials per thread (one global Q = 64 left
// ~1-2 loads per thread and 41 K workgroups for bottleneck1's stage: 56 us)
__global__ void reduce_fold_multi_kernel(RedTable t) {
  const int jb = red_job(t, blockIdx.x);
  const RedJob& J = t.j[jb];
  const int nb = cdiv(J.count, 256);
  const int local = blockIdx.x - t.blk0[jb];
  const int q = local / nb;
  const int i = (local - q * nb) * blockDim.x + threadIdx.x;
  if (i >= J.count) return;
  float s = 0.f;
  for (int k0 = q; k0 < J.S; k0 += 8 * J.Q) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u * J.Q;
      const float x = J.slab[(size_t)(k < J.S ? k : q) * J.stride + i];
      v[u] = k < J.S ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  J.slab[(size_t)q * J.stride + i] = s;
}

__global__ void reduce_final_multi_kernel(RedTable t) {
  const int jb = red_job(t, blockIdx.x);
  const RedJob& J = t.j[jb];
  const int i = (blockIdx.x - t.blk0[jb]) * blockDim.x + threadIdx.x;
  if (i >= J.count) return;
  const int S = J.S > RED_Q ? J.Q : J.S;
  float s = 0.f;
  for (int k0 = 0; k0 < S; k0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float x = J.slab[(size_t)(k0 + u < S ? k0 + u : 0) * J.stride + i];
      v[u] = k0 + u < S ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  const int o = J.C9 ? (i % J.C9) * 9 + i / J.C9 : i;
  J.out[o] = J.accumulate ? J.out[o] + s : s;
}

int reduce_slabs_multi(const RedTable& tin, hipStream_t st) {
  if (tin.n <= 0) return OK;
  RedTable t = tin;
  // the fold pass covers only the jobs with more than RED_Q partials
  RedTable f;
  for (int k = 0; k < t.n; ++k) {
    RedJob& J = t.j[k];
    if (J.S <= RED_Q) continue;
    J.Q = cdiv(J.S, 16) < RED_Q ? cdiv(J.S, 16) : RED_Q;
    f.j[f.n] = J;
    f.blk0[f.n] = f.blocks;
    f.blocks += cdiv(J.count, 256) * J.Q;
    f.n++;
    f.blk0[f.n] = f.blocks;
  }
  if (f.n) prof_launch(reduce_fold_multi_kernel, f.blocks, 256, 0, st, f);
  prof_launch(reduce_final_multi_kernel, t.blocks, 256, 0, st, t);
  return check_launch("reduce_slabs_multi");
}

// per-block column sums of D [M][N] (ld) -> part [P][N]  (bias gradients)
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* D, int M, int N, int ld,
                                                     int rows_per_block, float* part) {
  int n = blockIdx.x * 64 + (threadIdx.x & 63);
  int g = threadIdx.x >> 6;
  __shared__ float red[4][64];
  float s = 0.f;
  if (n < N) {
    int mb = blockIdx.y * rows_per_block, me = min(M, mb + rows_per_block);
    for (int m0 = mb + g; m0 < me; m0 += 32) {  // 8 rows per batch, loads first
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int m = m0 + 4 * u;
        const float t = ld1(D + (size_t)(m < me ? m : mb) * ld + n);
        v[u] = m < me ? t : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  }
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && n < N)
    part[(size_t)blockIdx.y * N + n] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                       red[2][threadIdx.x] + red[3][threadIdx.x];
}

int colsum_parts(int M) { int p = cdiv(M, 1024); return p > 1024 ? 1024 : p; }

int colsum(const void* D, int M, int N, int ld, float* part, int dtype, hipStream_t st) {
  int P = colsum_parts(M);
  int rpb = cdiv(M, P);
  dim3 grid(cdiv(N, 64), P);
  if (dtype == DT_F32) prof_launch(colsum_kernel<float>, grid, 256, 0, st, (const float*)D, M, N, ld, rpb, part);
  else if (dtype == DT_F16) prof_launch(colsum_kernel<f16>, grid, 256, 0, st, (const f16*)D, M, N, ld, rpb, part);
  else prof_launch(colsum_kernel<bf16>, grid, 256, 0, st, (const bf16*)D, M, N, ld, rpb, part);
  return check_launch("colsum");
}

}  // namespace fscnn
