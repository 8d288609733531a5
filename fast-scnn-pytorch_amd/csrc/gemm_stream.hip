// Streaming pointwise GEMM for the eval forward: C[m][n] = epi(sum_k A[m][k] * W[n][k]).
// Same contract as gemm_nt (kernels.hpp GemmArgs, b_trans = 0, no statistics) for the 1x1 convs
// whose whole weight slice fits in LDS: every K <= 128 fp32 / <= 256 bf16 conv of
// models/fast_scnn.py (:73 DSConv pw, :103 expand, :124-128 PPM, :198/:202 FFM, :230 classifier).
//
// Why a second kernel: at M = 262,144 pixels and K = 128 the tiled gemm_nt spends as long in its
// LDS-staged A tile and epilogue as in MFMA.  Here
//   * a workgroup owns one column group (16*NT output channels) and keeps that group's weights
//     [16*NT][K] in LDS for its whole life (loaded once);
//   * each wave streams its own 32-pixel chunks straight from HBM into registers (lane (li, lq)
//     loads pixel li's k-vector lq of every k-step: one 16-B load per MFMA operand), with no
//     workgroup barrier in the loop;
//   * the MFMA operands are swapped (weights as the A operand), so each lane's accumulator holds
//     4 CONSECUTIVE output channels of one pixel: the epilogue (BN fold, bias, residual, ReLU)
//     runs in registers and stores 16-B (fp32) / 8-B (bf16) NHWC vectors directly.
// The k summation order inside a 16x16xK MFMA step matches gemm_nt (4-element k quads for fp32,
// 8-element for bf16, steps in increasing k), so results agree with it to rounding of the
// accumulation order within the hardware MFMA.
#include "kernels.hpp"

namespace fscnn {

constexpr int GS_MW = 32;  // pixels per wave chunk (2 x 16-row MFMA tiles)

template <typename T>
struct GsMma;
template <>
struct GsMma<float> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.x), __uint_as_float(x.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.y), __uint_as_float(x.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.z), __uint_as_float(x.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(w.w), __uint_as_float(x.w), acc, 0, 0, 0);
  }
};
template <>
struct GsMma<bf16> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    i16x8 wv, xv;
    __builtin_memcpy(&wv, &w, 16);
    __builtin_memcpy(&xv, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, xv, acc, 0, 0, 0);
  }
};

template <>
struct GsMma<f16> {
  static __device__ __forceinline__ void run(const uint4& w, const uint4& x, f32x4& acc) {
    h16x8 wv, xv;
    __builtin_memcpy(&wv, &w, 16);
    __builtin_memcpy(&xv, &x, 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wv, xv, acc, 0, 0, 0);
  }
};

// zero the elements >= valid of a 16-B vector with selects only (no dynamic register indexing)
template <typename T>
__device__ __forceinline__ uint4 gs_tail(uint4 v, int valid) {
  constexpr int V = VecW<T>::V;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (V == 4) {
      w[j] = j < valid ? w[j] : 0u;
    } else {
      const uint32_t lo = (2 * j < valid) ? 0x0000FFFFu : 0u;
      const uint32_t hi = (2 * j + 1 < valid) ? 0xFFFF0000u : 0u;
      w[j] &= lo | hi;
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// NT: 16-column MFMA tiles per group; KS: k-steps (16 fp32 / 32 bf16 k each) covering K
template <typename T, int NT, int KS, bool TAIL>
__global__ __launch_bounds__(256, 2) void gemm_stream_kernel(GemmArgs a, int bpg) {
  constexpr int V = VecW<T>::V;     // elements per 16-B vector
  constexpr int KV = 4 * KS;        // 16-B vectors per weight row (4 per k-step)
  constexpr int WST = KV + 1;       // padded LDS row stride (vectors): conflict-free b128 reads
  constexpr int BN = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) uint4 s_w[];  // [BN][WST]
  float* s_sc = reinterpret_cast<float*>(s_w + BN * WST);       // [BN] scale, [BN] shift

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  // block -> (group, index within group) = blockIdx / bpg; bpg % 8 == 0 (when not capped) keeps
  // the blocks that stream the same pixel chunks for different groups on one XCD (shared A in L2)
  const int g = blockIdx.x / bpg;
  const int bi = blockIdx.x - g * bpg;
  const int n0 = g * BN;
  const T* A = (const T*)a.A;
  const T* B = (const T*)a.B;

  // ---- weights of the group -> LDS (zero rows n >= N, zero k >= K) ---------------------------
  for (int i = tid; i < BN * KV; i += 256) {
    const int r = i / KV, v = i - r * KV;
    const int n = n0 + r, k = v * V;
    const bool ok = n < a.N && k < a.K;
    const uint4 t = gs_tail<T>(*reinterpret_cast<const uint4*>(B + (ok ? (size_t)n * a.ldb + k : 0)),
                               ok ? a.K - k : 0);
    s_w[r * WST + v] = t;
  }
  for (int i = tid; i < BN; i += 256) {
    const int n = n0 + i < a.N ? n0 + i : 0;
    s_sc[i] = a.scale ? a.scale[n] : 1.f;
    s_sc[BN + i] = a.shift ? a.shift[n] : 0.f;
  }
  __syncthreads();

  const int nchunks = cdiv(a.M, GS_MW);
  const int wstride = bpg * 4;
  int c = bi * 4 + wave;
  if (c >= nchunks) return;

  // k-vector (4*s + lq) of pixel rows li, 16 + li of the chunk -> x[mt][s]
  uint4 xa[2][KS];
  auto loadx = [&](int chunk, uint4 (&r)[2][KS]) {
    const bool cok = chunk < nchunks;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = chunk * GS_MW + mt * 16 + li;
      const bool mok = cok && m < a.M;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int k = (4 * s + lq) * V;
        const bool ok = mok && k < a.K;
        r[mt][s] = *reinterpret_cast<const uint4*>(A + (ok ? (size_t)m * a.lda + k : 0));
      }
    }
    // zero invalid rows / the K tail (selects after all loads are in flight)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = chunk * GS_MW + mt * 16 + li;
      const bool mok = cok && m < a.M;
#pragma unroll
      for (int s = 0; s < KS; ++s) r[mt][s] = gs_tail<T>(r[mt][s], mok ? a.K - (4 * s + lq) * V : 0);
    }
  };

  T* Cp = (T*)a.C;
  const T* Rp = (const T*)a.R;
  // Small chunks (KS <= 4: 32 A registers or fewer) double-buffer the next chunk in registers;
  // the big fp32 tiles do not (it would push them past 256 VGPRs): there the co-resident waves
  // of a SIMD alternate their load and MFMA phases, and the MFMAs of step s wait only for step
  // s's loads.
  constexpr bool PF = KS <= 4;
  uint4 xn[2][PF ? KS : 1];
  if constexpr (PF) loadx(c, xa);
  for (; c < nchunks; c += wstride) {
    if constexpr (PF) loadx(c + wstride, xn);  // clamped / zeroed past the end
    else loadx(c, xa);
    f32x4 acc[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the weight fragments are loop-invariant: launder the LDS base so they are re-read per
    // chunk (cheap ds_read_b128) instead of being hoisted into NT*KS*4 registers
    int wb = li * WST + lq;
    asm volatile("" : "+v"(wb));
    const float* ssc = s_sc + (wb - li * WST - lq);  // same laundering for the epilogue table
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const uint4 w = s_w[wb + nt * 16 * WST + 4 * s];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) GsMma<T>::run(w, xa[mt][s], acc[mt][nt]);
      }
    }
    // ---- epilogue: lane holds channels n0 + 16nt + 4lq + r of pixel m ------------------------
    if constexpr (!TAIL) {  // whole 4-channel vectors, 16-B aligned rows (checked on the host)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int m = c * GS_MW + mt * 16 + li;
        const bool mok = m < a.M;
        const size_t mr = mok ? (size_t)m : 0;
        float rv[NT][4];
        if (Rp) {  // every residual load of the row before any store (R may alias C)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) ld4v(Rp + mr * a.ldr + n0 + nt * 16 + 4 * lq, rv[nt]);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int nl = nt * 16 + 4 * lq;
          const float4 sc = *reinterpret_cast<const float4*>(ssc + nl);
          const float4 sh = *reinterpret_cast<const float4*>(ssc + BN + nl);
          const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[mt][nt][r] * scv[r] + shv[r];
            if (Rp) v += rv[nt][r];
            o[r] = a.relu ? fmaxf(v, 0.f) : v;
          }
          if (mok) st4v(Cp + mr * a.ldc + n0 + nl, o);
        }
      }
    } else {  // column tail / unaligned rows (the 19-class classifier): scalar
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int m = c * GS_MW + mt * 16 + li;
        if (m >= a.M) continue;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int nl = nt * 16 + 4 * lq;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = n0 + nl + r;
            if (n >= a.N) continue;
            float v = acc[mt][nt][r] * ssc[nl + r] + ssc[BN + nl + r];
            if (Rp) v += ld1(Rp + (size_t)m * a.ldr + n);
            st1(Cp + (size_t)m * a.ldc + n, a.relu ? fmaxf(v, 0.f) : v);
          }
        }
      }
    }
    if constexpr (PF) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int s = 0; s < KS; ++s) xa[mt][s] = xn[mt][s];
    }
  }
}

static int gs_pick_nt(int N) {
  if (N <= 32) return 2;
  if (N <= 48) return 3;
  if (N <= 64) return 4;
  if (N % 96 == 0) return 6;
  return 8;
}

static bool gs_tail_needed(const GemmArgs& a, int nt) {
  return a.N % (16 * nt) != 0 || a.ldc % 4 != 0 || (a.R && a.ldr % 4 != 0);
}

bool gemm_stream_ok(const GemmArgs& a, int dtype) {
  const int KC = dtype == DT_F32 ? 16 : 32;  // k per step
  const int ks = cdiv(a.K, KC);
  if (a.part || a.bpart || a.b_trans) return false;
  if (!(ks == 1 || ks == 2 || ks == 3 || ks == 4 || ks == 6 || ks == 8)) return false;
  const int nt = gs_pick_nt(a.N);
  if (gs_tail_needed(a, nt) && nt != 2) return false;  // scalar-tail variant only for N <= 32
  const size_t lds = (size_t)16 * nt * (4 * ks + 1) * 16 + (size_t)2 * 16 * nt * 4;
  if (lds > 72 * 1024) return false;
  return a.M >= 4096;  // tiny GEMMs (PPM bins): loading a weight slice per block does not pay
}


template <typename T, int NT, bool TAIL>
static void gs_launch_ks(const GemmArgs& a, int ks, dim3 grid, size_t lds, int bpg,
                         hipStream_t st) {
  switch (ks) {
    case 1: gemm_stream_kernel<T, NT, 1, TAIL><<<grid, 256, lds, st>>>(a, bpg); break;
    case 2: gemm_stream_kernel<T, NT, 2, TAIL><<<grid, 256, lds, st>>>(a, bpg); break;
    case 3: gemm_stream_kernel<T, NT, 3, TAIL><<<grid, 256, lds, st>>>(a, bpg); break;
    case 4: gemm_stream_kernel<T, NT, 4, TAIL><<<grid, 256, lds, st>>>(a, bpg); break;
    case 6: gemm_stream_kernel<T, NT, 6, TAIL><<<grid, 256, lds, st>>>(a, bpg); break;
    default: gemm_stream_kernel<T, NT, 8, TAIL><<<grid, 256, lds, st>>>(a, bpg); break;
  }
}

template <typename T>
static void gs_launch(const GemmArgs& a, hipStream_t st) {
  constexpr int KC = 4 * VecW<T>::V;
  const int ks = cdiv(a.K, KC);
  const int nt = gs_pick_nt(a.N);
  const int groups = cdiv(a.N, 16 * nt);
  const size_t lds = (size_t)16 * nt * (4 * ks + 1) * 16 + (size_t)2 * 16 * nt * 4;
  const int nchunks = cdiv(a.M, GS_MW);
  // resident workgroups: LDS-limited (160 KB / CU), at most 2 per CU (measured: 3-4 slower)
  int per_cu = (int)((160 * 1024) / (lds + 1024));
  per_cu = per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu);
  int bpg = cdiv(256 * per_cu, groups);
  bpg = (bpg + 7) / 8 * 8;
  const int need = cdiv(nchunks, 4);
  if (bpg > need) bpg = need;
  if (bpg < 1) bpg = 1;
  dim3 grid((unsigned)(groups * bpg));
  switch (nt) {
    case 2:
      if (gs_tail_needed(a, nt)) gs_launch_ks<T, 2, true>(a, ks, grid, lds, bpg, st);
      else gs_launch_ks<T, 2, false>(a, ks, grid, lds, bpg, st);
      break;
    case 3: gs_launch_ks<T, 3, false>(a, ks, grid, lds, bpg, st); break;
    case 4: gs_launch_ks<T, 4, false>(a, ks, grid, lds, bpg, st); break;
    case 6: gs_launch_ks<T, 6, false>(a, ks, grid, lds, bpg, st); break;
    default: gs_launch_ks<T, 8, false>(a, ks, grid, lds, bpg, st); break;
  }
}

int gemm_stream(const GemmArgs& a, int dtype, hipStream_t st) {
  if (dtype == DT_F32) gs_launch<float>(a, st);
  else if (dtype == DT_F16) gs_launch<f16>(a, st);
  else gs_launch<bf16>(a, st);
  return check_launch("gemm_stream");
}

}  // namespace fscnn
