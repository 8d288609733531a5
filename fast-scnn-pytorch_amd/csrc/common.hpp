// Shared device/host helpers for the Fast-SCNN gfx950 kernels.
//
// Layout conventions: activations are NHWC ("[M rows = N*H*W][C channels]",
// channels contiguous) in the storage type T (float or bf16); every kernel computes in fp32.
// Per-channel BatchNorm statistics travel as "partial records" [part][3][C] = (mean, M2, count)
// merged with Chan's parallel formula, so every reduction is deterministic (fixed order) and
// free of the E[x^2]-E[x]^2 cancellation.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <type_traits>

#include <string>

namespace fscnn {

// DT_F16 is an input / output dtype (fp16 images in, fp16 logits out: the reference's fp16
// autocast I/O); the arithmetic of such a call runs in the plan's dtype (bf16 for cfg5).
enum DType : int { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

struct bf16 {
  uint16_t x;
};
struct f16 {  // IEEE half storage (inference plans of dtype DT_F16; fp16 I/O)
  uint16_t x;
};
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }
// a 16-bit input element of dtype code XT (1 bf16, 2 fp16) as fp32
template <int XT>
__device__ __forceinline__ float in16(uint16_t h) { return XT == 2 ? h2f(h) : bf2f(h); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // RNE; lowers to v_cvt_pk_bf16_f32 on gfx950
  return *reinterpret_cast<uint16_t*>(&h);
}

// Elements per 16-byte vector.
template <typename T> struct VecW;
template <> struct VecW<float> { static constexpr int V = 4; };
template <> struct VecW<bf16> { static constexpr int V = 8; };
template <> struct VecW<f16> { static constexpr int V = 8; };

// a 16-bit storage element <-> fp32 (bf16 or fp16), and fp32 rounded the way T stores it
template <typename T> __device__ __forceinline__ float s16_to(uint16_t h) {
  if constexpr (std::is_same<T, f16>::value) return h2f(h);
  else return bf2f(h);
}
template <typename T> __device__ __forceinline__ uint16_t s16_from(float f) {
  if constexpr (std::is_same<T, f16>::value) return f2h(f);
  else return f2bf(f);
}
template <typename T> __device__ __forceinline__ float round_as(float v) {
  if constexpr (sizeof(T) == 4) return v;
  else return s16_to<T>(s16_from<T>(v));
}

// ---- scalar load/store in storage type -------------------------------------------------------
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16* p) { return bf2f(p->x); }
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(bf16* p, float v) { p->x = f2bf(v); }
__device__ __forceinline__ float ld1(const f16* p) { return h2f(p->x); }
__device__ __forceinline__ void st1(f16* p, float v) { p->x = f2h(v); }

// ---- 16-byte vector load/store (p must be 16 B aligned) --------------------------------------
__device__ __forceinline__ void ldv(const float* p, float (&v)[4]) {
  float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
__device__ __forceinline__ void ldv(const bf16* p, float (&v)[8]) {
  uint4 t = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
__device__ __forceinline__ void ldv(const f16* p, float (&v)[8]) {
  uint4 t = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = h2f((uint16_t)(w[i] & 0xFFFFu));
    v[2 * i + 1] = h2f((uint16_t)(w[i] >> 16));
  }
}
__device__ __forceinline__ void stv(f16* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2h(v[2 * i]) | ((uint32_t)f2h(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void stv(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void stv(bf16* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

// raw 16-B vector in storage type -> floats (for code that keeps loads packed until use)
__device__ __forceinline__ void unpackv(const uint4& t, float (&v)[4]) {
  v[0] = __uint_as_float(t.x); v[1] = __uint_as_float(t.y);
  v[2] = __uint_as_float(t.z); v[3] = __uint_as_float(t.w);
}
__device__ __forceinline__ void unpackv(const uint4& t, float (&v)[8]) {
  const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
// raw 16-B vector of storage type T -> floats (bf16 / fp16 / fp32)
template <typename T>
__device__ __forceinline__ void unpack(const uint4& t, float (&v)[VecW<T>::V]) {
  if constexpr (sizeof(T) == 4) {
    unpackv(t, v);
  } else {
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = s16_to<T>((uint16_t)(w[i] & 0xFFFFu));
      v[2 * i + 1] = s16_to<T>((uint16_t)(w[i] >> 16));
    }
  }
}
__device__ __forceinline__ uint4 sel4(bool ok, const uint4& t) {
  return ok ? t : make_uint4(0u, 0u, 0u, 0u);
}

// ---- Chan parallel merge of (count, mean, M2) ------------------------------------------------
struct Welford {
  double n, mean, m2;
};
__device__ __forceinline__ Welford wf_merge(Welford a, Welford b) {
  double n = a.n + b.n;
  if (n == 0.0) return a;
  double d = b.mean - a.mean;
  double f = b.n / n;
  Welford r;
  r.n = n;
  r.mean = a.mean + d * f;
  r.m2 = a.m2 + b.m2 + d * d * a.n * f;
  return r;
}

// ---- in-launch hand-off between workgroups (MI355X_MICROARCH.md, inter-workgroup visibility) ----
// Per-XCD L2s are not coherent, and an agent-scope release fence writes back the XCD's whole L2
// (microseconds).  Small hand-offs therefore go write-through instead: every byte a workgroup
// publishes is stored with an `sc1` store (st_wt), each storing wave drains its stores
// (s_waitcnt vmcnt(0)), the workgroup barriers, and ONE lane adds to an agent-scope counter; the
// workgroup whose add returns expected-1 is the last arriver and reads the published bytes with
// `sc1` loads (ld_wt), which bypass its L1.  No workgroup ever waits for another (no spin), and
// the last arriver resets the counter for the next launch.
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every thread of the workgroup calls this after its st_wt stores; true in the last arriver
__device__ __forceinline__ bool arrive_last(unsigned* ctr, unsigned expected) {
  __shared__ unsigned s_old;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0 && threadIdx.z == 0)
    s_old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool last = s_old == expected - 1;
  // no instruction: keeps the compiler from hoisting the last arriver's sc1 loads above the add
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return last;
}
__device__ __forceinline__ void reset_counter(unsigned* ctr) {
  if (threadIdx.x == 0 && threadIdx.y == 0 && threadIdx.z == 0)
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- fp32 products on the bf16 matrix cores (eval GEMMs; gemm_stream.hip, gemm.hip) --------
// An fp32 value splits exactly into three bf16 terms by truncation, f = f0 + f1 + f2; with the
// same k permutation in both operands, six v_mfma_f32_16x16x32_bf16 give a.w to fp32 accuracy
// (the dropped a1w2 + a2w1 + a2w2 are below fp32's own product rounding).
__device__ __forceinline__ void gs_split3(const uint4& lo4, const uint4& hi4, uint4 (&t)[3]) {
  // 8 fp32 (k = 8lq .. 8lq+7 of one row) -> three bf16x8 vectors (truncation splits)
  const uint32_t f[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
  uint32_t p0[8], p1[8], p2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t b0 = f[e] & 0xFFFF0000u;
    const float r1 = __uint_as_float(f[e]) - __uint_as_float(b0);  // exact
    const uint32_t b1 = __float_as_uint(r1) & 0xFFFF0000u;
    const float r2 = r1 - __uint_as_float(b1);                       // exact, <= 8 bits
    p0[e] = b0;
    p1[e] = b1;
    p2[e] = __float_as_uint(r2) & 0xFFFF0000u;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const uint32_t* p = j == 0 ? p0 : (j == 1 ? p1 : p2);
    t[j] = make_uint4((p[0] >> 16) | p[1], (p[2] >> 16) | p[3], (p[4] >> 16) | p[5],
                      (p[6] >> 16) | p[7]);
  }
}

__device__ __forceinline__ void gs_mma_x3(const uint4 (&w)[3], const uint4 (&x)[3], f32x4& acc) {
  i16x8 a[3], b[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    __builtin_memcpy(&a[j], &w[j], 16);
    __builtin_memcpy(&b[j], &x[j], 16);
  }
  // smallest terms first
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
}

// LearningToDownsample.conv (conv0.hip, stem.hip): MFMA helpers for the im2col GEMM out[px][co] = sum_k patch[px][k] * W[co][k], K = 27 -> 32:
// lane (li, lq) supplies k = 8*lq .. 8*lq+7 for its row (pixel li / channel li).
template <int BF>
struct C0Mma;
template <>
struct C0Mma<2> {  // fp16 operands (inference plans of dtype fp16): v_mfma_f32_16x16x32_f16
  using Frag = h16x8;
  static __device__ __forceinline__ Frag pack(const float (&v)[8]) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (_Float16)v[e];
    return f;
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  }
};
template <>
struct C0Mma<1> {  // bf16 operands, one v_mfma_f32_16x16x32_bf16 per 16 px x 16 co
  using Frag = i16x8;
  static __device__ __forceinline__ Frag pack(const float (&v)[8]) {
    Frag f;
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (short)f2bf(v[e]);
    return f;
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
};
template <>
struct C0Mma<0> {  // fp32: the three-term bf16 split of both operands, six bf16 MFMAs (gs_mma_x3)
  // (r05: replaces 8 x v_mfma_f32_16x16x4_f32 = 256 matrix cycles per 16 px x 16 co by 96; the
  //  dropped split terms are below fp32's own product rounding)
  struct Frag { uint4 t[3]; };
  static __device__ __forceinline__ Frag pack(const float (&v)[8]) {
    Frag f;
    gs_split3(make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                         __float_as_uint(v[3])),
              make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]),
                         __float_as_uint(v[7])), f.t);
    return f;
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4& acc) {
    gs_mma_x3(a.t, b.t, acc);
  }
};

// ---- 4-element vectors (16 B fp32 / 8 B bf16) ------------------------------------------------
__device__ __forceinline__ void st4v(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st4v(bf16* p, const float (&v)[4]) {
  uint2 t;
  t.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  t.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = t;
}
__device__ __forceinline__ void ld4v(const float* p, float (&v)[4]) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
}
__device__ __forceinline__ void st4v(f16* p, const float (&v)[4]) {
  uint2 t;
  t.x = (uint32_t)f2h(v[0]) | ((uint32_t)f2h(v[1]) << 16);
  t.y = (uint32_t)f2h(v[2]) | ((uint32_t)f2h(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = t;
}
__device__ __forceinline__ void ld4v(const f16* p, float (&v)[4]) {
  const uint2 t = *reinterpret_cast<const uint2*>(p);
  v[0] = h2f((uint16_t)(t.x & 0xFFFFu)); v[1] = h2f((uint16_t)(t.x >> 16));
  v[2] = h2f((uint16_t)(t.y & 0xFFFFu)); v[3] = h2f((uint16_t)(t.y >> 16));
}
__device__ __forceinline__ void ld4v(const bf16* p, float (&v)[4]) {
  const uint2 t = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xFFFF0000u);
  v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xFFFF0000u);
}

// ---- lazily applied BatchNorm + ReLU of a producer whose activation is never stored ---------
// relu(fmaf(x, sc[j], sh[j])) on one raw 16-B vector of the storage type: exactly bn_apply's
// arithmetic (fp32 fma, ReLU, RNE back to the storage type), so a consumer that applies it while
// staging its operand sees the same bits bn_apply would have written.
template <typename T>
__device__ __forceinline__ uint4 bnrelu_vec(const uint4& t, const float* sc, const float* sh) {
  if constexpr (sizeof(T) == 4) {
    float v[4];
    unpackv(t, v);
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = __float_as_uint(fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f));
    return make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    float v[8];
    unpack<T>(t, v);
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = fmaxf(fmaf(v[2 * i], sc[2 * i], sh[2 * i]), 0.f);
      const float b = fmaxf(fmaf(v[2 * i + 1], sc[2 * i + 1], sh[2 * i + 1]), 0.f);
      w[i] = (uint32_t)s16_from<T>(a) | ((uint32_t)s16_from<T>(b) << 16);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---- BatchNorm backward applied while a consumer stages its operand -------------------------
// The dz of a train-mode BatchNorm(+ReLU) is never stored: its consumers (the conv's wgrad and
// dgrad) read dy and the saved pre-BN tensor z and form, per element,
//     dz = alpha * [fmaf(z, sc, sh) > 0] * dy + (gz * z + beta)       (rounded to the storage type)
// i.e. scale * (dy_r - mean(dy_r) - xhat * mean(dy_r * xhat)) with the BN-backward sums folded into
// per-channel (alpha, beta, gz) by bn_bwd_finalize; (sc, sh) is the forward BN affine that
// recomputes the ReLU mask (no ReLU: sc = 0, sh = 1).  Table: tab[c * 8 + {0..4}].
constexpr int BWDX_STRIDE = 8;
template <typename T>
__device__ __forceinline__ uint4 packv(const float (&o)[VecW<T>::V]) {
  if constexpr (sizeof(T) == 4) {
    return make_uint4(__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]),
                      __float_as_uint(o[3]));
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)s16_from<T>(o[2 * i]) | ((uint32_t)s16_from<T>(o[2 * i + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}
// per-lane coefficients of V consecutive channels c..c+V-1 (registers)
template <typename T>
struct BwdXCoef {
  float al[VecW<T>::V], be[VecW<T>::V], gz[VecW<T>::V], sc[VecW<T>::V], sh[VecW<T>::V];
  __device__ __forceinline__ void load(const float* tab, int c) {
#pragma unroll
    for (int j = 0; j < VecW<T>::V; ++j) {
      const float4 t = *reinterpret_cast<const float4*>(tab + (size_t)(c + j) * BWDX_STRIDE);
      al[j] = t.x; be[j] = t.y; gz[j] = t.z; sc[j] = t.w;
      sh[j] = tab[(size_t)(c + j) * BWDX_STRIDE + 4];
    }
  }
};
template <typename T>
__device__ __forceinline__ uint4 bwdx_apply(const uint4& dy, const uint4& z, const float* al,
                                            const float* be, const float* gz, const float* sc,
                                            const float* sh) {
  constexpr int V = VecW<T>::V;
  float g[V], zz[V], o[V];
  unpack<T>(dy, g);
  unpack<T>(z, zz);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const float gv = fmaf(zz[j], sc[j], sh[j]) > 0.f ? g[j] : 0.f;
    o[j] = fmaf(al[j], gv, fmaf(gz[j], zz[j], be[j]));
  }
  return packv<T>(o);
}

// ---- dropout keep-mask: a pure function of (seed, NCHW linear index) -------------------------
// Must match oracle/fast_scnn_ref.py:dropout_mask bit for bit.
// keep iff (hash >> 40) >= thr, thr = ceil(p * 2^24)  (<=> 24-bit uniform u >= p)
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t idx, uint32_t thr) {
  uint64_t z = idx * 0x9E3779B97F4A7C15ull + seed;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (uint32_t)(z >> 40) >= thr;
}
// Channel-owning sweeps (bn_bwd_apply, dropout): each thread keeps ONE channel vector's tables
// in registers and visits pixels p0, p0 + P, ...; P = pixels per grid sweep.  Up to 8 pixels per
// thread amortise the tables, while the grid keeps >= 1024 workgroups (4 per CU) when the tensor
// has that much work (measured r04, cfg3 step: 1024 -> 5.786 ms, 2048 -> 5.804, 4096 -> 5.835;
// a cap of 16 pixels per thread: no change).
inline unsigned chan_sweep(long long M, int CV) {
  long long ppt = M * CV / (1024LL * 256);
  ppt = ppt < 1 ? 1 : (ppt > 8 ? 8 : ppt);
  return (unsigned)((M + ppt - 1) / ppt);
}
inline uint32_t dropout_threshold(float p) {
  double t = (double)p * 16777216.0;
  uint32_t k = (uint32_t)t;
  return ((double)k < t) ? k + 1 : k;
}

// ---- align_corners=True source index (aten compute_source_index_and_lambda) ------------------
struct Lerp {
  int i0, i1;
  float l0, l1;
};
// l0 * a + l1 * b as ONE explicit form, fma(l0, a, round(l1 * b)): left to the compiler, the
// expression is contracted differently per kernel (hipcc's default -ffp-contract=fast applies to
// __fmul_rn / __fadd_rn too), and a 1-ulp difference between up_nchw and up_argmax flipped a
// cfg2 near-tie label; every kernel that evaluates the same bilinear tap pair now gets the same bits
__device__ __forceinline__ float lerp2(float l0, float a, float l1, float b) {
  return fmaf(l0, a, l1 * b);
}
__host__ __device__ __forceinline__ float ac_scale(int in, int out) {
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.0f;
}
__host__ __device__ __forceinline__ Lerp ac_lerp(int o, int in, int out, float scale) {
  Lerp r;
  if (in == out) {
    r.i0 = o; r.i1 = o; r.l0 = 1.0f; r.l1 = 0.0f;
    return r;
  }
  float real = scale * (float)o;
  int i0 = (int)floorf(real);
  if (i0 > in - 1) i0 = in - 1;
  float lam = real - (float)i0;
  lam = lam < 0.f ? 0.f : (lam > 1.f ? 1.f : lam);
  r.i0 = i0;
  r.i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  r.l1 = lam;
  r.l0 = 1.0f - lam;
  return r;
}

// ---- error reporting ----------------------------------------------------------------------------
void set_error(const char* fmt, ...);
const char* last_error();
int check_launch(const char* what);

enum Status : int { OK = 0, E_INVALID = -1, E_UNSUPPORTED = -2, E_HIP = -3 };

// ---- in-library launch profiler (bench.py roofline: HIP events on the launch stream) ---------
enum ProfKind : int {
  PK_NONE = 0, PK_CONV0_FWD, PK_DW_FWD, PK_DW_DGRAD, PK_DW_WGRAD, PK_GEMM_NT, PK_GEMM_TN,
  PK_BN_APPLY, PK_BN_BWD, PK_UP, PK_UP_BWD, PK_CE, PK_CONV0_WGRAD, PK_BN_BWD_RED, PK_BN_FIN,
  PK_PPM, PK_IR, PK_STEM, PK_DSCONV, PK_COUNT
};
constexpr int PK_ALL = 100;  // record every kind (per-launch layer report)
extern int g_prof_kind;  // kind being recorded (PK_NONE = off)
// layer the executor is issuing (per-launch report label); per thread: DataParallel replicas
// (train.py:170-171) run the executor from one worker thread per device
extern thread_local const char* g_prof_tag;
void prof_start(hipStream_t st);
void prof_stop(hipStream_t st, int kind, double bytes, double flops);
struct ProfScope {
  bool on;
  int kind;
  hipStream_t st;
  double bytes, flops;
  ProfScope(int k, hipStream_t s, double b, double f)
      : on(g_prof_kind == k || (g_prof_kind == PK_ALL && k != PK_NONE)), kind(k), st(s), bytes(b),
        flops(f) {
    if (on) prof_start(st);
  }
  ~ProfScope() {
    if (on) prof_stop(st, kind, bytes, flops);
  }
};

// Every kernel launch goes through prof_launch.  Inside a recording ProfScope the scope's first
// launch is issued by hipExtLaunchKernelGGL with the scope's event pair bound to the dispatch
// itself: the events carry the kernel's own start / end timestamps (what rocprofv3's kernel trace
// reads), not marker packets around it (each of which idles the stream ~7 us).  Otherwise it is a
// plain launch.
bool prof_take_ext(hipEvent_t& e0, hipEvent_t& e1);
// FSCNN_HOST_PROF=1 (diagnostics): host time spent in launches / stream forks, printed at exit
extern bool g_host_prof;
void host_prof_add(int what, double us);
double host_now_us();
template <typename F, typename... A>
inline void prof_launch(F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st, A... args) {
  hipEvent_t e0, e1;
  const double t0 = g_host_prof ? host_now_us() : 0.0;
  if (prof_take_ext(e0, e1))
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, st, e0, e1, 0u, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, lds, st, args...);
  if (g_host_prof) host_prof_add(0, host_now_us() - t0);
}

__host__ __device__ inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// ---- buffer operations: 32-bit offsets, range-checked (an out-of-range lane loads 0 / stores
// nothing), so edge handling needs no branch and a launch's memory-op count per step is fixed
constexpr uint32_t BUF_OOB = 0x80000000u;       // a buffer offset past every range
typedef unsigned int buf_v4u __attribute__((__vector_size__(16)));
typedef unsigned int buf_v2u __attribute__((__vector_size__(8)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[4],
                                       float*) {
  const buf_v4u t = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                   __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(t, r, off, 0, 0);
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[4],
                                       bf16*) {
  const buf_v2u t = {(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                   (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
  __builtin_amdgcn_raw_buffer_store_b64(t, r, off, 0, 0);
}
__device__ __forceinline__ void buf_st4(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[4],
                                       f16*) {
  const buf_v2u t = {(uint32_t)f2h(v[0]) | ((uint32_t)f2h(v[1]) << 16),
                   (uint32_t)f2h(v[2]) | ((uint32_t)f2h(v[3]) << 16)};
  __builtin_amdgcn_raw_buffer_store_b64(t, r, off, 0, 0);
}

// ---- phase stamps (tools/stamp_probe.py; off unless fscnn_debug_stamps set a buffer) ----------
// Lane 0 of every wave records the 100 MHz wall clock at numbered points of a kernel into
// stamps[(block * 4 + wave) * STAMP_SLOTS + slot] (vector stores): where a launch's time goes.
// Every instrumented launch takes its own STAMP_STRIDE region (stamp_region) and a layer label.
constexpr int STAMP_SLOTS = 8;
constexpr long long STAMP_STRIDE = 8192LL * 4 * STAMP_SLOTS;
extern unsigned long long* g_stamps;  // device buffer of the next launches, or null
unsigned long long* stamp_region();   // host: the next launch's region (null: off / full)
__device__ __forceinline__ void stamp(unsigned long long* st, int slot) {
  if (st && (threadIdx.x & 63) == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const size_t b = blockIdx.x + (size_t)gridDim.x * (blockIdx.y + (size_t)gridDim.y * blockIdx.z);
    if (b < 8192 && (threadIdx.x >> 6) < 4) {  // (waves 0-3 of larger workgroups)
      st[(b * 4 + (threadIdx.x >> 6)) * STAMP_SLOTS + slot] = t;
      if (slot == 0) {  // placement of the wave: XCC id << 32 | HW_ID (CU, SIMD, SE) in slot 7
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        st[(b * 4 + (threadIdx.x >> 6)) * STAMP_SLOTS + 7] = ((unsigned long long)(xcc & 15) << 32) | hw;
      }
    }
  }
}

}  // namespace fscnn
