// Streaming pointwise GEMM: C[m][n] = epi(sum_k A[m][k] * W[n][k]) for every 1x1 conv whose
// weight slice fits in LDS (K <= 128 fp32 / <= 256 bf16-fp16): models/fast_scnn.py :73 DSConv pw,
// :103 expand, :124-128 PPM, :198/:202 FFM, :230 classifier, and the dgrads of those shapes
// (the executor's dgrad reads a per-step transposed weight copy, so it is the same NT GEMM).
//
// Same contract as gemm_nt (kernels.hpp GemmArgs).  Why a second kernel: at M = 262,144 pixels
// and K = 64-128 the tiled gemm_nt spends as long in its LDS-staged A tile and block-wide
// epilogue as in MFMA.  Here
//   * a workgroup owns one column group (16*NT output channels) and keeps that group's weights
//     [16*NT][K] in LDS for its whole life (loaded once);
//   * each wave streams its own 32-pixel chunks straight from HBM into registers (lane (li, lq)
//     loads pixel li's k-vector lq of every k-step: one 16-B load per MFMA operand), with no
//     workgroup barrier in the loop; the next chunk's loads are in flight during this chunk's
//     MFMAs (register double buffer), and tail masks / the lazy BN are applied at the use site;
//   * the MFMA operands are swapped (weights as the A operand), so each lane's accumulator holds
//     4 CONSECUTIVE output channels of one pixel: the epilogue runs in registers and stores
//     16-B (fp32) / 8-B (16-bit) NHWC vectors directly.
// Training forms (template flags):
//   AT  the A operand is the raw conv output z of a BN+ReLU that is never stored; the GEMM
//       consumes relu(fmaf(z, a_scale[k], a_shift[k])) (bn_apply's arithmetic, bit-identical);
//   ST  per-channel BN statistics of the output: each lane keeps shifted sums (shift = the
//       channel's value at the wave's first pixel, broadcast) over its pixels; at the end the
//       lanes (xor butterfly, fixed order) and the 4 waves (Chan merge, fixed order) are folded
//       into ONE (mean, M2, count) record per workgroup -> part[bi][3][N] (bi < bpg, the
//       workgroup's index within its column group; gemm_stream_parts reports bpg);
//   BS  dgrad producing the dy of a BN: per-channel sum(g*mask), sum(g*mask*xhat) of the stored
//       (rounded) output, the mask recomputed from that BN's z -> bpart[bi][2][N].
// The k summation order inside a 16x16xK MFMA step matches gemm_nt (4-element k quads for fp32,
// 8-element for 16-bit, steps in increasing k).
#include "bn_finish.hpp"

namespace fscnn {

constexpr int GS_MW = 32;     // pixels per wave chunk (2 x 16-row MFMA tiles)
constexpr int GS_KMAX = 576;  // largest K of a lazily normalised (AT) A operand

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

// sum over the 16 lanes li of a 16-lane row (xor butterfly: every lane ends with the same sum)
__device__ __forceinline__ float gs_rowsum(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

// In-kernel BN finish (GemmArgs::tail).  Two arrival levels keep every fold one batch of loads
// deep (a single finisher walking all bpg <= 512 records was a chain of ~25 dependent sc1 round
// trips): workgroups arrive in teams of GS_TEAM; a team's last arriver folds the team's records
// into the team's first slot (in place, write-through) and arrives on the column group's
// counter; the group's last arriver folds the team records and finishes each channel with the
// finalize kernels' arithmetic (bn_finish.hpp).  Folds are fp64 sums in fixed order (thread
// slice sl takes records sl, sl + S, ... in increasing order; slices summed in order).
constexpr int GS_TEAM = 16;
constexpr int GS_CTR_TEAMS = 64;  // counters: [0, 64) groups, then cdiv(bpg, GS_TEAM) teams per group

template <bool FWD>
__device__ inline void gs_fold(const GemmArgs& a, int n0, int BN, int first, int count, int stride,
                               double (&sum)[3]) {
  __shared__ double s_f[3][256];
  const int tid = threadIdx.x;
  const int S = 256 / BN;
  const int col = tid % BN, sl = tid / BN;
  const int n = n0 + col;
  const int N = a.N;
  const float* base = FWD ? a.part : a.bpart;
  constexpr int R = FWD ? 3 : 2;
  constexpr int U = FWD ? 8 : 4;  // records per thread per batch (all loads issued before the sums)
  double t0 = 0.0, t1 = 0.0, t2 = 0.0;
  if (sl < S && n < N) {
    for (int i0 = sl; i0 < count; i0 += U * S) {
      float v[U][R];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * S;
        const float* rec = base + (size_t)(first + (i < count ? i : i0) * stride) * R * N;
#pragma unroll
        for (int j = 0; j < R; ++j) v[u][j] = ld_wt(rec + (size_t)j * N + n);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i0 + u * S >= count) break;
        if constexpr (FWD) {  // (mean, M2, count) -> (n, n*mean, M2 + n*mean^2)
          const double cn = v[u][2], m = v[u][0];
          t0 += cn;
          t1 += cn * m;
          t2 += (double)v[u][1] + cn * m * m;
        } else {
          t1 += v[u][0];
          t2 += v[u][1];
        }
      }
    }
  }
  s_f[0][tid] = t0;
  s_f[1][tid] = t1;
  s_f[2][tid] = t2;
  __syncthreads();
  sum[0] = sum[1] = sum[2] = 0.0;
  if (sl == 0) {
    for (int j = 0; j < S; ++j) {
      sum[0] += s_f[0][j * BN + col];
      sum[1] += s_f[1][j * BN + col];
      sum[2] += s_f[2][j * BN + col];
    }
  }
  __syncthreads();  // s_f reusable by the next fold
}

template <bool FWD>
__device__ inline void gs_finish(const GemmArgs& a, int g, int bi, int n0, int BN, int bpg) {
  unsigned* ctr = a.tail.counters;
  const int team = bi / GS_TEAM, nteam = cdiv(bpg, GS_TEAM);
  const int tsize = min(GS_TEAM, bpg - team * GS_TEAM);
  const int tid = threadIdx.x, col = tid % BN, n = n0 + col;
  const bool owner = tid < BN && n < a.N;  // slice 0 holds the folded sums
  if (!arrive_last(ctr + GS_CTR_TEAMS + g * nteam + team, (unsigned)tsize)) return;
  // the finish's per-channel inputs, in flight with the team fold (one round trip off the chain
  // of the group's last workgroup)
  BnFwdIn fin;
  BnBwdIn bin;
  if (owner) {
    if constexpr (FWD) fin = bn_fwd_load(a.tail.fwd, n);
    else bin = bn_bwd_load(a.tail.tab, n);
  }
  double s[3];
  gs_fold<FWD>(a, n0, BN, team * GS_TEAM, tsize, 1, s);
  if (owner) {  // the team record replaces slot team * GS_TEAM (every other reader is done)
    const int N = a.N;
    if constexpr (FWD) {
      float* rec = a.part + (size_t)team * GS_TEAM * 3 * N;
      const double mean = s[0] > 0.0 ? s[1] / s[0] : 0.0;
      st_wt(rec + n, (float)mean);
      st_wt(rec + N + n, s[0] > 0.0 ? (float)fmax(s[2] - s[0] * mean * mean, 0.0) : 0.f);
      st_wt(rec + 2 * N + n, (float)s[0]);
    } else {
      float* rec = a.bpart + (size_t)team * GS_TEAM * 2 * N;
      st_wt(rec + n, (float)s[1]);
      st_wt(rec + N + n, (float)s[2]);
    }
  }
  reset_counter(ctr + GS_CTR_TEAMS + g * nteam + team);
  if (!arrive_last(ctr + g, (unsigned)nteam)) return;
  gs_fold<FWD>(a, n0, BN, 0, nteam, GS_TEAM, s);
  if (owner) {
    if constexpr (FWD) bn_fwd_finish(a.tail.fwd, n, s[0], s[1], s[2], fin);
    else bn_bwd_finish(n, a.N, s[1], s[2], a.tail.count, a.tail.dgamma, a.tail.dbeta,
                       a.tail.coef, a.tail.tab, bin);
  }
  reset_counter(ctr + g);
}

// NT: 16-column MFMA tiles per group; KS: k-steps (16 fp32 / 32 16-bit k each) covering K
template <typename T, int NT, int KS, bool TAIL, bool AT, bool ST, bool BS>
__global__ __launch_bounds__(256, 2) void gemm_stream_kernel(GemmArgs a, int bpg) {
  constexpr int V = VecW<T>::V;     // elements per 16-B vector
  constexpr int KV = 4 * KS;        // 16-B vectors per weight row (4 per k-step)
  constexpr int KP = KV * V;        // K padded to whole k-steps
  constexpr int WST = KV + 1;       // padded LDS row stride (vectors): conflict-free b128 reads
  constexpr int BN = 16 * NT;
  constexpr bool SUMS = ST || BS;
  extern __shared__ __attribute__((aligned(16))) uint4 s_w[];  // [BN][WST]
  float* s_sc = reinterpret_cast<float*>(s_w + BN * WST);       // [BN] scale, [BN] shift
  float* s_at = s_sc + 2 * BN;                                  // AT: [KP] scale, [KP] shift
  float* s_bc = s_at + (AT ? 2 * KP : 0);                       // BS: [4][BN] mean/istd/sc/sh
  float* s_shf = s_bc + (BS ? 4 * BN : 0);                       // ST: [4 waves][BN] shifts

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  // block -> (group, index within group) = blockIdx / bpg; bpg % 8 == 0 (when not capped) keeps
  // the blocks that stream the same pixel chunks for different groups on one XCD (shared A in L2)
  const int g = blockIdx.x / bpg;
  const int bi = blockIdx.x - g * bpg;
  const int n0 = g * BN;
  const T* A = (const T*)a.A;
  const T* B = (const T*)a.B;
  stamp(a.stamps, 0);

  const int nchunks = cdiv(a.M, GS_MW);
  const int wstride = bpg * 4;
  int c = bi * 4 + wave;

  // Software pipeline over K-parts: a chunk's k-steps are loaded as NH parts of KH steps (a
  // whole chunk double-buffered would pass 256 VGPRs for K > 4 steps), and each part's loads are
  // in flight while the previous part computes — the next chunk's first part during this
  // chunk's last part (NH > 1) or during all of it (NH = 1).  Even parts live in xa, odd in xn.
  constexpr int NH =
      KS <= 4 ? 1 : (KS <= 8 ? 2 : (KS == 12 ? (BS ? 4 : 2) : (KS == 16 ? 4 : 6)));
  constexpr int KH = KS / NH;
  static_assert(KH * NH == KS && (NH == 1 || NH % 2 == 0), "k-steps split in an even part count");
  // k-vector (4*s + lq), s in half h, of pixel rows li, 16 + li -> r[mt][j] (raw, clamped loads)
  uint4 xa[2][KH], xn[2][KH];
  auto loadx = [&](int chunk, int h, uint4 (&r)[2][KH]) {
    const bool cok = chunk < nchunks;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = chunk * GS_MW + mt * 16 + li;
      const bool mok = cok && m < a.M;
#pragma unroll
      for (int j = 0; j < KH; ++j) {
        const int k = (4 * (h * KH + j) + lq) * V;
        const bool ok = mok && k < a.K;
        r[mt][j] = *reinterpret_cast<const uint4*>(A + (ok ? (size_t)m * a.lda + k : 0));
      }
    }
  };

  // ---- weights of the group -> LDS (zero rows n >= N, zero k >= K), per-column tables -------
  // Every global load of the prologue — the first chunk's A part included — is issued before the
  // first LDS store, in batches of WB vectors per thread: the workgroup waits out one memory
  // round trip per batch instead of one per loop trip (the stores of a rolled loop each waited
  // on their own load; the A part then stays in flight across the barrier, which waits on LDS
  // only).
  if (c < nchunks) loadx(c, 0, xa);
  float t_sc = 1.f, t_sh = 0.f, t_bc[4] = {0.f, 0.f, 0.f, 1.f};
  if (tid < BN) {  // BN <= 128 < 256 threads: one column each
    const int n = n0 + tid < a.N ? n0 + tid : 0;
    if (a.scale) t_sc = a.scale[n];
    if (a.shift) t_sh = a.shift[n];
    if constexpr (BS) {
      // ReLU mask of that BN recomputed as fmaf(z, scale, shift) > 0 (mode 2); mode 0 (no
      // ReLU) uses scale 0, shift 1 so both are the same select
      t_bc[0] = a.bmean[n];
      t_bc[1] = a.binvstd[n];
      if (a.bmode == 2) {
        t_bc[2] = a.bscale[n];
        t_bc[3] = a.bshift[n];
      }
    }
  }
  constexpr int ATI = AT ? (KP + 255) / 256 : 1;
  float t_at[ATI][2];
  if constexpr (AT) {
#pragma unroll
    for (int u = 0; u < ATI; ++u) {
      const int k = tid + u * 256;
      const bool ok = k < a.K;
      t_at[u][0] = ok ? a.a_scale[k] : 0.f;
      t_at[u][1] = ok ? a.a_shift[k] : 0.f;
    }
  }
  constexpr int WI = (BN * KV + 255) / 256;  // weight vectors per thread
  constexpr int WB = WI < 8 ? WI : 8;
#pragma unroll
  for (int u0 = 0; u0 < WI; u0 += WB) {
    uint4 t[WB];
#pragma unroll
    for (int u = 0; u < WB; ++u) {
      const int i = tid + (u0 + u) * 256;
      const int r = i / KV, v = i - r * KV;
      const int n = n0 + r, k = v * V;
      const bool ok = u0 + u < WI && i < BN * KV && n < a.N && k < a.K;
      t[u] = gs_tail<T>(*reinterpret_cast<const uint4*>(B + (ok ? (size_t)n * a.ldb + k : 0)),
                        ok ? a.K - k : 0);
    }
#pragma unroll
    for (int u = 0; u < WB; ++u) {
      const int i = tid + (u0 + u) * 256;
      const int r = i / KV, v = i - r * KV;
      if (u0 + u < WI && i < BN * KV) s_w[r * WST + v] = t[u];
    }
  }
  if (tid < BN) {
    s_sc[tid] = t_sc;
    s_sc[BN + tid] = t_sh;
    if constexpr (BS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s_bc[j * BN + tid] = t_bc[j];
    }
  }
  if constexpr (AT) {
#pragma unroll
    for (int u = 0; u < ATI; ++u) {
      const int k = tid + u * 256;
      if (k < KP) {
        s_at[k] = t_at[u][0];
        s_at[KP + k] = t_at[u][1];
      }
    }
  }
  __syncthreads();
  stamp(a.stamps, 1);

  // sums of channels n0 + 16nt + 4lq + r over this lane's pixels (ST: shifted by shf)
  float s1[SUMS ? NT : 1][4], s2[SUMS ? NT : 1][4];
  float cnt = 0.f;
  if constexpr (SUMS) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[nt][r] = 0.f; s2[nt][r] = 0.f; }
  }
  // ST shift of each channel: its value at the wave's first pixel, kept in LDS (s_shf[wave])
  float* wshf = s_shf + wave * BN;
  if constexpr (ST) {
    for (int i = lane; i < BN; i += 64) wshf[i] = 0.f;
  }
  bool first = true;

  // at the use site: lazy BN+ReLU (AT), then the row / K-tail zeroing
  auto prep = [&](int chunk, int h, uint4 (&r)[2][KH]) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = chunk * GS_MW + mt * 16 + li;
      const bool mok = m < a.M;
#pragma unroll
      for (int j = 0; j < KH; ++j) {
        const int k = (4 * (h * KH + j) + lq) * V;
        uint4 v = r[mt][j];
        if constexpr (AT) v = bnrelu_vec<T>(v, s_at + k, s_at + KP + k);
        r[mt][j] = gs_tail<T>(v, mok ? a.K - k : 0);
      }
    }
  };

  T* Cp = (T*)a.C;
  const T* Rp = (const T*)a.R;
  // output dropout: compiled into the one-k-step dgrad-with-partials forms only (the classifier
  // conv's dgrad, K = classes <= 32); elsewhere its registers would spill the BS kernels
  constexpr bool DROP_OK = BS && KS == 1;
  const bool drop = DROP_OK && a.drop_hw != 0;
  const uint64_t dseed = drop ? (a.drop_seed_ptr ? *a.drop_seed_ptr : a.drop_seed) + a.drop_seed_add : 0;
  const float dscale = 1.f / (1.f - a.drop_p);
  for (; c < nchunks; c += wstride) {
    f32x4 acc[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the weight fragments are loop-invariant: launder the LDS base so they are re-read per
    // chunk (cheap ds_read_b128) instead of being hoisted into NT*KS*4 registers
    int wb = li * WST + lq;
    asm volatile("" : "+v"(wb));
    const int wz = wb - li * WST - lq;  // 0, opaque to the compiler
    const float* ssc = s_sc + wz;       // same laundering for the epilogue tables
    const float* sbc = s_bc + wz;
    auto mma = [&](int h, uint4 (&r)[2][KH]) {
#pragma unroll
      for (int j = 0; j < KH; ++j) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint4 w = s_w[wb + nt * 16 * WST + 4 * (h * KH + j)];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) GsMma<T>::run(w, r[mt][j], acc[mt][nt]);
        }
      }
    };
    if constexpr (NH == 1) {
      loadx(c + wstride, 0, xn);  // clamped past the end
      prep(c, 0, xa);
      mma(0, xa);
    } else {
#pragma unroll
      for (int h = 0; h < NH; h += 2) {
        loadx(c, h + 1, xn);
        prep(c, h, xa);
        mma(h, xa);
        if (h + 2 < NH) loadx(c, h + 2, xa);
        else loadx(c + wstride, 0, xa);  // clamped past the end
        prep(c, h + 1, xn);
        mma(h + 1, xn);
      }
    }
    // ---- epilogue: lane holds channels n0 + 16nt + 4lq + r of pixel m ------------------------
    if constexpr (!TAIL) {  // whole 4-channel vectors, 16-B aligned rows (checked on the host)
      if constexpr (ST) {
        if (first) {  // per-channel shift: the value at the wave's first pixel (lane li = 0)
          if (li == 0) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
              const int nl = nt * 16 + 4 * lq;
#pragma unroll
              for (int r = 0; r < 4; ++r) wshf[nl + r] = acc[0][nt][r] * ssc[nl + r] + ssc[BN + nl + r];
            }
          }
          __builtin_amdgcn_wave_barrier();
          first = false;
        }
      }
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
        float zv[BS ? NT : 1][4];
        if constexpr (BS) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            ld4v((const T*)a.bz + mr * a.ldbz + n0 + nt * 16 + 4 * lq, zv[nt]);
        }
        if constexpr (SUMS) cnt += mok ? 1.f : 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int nl = nt * 16 + 4 * lq;
          const float4 sc = *reinterpret_cast<const float4*>(ssc + nl);
          const float4 sh = *reinterpret_cast<const float4*>(ssc + BN + nl);
          const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, shv[4] = {sh.x, sh.y, sh.z, sh.w};
          float shf[4] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (ST) {
            const float4 t = *reinterpret_cast<const float4*>(wshf + wz + nl);
            shf[0] = t.x; shf[1] = t.y; shf[2] = t.z; shf[3] = t.w;
          }
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[mt][nt][r] * scv[r] + shv[r];
            if constexpr (ST) {  // statistics of the value as stored (gemm_nt's convention)
              const float d = mok ? round_as<T>(v) - shf[r] : 0.f;
              s1[nt][r] += d;
              s2[nt][r] += d * d;
            }
            if (Rp) v += rv[nt][r];
            o[r] = a.relu ? fmaxf(v, 0.f) : v;
          }
          if (DROP_OK && drop) {  // the dropout kernel's law on the stored value (misc.hip dropout_kernel)
            const unsigned HW = (unsigned)a.drop_hw;
            const unsigned pn = (unsigned)mr / HW, hw = (unsigned)mr - pn * HW;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint64_t nchw = ((uint64_t)pn * a.N + (unsigned)(n0 + nl + r)) * HW + hw;
              o[r] = dropout_keep(dseed, nchw, a.drop_thr) ? round_as<T>(o[r]) * dscale : 0.f;
            }
          }
          if (mok && Cp) st4v(Cp + mr * a.ldc + n0 + nl, o);  // (C null: statistics only)
          if constexpr (BS) {  // partials of the value as stored, masked by that BN's ReLU
            const float4 bm = *reinterpret_cast<const float4*>(sbc + nl);
            const float4 bv = *reinterpret_cast<const float4*>(sbc + BN + nl);
            const float4 bs = *reinterpret_cast<const float4*>(sbc + 2 * BN + nl);
            const float4 bh = *reinterpret_cast<const float4*>(sbc + 3 * BN + nl);
            const float bmv[4] = {bm.x, bm.y, bm.z, bm.w}, biv[4] = {bv.x, bv.y, bv.z, bv.w};
            const float bsv[4] = {bs.x, bs.y, bs.z, bs.w}, bhv[4] = {bh.x, bh.y, bh.z, bh.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float gv = round_as<T>(o[r]);
              gv = (mok && fmaf(zv[nt][r], bsv[r], bhv[r]) > 0.f) ? gv : 0.f;
              s1[nt][r] += gv;
              s2[nt][r] += gv * (zv[nt][r] - bmv[r]) * biv[r];
            }
          }
        }
      }
    } else {  // column tail / unaligned rows (the 19-class classifier): scalar, no statistics
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
            if (Cp) st1(Cp + (size_t)m * a.ldc + n, a.relu ? fmaxf(v, 0.f) : v);
          }
        }
      }
    }
    if constexpr (NH == 1) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int j = 0; j < KH; ++j) xa[mt][j] = xn[mt][j];
    }
  }

  stamp(a.stamps, 2);
  if constexpr (SUMS) {
    // ---- one record per workgroup: lanes (xor butterfly), then the 4 waves (fixed order) ----
    cnt = gs_rowsum(cnt);  // pixels of this wave (every lane row covers the same pixels)
    __syncthreads();       // every wave is done with s_w: reuse it as the reduction scratch
    float* red = reinterpret_cast<float*>(s_w);  // [4 waves][3][BN]
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t1 = gs_rowsum(s1[nt][r]), t2 = gs_rowsum(s2[nt][r]);
        if (li == 0) {
          const int col = nt * 16 + 4 * lq + r;
          if constexpr (ST) {  // (count, mean, M2) of the wave from its shifted sums
            const float mean = cnt > 0.f ? wshf[col] + t1 / cnt : 0.f;
            const float m2 = cnt > 0.f ? fmaxf(t2 - t1 * (t1 / cnt), 0.f) : 0.f;
            red[(wave * 3 + 0) * BN + col] = cnt;
            red[(wave * 3 + 1) * BN + col] = mean;
            red[(wave * 3 + 2) * BN + col] = m2;
          } else {
            red[(wave * 3 + 0) * BN + col] = t1;
            red[(wave * 3 + 1) * BN + col] = t2;
          }
        }
      }
    __syncthreads();
    for (int col = tid; col < BN; col += 256) {
      const int n = n0 + col;
      if (n >= a.N) continue;
      if constexpr (ST) {
        float nn = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {  // Chan merge of the 4 waves, fixed order
          const float nb = red[(w * 3 + 0) * BN + col];
          if (nb <= 0.f) continue;
          const float mb = red[(w * 3 + 1) * BN + col], qb = red[(w * 3 + 2) * BN + col];
          const float tot = nn + nb, d = mb - mean;
          mean += d * (nb / tot);
          m2 += qb + d * d * (nn * nb / tot);
          nn = tot;
        }
        float* rec = a.part + (size_t)bi * 3 * a.N;  // write-through: read by the finisher
        st_wt(rec + n, mean);
        st_wt(rec + a.N + n, m2);
        st_wt(rec + 2 * a.N + n, nn);
      } else {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          t1 += red[(w * 3 + 0) * BN + col];
          t2 += red[(w * 3 + 1) * BN + col];
        }
        float* rec = a.bpart + (size_t)bi * 2 * a.N;
        st_wt(rec + n, t1);
        st_wt(rec + a.N + n, t2);
      }
    }
    stamp(a.stamps, 3);
    // ---- in-kernel finish by the column group's last workgroup (no finalize launch) ---------
    if (a.tail.counters) gs_finish<ST>(a, g, bi, n0, BN, bpg);
    stamp(a.stamps, 4);
  }
}

// column tile: the dgrad partial sums also hold a z row (NT <= 4); the forward statistics fit
// NT = 6 (NT = 8 spills)
// ---- fp32 GEMMs on the bf16 matrix cores (inference plans) ---------------------------------
// An fp32 value splits EXACTLY into three bf16 terms by truncation, f = f0 + f1 + f2 (each
// term carries the next 8 of the 24 significand bits), so
//   a.w = a0w0 + (a0w1 + a1w0) + (a0w2 + a1w1 + a2w0) + O(2^-23 |a||w|)
// with the dropped terms (a1w2, a2w1, a2w2) below fp32's own product rounding.  Six
// v_mfma_f32_16x16x32_bf16 per 32-k step (fp32 accumulation) replace eight 16x16x4 fp32 MFMAs
// per 16-k step: 6 x 16 vs 16 x 32 cycles per 32 k, ~5x the fp32 matrix rate, which is what
// bounds the K = 64-128 fp32 1x1 convs of the eval forward (fp32 MFMA: ~157 TFLOP/s).
// Same tile scheme as gemm_stream_kernel; no training forms (statistics stay exact fp32).
// KS: 32-k steps covering K (<= 4: K <= 128)
template <int NT, int KS, bool TAIL>
__global__ __launch_bounds__(256, 2) void gemm_stream_x3_kernel(GemmArgs a, int bpg) {
  constexpr int KV = 4 * KS;   // bf16x8 vectors per weight row and plane
  constexpr int WST = KV + 1;  // padded row stride
  constexpr int BN = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) uint4 s_w[];  // [3][BN][WST]
  float* s_sc = reinterpret_cast<float*>(s_w + 3 * BN * WST);   // [BN] scale, [BN] shift
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int g = blockIdx.x / bpg;
  const int bi = blockIdx.x - g * bpg;
  const int n0 = g * BN;
  const float* A = (const float*)a.A;
  const float* B = (const float*)a.B;
  for (int i = tid; i < BN * KV; i += 256) {
    const int r = i / KV, v = i - r * KV;
    const int n = n0 + r, k = v * 8;
    const bool ok = n < a.N && k < a.K;
    const float* src = B + (ok ? (size_t)n * a.ldb + k : 0);
    const uint4 lo4 = gs_tail<float>(*reinterpret_cast<const uint4*>(src), ok ? a.K - k : 0);
    const uint4 hi4 = gs_tail<float>(*reinterpret_cast<const uint4*>(src + 4), ok ? a.K - k - 4 : 0);
    uint4 t[3];
    gs_split3(lo4, hi4, t);
#pragma unroll
    for (int j = 0; j < 3; ++j) s_w[(j * BN + r) * WST + v] = t[j];
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
  // lane (li, lq) holds k = 32 s + 8 lq .. +7 of pixel rows li, 16 + li: two 16-B loads
  uint4 xa[2][KS][2], xn[2][KS][2];
  auto loadx = [&](int chunk, uint4 (&r)[2][KS][2]) {
    const bool cok = chunk < nchunks;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = chunk * GS_MW + mt * 16 + li;
      const bool mok = cok && m < a.M;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 32 * s + 8 * lq + 4 * h;
          const bool ok = mok && k < a.K;
          r[mt][s][h] = *reinterpret_cast<const uint4*>(A + (ok ? (size_t)m * a.lda + k : 0));
        }
    }
  };
  float* Cp = (float*)a.C;
  const float* Rp = (const float*)a.R;
  if (c < nchunks) loadx(c, xa);
  for (; c < nchunks; c += wstride) {
    loadx(c + wstride, xn);  // clamped past the end
    f32x4 acc[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    int wb = li * WST + lq;
    asm volatile("" : "+v"(wb));
    const float* ssc = s_sc + (wb - li * WST - lq);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      uint4 xs[2][3];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int m = c * GS_MW + mt * 16 + li;
        const bool mok = m < a.M;
        const int k = 32 * s + 8 * lq;
        gs_split3(gs_tail<float>(xa[mt][s][0], mok ? a.K - k : 0),
                  gs_tail<float>(xa[mt][s][1], mok ? a.K - k - 4 : 0), xs[mt]);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        uint4 w[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) w[j] = s_w[(j * BN + nt * 16) * WST + wb + 4 * s];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) gs_mma_x3(w, xs[mt], acc[mt][nt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = c * GS_MW + mt * 16 + li;
      const bool mok = m < a.M;
      const size_t mr = mok ? (size_t)m : 0;
      if constexpr (!TAIL) {
        float rv[NT][4];
        if (Rp) {
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) ld4v(Rp + mr * a.ldr + n0 + nt * 16 + 4 * lq, rv[nt]);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int nl = nt * 16 + 4 * lq;
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[mt][nt][r] * ssc[nl + r] + ssc[BN + nl + r];
            if (Rp) v += rv[nt][r];
            o[r] = a.relu ? fmaxf(v, 0.f) : v;
          }
          if (mok) st4v(Cp + mr * a.ldc + n0 + nl, o);
        }
      } else {
        if (!mok) continue;
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
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) xa[mt][s][h] = xn[mt][s][h];
  }
}

// eval-form fp32 GEMM on the bf16 matrix cores: FSCNN_F32_SPLIT=0 keeps exact fp32 MFMA
static bool gs_x3_on() {
  static const bool on = [] {
    const char* e = getenv("FSCNN_F32_SPLIT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The largest column tile count of the statistics forms above N = 64: 4.  Their per-lane
// shifted sums (8 NT registers) put the NT = 6 form at 256 VGPRs (2 waves per SIMD); measured
// r06, cfg3 bf16, same box, two pairs: cap 4 5.777 / 5.771 ms per step, NT = 6 (the previous
// choice for N % 96 == 0) 5.786 / 5.780, cap 3 5.841 / 5.808, cap 2 5.860 / 5.863.
// FSCNN_GS_ST_NT overrides it (tuning A/B; 0: no cap).
static int gs_st_nt_cap() {
  static const int v = [] {
    const char* e = getenv("FSCNN_GS_ST_NT");
    return e ? atoi(e) : 4;
  }();
  return v;
}

static int gs_pick_nt(const GemmArgs& a, int ks) {
  const int N = a.N;
  if (N <= 32) return 2;
  if (a.part && ks <= 8 && N > 64 && gs_st_nt_cap() > 0) {
    for (int nt = gs_st_nt_cap(); nt >= 2; --nt)
      if (N % (16 * nt) == 0) return nt;
  }
  if (ks > 8) return N % 64 == 0 ? 4 : (N % 48 == 0 ? 3 : 4);  // deep K: weights [<=64][K] in LDS
  if (N <= 48) return 3;
  if (N <= 64 || a.bpart) return 4;
  // statistics forms with ks > 2 cannot hold 6 column tiles in 256 VGPRs: 4 when N allows
  if (a.part && ks > 2 && N % 64 == 0) return 4;
  if (N % 96 == 0) return 6;
  return a.part ? 4 : 8;
}

static bool gs_tail_needed(const GemmArgs& a, int nt) {
  return a.N % (16 * nt) != 0 || a.ldc % 4 != 0 || (a.R && a.ldr % 4 != 0);
}

static size_t gs_lds(const GemmArgs& a, int nt, int ks, int kc) {
  size_t b = (size_t)16 * nt * (4 * ks + 1) * 16 + (size_t)2 * 16 * nt * 4;
  if (a.a_scale) b += (size_t)2 * ks * kc * 4;
  if (a.bpart) b += (size_t)4 * 16 * nt * 4;
  if (a.part) b += (size_t)4 * 16 * nt * 4;
  return b;  // >= the end-of-kernel reduction scratch [4][3][16 nt] (aliases the weights)
}

static int gs_bpg(const GemmArgs& a, int dtype, int& nt, int& ks, size_t& lds);

bool gemm_stream_ok(const GemmArgs& a, int dtype) {
  const int KC = dtype == DT_F32 ? 16 : 32;  // k per step
  const int ks = cdiv(a.K, KC);
  const bool sums = a.part || a.bpart;
  if (a.b_trans || (a.part && a.bpart)) return false;
  if (a.part && a.R) return false;
  // lazy BN on A: train-forward producers only (always with statistics)
  if (a.a_scale && (!a.a_shift || !a.part || a.K > GS_KMAX)) return false;
  // deep K (K = 384 / 512 / 576 16-bit: the projects and the expand dgrads) streams the chunk
  // in 2-6 register parts against a <= 64-column weight slice of up to 75 KB
  const bool deep = ks == 12 || ks == 16 || ks == 18;
  if (deep && dtype == DT_F32) return false;
  // (measured: at M <= 65536 each wave streams one or two chunks and the part-by-part load chain
  //  is slower than the tiled kernel; at M = 262,144, e.g. bottleneck1.0's expand dgrad, 10% faster)
  if (deep && a.M < 131072) return false;
  if (!(ks == 1 || ks == 2 || ks == 3 || ks == 4 || ks == 6 || ks == 8 || deep)) return false;
  const int nt = gs_pick_nt(a, ks);
  // keep the statistics forms within 256 VGPRs (measured: these would spill)
  if (sums && ks > 4 && nt > 4) return false;
  if (sums && nt == 4 && ks > 12) return false;
  if (a.part && nt > 4 && ks > 2) return false;
  if (a.bpart && dtype == DT_F32 && nt == 4 && ks > 2) return false;  // would spill
  if (gs_tail_needed(a, nt) && (nt != 2 || sums)) return false;  // scalar tail: N <= 32 only
  if (a.bpart && (!a.bz || a.ldbz % 4 || (a.bmode != 0 && a.bmode != 2))) return false;
  if (a.drop_hw && (!a.bpart || ks != 1 || gs_tail_needed(a, nt) || a.M % a.drop_hw)) return false;
  // two resident workgroups per CU (160 KB LDS, 1 KB reserved each)
  if (gs_lds(a, nt, ks, KC) > (deep ? 80 * 1024 - 1024 : 72 * 1024)) return false;
  // in-kernel BN finish: group counters [0, 64), then each group's team counters
  if (a.tail.counters) {
    int nt2, ks2;
    size_t lds2;
    const int bpg = gs_bpg(a, dtype, nt2, ks2, lds2);
    const int groups = cdiv(a.N, 16 * nt);
    if (groups > GS_CTR_TEAMS || GS_CTR_TEAMS + groups * cdiv(bpg, GS_TEAM) > BN_COUNTERS)
      return false;
  }
  return a.M >= 4096;  // tiny GEMMs (PPM bins): loading a weight slice per block does not pay
}

// workgroups per column group for `slots` resident workgroups shared by `groups` column groups:
// a multiple of 8 (XCD-aligned) that does not oversubscribe the slots.  The chunks are assigned
// statically (c += wstride), so workgroups past the resident slots run as a second round:
// rounding up (9 groups: 64 x 9 = 576 > 512) put 64 workgroups of every 576- / 768- /
// 384-channel launch there (measured: cfg3 step 6.62 -> 6.54 ms with this rounding down)
static int gs_fill_bpg(int slots, int groups) {
  const int b = slots / groups / 8 * 8;
  return b >= 8 ? b : (cdiv(slots, groups) + 7) / 8 * 8;
}

// workgroups per column group = the record count of the statistics forms
static int gs_bpg(const GemmArgs& a, int dtype, int& nt, int& ks, size_t& lds) {
  const int KC = dtype == DT_F32 ? 16 : 32;
  ks = cdiv(a.K, KC);
  nt = gs_pick_nt(a, ks);
  const int groups = cdiv(a.N, 16 * nt);
  lds = gs_lds(a, nt, ks, KC);
  const int nchunks = cdiv(a.M, GS_MW);
  // resident workgroups: LDS-limited (160 KB / CU), at most 2 per CU (measured: 3-4 slower)
  // (r04: the low-M dgrads with BN-backward partials at NT = 2 and 3 per CU measured equal)
  constexpr int cap = 2;
  int per_cu = (int)((160 * 1024) / (lds + 1024));
  per_cu = per_cu < 1 ? 1 : (per_cu > cap ? cap : per_cu);
  // (2 or 4 rounds of resident workgroups instead of one, for dynamic balance: measured r05
  //  6.16 / 6.50 vs 5.78 ms per cfg3 step -- each extra round pays the prologue and records again)
  int bpg = gs_fill_bpg(256 * per_cu, groups);
  const int need = cdiv(nchunks, 4);  // <= cdiv(M, 128) = gemm_parts(M): fits the record slots
  if (bpg > need) bpg = need;
  // the finish's team counters: [GS_CTR_TEAMS, BN_COUNTERS) shared by the groups
  const int tmax = (BN_COUNTERS - GS_CTR_TEAMS) / groups * GS_TEAM;
  if (bpg > tmax) bpg = tmax;
  if (bpg < 1) bpg = 1;
  return bpg;
}

int gemm_stream_parts(const GemmArgs& a, int dtype) {
  int nt, ks;
  size_t lds;
  return gs_bpg(a, dtype, nt, ks, lds);
}

template <typename T, int NT, bool TAIL, bool AT, bool ST, bool BS>
static void gs_launch_ks(const GemmArgs& a, int ks, dim3 grid, size_t lds, int bpg,
                         hipStream_t st) {
  constexpr bool SUMS = ST || BS;
  constexpr bool WIDE = SUMS && NT > 4;  // wide statistics tiles: K <= 2 k-steps only
  constexpr bool DEEP = sizeof(T) == 2 && NT <= 4 && !TAIL;
  switch (ks) {
    case 1: prof_launch(gemm_stream_kernel<T, NT, 1, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg); break;
    case 2: prof_launch(gemm_stream_kernel<T, NT, 2, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg); break;
    case 3:
      if constexpr (!WIDE) prof_launch(gemm_stream_kernel<T, NT, 3, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
      break;
    case 4:
      if constexpr (!WIDE) prof_launch(gemm_stream_kernel<T, NT, 4, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
      break;
    case 6:
      if constexpr (!WIDE) prof_launch(gemm_stream_kernel<T, NT, 6, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
      break;
    case 8:
      if constexpr (!WIDE) prof_launch(gemm_stream_kernel<T, NT, 8, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
      break;
    default:  // deep K: 16-bit, <= 4 column tiles, no scalar tail
      if constexpr (DEEP) {
        if (ks == 12) prof_launch(gemm_stream_kernel<T, NT, 12, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
        else if (ks == 16) prof_launch(gemm_stream_kernel<T, NT, 16, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
        else prof_launch(gemm_stream_kernel<T, NT, 18, TAIL, AT, ST, BS>, grid, 256, lds, st, a, bpg);
      }
      break;
  }
}

template <typename T, bool AT, bool ST, bool BS>
static void gs_launch_nt(const GemmArgs& a, int nt, int ks, dim3 grid, size_t lds, int bpg,
                         hipStream_t st) {
  constexpr bool SUMS = ST || BS;
  switch (nt) {
    case 2:
      if (!SUMS && gs_tail_needed(a, nt)) gs_launch_ks<T, 2, true, AT, false, false>(a, ks, grid, lds, bpg, st);
      else gs_launch_ks<T, 2, false, AT, ST, BS>(a, ks, grid, lds, bpg, st);
      break;
    case 3: gs_launch_ks<T, 3, false, AT, ST, BS>(a, ks, grid, lds, bpg, st); break;
    case 4: gs_launch_ks<T, 4, false, AT, ST, BS>(a, ks, grid, lds, bpg, st); break;
    case 6:
      if constexpr (!BS) gs_launch_ks<T, 6, false, AT, ST, false>(a, ks, grid, lds, bpg, st);
      break;
    default:
      if constexpr (!SUMS) gs_launch_ks<T, 8, false, AT, false, false>(a, ks, grid, lds, bpg, st);
      break;
  }
}

template <typename T>
static void gs_launch(const GemmArgs& a, int dtype, hipStream_t st) {
  int nt, ks;
  size_t lds;
  const int bpg = gs_bpg(a, dtype, nt, ks, lds);
  const int groups = cdiv(a.N, 16 * nt);
  dim3 grid((unsigned)(groups * bpg));
  const bool at = a.a_scale != nullptr;
  if (a.bpart) gs_launch_nt<T, false, false, true>(a, nt, ks, grid, lds, bpg, st);
  else if (a.part && at) gs_launch_nt<T, true, true, false>(a, nt, ks, grid, lds, bpg, st);
  else if (a.part) gs_launch_nt<T, false, true, false>(a, nt, ks, grid, lds, bpg, st);
  else gs_launch_nt<T, false, false, false>(a, nt, ks, grid, lds, bpg, st);
}

// fp32 eval GEMMs with K <= 128 on the bf16 matrix cores (gemm_stream_x3_kernel): the widest
// column tile whose three weight planes fit 72 KB of LDS
static bool gs_x3_launch(const GemmArgs& a, hipStream_t st) {
  if (!gs_x3_on() || a.part || a.bpart || a.a_scale || a.K > 128) return false;
  const int ks = cdiv(a.K, 32);
  auto lds_of = [&](int nt) { return (size_t)3 * 16 * nt * (4 * ks + 1) * 16 + (size_t)2 * 16 * nt * 4; };
  int nt = gs_pick_nt(a, ks);
  while (nt > 2 && lds_of(nt) > 72 * 1024) nt = nt == 8 ? 4 : (nt == 6 ? 3 : 2);
  if (lds_of(nt) > 72 * 1024) return false;
  const bool tail = gs_tail_needed(a, nt);
  if (tail && nt != 2) return false;
  const size_t lds = lds_of(nt);
  const int groups = cdiv(a.N, 16 * nt);
  int per_cu = (int)((160 * 1024) / (lds + 1024));
  per_cu = per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu);
  int bpg = gs_fill_bpg(256 * per_cu, groups);
  const int need = cdiv(cdiv(a.M, GS_MW), 4);
  if (bpg > need) bpg = need;
  if (bpg < 1) bpg = 1;
  const dim3 grid((unsigned)(groups * bpg));
#define X3(NT, KS, TL) prof_launch(gemm_stream_x3_kernel<NT, KS, TL>, grid, 256, lds, st, a, bpg)
#define X3K(NT, TL)                         \
  switch (ks) {                             \
    case 1: X3(NT, 1, TL); break;           \
    case 2: X3(NT, 2, TL); break;           \
    case 3: X3(NT, 3, TL); break;           \
    default: X3(NT, 4, TL); break;          \
  }
  switch (nt) {
    case 2: if (tail) { X3K(2, true) } else { X3K(2, false) } break;
    case 3: X3K(3, false) break;
    case 4: X3K(4, false) break;
    case 6: X3K(6, false) break;
    default: X3K(8, false) break;
  }
#undef X3K
#undef X3
  return true;
}

int gemm_stream(const GemmArgs& a, int dtype, hipStream_t st) {
  if (dtype == DT_F32) {
    if (!gs_x3_launch(a, st)) gs_launch<float>(a, dtype, st);
  } else if (dtype == DT_F16) {
    gs_launch<f16>(a, dtype, st);
  } else {
    gs_launch<bf16>(a, dtype, st);
  }
  return check_launch("gemm_stream");
}

}  // namespace fscnn
