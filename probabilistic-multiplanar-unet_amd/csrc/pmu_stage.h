// Branch-free operand staging shared by the conv kernels.
//
// A thread stages NI items of one frame into LDS: item i is the float4 of channels
// c..c+3 at frame pixel (ih[i], iw[i]) of image n, written to lds + dst[i].  All items of a
// thread use the same 4 channels, so the per-channel BN coefficients are loaded once; item
// addresses are clamped and masked so every load is issued before the first wait (the
// generic frame_value4 path branches per item and serialises one memory round trip per item).
#pragma once
#include "pmu_common.h"

constexpr int PMU_NO_ITEM = -0x4000;  // ih[i] marker: thread has no item i

__device__ __forceinline__ float4 pmu_bnrelu4(float4 x, float4 sc, float4 sh) {
  return make_float4(fmaxf(0.f, fmaf(x.x, sc.x, sh.x)), fmaxf(0.f, fmaf(x.y, sc.y, sh.y)),
                     fmaxf(0.f, fmaf(x.z, sc.z, sh.z)), fmaxf(0.f, fmaf(x.w, sc.w, sh.w)));
}
__device__ __forceinline__ float pmu_bnbwd1(float d, float z, float sc, float sh, float mu, float kx, float kc) {
  return fmaf(sc, fmaf(z, sc, sh) > 0.f ? d : 0.f, fmaf(kx, z - mu, kc));
}
// 4 operand values to LDS: fp32 (16 B at ((float*)lds)[dst]) or, for the bf16-MFMA kernels, rounded
// to bf16 (RNE, v_cvt_pk_bf16_f32) as 8 B at ((bf16*)lds)[dst]
typedef __bf16 pmu_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pmu_pk_bf16(float lo, float hi) {
  const pmu_bf16x2 r = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, r);
}
template <bool BF>
__device__ __forceinline__ void pmu_lds_store4(void* lds, int dst, float4 v) {
  if constexpr (BF) {
    *reinterpret_cast<uint2*>(reinterpret_cast<unsigned short*>(lds) + dst) = make_uint2(pmu_pk_bf16(v.x, v.y), pmu_pk_bf16(v.z, v.w));
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(lds) + dst) = v;
  }
}
__device__ __forceinline__ float4 pmu_max4(float4 a, float4 b) {
  return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
}

// AvgPool2d(2, 2, ceil_mode=True) of BN+ReLU values: v00 already transformed; the divisor is the
// number of window elements inside the input (the reference's ceil-mode windows at the edge)
__device__ __forceinline__ float4 pmu_avg4(float4 v00, const float4 (&x)[4], unsigned em, float4 sc, float4 sh) {
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 a = (em & 1u) ? pmu_bnrelu4(x[1], sc, sh) : z;
  const float4 b = (em & 2u) ? pmu_bnrelu4(x[2], sc, sh) : z;
  const float4 d = (em & 4u) ? pmu_bnrelu4(x[3], sc, sh) : z;
  const float cnt = (float)((1 + (em & 1u)) * (1 + ((em >> 1) & 1u)));
  return make_float4((((v00.x + a.x) + b.x) + d.x) / cnt, (((v00.y + a.y) + b.y) + d.y) / cnt,
                     (((v00.z + a.z) + b.z) + d.z) / cnt, (((v00.w + a.w) + b.w) + d.w) / cnt);
}

template <int MODE, int POOL, int NI, bool BF = false>
__device__ __forceinline__ void stage_items_fast(const DevSrc& s, int c, int n, const int (&ih)[NI],
                                                 const int (&iw)[NI], const int (&dst)[NI], void* lds) {
  float4 sc = make_float4(0, 0, 0, 0), sh = sc, mu = sc, kx = sc, kc = sc;
  if (MODE != PMU_SRC_RAW) {
    sc = *reinterpret_cast<const float4*>(s.coef + c);
    sh = *reinterpret_cast<const float4*>(s.coef + s.C + c);
  }
  if (MODE == PMU_SRC_BNBWD) {
    mu = *reinterpret_cast<const float4*>(s.coef + 2 * s.C + c);
    kx = *reinterpret_cast<const float4*>(s.coef + 3 * s.C + c);
    kc = *reinterpret_cast<const float4*>(s.coef + 4 * s.C + c);
  }
  constexpr bool P4 = POOL == PMU_POOL_MAX2 || POOL == PMU_POOL_AVG2CEIL;
  constexpr int NL = P4 ? 4 : 1;
  float4 xv[NI][NL];
  float4 zv[NI];
  bool ok[NI];
  unsigned em[NI];  // AvgPool2d(ceil): which of the window's (0,1), (1,0), (1,1) elements exist
  const long long rs = (long long)s.W * s.C;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    int hs = ih[i] - s.off_h, ws = iw[i] - s.off_w;
    if (P4) { hs *= 2; ws *= 2; }
    // max pool (floor) needs the whole window inside; avg pool (ceil) only its first element
    const int lim_h = (POOL == PMU_POOL_MAX2) ? s.H - 1 : s.H;
    const int lim_w = (POOL == PMU_POOL_MAX2) ? s.W - 1 : s.W;
    ok[i] = (ih[i] != PMU_NO_ITEM) && hs >= 0 && ws >= 0 && hs < lim_h && ws < lim_w;
    const long long idx = ok[i] ? (((long long)n * s.H + hs) * s.W + ws) * s.C + c : (long long)c;
    xv[i][0] = *reinterpret_cast<const float4*>(s.x + idx);
    if (POOL == PMU_POOL_MAX2) {
      xv[i][1] = *reinterpret_cast<const float4*>(s.x + idx + s.C);
      xv[i][2] = *reinterpret_cast<const float4*>(s.x + idx + rs);
      xv[i][3] = *reinterpret_cast<const float4*>(s.x + idx + rs + s.C);
    }
    if constexpr (POOL == PMU_POOL_AVG2CEIL) {
      const bool e01 = ok[i] && ws + 1 < s.W, e10 = ok[i] && hs + 1 < s.H;
      em[i] = (e01 ? 1u : 0u) | (e10 ? 2u : 0u) | ((e01 && e10) ? 4u : 0u);
      xv[i][1] = *reinterpret_cast<const float4*>(s.x + idx + (e01 ? s.C : 0));
      xv[i][2] = *reinterpret_cast<const float4*>(s.x + idx + (e10 ? rs : 0));
      xv[i][3] = *reinterpret_cast<const float4*>(s.x + idx + ((e01 && e10) ? rs + s.C : 0));
    }
    if (MODE == PMU_SRC_BNBWD) zv[i] = *reinterpret_cast<const float4*>(s.z + idx);
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (ih[i] == PMU_NO_ITEM) continue;
    float4 v;
    if (MODE == PMU_SRC_RAW) {
      v = xv[i][0];
    } else if (MODE == PMU_SRC_BNRELU) {
      v = pmu_bnrelu4(xv[i][0], sc, sh);
      if (POOL == PMU_POOL_MAX2) {
        v = pmu_max4(v, pmu_bnrelu4(xv[i][1], sc, sh));
        v = pmu_max4(v, pmu_bnrelu4(xv[i][2], sc, sh));
        v = pmu_max4(v, pmu_bnrelu4(xv[i][3], sc, sh));
      }
      if constexpr (POOL == PMU_POOL_AVG2CEIL) v = pmu_avg4(v, xv[i], em[i], sc, sh);
    } else {
      const float4 d = xv[i][0], z = zv[i];
      v = make_float4(pmu_bnbwd1(d.x, z.x, sc.x, sh.x, mu.x, kx.x, kc.x), pmu_bnbwd1(d.y, z.y, sc.y, sh.y, mu.y, kx.y, kc.y),
                      pmu_bnbwd1(d.z, z.z, sc.z, sh.z, mu.z, kx.z, kc.z), pmu_bnbwd1(d.w, z.w, sc.w, sh.w, mu.w, kx.w, kc.w));
    }
    if (!ok[i]) v = make_float4(0.f, 0.f, 0.f, 0.f);
    pmu_lds_store4<BF>(lds, dst[i], v);
  }
}

// Stage NI items of frame channels [cbase, cbase + span) — this thread's quad is cbase + 4*cq.
// Fast when the span lies inside one source (C % 4 == 0); generic otherwise.
template <int NI, bool BF = false>
__device__ __forceinline__ void stage_items(const DevFrame& F, int n, int cbase, int span, int cq,
                                            const int (&ih)[NI], const int (&iw)[NI], const int (&dst)[NI],
                                            void* lds) {
  const bool in0 = cbase + span <= F.C0;
  const bool in1 = F.nsrc > 1 && cbase >= F.C0 && cbase + span <= F.C;
  if (F.vec && (in0 || in1)) {
    const DevSrc& s = in0 ? F.s0 : F.s1;
    const int c = (in0 ? cbase : cbase - F.C0) + 4 * cq;
    if (s.pool == PMU_POOL_NONE) {
      if (s.mode == PMU_SRC_BNRELU) return stage_items_fast<PMU_SRC_BNRELU, PMU_POOL_NONE, NI, BF>(s, c, n, ih, iw, dst, lds);
      if (s.mode == PMU_SRC_BNBWD) return stage_items_fast<PMU_SRC_BNBWD, PMU_POOL_NONE, NI, BF>(s, c, n, ih, iw, dst, lds);
      return stage_items_fast<PMU_SRC_RAW, PMU_POOL_NONE, NI, BF>(s, c, n, ih, iw, dst, lds);
    }
    if (s.pool == PMU_POOL_MAX2 && s.mode == PMU_SRC_BNRELU)
      return stage_items_fast<PMU_SRC_BNRELU, PMU_POOL_MAX2, NI, BF>(s, c, n, ih, iw, dst, lds);
    if (s.pool == PMU_POOL_AVG2CEIL && s.mode == PMU_SRC_BNRELU)
      return stage_items_fast<PMU_SRC_BNRELU, PMU_POOL_AVG2CEIL, NI, BF>(s, c, n, ih, iw, dst, lds);
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
    if (ih[i] != PMU_NO_ITEM) pmu_lds_store4<BF>(lds, dst[i], frame_value4(F, n, ih[i], iw[i], cbase + 4 * cq));
}

// ---------------------------------------------------------------------------------------------
// Split staging for software-pipelined kernels: pmu_prefetch() issues every global load of a
// thread's NI items (and the chunk's BN coefficients) into registers; pmu_commit() applies the
// transform and writes LDS.  Between the two the caller runs MFMAs on the previous chunk, so the
// load latency is hidden inside the wave instead of relying on a second resident block.
// POOL and BWD (= BN-backward source) are compile-time; RAW vs BN+ReLU is a uniform runtime field
// so both halves of a concat frame share one register set.
// ---------------------------------------------------------------------------------------------
// F.s0 or F.s1 as a value, selected field by field (a select of the whole struct, or a call in each
// branch of an if, keeps the prefetch registers of the pipelined kernels in scratch)
__device__ __forceinline__ DevSrc pmu_pick_src(const DevFrame& F, bool second) {
  DevSrc r;
  r.x = second ? F.s1.x : F.s0.x;
  r.z = second ? F.s1.z : F.s0.z;
  r.coef = second ? F.s1.coef : F.s0.coef;
  r.mode = second ? F.s1.mode : F.s0.mode;
  r.pool = second ? F.s1.pool : F.s0.pool;
  r.C = second ? F.s1.C : F.s0.C;
  r.H = second ? F.s1.H : F.s0.H;
  r.W = second ? F.s1.W : F.s0.W;
  r.off_h = second ? F.s1.off_h : F.s0.off_h;
  r.off_w = second ? F.s1.off_w : F.s0.off_w;
  return r;
}

template <int POOL, bool BWD, int NI>
struct PmuPref {
  static constexpr int NL = (POOL == PMU_POOL_MAX2 || POOL == PMU_POOL_AVG2CEIL) ? 4 : 1;
  float4 x[NI][NL];
  float4 z[BWD ? NI : 1];
  float4 sc, sh, mu, kx, kc;
  unsigned okmask;
  unsigned em;  // AvgPool2d(ceil): 3 bits per item, which of the window's (0,1), (1,0), (1,1) exist
  int raw;
};

template <int POOL, bool BWD, int NI>
__device__ __forceinline__ void pmu_prefetch(const DevSrc& s, int c, int n, const int (&ih)[NI], const int (&iw)[NI],
                                             PmuPref<POOL, BWD, NI>& p) {
  p.raw = (s.mode == PMU_SRC_RAW);
  if (!p.raw) {
    p.sc = *reinterpret_cast<const float4*>(s.coef + c);
    p.sh = *reinterpret_cast<const float4*>(s.coef + s.C + c);
  }
  if (BWD) {
    p.mu = *reinterpret_cast<const float4*>(s.coef + 2 * s.C + c);
    p.kx = *reinterpret_cast<const float4*>(s.coef + 3 * s.C + c);
    p.kc = *reinterpret_cast<const float4*>(s.coef + 4 * s.C + c);
  }
  const long long rs = (long long)s.W * s.C;
  unsigned m = 0u, em = 0u;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    int hs = ih[i] - s.off_h, ws = iw[i] - s.off_w;
    if (POOL != PMU_POOL_NONE) { hs *= 2; ws *= 2; }
    const int lim_h = (POOL == PMU_POOL_MAX2) ? s.H - 1 : s.H;
    const int lim_w = (POOL == PMU_POOL_MAX2) ? s.W - 1 : s.W;
    const bool ok = (ih[i] != PMU_NO_ITEM) && hs >= 0 && ws >= 0 && hs < lim_h && ws < lim_w;
    m |= ok ? (1u << i) : 0u;
    const long long idx = ok ? (((long long)n * s.H + hs) * s.W + ws) * s.C + c : (long long)c;
    p.x[i][0] = *reinterpret_cast<const float4*>(s.x + idx);
    if (POOL == PMU_POOL_MAX2) {
      p.x[i][1] = *reinterpret_cast<const float4*>(s.x + idx + s.C);
      p.x[i][2] = *reinterpret_cast<const float4*>(s.x + idx + rs);
      p.x[i][3] = *reinterpret_cast<const float4*>(s.x + idx + rs + s.C);
    }
    if (POOL == PMU_POOL_AVG2CEIL) {  // ceil-mode windows: only the elements inside the input
      const bool e01 = ok && ws + 1 < s.W, e10 = ok && hs + 1 < s.H;
      em |= ((e01 ? 1u : 0u) | (e10 ? 2u : 0u) | ((e01 && e10) ? 4u : 0u)) << (3 * i);
      p.x[i][1] = *reinterpret_cast<const float4*>(s.x + idx + (e01 ? s.C : 0));
      p.x[i][2] = *reinterpret_cast<const float4*>(s.x + idx + (e10 ? rs : 0));
      p.x[i][3] = *reinterpret_cast<const float4*>(s.x + idx + ((e01 && e10) ? rs + s.C : 0));
    }
    if (BWD) p.z[i] = *reinterpret_cast<const float4*>(s.z + idx);
  }
  p.okmask = m;
  p.em = em;
}

struct PmuNoTee {
  __device__ __forceinline__ void operator()(int, float4) const {}
};

// tee(i, v) sees every committed item's operand value (e.g. to keep a bf16 copy for the backward)
template <int POOL, bool BWD, int NI, bool BF = false, class TEE = PmuNoTee>
__device__ __forceinline__ void pmu_commit(const PmuPref<POOL, BWD, NI>& p, const int (&ih)[NI], const int (&dst)[NI],
                                           void* lds, const TEE& tee = TEE()) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (ih[i] == PMU_NO_ITEM) continue;
    float4 v;
    if (BWD) {
      const float4 d = p.x[i][0], z = p.z[i];
      v = make_float4(pmu_bnbwd1(d.x, z.x, p.sc.x, p.sh.x, p.mu.x, p.kx.x, p.kc.x),
                      pmu_bnbwd1(d.y, z.y, p.sc.y, p.sh.y, p.mu.y, p.kx.y, p.kc.y),
                      pmu_bnbwd1(d.z, z.z, p.sc.z, p.sh.z, p.mu.z, p.kx.z, p.kc.z),
                      pmu_bnbwd1(d.w, z.w, p.sc.w, p.sh.w, p.mu.w, p.kx.w, p.kc.w));
    } else if (p.raw) {
      v = p.x[i][0];
    } else {
      v = pmu_bnrelu4(p.x[i][0], p.sc, p.sh);
      if (POOL == PMU_POOL_MAX2) {
        v = pmu_max4(v, pmu_bnrelu4(p.x[i][1], p.sc, p.sh));
        v = pmu_max4(v, pmu_bnrelu4(p.x[i][2], p.sc, p.sh));
        v = pmu_max4(v, pmu_bnrelu4(p.x[i][3], p.sc, p.sh));
      }
      if constexpr (POOL == PMU_POOL_AVG2CEIL) v = pmu_avg4(v, p.x[i], (p.em >> (3 * i)) & 7u, p.sc, p.sh);
    }
    if (!((p.okmask >> i) & 1u)) v = make_float4(0.f, 0.f, 0.f, 0.f);
    pmu_lds_store4<BF>(lds, dst[i], v);
    tee(i, v);
  }
}
