// 3x3 / pad 1 convolution in fp32 by Winograd F(4x4, 3x3) on f32 MFMA: the forward of nn.Conv2d at
// PMU/model/unet/unet_parts.py:15,18 and its input gradient, on a materialised NHWC operand (the
// tensor the weight gradient reads anyway), for images of at least 32 x 32 pixels.
//
// Every 4x4 block of output pixels ("tile") comes from the 6x6 operand patch d around it as
//   Y = A^T [ (G g G^T) .* (B^T d B) ] A
// i.e. 36 element-wise products per input/output channel pair for 16 outputs (2.25 per output, against
// 4 for F(2x2,3x3) in conv3x3_wino.hip and 9 for the direct sum).  The reduction over input channels
// becomes 36 independent GEMMs ("components")  M[c][tile][co] = sum_ci V[c][tile][ci] * U[c][ci][co].
// All arithmetic is fp32 (points 0, +-1, +-2, inf; U computed in double and rounded once): the result
// differs from the direct sum by rounding only (a few 1e-6 relative), far inside the 1e-3 parity bound.
//
// Block: 256 threads = 4 waves, one per SIMD (the 512-register file lets a wave hold 2 x 36 f32x4
// accumulators), 64 tiles (8 x 8 -> a 32 x 32 output patch) x 32 output channels.  Wave w owns the
// tiles of tile rows 2w, 2w+1 (lane & 15 -> tile) for both 16-channel halves of the 32 outputs: its
// V (the transformed patch, the MFMA A operand) feeds two MFMAs, so the input transform costs two
// VALU instructions per MFMA.  Per chunk of 8 input channels, double-buffered LDS stages receive the
// 34 x 34 x 8 operand image and the chunk's U (8 ch x 32 co x 36 comps) by global_load_lds (LDS-DMA:
// no registers, no VALU); each lane reads its tile's 6 x 6 patch for two channels as 36 ds_read_b64
// (conflict-free: halo pixels in groups of 4 with a pad unit, rows of 312 floats) and runs two MFMA
// steps (channel 2*kk + ks in k-slot kk = lane >> 4).
// Epilogue: A^T M A per lane (+bias), BN partial sums per block (forward) or the split dx store.
#include <string.h>
#include <stdlib.h>
#include <utility>
#include "pmu_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TX = 8, TY = 8;                 // tiles per block
constexpr int OW = 4 * TX, OH = 4 * TY;       // 32 x 32 output pixels
constexpr int HW = OW + 2, HH = OH + 2;       // 34 x 34 halo
constexpr int BK = 8;                         // input channels per chunk
constexpr int GP = 36;                        // floats per group of 4 halo pixels (4 x 8 ch + 1 pad unit)
constexpr int ROWF = 312;                     // floats per halo row: 8 groups + 2 px = 304, and 2*ROWF = 16 (mod 32) b64 units
constexpr int ROWU = ROWF / 4;                // 16-B units per halo row
constexpr int A_FLOATS = HH * ROWF;
constexpr int CO = 32;                        // output channels per block
constexpr int NC = 36;                        // Winograd components
constexpr int U_FLOATS = BK * CO * NC;        // one chunk of transformed weights [ch 8][co 32][comp 36]
constexpr int STAGE = A_FLOATS + U_FLOATS;
constexpr int NT = 512;
constexpr int A_UNITS = A_FLOATS / 4;
constexpr int NGL = (A_UNITS + NT - 1) / NT;  // operand DMA instructions per thread per chunk
constexpr int UGL = (U_FLOATS / 4 + NT - 1) / NT;  // U DMA rounds per chunk (the last one by waves 0-3)
constexpr int RED_FLOATS = 8 * 16 * 2;
static_assert(U_FLOATS % (4 * 256) == 0, "U of whole wave DMA instructions");
static_assert((2 * STAGE + RED_FLOATS) * 4 <= 160 * 1024, "LDS");

struct W4Args {
  const float* x;     // [N][H][W][KC]
  const float* wp;    // packed U [co block][chunk][ch 8][co 32][comp 36]
  const float* bias;
  float* out0;
  float* out1;
  float* part;        // [spatial blocks][2][NOUT] BN partial sums (fwd) or null
  int H, W, KC, NOUT, split, bw, bh, nco, cpb;
  int prio;           // 1: waves of component half 1 run at s_setprio 1 (PMU_WINO4_PRIO)
  int ts, tc;         // 2-D workgroup grouping (spatial x co-groups per group; tc = 0: co-groups fastest)
  int N;              // images (bounds checks of the debug build)
  // input gradient only: BatchNorm+ReLU backward partial sums of the layer that produced the operand
  // of this conv (dx is that layer's da): part[spatial][2][NOUT] += (sum g, sum g*xhat) with
  // g = dx * (z*scale+shift > 0), xhat = (z-mean)*invstd (pmu_bn_bwd_reduce's sums); null: none
  const float* bz;
  const float* bcoef;
  const float* bmean;
  const float* binv;
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// position of component c = 6a + b (half a / 3, local index cl = c - 18 (a / 3)) in a packed U row of 36
constexpr int upos(int ch, int cl) { return cl < 16 ? 16 * ch + cl : 32 + 2 * ch + (cl - 16); }

// U = G g G^T, G = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1]
__device__ __forceinline__ void g6(const double (&g)[3], double (&t)[6]) {
  t[0] = g[0] / 4.0;
  t[1] = -(g[0] + g[1] + g[2]) / 6.0;
  t[2] = -(g[0] - g[1] + g[2]) / 6.0;
  t[3] = g[0] / 24.0 + g[1] / 12.0 + g[2] / 6.0;
  t[4] = g[0] / 24.0 - g[1] / 12.0 + g[2] / 6.0;
  t[5] = g[2];
}

// One workgroup per (co block, chunk): the BK x CO filters are transformed into LDS in the packed
// order and the contiguous BK x CO x 36 segment is stored with consecutive float4s. Consecutive
// threads read consecutive filters: along the output channel for the input gradient (w[k][j..]),
// along the reduction channel for the forward (w[j][k..]).
__device__ __forceinline__ void pack_wino4_body(const float* __restrict__ w, int Cout, int Cin, int dgrad,
                                                float* __restrict__ wp, int bid) {
  constexpr int SEG = BK * CO * NC;
  __shared__ float4 seg4[SEG / 4];
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK;
  const int ch = bid % nch, jb = bid / nch;
  for (int f = threadIdx.x; f < BK * CO; f += blockDim.x) {
    const int col = dgrad ? f % CO : f / BK, kl = dgrad ? f / CO : f % BK;
    const int j = jb * CO + col, k = ch * BK + kl;
    double g[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double v = 0.0;
        if (j < NOUT && k < KC)  // dgrad: the input gradient convolves dz with w[co][ci] rotated by 180 degrees
          v = dgrad ? w[((long long)k * Cin + j) * 9 + (2 - a) * 3 + (2 - b)] : w[((long long)j * Cin + k) * 9 + a * 3 + b];
        g[a][b] = v;
      }
    double t[6][3];  // G g (columns)
    for (int b = 0; b < 3; ++b) {
      const double col3[3] = {g[0][b], g[1][b], g[2][b]};
      double o[6];
      g6(col3, o);
      for (int a = 0; a < 6; ++a) t[a][b] = o[a];
    }
    float u[36];     // (G g) G^T
    for (int a = 0; a < 6; ++a) {
      const double row3[3] = {t[a][0], t[a][1], t[a][2]};
      double o[6];
      g6(row3, o);
      for (int b = 0; b < 6; ++b) u[6 * a + b] = (float)o[b];
    }
    float row[36];   // the row in component-half order (upos)
    for (int c = 0; c < 36; ++c) row[upos(c / 18, c % 18)] = u[c];
    float4* d = seg4 + (kl * CO + col) * (NC / 4);
    for (int q = 0; q < 9; ++q) d[q] = make_float4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
  }
  __syncthreads();
  float4* dst = reinterpret_cast<float4*>(wp + (long long)bid * SEG);
  for (int i = threadIdx.x; i < SEG / 4; i += blockDim.x) dst[i] = seg4[i];
}
__global__ __launch_bounds__(256) void pack_wino4_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad,
                                                         float* __restrict__ wp) {
  pack_wino4_body(w, Cout, Cin, dgrad, wp, blockIdx.x);
}
__global__ __launch_bounds__(256) void pack_wino4_multi_kernel(const pmu_pack_job* __restrict__ jobs, int njobs,
                                                               int dgrad) {
  const pmu_pack_job& j = jobs[pmu_job_of(jobs, njobs, blockIdx.x)];
  pack_wino4_body(j.w, j.Cout, j.Cin, dgrad, (float*)j.dst, blockIdx.x - j.block0);
}

// B^T row on d0..d5, B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
__device__ __forceinline__ void bt6(float d0, float d1, float d2, float d3, float d4, float d5, float& r0, float& r1,
                                    float& r2, float& r3, float& r4, float& r5) {
  r0 = fmaf(-5.f, d2, fmaf(4.f, d0, d4));
  const float a = fmaf(-4.f, d2, d4), b = fmaf(-4.f, d1, d3);
  r1 = a + b;
  r2 = a - b;
  const float c = d4 - d2, e = d3 - d1;
  r3 = fmaf(2.f, e, c);
  r4 = fmaf(-2.f, e, c);
  r5 = fmaf(-5.f, d3, fmaf(4.f, d1, d5));
}

// V = B^T d B; v[6a + b]
__device__ __forceinline__ void input_transform4(const float (&d)[36], float (&v)[36]) {
  float t[36];
#pragma unroll
  for (int j = 0; j < 6; ++j)
    bt6(d[j], d[6 + j], d[12 + j], d[18 + j], d[24 + j], d[30 + j], t[j], t[6 + j], t[12 + j], t[18 + j], t[24 + j],
        t[30 + j]);
#pragma unroll
  for (int a = 0; a < 6; ++a)
    bt6(t[6 * a], t[6 * a + 1], t[6 * a + 2], t[6 * a + 3], t[6 * a + 4], t[6 * a + 5], v[6 * a], v[6 * a + 1],
        v[6 * a + 2], v[6 * a + 3], v[6 * a + 4], v[6 * a + 5]);
}

// A^T row on m0..m5, A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
__device__ __forceinline__ void at4(float m0, float m1, float m2, float m3, float m4, float m5, float& y0, float& y1,
                                    float& y2, float& y3) {
  const float s12 = m1 + m2, d12 = m1 - m2, s34 = m3 + m4, d34 = m3 - m4;
  y0 = m0 + s12 + s34;
  y1 = fmaf(2.f, d34, d12);
  y2 = fmaf(4.f, s34, s12);
  y3 = fmaf(8.f, d34, d12) + m5;
}

template <int OFF>
__device__ __forceinline__ float4 lds_b128(unsigned addr) {
  float4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ float2 lds_b64(unsigned addr) {
  float2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(p);
}

template <int OFF>
__device__ __forceinline__ float lds_b32(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
// patch element e (row e / 6, column e % 6) of this lane's tile: byte offset from the patch origin
template <int E>
struct PatchOff {
  static constexpr int value = ((E / 6) * ROWF + ((E % 6) >> 2) * GP + ((E % 6) & 3) * 8) * 4;
};
// elements E0 .. E0+N-1 of the 6x6 patch of this lane's tile for one channel (ds_read_b32 each)
template <int E0, int N>
__device__ __forceinline__ void load_patch_part(unsigned pa, float (&d)[36]) {
  if constexpr (N > 0) {
    d[E0] = lds_b32<PatchOff<E0>::value>(pa);
    load_patch_part<E0 + 1, N - 1>(pa, d);
  }
}
// s_waitcnt lgkmcnt(N) (vmcnt / expcnt left at their maxima; gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt");
  __builtin_amdgcn_s_waitcnt(0xC07F | (N << 8));
}

// component c = 6a + b of the 6x6 grid belongs to half CH = a / 3 (local index cl = c - 18 CH); a packed
// U row of 36 holds [half 0: cl 0..15 | half 1: cl 0..15 | half 0: cl 16,17 | half 1: cl 16,17], so a
// half is 4 b128 + 1 b64 reads

// the half CH of V = B^T d B: rows a = 3 CH .. 3 CH + 2 of the column pass, then their row pass;
// v[6 a' + b], a' = a - 3 CH
template <int CH>
__device__ __forceinline__ void input_transform_half(const float (&d)[36], float (&v)[18]) {
  float t[18];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const float d0 = d[j], d1 = d[6 + j], d2 = d[12 + j], d3 = d[18 + j], d4 = d[24 + j], d5 = d[30 + j];
    if (CH == 0) {
      t[j] = fmaf(-5.f, d2, fmaf(4.f, d0, d4));
      const float a = fmaf(-4.f, d2, d4), b = fmaf(-4.f, d1, d3);
      t[6 + j] = a + b;
      t[12 + j] = a - b;
    } else {
      const float c = d4 - d2, e = d3 - d1;
      t[j] = fmaf(2.f, e, c);
      t[6 + j] = fmaf(-2.f, e, c);
      t[12 + j] = fmaf(-5.f, d3, fmaf(4.f, d1, d5));
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
    bt6(t[6 * a], t[6 * a + 1], t[6 * a + 2], t[6 * a + 3], t[6 * a + 4], t[6 * a + 5], v[6 * a], v[6 * a + 1],
        v[6 * a + 2], v[6 * a + 3], v[6 * a + 4], v[6 * a + 5]);
}

// ---- one MFMA step (4 channels: channel 2*kk + ks in k-slot kk) of a wave -------------------------
// The wave's 18 components x 2 co halves = 36 MFMAs in 5 groups (4 components each, the last 2).  LDS
// reads in issue order: the step's patch (36 x b32), U groups 0..2 (one read per co half each), then
// group g + 3 after group g's MFMAs.  Being asm, the reads get no compiler waits: group g waits
// (lgkmcnt) for all but the reads issued after it (DS reads complete in order).
template <int CH, int G>
__device__ __forceinline__ void w4_uread(unsigned ua, float4 (&ur)[3][2], float2 (&ut)[2]) {
  if constexpr (G < 4) {
    ur[G % 3][0] = lds_b128<upos(CH, 4 * G) * 4>(ua);
    ur[G % 3][1] = lds_b128<(16 * NC + upos(CH, 4 * G)) * 4>(ua);
  } else {
    ut[0] = lds_b64<upos(CH, 16) * 4>(ua);
    ut[1] = lds_b64<(16 * NC + upos(CH, 16)) * 4>(ua);
  }
}

// PF: the next step's patch (channel +1) is read during this step's last two groups (12 + 24 reads,
// after the U reads: the counted waits stay <= 15), so the next step starts on landed data.
template <int CH, int G, bool PF>
__device__ __forceinline__ void w4_group(unsigned ua, const float (&v)[18], float4 (&ur)[3][2], float2 (&ut)[2],
                                         f32x4 (&acc)[2][18], unsigned pn, float (&dn)[36]) {
  if constexpr (G > 0) wait_lgkm<(PF && G == 4) ? 12 : 2 * ((G + 2 < 4 ? G + 2 : 4) - G)>();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (G < 4) {
    constexpr int c0 = 4 * G;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 q = ur[G % 3][h];
      acc[h][c0 + 0] = mfma16(v[c0 + 0], q.x, acc[h][c0 + 0]);
      acc[h][c0 + 1] = mfma16(v[c0 + 1], q.y, acc[h][c0 + 1]);
      acc[h][c0 + 2] = mfma16(v[c0 + 2], q.z, acc[h][c0 + 2]);
      acc[h][c0 + 3] = mfma16(v[c0 + 3], q.w, acc[h][c0 + 3]);
    }
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      acc[h][16] = mfma16(v[16], ut[h].x, acc[h][16]);
      acc[h][17] = mfma16(v[17], ut[h].y, acc[h][17]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (G + 3 <= 4) w4_uread<CH, G + 3>(ua, ur, ut);
  if constexpr (PF && G == 3) load_patch_part<0, 12>(pn, dn);
  if constexpr (PF && G == 4) load_patch_part<12, 24>(pn, dn);
}

// One chunk (two MFMA steps: channels 2*kk and 2*kk + 1).  pa = byte address of this lane's patch
// origin (channel 2*kk), ua = of its U row (channel 2*kk, co half 0).  PF: step 1's patch is read
// during step 0's MFMAs instead of after them.
template <int CH, bool PF>
__device__ __forceinline__ void w4_chunk(unsigned pa, unsigned ua, f32x4 (&acc)[2][18]) {
  float d[36], v[18];
  float4 ur[3][2];
  float2 ut[2];
  load_patch_part<0, 36>(pa, d);
  w4_uread<CH, 0>(ua, ur, ut);
  w4_uread<CH, 1>(ua, ur, ut);
  w4_uread<CH, 2>(ua, ur, ut);
  wait_lgkm<4>();  // the patch and U group 0
  __builtin_amdgcn_sched_barrier(0);
  input_transform_half<CH>(d, v);
  __builtin_amdgcn_sched_barrier(0);
  const unsigned pa1 = pa + 4, ua1 = ua + CO * NC * 4;
  w4_group<CH, 0, PF>(ua, v, ur, ut, acc, pa1, d);
  w4_group<CH, 1, PF>(ua, v, ur, ut, acc, pa1, d);
  w4_group<CH, 2, PF>(ua, v, ur, ut, acc, pa1, d);
  w4_group<CH, 3, PF>(ua, v, ur, ut, acc, pa1, d);
  w4_group<CH, 4, PF>(ua, v, ur, ut, acc, pa1, d);
  if constexpr (!PF) load_patch_part<0, 36>(pa1, d);
  w4_uread<CH, 0>(ua1, ur, ut);
  w4_uread<CH, 1>(ua1, ur, ut);
  w4_uread<CH, 2>(ua1, ur, ut);
  wait_lgkm<4>();  // step 1's patch and U group 0
  __builtin_amdgcn_sched_barrier(0);
  input_transform_half<CH>(d, v);
  __builtin_amdgcn_sched_barrier(0);
  w4_group<CH, 0, false>(ua1, v, ur, ut, acc, pa1, d);
  w4_group<CH, 1, false>(ua1, v, ur, ut, acc, pa1, d);
  w4_group<CH, 2, false>(ua1, v, ur, ut, acc, pa1, d);
  w4_group<CH, 3, false>(ua1, v, ur, ut, acc, pa1, d);
  w4_group<CH, 4, false>(ua1, v, ur, ut, acc, pa1, d);
}

// column j of the half-CH column pass of B^T d B (input_transform_half's first loop) for one channel
template <int CH>
__device__ __forceinline__ void w4_col_half(float d0, float d1, float d2, float d3, float d4, float d5, float& r0,
                                            float& r1, float& r2) {
  if (CH == 0) {
    r0 = fmaf(-5.f, d2, fmaf(4.f, d0, d4));
    const float a = fmaf(-4.f, d2, d4), b = fmaf(-4.f, d1, d3);
    r1 = a + b;
    r2 = a - b;
  } else {
    const float c = d4 - d2, e = d3 - d1;
    r0 = fmaf(2.f, e, c);
    r1 = fmaf(-2.f, e, c);
    r2 = fmaf(-5.f, d3, fmaf(4.f, d1, d5));
  }
}
// column J of this lane's 6x6 patch for both channels of its k-slot (2kk, 2kk + 1) as ds_read_b64: the
// five rows half CH uses (0-4 for CH 0, 1-5 for CH 1) — an asm read whose result is never used would let
// the compiler hand its register to a live value that the late LDS return then overwrites
template <int CH, int J>
__device__ __forceinline__ void w4_col_read(unsigned pa, float2 (&c)[5]) {
  c[0] = lds_b64<PatchOff<6 * CH + J>::value>(pa);
  c[1] = lds_b64<PatchOff<6 * CH + 6 + J>::value>(pa);
  c[2] = lds_b64<PatchOff<6 * CH + 12 + J>::value>(pa);
  c[3] = lds_b64<PatchOff<6 * CH + 18 + J>::value>(pa);
  c[4] = lds_b64<PatchOff<6 * CH + 24 + J>::value>(pa);
}
template <int CH, int J>
__device__ __forceinline__ void w4_col_tf(const float2 (&c)[5], float (&t0)[18], float (&t1)[18]) {
  if (CH == 0) {  // rows 0-4 (w4_col_half<0> does not read d5)
    w4_col_half<0>(c[0].x, c[1].x, c[2].x, c[3].x, c[4].x, 0.f, t0[J], t0[6 + J], t0[12 + J]);
    w4_col_half<0>(c[0].y, c[1].y, c[2].y, c[3].y, c[4].y, 0.f, t1[J], t1[6 + J], t1[12 + J]);
  } else {        // rows 1-5 (w4_col_half<1> does not read d0)
    w4_col_half<1>(0.f, c[0].x, c[1].x, c[2].x, c[3].x, c[4].x, t0[J], t0[6 + J], t0[12 + J]);
    w4_col_half<1>(0.f, c[0].y, c[1].y, c[2].y, c[3].y, c[4].y, t1[J], t1[6 + J], t1[12 + J]);
  }
}
template <int CH>
__device__ __forceinline__ void w4_row_pass(const float (&t)[18], float (&v)[18]) {
#pragma unroll
  for (int a = 0; a < 3; ++a)
    bt6(t[6 * a], t[6 * a + 1], t[6 * a + 2], t[6 * a + 3], t[6 * a + 4], t[6 * a + 5], v[6 * a], v[6 * a + 1],
        v[6 * a + 2], v[6 * a + 3], v[6 * a + 4], v[6 * a + 5]);
}

// One chunk with the patch read as ds_read_b64 channel pairs: both steps' patches (channels 2kk, 2kk + 1)
// arrive together, 30 b64 reads (the 5 x 6 elements this half uses) instead of 72 b32.  In a 32-lane group the 16 tiles x 2 k-slots cover
// all 64 banks once (tile columns 36 floats apart, tile rows 4 x 312 = 32 mod 64 floats, k-slots 2
// floats): conflict-free, where the b32 reads of one channel are 2-way (16 tiles x 2 channels on 32
// banks of 4-float DMA units).  The patch streams column by column through two 6-read register sets; each
// column's half column-pass runs for both channels as it lands, so the live state is the two channels'
// column-pass halves (t0, t1: 36 floats, as d[36] before), not 72 patch values.
template <int CH>
__device__ __forceinline__ void w4_chunk64(unsigned pa, unsigned ua, f32x4 (&acc)[2][18]) {
  float t0[18], t1[18], v[18];
  float2 cA[5], cB[5];
  float4 ur[3][2];
  float2 ut[2];
  w4_col_read<CH, 0>(pa, cA);
  w4_col_read<CH, 1>(pa, cB);
  wait_lgkm<5>();  // column 0 (reads complete in order)
  __builtin_amdgcn_sched_barrier(0);
  w4_col_tf<CH, 0>(cA, t0, t1);
  __builtin_amdgcn_sched_barrier(0);
  w4_col_read<CH, 2>(pa, cA);
  wait_lgkm<5>();
  __builtin_amdgcn_sched_barrier(0);
  w4_col_tf<CH, 1>(cB, t0, t1);
  __builtin_amdgcn_sched_barrier(0);
  w4_col_read<CH, 3>(pa, cB);
  wait_lgkm<5>();
  __builtin_amdgcn_sched_barrier(0);
  w4_col_tf<CH, 2>(cA, t0, t1);
  __builtin_amdgcn_sched_barrier(0);
  w4_col_read<CH, 4>(pa, cA);
  wait_lgkm<5>();
  __builtin_amdgcn_sched_barrier(0);
  w4_col_tf<CH, 3>(cB, t0, t1);
  __builtin_amdgcn_sched_barrier(0);
  w4_col_read<CH, 5>(pa, cB);
  // step 0's U groups 0-2 behind the last column (their registers are free until here)
  w4_uread<CH, 0>(ua, ur, ut);
  w4_uread<CH, 1>(ua, ur, ut);
  w4_uread<CH, 2>(ua, ur, ut);
  wait_lgkm<11>();  // column 4
  __builtin_amdgcn_sched_barrier(0);
  w4_col_tf<CH, 4>(cA, t0, t1);
  __builtin_amdgcn_sched_barrier(0);
  wait_lgkm<6>();   // column 5
  __builtin_amdgcn_sched_barrier(0);
  w4_col_tf<CH, 5>(cB, t0, t1);
  w4_row_pass<CH>(t0, v);
  __builtin_amdgcn_sched_barrier(0);
  wait_lgkm<4>();   // U group 0
  __builtin_amdgcn_sched_barrier(0);
  float dn[36];   // (unused: no patch prefetch in this form)
  w4_group<CH, 0, false>(ua, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 1, false>(ua, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 2, false>(ua, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 3, false>(ua, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 4, false>(ua, v, ur, ut, acc, 0u, dn);
  const unsigned ua1 = ua + CO * NC * 4;
  w4_uread<CH, 0>(ua1, ur, ut);
  w4_uread<CH, 1>(ua1, ur, ut);
  w4_uread<CH, 2>(ua1, ur, ut);
  w4_row_pass<CH>(t1, v);
  wait_lgkm<4>();  // step 1's U group 0
  __builtin_amdgcn_sched_barrier(0);
  w4_group<CH, 0, false>(ua1, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 1, false>(ua1, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 2, false>(ua1, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 3, false>(ua1, v, ur, ut, acc, 0u, dn);
  w4_group<CH, 4, false>(ua1, v, ur, ut, acc, 0u, dn);
}

// this half's share of Y = A^T M A for tile r of co half h: P[4p + q] = sum over the half's rows a of
// A^T[p][a] (M[a][:] A)[q]
template <int CH>
__device__ __forceinline__ void w4_partial(const f32x4 (&acc)[2][18], int h, int r, float (&P)[16]) {
  float R[3][4];
#pragma unroll
  for (int a = 0; a < 3; ++a)
    at4(acc[h][6 * a][r], acc[h][6 * a + 1][r], acc[h][6 * a + 2][r], acc[h][6 * a + 3][r], acc[h][6 * a + 4][r],
        acc[h][6 * a + 5][r], R[a][0], R[a][1], R[a][2], R[a][3]);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (CH == 0) {  // A^T columns 0..2: (1,0,0,0), (1,1,1,1), (1,-1,1,-1)
      const float s = R[1][q] + R[2][q], df = R[1][q] - R[2][q];
      P[q] = R[0][q] + s;
      P[4 + q] = df;
      P[8 + q] = s;
      P[12 + q] = df;
    } else {        // A^T columns 3..5: (1,2,4,8), (1,-2,4,-8), (0,0,0,1)
      const float s = R[0][q] + R[1][q], df = R[0][q] - R[1][q];
      P[q] = s;
      P[4 + q] = 2.f * df;
      P[8 + q] = 4.f * s;
      P[12 + q] = fmaf(8.f, df, R[2][q]);
    }
  }
}

// epilogue: lane holds M[comp (half CH)][tile 4*kk + r of the wave's group][co j0 + 16 h + (lane & 15)]
// in acc[h][cl][r].  The two waves of a tile group (halves 0 and 1) swap the partial outputs of the
// co half the other one finishes through xb (a free LDS stage), in two rounds of two tiles per lane;
// wave (tg, CH) then finishes co half CH: bias, store, BN partial sums.
template <bool DGRAD, bool BNR, int CH, int EXP = 0>
__device__ __forceinline__ void wino4_epilogue(const W4Args& a, int n, int h0, int w0, int j0, int spatial,
                                               const f32x4 (&acc)[2][18], float* xb, float* red, float bias) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kk = lane >> 4;
  const int tg = wave & 3, partner = tg + 4 * (1 - CH);
  const int j = j0 + 16 * CH + (lane & 15);
  const bool jok = j < a.NOUT;
  // this lane's output column: the forward's z, or the input gradient's dx0 / dx1 side of the split
  float* dst;
  int ld;
  if (!DGRAD) { dst = a.out0 + j; ld = a.NOUT; }
  else if (j < a.split) { dst = a.out0 + j; ld = a.split; }
  else { dst = a.out1 + (j - a.split); ld = a.NOUT - a.split; }
  float s1 = 0.f, s2 = 0.f, sink = 0.f;
  float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
  if (BNR && jok) {
    bsc = a.bcoef[j];
    bsh = a.bcoef[a.NOUT + j];
    bmu = a.bmean[j];
    bis = a.binv[j];
  }
#pragma unroll
  for (int rho = 0; rho < 2; ++rho) {
    if (rho) __syncthreads();  // round 0's reads are done before xb is rewritten
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      float P[16];
      w4_partial<CH>(acc, 1 - CH, 2 * rho + rr, P);
#pragma unroll
      for (int e = 0; e < 16; ++e) xb[((wave * 2 + rr) * 16 + e) * 64 + lane] = P[e];
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int r = 2 * rho + rr;
      const int t = 4 * kk + r;  // tile within the group
      const int oh = h0 + 4 * (2 * tg + (t >> 3)), ow = w0 + 4 * (t & 7);
      // the producer's z under this tile's 16 outputs, loaded before the output transform so the
      // loads are in flight together (issued one per store, each waited for on its own)
      float zt[16];
      if (BNR && EXP == 8) {  // timing experiment: one z load (the column's first pixel) for all 16
        const float z0 = a.bz[min(j, a.NOUT - 1)];
#pragma unroll
        for (int e = 0; e < 16; ++e) zt[e] = z0;
      } else if (BNR) {
        const int jc = min(j, a.NOUT - 1);  // clamped: every lane loads (no branch per load), unused ones ignored
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int hh2 = oh + (e >> 2), ww = ow + (e & 3);
          const long long pix = ((long long)n * a.H + min(hh2, a.H - 1)) * a.W + min(ww, a.W - 1);
          zt[e] = a.bz[pix * a.NOUT + jc];
        }
      }
      float P[16];
      w4_partial<CH>(acc, CH, r, P);
      // the partner's 16 partial outputs read together and held in registers before any store branch:
      // read where they are used, the compiler sank each ds_read into its output's store branch (the
      // plain input gradient uses v only there) and waited lgkmcnt(0) right behind it — 16 serial LDS
      // round trips per tile
      float xv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) xv[e] = xb[((partner * 2 + rr) * 16 + e) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 16; ++e) asm volatile("" : "+v"(xv[e]));
      // values, masks and BN sums unconditional, only the stores predicated (see conv3x3_wino2h.hip:
      // a global value first consumed inside a per-output branch cost a vmcnt(0) per store); one row
      // pointer per output row, 32-bit column offsets
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int hh2 = oh + p;
        float* rowp = dst + (long long)((long long)n * a.H + min(hh2, a.H - 1)) * a.W * ld;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ww = ow + q;
          const float v = P[4 * p + q] + xv[4 * p + q] + bias;
          const bool ok = jok && hh2 < a.H && ww < a.W;
          if (!DGRAD) {
            const float m = ok ? v : 0.f;
            s1 += m;
            s2 = fmaf(m, m, s2);
          } else if (BNR) {
            const float zz = zt[4 * p + q];
            const float g = (ok && fmaf(zz, bsc, bsh) > 0.f) ? v : 0.f;
            s1 += g;
            s2 = fmaf(g, (zz - bmu) * bis, s2);
          }
          if (EXP == 6) {  // timing experiment: no stores (the values kept live through one sum)
            sink += ok ? v : 0.f;
            continue;
          }
          if (!ok) continue;
          PMU_DCHECK((((long long)n * a.H + hh2) * a.W + ww) < (long long)a.N * a.H * a.W && j < a.NOUT, PMU_DBG_OUTPUT);
          rowp[(unsigned)(ww * ld)] = v;
        }
      }
    }
  }
  if (EXP == 6 && a.N < 0) dst[0] = sink;  // (never true: keeps the experiment's values live)
  if (a.part) {  // forward: BN partial sums of the output; input gradient: of the producer's BN backward
    s1 += __shfl_xor(s1, 16, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (lane < 16) {
      red[(wave * 16 + lane) * 2 + 0] = s1;
      red[(wave * 16 + lane) * 2 + 1] = s2;
    }
    __syncthreads();
    if (tid < CO) {  // channel tid: half tid >> 4, summed over the 4 tile groups (waves 4*half + tg) in order
      const int jj = j0 + tid, hf = tid >> 4, l = tid & 15;
      if (jj < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          t1 += red[((4 * hf + g) * 16 + l) * 2 + 0];
          t2 += red[((4 * hf + g) * 16 + l) * 2 + 1];
        }
        PMU_DCHECK(spatial < (long long)a.N * a.bh * a.bw, PMU_DBG_WORKSPACE);
        a.part[((long long)spatial * 2 + 0) * a.NOUT + jj] = t1;
        a.part[((long long)spatial * 2 + 1) * a.NOUT + jj] = t2;
      }
    }
  }
  __syncthreads();  // the exchange reads are done before the next pass's DMA refills xb's stage
}

struct W4Block {
  int n, h0, w0, cob0, spatial, nchunks, npass;
  unsigned gin;    // operand units inside the input (DMA'd)
  unsigned gzero;  // image units outside it (zero, written once; restored after an exchange in their stage)
};

// the pass / chunk pipeline of a wave of component half CH (waves 4 CH .. 4 CH + 3); PM: the patch read —
// 0 b32 per channel, 1 b32 with step 1's patch read under step 0's MFMAs, 2 b64 channel pairs (default)
template <bool DGRAD, bool BNR, int CH, int PM, int EXP = 0>
__device__ __forceinline__ void wino4_main(const W4Args& a, const W4Block& B, const unsigned (&goff)[NGL],
                                           float* smem) {
  float* red = smem + 2 * STAGE;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nchunks = B.nchunks, total = B.npass * nchunks;
  const float* wsrc = a.wp + (long long)B.cob0 * nchunks * U_FLOATS;
  const unsigned uoff = 16u * tid;
  const int wave_off = wave * 256;
  const unsigned gin = B.gin;
#define PMU_GLDS(S, D)                                                                                      \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S),                     \
                                   (__attribute__((address_space(3))) void*)(D), 16, 0, 0);
  // Passes walk the chunks in alternating (serpentine) order: a pass starts on the chunks the previous
  // pass fetched last, which are still in the XCD's L2 (~3 of a workgroup's 37-KB chunk images fit its
  // share), instead of on chunk 0, fetched longest ago.  The direction follows the co-block's parity,
  // not the pass index, so an output's summation order does not depend on cpb (launches split over
  // images stay bit-equal to whole ones).
#define PMU_FETCH4(GI, BUF)                                                                                 \
  {                                                                                                        \
    const int p_ = (GI) / nchunks;                                                                         \
    const int c_ = (GI) - p_ * nchunks;                                                                    \
    const int cs_ = ((B.cob0 + p_) & 1) ? nchunks - 1 - c_ : c_;                                           \
    const int k0_ = cs_ * BK;                                                                              \
    PMU_DCHECK(k0_ + BK <= a.KC, PMU_DBG_OPERAND);                                                         \
    float* b_ = (BUF);                                                                                     \
    const char* xb_ = reinterpret_cast<const char*>(a.x + k0_);                                            \
    _Pragma("unroll") for (int r = 0; r < NGL; ++r)                                                        \
      if ((gin >> r) & 1u) PMU_GLDS(xb_ + goff[r], b_ + 4 * (r * NT) + wave_off)                           \
    const char* s_ = reinterpret_cast<const char*>(wsrc + ((long long)p_ * nchunks + cs_) * U_FLOATS) + uoff; \
    float* d_ = b_ + A_FLOATS + wave_off;                                                                  \
    _Pragma("unroll") for (int r = 0; r < UGL; ++r)                                                        \
      if (r * NT * 4 + (wave + 1) * 256 <= U_FLOATS) PMU_GLDS(s_ + 16 * NT * r, d_ + 4 * NT * r)          \
  }
  const int t = lane & 15, kk = lane >> 4, tg = wave & 3;
  const int pbase = 4 * (2 * tg + (t >> 3)) * ROWF + GP * (t & 7) + 2 * kk;
  const int ubase = A_FLOATS + (2 * kk * CO + t) * NC;
  f32x4 acc[2][18];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int c = 0; c < 18; ++c) acc[h][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  PMU_FETCH4(0, smem)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int p = 0; p < B.npass; ++p) {
    const int j0 = (B.cob0 + p) * CO;
    const int jb = j0 + 16 * CH + t;
    const float bias = (!DGRAD && a.bias && jb < a.NOUT) ? a.bias[jb] : 0.f;
    int gi = p * nchunks;
    for (int ch = 0; ch < nchunks; ++ch, ++gi) {
      float* cur = smem + (gi & 1) * STAGE;
      if (gi + 1 < total) PMU_FETCH4(gi + 1, smem + ((gi + 1) & 1) * STAGE)
      const unsigned pa = lds_addr(cur + pbase), ua = lds_addr(cur + ubase);
      if constexpr (PM == 2) w4_chunk64<CH>(pa, ua, acc);
      else w4_chunk<CH, PM == 1>(pa, ua, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next chunk's DMA has landed
      __syncthreads();
    }
    // launder the block origin so the epilogue's address arithmetic is not hoisted out of the pass
    // loop (it would be held, and spilled, across the MFMA loop)
    int ne = B.n, h0e = B.h0, w0e = B.w0;
    asm volatile("" : "+s"(ne), "+s"(h0e), "+s"(w0e));
    float* xb = smem + ((gi - 1) & 1) * STAGE;
    wino4_epilogue<DGRAD, BNR, CH, EXP>(a, ne, h0e, w0e, j0, B.spatial, acc, xb, red, bias);
    if (p + 1 < B.npass) {  // block-uniform: every wave takes the barrier
      // the exchange overwrote xb's stage: restore its zero units (each thread its own) before the
      // next pass reads it
#pragma unroll
      for (int r = 0; r < NGL; ++r)
        if ((B.gzero >> r) & 1u) *reinterpret_cast<float4*>(xb + 4 * (r * NT + tid)) = make_float4(0.f, 0.f, 0.f, 0.f);
      __syncthreads();
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int c = 0; c < 18; ++c) acc[h][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#undef PMU_FETCH4
#undef PMU_GLDS
}

// A workgroup walks a.cpb output-channel blocks of one spatial block in passes; the flat
// (pass, chunk) sequence is one DMA pipeline, so the next pass's first chunk lands under this
// pass's epilogue.  Waves 0-3 compute components 0..17 (rows 0-2 of the 6x6 grid), waves 4-7 the
// rest, each for its tile group's 16 tiles x all 32 output channels.
// BNR (input gradient only): the producer's BN-backward partial sums in the epilogue (a.bz set) — a
// compile-time choice, so the z loads and their uses sit in straight-line code
// EXP (timing experiments, experiments build, PMU_WINO4_EXP; wrong results on purpose): 6 = no output
// stores, 8 = no z loads in the BN-backward epilogue
template <bool DGRAD, bool BNR, int PM, int EXP = 0>
__global__ __launch_bounds__(NT, 1) void conv3x3_wino4_kernel(W4Args a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE + RED_FLOATS];
  const int tid = threadIdx.x;
  const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
  const int ncog = (a.nco + a.cpb - 1) / a.cpb;
  W4Block B;
  int cg, sp;
  if (a.tc > 0) {
    // 2-D grouping (the host checked ncog % tc == 0 and spatial % ts == 0): an XCD's consecutive
    // workgroups cover ts spatial blocks x tc co-groups, so its L2 holds ts operand images and tc U
    // slices at a time instead of 1 image and all U slices
    const int gsz = a.ts * a.tc, g = lb / gsz, i = lb - g * gsz;
    const int gpr = ncog / a.tc;
    cg = (g % gpr) * a.tc + i % a.tc;
    sp = (g / gpr) * a.ts + i / a.tc;
  } else {
    cg = lb % ncog;
    sp = lb / ncog;
  }
  B.cob0 = cg * a.cpb;
  B.spatial = sp;
  const int bx = sp % a.bw; sp /= a.bw;
  const int by = sp % a.bh;
  B.n = sp / a.bh;
  B.h0 = by * OH;
  B.w0 = bx * OW;
  const int KC = a.KC;
  B.nchunks = KC / BK;
  B.npass = a.cpb < a.nco - B.cob0 ? a.cpb : a.nco - B.cob0;
  PMU_DCHECK(B.n < a.N && B.cob0 < a.nco, PMU_DBG_GRID);

  // this thread's operand units: byte offset of chunk 0 (< 2^32, host-checked) and whether the unit
  // is inside the input; units of the image outside it are zeroed in both stages once
  unsigned goff[NGL];
  unsigned gin = 0u, gzero = 0u;
#pragma unroll
  for (int r = 0; r < NGL; ++r) {
    const int u = r * NT + tid;
    const int hr = u / ROWU, wu = u - hr * ROWU;
    const int g = wu / 9, w9 = wu - 9 * g;
    const int px = 4 * g + (w9 >> 1);
    const bool data = u < A_UNITS && w9 < 8 && px < HW;
    const int h = B.h0 - 1 + hr, w = B.w0 - 1 + px;
    const bool in = data && h >= 0 && w >= 0 && h < a.H && w < a.W;
    goff[r] = in ? (unsigned)(((((long long)B.n * a.H + h) * a.W + w) * KC + 4 * (w9 & 1)) * 4) : 0u;
    PMU_DCHECK(!in || (((long long)B.n * a.H + h) * a.W + w) < (long long)a.N * a.H * a.W, PMU_DBG_OPERAND);
    gin |= in ? (1u << r) : 0u;
    gzero |= (data && !in) ? (1u << r) : 0u;
    if (data && !in) {
      *reinterpret_cast<float4*>(smem + 4 * u) = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(smem + STAGE + 4 * u) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  B.gin = gin;
  B.gzero = gzero;
  if (a.prio && (tid >> 8)) __builtin_amdgcn_s_setprio(1);
  if (tid >> 8) wino4_main<DGRAD, BNR, 1, PM, EXP>(a, B, goff, smem);
  else wino4_main<DGRAD, BNR, 0, PM, EXP>(a, B, goff, smem);
}

int launch_wino4(const float* x, int KC, int N, int H, int W, const float* wp, const float* bias, int NOUT,
                 float* out0, float* out1, int split, float* part, bool dgrad, void* stream,
                 const float* bz = nullptr, const float* bcoef = nullptr, const float* bmean = nullptr,
                 const float* binv = nullptr) {
  PMU_REQUIRE(x && wp && out0 && KC > 0 && KC % BK == 0 && NOUT > 0 && N > 0 && H > 0 && W > 0);
  const long long img_bytes = (long long)H * W * (KC > NOUT ? KC : NOUT) * 4;
  if ((long long)N * img_bytes >= (1LL << 32)) {  // 32-bit DMA byte offsets: split over images
    const long long tiles = (long long)pmu_cdiv(W, OW) * pmu_cdiv(H, OH);
    return pmu_image_chunks(N, img_bytes, [&](int n0, int nn) {
      const long long px = (long long)n0 * H * W;
      return launch_wino4(x + px * KC, KC, nn, H, W, wp, bias, NOUT, out0 + px * split,
                  out1 ? out1 + px * (NOUT - split) : nullptr, split,
                  part ? part + (long long)n0 * tiles * 2 * NOUT : nullptr, dgrad, stream,
                  bz ? bz + px * NOUT : nullptr, bcoef, bmean, binv);
    });
  }
  W4Args a;
  memset(&a, 0, sizeof(a));
  a.x = x; a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part;
  a.H = H; a.W = W; a.KC = KC; a.NOUT = NOUT; a.split = split;
  a.N = N;
  a.bz = bz; a.bcoef = bcoef; a.bmean = bmean; a.binv = binv;
  a.bw = pmu_cdiv(W, OW);
  a.bh = pmu_cdiv(H, OH);
  a.nco = pmu_cdiv(NOUT, CO);
  const long long spatial = (long long)a.bw * a.bh * N;
  // co-block passes per workgroup (the per-workgroup prologue is paid once per pass group) while
  // keeping >= PMU_WINO4_MINWG workgroups; PMU_WINO4_CPB forces a value (A/B)
  static const int cpb_env = [] {
    const char* e = getenv("PMU_WINO4_CPB");
    return e ? atoi(e) : 0;
  }();
  static const long long min_wg = [] {
    const char* e = getenv("PMU_WINO4_MINWG");
    return e ? atoll(e) : 1024LL;
  }();
  int cpb = 1;
  if (cpb_env > 0) {
    cpb = cpb_env < a.nco ? cpb_env : a.nco;
  } else {
    while (cpb * 2 <= a.nco && spatial * pmu_cdiv(a.nco, cpb * 2) >= min_wg) cpb *= 2;
  }
  a.cpb = cpb;
  // patch read (A/B, experiments build): PMU_WINO4_PF=1 b32 with prefetch, PMU_WINO4_B32=1 b32; default b64 pairs
  static const int pf = [] {
    const char* e = pmu_variant_env("PMU_WINO4_PF");
    return e ? atoi(e) : 0;
  }();
  static const int b32 = [] {
    const char* e = pmu_variant_env("PMU_WINO4_B32");
    return e ? atoi(e) : 0;
  }();
  const int pm = pf ? 1 : b32 ? 0 : 2;
  static const int prio = [] {  // PMU_WINO4_PRIO=1: waves of component half 1 at s_setprio 1 (A/B)
    const char* e = pmu_variant_env("PMU_WINO4_PRIO");
    return e ? atoi(e) : 0;
  }();
  a.prio = prio;
  static const int grp = [] {  // PMU_WINO4_GROUP=0: co-groups fastest (A/B)
    const char* e = pmu_variant_env("PMU_WINO4_GROUP");
    return e ? atoi(e) : 1;
  }();
  {
    const int ncog = pmu_cdiv(a.nco, cpb);
    a.tc = 0; a.ts = 0;
    if (grp) {
      const int tc = ncog < 8 ? ncog : 8, ts = 32 / tc;
      if (ncog % tc == 0 && spatial % ts == 0 && tc > 1 && ts > 1) { a.tc = tc; a.ts = ts; }
    }
  }
  const long long blocks = (long long)pmu_cdiv(a.nco, cpb) * spatial;
  PMU_REQUIRE(blocks < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)blocks);
#ifdef PMU_EXPERIMENTS
  static const int exp_v = [] {
    const char* e = pmu_variant_env("PMU_WINO4_EXP");
    return e ? atoi(e) : 0;
  }();
  if (dgrad && pm == 2 && (exp_v == 6 || exp_v == 8)) {
    if (bz && exp_v == 6) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, true, 2, 6>), grid, dim3(NT), 0, st, a);
    else if (bz) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, true, 2, 8>), grid, dim3(NT), 0, st, a);
    else if (exp_v == 6) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, false, 2, 6>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_wino4_kernel<true, false, 2>), grid, dim3(NT), 0, st, a);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  if (dgrad && bz && pm == 0) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, true, 0>), grid, dim3(NT), 0, st, a);
  else if (dgrad && bz) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, true, 2>), grid, dim3(NT), 0, st, a);
  else if (dgrad && pm == 1) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, false, 1>), grid, dim3(NT), 0, st, a);
  else if (dgrad && pm == 0) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, false, 0>), grid, dim3(NT), 0, st, a);
  else if (dgrad) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, false, 2>), grid, dim3(NT), 0, st, a);
  else if (pm == 1) hipLaunchKernelGGL((conv3x3_wino4_kernel<false, false, 1>), grid, dim3(NT), 0, st, a);
  else if (pm == 0) hipLaunchKernelGGL((conv3x3_wino4_kernel<false, false, 0>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((conv3x3_wino4_kernel<false, false, 2>), grid, dim3(NT), 0, st, a);
#else
  (void)pm;
  if (dgrad && bz) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, true, 2>), grid, dim3(NT), 0, st, a);
  else if (dgrad) hipLaunchKernelGGL((conv3x3_wino4_kernel<true, false, 2>), grid, dim3(NT), 0, st, a);
  else return PMU_ERR_ARG;  // the F(4x4) forward is an experiments-build kernel (see pmu_conv3x3_fwd_wino4)
#endif
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

extern "C" int pmu_conv3x3_tiles_wino4(int N, int H, int W) { return N * pmu_cdiv(H, OH) * pmu_cdiv(W, OW); }

extern "C" size_t pmu_conv3x3_packed_size_wino4(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  return (size_t)pmu_cdiv(NOUT, CO) * pmu_cdiv(KC, BK) * U_FLOATS * sizeof(float);
}

extern "C" int pmu_conv3x3_pack_wino4(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const unsigned segs = (unsigned)(pmu_cdiv(NOUT, CO) * pmu_cdiv(KC, BK));  // one workgroup per segment
  hipLaunchKernelGGL(pack_wino4_kernel, dim3(segs), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

#ifdef PMU_EXPERIMENTS
// The F(4x4) forward: built, tested (tests/test_wino4_gpu.py) and measured (+41 slices/s on c2), but its
// fp32 rounding enters the BatchNorm statistics and breaks the model-level 1e-3 / Dice contract
// (DESIGN.md §3a), so it ships only in the experiments build (include/pmunet_hip_experiments.h).
extern "C" int pmu_conv3x3_fwd_wino4(const float* xt, int Cin, int N, int H, int W, const float* wp, const float* bias,
                                     int Cout, float* z, float* part, void* stream) {
  return launch_wino4(xt, Cin, N, H, W, wp, bias, Cout, z, nullptr, Cout, part, false, stream);
}
#endif

extern "C" int pmu_conv3x3_dgrad_wino4(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                       int Csplit, float* dx0, float* dx1, void* stream) {
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  return launch_wino4(dzt, Cout, N, H, W, wp, nullptr, Cin, dx0, dx1, Csplit, nullptr, true, stream);
}

// The input gradient fused with the BatchNorm+ReLU backward reduction of the layer whose output
// this conv consumed (dx = that layer's da): part[pmu_conv3x3_tiles_wino4 rows][2][Cin] as
// pmu_bn_bwd_reduce would compute them from (dx, z) — dx is not read back.
extern "C" int pmu_conv3x3_dgrad_wino4_bnr(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                           float* dx, const float* z, const float* coef, const float* mean,
                                           const float* invstd, float* part, void* stream) {
  PMU_REQUIRE(z && coef && mean && invstd && part);
  return launch_wino4(dzt, Cout, N, H, W, wp, nullptr, Cin, dx, nullptr, Cin, part, true, stream, z, coef, mean,
                      invstd);
}

extern "C" int pmu_conv3x3_pack_wino4_blocks(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  return pmu_cdiv(NOUT, CO) * pmu_cdiv(KC, BK);
}

extern "C" int pmu_conv3x3_pack_wino4_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream) {
  PMU_REQUIRE(jobs && njobs > 0 && blocks > 0);
  hipLaunchKernelGGL(pack_wino4_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, jobs, njobs,
                     dgrad);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
