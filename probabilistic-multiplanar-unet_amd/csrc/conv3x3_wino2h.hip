// 3x3 / pad 1 convolution in fp32 by Winograd F(2x2, 3x3), high-occupancy variant: the forward of
// nn.Conv2d at PMU/model/unet/unet_parts.py:15,18 (and its input gradient) on a materialised NHWC
// operand, the same arithmetic as conv3x3_wino.hip's raw kernel (16 products per 2x2 tile per channel
// pair; transforms with coefficients 0, +-1, +-1/2; results equal the direct sum to fp32 rounding).
//
// Block: 1024 threads = 16 waves, four per SIMD (the weight gradient measured 12% faster going from
// two to four waves per SIMD): 64 tiles (8 x 8 -> a 16 x 16 output patch) x 64 output channels.
// Wave w = (tile group tg = w & 3: tile rows 2tg, 2tg+1; component half ch = (w >> 2) & 1: rows
// 2ch, 2ch+1 of the 4x4 component grid; channel group cg = w >> 3: 32 outputs).  A wave keeps 8
// components x 2 co halves = 16 f32x4 accumulators (64 registers, < 128 in all), forms only its half
// of V = B^T d B (16 VALU for 16 MFMAs) and the two component halves of a tile group swap partial
// outputs through a free LDS stage in the epilogue.  Per chunk of 8 input channels (two MFMA steps),
// double-buffered stages receive the 18 x 18 x 8 operand image (2-pixel groups + a pad unit) and U
// (8 ch x 64 co x 16 comps, rows padded to 20 floats) by LDS-DMA; the patch is read per step as 16
// ds_read_b32.
#include <string.h>
#include <stdlib.h>
#include "pmu_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TX = 8, TY = 8;                 // tiles per block
constexpr int OW = 2 * TX, OH = 2 * TY;       // 16 x 16 output pixels
constexpr int HW = OW + 2, HH = OH + 2;       // 18 x 18 halo
constexpr int BK = 8;                         // input channels per chunk
constexpr int GP = 20;                        // floats per group of 2 halo pixels (2 x 8 ch + 1 pad unit)
constexpr int ROWF = 208;                     // floats per halo row (9 groups = 180, padded to 16 mod 32:
                                              // the wave's two tile rows 2 ROWF = 32 mod 64 floats apart,
                                              // conflict-free ds_read_b64 patch pairs, see w2_pair)
constexpr int ROWU = ROWF / 4;
constexpr int A_FLOATS = HH * ROWF;
[[maybe_unused]] constexpr int NC = 16;       // Winograd components
constexpr int NCP = 16;                       // floats per U row: the 16 components as four 16-B units, unit q
                                              // of row r stored at q ^ u_swz(r) (the lanes' b128 U reads
                                              // conflict-free without a pad unit, see u_swz)
constexpr int A_UNITS = A_FLOATS / 4;

// U row r = kl * CO + co (channel in chunk, output channel in block) keeps its 16-B unit q at q ^ u_swz(r):
// 16 lanes reading rows r .. r + 15 (one b128 phase) then cover the 64 banks once — rows 4 apart, 256 B
// = 64 banks apart, land on different units.  Every lane's row is 32 cg + 16 h + t (+ CO per channel, CO a
// multiple of 16), so u_swz(row) = (t >> 2) & 3 for the lane's t = lane & 15.
__host__ __device__ constexpr int u_swz(int row) { return (row >> 2) & 3; }

// block geometry by output channels per block: 64 (1024 threads, 16 waves, one block per CU) or 32
// (512 threads, 8 waves, 67 KB of LDS: two blocks per CU, PMU_WINO2H_CO=32)
template <int CO_>
struct W2Cfg {
  static constexpr int CO = CO_;
  static constexpr int NT = 16 * CO_;
  static constexpr int NW = NT / 64;
  static constexpr int U_FLOATS = BK * CO_ * NCP;          // [ch 8][co][comp 16, units swizzled]
  static constexpr int STAGE = A_FLOATS + U_FLOATS;
  static constexpr int NGL = (A_UNITS + NT - 1) / NT;
  static constexpr int UGL = (U_FLOATS / 4 + NT - 1) / NT;  // U DMA rounds (the last one by the first waves)
  static constexpr int RED_FLOATS = NW * 16 * 2;
  static constexpr int XB_FLOATS = NW * 2 * 4 * 64;         // one exchange round: waves x 2 tiles x 4 outputs x lanes
  static_assert(U_FLOATS % (4 * 64) == 0, "U of whole wave DMA instructions");
  static_assert(XB_FLOATS <= STAGE, "exchange round fits a stage");
  static_assert((2 * STAGE + RED_FLOATS) * 4 <= 160 * 1024, "LDS");
};

struct W2Args {
  const float* x;     // [N][H][W][KC]
  const float* wp;    // packed U [co block][chunk][ch 8][co 64][comp 16, units swizzled by u_swz]
  const float* bias;
  float* out0;
  float* out1;
  float* part;        // [spatial blocks][2][NOUT] BN partial sums (fwd) or null
  int H, W, KC, NOUT, split, bw, bh, nco, cpb;
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

__device__ __forceinline__ void wino2_u(const float (&g)[3][3], float (&u)[16]) {
  float t[4][3];
  for (int b = 0; b < 3; ++b) {
    t[0][b] = g[0][b];
    t[1][b] = 0.5f * (g[0][b] + g[1][b] + g[2][b]);
    t[2][b] = 0.5f * (g[0][b] - g[1][b] + g[2][b]);
    t[3][b] = g[2][b];
  }
  for (int a = 0; a < 4; ++a) {
    u[4 * a + 0] = t[a][0];
    u[4 * a + 1] = 0.5f * (t[a][0] + t[a][1] + t[a][2]);
    u[4 * a + 2] = 0.5f * (t[a][0] - t[a][1] + t[a][2]);
    u[4 * a + 3] = t[a][2];
  }
}

// U = G g G^T, G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1]; one thread per (co block, chunk,
// channel, co) writes its 16 components (c = 4a + b) as 4 float4 (input-gradient packing: consecutive
// threads read consecutive filters w[co][ci..])
template <int CO>
__device__ __forceinline__ void pack_wino2h_body(const float* __restrict__ w, int Cout, int Cin, int dgrad,
                                                 float* __restrict__ wp, int bid, int nblk) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int nch = (KC + BK - 1) / BK, ncob = (NOUT + CO - 1) / CO;
  const long long total = (long long)ncob * nch * BK * CO;
  for (long long e = (long long)bid * blockDim.x + threadIdx.x; e < total; e += (long long)nblk * blockDim.x) {
    const int col = (int)(e % CO);
    long long r = e / CO;
    const int kl = (int)(r % BK); r /= BK;
    const int ch = (int)(r % nch);
    const int jb = (int)(r / nch);
    const int j = jb * CO + col, k = ch * BK + kl;
    float g[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        float v = 0.f;
        if (j < NOUT && k < KC)  // dgrad: the input gradient convolves dz with w[co][ci] rotated by 180 degrees
          v = dgrad ? w[((long long)k * Cin + j) * 9 + (2 - a) * 3 + (2 - b)] : w[((long long)j * Cin + k) * 9 + a * 3 + b];
        g[a][b] = v;
      }
    float u[16];
    wino2_u(g, u);
    float* dst = wp + (((long long)jb * nch + ch) * BK + kl) * (CO * NCP) + col * NCP;
    const int sw = u_swz(kl * CO + col);
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(dst + 4 * (q ^ sw)) = make_float4(u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]);
  }
}
template <int CO>
__global__ void pack_wino2h_kernel(const float* __restrict__ w, int Cout, int Cin, int dgrad, float* __restrict__ wp) {
  pack_wino2h_body<CO>(w, Cout, Cin, dgrad, wp, blockIdx.x, gridDim.x);
}

// Forward packing, one workgroup per (co block, chunk): the 8 x CO filters w[co][ci0..ci0+7] are read
// along ci (8 lanes cover 288 contiguous bytes), transformed into LDS in the packed order, and the
// workgroup's contiguous BK x CO x NCP segment is stored with consecutive float4s.
template <int CO>
__device__ __forceinline__ void pack_wino2h_fwd_body(const float* __restrict__ w, int Cout, int Cin,
                                                     float* __restrict__ wp, int bid) {
  constexpr int SEG = BK * CO * NCP;
  __shared__ float4 seg4[SEG / 4];
  const int nch = (Cin + BK - 1) / BK;
  const int ch = bid % nch, jb = bid / nch;
  for (int f = threadIdx.x; f < BK * CO; f += blockDim.x) {
    const int kl = f % BK, col = f / BK;
    const int j = jb * CO + col, k = ch * BK + kl;
    float g[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) g[a][b] = (j < Cout && k < Cin) ? w[((long long)j * Cin + k) * 9 + a * 3 + b] : 0.f;
    float u[16];
    wino2_u(g, u);
    float4* d = seg4 + (kl * CO + col) * (NCP / 4);
    const int sw = u_swz(kl * CO + col);
    for (int q = 0; q < 4; ++q) d[q ^ sw] = make_float4(u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]);
  }
  __syncthreads();
  float4* dst = reinterpret_cast<float4*>(wp + (long long)bid * SEG);
  for (int i = threadIdx.x; i < SEG / 4; i += blockDim.x) dst[i] = seg4[i];
}
template <int CO>
__global__ __launch_bounds__(256) void pack_wino2h_fwd_kernel(const float* __restrict__ w, int Cout, int Cin,
                                                              float* __restrict__ wp) {
  pack_wino2h_fwd_body<CO>(w, Cout, Cin, wp, blockIdx.x);
}
__global__ __launch_bounds__(256) void pack_wino2h_multi_kernel(const pmu_pack_job* __restrict__ jobs, int njobs,
                                                                int dgrad) {
  const pmu_pack_job& j = jobs[pmu_job_of(jobs, njobs, blockIdx.x)];
  const int bid = blockIdx.x - j.block0;
  if (dgrad) pack_wino2h_body<64>(j.w, j.Cout, j.Cin, 1, (float*)j.dst, bid, j.nblocks);
  else pack_wino2h_fwd_body<64>(j.w, j.Cout, j.Cin, (float*)j.dst, bid);
}

template <int OFF>
__device__ __forceinline__ float2 lds_b64(unsigned addr) {
  float2 v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ float lds_b32(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ float4 lds_b128(unsigned addr) {
  float4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(p);
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N <= 15, "lgkmcnt");
  __builtin_amdgcn_s_waitcnt(0xC07F | (N << 8));
}

// patch element (i, j) of this lane's tile: byte offset from the patch origin
#define PMU_W2P(I, J) ((((I) * ROWF) + ((J) >> 1) * GP + ((J) & 1) * 8) * 4)

// one MFMA step (channel 2*kk + ks in k-slot kk): patch (16 x b32), U (2 groups x 2 co halves x b128),
// half CH of B^T d B (rows 2CH, 2CH+1; B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]), 16 MFMAs
template <int CH>
__device__ __forceinline__ void w2_step(unsigned pa, unsigned ua0, unsigned ua1, f32x4 (&acc)[2][8]) {
  float d[16];
#define PMU_RD(I, J) d[4 * (I) + (J)] = lds_b32<PMU_W2P(I, J)>(pa);
  PMU_RD(0, 0) PMU_RD(0, 1) PMU_RD(0, 2) PMU_RD(0, 3) PMU_RD(1, 0) PMU_RD(1, 1) PMU_RD(1, 2) PMU_RD(1, 3)
  PMU_RD(2, 0) PMU_RD(2, 1) PMU_RD(2, 2) PMU_RD(2, 3) PMU_RD(3, 0) PMU_RD(3, 1) PMU_RD(3, 2) PMU_RD(3, 3)
#undef PMU_RD
  // U of this half: components 8CH .. 8CH+7 (units 2CH at ua0, 2CH + 1 at ua1) of co half h at row
  // offset 16*NCP*h
  const float4 u00 = lds_b128<0>(ua0);
  const float4 u10 = lds_b128<16 * NCP * 4>(ua0);
  const float4 u01 = lds_b128<0>(ua1);
  const float4 u11 = lds_b128<16 * NCP * 4>(ua1);
  wait_lgkm<2>();  // the patch and U group 0
  __builtin_amdgcn_sched_barrier(0);
  float t[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (CH == 0) {
      t[0][j] = d[j] - d[8 + j];
      t[1][j] = d[4 + j] + d[8 + j];
    } else {
      t[0][j] = d[8 + j] - d[4 + j];
      t[1][j] = d[4 + j] - d[12 + j];
    }
  }
  float v[8];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    v[4 * a + 0] = t[a][0] - t[a][2];
    v[4 * a + 1] = t[a][1] + t[a][2];
    v[4 * a + 2] = t[a][2] - t[a][1];
    v[4 * a + 3] = t[a][1] - t[a][3];
  }
  __builtin_amdgcn_sched_barrier(0);
  acc[0][0] = mfma16(v[0], u00.x, acc[0][0]);
  acc[1][0] = mfma16(v[0], u10.x, acc[1][0]);
  acc[0][1] = mfma16(v[1], u00.y, acc[0][1]);
  acc[1][1] = mfma16(v[1], u10.y, acc[1][1]);
  acc[0][2] = mfma16(v[2], u00.z, acc[0][2]);
  acc[1][2] = mfma16(v[2], u10.z, acc[1][2]);
  acc[0][3] = mfma16(v[3], u00.w, acc[0][3]);
  acc[1][3] = mfma16(v[3], u10.w, acc[1][3]);
  __builtin_amdgcn_sched_barrier(0);
  wait_lgkm<0>();
  __builtin_amdgcn_sched_barrier(0);
  acc[0][4] = mfma16(v[4], u01.x, acc[0][4]);
  acc[1][4] = mfma16(v[4], u11.x, acc[1][4]);
  acc[0][5] = mfma16(v[5], u01.y, acc[0][5]);
  acc[1][5] = mfma16(v[5], u11.y, acc[1][5]);
  acc[0][6] = mfma16(v[6], u01.z, acc[0][6]);
  acc[1][6] = mfma16(v[6], u11.z, acc[1][6]);
  acc[0][7] = mfma16(v[7], u01.w, acc[0][7]);
  acc[1][7] = mfma16(v[7], u11.w, acc[1][7]);
  __builtin_amdgcn_sched_barrier(0);
}

// half CH of B^T d B from the column-pass halves t[a][j] (a = 0, 1): v[4a + b]
__device__ __forceinline__ void w2_rows(const float (&t)[2][4], float (&v)[8]) {
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    v[4 * a + 0] = t[a][0] - t[a][2];
    v[4 * a + 1] = t[a][1] + t[a][2];
    v[4 * a + 2] = t[a][2] - t[a][1];
    v[4 * a + 3] = t[a][1] - t[a][3];
  }
}

// 16 MFMAs of one step on v with U groups (u00, u10) and (u01, u11); the second group waited for here
// (W: lgkmcnt allowing the reads issued after it)
template <int W>
__device__ __forceinline__ void w2_mfma(const float (&v)[8], float4 u00, float4 u10, float4 u01, float4 u11,
                                        f32x4 (&acc)[2][8]) {
  acc[0][0] = mfma16(v[0], u00.x, acc[0][0]);
  acc[1][0] = mfma16(v[0], u10.x, acc[1][0]);
  acc[0][1] = mfma16(v[1], u00.y, acc[0][1]);
  acc[1][1] = mfma16(v[1], u10.y, acc[1][1]);
  acc[0][2] = mfma16(v[2], u00.z, acc[0][2]);
  acc[1][2] = mfma16(v[2], u10.z, acc[1][2]);
  acc[0][3] = mfma16(v[3], u00.w, acc[0][3]);
  acc[1][3] = mfma16(v[3], u10.w, acc[1][3]);
  __builtin_amdgcn_sched_barrier(0);
  wait_lgkm<W>();
  __builtin_amdgcn_sched_barrier(0);
  acc[0][4] = mfma16(v[4], u01.x, acc[0][4]);
  acc[1][4] = mfma16(v[4], u11.x, acc[1][4]);
  acc[0][5] = mfma16(v[5], u01.y, acc[0][5]);
  acc[1][5] = mfma16(v[5], u11.y, acc[1][5]);
  acc[0][6] = mfma16(v[6], u01.z, acc[0][6]);
  acc[1][6] = mfma16(v[6], u11.z, acc[1][6]);
  acc[0][7] = mfma16(v[7], u01.w, acc[0][7]);
  acc[1][7] = mfma16(v[7], u11.w, acc[1][7]);
  __builtin_amdgcn_sched_barrier(0);
}

// Both MFMA steps of a chunk (channels 2kk, 2kk + 1 of k-slot kk) with the patch read as ds_read_b64
// channel pairs, and only the three patch rows this component half uses (rows CH .. CH + 2): 12 b64 reads
// per chunk instead of 2 x 16 b32.  Bank map of a 32-lane group (b64: dword banks mod 64): tile columns
// GP = 20 floats apart, the wave's two tile rows 2 ROWF = 32 (mod 64) apart, the k-slot pair 2 floats:
// the 16 tiles x 2 k-slots cover the 64 banks once (the b32 reads of one channel were 2-way: tile rows
// 368 = 16 (mod 32) apart put both rows of tiles on the same 8 bank quads).
template <int CH, int CO>
__device__ __forceinline__ void w2_pair(unsigned pa, unsigned ua0, f32x4 (&acc)[2][8]) {
  float2 c[3][4];
#define PMU_RD2(I, J) c[I][J] = lds_b64<PMU_W2P(CH + (I), J)>(pa);
  PMU_RD2(0, 0) PMU_RD2(0, 1) PMU_RD2(0, 2) PMU_RD2(0, 3) PMU_RD2(1, 0) PMU_RD2(1, 1) PMU_RD2(1, 2) PMU_RD2(1, 3)
  PMU_RD2(2, 0) PMU_RD2(2, 1) PMU_RD2(2, 2) PMU_RD2(2, 3)
#undef PMU_RD2
  wait_lgkm<0>();  // the patch
  __builtin_amdgcn_sched_barrier(0);
  // column pass (rows CH .. CH+2 of d as c[0..2]): CH 0: (d0 - d2, d1 + d2); CH 1: (d2 - d1, d1 - d3)
  float t0[2][4], t1[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (CH == 0) {
      t0[0][j] = c[0][j].x - c[2][j].x;
      t0[1][j] = c[1][j].x + c[2][j].x;
      t1[0][j] = c[0][j].y - c[2][j].y;
      t1[1][j] = c[1][j].y + c[2][j].y;
    } else {
      t0[0][j] = c[1][j].x - c[0][j].x;
      t0[1][j] = c[0][j].x - c[2][j].x;
      t1[0][j] = c[1][j].y - c[0][j].y;
      t1[1][j] = c[0][j].y - c[2][j].y;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // U after the patch is consumed (at the 128-register cap of four waves per SIMD the patch pairs and U
  // together spilled; the SIMD's other waves cover the U read latency)
  // (unit 2CH + 1 at ua0 ^ 16, formed at each use: one register fewer live across the MFMAs)
  float4 u00 = lds_b128<0>(ua0);
  float4 u10 = lds_b128<16 * NCP * 4>(ua0);
  float4 u01 = lds_b128<0>(ua0 ^ 16u);
  float4 u11 = lds_b128<16 * NCP * 4>(ua0 ^ 16u);
  float v[8];
  w2_rows(t0, v);
  wait_lgkm<2>();  // U group 0
  __builtin_amdgcn_sched_barrier(0);
  w2_mfma<0>(v, u00, u10, u01, u11, acc);
  const unsigned ub = ua0 + CO * NCP * 4;  // step 1: the next channel's rows, CO rows on (same swizzle)
  u00 = lds_b128<0>(ub);
  u10 = lds_b128<16 * NCP * 4>(ub);
  u01 = lds_b128<0>(ub ^ 16u);
  u11 = lds_b128<16 * NCP * 4>(ub ^ 16u);
  w2_rows(t1, v);
  wait_lgkm<2>();  // step 1's U group 0
  __builtin_amdgcn_sched_barrier(0);
  w2_mfma<0>(v, u00, u10, u01, u11, acc);
}

// this half's share of Y = A^T M A (A^T = [1 1 1 0; 0 1 -1 -1]) for tile r of co half h:
// P[2p + q] = sum over the half's rows a of A^T[p][a] (M[a][:] A)[q]
template <int CH>
__device__ __forceinline__ void w2_partial(const f32x4 (&acc)[2][8], int h, int r, float (&P)[4]) {
  float R[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float m0 = acc[h][4 * a][r], m1 = acc[h][4 * a + 1][r], m2 = acc[h][4 * a + 2][r], m3 = acc[h][4 * a + 3][r];
    R[a][0] = m0 + m1 + m2;
    R[a][1] = m1 - m2 - m3;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (CH == 0) {  // rows 0, 1: A^T columns (1, 0), (1, 1)
      P[q] = R[0][q] + R[1][q];
      P[2 + q] = R[1][q];
    } else {        // rows 2, 3: A^T columns (1, -1), (0, -1)
      P[q] = R[0][q];
      P[2 + q] = -R[0][q] - R[1][q];
    }
  }
}

// epilogue: lane holds M[comp (half CH)][tile 4*kk + r of the group][co j0 + 32 cg + 16 h + (lane & 15)];
// the two component halves of (tg, cg) swap the partial outputs of the co half the other finishes
// through xb (a free LDS stage), in two rounds of two tiles per lane
template <bool DGRAD, bool BNR, int CH, int CO, bool NOST = false>
__device__ __forceinline__ void wino2h_epilogue(const W2Args& a, int n, int h0, int w0, int j0, int spatial,
                                                const f32x4 (&acc)[2][8], float* xb, float* red, float bias) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kk = lane >> 4;
  const int tg = wave & 3, cg = wave >> 3, partner = tg + 4 * (1 - CH) + 8 * cg;
  const int j = j0 + 32 * cg + 16 * CH + (lane & 15);
  const bool jok = j < a.NOUT;
  // this lane's output column: the forward's z, or the input gradient's dx0 / dx1 side of the split
  float* dst;
  int ld;
  if (!DGRAD) { dst = a.out0 + j; ld = a.NOUT; }
  else if (j < a.split) { dst = a.out0 + j; ld = a.split; }
  else { dst = a.out1 + (j - a.split); ld = a.NOUT - a.split; }
  float s1 = 0.f, s2 = 0.f;
  float bsc = 0.f, bsh = 0.f, bmu = 0.f, bis = 0.f;
  if (BNR && jok) {
    bsc = a.bcoef[j];
    bsh = a.bcoef[a.NOUT + j];
    bmu = a.bmean[j];
    bis = a.binv[j];
  }
  // (BNR) the producer's z under a round's two tiles (4 outputs each), loaded at the start of the round,
  // before its stores: loaded per tile between the stores, each tile's z waited (in-order vmcnt) for
  // every earlier store of the epilogue — four HBM round trips per wave behind the stores, now one (the
  // second round's).  All four tiles' z up front spilled 18 VGPRs.  Clamped addresses: every lane loads,
  // unused values are ignored.
  float zt2[2][4];
#pragma unroll
  for (int rho = 0; rho < 2; ++rho) {
    if (BNR) {
      const int jc = min(j, a.NOUT - 1);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int t = 4 * kk + 2 * rho + rr;
        const int oh = h0 + 2 * (2 * tg + (t >> 3)), ow = w0 + 2 * (t & 7);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long long pix = ((long long)n * a.H + min(oh + (e >> 1), a.H - 1)) * a.W + min(ow + (e & 1), a.W - 1);
          zt2[rr][e] = a.bz[pix * a.NOUT + jc];
        }
      }
    }
    if (rho) __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      float P[4];
      w2_partial<CH>(acc, 1 - CH, 2 * rho + rr, P);
#pragma unroll
      for (int e = 0; e < 4; ++e) xb[((wave * 2 + rr) * 4 + e) * 64 + lane] = P[e];
    }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      const int r = 2 * rho + rr;
      const int t = 4 * kk + r;
      const int oh = h0 + 2 * (2 * tg + (t >> 3)), ow = w0 + 2 * (t & 7);
      const float (&zt)[4] = zt2[rr];
      float P[4];
      w2_partial<CH>(acc, CH, r, P);
      // the partner's partial outputs read together and held in registers before any store branch (read
      // where used, the plain input gradient's ds_reads sank into the store branches, each followed by
      // an lgkmcnt(0): serial LDS round trips).  Values, masks and BN sums are formed unconditionally
      // and only the stores are predicated: a global-memory value (bias, z) first consumed inside a
      // per-output branch made the compiler wait vmcnt(0) in every branch, i.e. for every earlier store
      // of the epilogue to complete.
      float xv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[e] = xb[((partner * 2 + rr) * 4 + e) * 64 + lane];
#pragma unroll
      for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(xv[e]));
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int hh = oh + p;
        float* rowp = dst + (long long)((long long)n * a.H + min(hh, a.H - 1)) * a.W * ld;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ww = ow + q;
          const float v = P[2 * p + q] + xv[2 * p + q] + bias;
          const bool ok = jok && hh < a.H && ww < a.W;
          if (!DGRAD) {
            const float m = ok ? v : 0.f;
            s1 += m;
            s2 = fmaf(m, m, s2);
          } else if (BNR) {
            const float zz = zt[2 * p + q];
            const float g = (ok && fmaf(zz, bsc, bsh) > 0.f) ? v : 0.f;
            s1 += g;
            s2 = fmaf(g, (zz - bmu) * bis, s2);
          }
          if (!ok || NOST) continue;
          PMU_DCHECK((((long long)n * a.H + hh) * a.W + ww) < (long long)a.N * a.H * a.W && j < a.NOUT, PMU_DBG_OUTPUT);
          rowp[(unsigned)(ww * ld)] = v;
        }
      }
    }
  }
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
    if (tid < CO) {  // channel tid = 32 cg + 16 h + l, summed over the 4 tile groups in order
      const int jj = j0 + tid, cgg = tid >> 5, hf = (tid >> 4) & 1, l = tid & 15;
      if (jj < a.NOUT) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int wv = g + 4 * hf + 8 * cgg;
          t1 += red[(wv * 16 + l) * 2 + 0];
          t2 += red[(wv * 16 + l) * 2 + 1];
        }
        PMU_DCHECK(spatial < (long long)a.N * a.bh * a.bw, PMU_DBG_WORKSPACE);
        a.part[((long long)spatial * 2 + 0) * a.NOUT + jj] = t1;
        a.part[((long long)spatial * 2 + 1) * a.NOUT + jj] = t2;
      }
    }
  }
  __syncthreads();  // the exchange reads are done before the next pass reuses xb's stage
}

struct W2Block {
  int n, h0, w0, cob0, spatial, nchunks, npass;
  unsigned gin, gzero;
};

// EXP (timing experiments, experiments build, PMU_WINO2H_EXP; wrong results on purpose): 1 = no restaging
// (every chunk reads stage 0, no DMA after the first; the chunk barrier kept), 2 = that without the barrier,
// 3 = the DMA issued as usual but never waited for (a bare s_barrier per chunk), 4 = only the operand image
// restaged (U DMA'd for the first chunk only), 5 = only U restaged, 6 = no z stores, 7 = 3 in the first chunk
// of every pass after the first only
template <bool DGRAD, bool BNR, int CH, int CO_, bool P64, int EXP = 0>
__device__ __forceinline__ void wino2h_main(const W2Args& a, const W2Block& B, const unsigned (&goff)[W2Cfg<CO_>::NGL],
                                            float* smem) {
  using C = W2Cfg<CO_>;
  constexpr int CO = C::CO, NT = C::NT, NGL = C::NGL, UGL = C::UGL, U_FLOATS = C::U_FLOATS, STAGE = C::STAGE;
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
  // serpentine chunk order over the passes (as conv3x3_wino4.hip): a pass begins on the chunks the
  // previous one fetched last, still in L2; direction by co-block parity (independent of cpb)
#define PMU_FETCH2(GI, BUF)                                                                                 \
  {                                                                                                        \
    const int p_ = (GI) / nchunks;                                                                         \
    const int c_ = (GI) - p_ * nchunks;                                                                    \
    const int cs_ = ((B.cob0 + p_) & 1) ? nchunks - 1 - c_ : c_;                                           \
    const int k0_ = cs_ * BK;                                                                              \
    PMU_DCHECK(k0_ + BK <= a.KC, PMU_DBG_OPERAND);                                                         \
    float* b_ = (BUF);                                                                                     \
    const char* xb_ = reinterpret_cast<const char*>(a.x + k0_);                                            \
    _Pragma("unroll") for (int r = 0; r < NGL; ++r)                                                        \
      if (EXP != 5 && ((gin >> r) & 1u)) PMU_GLDS(xb_ + goff[r], b_ + 4 * (r * NT) + wave_off)             \
    const char* s_ = reinterpret_cast<const char*>(wsrc + ((long long)p_ * nchunks + cs_) * U_FLOATS) + uoff; \
    float* d_ = b_ + A_FLOATS + wave_off;                                                                  \
    _Pragma("unroll") for (int r = 0; r < UGL; ++r)                                                        \
      if (EXP != 4 && r * NT * 4 + (wave + 1) * 256 <= U_FLOATS) PMU_GLDS(s_ + 16 * NT * r, d_ + 4 * NT * r) \
  }
  const int t = lane & 15, kk = lane >> 4, tg = wave & 3, cg = wave >> 3;
  const int pbase = 2 * (2 * tg + (t >> 3)) * ROWF + GP * (t & 7) + 2 * kk;
  const int ubase = A_FLOATS + (2 * kk * CO + 32 * cg + t) * NCP;
  static_assert(CO % 16 == 0, "u_swz of every row a lane reads is (t >> 2) & 3");
  // byte offset of unit 2CH of the lane's row in a stage; unit 2CH + 1 is at that ^ 16 (rows 64-B aligned:
  // smem aligned to 64, A_FLOATS and STAGE multiples of 16 floats)
  const unsigned uoff0 = 4u * ubase + 16u * ((2 * CH) ^ ((t >> 2) & 3));
  f32x4 acc[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[h][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  PMU_FETCH2(0, smem)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int p = 0; p < B.npass; ++p) {
    const int j0 = (B.cob0 + p) * CO;
    const int jb = j0 + 32 * cg + 16 * CH + t;
    const float bias = (!DGRAD && a.bias && jb < a.NOUT) ? a.bias[jb] : 0.f;
    int gi = p * nchunks;
    for (int ch = 0; ch < nchunks; ++ch, ++gi) {
      float* cur = smem + ((EXP == 1 || EXP == 2) ? 0 : (gi & 1) * STAGE);
      if (gi + 1 < total && EXP != 1 && EXP != 2) PMU_FETCH2(gi + 1, smem + ((gi + 1) & 1) * STAGE)
      const unsigned pa = lds_addr(cur + pbase), ua0 = lds_addr(cur) + uoff0, ua1 = ua0 ^ 16u;
      if constexpr (P64) {
        w2_pair<CH, CO>(pa, ua0, acc);                   // channels 2*kk, 2*kk + 1
      } else {
        w2_step<CH>(pa, ua0, ua1, acc);                  // channel 2*kk
        w2_step<CH>(pa + 4, ua0 + CO * NCP * 4, ua1 + CO * NCP * 4, acc);  // channel 2*kk + 1
      }
      if (EXP == 3 || (EXP == 7 && ch == 0 && p > 0)) {  // timing experiment: the DMA issued but never
        // waited for (a bare barrier); 7: only in a pass's first chunk, where the wait also covers the previous
        // pass's epilogue stores (in-order vmcnt)
        __builtin_amdgcn_s_barrier();
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next chunk's DMA has landed
        if (EXP != 2) __syncthreads();
      }
    }
    int ne = B.n, h0e = B.h0, w0e = B.w0;
    asm volatile("" : "+s"(ne), "+s"(h0e), "+s"(w0e));
    float* xb = smem + ((gi - 1) & 1) * STAGE;
    wino2h_epilogue<DGRAD, BNR, CH, CO, EXP == 6>(a, ne, h0e, w0e, j0, B.spatial, acc, xb, red, bias);
    if (p + 1 < B.npass) {  // block-uniform: restore the zero units the exchange overwrote
#pragma unroll
      for (int r = 0; r < NGL; ++r)
        if ((B.gzero >> r) & 1u) *reinterpret_cast<float4*>(xb + 4 * (r * NT + tid)) = make_float4(0.f, 0.f, 0.f, 0.f);
      __syncthreads();
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[h][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#undef PMU_FETCH2
#undef PMU_GLDS
}

// BNR (input gradient only): the producer's BN-backward partial sums in the epilogue (a.bz set) — a
// compile-time choice, so the z loads and their uses sit in straight-line code
template <bool DGRAD, bool BNR, int CO_, bool P64 = true, int EXP = 0>
// 64 channels: 1024 threads = four waves per SIMD (<= 128 VGPRs implied); 32 channels: 512 threads,
// capped at 128 VGPRs (four waves per SIMD) so two workgroups share a CU (at 132 VGPRs only one fit)
__global__ __launch_bounds__(16 * CO_, CO_ == 32 ? 4 : 1) void conv3x3_wino2h_kernel(W2Args a) {
  using C = W2Cfg<CO_>;
  constexpr int NT = C::NT, NGL = C::NGL, STAGE = C::STAGE;
  __shared__ __attribute__((aligned(64))) float smem[2 * STAGE + C::RED_FLOATS];
  static_assert(A_FLOATS % 16 == 0 && STAGE % 16 == 0, "U rows 64-B aligned (ua1 = ua0 ^ 16)");
  const int tid = threadIdx.x;
  const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
  const int ncog = (a.nco + a.cpb - 1) / a.cpb;
  W2Block B;
  B.cob0 = (lb % ncog) * a.cpb;
  int sp = lb / ncog;
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
  unsigned goff[NGL];
  unsigned gin = 0u, gzero = 0u;
#pragma unroll
  for (int r = 0; r < NGL; ++r) {
    const int u = r * NT + tid;
    const int hr = u / ROWU, wu = u - hr * ROWU;
    const int g = wu / 5, w5 = wu - 5 * g;
    const int px = 2 * g + (w5 >> 1);
    const bool data = u < A_UNITS && w5 < 4 && px < HW;
    const int h = B.h0 - 1 + hr, w = B.w0 - 1 + px;
    const bool in = data && h >= 0 && w >= 0 && h < a.H && w < a.W;
    goff[r] = in ? (unsigned)(((((long long)B.n * a.H + h) * a.W + w) * KC + 4 * (w5 & 1)) * 4) : 0u;
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
  if ((tid >> 8) & 1) wino2h_main<DGRAD, BNR, 1, CO_, P64, EXP>(a, B, goff, smem);
  else wino2h_main<DGRAD, BNR, 0, CO_, P64, EXP>(a, B, goff, smem);
}

// output channels per block (PMU_WINO2H_CO=32: 512-thread blocks, two per CU; A/B)
static int w2h_co() {
  static const int v = [] {
    const char* e = pmu_variant_env("PMU_WINO2H_CO");
    return (e && atoi(e) == 32) ? 32 : 64;
  }();
  return v;
}

int launch_wino2h(const float* x, int KC, int N, int H, int W, const float* wp, const float* bias, int NOUT,
                  float* out0, float* out1, int split, float* part, bool dgrad, void* stream,
                 const float* bz = nullptr, const float* bcoef = nullptr, const float* bmean = nullptr,
                 const float* binv = nullptr) {
  PMU_REQUIRE(x && wp && out0 && KC > 0 && KC % BK == 0 && NOUT > 0 && N > 0 && H > 0 && W > 0);
  const long long img_bytes = (long long)H * W * (KC > NOUT ? KC : NOUT) * 4;
  if ((long long)N * img_bytes >= (1LL << 32)) {  // 32-bit DMA byte offsets: split over images
    const long long tiles = (long long)pmu_cdiv(W, OW) * pmu_cdiv(H, OH);
    return pmu_image_chunks(N, img_bytes, [&](int n0, int nn) {
      const long long px = (long long)n0 * H * W;
      return launch_wino2h(x + px * KC, KC, nn, H, W, wp, bias, NOUT, out0 + px * split,
                  out1 ? out1 + px * (NOUT - split) : nullptr, split,
                  part ? part + (long long)n0 * tiles * 2 * NOUT : nullptr, dgrad, stream,
                  bz ? bz + px * NOUT : nullptr, bcoef, bmean, binv);
    });
  }
  W2Args a;
  memset(&a, 0, sizeof(a));
  a.x = x; a.wp = wp; a.bias = bias; a.out0 = out0; a.out1 = out1; a.part = part;
  a.H = H; a.W = W; a.KC = KC; a.NOUT = NOUT; a.split = split;
  a.N = N;
  a.bz = bz; a.bcoef = bcoef; a.bmean = bmean; a.binv = binv;
  a.bw = pmu_cdiv(W, OW);
  a.bh = pmu_cdiv(H, OH);
  const int CO = w2h_co();
  a.nco = pmu_cdiv(NOUT, CO);
  const long long spatial = (long long)a.bw * a.bh * N;
  static const int cpb_env = [] {
    const char* e = getenv("PMU_WINO2H_CPB");
    return e ? atoi(e) : 0;
  }();
  static const long long min_wg = [] {
    const char* e = getenv("PMU_WINO2H_MINWG");
    return e ? atoll(e) : 1024LL;
  }();
  int cpb = 1;
  if (cpb_env > 0) {
    cpb = cpb_env < a.nco ? cpb_env : a.nco;
  } else {
    while (cpb * 2 <= a.nco && spatial * pmu_cdiv(a.nco, cpb * 2) >= min_wg) cpb *= 2;
  }
  a.cpb = cpb;
  const long long blocks = (long long)pmu_cdiv(a.nco, cpb) * spatial;
  PMU_REQUIRE(blocks < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)blocks);
  const bool bnr = dgrad && bz;
#ifdef PMU_EXPERIMENTS
  // PMU_WINO2H_B32=1 (A/B): the patch read per channel as ds_read_b32 (w2_step), the round-5 kernel
  static const int b32 = [] {
    const char* e = pmu_variant_env("PMU_WINO2H_B32");
    return e ? atoi(e) : 0;
  }();
  static const int exp_v = [] {
    const char* e = pmu_variant_env("PMU_WINO2H_EXP");
    return e ? atoi(e) : 0;
  }();
  if (exp_v && CO == 64 && !dgrad) {
    if (exp_v == 1) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 1>), grid, dim3(1024), 0, st, a);
    else if (exp_v == 2) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 2>), grid, dim3(1024), 0, st, a);
    else if (exp_v == 4) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 4>), grid, dim3(1024), 0, st, a);
    else if (exp_v == 5) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 5>), grid, dim3(1024), 0, st, a);
    else if (exp_v == 6) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 6>), grid, dim3(1024), 0, st, a);
    else if (exp_v == 7) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 7>), grid, dim3(1024), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, true, 3>), grid, dim3(1024), 0, st, a);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  if (b32 && CO == 64) {
    if (bnr) hipLaunchKernelGGL((conv3x3_wino2h_kernel<true, true, 64, false>), grid, dim3(1024), 0, st, a);
    else if (dgrad) hipLaunchKernelGGL((conv3x3_wino2h_kernel<true, false, 64, false>), grid, dim3(1024), 0, st, a);
    else hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64, false>), grid, dim3(1024), 0, st, a);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
#endif
  if (CO == 32 && bnr) hipLaunchKernelGGL((conv3x3_wino2h_kernel<true, true, 32, false>), grid, dim3(512), 0, st, a);
  else if (CO == 32 && dgrad) hipLaunchKernelGGL((conv3x3_wino2h_kernel<true, false, 32, false>), grid, dim3(512), 0, st, a);
  else if (CO == 32) hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 32, false>), grid, dim3(512), 0, st, a);
  else if (bnr) hipLaunchKernelGGL((conv3x3_wino2h_kernel<true, true, 64>), grid, dim3(1024), 0, st, a);
  else if (dgrad) hipLaunchKernelGGL((conv3x3_wino2h_kernel<true, false, 64>), grid, dim3(1024), 0, st, a);
  else hipLaunchKernelGGL((conv3x3_wino2h_kernel<false, false, 64>), grid, dim3(1024), 0, st, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

}  // namespace

extern "C" int pmu_conv3x3_tiles_wino2h(int N, int H, int W) { return N * pmu_cdiv(H, OH) * pmu_cdiv(W, OW); }

extern "C" size_t pmu_conv3x3_packed_size_wino2h(int Cout, int Cin, int dgrad) {
  const int NOUT = dgrad ? Cin : Cout, KC = dgrad ? Cout : Cin;
  const int CO = w2h_co();
  return (size_t)pmu_cdiv(NOUT, CO) * pmu_cdiv(KC, BK) * (BK * CO * NCP) * sizeof(float);
}

extern "C" int pmu_conv3x3_pack_wino2h(const float* w, int Cout, int Cin, int dgrad, float* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cout > 0 && Cin > 0);
  const long long total = (long long)pmu_conv3x3_packed_size_wino2h(Cout, Cin, dgrad) / sizeof(float) / NCP;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  if (!dgrad) {  // one workgroup per (co block, chunk) segment
    const unsigned segs = (unsigned)(pmu_cdiv(Cout, w2h_co()) * pmu_cdiv(Cin, BK));
    if (w2h_co() == 32)
      hipLaunchKernelGGL(pack_wino2h_fwd_kernel<32>, dim3(segs), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, wp);
    else
      hipLaunchKernelGGL(pack_wino2h_fwd_kernel<64>, dim3(segs), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, wp);
  } else if (w2h_co() == 32)
    hipLaunchKernelGGL(pack_wino2h_kernel<32>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad, wp);
  else
    hipLaunchKernelGGL(pack_wino2h_kernel<64>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_conv3x3_fwd_wino2h(const float* xt, int Cin, int N, int H, int W, const float* wp, const float* bias,
                                      int Cout, float* z, float* part, void* stream) {
  return launch_wino2h(xt, Cin, N, H, W, wp, bias, Cout, z, nullptr, Cout, part, false, stream);
}

extern "C" int pmu_conv3x3_dgrad_wino2h(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                        int Csplit, float* dx0, float* dx1, void* stream) {
  PMU_REQUIRE(Csplit > 0 && Csplit <= Cin && (Csplit == Cin || dx1));
  return launch_wino2h(dzt, Cout, N, H, W, wp, nullptr, Cin, dx0, dx1, Csplit, nullptr, true, stream);
}

// As pmu_conv3x3_dgrad_wino4_bnr (part rows = pmu_conv3x3_tiles_wino2h).
extern "C" int pmu_conv3x3_dgrad_wino2h_bnr(const float* dzt, int Cout, int N, int H, int W, const float* wp, int Cin,
                                            float* dx, const float* z, const float* coef, const float* mean,
                                            const float* invstd, float* part, void* stream) {
  PMU_REQUIRE(z && coef && mean && invstd && part);
  return launch_wino2h(dzt, Cout, N, H, W, wp, nullptr, Cin, dx, nullptr, Cin, part, true, stream, z, coef, mean,
                       invstd);
}

static int pack_wino2h_grid(int Cout, int Cin, int dgrad) {
  if (!dgrad) return pmu_cdiv(Cout, w2h_co()) * pmu_cdiv(Cin, BK);
  const long long total = (long long)pmu_conv3x3_packed_size_wino2h(Cout, Cin, dgrad) / sizeof(float) / NCP;
  return (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
}

extern "C" int pmu_conv3x3_pack_wino2h_blocks(int Cout, int Cin, int dgrad) { return pack_wino2h_grid(Cout, Cin, dgrad); }

extern "C" int pmu_conv3x3_pack_wino2h_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream) {
  PMU_REQUIRE(jobs && njobs > 0 && blocks > 0 && w2h_co() == 64);
  hipLaunchKernelGGL(pack_wino2h_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, jobs, njobs,
                     dgrad);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
