// Weight gradient of the 3x3 / pad 1 convolution in fp32 by Winograd F(4x4, 3x3) (the autograd of
// nn.Conv2d w.r.t. its weight, PMU/model/unet/unet_parts.py:15,18), on the materialised operands
// (xt = the conv's input operand, dzt = dL/dz; both NHWC fp32) — the F(2x2) kernel's scheme
// (wgrad3x3_wino.hip) with 4x4 output tiles:
//     dL/dg = G^T [ sum over tiles (A dY A^T) .* (B^T X B) ] G,
// A (6x4) = [1 0 0 0; 1 1 1 1; 1 -1 1 -1; 1 2 4 8; 1 -2 4 -8; 0 0 0 1] (A^T of the forward),
// B^T (6x6) = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1],
// G (6x3) = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6; 1/24 -1/12 1/6; 0 0 1].
// 36 per-component GEMMs over the tiles, 36 products per 4x4 tile and channel pair: 2.25 per output
// pixel where F(2x2) takes 4 (1.78x fewer MFMA flops).  fp32 accumulation; the output transform in
// fp64 in the reduce.  fp32 rounding (tools/wgrad_err.py): ~1.3e-6 of rms |dw| vs F(2x2)'s 2.2e-7 —
// no BatchNorm sits behind a weight gradient to amplify it (the reason the forward stays F(2x2)).
//
// Block: 768 threads = 12 waves (3 per SIMD), 32 output x 64 input channels; wave w owns component
// row i = w % 6 (components 6i .. 6i+5) for input-channel half w / 6: acc[6] of 32x32 f32 (96
// registers, v_mfma_f32_32x32x2_f32).  K = tiles, in K-tiles of 8 x 16 output pixels (2 x 4 Winograd
// tiles, 4 MFMA steps of 2 tiles: k = lane >> 5); the next K-tile's dz image (128 px x 32 co) and x
// halo image (10 x 18 px x 64 ci) arrive by LDS-DMA during the current one's MFMAs (two 61 KB
// stages).  Row i of A dY A^T needs dY rows {0} / {0..3} / {3} and row i of B^T X B patch rows
// {0,2,4} / {1..4} / {1,3,5}: a step reads 22-40 values (b32, the lanes of a half read one pixel's
// consecutive channels: conflict-free) and spends ~60 VALU on 6 MFMAs.  Split-K over blocks into
// slabs ws[split][36][Cout][Cin], summed in a fixed order by the reduce (deterministic).
#include <stdlib.h>
#include <string.h>
#include "pmu_common.h"

// Measured equal to F(2x2) over the c2 shapes (10.29 vs 10.29 ms, LDS-read bound) and off
// in the engine: experiments build only (include/pmunet_hip_experiments.h).
#ifdef PMU_EXPERIMENTS
namespace {

constexpr int NT = 768;
constexpr int WCO = 32, WCI = 64;
constexpr int TH = 8, TW = 16;
constexpr int HH = TH + 2, HWD = TW + 2;
constexpr int DLS = WCO, XLS = WCI;
constexpr int D_FLOATS = TH * TW * DLS;
constexpr int X_FLOATS = HH * HWD * XLS;
constexpr int SLOT = D_FLOATS + X_FLOATS;
constexpr int D_UPX = DLS / 4, X_UPX = XLS / 4;
constexpr int D_UNITS = TH * TW * D_UPX;
constexpr int W_UNITS = D_UNITS + HH * HWD * X_UPX;
constexpr int W_NGL = (W_UNITS + NT - 1) / NT;
constexpr int NCOMP = 36;
static_assert(2 * SLOT * 4 <= 160 * 1024, "two stages fit the LDS");

struct Wg4Args {
  const float* dz;  // [N][H][W][Cout]
  const float* x;   // [N][H][W][Cin]
  float* ws;        // [nsplit][36][Cout][Cin]
  int N, H, W, Cout, Cin, tiles_w, tiles_h, ntiles, nsplit, nco;
};

__device__ __forceinline__ void wg4_dma(const Wg4Args& a, int tile, int co0, int ci0, int tid, float* slot) {
  int t = tile;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t, h0 = th * TH, w0 = tw * TW;
  PMU_DCHECK(n < a.N, PMU_DBG_GRID);
  const int wbase = (tid >> 6) * 256;
#pragma unroll 1
  for (int r = 0; r < W_NGL; ++r) {  // (not unrolled: six rounds' 64-bit addresses beside 96 accumulators spill)
    const int u = r * NT + tid;
    const bool isd = u < D_UNITS;
    const int pd = u / D_UPX, qd = u - pd * D_UPX;
    const int v = u - D_UNITS;
    const int px = v / X_UPX, qx = v - px * X_UPX;
    const int hr = px / HWD, hc = px - hr * HWD;
    const int h = isd ? h0 + pd / TW : h0 - 1 + hr;
    const int w = isd ? w0 + pd % TW : w0 - 1 + hc;
    const bool data = u < W_UNITS;
    const bool in = data && h >= 0 && w >= 0 && h < a.H && w < a.W;
    const long long pix = ((long long)n * a.H + h) * a.W + w;
    PMU_DCHECK(!in || pix < (long long)a.N * a.H * a.W, PMU_DBG_OPERAND);
    const float* src = isd ? a.dz + pix * a.Cout + co0 + 4 * qd : a.x + pix * a.Cin + ci0 + 4 * qx;
    if (in)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(slot + 4 * r * NT + wbase), 16, 0, 0);
    else if (data)
      *reinterpret_cast<float4*>(slot + 4 * u) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int OFF>
__device__ __forceinline__ float lds_b32(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(p);
}

// rows of dY (A row i) and of the x patch (B^T row i) a component row needs
template <int ROW> struct RowSet;
template <> struct RowSet<0> { static constexpr int nd = 1, d0 = 0, nx = 3, x[4] = {0, 2, 4, 0}; };
template <> struct RowSet<1> { static constexpr int nd = 4, nx = 4, x[4] = {1, 2, 3, 4}; };
template <> struct RowSet<2> { static constexpr int nd = 4, nx = 4, x[4] = {1, 2, 3, 4}; };
template <> struct RowSet<3> { static constexpr int nd = 4, nx = 4, x[4] = {1, 2, 3, 4}; };
template <> struct RowSet<4> { static constexpr int nd = 4, nx = 4, x[4] = {1, 2, 3, 4}; };
template <> struct RowSet<5> { static constexpr int nd = 1, d0 = 3, nx = 3, x[4] = {1, 3, 5, 0}; };

struct Ops {
  float d[4][4];  // dY rows (tile, co): [row slot][col]
  float x[4][6];  // patch rows (tile, ci): [row slot][col]
};

// step s: tiles t = 2s + k (k = lane >> 5): tile row ty = s >> 1, tile column 2 (s & 1) + k; the
// lane's base addresses already hold the k and channel offsets
template <int ROW, int S>
__device__ __forceinline__ void wg4_read_d(unsigned dbase, Ops& o) {
  using R = RowSet<ROW>;
  constexpr int ty = S >> 1, tx0 = 2 * (S & 1);
  constexpr int doff = (4 * ty * TW + 4 * tx0) * DLS;
  if constexpr (R::nd == 1) {
    constexpr int r = R::d0;
    o.d[0][0] = lds_b32<4 * (doff + (r * TW + 0) * DLS)>(dbase);
    o.d[0][1] = lds_b32<4 * (doff + (r * TW + 1) * DLS)>(dbase);
    o.d[0][2] = lds_b32<4 * (doff + (r * TW + 2) * DLS)>(dbase);
    o.d[0][3] = lds_b32<4 * (doff + (r * TW + 3) * DLS)>(dbase);
  } else {
#define PMU_RDD(R_, C_) o.d[R_][C_] = lds_b32<4 * (doff + ((R_) * TW + (C_)) * DLS)>(dbase);
    PMU_RDD(0, 0) PMU_RDD(0, 1) PMU_RDD(0, 2) PMU_RDD(0, 3) PMU_RDD(1, 0) PMU_RDD(1, 1) PMU_RDD(1, 2) PMU_RDD(1, 3)
    PMU_RDD(2, 0) PMU_RDD(2, 1) PMU_RDD(2, 2) PMU_RDD(2, 3) PMU_RDD(3, 0) PMU_RDD(3, 1) PMU_RDD(3, 2) PMU_RDD(3, 3)
#undef PMU_RDD
  }
}
template <int ROW, int S>
__device__ __forceinline__ void wg4_read_x(unsigned xbase, Ops& o) {
  using R = RowSet<ROW>;
  constexpr int ty = S >> 1, tx0 = 2 * (S & 1);
  constexpr int xoff = (4 * ty * HWD + 4 * tx0) * XLS;
#define PMU_RDX(I_, C_) o.x[I_][C_] = lds_b32<4 * (D_FLOATS + xoff + (R::x[I_] * HWD + (C_)) * XLS)>(xbase);
#define PMU_RDXROW(I_) PMU_RDX(I_, 0) PMU_RDX(I_, 1) PMU_RDX(I_, 2) PMU_RDX(I_, 3) PMU_RDX(I_, 4) PMU_RDX(I_, 5)
  PMU_RDXROW(0) PMU_RDXROW(1) PMU_RDXROW(2)
  if constexpr (R::nx == 4) { PMU_RDXROW(3) }
#undef PMU_RDXROW
#undef PMU_RDX
}

// z = row ROW of A dY A^T (6 values), v = row ROW of B^T X B (6 values)
template <int ROW>
__device__ __forceinline__ void wg4_xform_z(const Ops& o, float (&z)[6]) {
  float r[4];
  if constexpr (ROW == 0 || ROW == 5) {
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = o.d[0][c];
  } else {
    // A row: (1, a1, a2, a3)
    constexpr float a1 = ROW == 1 ? 1.f : ROW == 2 ? -1.f : ROW == 3 ? 2.f : -2.f;
    constexpr float a2 = ROW <= 2 ? 1.f : 4.f;
    constexpr float a3 = ROW == 1 ? 1.f : ROW == 2 ? -1.f : ROW == 3 ? 8.f : -8.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) r[c] = fmaf(a3, o.d[3][c], fmaf(a2, o.d[2][c], fmaf(a1, o.d[1][c], o.d[0][c])));
  }
  {
    const float e = r[0] + r[2], od = r[1] + r[3];
    const float e4 = fmaf(4.f, r[2], r[0]), o8 = fmaf(8.f, r[3], 2.f * r[1]);
    z[0] = r[0];
    z[1] = e + od;
    z[2] = e - od;
    z[3] = e4 + o8;
    z[4] = e4 - o8;
    z[5] = r[3];
  }
}
template <int ROW>
__device__ __forceinline__ void wg4_xform_v(const Ops& o, float (&v)[6]) {
  // q = B^T row ROW applied to the patch rows (6 columns)
  float q[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    if constexpr (ROW == 0) q[c] = fmaf(4.f, o.x[0][c], fmaf(-5.f, o.x[1][c], o.x[2][c]));           // 4x0 - 5x2 + x4
    else if constexpr (ROW == 1) q[c] = fmaf(-4.f, o.x[0][c] + o.x[1][c], o.x[2][c] + o.x[3][c]);    // -4x1 - 4x2 + x3 + x4
    else if constexpr (ROW == 2) q[c] = fmaf(4.f, o.x[0][c] - o.x[1][c], o.x[3][c] - o.x[2][c]);     // 4x1 - 4x2 - x3 + x4
    else if constexpr (ROW == 3) q[c] = fmaf(2.f, o.x[2][c] - o.x[0][c], o.x[3][c] - o.x[1][c]);     // -2x1 - x2 + 2x3 + x4
    else if constexpr (ROW == 4) q[c] = fmaf(2.f, o.x[0][c] - o.x[2][c], o.x[3][c] - o.x[1][c]);     // 2x1 - x2 - 2x3 + x4
    else q[c] = fmaf(4.f, o.x[0][c], fmaf(-5.f, o.x[1][c], o.x[2][c]));                               // 4x1 - 5x3 + x5
  }
  // v[j] = sum_c q[c] B^T[j][c]
  v[0] = fmaf(4.f, q[0], fmaf(-5.f, q[2], q[4]));
  v[1] = fmaf(-4.f, q[1] + q[2], q[3] + q[4]);
  v[2] = fmaf(4.f, q[1] - q[2], q[4] - q[3]);
  v[3] = fmaf(2.f, q[3] - q[1], q[4] - q[2]);
  v[4] = fmaf(2.f, q[1] - q[3], q[4] - q[2]);
  v[5] = fmaf(4.f, q[1], fmaf(-5.f, q[3], q[5]));
}

template <int ROW>
__device__ __forceinline__ void wg4_main(const Wg4Args& a, int co0, int ci0, int half, int split, int t_beg,
                                         int t_end, float* smem) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int k = lane >> 5;
  f32x16 acc[6];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  // lane bases: tile column k of the step's tile pair, channel lane & 31 (dz) / 32 half + lane & 31 (x)
  const int doffl = (4 * k) * DLS + (lane & 31);
  const int xoffl = (4 * k) * XLS + 32 * half + (lane & 31);

  if (t_beg < t_end) wg4_dma(a, t_beg, co0, ci0, tid, smem);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  for (int tile = t_beg; tile < t_end; ++tile) {
    const int cur = (tile - t_beg) & 1;
    if (tile + 1 < t_end) wg4_dma(a, tile + 1, co0, ci0, tid, smem + (cur ^ 1) * SLOT);
    const float* slot = smem + cur * SLOT;
    const unsigned dbase = lds_addr(slot + doffl), xbase = lds_addr(slot + xoffl);
    Ops o;
    float z[6], v[6];
    // a step's reads, then its transforms and MFMAs (no read-ahead: the 40 operand registers of a
    // second step do not fit beside 96 accumulators at 3 waves per SIMD; the SIMD's other two
    // waves cover this one's LDS latency)
#define PMU_W4G_STEP(S_)                                                                   \
    wg4_read_d<ROW, S_>(dbase, o);                                                         \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    wg4_read_x<ROW, S_>(xbase, o);                                                         \
    wg4_xform_z<ROW>(o, z);                                                                \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    wg4_xform_v<ROW>(o, v);                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    _Pragma("unroll") for (int j = 0; j < 6; ++j) acc[j] = mfma_f32_32x32x2(z[j], v[j], acc[j]); \
    __builtin_amdgcn_sched_barrier(0);
    PMU_W4G_STEP(0)
    PMU_W4G_STEP(1)
    PMU_W4G_STEP(2)
    PMU_W4G_STEP(3)
#undef PMU_W4G_STEP
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // slab: ws[split][6 ROW + j][co][ci], D row = co (acc_row), col = ci (lane & 31)
  const int ci = ci0 + 32 * half + (lane & 31);
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + acc_row(r, lane);
      PMU_DCHECK(split < a.nsplit && co < a.Cout && ci < a.Cin, PMU_DBG_WORKSPACE);
      a.ws[(((long long)split * NCOMP + 6 * ROW + j) * a.Cout + co) * a.Cin + ci] = acc[j][r];
    }
}

__global__ __launch_bounds__(NT, 1) void wgrad3x3_wino4_kernel(Wg4Args a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * SLOT];
  const int wave = threadIdx.x >> 6;
  const int row = wave % 6, half = wave / 6;
  const int lb = pmu_xcd_block(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int nmn = gridDim.x;
  const int mn = lb % nmn, split = lb / nmn;
  const int co0 = (mn % a.nco) * WCO, ci0 = (mn / a.nco) * WCI;
  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);
  switch (row) {  // wave-uniform: one specialised body per component row
    case 0: wg4_main<0>(a, co0, ci0, half, split, t_beg, t_end, smem); break;
    case 1: wg4_main<1>(a, co0, ci0, half, split, t_beg, t_end, smem); break;
    case 2: wg4_main<2>(a, co0, ci0, half, split, t_beg, t_end, smem); break;
    case 3: wg4_main<3>(a, co0, ci0, half, split, t_beg, t_end, smem); break;
    case 4: wg4_main<4>(a, co0, ci0, half, split, t_beg, t_end, smem); break;
    default: wg4_main<5>(a, co0, ci0, half, split, t_beg, t_end, smem); break;
  }
}

// dw[co][ci][3][3] = G^T (sum over splits of M) G in fp64.  Block = 16 consecutive (co, ci) elements
// x 36 components (576 threads): thread (comp, e) sums its slab column over the splits (4 interleaved
// partial sums combined in a fixed order: deterministic); 16 threads apply the output transform.
__global__ __launch_bounds__(576) void wgrad_wino4_reduce_kernel(const float* __restrict__ ws, int nsplit,
                                                                 long long CC, float* __restrict__ dw) {
  __shared__ float mm[NCOMP][17];
  const int c = threadIdx.x >> 4, el = threadIdx.x & 15;
  const long long e = (long long)blockIdx.x * 16 + el;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (e < CC) {
    const float* p = ws + (long long)c * CC + e;
    const long long st = (long long)NCOMP * CC;
    int sp = 0;
    for (; sp + 3 < nsplit; sp += 4) {
      s0 += p[(long long)sp * st];
      s1 += p[(long long)(sp + 1) * st];
      s2 += p[(long long)(sp + 2) * st];
      s3 += p[(long long)(sp + 3) * st];
    }
    for (; sp < nsplit; ++sp) s0 += p[(long long)sp * st];
  }
  mm[c][el] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (threadIdx.x >= 16 || e >= CC) return;
  const double G[6][3] = {{0.25, 0., 0.},
                          {-1. / 6, -1. / 6, -1. / 6},
                          {-1. / 6, 1. / 6, -1. / 6},
                          {1. / 24, 1. / 12, 1. / 6},
                          {1. / 24, -1. / 12, 1. / 6},
                          {0., 0., 1.}};
  double t[3][6];  // G^T M
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double s = 0.;
#pragma unroll
      for (int r = 0; r < 6; ++r) s += G[r][i] * (double)mm[6 * r + j][el];
      t[i][j] = s;
    }
  float* o = dw + e * 9;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      double s = 0.;
#pragma unroll
      for (int j = 0; j < 6; ++j) s += t[i][j] * G[j][b];
      o[3 * i + b] = (float)s;
    }
}

void wg4_geometry(int N, int H, int W, int Cout, int Cin, Wg4Args& a) {
  a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.Cin = Cin;
  a.tiles_w = pmu_cdiv(W, TW);
  a.tiles_h = pmu_cdiv(H, TH);
  a.ntiles = N * a.tiles_w * a.tiles_h;
  a.nco = Cout / WCO;
  const int blocks_mn = a.nco * (Cin / WCI);
  static const int target_env = [] {  // PMU_WG4_BLOCKS: workgroups the split-K aims for
    const char* e = getenv("PMU_WG4_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  const int target = target_env > 0 ? target_env : 256;  // one 768-thread workgroup per CU
  int s = target / blocks_mn;
  if (s < 1) s = 1;
  if (s > a.ntiles) s = a.ntiles;
  a.nsplit = s;
}

}  // namespace

extern "C" size_t pmu_conv3x3_wgrad_ws_wino4(int N, int H, int W, int Cin, int Cout) {
  if (N <= 0 || H <= 0 || W <= 0 || Cout <= 0 || Cin <= 0 || Cout % WCO != 0 || Cin % WCI != 0) return 0;
  Wg4Args a;
  wg4_geometry(N, H, W, Cout, Cin, a);
  return (size_t)a.nsplit * NCOMP * Cout * Cin * sizeof(float);
}

extern "C" int pmu_conv3x3_wgrad_wino4(const float* dzt, const float* xt, int N, int H, int W, int Cout, int Cin,
                                       float* dw, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(dzt && xt && dw && ws && N > 0 && H > 0 && W > 0);
  PMU_REQUIRE(Cout % WCO == 0 && Cin % WCI == 0);
  Wg4Args a;
  a.dz = dzt; a.x = xt; a.ws = ws;
  wg4_geometry(N, H, W, Cout, Cin, a);
  PMU_REQUIRE(ws_bytes >= (size_t)a.nsplit * NCOMP * Cout * Cin * sizeof(float));
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(a.nco * (Cin / WCI)), (unsigned)a.nsplit);
  hipLaunchKernelGGL(wgrad3x3_wino4_kernel, grid, dim3(NT), 0, st, a);
  PMU_CHECK_LAUNCH();
  const long long CC = (long long)Cout * Cin;
  hipLaunchKernelGGL(wgrad_wino4_reduce_kernel, dim3((unsigned)((CC + 15) / 16)), dim3(576), 0, st, (const float*)ws,
                     a.nsplit, CC, dw);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
#endif  // PMU_EXPERIMENTS
