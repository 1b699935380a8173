// Weight gradient of the 3x3 / pad 1 convolution in fp32 by Winograd F(2x2, 3x3) (the autograd of
// nn.Conv2d w.r.t. its weight, PMU/model/unet/unet_parts.py:15,18), on the materialised operands the
// forward and input-gradient kernels tee (xt = the conv's input operand, dzt = dL/dz; both NHWC fp32).
//
// For a 2x2 output tile with gradient block dY (per output channel) and 4x4 input patch X (per input
// channel), the forward is Y = A^T [(G g G^T) .* (B^T X B)] A, so
//     dL/dg = G^T [ (A dY A^T) .* (B^T X B) ] G     (summed over tiles)
// i.e. 16 per-component GEMMs over the tiles, M[c][co][ci] = sum_t Z[c][t][co] V[c][t][ci] with
// Z = A dY A^T, V = B^T X B, followed by the 3x4x4x3 output transform G^T M G — 16 products per tile
// and channel pair where the direct sum takes 36.  fp32 throughout; the result differs from the
// direct sum by fp32 rounding only.
//
// Block: 512 threads, 32 output x 64 input channels, all 16 components; wave w owns the 16 x 16
// (co, ci) fragment (w & 1, w >> 1) for every component (acc[16] of v_mfma_f32_16x16x4_f32, 64
// registers).  K = tiles, in K-tiles of 128 output pixels (8 x 16 = 32 Winograd tiles, 8 MFMA steps);
// the next K-tile's dzt / xt images are fetched by LDS-DMA (global_load_lds) during the current
// one's MFMAs (double-buffered LDS, 145 KB).  Split-K over blocks: each writes M for its tile range to a slab, and the
// reduce kernel sums the slabs in a fixed order (deterministic) and applies G^T M G.
#include <stdlib.h>
#include <string.h>
#include "pmu_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;
constexpr int WCO = 32, WCI = 64;        // channels per block
constexpr int TH = 8, TW = 16;           // output pixels per K-tile
constexpr int NSTEP = (TH / 2) * (TW / 2) / 4;  // MFMA steps (4 Winograd tiles each) per K-tile
constexpr int HH = TH + 2, HWD = TW + 2; // 10 x 18 operand halo
// LDS floats per dz / x pixel: unpadded — the row-split kernel's 32-lane read groups all read one
// pixel's consecutive channels (conflict-free at any pitch), and the DMA then moves no pad units.
// (The 16x16x4 kernel's groups span two tiles and bank 2-way at this pitch; it is the fallback.)
constexpr int DLS = WCO;
constexpr int XLS = WCI;
constexpr int D_FLOATS = TH * TW * DLS;
constexpr int X_FLOATS = HH * HWD * XLS;
constexpr int SLOT = D_FLOATS + X_FLOATS;

struct WgwArgs {
  const float* dz;  // [N][H][W][Cout]
  const float* x;   // [N][H][W][Cin]
  float* ws;        // [nsplit][16][Cout][Cin]
  int N, H, W, Cout, Cin, tiles_w, tiles_h, ntiles, nsplit, nco;
  int prio;         // 1: waves 4-7 run at s_setprio 1 (PMU_WINO_PRIO)
};

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void wgw_origin(const WgwArgs& a, int tile, int& n, int& h0, int& w0) {
  int t = tile;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  n = t; h0 = th * TH; w0 = tw * TW;
  PMU_DCHECK(n < a.N, PMU_DBG_GRID);
}

// LDS-DMA staging of one K-tile: the slot is the dz image (128 px x 8 units) followed by the
// x halo image (180 px x 16 units); each global_load_lds wave-instruction fills 64 consecutive
// units, its lanes' global sources chosen per unit.  Units outside the input are zeroed with a
// ds_write instead (their DMA lanes masked); pad units are not written.
constexpr int D_UPX = DLS / 4, X_UPX = XLS / 4;
constexpr int D_UNITS = TH * TW * D_UPX;
constexpr int W_UNITS = D_UNITS + HH * HWD * X_UPX;
[[maybe_unused]] constexpr int W_NGL = (W_UNITS + NT - 1) / NT;
static_assert(D_UNITS * 4 == D_FLOATS && W_UNITS * 4 == SLOT, "slot = dz image + x image");

// block geometry by output-channel width: 32 (512 threads) or 64 (1024 threads: 4 waves per SIMD,
// the x halo image shared by twice the output channels; PMU_WGW64)
template <int WCO_>
struct WgwCfg {
  static constexpr int WCO = WCO_, NT = 16 * WCO_, DLS = WCO_;
  static constexpr int D_FLOATS = TH * TW * DLS;
  static constexpr int SLOT = D_FLOATS + X_FLOATS;
  static constexpr int D_UPX = DLS / 4;
  static constexpr int D_UNITS = TH * TW * D_UPX;
  static constexpr int W_UNITS = D_UNITS + HH * HWD * X_UPX;
  static constexpr int W_NGL = (W_UNITS + NT - 1) / NT;
};

template <int WCO_ = 32>
__device__ __forceinline__ void wgw_dma(const WgwArgs& a, int tile, int co0, int ci0, int tid, float* slot) {
  using C = WgwCfg<WCO_>;
  int n, h0, w0;
  wgw_origin(a, tile, n, h0, w0);
  const int wbase = (tid >> 6) * 256;
#pragma unroll
  for (int r = 0; r < C::W_NGL; ++r) {
    const int u = r * C::NT + tid;
    // dz image unit (u < D_UNITS) or x halo unit, branch-free
    const bool isd = u < C::D_UNITS;
    const int pd = u / C::D_UPX, qd = u - pd * C::D_UPX;
    const int v = u - C::D_UNITS;
    const int px = v / X_UPX, qx = v - px * X_UPX;
    const int hr = px / HWD, hc = px - hr * HWD;
    const int h = isd ? h0 + (pd >> 4) : h0 - 1 + hr;
    const int w = isd ? w0 + (pd & 15) : w0 - 1 + hc;
    const bool data = isd ? qd < C::WCO / 4 : (u < C::W_UNITS && qx < WCI / 4);
    const bool in = data && h >= 0 && w >= 0 && h < a.H && w < a.W;
    const long long pix = ((long long)n * a.H + h) * a.W + w;
    PMU_DCHECK(!in || pix < (long long)a.N * a.H * a.W, PMU_DBG_OPERAND);
    const float* src = isd ? a.dz + pix * a.Cout + co0 + 4 * qd : a.x + pix * a.Cin + ci0 + 4 * qx;
    if (in)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(slot + 4 * r * C::NT + wbase), 16, 0, 0);
    else if (data)
      *reinterpret_cast<float4*>(slot + 4 * u) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// operand values of one MFMA step: tiles 4s..4s+3 (k = lane >> 4), this lane's co (dz 2x2) and ci (x 4x4)
struct WgwOps {
  float d[4];
  float x[16];
};
__device__ __forceinline__ void wgw_read(const float* slot, int s, int lane, int cf, int pf, WgwOps& o) {
  const int t = 4 * s + (lane >> 4);
  const int ty = t >> 3, tx = t & 7;
  const float* dp = slot + ((2 * ty) * TW + 2 * tx) * DLS + cf * 16 + (lane & 15);
  const float* xp = slot + D_FLOATS + ((2 * ty) * HWD + 2 * tx) * XLS + pf * 16 + (lane & 15);
  o.d[0] = dp[0]; o.d[1] = dp[DLS]; o.d[2] = dp[TW * DLS]; o.d[3] = dp[(TW + 1) * DLS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) o.x[4 * i + j] = xp[(i * HWD + j) * XLS];
}

template <bool NOXF = false>
__device__ __forceinline__ void wgw_mfmas(const WgwOps& o, f32x4 (&acc)[16]) {
  // Z = A dY A^T, A = [1 0; 1 1; 1 -1; 0 -1]
  const float d00 = o.d[0], d01 = o.d[1], d10 = o.d[2], d11 = o.d[3];
  float r[4][2];  // A dY
  r[0][0] = d00; r[0][1] = d01;
  r[1][0] = d00 + d10; r[1][1] = d01 + d11;
  r[2][0] = d00 - d10; r[2][1] = d01 - d11;
  r[3][0] = -d10; r[3][1] = -d11;
  float z[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    z[4 * i + 0] = r[i][0];
    z[4 * i + 1] = r[i][0] + r[i][1];
    z[4 * i + 2] = r[i][0] - r[i][1];
    z[4 * i + 3] = -r[i][1];
  }
  // V = B^T X B, B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
  float tt[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    tt[0][j] = o.x[j] - o.x[8 + j];
    tt[1][j] = o.x[4 + j] + o.x[8 + j];
    tt[2][j] = o.x[8 + j] - o.x[4 + j];
    tt[3][j] = o.x[4 + j] - o.x[12 + j];
  }
  float v[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[4 * i + 0] = tt[i][0] - tt[i][2];
    v[4 * i + 1] = tt[i][1] + tt[i][2];
    v[4 * i + 2] = tt[i][2] - tt[i][1];
    v[4 * i + 3] = tt[i][1] - tt[i][3];
  }
  if (NOXF) {  // timing experiment only: operands untransformed
#pragma unroll
    for (int c = 0; c < 16; ++c) { z[c] = o.x[c]; v[c] = o.x[c]; }
  }
  __builtin_amdgcn_sched_barrier(0);  // all components first: the MFMAs then issue back to back
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = mfma16(z[c], v[c], acc[c]);
}

// EXP (timing experiments, PMU_WINO_EXP): 1 = no restaging (every K-tile reuses the first),
// 3 = no operand transforms; results are wrong for EXP != 0
template <int EXP = 0>
__global__ __launch_bounds__(NT, 1) void wgrad3x3_wino_kernel(WgwArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cf = wave & 1, pf = wave >> 1;
  // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs; remap so each XCD runs a
  // contiguous range of logical blocks — the (co, ci) blocks of one split share its K-tiles in L2
  const int nmn = gridDim.x, nb = nmn * gridDim.y, id = blockIdx.y * nmn + blockIdx.x;
  const int xc = id & 7, q8 = nb >> 3, r8 = nb & 7;
  const int lb = xc * q8 + (xc < r8 ? xc : r8) + (id >> 3);
  const int mn = lb % nmn, split = lb / nmn;
  const int co0 = (mn % a.nco) * WCO, ci0 = (mn / a.nco) * WCI;
  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);

  f32x4 acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (t_beg < t_end) wgw_dma(a, t_beg, co0, ci0, tid, smem);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  for (int tile = t_beg; tile < t_end; ++tile) {
    const int cur = (tile - t_beg) & 1;
    const bool more = tile + 1 < t_end;
    if (more && EXP != 1) wgw_dma(a, tile + 1, co0, ci0, tid, smem + (cur ^ 1) * SLOT);  // lands during the MFMAs
    const float* slot = smem + (EXP == 1 ? 0 : cur * SLOT);
    // each step's LDS reads are issued before the previous step's MFMAs
    WgwOps ops[2];
    wgw_read(slot, 0, lane, cf, pf, ops[0]);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < NSTEP) wgw_read(slot, s + 1, lane, cf, pf, ops[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      wgw_mfmas<EXP == 3>(ops[s & 1], acc);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // slab: ws[split][c][co][ci], D row = co (4*(lane>>4) + r), col = ci (lane & 15)
  const int ci = ci0 + pf * 16 + (lane & 15);
#pragma unroll
  for (int c = 0; c < 16; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + cf * 16 + 4 * (lane >> 4) + r;
      PMU_DCHECK(split < a.nsplit && co < a.Cout && ci < a.Cin, PMU_DBG_WORKSPACE);
      a.ws[(((long long)split * 16 + c) * a.Cout + co) * a.Cin + ci] = acc[c][r];
    }
}

// ---------------------------------------------------------------------------------------------
// Row-split variant on v_mfma_f32_32x32x2_f32 (the default): wave w owns component row i = w & 3
// (components 4i..4i+3) for 32 output x 32 input channels (half w >> 2 of the block's 64), acc[4] of
// 32x32 (64 registers).  A step covers 2 Winograd tiles (k = lane >> 5).  Row i of B^T X B needs
// only 2 of the 4 patch rows (tt = x[ra] + s x[rb]) and row i of A dY A^T one combination of the
// dz rows, so a step costs 12 LDS reads and ~15 VALU for 4 MFMAs of 64 cycles — half the transform
// work per MFMA cycle of the 16x16x4 layout above.
// ---------------------------------------------------------------------------------------------
constexpr int NSTEP2 = (TH / 2) * (TW / 2) / 2;  // 2 tiles per step


template <int OFF>
__device__ __forceinline__ float lds_b32(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(p);
}

struct WgwOps2 {
  float d[4];   // dz 2x2 of (tile, co)
  float xa[4];  // patch row ra of (tile, ci)
  float xb[4];  // patch row rb
};

template <int EXP = 0, int WCO_ = 32>
__global__ __launch_bounds__(16 * WCO_, 1) void wgrad3x3_wino32_kernel(WgwArgs a) {
  using C = WgwCfg<WCO_>;
  __shared__ __attribute__((aligned(16))) float smem[2 * C::SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = wave & 3, half = (wave >> 2) & 1, cg = wave >> 3;  // cg: 32-channel group of WCO_ = 64
  // B^T row `row` = x[ra] + sx * x[rb]; A row `row` of dY: alpha * d0 + beta * d1
  const int ra = row == 0 ? 0 : row == 2 ? 2 : 1;
  const int rb = row == 0 ? 2 : row == 1 ? 2 : row == 2 ? 1 : 3;
  const float sx = row == 1 ? 1.f : -1.f;
  const float alpha = row == 3 ? 0.f : 1.f;
  const float beta = row == 0 ? 0.f : row == 1 ? 1.f : -1.f;
  const int nmn = gridDim.x, nb = nmn * gridDim.y, id = blockIdx.y * nmn + blockIdx.x;
  const int xc = id & 7, q8 = nb >> 3, r8 = nb & 7;
  const int lb = xc * q8 + (xc < r8 ? xc : r8) + (id >> 3);
  const int mn = lb % nmn, split = lb / nmn;
  const int co0 = (mn % a.nco) * C::WCO, ci0 = (mn / a.nco) * WCI;
  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);

  f32x16 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  if (a.prio && half) __builtin_amdgcn_s_setprio(1);  // the younger half wins VALU arbitration

  // Operand reads as explicit ds_read_b32 (asm): the compiler's own waits put an lgkmcnt(0)
  // right after each step's read-ahead (its counter bookkeeping gave up), exposing the LDS latency
  // every step.  Here a step waits for its operands — read one step earlier — before issuing the
  // next step's reads, as the forward kernel does.  Per lane: three base addresses per K-tile, a
  // compile-time offset per step and value.  Step s covers tiles t = 2s + h (h = lane >> 5):
  // ty = s >> 2, tx = 2 (s & 3) + h.
  const int hl = lane >> 5;
  const int db = (rb - ra) * HWD * XLS;
  unsigned dbase = 0, xabase = 0, xbbase = 0;
  auto set_bases = [&](const float* slot) {
    dbase = lds_addr(slot + (2 * hl) * C::DLS + 32 * cg + (lane & 31));
    xabase = lds_addr(slot + C::D_FLOATS + ra * HWD * XLS + (2 * hl) * XLS + 32 * half + (lane & 31));
    xbbase = xabase + 4u * (unsigned)db;
  };
  auto read = [&](int s, WgwOps2& o) {
    const unsigned dstep = 4u * (unsigned)((2 * (s >> 2) * TW + 4 * (s & 3)) * C::DLS);
    const unsigned xstep = 4u * (unsigned)((2 * (s >> 2) * HWD + 4 * (s & 3)) * XLS);
    const unsigned da = dbase + dstep, xa = xabase + xstep, xb = xbbase + xstep;
    o.d[0] = lds_b32<0>(da);
    o.d[1] = lds_b32<4 * C::DLS>(da);
    o.d[2] = lds_b32<4 * TW * C::DLS>(da);
    o.d[3] = lds_b32<4 * (TW + 1) * C::DLS>(da);
    o.xa[0] = lds_b32<0>(xa);
    o.xa[1] = lds_b32<4 * XLS>(xa);
    o.xa[2] = lds_b32<8 * XLS>(xa);
    o.xa[3] = lds_b32<12 * XLS>(xa);
    o.xb[0] = lds_b32<0>(xb);
    o.xb[1] = lds_b32<4 * XLS>(xb);
    o.xb[2] = lds_b32<8 * XLS>(xb);
    o.xb[3] = lds_b32<12 * XLS>(xb);
  };
  if (t_beg < t_end) wgw_dma<WCO_>(a, t_beg, co0, ci0, tid, smem);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  for (int tile = t_beg; tile < t_end; ++tile) {
    const int cur = (tile - t_beg) & 1;
    const bool more = tile + 1 < t_end;
    if (more && EXP != 1) wgw_dma<WCO_>(a, tile + 1, co0, ci0, tid, smem + (cur ^ 1) * C::SLOT);
    set_bases(smem + (EXP == 1 ? 0 : cur * C::SLOT));
    WgwOps2 ops[2];
    read(0, ops[0]);
#pragma unroll
    for (int s = 0; s < NSTEP2; ++s) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // step s's operands (read one step ago)
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < NSTEP2) read(s + 1, ops[(s + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const WgwOps2& o = ops[s & 1];
      // Z row: r = alpha * dY[0] + beta * dY[1] (2 columns), then [r0, r0 + r1, r0 - r1, -r1]
      const float r0 = fmaf(beta, o.d[2], alpha * o.d[0]);
      const float r1 = fmaf(beta, o.d[3], alpha * o.d[1]);
      float z[4] = {r0, r0 + r1, r0 - r1, -r1};
      // V row: tt = x[ra] + sx * x[rb], then [t0 - t2, t1 + t2, t2 - t1, t1 - t3]
      float tt[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) tt[j] = fmaf(sx, o.xb[j], o.xa[j]);
      float v[4] = {tt[0] - tt[2], tt[1] + tt[2], tt[2] - tt[1], tt[1] - tt[3]};
      if (EXP == 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k) { z[k] = o.d[k]; v[k] = o.xa[k]; }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = mfma_f32_32x32x2(z[k], v[k], acc[k]);
      __builtin_amdgcn_sched_barrier(0);  // the next step's wait stays behind these MFMAs
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // slab: ws[split][4*row + k][co][ci], D row = co (acc_row), col = ci (lane & 31)
  const int ci = ci0 + 32 * half + (lane & 31);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + 32 * cg + acc_row(r, lane);
      PMU_DCHECK(split < a.nsplit && co < a.Cout && ci < a.Cin, PMU_DBG_WORKSPACE);
      a.ws[(((long long)split * 16 + 4 * row + k) * a.Cout + co) * a.Cin + ci] = acc[k][r];
    }
}

// dw[co][ci][3][3] = G^T (sum over splits of M) G, G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1].
// Block = 64 consecutive (co, ci) elements x 16 components x 4 split residues (1024 threads): thread
// (q = t >> 8, comp = (t >> 4) & 15, four elements (t & 15) * 4 ...) sums splits q, q + 4, ... of its
// float4 slab column (residue 0 also the tail past the last full group of 4), the four partial sums meet
// in LDS in the fixed order (s0 + s1) + (s2 + s3) — deterministic — and 64 threads apply the output
// transform.  (16 B per load: the 4-B loads of one thread per (element, residue) kept ~1/4 of the
// bytes in flight and left the reduction latency-bound at ~21 us whatever the layer.)
__global__ __launch_bounds__(1024) void wgrad_wino_reduce_kernel(const float* __restrict__ ws, int nsplit, int Cout,
                                                                 int Cin, float* __restrict__ dw) {
  __shared__ float red[4][16][65];
  const long long CC = (long long)Cout * Cin;  // a multiple of 64 (pmu_conv3x3_wgrad_wino)
  const int q = threadIdx.x >> 8, c = (threadIdx.x >> 4) & 15, e4 = (threadIdx.x & 15) * 4;
  const long long e = (long long)blockIdx.x * 64 + e4;
  const float* p = ws + (long long)c * CC + e;
  const long long st = 16 * CC;
  const int full = nsplit >> 2;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int k = 0; k < full; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(p + (long long)(4 * k + q) * st);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  if (q == 0)
    for (int sp = 4 * full; sp < nsplit; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(p + (long long)sp * st);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  red[q][c][e4 + 0] = s.x;
  red[q][c][e4 + 1] = s.y;
  red[q][c][e4 + 2] = s.z;
  red[q][c][e4 + 3] = s.w;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int el = threadIdx.x;
  float m[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) m[k] = (red[0][k][el] + red[1][k][el]) + (red[2][k][el] + red[3][k][el]);
  float t[3][4];  // G^T M
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float h = 0.5f * (m[4 + k] + m[8 + k]);
    t[0][k] = m[k] + h;
    t[1][k] = 0.5f * (m[4 + k] - m[8 + k]);
    t[2][k] = h + m[12 + k];
  }
  float* o = dw + ((long long)blockIdx.x * 64 + el) * 9;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float h = 0.5f * (t[i][1] + t[i][2]);
    o[3 * i + 0] = t[i][0] + h;
    o[3 * i + 1] = 0.5f * (t[i][1] - t[i][2]);
    o[3 * i + 2] = h + t[i][3];
  }
}

// 64-channel blocks when Cout allows (PMU_WGW64=0: the 32-channel, 512-thread blocks everywhere)
static bool wgw_v16() {  // PMU_WGRAD_WINO=16x16: the 16x16x4 layout (all components per wave)
  static const bool v = [] {
    const char* e = pmu_variant_env("PMU_WGRAD_WINO");
    return e && strcmp(e, "16x16") == 0;
  }();
  return v;
}
static int wgw_wco(int Cout) {
  static const bool w64 = [] {
    const char* e = pmu_variant_env("PMU_WGW64");
    return !(e && atoi(e) == 0);
  }();
  return (w64 && !wgw_v16() && Cout % 64 == 0) ? 64 : 32;
}

void wgw_geometry(int N, int H, int W, int Cout, int Cin, WgwArgs& a) {
  a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.Cin = Cin;
  a.tiles_w = pmu_cdiv(W, TW);
  a.tiles_h = pmu_cdiv(H, TH);
  a.ntiles = N * a.tiles_w * a.tiles_h;
  a.nco = Cout / wgw_wco(Cout);
  const int blocks_mn = a.nco * (Cin / WCI);
  static const int target_env = [] {  // PMU_WGW_BLOCKS: workgroups the split-K aims for (A/B)
    const char* e = getenv("PMU_WGW_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  // one wave of workgroups: 256 of the 1024-thread 64-channel blocks (one per CU; 320 / 512 / 768
  // measured 19.2 / 13.4 / 14.2 ms vs 12.9-13.0 ms per c2 step), 512 of the 512-thread ones (two per CU)
  const int target = target_env > 0 ? target_env : (wgw_wco(Cout) == 64 ? 256 : 512);
  int s = target / blocks_mn;
  if (s < 1) s = 1;
  if (s > a.ntiles) s = a.ntiles;
  a.nsplit = s;
}

}  // namespace

extern "C" size_t pmu_conv3x3_wgrad_ws_wino(int N, int H, int W, int Cin, int Cout) {
  if (Cout % WCO != 0 || Cin % WCI != 0) return 0;
  WgwArgs a;
  wgw_geometry(N, H, W, Cout, Cin, a);
  return (size_t)a.nsplit * 16 * Cout * Cin * sizeof(float);
}

static int wino_prio() {  // PMU_WINO_PRIO=0|1 (A/B of static wave priority)
  static const int v = [] {
    const char* e = pmu_variant_env("PMU_WINO_PRIO");
    return e ? atoi(e) : 0;
  }();
  return v;
}

extern "C" int pmu_conv3x3_wgrad_wino(const float* dzt, const float* xt, int N, int H, int W, int Cout, int Cin,
                                      float* dw, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(dzt && xt && dw && ws && N > 0 && H > 0 && W > 0);
  PMU_REQUIRE(Cout % WCO == 0 && Cin % WCI == 0);
  WgwArgs a;
  a.dz = dzt; a.x = xt; a.ws = ws;
  wgw_geometry(N, H, W, Cout, Cin, a);
  a.prio = wino_prio();
  PMU_REQUIRE(ws_bytes >= (size_t)a.nsplit * 16 * Cout * Cin * sizeof(float));
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)(a.nco * (Cin / WCI)), (unsigned)a.nsplit);
  const bool v16 = wgw_v16();
#ifdef PMU_EXPERIMENTS
  // timing experiments (wrong results for EXP != 0): only in `make EXPERIMENTS=1` builds
  static const int exp_ = [] {
    const char* e = pmu_variant_env("PMU_WINO_EXP");
    return e ? atoi(e) : 0;
  }();
  if (exp_ == 1 || exp_ == 3) {
    const bool w64 = wgw_wco(Cout) == 64;  // (the shipped 1024-thread layout when it applies)
    if (v16 && exp_ == 1) hipLaunchKernelGGL((wgrad3x3_wino_kernel<1>), grid, dim3(NT), 0, st, a);
    else if (v16) hipLaunchKernelGGL((wgrad3x3_wino_kernel<3>), grid, dim3(NT), 0, st, a);
    else if (exp_ == 1 && w64) hipLaunchKernelGGL((wgrad3x3_wino32_kernel<1, 64>), grid, dim3(1024), 0, st, a);
    else if (w64) hipLaunchKernelGGL((wgrad3x3_wino32_kernel<3, 64>), grid, dim3(1024), 0, st, a);
    else if (exp_ == 1) hipLaunchKernelGGL((wgrad3x3_wino32_kernel<1>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((wgrad3x3_wino32_kernel<3>), grid, dim3(NT), 0, st, a);
  } else
#endif
  if (v16)  // the 16x16x4 layout (all components per wave)
    hipLaunchKernelGGL((wgrad3x3_wino_kernel<0>), grid, dim3(NT), 0, st, a);
  else if (wgw_wco(Cout) == 64)
    hipLaunchKernelGGL((wgrad3x3_wino32_kernel<0, 64>), grid, dim3(1024), 0, st, a);
  else
    hipLaunchKernelGGL((wgrad3x3_wino32_kernel<0>), grid, dim3(NT), 0, st, a);
  PMU_CHECK_LAUNCH();
  const long long CC = (long long)Cout * Cin;  // Cout % WCO, Cin % WCI: a multiple of 64
  hipLaunchKernelGGL(wgrad_wino_reduce_kernel, dim3((unsigned)(CC / 64)), dim3(1024), 0, st, (const float*)ws,
                     a.nsplit, Cout, Cin, dw);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
