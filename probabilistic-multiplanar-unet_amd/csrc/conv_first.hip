// First layer of the U-Net / prior / posterior (Cin <= 4 input planes): conv3x3 forward with BN
// partial sums, and its weight gradient, on the VALU (K = 9*Cin is too short for MFMA tiles).
// Reference: the first DoubleConv conv of PMU/model/unet/unet_parts.py:15 and Encoder conv of
// PMU/model/probabilistic_unet/probabilistic_unet.py:38 (posterior input = cat(image, mask), :88).
#include "pmu_stage.h"

namespace {

// ---------------------------------------------------------------------------------
// First layer: Cin <= 4 input planes (NCHW-style, one pointer per channel), VALU.
// ---------------------------------------------------------------------------------
struct FirstArgs {
  const float* planes[4];
  int Cin, N, H, W, Cout;
  const float* w;
  const float* bias;
  float* z;
  float* part;
};

// Tiled forward: a block walks FT_TPB consecutive 8 x 32 output-pixel tiles of one image row band x
// all Cout.  Each tile's (8+2) x (32+2) x CIN input patch is staged in LDS (zero halo; the next tile's
// patch values are loaded into registers under the current tile's FMAs, so only a block's first
// patch load is exposed), each thread keeps its channel quad's 9*CIN weight float4 in registers, and
// per pixel reads the 9*CIN inputs from LDS (one address per pixel: broadcast over the quad lanes)
// into packed 2-wide FMAs.  BN partial sums: one row per tile (pmu_conv_first_tiles rows).
constexpr int FT_H = 8, FT_W = 32, FT_PH = FT_H + 2, FT_PW = FT_W + 2;
constexpr int FT_TPB = 4;  // tiles per forward block (one block per tile exposed each patch load: 0.35 ms at c5)

typedef float pmu_f2 __attribute__((ext_vector_type(2)));
typedef float pmu_f32x4 __attribute__((ext_vector_type(4)));

// the (8+2) x (32+2) x CIN patch values of one tile this thread stages (zero outside the image)
template <int CIN>
__device__ __forceinline__ void first_patch_load(const float* const (&planes)[4], int tile, int tiles_w, int tiles_h,
                                                 int H, int W, float (&pv)[(CIN * FT_PH * FT_PW + 255) / 256]) {
  constexpr int PE = CIN * FT_PH * FT_PW, NPE = (PE + 255) / 256;
  int t = tile;
  const int tw = t % tiles_w; t /= tiles_w;
  const int th = t % tiles_h;
  const int n = t / tiles_h;
  const int h0 = th * FT_H, w0 = tw * FT_W;
  const unsigned HW = (unsigned)H * (unsigned)W;
#pragma unroll
  for (int q = 0; q < NPE; ++q) {
    const int e = threadIdx.x + 256 * q;
    const int ci = e / (FT_PH * FT_PW), r = e - ci * (FT_PH * FT_PW);
    const int ph = r / FT_PW, pw = r - ph * FT_PW;
    const int h = h0 - 1 + ph, w = w0 - 1 + pw;
    float v = 0.f;
    if (e < PE && h >= 0 && h < H && w >= 0 && w < W) v = planes[ci][(unsigned)n * HW + (unsigned)(h * W + w)];
    pv[q] = v;
  }
}

// (three waves per SIMD fit the 9 * CIN weight pairs up to CIN = 3; CIN = 4 at that cap spilled 267 registers)
template <int CIN>
__global__ __launch_bounds__(256, CIN >= 4 ? 2 : 3) void conv_first_fwd_tile_kernel(FirstArgs a, int tiles_w, int tiles_h, int ntiles) {
  constexpr int PE = CIN * FT_PH * FT_PW, NPE = (PE + 255) / 256;
  __shared__ float patch[PE];
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x;
  const int CQ = a.Cout >> 2, npl = 256 / CQ;
  const int cq = tid % CQ, pl = tid / CQ;
  const unsigned HW = (unsigned)a.H * (unsigned)a.W;
  pmu_f2 wlo[CIN * 9], whi[CIN * 9];  // w[co = 4cq + {0,1}], w[4cq + {2,3}] per (ci, tap)
#pragma unroll
  for (int k = 0; k < CIN * 9; ++k) {
    wlo[k] = pmu_f2{a.w[(4 * cq + 0) * CIN * 9 + k], a.w[(4 * cq + 1) * CIN * 9 + k]};
    whi[k] = pmu_f2{a.w[(4 * cq + 2) * CIN * 9 + k], a.w[(4 * cq + 3) * CIN * 9 + k]};
  }
  pmu_f2 blo = {0.f, 0.f}, bhi = {0.f, 0.f};
  if (a.bias) {
    blo = pmu_f2{a.bias[4 * cq], a.bias[4 * cq + 1]};
    bhi = pmu_f2{a.bias[4 * cq + 2], a.bias[4 * cq + 3]};
  }
  const int t_beg = blockIdx.x * FT_TPB, t_end = min(ntiles, t_beg + FT_TPB);
  float pv[NPE];
  first_patch_load<CIN>(a.planes, t_beg, tiles_w, tiles_h, a.H, a.W, pv);
  for (int tile = t_beg; tile < t_end; ++tile) {
    __syncthreads();  // the previous tile's patch and partial-sum reads are done
#pragma unroll
    for (int q = 0; q < NPE; ++q)
      if (tid + 256 * q < PE) patch[tid + 256 * q] = pv[q];
    __syncthreads();
    if (tile + 1 < t_end) first_patch_load<CIN>(a.planes, tile + 1, tiles_w, tiles_h, a.H, a.W, pv);
    int t = tile;
    const int tw = t % tiles_w; t /= tiles_w;
    const int th = t % tiles_h;
    const int n = t / tiles_h;
    const int h0 = th * FT_H, w0 = tw * FT_W;
    pmu_f2 s1lo = {0.f, 0.f}, s1hi = {0.f, 0.f}, s2lo = {0.f, 0.f}, s2hi = {0.f, 0.f};
    for (int i = pl; i < FT_H * FT_W; i += npl) {
      const int r = i / FT_W, c = i - r * FT_W;
      const int h = h0 + r, w = w0 + c;
      if (h >= a.H || w >= a.W) continue;
      pmu_f2 olo = blo, ohi = bhi;
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const float x = patch[(ci * FT_PH + r + tap / 3) * FT_PW + c + tap % 3];
          const pmu_f2 x2 = {x, x};
          olo = __builtin_elementwise_fma(x2, wlo[ci * 9 + tap], olo);
          ohi = __builtin_elementwise_fma(x2, whi[ci * 9 + tap], ohi);
        }
      const unsigned p = (unsigned)n * HW + (unsigned)(h * a.W + w);
      *reinterpret_cast<float4*>(a.z + (size_t)p * a.Cout + 4 * cq) = make_float4(olo.x, olo.y, ohi.x, ohi.y);
      s1lo += olo; s1hi += ohi;
      s2lo = __builtin_elementwise_fma(olo, olo, s2lo);
      s2hi = __builtin_elementwise_fma(ohi, ohi, s2hi);
    }
    if (!a.part) continue;  // (block-uniform)
    // BN partial sums of this tile: one row per tile, in the one-tile-per-block order
    red[tid * 8 + 0] = s1lo.x; red[tid * 8 + 1] = s1lo.y; red[tid * 8 + 2] = s1hi.x; red[tid * 8 + 3] = s1hi.y;
    red[tid * 8 + 4] = s2lo.x; red[tid * 8 + 5] = s2lo.y; red[tid * 8 + 6] = s2hi.x; red[tid * 8 + 7] = s2hi.y;
    __syncthreads();
    // (one thread per (channel quad, value) instead, the same sums in the same order: 406 vs 382 us at c5)
    if (tid < CQ) {
      float t1[4] = {0, 0, 0, 0}, t2[4] = {0, 0, 0, 0};
      for (int l = 0; l < npl; ++l) {
        const int src = l * CQ + tid;
#pragma unroll
        for (int e = 0; e < 4; ++e) { t1[e] += red[src * 8 + e]; t2[e] += red[src * 8 + 4 + e]; }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a.part[((long long)tile * 2 + 0) * a.Cout + 4 * tid + e] = t1[e];
        a.part[((long long)tile * 2 + 1) * a.Cout + 4 * tid + e] = t2[e];
      }
    }
  }
}

// MFMA form of the tiled forward (Cout = 16 MT, MT = 1, 2, 4; the engine's first layers): z[px][c] =
// bias[c] + sum over k = 9 ci + tap of w[c][k] * patch[px][k], as D[c][px] on v_mfma_f32_16x16x4f32 with
// K = 9 CIN taps in steps of 4 (zero-padded).  A = w (lane (i, kk): w[16 m + i][4 s + kk], held in
// registers), B = patch (lane (j, kk): pixel j's tap 4 s + kk, from the tile's LDS patch), so each lane
// ends with 4 consecutive channels of one pixel: one 16-B z store per M tile.  A wave takes 16 pixels
// of its tile at a time (4 groups per tile); the per-tile BN partial sums are summed over a group's 16
// pixel lanes by DPP row sums, then over the 4 waves in order.  The fp32 sums of the VALU kernel come in
// another order (z equal to within its rounding); one part row per tile as before.
template <int CIN, int MT>
__global__ __launch_bounds__(256) void conv_first_fwd_mfma_kernel(FirstArgs a, int tiles_w, int tiles_h, int ntiles) {
  constexpr int K9 = CIN * 9, KS = (K9 + 3) / 4, PE = CIN * FT_PH * FT_PW, NPE = (PE + 255) / 256;
  constexpr int COUT = 16 * MT, GPT = FT_H * FT_W / 64;  // 16-pixel groups per wave and tile
  __shared__ float patch[PE];
  __shared__ float red[4 * 2 * COUT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const unsigned HW = (unsigned)a.H * (unsigned)a.W;
  float wa[MT][KS];  // A operand: w[16 m + li][4 s + lk]
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int k = 4 * st + lk;
      wa[m][st] = k < K9 ? a.w[(16 * m + li) * K9 + k] : 0.f;
    }
  int koff[KS];  // B operand: the lane's tap 4 s + lk as a patch offset (-1: padding)
#pragma unroll
  for (int st = 0; st < KS; ++st) {
    const int k = 4 * st + lk, ci = k / 9, t = k - 9 * (k / 9);
    koff[st] = k < K9 ? (ci * FT_PH + t / 3) * FT_PW + t % 3 : -1;
  }
  float4 bq[MT];  // bias of the lane's output channels 16 m + 4 lk .. + 3
#pragma unroll
  for (int m = 0; m < MT; ++m)
    bq[m] = a.bias ? *reinterpret_cast<const float4*>(a.bias + 16 * m + 4 * lk) : make_float4(0.f, 0.f, 0.f, 0.f);
  const int t_beg = blockIdx.x * FT_TPB, t_end = min(ntiles, t_beg + FT_TPB);
  float pv[NPE];
  first_patch_load<CIN>(a.planes, t_beg, tiles_w, tiles_h, a.H, a.W, pv);
  for (int tile = t_beg; tile < t_end; ++tile) {
    __syncthreads();  // the previous tile's patch and partial-sum reads are done
#pragma unroll
    for (int q = 0; q < NPE; ++q)
      if (tid + 256 * q < PE) patch[tid + 256 * q] = pv[q];
    __syncthreads();
    if (tile + 1 < t_end) first_patch_load<CIN>(a.planes, tile + 1, tiles_w, tiles_h, a.H, a.W, pv);
    int t = tile;
    const int tw = t % tiles_w; t /= tiles_w;
    const int th = t % tiles_h;
    const int n = t / tiles_h;
    const int h0 = th * FT_H, w0 = tw * FT_W;
    float s1[MT][4], s2[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) { s1[m][e] = 0.f; s2[m][e] = 0.f; }
#pragma unroll 1
    for (int gi = 0; gi < GPT; ++gi) {
      const int q0 = (wave * GPT + gi) * 16;  // the group's first pixel in the tile (16 in one tile row)
      const int r = q0 / FT_W, c = q0 - r * FT_W + li;
      float b[KS];
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        const float v = patch[(koff[st] < 0 ? 0 : koff[st]) + r * FT_PW + c];
        b[st] = koff[st] < 0 ? 0.f : v;
      }
      pmu_f32x4 acc[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        acc[m] = pmu_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < KS; ++st) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[m][st], b[st], acc[m], 0, 0, 0);
      }
      const int h = h0 + r, w = w0 + c;
      const bool ok = h < a.H && w < a.W;
      const unsigned p = (unsigned)n * HW + (unsigned)(min(h, a.H - 1) * a.W + min(w, a.W - 1));
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const float4 zv = make_float4(acc[m][0] + bq[m].x, acc[m][1] + bq[m].y, acc[m][2] + bq[m].z, acc[m][3] + bq[m].w);
        const float zz[4] = {zv.x, zv.y, zv.z, zv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = ok ? zz[e] : 0.f;
          s1[m][e] += v;
          s2[m][e] = fmaf(v, v, s2[m][e]);
        }
        if (ok) *reinterpret_cast<float4*>(a.z + (size_t)p * COUT + 16 * m + 4 * lk) = zv;
      }
    }
    if (!a.part) continue;  // (block-uniform)
    // over the 16 pixel lanes of each channel quad (a DPP row), then over the 4 waves in order
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t1 = pmu_group_sum(s1[m][e], 16), t2 = pmu_group_sum(s2[m][e], 16);
        if (li == 0) {
          red[(wave * 2 + 0) * COUT + 16 * m + 4 * lk + e] = t1;
          red[(wave * 2 + 1) * COUT + 16 * m + 4 * lk + e] = t2;
        }
      }
    __syncthreads();
    for (int o = tid; o < 2 * COUT; o += 256) {
      const int rr = o / COUT, cc = o - rr * COUT;
      float v = 0.f;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv) v += red[(wv * 2 + rr) * COUT + cc];
      a.part[((long long)tile * 2 + rr) * a.Cout + cc] = v;
    }
  }
}

struct FirstWgArgs {
  DevFrame dz;
  const float* planes[4];
  int Cin, Cout;
  float* ws;  // [blocks][Cout][Cin*9]
};

constexpr int FWPIX = 1024;  // pixels per block

// thread = (co, pixel group); accumulates Cin*9 products over its pixels
__global__ __launch_bounds__(256) void conv_first_wgrad_kernel(FirstWgArgs a) {
  __shared__ float red[256 * 36];
  const int tid = threadIdx.x;
  const int npg = 256 / a.Cout;
  const int co = tid % a.Cout, pg = tid / a.Cout;
  const DevFrame& D = a.dz;
  const int H = D.H, W = D.W;
  const long long P = (long long)D.N * H * W;
  const long long p0 = (long long)blockIdx.x * FWPIX;
  const int K9 = a.Cin * 9;
  float acc[36];
#pragma unroll
  for (int k = 0; k < 36; ++k) acc[k] = 0.f;
  for (int i = pg; i < FWPIX; i += npg) {
    const long long p = p0 + i;
    if (p >= P) break;
    const int w = (int)(p % W);
    const int h = (int)((p / W) % H);
    const int n = (int)(p / ((long long)W * H));
    const float g = frame_value(D, n, h, w, co);
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      if (ci >= a.Cin) break;
      const float* pl_ = a.planes[ci] + (long long)n * H * W;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int hh = h + tap / 3 - 1, ww = w + tap % 3 - 1;
        const float x = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? pl_[hh * W + ww] : 0.f;
        acc[ci * 9 + tap] = fmaf(g, x, acc[ci * 9 + tap]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 36; ++k) red[tid * 36 + k] = acc[k];
  __syncthreads();
  for (int o = tid; o < a.Cout * K9; o += 256) {
    const int c = o / K9, k = o - c * K9;
    float s = 0.f;
    for (int l = 0; l < npg; ++l) s += red[(l * a.Cout + c) * 36 + k];
    a.ws[(long long)blockIdx.x * a.Cout * K9 + o] = s;
  }
}

// Fast path (dz = one unpooled BN-backward source, Cout % 4 == 0, tiled): a block walks FW_TPB consecutive 8 x 32 pixel tiles (the tile order of the
// forward).  Each tile's (8+2) x (32+2) x CIN input patch goes through LDS (the next tile's patch
// values are loaded into registers under the current tile's FMAs), so the 9*CIN input reads per
// pixel are LDS broadcasts instead of the global loads of the untiled kernel; dz is formed from
// float4 loads of da and z (BN-backward coefficients of the thread's channel quad in registers).
constexpr int FW_TPB = 16;  // tiles per block

// XB: da stored as bf16 (the second conv's *_dxb input gradient)
template <int CIN, bool XB = false>
__global__ __launch_bounds__(256) void conv_first_wgrad_tile_kernel(FirstWgArgs a, int tiles_w, int tiles_h,
                                                                    int ntiles) {
  constexpr int K9 = CIN * 9, PE = CIN * FT_PH * FT_PW, NPE = (PE + 255) / 256;
  __shared__ float patch[PE];
  __shared__ float red[512 * K9];  // [slot][Cout][K9]: 4 slots x Cout <= 128, or 1 slot x Cout = 256
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DevSrc& s = a.dz.s0;
  const int Cout = a.Cout, CQ = Cout >> 2, PG = 256 / CQ;
  const int cq = tid % CQ, pg = tid / CQ;
  const int H = a.dz.H, W = a.dz.W;
  const unsigned HW = (unsigned)H * (unsigned)W;
  const int c = 4 * cq;
  const float4 sc = *reinterpret_cast<const float4*>(s.coef + c);
  const float4 sh = *reinterpret_cast<const float4*>(s.coef + Cout + c);
  const float4 mu = *reinterpret_cast<const float4*>(s.coef + 2 * Cout + c);
  const float4 kx = *reinterpret_cast<const float4*>(s.coef + 3 * Cout + c);
  const float4 kc = *reinterpret_cast<const float4*>(s.coef + 4 * Cout + c);
  pmu_f2 acc[2][K9];  // channels {4cq, 4cq+1} and {4cq+2, 4cq+3}
#pragma unroll
  for (int k = 0; k < K9; ++k) { acc[0][k] = pmu_f2{0.f, 0.f}; acc[1][k] = pmu_f2{0.f, 0.f}; }
  const int t_beg = blockIdx.x * FW_TPB, t_end = min(ntiles, t_beg + FW_TPB);
  float pv[NPE];
  auto load_patch = [&](int tile) { first_patch_load<CIN>(a.planes, tile, tiles_w, tiles_h, H, W, pv); };
  // da / z of the thread's pixels two iterations ahead (flat (tile, pixel) order, crossing tile
  // boundaries): a pixel's float4 loads were consumed right after issue, one global round trip per
  // pixel with two waves per SIMD to cover it (0.61 ms at c5 for 2.1 GB)
  const int per_tile = (FT_H * FT_W) / PG;  // PG divides 256
  const int nj = (t_end - t_beg) * per_tile;
  auto pixel_of = [&](int j, size_t& p, int& r, int& cc, bool& ok) {
    const int jj = j < nj ? j : nj - 1;
    int t = t_beg + jj / per_tile;
    const int i = pg + (jj - (jj / per_tile) * per_tile) * PG;
    r = i / FT_W;
    cc = i - r * FT_W;
    const int tw = t % tiles_w; t /= tiles_w;
    const int th = t % tiles_h;
    const int n = t / tiles_h;
    const int h = th * FT_H + r, w = tw * FT_W + cc;
    ok = j < nj && h < H && w < W;
    p = (size_t)((unsigned)n * HW + (unsigned)(min(h, H - 1) * W + min(w, W - 1)));
  };
  float4 dq[2], zq[2];
  auto issue = [&](int j, int slot) {
    size_t p; int r, cc; bool ok;
    pixel_of(j, p, r, cc, ok);
    dq[slot] = XB ? pmu_ld4(reinterpret_cast<const unsigned short*>(s.x) + p * Cout + c)
                  : *reinterpret_cast<const float4*>(s.x + p * Cout + c);
    zq[slot] = *reinterpret_cast<const float4*>(s.z + p * Cout + c);
  };
  auto consume = [&](int j, int slot) {
    size_t p; int r, cc; bool ok;
    pixel_of(j, p, r, cc, ok);
    const float4 d = dq[slot], z = zq[slot];
    pmu_f2 glo = {pmu_bnbwd1(d.x, z.x, sc.x, sh.x, mu.x, kx.x, kc.x), pmu_bnbwd1(d.y, z.y, sc.y, sh.y, mu.y, kx.y, kc.y)};
    pmu_f2 ghi = {pmu_bnbwd1(d.z, z.z, sc.z, sh.z, mu.z, kx.z, kc.z), pmu_bnbwd1(d.w, z.w, sc.w, sh.w, mu.w, kx.w, kc.w)};
    if (!ok) { glo = pmu_f2{0.f, 0.f}; ghi = pmu_f2{0.f, 0.f}; }
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const float x = patch[(ci * FT_PH + r + tap / 3) * FT_PW + cc + tap % 3];
        const pmu_f2 x2 = {x, x};
        acc[0][ci * 9 + tap] = __builtin_elementwise_fma(glo, x2, acc[0][ci * 9 + tap]);
        acc[1][ci * 9 + tap] = __builtin_elementwise_fma(ghi, x2, acc[1][ci * 9 + tap]);
      }
  };
  if (t_beg < t_end) {
    load_patch(t_beg);
    issue(0, 0);
    issue(1, 1);
  }
  for (int tile = t_beg; tile < t_end; ++tile) {
    __syncthreads();  // the previous tile's patch reads are done
#pragma unroll
    for (int q = 0; q < NPE; ++q)
      if (tid + 256 * q < PE) patch[tid + 256 * q] = pv[q];
    __syncthreads();
    if (tile + 1 < t_end) load_patch(tile + 1);  // in flight under this tile's FMAs
    const int j0 = (tile - t_beg) * per_tile;
    for (int ii = 0; ii < per_tile; ii += 2) {  // per_tile = Cout / 4 is even (first_wgrad_fast)
      const int j = j0 + ii;
      consume(j, 0);
      issue(j + 2, 0);
      consume(j + 1, 1);
      issue(j + 3, 1);
    }
  }
  // reduce over the pixel groups inside the wave (lanes with equal cq are CQ apart), then waves
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int k = 0; k < K9; ++k) {
      float v0 = acc[hf][k].x, v1 = acc[hf][k].y;
      for (int off = CQ; off < 64; off <<= 1) {
        v0 += __shfl_xor(v0, off, 64);
        v1 += __shfl_xor(v1, off, 64);
      }
      acc[hf][k] = pmu_f2{v0, v1};
    }
  const int cq_per_wave = CQ < 64 ? CQ : 64;
  const int nwr = CQ < 64 ? 4 : 1;
  __syncthreads();
  if (lane < cq_per_wave) {
    const int slot = CQ < 64 ? wave : 0;
#pragma unroll
    for (int k = 0; k < K9; ++k) {
      red[(slot * Cout + c + 0) * K9 + k] = acc[0][k].x;
      red[(slot * Cout + c + 1) * K9 + k] = acc[0][k].y;
      red[(slot * Cout + c + 2) * K9 + k] = acc[1][k].x;
      red[(slot * Cout + c + 3) * K9 + k] = acc[1][k].y;
    }
  }
  __syncthreads();
  for (int o = tid; o < Cout * K9; o += 256) {
    float v = 0.f;
    for (int wv = 0; wv < nwr; ++wv) v += red[wv * Cout * K9 + o];
    a.ws[(long long)blockIdx.x * Cout * K9 + o] = v;
  }
}

// MFMA form of the tiled weight gradient (Cout = 16 MT, MT = 1, 2, 4; the engine's first layers): per
// output channel and tap dw[c][k] = sum over pixels g[px][c] * patch[px][k], i.e. a GEMM with M = Cout,
// N = 9 CIN taps (padded to 16 NN), K = pixels, on v_mfma_f32_16x16x4f32 (fp32, as the first layer runs
// under autocast).  Lane (i, k) = (lane & 15, lane >> 4) supplies the A element g[px_k][MT i + m] of M tile
// m (so its MT channels are consecutive: one 4 MT-byte z load and one da load per pixel, 256 / 128 B per
// 16 lanes) and the B element patch[px_k][tap i + 16 nt].  A wave takes 64 of a tile's 256 pixels, four at
// a time, with the loads of the next DEPTH groups in flight; accumulators MT x NN x 4 registers instead
// of the VALU kernel's 4 x 27 per thread (at 210 VGPRs, two waves per SIMD and two pixels in flight:
// 0.54 ms for c5's 2.1 GB, latency-bound).  Same per-block rows (ws) and row sum as the VALU kernel.
template <int CIN, int MT, bool XB>
__global__ __launch_bounds__(256) void conv_first_wgrad_mfma_kernel(FirstWgArgs a, int tiles_w, int tiles_h,
                                                                    int ntiles) {
  constexpr int K9 = CIN * 9, NN = (K9 + 15) / 16, PE = CIN * FT_PH * FT_PW, NPE = (PE + 255) / 256;
  // (DEPTH 8 at c5: 446 vs 380 us)
  constexpr int COUT = 16 * MT, DEPTH = 4, ITS = FT_H * FT_W / 16;  // 4-pixel groups per wave and tile
  static_assert(ITS % DEPTH == 0, "groups per tile");
  __shared__ float patch[PE];
  __shared__ float red[4 * COUT * K9];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const DevSrc& s = a.dz.s0;
  const int H = a.dz.H, W = a.dz.W;
  const unsigned HW = (unsigned)H * (unsigned)W;
  float sc[MT], sh[MT], mu[MT], kx[MT], kc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int c = MT * li + m;
    sc[m] = s.coef[c];
    sh[m] = s.coef[COUT + c];
    mu[m] = s.coef[2 * COUT + c];
    kx[m] = s.coef[3 * COUT + c];
    kc[m] = s.coef[4 * COUT + c];
  }
  int toff[NN];  // the lane's tap of N tile nt: its offset in the patch (-1: padding tap)
#pragma unroll
  for (int nt = 0; nt < NN; ++nt) {
    const int j = li + 16 * nt, ci = j / 9, t = j - 9 * (j / 9);
    toff[nt] = j < K9 ? (ci * FT_PH + t / 3) * FT_PW + t % 3 : -1;
  }
  pmu_f32x4 acc[MT][NN];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) acc[m][nt] = pmu_f32x4{0.f, 0.f, 0.f, 0.f};
  const int t_beg = blockIdx.x * FW_TPB, t_end = min(ntiles, t_beg + FW_TPB);
  const int nj = (t_end - t_beg) * ITS;
  float pv[NPE];
  auto load_patch = [&](int tile) { first_patch_load<CIN>(a.planes, tile, tiles_w, tiles_h, H, W, pv); };
  // group j (flat over the block's tiles): the lane's pixel (clamped past the end: a valid address)
  auto pixel_of = [&](int j, unsigned& p, int& r, int& c, bool& ok) __attribute__((always_inline)) {
    const int jj = j < nj ? j : nj - 1;
    int t = t_beg + jj / ITS;
    const int q = wave * (FT_H * FT_W / 4) + (jj - (jj / ITS) * ITS) * 4 + lk;
    r = q / FT_W;
    c = q - r * FT_W;
    const int tw = t % tiles_w; t /= tiles_w;
    const int th = t % tiles_h;
    const int n = t / tiles_h;
    const int h = th * FT_H + r, w = tw * FT_W + c;
    ok = j < nj && h < H && w < W;
    p = (unsigned)n * HW + (unsigned)(min(h, H - 1) * W + min(w, W - 1));
  };
  float zq[DEPTH][MT], dq[DEPTH][MT];
  unsigned dqb[DEPTH][(MT + 1) / 2];  // (XB) raw bf16 pairs
  auto issue = [&](int j, int slot) __attribute__((always_inline)) {
    unsigned p; int r, c; bool ok;
    pixel_of(j, p, r, c, ok);
    const size_t e = (size_t)p * COUT + MT * li;
    const float* zp = s.z + e;
    if constexpr (MT == 4) {
      const float4 v = *reinterpret_cast<const float4*>(zp);
      zq[slot][0] = v.x; zq[slot][1] = v.y; zq[slot][2] = v.z; zq[slot][3] = v.w;
    } else if constexpr (MT == 2) {
      const float2 v = *reinterpret_cast<const float2*>(zp);
      zq[slot][0] = v.x; zq[slot][1] = v.y;
    } else {
      zq[slot][0] = *zp;
    }
    if constexpr (XB) {
      const unsigned short* dp = reinterpret_cast<const unsigned short*>(s.x) + e;
      if constexpr (MT == 4) {
        const uint2 v = *reinterpret_cast<const uint2*>(dp);
        dqb[slot][0] = v.x; dqb[slot][1] = v.y;
      } else if constexpr (MT == 2) {
        dqb[slot][0] = *reinterpret_cast<const unsigned*>(dp);
      } else {
        dqb[slot][0] = *dp;
      }
    } else {
      const float* dp = s.x + e;
      if constexpr (MT == 4) {
        const float4 v = *reinterpret_cast<const float4*>(dp);
        dq[slot][0] = v.x; dq[slot][1] = v.y; dq[slot][2] = v.z; dq[slot][3] = v.w;
      } else if constexpr (MT == 2) {
        const float2 v = *reinterpret_cast<const float2*>(dp);
        dq[slot][0] = v.x; dq[slot][1] = v.y;
      } else {
        dq[slot][0] = *dp;
      }
    }
  };
  auto consume = [&](int j, int slot) __attribute__((always_inline)) {
    unsigned p; int r, c; bool ok;
    pixel_of(j, p, r, c, ok);
    float g[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float d;
      if constexpr (XB) d = pmu_bf16_f32((unsigned short)(dqb[slot][m >> 1] >> (16 * (m & 1))));
      else d = dq[slot][m];
      g[m] = ok ? pmu_bnbwd1(d, zq[slot][m], sc[m], sh[m], mu[m], kx[m], kc[m]) : 0.f;
    }
    float b[NN];
#pragma unroll
    for (int nt = 0; nt < NN; ++nt) {
      const float v = patch[(toff[nt] < 0 ? 0 : toff[nt]) + r * FT_PW + c];
      b[nt] = toff[nt] < 0 ? 0.f : v;
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int nt = 0; nt < NN; ++nt) acc[m][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(g[m], b[nt], acc[m][nt], 0, 0, 0);
  };
  if (t_beg < t_end) {
    load_patch(t_beg);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) issue(d, d);
  }
  for (int tile = t_beg; tile < t_end; ++tile) {
    __syncthreads();  // the previous tile's patch reads are done
#pragma unroll
    for (int q = 0; q < NPE; ++q)
      if (tid + 256 * q < PE) patch[tid + 256 * q] = pv[q];
    __syncthreads();
    if (tile + 1 < t_end) load_patch(tile + 1);  // in flight under this tile's MFMAs
    const int j0 = (tile - t_beg) * ITS;
    for (int ii = 0; ii < ITS; ii += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        consume(j0 + ii + d, d);
        issue(j0 + ii + d + DEPTH, d);
      }
    }
  }
  // accumulator element e of (m, nt): channel MT (4 lk + e) + m, tap li + 16 nt; the 4 waves' sums in order
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int nt = 0; nt < NN; ++nt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = li + 16 * nt;
        if (j < K9) red[(wave * COUT + MT * (4 * lk + e) + m) * K9 + j] = acc[m][nt][e];
      }
  __syncthreads();
  for (int o = tid; o < COUT * K9; o += 256) {
    float v = 0.f;
#pragma unroll
    for (int wv = 0; wv < 4; ++wv) v += red[wv * COUT * K9 + o];
    a.ws[(long long)blockIdx.x * COUT * K9 + o] = v;
  }
}

// out[o] = sum_r ws[r][o]: block = 64 outputs x 4 row phases (fixed order), fp64 accumulation
__global__ __launch_bounds__(1024) void rows_sum4_kernel(const float* __restrict__ ws, int R, int Wd,
                                                         float* __restrict__ out) {
  __shared__ double red[1024];
  const int o = blockIdx.x * 64 + (threadIdx.x & 63);
  const double t = pmu_colsum64x16(ws, R, Wd, o, red);
  if (threadIdx.x < 64 && o < Wd) out[o] = (float)t;
}

// dw[o] = sum_b ws[b][o]
__global__ void rows_sum_kernel(const float* __restrict__ ws, int R, int Wd, float* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= Wd) return;
  double s = 0.0;
  for (int r = 0; r < R; ++r) s += ws[(long long)r * Wd + o];
  out[o] = (float)s;
}

}  // namespace

// rows of the forward's BN partial sums: one per 8 x 32 tile
extern "C" int pmu_conv_first_tiles(int N, int H, int W) {
  return N * pmu_cdiv(H, FT_H) * pmu_cdiv(W, FT_W);
}

extern "C" int pmu_conv_first_fwd(const float* const* planes, int Cin, int N, int H, int W,
                                  const float* w, const float* bias, int Cout, float* z, float* part,
                                  void* stream) {
  PMU_REQUIRE(planes && Cin >= 1 && Cin <= 4 && N > 0 && H > 0 && W > 0 && w && z);
  PMU_REQUIRE(Cout >= 4 && Cout <= 256 && Cout % 4 == 0 && 256 % (Cout / 4) == 0);
  PMU_REQUIRE((long long)N * H * W < (1LL << 31));
  FirstArgs a;
  for (int i = 0; i < 4; ++i) a.planes[i] = i < Cin ? planes[i] : nullptr;
  for (int i = 0; i < Cin; ++i) PMU_REQUIRE(planes[i]);
  a.Cin = Cin; a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.w = w; a.bias = bias; a.z = z; a.part = part;
  const int tw = pmu_cdiv(W, FT_W), th = pmu_cdiv(H, FT_H), nt = N * tw * th;
  const dim3 grid((unsigned)pmu_cdiv(nt, FT_TPB));
  hipStream_t st = (hipStream_t)stream;
#define PMU_FFM_LAUNCH(MTV)                                                                                       \
  switch (Cin) {                                                                                                  \
    case 1: hipLaunchKernelGGL((conv_first_fwd_mfma_kernel<1, MTV>), grid, dim3(256), 0, st, a, tw, th, nt); break; \
    case 2: hipLaunchKernelGGL((conv_first_fwd_mfma_kernel<2, MTV>), grid, dim3(256), 0, st, a, tw, th, nt); break; \
    case 3: hipLaunchKernelGGL((conv_first_fwd_mfma_kernel<3, MTV>), grid, dim3(256), 0, st, a, tw, th, nt); break; \
    default: hipLaunchKernelGGL((conv_first_fwd_mfma_kernel<4, MTV>), grid, dim3(256), 0, st, a, tw, th, nt); break; \
  }
  // MFMA form for three or four planes (c5: 382 -> 348 us); with one plane the VALU kernel is faster
  // (c2: 110 vs 124 us; 9 taps are three MFMA steps of the padded K)
  if (Cin >= 3 && Cout == 64) { PMU_FFM_LAUNCH(4) }
  else if (Cin >= 3 && Cout == 32) { PMU_FFM_LAUNCH(2) }
  else if (Cin >= 3 && Cout == 16) { PMU_FFM_LAUNCH(1) }
  else switch (Cin) {
    case 1: hipLaunchKernelGGL(conv_first_fwd_tile_kernel<1>, grid, dim3(256), 0, st, a, tw, th, nt); break;
    case 2: hipLaunchKernelGGL(conv_first_fwd_tile_kernel<2>, grid, dim3(256), 0, st, a, tw, th, nt); break;
    case 3: hipLaunchKernelGGL(conv_first_fwd_tile_kernel<3>, grid, dim3(256), 0, st, a, tw, th, nt); break;
    default: hipLaunchKernelGGL(conv_first_fwd_tile_kernel<4>, grid, dim3(256), 0, st, a, tw, th, nt); break;
  }
#undef PMU_FFM_LAUNCH
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

static bool first_wgrad_fast(const pmu_frame* dz, int Cout) {
  const pmu_src& s = dz->src[0];
  return s.mode == PMU_SRC_BNBWD && s.pool == PMU_POOL_NONE && s.off_h == 0 && s.off_w == 0 && s.H == dz->H &&
         s.W == dz->W && Cout % 8 == 0 && Cout <= 256 && 256 % (Cout / 4) == 0;  // (Cout / 4 pixels per tile
                                                                                  // and thread: paired)
}

extern "C" size_t pmu_conv_first_wgrad_ws(int N, int H, int W, int Cin, int Cout) {
  const long long P = (long long)N * H * W;
  const size_t slow = (size_t)pmu_cdiv(P, FWPIX) * Cout * Cin * 9 * sizeof(float);
  const size_t fast = (size_t)pmu_cdiv(N * pmu_cdiv(H, FT_H) * pmu_cdiv(W, FT_W), FW_TPB) * Cout * Cin * 9 *
                      sizeof(float);
  return slow > fast ? slow : fast;
}

extern "C" int pmu_conv_first_wgrad(const pmu_frame* dz, const float* const* planes, int Cin, int Cout,
                                    float* dw, float* ws, size_t ws_bytes, void* stream) {
  // (dz's da may be bf16-stored: the tiled kernel below takes it, the generic one reads through src_xform)
  PMU_REQUIRE(valid_frame(dz, true) && dz->nsrc == 1 && dz->src[0].C == Cout && planes && dw && ws);
  PMU_REQUIRE((dz->src[0].dtype & PMU_DT_Z_BF16) == 0);
  PMU_REQUIRE(Cin >= 1 && Cin <= 4 && Cout >= 1 && Cout <= 256 && 256 % Cout == 0);
  PMU_REQUIRE(ws_bytes >= pmu_conv_first_wgrad_ws(dz->N, dz->H, dz->W, Cin, Cout));
  FirstWgArgs a;
  a.dz = make_dev_frame(dz);
  for (int i = 0; i < 4; ++i) a.planes[i] = i < Cin ? planes[i] : nullptr;
  for (int i = 0; i < Cin; ++i) PMU_REQUIRE(planes[i]);
  a.Cin = Cin; a.Cout = Cout; a.ws = ws;
  hipStream_t st = (hipStream_t)stream;
  const long long P = (long long)dz->N * dz->H * dz->W;
  int nb;
  if (first_wgrad_fast(dz, Cout)) {
    const int tw = pmu_cdiv(dz->W, FT_W), th = pmu_cdiv(dz->H, FT_H), nt = dz->N * tw * th;
    PMU_REQUIRE(P < (1LL << 31));
    nb = pmu_cdiv(nt, FW_TPB);
#define PMU_FW_LAUNCH(XBV)                                                                                         \
  switch (Cin) {                                                                                                  \
    case 1: hipLaunchKernelGGL((conv_first_wgrad_tile_kernel<1, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
    case 2: hipLaunchKernelGGL((conv_first_wgrad_tile_kernel<2, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
    case 3: hipLaunchKernelGGL((conv_first_wgrad_tile_kernel<3, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
    default: hipLaunchKernelGGL((conv_first_wgrad_tile_kernel<4, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
  }
#define PMU_FWM_LAUNCH(MTV, XBV)                                                                                  \
  switch (Cin) {                                                                                                  \
    case 1: hipLaunchKernelGGL((conv_first_wgrad_mfma_kernel<1, MTV, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
    case 2: hipLaunchKernelGGL((conv_first_wgrad_mfma_kernel<2, MTV, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
    case 3: hipLaunchKernelGGL((conv_first_wgrad_mfma_kernel<3, MTV, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
    default: hipLaunchKernelGGL((conv_first_wgrad_mfma_kernel<4, MTV, XBV>), dim3((unsigned)nb), dim3(256), 0, st, a, tw, th, nt); break; \
  }
    const bool xb = dz->src[0].dtype & PMU_DT_X_BF16;
    if (Cout == 64) { if (xb) PMU_FWM_LAUNCH(4, true) else PMU_FWM_LAUNCH(4, false) }
    else if (Cout == 32) { if (xb) PMU_FWM_LAUNCH(2, true) else PMU_FWM_LAUNCH(2, false) }
    else if (Cout == 16) { if (xb) PMU_FWM_LAUNCH(1, true) else PMU_FWM_LAUNCH(1, false) }
    else if (xb) PMU_FW_LAUNCH(true)
    else PMU_FW_LAUNCH(false)
#undef PMU_FW_LAUNCH
#undef PMU_FWM_LAUNCH
  } else {
    nb = pmu_cdiv(P, FWPIX);
    hipLaunchKernelGGL(conv_first_wgrad_kernel, dim3((unsigned)nb), dim3(256), 0, st, a);
  }
  PMU_CHECK_LAUNCH();
  const int Wd = Cout * Cin * 9;
  hipLaunchKernelGGL(rows_sum4_kernel, dim3((unsigned)pmu_cdiv(Wd, 64)), dim3(1024), 0, st, (const float*)ws, nb, Wd,
                     dw);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
