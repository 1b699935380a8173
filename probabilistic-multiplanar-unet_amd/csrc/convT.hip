// ConvTranspose2d(Cin, Cout, kernel 2, stride 2) of Up (PMU/model/unet/unet_parts.py:52)
// forward and backward as GEMMs on f32 MFMA.
//
// The 2x2/s2 transposed conv never overlaps: u[n][2i+a][2j+b][co] = sum_ci x[n][i][j][ci] w[ci][co][a][b] + b[co]
//   forward : C[pix][co*4+ab] = act(x)[pix][ci] . W[ci][co*4+ab]       (M=pixels, N=4Cout, K=Cin)
//   dgrad   : dx[pix][ci] = sum_{ab,co} du[2i+a][2j+b][co] W[ci][co*4+ab] (M=pixels, N=Cin, K=4Cout)
//   wgrad   : dW[ci][co*4+ab] = sum_pix act(x)[pix][ci] du[2i+a][2j+b][co] (M=Cin, N=4Cout, K=pixels, split-K)
// du is the gradient of the concat's "up" half in the skip's frame; the convT output sits at
// (off_h, off_w) inside it (F.pad, unet_parts.py:58-62).
// Tile 128x128x16, 4 waves (2x2), wave tile 64x64 = 2x2 32x32 accumulators, LDS rows k-contiguous.
#include <cstdlib>
#include "pmu_stage.h"

namespace {

constexpr int GM = 128, GN = 128, GK = 16, GLS = 20;

struct PixDecode {
  int H, W;
  __device__ __forceinline__ void operator()(long long m, int& n, int& i, int& j) const {
    j = (int)(m % W);
    const long long t = m / W;
    i = (int)(t % H);
    n = (int)(t / H);
  }
};

// A[m=pixel][k=channel] = act(frame)
struct ActRowA {
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC = true;
  DevFrame f;
  PixDecode pd;
  __device__ float load(long long m, int k) const {
    int n, i, j; pd(m, n, i, j);
    return frame_value(f, n, i, j, k);
  }
  __device__ float4 load4(long long m, int k) const {
    int n, i, j; pd(m, n, i, j);
    return frame_value4(f, n, i, j, k);
  }
};
// B[k=ci][n] = W[ci*NN + n]
struct WKN_B {
  static constexpr bool KCONTIG = false;
  const float* w;
  int NN;
  __device__ float load(int k, int n) const { return w[(long long)k * NN + n]; }
};
// A[m=pixel][k'=ab*Cout+co] = du gathered
struct DuGatherA {
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC = true;
  const float* du;
  int Hd, Wd, off_h, off_w, Cout;
  PixDecode pd;
  __device__ __forceinline__ long long idx(long long m, int k) const {
    int n, i, j; pd(m, n, i, j);
    const int ab = k / Cout, co = k - ab * Cout;
    const int hh = off_h + 2 * i + (ab >> 1), ww = off_w + 2 * j + (ab & 1);
    return (((long long)n * Hd + hh) * Wd + ww) * Cout + co;
  }
  __device__ float load(long long m, int k) const { return du[idx(m, k)]; }
  __device__ float4 load4(long long m, int k) const {
    if ((Cout & 3) == 0) return *reinterpret_cast<const float4*>(du + idx(m, k));
    return make_float4(du[idx(m, k)], du[idx(m, k + 1)], du[idx(m, k + 2)], du[idx(m, k + 3)]);
  }
};
// B[k'=ab*Cout+co][n=ci] = W[ci][co*4+ab]
struct WT_B {
  static constexpr bool KCONTIG = true;
  const float* w;
  int Cout;
  __device__ float load(int k, int n) const {
    const int ab = k / Cout, co = k - ab * Cout;
    return w[(long long)n * Cout * 4 + co * 4 + ab];
  }
};
struct ScatterEp {  // convT forward output
  float* u;
  const float* bias;
  int H, W, Cout;
  PixDecode pd;
  __device__ void store(long long m, int col, float v, int) const {
    int n, i, j; pd(m, n, i, j);
    const int co = col >> 2, a = (col >> 1) & 1, b = col & 1;
    u[(((long long)n * 2 * H + 2 * i + a) * (2 * W) + 2 * j + b) * Cout + co] = v + (bias ? bias[co] : 0.f);
  }
};
struct RowEp {  // plain row-major store C[m][n]
  float* out;
  int ld;
  __device__ void store(long long m, int col, float v, int) const { out[m * ld + col] = v; }
};

template <class AL, class BL, class EP>
__global__ __launch_bounds__(256, 2) void gemm_kernel(AL al, BL bl, EP ep, long long M, int N, long long K, int cps) {
  __shared__ __attribute__((aligned(16))) float As[GM * GLS];
  __shared__ __attribute__((aligned(16))) float Bs[GN * GLS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)blockIdx.x * GM;
  const int n0 = blockIdx.y * GN;
  const int split = blockIdx.z;
  const long long nch = (K + GK - 1) / GK;
  const long long c_beg = (long long)split * cps;
  long long c_end = c_beg + cps;
  if (c_end > nch) c_end = nch;
  const int hsel = (lane >> 5) * 8;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (long long ch = c_beg; ch < c_end; ++ch) {
    const long long k0 = ch * GK;
    // ---- A tile [GM][GK]
    if constexpr (AL::KCONTIG && AL::VEC) {
      for (int it = tid; it < GM * GK / 4; it += 256) {
        const int ml = it >> 2, kq = (it & 3) * 4;
        const long long m = m0 + ml, k = k0 + kq;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < M) {
          if (k + 3 < K) v = al.load4(m, (int)k);
          else {
            float t[4];
            for (int e = 0; e < 4; ++e) t[e] = (k + e < K) ? al.load(m, (int)(k + e)) : 0.f;
            v = make_float4(t[0], t[1], t[2], t[3]);
          }
        }
        *reinterpret_cast<float4*>(As + ml * GLS + kq) = v;
      }
    } else if constexpr (AL::KCONTIG) {
      for (int it = tid; it < GM * GK; it += 256) {
        const int ml = it / GK, kl = it % GK;
        const long long m = m0 + ml, k = k0 + kl;
        As[ml * GLS + kl] = (m < M && k < K) ? al.load(m, k) : 0.f;
      }
    } else {
      for (int it = tid; it < GM * GK; it += 256) {
        const int kl = it / GM, ml = it % GM;
        const long long m = m0 + ml, k = k0 + kl;
        As[ml * GLS + kl] = (m < M && k < K) ? al.load(m, k) : 0.f;
      }
    }
    // ---- B tile, stored [GN][GK]
    if constexpr (BL::KCONTIG) {
      for (int it = tid; it < GN * GK; it += 256) {
        const int nl = it / GK, kl = it % GK;
        const int n = n0 + nl;
        const long long k = k0 + kl;
        Bs[nl * GLS + kl] = (n < N && k < K) ? bl.load(k, n) : 0.f;
      }
    } else {
      for (int it = tid; it < GN * GK; it += 256) {
        const int kl = it / GN, nl = it % GN;
        const int n = n0 + nl;
        const long long k = k0 + kl;
        Bs[nl * GLS + kl] = (n < N && k < K) ? bl.load(k, n) : 0.f;
      }
    }
    __syncthreads();
    float av[2][8], bv[2][8];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float* pa = As + (wm * 64 + f * 32 + (lane & 31)) * GLS + hsel;
      const float4 x0 = *reinterpret_cast<const float4*>(pa), x1 = *reinterpret_cast<const float4*>(pa + 4);
      av[f][0] = x0.x; av[f][1] = x0.y; av[f][2] = x0.z; av[f][3] = x0.w;
      av[f][4] = x1.x; av[f][5] = x1.y; av[f][6] = x1.z; av[f][7] = x1.w;
      const float* pb = Bs + (wn * 64 + f * 32 + (lane & 31)) * GLS + hsel;
      const float4 y0 = *reinterpret_cast<const float4*>(pb), y1 = *reinterpret_cast<const float4*>(pb + 4);
      bv[f][0] = y0.x; bv[f][1] = y0.y; bv[f][2] = y0.z; bv[f][3] = y0.w;
      bv[f][4] = y1.x; bv[f][5] = y1.y; bv[f][6] = y1.z; bv[f][7] = y1.w;
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = mfma_f32_32x32x2(av[fm][s], bv[fn][s], acc[fm][fn]);
    __syncthreads();
  }
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) {
    const int col = n0 + wn * 64 + fn * 32 + (lane & 31);
    if (col >= N) continue;
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = m0 + wm * 64 + fm * 32 + acc_row(r, lane);
        if (m < M) ep.store(m, col, acc[fm][fn][r], split);
      }
  }
}

// ---------------------------------------------------------------------------------
// Weight gradient: dW[ci][co][a][b] = sum_{n,i,j} act[n,i,j,ci] * du[n, oh+2i+a, ow+2j+b, co]
// Block: 64 ci (M) x 64 co (N) x 4 taps; split-K over 32-pixel tiles of the convT input.
// LDS: X[32 px][64 ci], D[4 taps][32 px][64 co]; wave w owns (ci frag w>>1, co frag w&1) x 4 taps
// and reuses its A fragment (act) across the 4 taps.  Blocks of ci-block 0 also accumulate the
// bias gradient sum du[..][co] from the staged D tile.
// ---------------------------------------------------------------------------------
constexpr int TB = 64;    // ci / co per block
constexpr int TPIX = 32;  // pixels per K tile

struct TwArgs {
  DevFrame act;
  const float* du;
  int Hd, Wd, off_h, off_w, Cout, Cin;
  int twl, tiles_w, tiles_h, ntiles, nsplit;
  float* ws;   // [split][4][Cin][Cout]
  float* bws;  // [split][Cout] or null
};

__global__ __launch_bounds__(256, 2) void convT_wgrad_kernel(TwArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[TPIX * TB + 4 * TPIX * TB];
  float* Xs = smem;
  float* Ds = smem + TPIX * TB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int TW = 1 << a.twl, TH = TPIX >> a.twl;
  const int nci = (a.Cin + TB - 1) / TB;
  // (channel block, split) in XCD order, channel blocks fastest (see wgrad3x3_bf16.hip)
  const int nblk = gridDim.x;
  const int lbk = pmu_xcd_block(blockIdx.y * nblk + blockIdx.x, nblk * gridDim.y);
  const int ci0 = (lbk % nblk % nci) * TB, co0 = (lbk % nblk / nci) * TB;
  const int split = lbk / nblk;
  const int cif = wave >> 1, cof = wave & 1;
  const bool do_bias = (a.bws != nullptr) && ci0 == 0;
  const bool vec = (a.Cout & 3) == 0;
  const DevFrame& X = a.act;
  const int H = X.H, W = X.W;

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum = 0.f;

  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);
  for (int tile = t_beg; tile < t_end; ++tile) {
    int t = tile;
    const int tw = t % a.tiles_w; t /= a.tiles_w;
    const int th = t % a.tiles_h; t /= a.tiles_h;
    const int n = t;
    const int i0 = th * TH, j0 = tw * TW;
    for (int it = tid; it < TPIX * 16; it += 256) {
      const int px = it >> 4, cq = it & 15;
      const float4 v = frame_value4(X, n, i0 + (px >> a.twl), j0 + (px & (TW - 1)), ci0 + 4 * cq);
      *reinterpret_cast<float4*>(Xs + px * TB + 4 * cq) = v;
    }
    for (int it = tid; it < 4 * TPIX * 16; it += 256) {
      const int cq = it & 15, px = (it >> 4) & (TPIX - 1), ab = it >> 9;
      const int i = i0 + (px >> a.twl), j = j0 + (px & (TW - 1));
      const int co = co0 + 4 * cq;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < H && j < W && co < a.Cout) {
        const long long base = (((long long)n * a.Hd + a.off_h + 2 * i + (ab >> 1)) * a.Wd + a.off_w + 2 * j + (ab & 1)) * a.Cout;
        if (vec && co + 3 < a.Cout) v = *reinterpret_cast<const float4*>(a.du + base + co);
        else {
          v.x = a.du[base + co];
          v.y = co + 1 < a.Cout ? a.du[base + co + 1] : 0.f;
          v.z = co + 2 < a.Cout ? a.du[base + co + 2] : 0.f;
          v.w = co + 3 < a.Cout ? a.du[base + co + 3] : 0.f;
        }
      }
      *reinterpret_cast<float4*>(Ds + (ab * TPIX + px) * TB + 4 * cq) = v;
    }
    __syncthreads();
    if (do_bias) {  // thread -> (co = tid & 63, tap = tid >> 6): sum over the tile's pixels
      const float* d = Ds + (tid >> 6) * TPIX * TB + (tid & 63);
#pragma unroll 8
      for (int px = 0; px < TPIX; ++px) bsum += d[px * TB];
    }
#pragma unroll 4
    for (int ks = 0; ks < TPIX / 2; ++ks) {
      const int px = 2 * ks + (lane >> 5);
      const float av = Xs[px * TB + cif * 32 + (lane & 31)];
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const float bv = Ds[(ab * TPIX + px) * TB + cof * 32 + (lane & 31)];
        acc[ab] = mfma_f32_32x32x2(av, bv, acc[ab]);
      }
    }
    __syncthreads();
  }
  const int co = co0 + cof * 32 + (lane & 31);
  if (co < a.Cout) {
#pragma unroll
    for (int ab = 0; ab < 4; ++ab)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + cif * 32 + acc_row(r, lane);
        if (ci < a.Cin) a.ws[(((long long)split * 4 + ab) * a.Cin + ci) * a.Cout + co] = acc[ab][r];
      }
  }
  if (do_bias) {
    Xs[tid] = bsum;  // LDS no longer read by the MFMA loop (last barrier passed)
    __syncthreads();
    if (tid < 64 && co0 + tid < a.Cout)
      a.bws[(long long)split * a.Cout + co0 + tid] = Xs[tid] + Xs[64 + tid] + Xs[128 + tid] + Xs[192 + tid];
  }
}

// registers of one in-flight tile of convT_wgrad_pipe_kernel (a struct passed by reference to
// inlined functions stays in VGPRs; captured by a lambda it was placed in scratch)
struct TwRegs {
  float4 rx0, rx1, rd[8];
  bool ox0, ox1;
  unsigned od;
};

__device__ __forceinline__ void tw_load(const TwArgs& a, int tile, int ci0, int co0, int tid, TwRegs& g) {
  const DevSrc& xs = a.act.s0;
  const int H = a.act.H, W = a.act.W;
  const int TW = 1 << a.twl, TH = TPIX >> a.twl;
  const int cq = tid & 15;
  int t = tile;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const long long n = t;
  const int i0 = th * TH, j0 = tw * TW;
  const int px = tid >> 4;  // act items tid and tid + 256: pixels px and px + 16
  const int i = i0 + (px >> a.twl), j = j0 + (px & (TW - 1));
  g.ox0 = i < H && j < W;
  g.rx0 = *reinterpret_cast<const float4*>(xs.x + (g.ox0 ? ((n * H + i) * W + j) * xs.C : 0) + ci0 + 4 * cq);
  const int px1 = px + 16;
  const int i1 = i0 + (px1 >> a.twl), j1 = j0 + (px1 & (TW - 1));
  g.ox1 = i1 < H && j1 < W;
  g.rx1 = *reinterpret_cast<const float4*>(xs.x + (g.ox1 ? ((n * H + i1) * W + j1) * xs.C : 0) + ci0 + 4 * cq);
  unsigned od = 0u;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int it = tid + 256 * r;
    const int p = (it >> 4) & (TPIX - 1), ab = it >> 9;
    const int ii = i0 + (p >> a.twl), jj = j0 + (p & (TW - 1));
    const bool ok = ii < H && jj < W;
    od |= ok ? (1u << r) : 0u;
    const long long base =
        ok ? ((n * a.Hd + a.off_h + 2 * ii + (ab >> 1)) * a.Wd + a.off_w + 2 * jj + (ab & 1)) * a.Cout : 0;
    g.rd[r] = *reinterpret_cast<const float4*>(a.du + base + co0 + 4 * cq);
  }
  g.od = od;
}

__device__ __forceinline__ void tw_store(const TwRegs& g, int tid, float4 xsc, float4 xsh, float* buf) {
  float* Xs = buf;
  float* Ds = buf + TPIX * TB;
  const int cq = tid & 15, px = tid >> 4;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 x0 = pmu_bnrelu4(g.rx0, xsc, xsh), x1 = pmu_bnrelu4(g.rx1, xsc, xsh);
  if (!g.ox0) x0 = z4;
  if (!g.ox1) x1 = z4;
  *reinterpret_cast<float4*>(Xs + px * TB + 4 * cq) = x0;
  *reinterpret_cast<float4*>(Xs + (px + 16) * TB + 4 * cq) = x1;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int it = tid + 256 * r;
    const int p = (it >> 4) & (TPIX - 1), ab = it >> 9;
    float4 v = g.rd[r];  // value select (a select of the two lvalues becomes an address select -> scratch)
    if (!((g.od >> r) & 1u)) v = z4;
    *reinterpret_cast<float4*>(Ds + (ab * TPIX + p) * TB + 4 * cq) = v;
  }
}

// Pipelined variant (act = one unpooled BN+ReLU source, Cin and Cout multiples of TB): the next
// tile's 2 act float4 and 8 du float4 per thread are loaded into registers before the current
// tile's 64 MFMAs per wave and written to the other half of a double-buffered LDS ring after them
// (2 x 40 KB: still 2 blocks per CU), one barrier per tile.
__global__ __launch_bounds__(256, 2) void convT_wgrad_pipe_kernel(TwArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (TPIX * TB + 4 * TPIX * TB)];
  constexpr int SL = TPIX * TB + 4 * TPIX * TB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nci = a.Cin / TB, nblk = nci * (a.Cout / TB);
  // 1-D grid, XCD-aware order: workgroups are dealt round-robin over the 8 XCDs; remap so each XCD
  // runs a contiguous range of logical blocks, i.e. all channel blocks of one K split (the same
  // pixels) run together on one XCD and share their du / act tiles through its L2
  const int nb = gridDim.x, x = blockIdx.x & 7, q = nb >> 3, rr = nb & 7;
  const int lb = x * q + (x < rr ? x : rr) + (blockIdx.x >> 3);
  const int bx = lb % nblk;
  const int ci0 = (bx % nci) * TB, co0 = (bx / nci) * TB;
  const int split = lb / nblk;
  const int cif = wave >> 1, cof = wave & 1;
  const bool do_bias = (a.bws != nullptr) && ci0 == 0;
  const DevSrc& xs = a.act.s0;
  const int cq = tid & 15;
  const float4 xsc = *reinterpret_cast<const float4*>(xs.coef + ci0 + 4 * cq);
  const float4 xsh = *reinterpret_cast<const float4*>(xs.coef + xs.C + ci0 + 4 * cq);

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum = 0.f;

  TwRegs rg;

  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);
  if (t_beg < t_end) {
    tw_load(a, t_beg, ci0, co0, tid, rg);
    tw_store(rg, tid, xsc, xsh, smem);
  }
  __syncthreads();
  for (int tile = t_beg; tile < t_end; ++tile) {
    const int cur = (tile - t_beg) & 1;
    const bool more = tile + 1 < t_end;
    if (more) tw_load(a, tile + 1, ci0, co0, tid, rg);
    const float* Xs = smem + cur * SL;
    const float* Ds = Xs + TPIX * TB;
    if (do_bias) {  // thread -> (co = tid & 63, tap = tid >> 6): sum over the tile's pixels
      const float* d = Ds + (tid >> 6) * TPIX * TB + (tid & 63);
#pragma unroll 8
      for (int px = 0; px < TPIX; ++px) bsum += d[px * TB];
    }
#pragma unroll
    for (int ks = 0; ks < TPIX / 2; ++ks) {
      const int px = 2 * ks + (lane >> 5);
      const float av = Xs[px * TB + cif * 32 + (lane & 31)];
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        const float bv = Ds[(ab * TPIX + px) * TB + cof * 32 + (lane & 31)];
        acc[ab] = mfma_f32_32x32x2(av, bv, acc[ab]);
      }
    }
    if (more) tw_store(rg, tid, xsc, xsh, smem + (cur ^ 1) * SL);
    __syncthreads();
  }
  const int co = co0 + cof * 32 + (lane & 31);
#pragma unroll
  for (int ab = 0; ab < 4; ++ab)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ci = ci0 + cif * 32 + acc_row(r, lane);
      a.ws[(((long long)split * 4 + ab) * a.Cin + ci) * a.Cout + co] = acc[ab][r];
    }
  if (do_bias) {
    smem[tid] = bsum;  // LDS no longer read by the MFMA loop (last barrier passed)
    __syncthreads();
    if (tid < 64) a.bws[(long long)split * a.Cout + co0 + tid] = smem[tid] + smem[64 + tid] + smem[128 + tid] + smem[192 + tid];
  }
}

// dW[ci][co][a][b] = sum_s ws[s][ab][ci][co]: a block owns 64 consecutive elements, its 4 waves sum
// the splits s = g, g+4, ... and wave 0 adds the 4 partials in order (deterministic)
__global__ __launch_bounds__(256) void convT_wreduce_kernel(const float* __restrict__ ws, int nsplit, int Cin, int Cout,
                                                            float* __restrict__ dw) {
  __shared__ float red[4][64];
  const long long CC = (long long)Cin * Cout;
  const long long E = 4 * CC;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + lane;  // (ab*Cin + ci)*Cout + co
  float s0 = 0.f, s1 = 0.f;
  if (e < E) {
    int sp = g;
    for (; sp + 4 < nsplit; sp += 8) {
      s0 += ws[(long long)sp * E + e];
      s1 += ws[(long long)(sp + 4) * E + e];
    }
    for (; sp < nsplit; sp += 4) s0 += ws[(long long)sp * E + e];
  }
  red[g][lane] = s0 + s1;
  __syncthreads();
  if (g == 0 && e < E) {
    const float s = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    const int ab = (int)(e / CC);
    const long long cc = e - ab * CC;  // ci*Cout + co
    dw[cc * 4 + ab] = s;
  }
}

__global__ void rows_sum_f32_kernel(const float* __restrict__ ws, int R, int Wd, float* __restrict__ out) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= Wd) return;
  double s = 0.0;
  for (int r = 0; r < R; ++r) s += ws[(long long)r * Wd + o];
  out[o] = (float)s;
}

// ---------------------------------------------------------------------------------
// Pipelined ConvT forward / dgrad GEMM (the common case: Cin, Cout multiples of 16, the forward
// operand a single unpooled BN+ReLU source).  128x128x16 tiles, 4 waves of 64x64, double-buffered
// LDS: the next chunk's global loads are issued before the current chunk's MFMAs and written to
// the other buffer afterwards, so one barrier per chunk and the load latency hides under MFMAs.
// Both B operands come pre-packed k-contiguous (pmu_convT2x2_pack):
//   forward: Bp[n = ab*Cout + co][ci] = W[ci][co][ab]   (N ordered (ab, co): the scatter epilogue
//            writes 32 consecutive channels of one output pixel per fragment column block)
//   dgrad  : Bp[ci][k' = ab*Cout + co] = W[ci][co][ab]
// ---------------------------------------------------------------------------------
constexpr int PM = 128, PN = 128, PK = 16, PLS = 20;

struct PipeArgs {
  const float* a;      // fwd: z [M][Cin] (pre-BN);  dgrad: du [N][Hd][Wd][Cout]
  const float* coef;   // fwd: [scale|shift] of the BN feeding the convT
  const float* bp;     // packed B [Ncols][K]
  const float* bias;   // fwd: [Cout]
  float* out;          // fwd: u [N][2H][2W][Cout];  dgrad: dx [M][Cin]
  long long M;
  int Ncols, K;        // GEMM N and K
  int H, W, Cin, Cout;
  int Hd, Wd, off_h, off_w;
  int lw, lh;          // fwd: log2 W, log2 H when powers of two, else -1
  int nnb, xcd;        // column blocks; 1: 1-D XCD-ordered grid, column blocks fastest
  int ldo;             // fwd: output pixel stride (floats; Cout, or the concat operand's width)
};

template <int OFF>
__device__ __forceinline__ float4 ct_lds_b128(unsigned addr) {
  float4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned ct_lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(p);
}

// PF2: the operands of chunk c + 2 are loaded while chunk c's MFMAs run (two register sets in
// alternation), so a chunk's global loads have two chunks' MFMAs (2 x 2048 cycles per wave) to land
// before their LDS store instead of one
template <bool DGRAD, int EXP = 0, bool PF2 = false>
__global__ __launch_bounds__(256, 2) void convT_pipe_kernel(PipeArgs p) {
  __shared__ __attribute__((aligned(16))) float As[2][PM * PLS];
  __shared__ __attribute__((aligned(16))) float Bs[2][PN * PLS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // with p.xcd the column blocks of one row block run back to back on one XCD, so the A rows (the
  // big operand) come from HBM once and are re-read from that XCD's L2
  long long mb;
  int nb_;
  if (p.xcd) {
    const int lb = pmu_xcd_block(blockIdx.x, gridDim.x);
    nb_ = lb % p.nnb;
    mb = lb / p.nnb;
  } else {
    mb = blockIdx.x;
    nb_ = blockIdx.y;
  }
  const long long m0 = mb * PM;
  const int n0 = nb_ * PN;
  const int hsel = (lane >> 5) * 8;
  // this thread's two A rows and two B rows (fixed over the K loop), 4 consecutive k each
  const int kq = (tid & 3) * 4;
  const int rl0 = tid >> 2, rl1 = rl0 + 64;
  const bool rok0 = m0 + rl0 < p.M, rok1 = m0 + rl1 < p.M;
  // A row base: fwd = row start of z; dgrad = du element of (2i, 2j) of the row's pixel, ab added per chunk
  auto row_base = [&](long long m) -> long long {
    if constexpr (DGRAD) {
      const int j = (int)(m % p.W);
      const long long t = m / p.W;
      const int i = (int)(t % p.H);
      const long long n = t / p.H;
      return ((n * p.Hd + p.off_h + 2 * i) * p.Wd + p.off_w + 2 * j) * p.Cout;
    } else {
      return m * p.Cin;
    }
  };
  const long long ab0 = row_base(rok0 ? m0 + rl0 : 0), ab1 = row_base(rok1 ? m0 + rl1 : 0);
  const float* br0 = p.bp + (long long)(n0 + rl0) * p.K + kq;
  const float* br1 = p.bp + (long long)(n0 + rl1) * p.K + kq;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // staging as macros over plain locals (captured by a lambda, the DGRAD registers went to scratch);
  // set S (0, or 1 for PF2's second set)
  float4 ra0_0, ra1_0, rb0_0, rb1_0, rsc_0, rsh_0;
  float4 ra0_1, ra1_1, rb0_1, rb1_1, rsc_1, rsh_1;
#define PMU_TLOAD(K0, S)                                                                                    \
  {                                                                                                        \
    const int k0_ = (K0);                                                                                  \
    long long off_ = k0_ + kq;                                                                             \
    if constexpr (DGRAD) {                                                                                 \
      const int ab_ = k0_ / p.Cout;                                                                        \
      off_ = ((long long)(ab_ >> 1) * p.Wd + (ab_ & 1)) * p.Cout + (k0_ - ab_ * p.Cout) + kq;              \
    } else { /* the chunk's BN coefficients travel with its operand (loaded under the MFMAs too) */       \
      rsc_##S = *reinterpret_cast<const float4*>(p.coef + k0_ + kq);                                       \
      rsh_##S = *reinterpret_cast<const float4*>(p.coef + p.Cin + k0_ + kq);                               \
    }                                                                                                      \
    /* unconditional: rows past M read row 0 (row_base) and are zeroed at the store; a guarded */        \
    /* load became 4 branchy dword loads per row */                                                        \
    ra0_##S = *reinterpret_cast<const float4*>(p.a + ab0 + off_);                                          \
    ra1_##S = *reinterpret_cast<const float4*>(p.a + ab1 + off_);                                          \
    rb0_##S = *reinterpret_cast<const float4*>(br0 + k0_);                                                 \
    rb1_##S = *reinterpret_cast<const float4*>(br1 + k0_);                                                 \
  }
#define PMU_TBN(V, S) make_float4(fmaxf(0.f, fmaf((V).x, rsc_##S.x, rsh_##S.x)), fmaxf(0.f, fmaf((V).y, rsc_##S.y, rsh_##S.y)), \
                                  fmaxf(0.f, fmaf((V).z, rsc_##S.z, rsh_##S.z)), fmaxf(0.f, fmaf((V).w, rsc_##S.w, rsh_##S.w)))
#define PMU_TSTORE(BUF, S)                                                                                  \
  {                                                                                                        \
    if constexpr (!DGRAD && EXP != 2) { /* BN + ReLU of the producer, in registers */                     \
      ra0_##S = PMU_TBN(ra0_##S, S);                                                                       \
      ra1_##S = PMU_TBN(ra1_##S, S);                                                                       \
    }                                                                                                      \
    if (!rok0) ra0_##S = make_float4(0.f, 0.f, 0.f, 0.f); /* rows past M stay zero */                      \
    if (!rok1) ra1_##S = make_float4(0.f, 0.f, 0.f, 0.f);                                                  \
    *reinterpret_cast<float4*>(&As[BUF][rl0 * PLS + kq]) = ra0_##S;                                        \
    *reinterpret_cast<float4*>(&As[BUF][rl1 * PLS + kq]) = ra1_##S;                                        \
    *reinterpret_cast<float4*>(&Bs[BUF][rl0 * PLS + kq]) = rb0_##S;                                        \
    *reinterpret_cast<float4*>(&Bs[BUF][rl1 * PLS + kq]) = rb1_##S;                                        \
  }

  const int nch = p.K / PK;
  // one chunk's MFMAs on LDS buffer CUR
  auto chunk_mfma = [&](int cur) __attribute__((always_inline)) {
    // the chunk's operands in two halves (k-steps 0-3, then 4-7), the second half's reads in flight
    // under the first half's 16 MFMAs (one wait for all eight reads exposed the LDS latency)
    // (explicit ds_read_b128 + waits: the compiler's own wait was one lgkmcnt(0) for all eight)
    float4 av[2][2], bv[2][2];  // [half][fragment]
    const unsigned aa = ct_lds_addr(&As[cur][(wm * 64 + (lane & 31)) * PLS + hsel]);
    const unsigned ba = ct_lds_addr(&Bs[cur][(wn * 64 + (lane & 31)) * PLS + hsel]);
    __builtin_amdgcn_sched_barrier(0);
    av[0][0] = ct_lds_b128<0>(aa);
    bv[0][0] = ct_lds_b128<0>(ba);
    av[0][1] = ct_lds_b128<32 * PLS * 4>(aa);
    bv[0][1] = ct_lds_b128<32 * PLS * 4>(ba);
    av[1][0] = ct_lds_b128<16>(aa);
    bv[1][0] = ct_lds_b128<16>(ba);
    av[1][1] = ct_lds_b128<32 * PLS * 4 + 16>(aa);
    bv[1][1] = ct_lds_b128<32 * PLS * 4 + 16>(ba);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      __builtin_amdgcn_sched_barrier(0);
      if (hf == 0) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn) {
            const float4 x = av[hf][fm], y = bv[hf][fn];
            const float xa = s == 0 ? x.x : s == 1 ? x.y : s == 2 ? x.z : x.w;
            const float yb = s == 0 ? y.x : s == 1 ? y.y : s == 2 ? y.z : y.w;
            acc[fm][fn] = mfma_f32_32x32x2(xa, yb, acc[fm][fn]);
          }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  PMU_TLOAD(0, 0)
  PMU_TSTORE(0, 0)
  __syncthreads();
  if constexpr (!PF2) {
    for (int c = 0; c < nch; ++c) {
      const int cur = c & 1;
      if (c + 1 < nch) PMU_TLOAD((c + 1) * PK, 0)
      chunk_mfma(cur);
      if (c + 1 < nch) PMU_TSTORE(cur ^ 1, 0)
      __syncthreads();
    }
  } else {
    // set 1 holds chunk c + 1 at even c, set 0 at odd c: chunk c + 2 goes into the set chunk c came in
    if (nch > 1) PMU_TLOAD(PK, 1)
    for (int c = 0; c < nch; c += 2) {
      if (c + 2 < nch) PMU_TLOAD((c + 2) * PK, 0)
      chunk_mfma(0);
      if (c + 1 < nch) PMU_TSTORE(1, 1)
      __syncthreads();
      if (c + 1 >= nch) break;
      if (c + 3 < nch) PMU_TLOAD((c + 3) * PK, 1)
      chunk_mfma(1);
      if (c + 2 < nch) PMU_TSTORE(0, 0)
      __syncthreads();
    }
  }
#undef PMU_TLOAD
#undef PMU_TBN
#undef PMU_TSTORE
  // epilogue
#pragma unroll
  for (int fn = 0; fn < 2; ++fn) {
    const int col = n0 + wn * 64 + fn * 32 + (lane & 31);
    if constexpr (DGRAD) {
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long m = m0 + wm * 64 + fm * 32 + acc_row(r, lane);
          if (m < p.M) p.out[m * p.Cin + col] = acc[fm][fn][r];
        }
    } else {
      const int ab = col / p.Cout, co = col - ab * p.Cout;
      float b = p.bias ? p.bias[co] : 0.f;
      // consumed here, unconditionally: first consumed inside the per-output store branches (the compiler
      // sinks the add into them), the bias made each branch wait vmcnt(0), i.e. for every earlier store
      asm volatile("" : "+v"(b));
      const unsigned Wu = (unsigned)p.W, Hu = (unsigned)p.H;  // 32-bit decode (M < 2^31, host-checked)
      const int ldo = p.ldo;
      float* outc = p.out + (long long)(ab >> 1) * 2 * p.W * ldo + (ab & 1) * ldo + co;
      const bool full = m0 + PM <= p.M;
      if (p.lw >= 0 && p.lh >= 0) {  // power-of-two H, W: shift/mask decode
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned m = (unsigned)(m0 + wm * 64 + fm * 32 + acc_row(r, lane));
            if (EXP == 1 && acc[fm][fn][r] != -1.2345f) continue;
            // the bias added outside the store's branch: first consumed inside it, it made the
            // compiler wait vmcnt(0) — for every earlier store — in each branch
            const float v = acc[fm][fn][r] + b;
            if (full || m < (unsigned)p.M) {
              const unsigned j = m & (Wu - 1), t = m >> p.lw;
              const unsigned i = t & (Hu - 1), n = t >> p.lh;
              outc[(size_t)(((n * 2 * Hu + 2 * i) * (2 * Wu) + 2 * j)) * (unsigned)ldo] = v;
            }
          }
      } else {
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned m = (unsigned)(m0 + wm * 64 + fm * 32 + acc_row(r, lane));
            const float v = acc[fm][fn][r] + b;
            if (m < (unsigned)p.M) {
              const unsigned t = m / Wu, j = m - t * Wu;
              const unsigned n = t / Hu, i = t - n * Hu;
              outc[((long long)(n * 2 * Hu + 2 * i) * (2 * Wu) + 2 * j) * ldo] = v;
            }
          }
      }
    }
  }
}

// packed B operands (see above); e over Cin*Cout*4
__device__ __forceinline__ void convT_pack_one(const float* __restrict__ w, int Cin, int Cout, int dgrad,
                                               float* __restrict__ wp, long long e) {
  const long long E = 4LL * Cin * Cout;
  if (e >= E) return;
  // read-coalesced: e = (ci*Cout + co)*4 + ab
  const int ab = (int)(e & 3);
  const long long cc = e >> 2;
  const int co = (int)(cc % Cout), ci = (int)(cc / Cout);
  const float v = w[e];
  if (dgrad) wp[(long long)ci * 4 * Cout + ab * Cout + co] = v;
  else wp[((long long)ab * Cout + co) * Cin + ci] = v;
}
__global__ void convT_pack_kernel(const float* __restrict__ w, int Cin, int Cout, int dgrad, float* __restrict__ wp) {
  convT_pack_one(w, Cin, Cout, dgrad, wp, (long long)blockIdx.x * blockDim.x + threadIdx.x);
}
// job: Cout = the ConvTranspose2d's Cin, Cin = its Cout (w [Cin][Cout][2][2])
__global__ void convT_pack_multi_kernel(const pmu_pack_job* __restrict__ jobs, int njobs, int dgrad) {
  const pmu_pack_job& j = jobs[pmu_job_of(jobs, njobs, blockIdx.x)];
  convT_pack_one(j.w, j.Cout, j.Cin, dgrad, (float*)j.dst, (long long)(blockIdx.x - j.block0) * blockDim.x + threadIdx.x);
}

static bool pipe_ok_fwd(const pmu_frame* in, int Cout) {
  const pmu_src& s = in->src[0];
  return in->nsrc == 1 && s.mode == PMU_SRC_BNRELU && s.pool == PMU_POOL_NONE && s.off_h == 0 && s.off_w == 0 &&
         s.H == in->H && s.W == in->W && s.C % PK == 0 && Cout % PK == 0 && (4 * Cout) % PN == 0;
}

static void convT_wgrad_geometry(int N, int H, int W, int Cin, int Cout, int* twl, int* tiles_w, int* tiles_h,
                                 int* ntiles, int* nsplit) {
  *twl = (W > 4) ? 3 : 2;  // 4x8 or 8x4 pixel tiles
  const int TW = 1 << *twl, TH = TPIX / TW;
  *tiles_w = pmu_cdiv(W, TW);
  *tiles_h = pmu_cdiv(H, TH);
  *ntiles = N * *tiles_w * *tiles_h;
  const int bmn = pmu_cdiv(Cin, TB) * pmu_cdiv(Cout, TB);
  static const int target = [] {  // PMU_CONVT_WBLOCKS: workgroups the split-K aims for (A/B)
    const char* e = getenv("PMU_CONVT_WBLOCKS");
    return e ? atoi(e) : 512;  // one wave of the 2-per-CU workgroups: 1.68 -> 1.54 ms per c2 step (1024 before)
  }();
  int sp = target / bmn;
  if (sp < 1) sp = 1;
  if (sp > *ntiles) sp = *ntiles;
  *nsplit = sp;
}

}  // namespace

static void pipe_grid(PipeArgs& p, int nnb) {
  static const int xcd = [] {
    const char* e = pmu_variant_env("PMU_CONVT_XCD");
    return e ? atoi(e) : 1;
  }();
  p.nnb = nnb;
  p.xcd = xcd && (long long)pmu_cdiv(p.M, PM) * nnb < (1LL << 31);
}

extern "C" size_t pmu_convT2x2_packed_size(int Cin, int Cout) {
  return (Cin > 0 && Cout > 0) ? (size_t)4 * Cin * Cout * sizeof(float) : 0;
}

extern "C" int pmu_convT2x2_pack(const float* w, int Cin, int Cout, int dgrad, float* wp, void* stream) {
  PMU_REQUIRE(w && wp && Cin > 0 && Cout > 0);
  const long long E = 4LL * Cin * Cout;
  hipLaunchKernelGGL(convT_pack_kernel, dim3((unsigned)pmu_cdiv(E, 256)), dim3(256), 0, (hipStream_t)stream, w, Cin,
                     Cout, dgrad, wp);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

static int convT_fwd(const pmu_frame* in, const float* w, const float* wp, const float* bias, int Cout, float* u,
                     int ldo, void* stream) {
  PMU_REQUIRE(valid_frame(in) && w && u && Cout > 0 && ldo >= Cout);
  const long long M = (long long)in->N * in->H * in->W;
  if (wp && pipe_ok_fwd(in, Cout) && M < (1LL << 31)) {
    PipeArgs p{};
    p.a = in->src[0].x; p.coef = in->src[0].coef; p.bp = wp; p.bias = bias; p.out = u;
    p.M = M; p.Ncols = 4 * Cout; p.K = in->src[0].C;
    p.H = in->H; p.W = in->W; p.Cin = in->src[0].C; p.Cout = Cout; p.ldo = ldo;
    auto log2_or = [](int v) { return (v & (v - 1)) == 0 ? __builtin_ctz((unsigned)v) : -1; };
    p.lw = log2_or(in->W); p.lh = log2_or(in->H);
    // the output index (((n*2H + 2i)*2W + 2j)*Cout + co) stays 32-bit in the shift path
    if (4LL * M * ldo >= (1LL << 32)) p.lw = -1;
    pipe_grid(p, p.Ncols / PN);
    const dim3 grid = p.xcd ? dim3((unsigned)(pmu_cdiv(M, PM) * p.nnb)) : dim3((unsigned)pmu_cdiv(M, PM), (unsigned)p.nnb);
#ifdef PMU_EXPERIMENTS
    // timing experiments (wrong results): only in `make EXPERIMENTS=1` builds
    static const int exp = [] {
      const char* e = pmu_variant_env("PMU_CONVT_EXP");
      return e ? atoi(e) : 0;
    }();
    static const int pf1 = [] {  // PMU_CONVT_PF2=0: one chunk of prefetch (the round-5 kernel; A/B)
      const char* e = pmu_variant_env("PMU_CONVT_PF2");
      return e ? atoi(e) == 0 : 0;
    }();
    if (exp == 1) hipLaunchKernelGGL((convT_pipe_kernel<false, 1>), grid, dim3(256), 0, (hipStream_t)stream, p);
    else if (exp == 2) hipLaunchKernelGGL((convT_pipe_kernel<false, 2>), grid, dim3(256), 0, (hipStream_t)stream, p);
    else if (pf1) hipLaunchKernelGGL((convT_pipe_kernel<false>), grid, dim3(256), 0, (hipStream_t)stream, p);
    else
#endif
    // two chunks of prefetch: kbench over the c2 shapes 1.56 -> 1.42 ms (the K = 1024 layer -22%)
    hipLaunchKernelGGL((convT_pipe_kernel<false, 0, true>), grid, dim3(256), 0, (hipStream_t)stream, p);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  PMU_REQUIRE(ldo == Cout);  // (the strided output is the pipelined kernel's)
  ActRowA al{make_dev_frame(in), PixDecode{in->H, in->W}};
  const int Cin = al.f.C;
  WKN_B bl{w, 4 * Cout};
  ScatterEp ep{u, bias, in->H, in->W, Cout, PixDecode{in->H, in->W}};
  const int N = 4 * Cout;
  const long long nch = (Cin + GK - 1) / GK;
  dim3 grid((unsigned)pmu_cdiv(M, GM), (unsigned)pmu_cdiv(N, GN), 1);
  hipLaunchKernelGGL((gemm_kernel<ActRowA, WKN_B, ScatterEp>), grid, dim3(256), 0, (hipStream_t)stream, al, bl, ep, M,
                     N, (long long)Cin, (int)nch);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_convT2x2_fwd(const pmu_frame* in, const float* w, const float* wp, const float* bias, int Cout,
                                float* u, void* stream) {
  return convT_fwd(in, w, wp, bias, Cout, u, Cout, stream);
}

// The transposed conv written straight into channels [0, Cout) of a wider NHWC tensor whose pixels are
// ldo floats apart: the up-sampled half of the Up block's concat operand (unet_parts.py:52,66), so
// the operand materialisation copies only the skip half.  Pipelined path only (wp, pmu_convT2x2_fwd_ld_ok).
extern "C" int pmu_convT2x2_fwd_ld_ok(const pmu_frame* in, int Cout) {
  return valid_frame(in) && pipe_ok_fwd(in, Cout) && (long long)in->N * in->H * in->W < (1LL << 31);
}
extern "C" int pmu_convT2x2_fwd_ld(const pmu_frame* in, const float* w, const float* wp, const float* bias, int Cout,
                                   float* u, int ldo, void* stream) {
  PMU_REQUIRE(wp && pmu_convT2x2_fwd_ld_ok(in, Cout));
  return convT_fwd(in, w, wp, bias, Cout, u, ldo, stream);
}

extern "C" int pmu_convT2x2_dgrad(const float* du, int Hd, int Wd, int off_h, int off_w, const float* w,
                                  const float* wp, int N, int H, int W, int Cin, int Cout, float* dx, void* stream) {
  PMU_REQUIRE(du && w && dx && N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0);
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  const long long M = (long long)N * H * W;
  if (wp && Cout % PK == 0 && Cin % PN == 0) {
    PipeArgs p{};
    p.a = du; p.bp = wp; p.out = dx;
    p.M = M; p.Ncols = Cin; p.K = 4 * Cout;
    p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
    p.Hd = Hd; p.Wd = Wd; p.off_h = off_h; p.off_w = off_w;
    pipe_grid(p, Cin / PN);
    const dim3 grid = p.xcd ? dim3((unsigned)(pmu_cdiv(M, PM) * p.nnb)) : dim3((unsigned)pmu_cdiv(M, PM), (unsigned)p.nnb);
#ifdef PMU_EXPERIMENTS
    static const int pf2 = [] {
      const char* e = pmu_variant_env("PMU_CONVT_PF2");
      return e ? atoi(e) : 0;
    }();
    if (pf2) hipLaunchKernelGGL((convT_pipe_kernel<true, 0, true>), grid, dim3(256), 0, (hipStream_t)stream, p);
    else
#endif
    // (two chunks of prefetch measured equal here: 1.249 vs 1.244 ms over the c2 shapes)
    hipLaunchKernelGGL(convT_pipe_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, p);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  DuGatherA al{du, Hd, Wd, off_h, off_w, Cout, PixDecode{H, W}};
  WT_B bl{w, Cout};
  RowEp ep{dx, Cin};
  const long long K = 4LL * Cout;
  dim3 grid((unsigned)pmu_cdiv(M, GM), (unsigned)pmu_cdiv(Cin, GN), 1);
  hipLaunchKernelGGL((gemm_kernel<DuGatherA, WT_B, RowEp>), grid, dim3(256), 0, (hipStream_t)stream, al, bl, ep, M,
                     Cin, K, (int)((K + GK - 1) / GK));
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" size_t pmu_convT2x2_wgrad_ws(int N, int H, int W, int Cin, int Cout) {
  int twl, tw, th, nt, ns;
  convT_wgrad_geometry(N, H, W, Cin, Cout, &twl, &tw, &th, &nt, &ns);
  return (size_t)ns * (4 * (size_t)Cin * Cout + Cout) * sizeof(float);
}

extern "C" int pmu_convT2x2_wgrad(const float* du, int Hd, int Wd, int off_h, int off_w, const pmu_frame* act,
                                  int Cout, float* dw, float* dbias, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(du && valid_frame(act) && dw && ws && Cout > 0);
  const int N = act->N, H = act->H, W = act->W;
  PMU_REQUIRE(off_h >= 0 && off_w >= 0 && off_h + 2 * H <= Hd && off_w + 2 * W <= Wd);
  TwArgs a;
  a.act = make_dev_frame(act);
  a.du = du; a.Hd = Hd; a.Wd = Wd; a.off_h = off_h; a.off_w = off_w; a.Cout = Cout; a.Cin = a.act.C;
  convT_wgrad_geometry(N, H, W, a.Cin, Cout, &a.twl, &a.tiles_w, &a.tiles_h, &a.ntiles, &a.nsplit);
  PMU_REQUIRE(ws_bytes >= pmu_convT2x2_wgrad_ws(N, H, W, a.Cin, Cout));
  a.ws = ws;
  a.bws = dbias ? ws + (size_t)a.nsplit * 4 * a.Cin * Cout : nullptr;
  dim3 grid((unsigned)(pmu_cdiv(a.Cin, TB) * pmu_cdiv(Cout, TB)), (unsigned)a.nsplit);
  const pmu_src& xs = act->src[0];
  const bool pipe = act->nsrc == 1 && xs.mode == PMU_SRC_BNRELU && xs.pool == PMU_POOL_NONE && xs.off_h == 0 &&
                    xs.off_w == 0 && xs.H == act->H && xs.W == act->W && a.Cin % TB == 0 && Cout % TB == 0;
  if (pipe)
    hipLaunchKernelGGL(convT_wgrad_pipe_kernel, dim3(grid.x * grid.y), dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(convT_wgrad_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
  PMU_CHECK_LAUNCH();
  const long long E = 4LL * a.Cin * Cout;
  hipLaunchKernelGGL(convT_wreduce_kernel, dim3((unsigned)pmu_cdiv(E, 64)), dim3(256), 0, (hipStream_t)stream,
                     (const float*)ws, a.nsplit, a.Cin, Cout, dw);
  PMU_CHECK_LAUNCH();
  if (dbias) {
    hipLaunchKernelGGL(rows_sum_f32_kernel, dim3((unsigned)pmu_cdiv(Cout, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)a.bws, a.nsplit, Cout, dbias);
    PMU_CHECK_LAUNCH();
  }
  return PMU_OK;
}

extern "C" int pmu_convT2x2_pack_blocks(int Cin, int Cout, int dgrad) {
  (void)dgrad;
  return pmu_cdiv(4LL * Cin * Cout, 256);
}

// jobs[]: .Cout = the ConvTranspose2d's in_channels, .Cin = its out_channels (w [Cin][Cout][2][2])
extern "C" int pmu_convT2x2_pack_multi(const pmu_pack_job* jobs, int njobs, int blocks, int dgrad, void* stream) {
  PMU_REQUIRE(jobs && njobs > 0 && blocks > 0);
  hipLaunchKernelGGL(convT_pack_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, jobs, njobs,
                     dgrad);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
