// Weight gradient of the 3x3 / pad 1 convolution on f32 MFMA (autograd of nn.Conv2d w.r.t. its
// weight at PMU/model/unet/unet_parts.py:15,18 and PMU/model/probabilistic_unet/probabilistic_unet.py:38,43).
//
//   dw[co][ci][kh][kw] = sum_{n,h,w} dz[n,h,w,co] * act[n, h+kh-1, w+kw-1, ci]
//
// GEMM view: M = Cout (64 per block), N = Cin (64 per block), 9 taps, K = pixels, split over
// blocks (split-K); each block writes an fp32 slab ws[split][tap][co][ci] and wgrad_reduce sums
// the slabs in a fixed order (bitwise reproducible, no float atomics).
//
// Block: 12 waves = 4 (co frag, ci frag) pairs x 3 kernel rows (kh); each wave keeps only the 3
// accumulators of its row (48 VGPRs), so the block can keep a whole tile of global loads in flight.
// Per K tile (64 output pixels, TH x TW) the block stages dz[64 px][64 co] (BN+ReLU backward applied
// on the fly) and the (TH+2) x (TW+2) halo of the BN+ReLU(+max-pool)(+concat) activation into a
// double-buffered LDS ring: the next tile's global loads are issued before the current tile's MFMAs
// and transformed/stored after them (1 block per CU, 88 KB LDS).
#include "pmu_stage.h"

namespace {

constexpr int WB = 64;        // co and ci per block
constexpr int WPIX = 64;      // pixels per K tile
constexpr int MAX_HPX = 108;  // (4+2)*(16+2) = 108, (8+2)*(8+2) = 100
constexpr int WLS = 64;       // LDS row stride (b32 reads, lanes consecutive)
constexpr int SLOT = WPIX * WLS + MAX_HPX * WLS;
constexpr int NT = 768;       // threads per block
constexpr int ND = 2;         // dz items per thread: ceil(64*16 / 768)
constexpr int NX = 3;         // halo items per thread: ceil(108*16 / 768)

struct WgArgs {
  DevFrame dz, act;
  float* ws;
  int Cout, Cin;
  int twl, tiles_w, tiles_h, ntiles, nsplit;
};

// in-flight raw loads of one tile for this thread
struct TileRegs {
  float4 d[ND], dz[ND];
  float4 x[NX][4];
  bool dok[ND], xok[NX];
  unsigned xem[NX];  // avg pool (ceil): window elements present
};

// fast-path descriptor: the block's 64 dz channels and 64 act channels each lie in one source
struct FastOps {
  DevSrc ds, xs;
  int dc, xc;  // this thread's channel quad inside each source
};

template <bool RAW>
__device__ __forceinline__ void tile_load(const FastOps& f, int n, int h0, int w0, int twl, int HW2, int HP, int tid,
                                          TileRegs& r) {
  const int TW = 1 << twl;
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int it = tid + NT * i;
    const int px = it >> 4;
    const int h = h0 + (px >> twl), w = w0 + (px & (TW - 1));
    r.dok[i] = it < WPIX * 16 && h < f.ds.H && w < f.ds.W;
    const long long idx = r.dok[i] ? (((long long)n * f.ds.H + h) * f.ds.W + w) * f.ds.C + f.dc : (long long)f.dc;
    r.d[i] = *reinterpret_cast<const float4*>(f.ds.x + idx);
    if constexpr (!RAW) r.dz[i] = *reinterpret_cast<const float4*>(f.ds.z + idx);
  }
  const DevSrc& s = f.xs;
  const bool mp = !RAW && s.pool == PMU_POOL_MAX2, ap = !RAW && s.pool == PMU_POOL_AVG2CEIL;
  const long long rs = (long long)s.W * s.C;
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int it = tid + NT * i;
    const int hp = it >> 4;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    int hs = h0 - 1 + hr - s.off_h, ws = w0 - 1 + hc - s.off_w;
    if (mp || ap) { hs *= 2; ws *= 2; }
    const int lh = mp ? s.H - 1 : s.H, lw = mp ? s.W - 1 : s.W;
    r.xok[i] = it < HP * 16 && hs >= 0 && ws >= 0 && hs < lh && ws < lw;
    const long long idx = r.xok[i] ? (((long long)n * s.H + hs) * s.W + ws) * s.C + f.xc : (long long)f.xc;
    r.x[i][0] = *reinterpret_cast<const float4*>(s.x + idx);
    if (mp) {
      r.x[i][1] = *reinterpret_cast<const float4*>(s.x + idx + s.C);
      r.x[i][2] = *reinterpret_cast<const float4*>(s.x + idx + rs);
      r.x[i][3] = *reinterpret_cast<const float4*>(s.x + idx + rs + s.C);
    }
    if (ap) {
      const bool e01 = r.xok[i] && ws + 1 < s.W, e10 = r.xok[i] && hs + 1 < s.H;
      r.xem[i] = (e01 ? 1u : 0u) | (e10 ? 2u : 0u) | ((e01 && e10) ? 4u : 0u);
      r.x[i][1] = *reinterpret_cast<const float4*>(s.x + idx + (e01 ? s.C : 0));
      r.x[i][2] = *reinterpret_cast<const float4*>(s.x + idx + (e10 ? rs : 0));
      r.x[i][3] = *reinterpret_cast<const float4*>(s.x + idx + ((e01 && e10) ? rs + s.C : 0));
    }
  }
}

template <bool RAW>
__device__ __forceinline__ void tile_store(const FastOps& f, const TileRegs& r, int HP, int tid, float* slot) {
  float* Ds = slot;
  float* Xs = slot + WPIX * WLS;
  const int cq = tid & 15;
  if constexpr (RAW) {  // both operands already materialised (teed by the fwd / dgrad kernels)
#pragma unroll
    for (int i = 0; i < ND; ++i) {
      const int it = tid + NT * i;
      if (it >= WPIX * 16) continue;
      float4 v = r.d[i];
      if (!r.dok[i]) v = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(Ds + (it >> 4) * WLS + 4 * cq) = v;
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int it = tid + NT * i;
      if (it >= HP * 16) continue;
      float4 v = r.x[i][0];
      if (!r.xok[i]) v = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(Xs + (it >> 4) * WLS + 4 * cq) = v;
    }
    return;
  }
  // coefficients re-read per tile (L1/L2 hits) rather than held in 28 VGPRs across the MFMA loop
  const float* dco = f.ds.coef + f.dc;
  const int dC = f.ds.C;
  const float4 dsc = *reinterpret_cast<const float4*>(dco), dsh = *reinterpret_cast<const float4*>(dco + dC);
  const float4 dmu = *reinterpret_cast<const float4*>(dco + 2 * dC), dkx = *reinterpret_cast<const float4*>(dco + 3 * dC);
  const float4 dkc = *reinterpret_cast<const float4*>(dco + 4 * dC);
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    const int it = tid + NT * i;
    if (it >= WPIX * 16) continue;
    const float4 d = r.d[i], z = r.dz[i];
    float4 v = make_float4(pmu_bnbwd1(d.x, z.x, dsc.x, dsh.x, dmu.x, dkx.x, dkc.x),
                           pmu_bnbwd1(d.y, z.y, dsc.y, dsh.y, dmu.y, dkx.y, dkc.y),
                           pmu_bnbwd1(d.z, z.z, dsc.z, dsh.z, dmu.z, dkx.z, dkc.z),
                           pmu_bnbwd1(d.w, z.w, dsc.w, dsh.w, dmu.w, dkx.w, dkc.w));
    if (!r.dok[i]) v = make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(Ds + (it >> 4) * WLS + 4 * cq) = v;
  }
  const bool mp = f.xs.pool == PMU_POOL_MAX2, ap = f.xs.pool == PMU_POOL_AVG2CEIL;
  const bool raw = f.xs.mode == PMU_SRC_RAW;
  float4 xsc = make_float4(0.f, 0.f, 0.f, 0.f), xsh = xsc;
  if (!raw) {
    xsc = *reinterpret_cast<const float4*>(f.xs.coef + f.xc);
    xsh = *reinterpret_cast<const float4*>(f.xs.coef + f.xs.C + f.xc);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int it = tid + NT * i;
    if (it >= HP * 16) continue;
    float4 v;
    if (raw) {
      v = r.x[i][0];
    } else {
      v = pmu_bnrelu4(r.x[i][0], xsc, xsh);
      if (mp) {
        v = pmu_max4(v, pmu_bnrelu4(r.x[i][1], xsc, xsh));
        v = pmu_max4(v, pmu_bnrelu4(r.x[i][2], xsc, xsh));
        v = pmu_max4(v, pmu_bnrelu4(r.x[i][3], xsc, xsh));
      }
      if (ap) v = pmu_avg4(v, r.x[i], r.xem[i], xsc, xsh);
    }
    if (!r.xok[i]) v = make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(Xs + (it >> 4) * WLS + 4 * cq) = v;
  }
}

// generic synchronous staging (mixed-source blocks, avg pool, channel counts not multiple of 4)
__device__ __forceinline__ void tile_stage_generic(const DevFrame& D, const DevFrame& X, int n, int h0, int w0, int twl, int HW2,
                                   int HP, int co0, int ci0, int tid, float* slot) {
  float* Ds = slot;
  float* Xs = slot + WPIX * WLS;
  const int TW = 1 << twl;
  for (int it = tid; it < WPIX * 16; it += NT) {
    const int px = it >> 4, cq = it & 15;
    *reinterpret_cast<float4*>(Ds + px * WLS + 4 * cq) =
        frame_value4(D, n, h0 + (px >> twl), w0 + (px & (TW - 1)), co0 + 4 * cq);
  }
  for (int it = tid; it < HP * 16; it += NT) {
    const int hp = it >> 4, cq = it & 15;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    *reinterpret_cast<float4*>(Xs + hp * WLS + 4 * cq) = frame_value4(X, n, h0 - 1 + hr, w0 - 1 + hc, ci0 + 4 * cq);
  }
}

// MODE 1 (fast): every block's 64 dz channels / 64 act channels lie in one source each (host-checked);
// MODE 2 (raw): additionally both frames are single RAW sources (the operands the conv kernels teed);
// MODE 0 stages synchronously through frame_value4.
// TWL = log2 of the pixel-tile width (compile-time: with the K loop fully unrolled every LDS
// operand address is the wave's base plus an immediate offset, no per-step VALU).
template <int MODE, int TWL>
__global__ __launch_bounds__(NT, 3) void wgrad3x3_kernel(WgArgs a) {
  constexpr bool FAST = MODE > 0, RAW = MODE == 2;
  __shared__ __attribute__((aligned(16))) float smem[2 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int TW = 1 << TWL, TH = WPIX >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  const int nco = pmu_cdiv_dev(a.Cout, WB);
  const int co0 = (blockIdx.x % nco) * WB, ci0 = (blockIdx.x / nco) * WB;
  const int split = blockIdx.y;
  const int pair = wave & 3, kh = wave >> 2;
  const int cof = pair >> 1, cif = pair & 1;
  const DevFrame& D = a.dz;
  const DevFrame& X = a.act;

  // fast path if both 64-channel blocks sit inside one source each
  const bool x_in0 = ci0 + WB <= X.C0;
  const DevSrc& xsrc = x_in0 ? X.s0 : X.s1;
  FastOps f;
  if constexpr (FAST) {
    const int cq = tid & 15;
    f.ds = D.s0;
    f.dc = co0 + 4 * cq;
    f.xs = xsrc;
    f.xc = (x_in0 ? ci0 : ci0 - X.C0) + 4 * cq;
  }

  f32x16 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);
  auto origin = [&](int tile, int& n, int& h0, int& w0) {
    int t = tile;
    const int tw = t % a.tiles_w; t /= a.tiles_w;
    const int th = t % a.tiles_h; t /= a.tiles_h;
    n = t; h0 = th * TH; w0 = tw * TW;
  };

  TileRegs regs;
  {
    int n, h0, w0;
    origin(t_beg, n, h0, w0);
    if constexpr (FAST) {
      tile_load<RAW>(f, n, h0, w0, TWL, HW2, HP, tid, regs);
      tile_store<RAW>(f, regs, HP, tid, smem);
    } else {
      tile_stage_generic(D, X, n, h0, w0, TWL, HW2, HP, co0, ci0, tid, smem);
    }
  }
  __syncthreads();

  for (int tile = t_beg; tile < t_end; ++tile) {
    const int cur = (tile - t_beg) & 1;
    const bool more = tile + 1 < t_end;
    int nn = 0, nh0 = 0, nw0 = 0;
    if (more) {
      origin(tile + 1, nn, nh0, nw0);
      if constexpr (FAST) tile_load<RAW>(f, nn, nh0, nw0, TWL, HW2, HP, tid, regs);  // in flight during the MFMAs
    }
    const float* Ds = smem + cur * SLOT;
    const float* Xs = Ds + WPIX * WLS;
    // lane half h takes pixels 2ks+h; TW is even, so both halves of a step share the row
    const int h = lane >> 5;
    const float* da = Ds + h * WLS + cof * 32 + (lane & 31);
    const float* xa = Xs + (kh * HW2 + h) * WLS + cif * 32 + (lane & 31);
#pragma unroll 8
    for (int ks = 0; ks < WPIX / 2; ++ks) {
      const int px0 = 2 * ks;  // constant within an unrolled group: immediate LDS offsets
      const int r = px0 >> TWL, c = px0 & (TW - 1);
      const float av = da[px0 * WLS];
      const float* xb = xa + (r * HW2 + c) * WLS;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) acc[kw] = mfma_f32_32x32x2(av, xb[kw * WLS], acc[kw]);
    }
    if (more) {
      float* nxt = smem + (cur ^ 1) * SLOT;
      if constexpr (FAST) tile_store<RAW>(f, regs, HP, tid, nxt);
      else tile_stage_generic(D, X, nn, nh0, nw0, TWL, HW2, HP, co0, ci0, tid, nxt);
    }
    __syncthreads();
  }

  // slab write: ws[split][tap][co][ci]
  const int ci = ci0 + cif * 32 + (lane & 31);
  if (ci < a.Cin) {
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int tap = kh * 3 + kw;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + cof * 32 + acc_row(r, lane);
        if (co < a.Cout) a.ws[(((long long)split * 9 + tap) * a.Cout + co) * a.Cin + ci] = acc[kw][r];
      }
    }
  }
}


static void wgrad_geometry(int N, int H, int W, int Cin, int Cout, int* twl, int* tiles_w, int* tiles_h,
                           int* ntiles, int* nsplit) {
  *twl = (W > 8) ? 4 : 3;
  const int TW = 1 << *twl, TH = WPIX / TW;
  *tiles_w = pmu_cdiv(W, TW);
  *tiles_h = pmu_cdiv(H, TH);
  *ntiles = N * *tiles_w * *tiles_h;
  const int blocks_mn = pmu_cdiv(Cout, WB) * pmu_cdiv(Cin, WB);
  int s = 512 / blocks_mn;  // ~2 blocks per CU over the launch
  if (s < 1) s = 1;
  if (s > *ntiles) s = *ntiles;
  *nsplit = s;
}

}  // namespace

extern "C" size_t pmu_conv3x3_wgrad_ws(int N, int H, int W, int Cin, int Cout) {
  int twl, tw, th, nt, ns;
  wgrad_geometry(N, H, W, Cin, Cout, &twl, &tw, &th, &nt, &ns);
  return (size_t)ns * 9 * Cout * Cin * sizeof(float);
}

extern "C" int pmu_conv3x3_wgrad(const pmu_frame* dz, const pmu_frame* act, int Cout, float* dw, float* ws,
                                 size_t ws_bytes, void* stream) {
  PMU_REQUIRE(valid_frame(dz) && valid_frame(act) && dw && ws);
  PMU_REQUIRE(dz->N == act->N && dz->H == act->H && dz->W == act->W);
  const int Cin = act->src[0].C + (act->nsrc > 1 ? act->src[1].C : 0);
  PMU_REQUIRE(dz->nsrc == 1 && dz->src[0].C == Cout);
  WgArgs a;
  a.dz = make_dev_frame(dz);
  a.act = make_dev_frame(act);
  a.ws = ws; a.Cout = Cout; a.Cin = Cin;
  wgrad_geometry(dz->N, dz->H, dz->W, Cin, Cout, &a.twl, &a.tiles_w, &a.tiles_h, &a.ntiles, &a.nsplit);
  PMU_REQUIRE(ws_bytes >= (size_t)a.nsplit * 9 * Cout * Cin * sizeof(float));
  dim3 grid((unsigned)(pmu_cdiv(Cout, WB) * pmu_cdiv(Cin, WB)), (unsigned)a.nsplit);
  // fast kernel only if every (co block, ci block) lies inside one source of each frame
  const pmu_src& d0 = dz->src[0];
  bool fast = a.dz.vec && d0.mode == PMU_SRC_BNBWD && d0.pool == PMU_POOL_NONE && Cout % WB == 0;
  fast = fast && a.act.vec && (a.act.C0 % WB == 0) && (Cin % WB == 0);
  for (int i = 0; i < act->nsrc; ++i) {
    const pmu_src& s = act->src[i];
    fast = fast && s.mode != PMU_SRC_BNBWD && (s.pool == PMU_POOL_NONE || s.mode == PMU_SRC_BNRELU);
  }
  const bool raw = a.dz.vec && d0.mode == PMU_SRC_RAW && d0.pool == PMU_POOL_NONE && Cout % WB == 0 &&
                   a.act.vec && act->nsrc == 1 && act->src[0].mode == PMU_SRC_RAW &&
                   act->src[0].pool == PMU_POOL_NONE && Cin % WB == 0;
  const int mode = raw ? 2 : fast ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
#define PMU_WG_LAUNCH(M, T) hipLaunchKernelGGL((wgrad3x3_kernel<M, T>), grid, dim3(NT), 0, st, a)
  if (a.twl == 4) {
    if (mode == 2) PMU_WG_LAUNCH(2, 4); else if (mode == 1) PMU_WG_LAUNCH(1, 4); else PMU_WG_LAUNCH(0, 4);
  } else {
    if (mode == 2) PMU_WG_LAUNCH(2, 3); else if (mode == 1) PMU_WG_LAUNCH(1, 3); else PMU_WG_LAUNCH(0, 3);
  }
#undef PMU_WG_LAUNCH
  PMU_CHECK_LAUNCH();
  const long long E = 9LL * Cout * Cin;
  hipLaunchKernelGGL(pmu_splitk_reduce9_kernel, dim3((unsigned)pmu_cdiv(E, 64)), dim3(256), 0, st, (const float*)ws,
                     a.nsplit, (long long)Cout * Cin, dw);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
