// Weight gradient of the 3x3 / pad 1 convolution on bf16 MFMA (config c5): autograd of nn.Conv2d
// w.r.t. its weight (PMU/model/unet/unet_parts.py:15,18; PMU/model/probabilistic_unet/probabilistic_unet.py:38,43)
// with torch.autocast(bfloat16) arithmetic: bf16 operands, fp32 sums, fp32 dw.
//
//   dw[co][ci][kh][kw] = sum_{n,h,w} dzt[n,h,w,co] * xt[n, h+kh-1, w+kw-1, ci]
//
// dzt / xt are the bf16 operands materialised once (pmu_frame_to_bf16: the BN+ReLU backward of dz,
// the BN+ReLU(+pool)(+concat) activation), NHWC with channels padded to a multiple of 8.
// GEMM view: M = Cout (WCO per block), N = Cin (64 per block), K = pixels split over blocks.
// The K dimension sits on MFMA register elements (8 consecutive pixels per lane half), so both
// operands are read from channel-contiguous LDS rows with ds_read_b64_tr_b16: a 16-lane group
// reads 4 pixel rows x 16 channels and receives them column-major, every lane supplying its own
// row address — the 3x3 tap shift is just a different row address, no im2col, no transposed copy.
// Block: 12 waves = (WCO/32/FCO co groups) x 2 ci fragments x 3 kernel rows; each wave keeps
// FCO x 3 (kw) accumulators.  Pixel tiles of 64 (TH x TW) are double-buffered in LDS with the next
// tile's global loads in flight during the current tile's MFMAs.  Split-K slabs
// ws[split][tap][co][ci] are summed in a fixed order (bitwise reproducible, no float atomics).
#include "pmu_stage.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int WCI = 64;     // ci per block
constexpr int NT = 768;     // 12 waves
// pixels per K tile: 128 for 64-channel blocks (the 512^2 / 64-channel shapes are load-latency-bound
// per tile: 0.49 -> 0.42 ms at 64 -> 64, 0.79 -> 0.70 ms at 128 -> 64), 64 for 128-channel blocks
// (at 128 they spill past the 3-waves-per-SIMD register cap and lose 15%)
__host__ __device__ constexpr int wpix_of(int wco) { return wco == 64 ? 128 : 64; }
// the tile's halo image: (TH + 2) x (TW + 2) pixels, TW = 16 or 8
__host__ __device__ constexpr int hpx_of(int px) { return px == 128 ? 180 : 108; }
constexpr int XS = WCI + 32;  // X row stride (bf16): 192 B = 64 mod 256 -> tr reads conflict-free

struct WgbArgs {
  const unsigned short* dzt;
  const unsigned short* xt;
  float* ws;
  int N, H, W, Cout, Cin, Cop, Cip;
  int tiles_w, tiles_h, ntiles, nsplit;
};

template <int WCO>
struct Geo {
  static constexpr int WPIX = wpix_of(WCO);
  static constexpr int MAX_HPX = hpx_of(WPIX);
  static constexpr int DS = WCO + 32;                 // D row stride (bf16): 320 B / 192 B
  static constexpr int D_ELEMS = WPIX * DS;
  static constexpr int SLOT = D_ELEMS + MAX_HPX * XS;  // one ring slot (bf16 elements)
  static constexpr int DU = WPIX * WCO / 8;            // 16-B units of a D tile
  static constexpr int ND = (DU + NT - 1) / NT;
  static constexpr int NX = (MAX_HPX * WCI / 8 + NT - 1) / NT;
  static_assert(2 * SLOT * 2 <= 160 * 1024, "two ring slots in LDS");
  static constexpr int FCO = WCO / 64;                 // co fragments per wave (12 waves)
};

// component-wise select (a select of whole uint4 values is lowered through scratch)
__device__ __forceinline__ uint4 keep_if(bool ok, uint4 v) {
  return make_uint4(ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u);
}
__device__ __forceinline__ s16x4 tr_read(const unsigned short* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
__device__ __forceinline__ bf16x8 frag_of(s16x4 lo, s16x4 hi) {
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// The next K tile rides in registers under the MFMAs.  Out-of-range units are zeroed when they are
// STORED (okd / okx bit masks): zeroing them at load time made the compiler wait for the loads
// right there (vmcnt before the MFMAs), exposing the whole global-load latency every tile.
template <int WCO, int TWL>
struct TileIO {
  uint4 d[Geo<WCO>::ND], x[Geo<WCO>::NX];
  unsigned okd, okx;
};

template <int WCO, int TWL>
__device__ __forceinline__ void tile_load(const WgbArgs& a, int tile, int co0, int ci0, int tid, TileIO<WCO, TWL>& r) {
  using G = Geo<WCO>;
  constexpr int TW = 1 << TWL, TH = G::WPIX >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  int t = tile;
  const int tw = t % a.tiles_w; t /= a.tiles_w;
  const int th = t % a.tiles_h; t /= a.tiles_h;
  const int n = t, h0 = th * TH, w0 = tw * TW;
  PMU_DCHECK(n < a.N, PMU_DBG_GRID);
  r.okd = 0u;
  r.okx = 0u;
#pragma unroll
  for (int i = 0; i < G::ND; ++i) {
    const int u = tid + NT * i;
    const int px = u / (WCO / 8), cu = u % (WCO / 8);
    const int h = h0 + (px >> TWL), w = w0 + (px & (TW - 1));
    const int c = co0 + 8 * cu;
    const bool ok = (G::DU % NT == 0 || u < G::DU) && h < a.H && w < a.W && c < a.Cop;
    const long long idx = ok ? (((long long)n * a.H + h) * a.W + w) * a.Cop + c : 0;
    r.d[i] = *reinterpret_cast<const uint4*>(a.dzt + idx);
    r.okd |= ok ? (1u << i) : 0u;
  }
#pragma unroll
  for (int i = 0; i < G::NX; ++i) {
    const int u = tid + NT * i;
    const int hp = u / (WCI / 8), cu = u % (WCI / 8);
    const int hr = hp / HW2, hc = hp - hr * HW2;
    const int h = h0 - 1 + hr, w = w0 - 1 + hc;
    const int c = ci0 + 8 * cu;
    const bool ok = u < HP * (WCI / 8) && h >= 0 && w >= 0 && h < a.H && w < a.W && c < a.Cip;
    const long long idx = ok ? (((long long)n * a.H + h) * a.W + w) * a.Cip + c : 0;
    r.x[i] = *reinterpret_cast<const uint4*>(a.xt + idx);
    r.okx |= ok ? (1u << i) : 0u;
  }
}

template <int WCO, int TWL>
__device__ __forceinline__ void tile_store(const TileIO<WCO, TWL>& r, int tid, unsigned short* slot) {
  using G = Geo<WCO>;
  constexpr int TW = 1 << TWL, TH = G::WPIX >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
  unsigned short* Ds = slot;
  unsigned short* Xs = slot + G::D_ELEMS;
#pragma unroll
  for (int i = 0; i < G::ND; ++i) {
    const int u = tid + NT * i;
    if (G::DU % NT != 0 && u >= G::DU) continue;
    const int px = u / (WCO / 8), cu = u % (WCO / 8);
    *reinterpret_cast<uint4*>(Ds + px * G::DS + 8 * cu) = keep_if((r.okd >> i) & 1u, r.d[i]);
  }
#pragma unroll
  for (int i = 0; i < G::NX; ++i) {
    const int u = tid + NT * i;
    if (u >= HP * (WCI / 8)) continue;
    const int hp = u / (WCI / 8), cu = u % (WCI / 8);
    *reinterpret_cast<uint4*>(Xs + hp * XS + 8 * cu) = keep_if((r.okx >> i) & 1u, r.x[i]);
  }
}

template <int WCO, int TWL>
__global__ __launch_bounds__(NT, 3) void wgrad3x3_bf16_kernel(WgbArgs a) {
  using G = Geo<WCO>;
  constexpr int TW = 1 << TWL, HW2 = TW + 2;
  constexpr int FCO = G::FCO > 0 ? G::FCO : 1;
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * G::SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nco = pmu_cdiv_dev(a.Cout, WCO);
  // (channel block, split) in XCD order, channel blocks fastest: the blocks of one split walk the same
  // pixel tiles in step on one XCD, so its L2 serves each tile to all of them (in launch order they
  // sat on different XCDs and each fetched every tile from HBM)
  const int nblk = gridDim.x;
  const int lbk = pmu_xcd_block(blockIdx.y * nblk + blockIdx.x, nblk * gridDim.y);
  const int blk = lbk % nblk;
  const int co0 = (blk % nco) * WCO, ci0 = (blk / nco) * WCI;
  const int split = lbk / nblk;
  // wave -> (co group, ci fragment, kernel row)
  const int kh = wave % 3, cif = (wave / 3) & 1, cog = wave / 6;  // cog < 2
  // WCO = 64: 2 co groups of one fragment; WCO = 128: 2 co groups of two fragments
  const int cbase = cog * 32 * FCO;

  f32x16 acc[FCO][3];
#pragma unroll
  for (int f = 0; f < FCO; ++f)
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][t][r] = 0.f;

  const int t_beg = (int)(((long long)a.ntiles * split) / a.nsplit);
  const int t_end = (int)(((long long)a.ntiles * (split + 1)) / a.nsplit);

  // transposed-read lane roles: half h takes pixels 8h..8h+7 of a 16-pixel k-step, group g the
  // column block 16g, lane 4q+p supplies row q (pixel 4t+q of the half) and columns 4p..4p+3
  const int h = lane >> 5, g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
  const int dcol = cbase + 16 * g + 4 * p;
  const int xcol = cif * 32 + 16 * g + 4 * p;

  TileIO<WCO, TWL> io;
  if (t_beg < t_end) {
    tile_load<WCO, TWL>(a, t_beg, co0, ci0, tid, io);
    tile_store<WCO, TWL>(io, tid, smem);
  }
  __syncthreads();

  for (int tile = t_beg; tile < t_end; ++tile) {
    const int cur = (tile - t_beg) & 1;
    const bool more = tile + 1 < t_end;
    if (more) tile_load<WCO, TWL>(a, tile + 1, co0, ci0, tid, io);  // in flight during the MFMAs
    const unsigned short* Ds = smem + cur * G::SLOT;
    const unsigned short* Xs = Ds + G::D_ELEMS;
#pragma unroll
    for (int ks = 0; ks < G::WPIX / 16; ++ks) {
      bf16x8 af[FCO], bf[3];
      s16x4 lo, hi;
      // pixel rows of this lane's two reads: 16ks + 8h + 4t + q, t = 0, 1 (same tile row: TW >= 8)
      const int pk0 = 16 * ks + 8 * h + q, pk1 = pk0 + 4;
#pragma unroll
      for (int f = 0; f < FCO; ++f) {
        lo = tr_read(Ds + pk0 * G::DS + dcol + 32 * f);
        hi = tr_read(Ds + pk1 * G::DS + dcol + 32 * f);
        af[f] = frag_of(lo, hi);
      }
      const int r0 = pk0 >> TWL, c0 = pk0 & (TW - 1), r1 = pk1 >> TWL, c1 = pk1 & (TW - 1);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        lo = tr_read(Xs + ((r0 + kh) * HW2 + c0 + kw) * XS + xcol);
        hi = tr_read(Xs + ((r1 + kh) * HW2 + c1 + kw) * XS + xcol);
        bf[kw] = frag_of(lo, hi);
      }
#pragma unroll
      for (int f = 0; f < FCO; ++f)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          acc[f][kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[f], bf[kw], acc[f][kw], 0, 0, 0);
    }
    if (more) tile_store<WCO, TWL>(io, tid, smem + (cur ^ 1) * G::SLOT);
    __syncthreads();
  }

  // slab write: ws[split][tap][co][ci]; D rows = co (A rows), columns = ci (lanes)
  const int ci = ci0 + cif * 32 + (lane & 31);
  if (ci < a.Cin) {
#pragma unroll
    for (int f = 0; f < FCO; ++f)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + cbase + 32 * f + acc_row(r, lane);
          PMU_DCHECK(split < a.nsplit && ci < a.Cin, PMU_DBG_WORKSPACE);
          if (co < a.Cout) a.ws[(((long long)split * 9 + tap) * a.Cout + co) * a.Cin + ci] = acc[f][kw][r];
        }
      }
  }
}


// operand materialisation: out[p][c] = bf16(frame value), channels [C, Cpad) zero
__global__ __launch_bounds__(256) void frame_to_bf16_kernel(DevFrame f, int Cpad, unsigned short* __restrict__ out) {
  const int nq = Cpad / 4;
  const long long total = (long long)f.N * f.H * f.W * nq;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int cq = (int)(e % nq);
    long long pix = e / nq;
    const int w = (int)(pix % f.W);
    long long t = pix / f.W;
    const int h = (int)(t % f.H);
    const int n = (int)(t / f.H);
    const float4 v = frame_value4(f, n, h, w, 4 * cq);
    *reinterpret_cast<uint2*>(out + pix * Cpad + 4 * cq) = make_uint2(pmu_pk_bf16(v.x, v.y), pmu_pk_bf16(v.z, v.w));
  }
}

// Fast path: one 16-B unit (8 channels) per thread, 32-bit pixel decode; every source's channel
// count is a multiple of 8 (a unit never straddles the concat) and the output has < 2^31 units.
// (ldo: output pixel stride in elements, >= Cpad — a wider tensor's first Cpad channels)
__global__ __launch_bounds__(256) void frame_to_bf16_fast_kernel(DevFrame f, int Cpad, unsigned total,
                                                                 unsigned short* __restrict__ out, int ldo) {
  const unsigned nu = (unsigned)Cpad / 8u, Wu = (unsigned)f.W, Hu = (unsigned)f.H;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const unsigned pix = e / nu, cu = e - pix * nu;
    const unsigned t = pix / Wu, w = pix - t * Wu;
    const unsigned n = t / Hu, h = t - n * Hu;
    const int c = 8 * (int)cu;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (c < f.C) {
      const bool second = f.nsrc > 1 && c >= f.C0;
      const DevSrc& s = second ? f.s1 : f.s0;
      const int cs = c - (second ? f.C0 : 0);
      const int hs = (int)h - s.off_h, ws = (int)w - s.off_w;
      a = src_value4(s, (int)n, hs, ws, cs);
      b = src_value4(s, (int)n, hs, ws, cs + 4);
    }
    *reinterpret_cast<uint4*>(out + (size_t)pix * ldo + c) =
        make_uint4(pmu_pk_bf16(a.x, a.y), pmu_pk_bf16(a.z, a.w), pmu_pk_bf16(b.x, b.y), pmu_pk_bf16(b.z, b.w));
  }
}

// operand materialisation in fp32: out[p][c] = frame value (e.g. a max-pooled BN+ReLU activation,
// consumed as a RAW source so the conv kernels need no pooled staging variant)
__global__ __launch_bounds__(256) void frame_to_f32_kernel(DevFrame f, float* __restrict__ out) {
  const int nq = (f.C + 3) / 4;
  const long long total = (long long)f.N * f.H * f.W * nq;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int cq = (int)(e % nq);
    long long pix = e / nq;
    const int w = (int)(pix % f.W);
    long long t = pix / f.W;
    const int h = (int)(t % f.H);
    const int n = (int)(t / f.H);
    const float4 v = frame_value4(f, n, h, w, 4 * cq);
    float* o = out + pix * f.C + 4 * cq;
    if (f.C % 4 == 0) {
      *reinterpret_cast<float4*>(o) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int k = 0; k < 4 && 4 * cq + k < f.C; ++k) o[k] = vv[k];
    }
  }
}

// Fast path of the fp32 materialisation: one float4 (4 channels) per thread, 32-bit pixel decode;
// every source's channel count is a multiple of 4 and the output has < 2^31 units.
__global__ __launch_bounds__(256) void frame_to_f32_fast_kernel(DevFrame f, unsigned total, float* __restrict__ out,
                                                                int ldo) {
  const unsigned nu = (unsigned)f.C / 4u, Wu = (unsigned)f.W, Hu = (unsigned)f.H;
  for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const unsigned pix = e / nu, cu = e - pix * nu;
    const unsigned t = pix / Wu, w = pix - t * Wu;
    const unsigned n = t / Hu, h = t - n * Hu;
    const int c = 4 * (int)cu;
    const bool second = f.nsrc > 1 && c >= f.C0;
    const DevSrc& s = second ? f.s1 : f.s0;
    const int cs = c - (second ? f.C0 : 0);
    *reinterpret_cast<float4*>(out + (size_t)pix * ldo + c) =
        src_value4(s, (int)n, (int)h - s.off_h, (int)w - s.off_w, cs);
  }
}

// ---- streaming materialisation ------------------------------------------------------------
// The frame_to_* passes are HBM-bound (c5: 38 per step, 19% of its kernel time; c2: 34, 7%).  The
// generic kernels above take one 8-channel unit per thread per step, re-load the unit's BN
// coefficients every step, and (vmcnt counts loads and stores in order) wait for a step's stores
// before the next step's loads can be consumed: 4.8-5.2 TB/s, 3.3-3.8 TB/s max-pooled.  This path
// takes the common frames — one fp32 source, no offset, C = Cpad a multiple of 8 with C / 8 a power
// of two up to 256 (every UNet width) — with a thread owning one channel unit for the whole launch
// (coefficients loaded once) and U pixels per step, the next step's loads issued before this step's
// stores.  Same per-element arithmetic as src_xform4 / src_value4: bit-identical output.  Measured
// (profiles/r03/kbench_frame_c5.txt): max-pooled 3.7-4.0 -> 5.2-6.6 TB/s; the flat passes over
// the 512^2 / 256^2 maps gain only from the nontemporal policy below (about 5.0 -> 5.5 TB/s).
struct StreamArgs {
  const float* x;
  const float* z;
  const float* coef;
  void* out;
  int C, lg;         // channels; log2(C / 8)
  int H, W, SH, SW;  // frame H x W; source SH x SW (POOL: the 2x2 windows' map, floor mode)
  unsigned P;        // frame pixels N * H * W
  int ldo;           // output pixel stride in elements
  void* out2;        // SKIP: the unpooled values (each 2x2 window's four), pixel stride ldo2
  int ldo2;
};

// XB (BNBWD only): x (the activation gradient da) stored as bf16 — one 16-B load of its 8 channels
// (xb), converted when the step is stored; v[0], v[1] then hold z
template <int MODE, bool POOL, bool XB = false>
struct StreamLd {
  static constexpr int NV = POOL ? 8 : (MODE == PMU_SRC_BNBWD ? (XB ? 2 : 4) : 2);
  float4 v[NV];
  uint4 xb;
};

typedef float stream_f4 __attribute__((ext_vector_type(4)));
typedef unsigned stream_u4 __attribute__((ext_vector_type(4)));
template <int NT>
__device__ __forceinline__ float4 stream_ld4(const float* p) {
  if (NT & 1) {
    const stream_f4 v = __builtin_nontemporal_load(reinterpret_cast<const stream_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  return pmu_ld4(p);
}

template <int MODE, bool POOL, int NT, bool XB = false>
__device__ __forceinline__ void stream_load(const StreamArgs& a, unsigned p, int c, StreamLd<MODE, POOL, XB>& d) {
  if (XB) {  // (BNBWD, unpooled)
    const size_t o = (size_t)p * a.C + c;
    const uint4* xp = reinterpret_cast<const uint4*>(reinterpret_cast<const unsigned short*>(a.x) + o);
    if (NT & 1) {
      const stream_u4 v = __builtin_nontemporal_load(reinterpret_cast<const stream_u4*>(xp));
      d.xb = make_uint4(v.x, v.y, v.z, v.w);
    } else {
      d.xb = *xp;
    }
    d.v[0] = stream_ld4<NT>(a.z + o);
    d.v[1] = stream_ld4<NT>(a.z + o + 4);
  } else if (!POOL) {
    const size_t o = (size_t)p * a.C + c;
    d.v[0] = stream_ld4<NT>(a.x + o);
    d.v[1] = stream_ld4<NT>(a.x + o + 4);
    if constexpr (MODE == PMU_SRC_BNBWD) {
      d.v[2] = stream_ld4<NT>(a.z + o);
      d.v[3] = stream_ld4<NT>(a.z + o + 4);
    }
  } else {
    const unsigned t = p / (unsigned)a.W, w = p - t * (unsigned)a.W;
    const unsigned n = t / (unsigned)a.H, h = t - n * (unsigned)a.H;
    const size_t b = (((size_t)n * a.SH + 2 * h) * a.SW + 2 * w) * a.C + c;
    const size_t rs = (size_t)a.SW * a.C;
    const size_t o[4] = {b, b + a.C, b + rs, b + rs + a.C};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d.v[2 * k] = stream_ld4<NT>(a.x + o[k]);
      d.v[2 * k + 1] = stream_ld4<NT>(a.x + o[k] + 4);
    }
  }
}

__device__ __forceinline__ float4 bnrelu4(float4 x, float4 sc, float4 sh) {
  return make_float4(fmaxf(0.f, fmaf(x.x, sc.x, sh.x)), fmaxf(0.f, fmaf(x.y, sc.y, sh.y)),
                     fmaxf(0.f, fmaf(x.z, sc.z, sh.z)), fmaxf(0.f, fmaf(x.w, sc.w, sh.w)));
}
__device__ __forceinline__ float4 max4(float4 a, float4 t) {
  return make_float4(fmaxf(a.x, t.x), fmaxf(a.y, t.y), fmaxf(a.z, t.z), fmaxf(a.w, t.w));
}
__device__ __forceinline__ float bnbwd1(float x, float z, float sc, float sh, float mu, float kx, float kc) {
  return fmaf(sc, fmaf(z, sc, sh) > 0.f ? x : 0.f, fmaf(kx, z - mu, kc));
}
__device__ __forceinline__ float4 bnbwd4(float4 x, float4 z, float4 sc, float4 sh, float4 mu, float4 kx, float4 kc) {
  return make_float4(bnbwd1(x.x, z.x, sc.x, sh.x, mu.x, kx.x, kc.x), bnbwd1(x.y, z.y, sc.y, sh.y, mu.y, kx.y, kc.y),
                     bnbwd1(x.z, z.z, sc.z, sh.z, mu.z, kx.z, kc.z), bnbwd1(x.w, z.w, sc.w, sh.w, mu.w, kx.w, kc.w));
}

// 8 channels (r0, r1) at element offset e of a bf16 / fp32 NHWC tensor
template <bool BF, int NT>
__device__ __forceinline__ void stream_st8(void* out, size_t e, float4 r0, float4 r1) {
  if (BF) {
    uint4* o = reinterpret_cast<uint4*>(static_cast<unsigned short*>(out) + e);
    const uint4 v = make_uint4(pmu_pk_bf16(r0.x, r0.y), pmu_pk_bf16(r0.z, r0.w), pmu_pk_bf16(r1.x, r1.y),
                               pmu_pk_bf16(r1.z, r1.w));
    if (NT & 2) __builtin_nontemporal_store(stream_u4{v.x, v.y, v.z, v.w}, reinterpret_cast<stream_u4*>(o));
    else *o = v;
  } else {
    float4* o = reinterpret_cast<float4*>(static_cast<float*>(out) + e);
    if (NT & 2) {
      __builtin_nontemporal_store(stream_f4{r0.x, r0.y, r0.z, r0.w}, reinterpret_cast<stream_f4*>(o));
      __builtin_nontemporal_store(stream_f4{r1.x, r1.y, r1.z, r1.w}, reinterpret_cast<stream_f4*>(o + 1));
    } else {
      o[0] = r0;
      o[1] = r1;
    }
  }
}

// SKIP (POOL only, even source dims): the four values of each window also written unpooled to out2 —
// the skip half of the Up block's concat operand, made in the same pass as the max-pooled operand of
// the next level's first conv (one read of the activation instead of two)
template <int MODE, bool POOL, bool BF, int U, int NT, bool SKIP = false, bool XB = false>
__global__ __launch_bounds__(256) void frame_stream_kernel(StreamArgs a) {
  const int tid = threadIdx.x;
  const int c = 8 * (tid & ((1 << a.lg) - 1));
  const unsigned pb = 256u >> a.lg;  // pixels per U-slice of a block step
  // this thread's channel unit is fixed: its coefficients in registers for the whole launch
  float4 sc[2], sh[2], mu[2], kx[2], kc[2];
  if (MODE != PMU_SRC_RAW) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      sc[k] = pmu_ld4(a.coef + c + 4 * k);
      sh[k] = pmu_ld4(a.coef + a.C + c + 4 * k);
      if (MODE == PMU_SRC_BNBWD) {
        mu[k] = pmu_ld4(a.coef + 2 * a.C + c + 4 * k);
        kx[k] = pmu_ld4(a.coef + 3 * a.C + c + 4 * k);
        kc[k] = pmu_ld4(a.coef + 4 * a.C + c + 4 * k);
      }
    }
  }
  const unsigned span = pb * U, stride = span * gridDim.x;
  const unsigned pr = (unsigned)(tid >> a.lg), plast = a.P - 1;
  // Two register sets in ping-pong (a copy between them would wait for the loads it copies): the
  // loads of step s+1 are in flight while step s stores.  Loads are unconditional, the pixel clamped
  // to the last one (a load under a branch makes the compiler wait for every outstanding load before
  // the first store), and the loop runs on the block's uniform base.
  StreamLd<MODE, POOL, XB> A[U], B[U];
  auto load = [&](StreamLd<MODE, POOL, XB>* d, unsigned base) {
#pragma unroll
    for (int j = 0; j < U; ++j) stream_load<MODE, POOL, NT, XB>(a, min(base + pr + j * pb, plast), c, d[j]);
  };
  auto store = [&](const StreamLd<MODE, POOL, XB>* d, unsigned base) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      // past the end: the clamped pixel's own value rewritten to it (identical bytes), so the stores
      // are unconditional too and the compiler can count the loads still in flight at each store
      const unsigned p = min(base + pr + j * pb, plast);
      float4 r[2], tq[4][2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (POOL) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            tq[q][k] = d[j].v[2 * q + k];
            if (MODE == PMU_SRC_BNRELU) tq[q][k] = bnrelu4(tq[q][k], sc[k], sh[k]);
          }
          float4 m = tq[0][k];
#pragma unroll
          for (int q = 1; q < 4; ++q) m = max4(m, tq[q][k]);
          r[k] = m;
        } else if (MODE == PMU_SRC_BNRELU) {
          r[k] = bnrelu4(d[j].v[k], sc[k], sh[k]);
        } else if (MODE == PMU_SRC_BNBWD && XB) {
          const unsigned u0 = k ? d[j].xb.z : d[j].xb.x, u1 = k ? d[j].xb.w : d[j].xb.y;
          const float4 xv = make_float4(__uint_as_float(u0 << 16), __uint_as_float(u0 & 0xffff0000u),
                                        __uint_as_float(u1 << 16), __uint_as_float(u1 & 0xffff0000u));
          r[k] = bnbwd4(xv, d[j].v[k], sc[k], sh[k], mu[k], kx[k], kc[k]);
        } else if (MODE == PMU_SRC_BNBWD) {
          r[k] = bnbwd4(d[j].v[k], d[j].v[2 + k], sc[k], sh[k], mu[k], kx[k], kc[k]);
        } else {
          r[k] = d[j].v[k];
        }
      }
      stream_st8<BF, NT>(a.out, (size_t)p * a.ldo + c, r[0], r[1]);
      if constexpr (POOL && SKIP) {
        const unsigned t = p / (unsigned)a.W, w = p - t * (unsigned)a.W;
        const unsigned n = t / (unsigned)a.H, h = t - n * (unsigned)a.H;
        const size_t sp = ((size_t)n * a.SH + 2 * h) * a.SW + 2 * w;
        const size_t so[4] = {sp, sp + 1, sp + a.SW, sp + a.SW + 1};
#pragma unroll
        for (int q = 0; q < 4; ++q) stream_st8<BF, NT>(a.out2, so[q] * a.ldo2 + c, tq[q][0], tq[q][1]);
      }
    }
  };
  unsigned base = blockIdx.x * span;
  load(A, base);
  // (sched_barrier: keeps the scheduler from hoisting a step's arithmetic, which waits for its loads,
  // above the issue of the next step's loads)
  for (; base < a.P; base += 2 * stride) {
    load(B, base + stride);
    __builtin_amdgcn_sched_barrier(0);
    store(A, base);
    // no exit between the halves (a step past the end rewrites the last pixel): a mid-loop exit
    // shares the latch, and the compiler then waits at the loop head for loads that path left pending
    load(A, base + 2 * stride);
    __builtin_amdgcn_sched_barrier(0);
    store(B, base + stride);
  }
}

// A frame the streaming path takes (see above); PMU_FRAME_STREAM=0 forces the generic kernels (the
// tests compare the two).
static bool stream_ok(const pmu_frame* f, int Cout) {
  if (f->nsrc != 1) return false;
  const pmu_src& s = f->src[0];
  // (bf16 storage: only the activation gradient of an unpooled BN-backward source, the *_dxb dx)
  if (s.dtype != 0 && !(s.dtype == PMU_DT_X_BF16 && s.mode == PMU_SRC_BNBWD && s.pool == PMU_POOL_NONE)) return false;
  if (s.off_h != 0 || s.off_w != 0 || s.C != Cout || s.C % 8 != 0) return false;
  const int nu = s.C / 8;
  if (nu > 256 || (nu & (nu - 1)) != 0) return false;
  if (s.pool == PMU_POOL_AVG2CEIL || (s.pool == PMU_POOL_MAX2 && s.mode == PMU_SRC_BNBWD)) return false;
  if (s.pool == PMU_POOL_NONE && (s.H != f->H || s.W != f->W)) return false;
  if (s.pool == PMU_POOL_MAX2 && (s.H / 2 != f->H || s.W / 2 != f->W)) return false;
  if ((long long)f->N * f->H * f->W >= (1LL << 31)) return false;
  const char* e = getenv("PMU_FRAME_STREAM");
  return !(e && e[0] == '0');
}

template <bool BF, int NT, int U_POOL, int U_FLAT, int U_BWD>
static void launch_stream_nt(const pmu_src& s, dim3 grid, dim3 blk, hipStream_t st, const StreamArgs& a) {
  if (a.out2) {  // (pool_skip_ok: BNRELU, max-pooled)
    hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_BNRELU, true, BF, U_POOL, NT, true>), grid, blk, 0, st, a);
  } else if (s.pool == PMU_POOL_MAX2) {
    if (s.mode == PMU_SRC_BNRELU) hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_BNRELU, true, BF, U_POOL, NT>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_RAW, true, BF, U_POOL, NT>), grid, blk, 0, st, a);
  } else if (s.mode == PMU_SRC_BNRELU) {
    hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_BNRELU, false, BF, U_FLAT, NT>), grid, blk, 0, st, a);
  } else if (s.mode == PMU_SRC_BNBWD && s.dtype == PMU_DT_X_BF16) {
    hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_BNBWD, false, BF, U_BWD, NT, false, true>), grid, blk, 0, st, a);
  } else if (s.mode == PMU_SRC_BNBWD) {
    hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_BNBWD, false, BF, U_BWD, NT>), grid, blk, 0, st, a);
  } else {
    hipLaunchKernelGGL((frame_stream_kernel<PMU_SRC_RAW, false, BF, U_FLAT, NT>), grid, blk, 0, st, a);
  }
}

template <bool BF>
static int launch_stream(const pmu_frame* f, void* out, int ldo, hipStream_t st, void* out2 = nullptr, int ldo2 = 0) {
  const pmu_src& s = f->src[0];
  StreamArgs a;
  a.x = s.x; a.z = s.z; a.coef = s.coef; a.out = out;
  a.out2 = out2; a.ldo2 = ldo2;
  a.C = s.C;
  a.lg = 0;
  while ((8 << a.lg) < s.C) ++a.lg;
  a.H = f->H; a.W = f->W; a.SH = s.H; a.SW = s.W;
  a.P = (unsigned)((long long)f->N * f->H * f->W);
  a.ldo = ldo;
  static const int max_blocks = [] {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return 8 * cus;
  }();
  constexpr int U_POOL = 1, U_FLAT = 2, U_BWD = 2;
  const int U = s.pool == PMU_POOL_MAX2 ? U_POOL : s.mode == PMU_SRC_BNBWD ? U_BWD : U_FLAT;
  const long long span = (256LL >> a.lg) * U;
  long long g = ((long long)a.P + span - 1) / span;
  if (g > max_blocks) g = max_blocks;
  const dim3 grid((unsigned)g), blk(256);
  // cache policy (measured per shape, tools/kbench_frame.py, and per step): nontemporal loads and
  // stores for the bf16 passes over sources larger than the 256 MB last-level cache's share they
  // would thrash (c5 512^2 / 256^2 levels: -8..-10%), plain below it and for the fp32 passes (c2:
  // nontemporal measured +18% there)
  const char* ne = pmu_variant_env("PMU_FRAME_NT");
  const size_t xbytes = (size_t)f->N * s.H * s.W * s.C * sizeof(float);
  const bool nt = ne ? (atoi(ne) & 3) == 3 : (BF && xbytes >= ((size_t)128 << 20));
  if (nt) launch_stream_nt<BF, 3, U_POOL, U_FLAT, U_BWD>(s, grid, blk, st, a);
  else launch_stream_nt<BF, 0, U_POOL, U_FLAT, U_BWD>(s, grid, blk, st, a);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

static int pad8(int c) { return (c + 7) & ~7; }

static void geometry(int N, int H, int W, int Cin, int Cout, int* wco, int* twl, int* tiles_w, int* tiles_h,
                     int* ntiles, int* nsplit) {
  *wco = Cout > 64 ? 128 : 64;
  *twl = (W > 8) ? 4 : 3;
  const int TW = 1 << *twl, TH = wpix_of(*wco) / TW;
  *tiles_w = pmu_cdiv(W, TW);
  *tiles_h = pmu_cdiv(H, TH);
  *ntiles = N * *tiles_w * *tiles_h;
  const int blocks_mn = pmu_cdiv(Cout, *wco) * pmu_cdiv(Cin, WCI);
  static const int target = [] {  // PMU_WGB_BLOCKS: workgroups the split-K aims for (A/B)
    const char* e = getenv("PMU_WGB_BLOCKS");
    return e ? atoi(e) : 256;
  }();
  // one round of one block per CU: c5 6.41 -> 5.9 ms per step (512: two rounds; 128 / 192: 9.8 / 7.2 ms)
  int s = target / blocks_mn;
  if (s < 1) s = 1;
  if (s > *ntiles) s = *ntiles;
  *nsplit = s;
}

}  // namespace

extern "C" int pmu_frame_to_bf16(const pmu_frame* f, int Cpad, unsigned short* out, void* stream) {
  PMU_REQUIRE(valid_frame(f, true) && out && Cpad % 4 == 0);
  const int C = f->src[0].C + (f->nsrc > 1 ? f->src[1].C : 0);
  PMU_REQUIRE(Cpad >= C);
  if (stream_ok(f, Cpad)) return launch_stream<true>(f, out, Cpad, (hipStream_t)stream);
  const long long units = (long long)f->N * f->H * f->W * (Cpad / 8);
  bool fast = Cpad % 8 == 0 && units < (1LL << 31);
  for (int i = 0; i < f->nsrc; ++i) fast = fast && f->src[i].C % 8 == 0;
  if (fast) {
    long long g = (units + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(frame_to_bf16_fast_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                       make_dev_frame(f), Cpad, (unsigned)units, out, Cpad);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  const long long total = (long long)f->N * f->H * f->W * (Cpad / 4);
  long long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(frame_to_bf16_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, make_dev_frame(f),
                     Cpad, out);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_frame_to_f32(const pmu_frame* f, float* out, void* stream) {
  PMU_REQUIRE(valid_frame(f, true) && out);
  if (stream_ok(f, f->src[0].C)) return launch_stream<false>(f, out, f->src[0].C, (hipStream_t)stream);
  const DevFrame d = make_dev_frame(f);
  const long long units = (long long)d.N * d.H * d.W * (d.C / 4);
  if (d.vec && units < (1LL << 31)) {
    long long g = (units + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(frame_to_f32_fast_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, d,
                       (unsigned)units, out, d.C);
    PMU_CHECK_LAUNCH();
    return PMU_OK;
  }
  const long long total = (long long)d.N * d.H * d.W * ((d.C + 3) / 4);
  long long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(frame_to_f32_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, d, out);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" size_t pmu_conv3x3_wgrad_ws_bf16(int N, int H, int W, int Cin, int Cout) {
  int wco, twl, tw, th, nt, ns;
  geometry(N, H, W, Cin, Cout, &wco, &twl, &tw, &th, &nt, &ns);
  return (size_t)ns * 9 * Cout * Cin * sizeof(float);
}

extern "C" int pmu_conv3x3_wgrad_bf16(const unsigned short* dzt, const unsigned short* xt, int N, int H, int W,
                                      int Cout, int Cin, float* dw, float* ws, size_t ws_bytes, void* stream) {
  PMU_REQUIRE(dzt && xt && dw && ws && N > 0 && H > 0 && W > 0 && Cout > 0 && Cin > 0);
  WgbArgs a;
  a.dzt = dzt; a.xt = xt; a.ws = ws;
  a.N = N; a.H = H; a.W = W; a.Cout = Cout; a.Cin = Cin; a.Cop = pad8(Cout); a.Cip = pad8(Cin);
  int wco, twl;
  geometry(N, H, W, Cin, Cout, &wco, &twl, &a.tiles_w, &a.tiles_h, &a.ntiles, &a.nsplit);
  PMU_REQUIRE(ws_bytes >= (size_t)a.nsplit * 9 * Cout * Cin * sizeof(float));
  dim3 grid((unsigned)(pmu_cdiv(Cout, wco) * pmu_cdiv(Cin, WCI)), (unsigned)a.nsplit);
  hipStream_t st = (hipStream_t)stream;
  if (wco == 128) {
    if (twl == 4) hipLaunchKernelGGL((wgrad3x3_bf16_kernel<128, 4>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((wgrad3x3_bf16_kernel<128, 3>), grid, dim3(NT), 0, st, a);
  } else {
    if (twl == 4) hipLaunchKernelGGL((wgrad3x3_bf16_kernel<64, 4>), grid, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((wgrad3x3_bf16_kernel<64, 3>), grid, dim3(NT), 0, st, a);
  }
  PMU_CHECK_LAUNCH();
  const long long E = 9LL * Cout * Cin;
  hipLaunchKernelGGL(pmu_splitk_reduce9_kernel, dim3((unsigned)pmu_cdiv(E, 64)), dim3(256), 0, st, (const float*)ws,
                     a.nsplit, (long long)Cout * Cin, dw);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

// Diagnostic: resident blocks per CU of the main kernel of this file (hipOccupancy API).
extern "C" int pmu_occupancy_wgrad3x3_bf16(int* blocks_per_cu) {
  PMU_REQUIRE(blocks_per_cu);
  int n = 0;
  const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(wgrad3x3_bf16_kernel<128, 4>), 768, 0);
  if (e != hipSuccess) return (int)e;
  *blocks_per_cu = n;
  return PMU_OK;
}

// The frame written into the first channels of a wider NHWC tensor (pixel stride ldo): the skip half
// of the Up block's concat operand, whose other half the transposed conv writes in place
// (pmu_convT2x2_fwd_ld / pmu_convT2x2_fwd_dma_ld).  Vector paths only (channel counts of 4 / 8).
extern "C" int pmu_frame_to_f32_ld(const pmu_frame* f, float* out, int ldo, void* stream) {
  PMU_REQUIRE(valid_frame(f, true) && out);
  const DevFrame d = make_dev_frame(f);
  const long long units = (long long)d.N * d.H * d.W * (d.C / 4);
  PMU_REQUIRE(d.vec && units < (1LL << 31) && ldo >= d.C && ldo % 4 == 0 && (long long)d.N * d.H * d.W * ldo < (1LL << 32));
  if (stream_ok(f, d.C) && ldo % 8 == 0) return launch_stream<false>(f, out, ldo, (hipStream_t)stream);
  long long g = (units + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(frame_to_f32_fast_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, d,
                     (unsigned)units, out, ldo);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

extern "C" int pmu_frame_to_bf16_ld(const pmu_frame* f, int Cpad, unsigned short* out, int ldo, void* stream) {
  PMU_REQUIRE(valid_frame(f, true) && out && Cpad % 8 == 0 && ldo >= Cpad && ldo % 8 == 0);
  const int C = f->src[0].C + (f->nsrc > 1 ? f->src[1].C : 0);
  PMU_REQUIRE(Cpad >= C);
  const long long units = (long long)f->N * f->H * f->W * (Cpad / 8);
  bool fast = units < (1LL << 31);
  for (int i = 0; i < f->nsrc; ++i) fast = fast && f->src[i].C % 8 == 0;
  PMU_REQUIRE(fast);
  if (stream_ok(f, Cpad)) return launch_stream<true>(f, out, ldo, (hipStream_t)stream);
  long long g = (units + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(frame_to_bf16_fast_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     make_dev_frame(f), Cpad, (unsigned)units, out, ldo);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}

// The max-pooled BN+ReLU operand of a down block's first conv and, in the same pass, the unpooled
// activation into the first channels of the Up block's concat operand (pixel stride ldo_skip; see
// pmu_frame_to_bf16_ld): one read of the activation instead of two.  f: the pooled frame (one fp32
// BN+ReLU source, max-pooled, even source dims, channels a power-of-two multiple of 8 up to 2048).
extern "C" int pmu_frame_pool_skip_ok(const pmu_frame* f) {
  if (!valid_frame(f, true) || !stream_ok(f, f->src[0].C)) return 0;
  const pmu_src& s = f->src[0];
  return s.pool == PMU_POOL_MAX2 && s.mode == PMU_SRC_BNRELU && s.H == 2 * f->H && s.W == 2 * f->W &&
         (long long)f->N * s.H * s.W < (1LL << 31);
}

extern "C" int pmu_frame_to_bf16_pool_skip(const pmu_frame* f, unsigned short* out, unsigned short* skip, int ldo_skip,
                                           void* stream) {
  PMU_REQUIRE(out && skip && pmu_frame_pool_skip_ok(f) && ldo_skip >= f->src[0].C && ldo_skip % 8 == 0);
  return launch_stream<true>(f, out, f->src[0].C, (hipStream_t)stream, skip, ldo_skip);
}

extern "C" int pmu_frame_to_f32_pool_skip(const pmu_frame* f, float* out, float* skip, int ldo_skip, void* stream) {
  PMU_REQUIRE(out && skip && pmu_frame_pool_skip_ok(f) && ldo_skip >= f->src[0].C && ldo_skip % 8 == 0);
  return launch_stream<false>(f, out, f->src[0].C, (hipStream_t)stream, skip, ldo_skip);
}
