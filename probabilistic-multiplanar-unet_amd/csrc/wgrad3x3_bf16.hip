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
constexpr int WPIX = 64;    // pixels per K tile
constexpr int NT = 768;     // 12 waves
constexpr int MAX_HPX = 108;
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
  static constexpr int DS = WCO + 32;                 // D row stride (bf16): 320 B / 192 B
  static constexpr int D_ELEMS = WPIX * DS;
  static constexpr int SLOT = D_ELEMS + MAX_HPX * XS;  // one ring slot (bf16 elements)
  static constexpr int DU = WPIX * WCO / 8;            // 16-B units of a D tile
  static constexpr int ND = (DU + NT - 1) / NT;
  static constexpr int NX = (MAX_HPX * WCI / 8 + NT - 1) / NT;
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
  constexpr int TW = 1 << TWL, TH = WPIX >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
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
  constexpr int TW = 1 << TWL, TH = WPIX >> TWL, HW2 = TW + 2, HP = (TH + 2) * HW2;
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
  const int co0 = (blockIdx.x % nco) * WCO, ci0 = (blockIdx.x / nco) * WCI;
  const int split = blockIdx.y;
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
    for (int ks = 0; ks < WPIX / 16; ++ks) {
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

static int pad8(int c) { return (c + 7) & ~7; }

static void geometry(int N, int H, int W, int Cin, int Cout, int* wco, int* twl, int* tiles_w, int* tiles_h,
                     int* ntiles, int* nsplit) {
  *wco = Cout > 64 ? 128 : 64;
  *twl = (W > 8) ? 4 : 3;
  const int TW = 1 << *twl, TH = WPIX / TW;
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
  long long g = (units + 255) / 256;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(frame_to_bf16_fast_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     make_dev_frame(f), Cpad, (unsigned)units, out, ldo);
  PMU_CHECK_LAUNCH();
  return PMU_OK;
}
